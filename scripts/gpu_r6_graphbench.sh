#!/bin/bash
# Round 6: the non-deterministic graph test once more, then graph vs eager benches at configs 2 / 3.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/capture
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "graph_replay_matches" > $OUT/graphtest2.log 2>&1
grep -E "PASS|FAIL|worst" $OUT/graphtest2.log | cut -c1-600
B="--no-cpu-baseline --no-parity --steps 30 --warmup 5"
for c in 2 3; do
  timeout -k 10 400 python bench.py $B --config $c --graph 1 > $OUT/graph_c$c.json 2> $OUT/graph_c$c.err || exit 1
  timeout -k 10 400 python bench.py $B --config $c > $OUT/eager_c$c.json 2> $OUT/eager_c$c.err || exit 1
done
for f in graph_c2 eager_c2 graph_c3 eager_c3; do python -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',round(d['value'],3),round(d['ms_per_step'],3))"; done

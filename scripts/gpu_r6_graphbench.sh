#!/bin/bash
# Round 6: graph vs eager bench lines at configs 2 / 3 (after the K1 backward pool fix), then the
# config-3 captured step under rocprofv3 (wall vs kernel busy of the replayed steps; the bench's
# 10 eager profiling steps after the timed ones are skipped).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/graph
mkdir -p $OUT
export PYTHONUNBUFFERED=1
B="--no-cpu-baseline --no-parity --steps 30 --warmup 5"
for c in 2 3; do
  timeout -k 10 400 python bench.py $B --config $c --graph 1 > $OUT/graph_c$c.json 2> $OUT/graph_c$c.err || exit 1
  timeout -k 10 400 python bench.py $B --config $c > $OUT/eager_c$c.json 2> $OUT/eager_c$c.err || exit 1
done
for f in graph_c2 eager_c2 graph_c3 eager_c3; do python -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',round(d['value'],3),round(d['ms_per_step'],3))"; done
SKIP_MARKS=10 bash scripts/gpu_r4_benchprof.sh r6_c3graph --config 3 --graph 1 --no-cpu-baseline --no-parity --steps 20 --warmup 5

#!/bin/bash
# Round 5: the whole GPU suite with the single-process graph test on (the context it faulted in
# before the capture fixes), then graph vs eager benches at configs 2 and 3 with rocprof traces
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/y
mkdir -p $OUT
export PYTHONUNBUFFERED=1
VFD_TEST_GRAPHS=1 timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $OUT/suite.log 2>&1
rc=$?; tail -3 $OUT/suite.log; [ $rc = 0 ] || exit $rc
B="--no-cpu-baseline --no-parity --steps 20 --warmup 5"
for c in 2 3; do
  timeout -k 10 300 python bench.py $B --config $c --graph 1 > $OUT/graph_c$c.json 2> $OUT/graph_c$c.err || exit 1
  timeout -k 10 300 python bench.py $B --config $c > $OUT/eager_c$c.json 2> $OUT/eager_c$c.err || exit 1
  python -c "import json;g=json.load(open('$OUT/graph_c$c.json'));e=json.load(open('$OUT/eager_c$c.json'));print('config $c graph',g['ms_per_step'],'eager',e['ms_per_step'])"
done

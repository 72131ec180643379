#!/bin/bash
# Round 5: the captured step WITH the batched pairs and the pose branch's stream
# (VFD_GRAPH_BRANCHES=1): the graph-replay test in isolation, then graph vs eager benches
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/bb
mkdir -p $OUT
export PYTHONUNBUFFERED=1
VFD_GRAPH_BRANCHES=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "graph" > $OUT/test.log 2>&1
rc=$?; tail -3 $OUT/test.log; [ $rc = 0 ] || exit $rc
B="--no-cpu-baseline --no-parity --steps 30 --warmup 5"
VFD_GRAPH_BRANCHES=1 timeout -k 10 300 python bench.py $B --graph 1 > $OUT/graph_br.json 2> $OUT/graph_br.err || exit 1
timeout -k 10 300 python bench.py $B > $OUT/eager.json 2> $OUT/eager.err || exit 1
VFD_GRAPH_BRANCHES=1 timeout -k 10 300 python bench.py $B --graph 1 --config 3 > $OUT/graph_br_c3.json 2> $OUT/graph_br_c3.err || exit 1
timeout -k 10 300 python bench.py $B --config 3 > $OUT/eager_c3.json 2> $OUT/eager_c3.err || exit 1
for f in graph_br eager graph_br_c3 eager_c3; do python -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',d['value'],d['ms_per_step'])"; done

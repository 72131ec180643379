#!/bin/bash
# Round 6: which captured-step configuration is both correct and fast?
#  (1) single-stream capture (VFD_BRANCH_STREAMS=0), MIOpen as tuned: graph-vs-eager x3 (diag_graphtest)
#  (2) benches: graph single-stream; graph branch + MIOpen deterministic solvers (empty db, immediate mode)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/capture
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for i in 1 2 3; do
  VFD_BRANCH_STREAMS=0 timeout -k 10 300 python tools/diag_graphtest.py --self 0 > $OUT/gtmode.log 2>&1 || { tail -5 $OUT/gtmode.log; exit 1; }
  grep "^pre" $OUT/gtmode.log
done
B="--no-cpu-baseline --no-parity --steps 30 --warmup 5"
for c in 2 3; do
  VFD_BRANCH_STREAMS=0 timeout -k 10 400 python bench.py $B --config $c --graph 1 > $OUT/graph1s_c$c.json 2> $OUT/graph1s_c$c.err || exit 1
  VFD_DIAG_MIOPEN_DET=1 MIOPEN_DEBUG_CONVOLUTION_DETERMINISTIC=1 MIOPEN_USER_DB_PATH=$(mktemp -d) timeout -k 10 600 python bench.py $B --config $c --graph 1 --conv-autotune 0 > $OUT/graphdet_c$c.json 2> $OUT/graphdet_c$c.err || exit 1
done
for f in graph1s_c2 graphdet_c2 graph1s_c3 graphdet_c3; do python -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',round(d['value'],3),round(d['ms_per_step'],3))"; done

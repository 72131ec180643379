#!/bin/bash
# Round 6: after giving the K1 planned backward its own split-tile pool: the non-deterministic
# branch-stream capture vs eager x3, the bitwise deterministic workers, the graph tests.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/capture
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for i in 1 2 3; do
  timeout -k 10 300 python tools/diag_graphtest.py --self 0 > $OUT/gtfix.log 2>&1 || { tail -5 $OUT/gtfix.log; exit 1; }
  grep "^pre" $OUT/gtfix.log
done
bash scripts/gpu_r6_graphdet.sh || exit 1
bash scripts/gpu_r6_graphtests.sh

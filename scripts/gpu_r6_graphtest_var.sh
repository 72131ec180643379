#!/bin/bash
# Round 6: the graph test's sequence (tools/diag_graphtest.py) with MIOpen's deterministic solvers
# only, then with only the VFD kernels deterministic: which non-deterministic path races in the replay?
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/capture
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for env in "VFD_DIAG_MIOPEN_DET=1" "VFD_DIAG_MIOPEN_DET=1" "VFD_DETERMINISTIC=1" "VFD_DETERMINISTIC=1" "VFD_X=0" "VFD_X=0"; do
  env $env timeout -k 10 300 python tools/diag_graphtest.py --self 1 > $OUT/gtvar.log 2>&1 || { tail -5 $OUT/gtvar.log; exit 1; }
  grep "^pre" $OUT/gtvar.log
done

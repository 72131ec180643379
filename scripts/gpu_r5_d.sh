#!/bin/bash
# Round 5 step D: MIOpen solver picks of the reduced step, pose pairs on / off (eager only).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/d
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for P in 1 0; do
  VFD_POSE_PAIRS=$P MIOPEN_ENABLE_LOGGING=1 MIOPEN_LOG_LEVEL=5 timeout -k 10 300 python tools/diag_miopen_solvers.py --config 0 \
    > $OUT/pairs$P.out 2> $OUT/pairs$P.err || exit 1
  gzip -f $OUT/pairs$P.err
done
ls -la $OUT

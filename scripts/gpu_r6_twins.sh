#!/bin/bash
# Round 6: twin-model gradient comparison (tools/diag_twins.py) with / without the branch stream
# and a preceding eager step.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/capture
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for args in "--branch 1 --pre 1" "--branch 1 --pre 0" "--branch 0 --pre 1"; do
  timeout -k 10 300 python tools/diag_twins.py $args > $OUT/twins.log 2>&1 || exit 1
  grep -A5 "^branch" $OUT/twins.log
done

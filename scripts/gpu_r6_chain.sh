#!/bin/bash
# Round 6: the stage-by-stage gradient chain at the reduced and the full (config 2) shape.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/chain
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "gradient_chain" > $OUT/tests.log 2>&1
rc=$?; grep -a "loss path\|nets (\|PASSED\|FAILED\|^E " $OUT/tests.log | head -20; exit $rc

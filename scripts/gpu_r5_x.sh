#!/bin/bash
# Round 5: the parity file with the single-process graph-replay test enabled (after the capture
# fixes: kernel zero fills, gc before warm-up / capture, no host->device copies in the capture)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/x
mkdir -p $OUT
export PYTHONUNBUFFERED=1 VFD_TEST_GRAPHS=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > $OUT/parity.log 2>&1
rc=$?; tail -4 $OUT/parity.log; exit $rc

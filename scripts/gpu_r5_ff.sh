#!/bin/bash
# Round 5: determinism test incl. the branch-stream vs single-stream comparison
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5/ff
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_gpu_parity.py -k deterministic > gpurun_out/r5/ff/det.log 2>&1
rc=$?; tail -3 gpurun_out/r5/ff/det.log; exit $rc

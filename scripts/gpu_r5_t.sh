#!/bin/bash
# Round 5: the GPU suite WITH the graph tests (VFD_TEST_GRAPHS=1) after the round-5 capture fixes
# (zero fills as kernels instead of hipMemsetAsync nodes, gc before warm-up / capture, no
# host->device copies in the captured step)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/t
mkdir -p $OUT
export PYTHONUNBUFFERED=1 VFD_TEST_GRAPHS=1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $OUT/suite.log 2>&1
rc=$?; tail -5 $OUT/suite.log; exit $rc

#!/bin/bash
# K3C micro timings only (forward / data / weight gradient vs MIOpen) at config 2, then the K3C parity tests.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/micro_projconv.py --config 2 > gpurun_out/micro_projconv.txt 2>&1 || exit $?
cat gpurun_out/micro_projconv.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "proj_conv_matches" tests/test_gpu_fullsize.py > gpurun_out/k3c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/k3c_tests.log
exit $rc

#!/bin/bash
# K3C iteration: parity of the fused forward / data / weight gradients, then the micro timings.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "proj_conv_matches or deterministic" tests/test_gpu_fullsize.py tests/test_gpu_parity.py > gpurun_out/k3c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/k3c_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/micro_projconv.py --config 2 > gpurun_out/micro_projconv.txt 2>&1 || exit $?
cat gpurun_out/micro_projconv.txt

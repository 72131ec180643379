#!/bin/bash
# K3C data-gradient A/B: eight compute waves (default) vs the loader/compute split (VFD_PCD4=1), then parity.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/micro_projconv.py --config 2 > gpurun_out/micro_pcd8.txt 2>&1 || exit $?
VFD_PCD4=1 timeout -k 10 300 python -u tools/micro_projconv.py --config 2 > gpurun_out/micro_pcd4.txt 2>&1 || exit $?
grep dgrad gpurun_out/micro_pcd8.txt gpurun_out/micro_pcd4.txt; grep wgrad gpurun_out/micro_pcd8.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "proj_conv_matches" tests/test_gpu_fullsize.py > gpurun_out/k3c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/k3c_tests.log
exit $rc

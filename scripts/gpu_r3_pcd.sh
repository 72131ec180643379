#!/bin/bash
# K3C data-gradient A/B: 128-n tiles (one 32-column block per wave, default) vs 256-n tiles (VFD_PD_NB=2), then parity.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/micro_projconv.py --config 2 > gpurun_out/micro_nb1.txt 2>&1 || exit $?
VFD_LIB=variants/libvfd_nb2.so timeout -k 10 300 python -u tools/micro_projconv.py --config 2 > gpurun_out/micro_nb2.txt 2>&1 || exit $?
grep dgrad gpurun_out/micro_nb1.txt gpurun_out/micro_nb2.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "proj_conv_matches" tests/test_gpu_fullsize.py > gpurun_out/k3c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/k3c_tests.log
exit $rc

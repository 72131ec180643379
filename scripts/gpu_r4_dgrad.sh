#!/bin/bash
# round 4: the folded K3C data gradient (fp32 + bf16) — tests, then timings at the step shapes;
# also the pcdf (gen 1) variant for the A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 600 --timeout-method thread -m gpu \
  -k "dgrad_matches or dgrad_bf16 or proj_conv_matches_k3 or proj_conv_bf16 or folded_matches" > gpurun_out/r4/dgrad_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4/dgrad_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/micro_convbwd_capi.py --shapes c2,c3,c4,c5 > gpurun_out/r4/dgrad_micro.txt 2>&1 || exit $?
cat gpurun_out/r4/dgrad_micro.txt
if [ -f variants/libvfd_pcd1.so ]; then
  VFD_LIB=variants/libvfd_pcd1.so timeout -k 10 300 python tools/micro_convbwd_capi.py --ops dgrad --shapes c2,c4 > gpurun_out/r4/dgrad_micro_gen1.txt 2>&1 || exit $?
  cat gpurun_out/r4/dgrad_micro_gen1.txt
fi

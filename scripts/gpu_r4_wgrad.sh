#!/bin/bash
# round 4: bf16 weight gradients (K3C / K2C) — tests, timings vs MIOpen
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 600 --timeout-method thread -m gpu \
  -k "wgrad_bf16 or proj_conv_bf16 or pad_conv_bf16" > gpurun_out/r4/wgrad_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4/wgrad_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/r4/wgrad_tests.log | head -20; exit $rc; }
timeout -k 10 300 python tools/micro_convbwd_capi.py --ops wgrad_bf16,wgrad_bf16_miopen,pwgrad_bf16,pwgrad_bf16_miopen --shapes c3,c5 > gpurun_out/r4/wgrad_micro.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r4/wgrad_micro.txt

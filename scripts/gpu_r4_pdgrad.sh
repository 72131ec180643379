#!/bin/bash
# round 4: K2C data gradient (ppd) — tests, timings vs MIOpen
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 600 --timeout-method thread -m gpu \
  -k "pad_conv" > gpurun_out/r4/pdgrad_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4/pdgrad_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/r4/pdgrad_tests.log | head -20; exit $rc; }
timeout -k 10 300 python tools/micro_convbwd_capi.py --ops pdgrad,pdgrad_bf16,pdgrad_miopen --shapes c2,c3,c5 > gpurun_out/r4/pdgrad_micro.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r4/pdgrad_micro.txt

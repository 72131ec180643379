#!/bin/bash
# round 4: bf16 dgrad on 16x16 tiles (pch) — tests + timings vs pcg (bf1d) and the no-staging bound
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread -m gpu \
  -k "dgrad_bf16" > gpurun_out/r4/dgrad4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4/dgrad4_tests.log; [ $rc -eq 0 ] || exit $rc
for V in main bf1d; do
  if [ $V = main ]; then unset VFD_LIB; else export VFD_LIB=variants/libvfd_$V.so; fi
  echo "== $V"
  timeout -k 10 300 python tools/micro_convbwd_capi.py --ops dgrad_bf16 --shapes c2,c3,c5 > gpurun_out/r4/dgrad4_$V.txt 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/r4/dgrad4_$V.txt
done

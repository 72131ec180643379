#!/bin/bash
# round 4: K3C bf16 gradient kernels — parity tests (TESTK), then C-ABI micro timings of variant builds
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
if [ -n "$TESTK" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 500 --timeout-method thread -m gpu \
    -k "$TESTK" > gpurun_out/r4/k3c_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/r4/k3c_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for v in ${VARIANTS:-main}; do
  if [ "$v" = main ]; then lib=vfdepth_amd/libvfd_hip.so; else lib=variants/libvfd_$v.so; fi
  echo "== $v"
  VFD_LIB=$lib timeout -k 10 300 python tools/micro_convbwd_capi.py --ops ${OPS:-dgrad_bf16,wgrad_bf16} --shapes ${SHAPES:-c3} > gpurun_out/r4/k3c_$v.txt 2>&1 || { tail -5 gpurun_out/r4/k3c_$v.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/r4/k3c_$v.txt
done

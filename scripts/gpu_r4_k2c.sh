#!/bin/bash
# round 4: K2C bf16 forward / data gradient loader + prefetch variants — parity tests, then timings
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread -m gpu \
    -k "${TESTK:-pad_conv}" > gpurun_out/r4/k2c_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/r4/k2c_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/r4/k2c_tests.log | head -20; exit $rc; }
fi
OPS=${OPS:-pfwd_bf16,pdgrad_bf16}
for v in ${VARIANTS:-main head}; do
  if [ "$v" = main ]; then lib=vfdepth_amd/libvfd_hip.so; else lib=variants/libvfd_$v.so; fi
  echo "== $v"
  VFD_LIB=$lib timeout -k 10 300 python tools/micro_convbwd_capi.py --ops $OPS --shapes ${SHAPES:-c3,c2} \
    > gpurun_out/r4/k2c_$v.txt 2>&1 || { tail -5 gpurun_out/r4/k2c_$v.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/r4/k2c_$v.txt
done

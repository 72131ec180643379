#!/bin/bash
# round 4: where pcg's time goes — no-staging / no-B-load timing variants (outputs invalid, timing only)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
for V in nostage nob nostnob; do
  export VFD_LIB=variants/libvfd_$V.so
  echo "== $V"
  timeout -k 10 300 python tools/micro_convbwd_capi.py --shapes c2,c3 > gpurun_out/r4/dgrad3_$V.txt 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/r4/dgrad3_$V.txt
done

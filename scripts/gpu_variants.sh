#!/bin/bash
# micro_fusion (K3 backward) under library variants built by tools/build_variant.py
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in "$@"; do
  echo "== $v" >> gpurun_out/variants.txt
  if [ "$v" = base ]; then
    timeout -k 10 120 python tools/micro_fusion.py --ops vproj >> gpurun_out/variants.txt 2>&1 || exit 1
  else
    VFD_LIB=variants/libvfd_$v.so timeout -k 10 120 python tools/micro_fusion.py --ops vproj >> gpurun_out/variants.txt 2>&1 || exit 1
  fi
done

#!/bin/bash
# Time every variants/libvfd_*.so with the fusion micro-benchmark ($1 = ops).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/variants
export PYTHONUNBUFFERED=1
for lib in variants/libvfd_*.so; do
  n=$(basename $lib .so)
  VFD_LIB=$PWD/$lib timeout -k 10 120 python tools/micro_fusion.py --iters 20 --ops ${1:-pose} > gpurun_out/variants/$n.txt 2>&1 || exit $?
done

#!/bin/bash
# Kernel table of a short bench for every variants/libvfd_*.so.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/bvar
export PYTHONUNBUFFERED=1
for lib in variants/libvfd_*.so; do
  n=$(basename $lib .so)
  VFD_LIB=$PWD/$lib timeout -k 10 240 python bench.py --steps 5 --warmup 3 --kernel-table --no-cpu-baseline > gpurun_out/bvar/$n.json 2> gpurun_out/bvar/$n.err || exit $?
done

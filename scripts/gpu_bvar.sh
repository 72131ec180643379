#!/bin/bash
# Bench kernel table for every variants/libvfd_*.so ($1 = grep pattern for the lines to keep).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/bvar
export PYTHONUNBUFFERED=1
for lib in variants/libvfd_*.so; do
  n=$(basename $lib .so)
  VFD_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --kernel-table --steps 5 --warmup 2 > gpurun_out/bvar/$n.json 2> gpurun_out/bvar/$n.err || exit $?
done

#!/bin/bash
# Config 5 (640x960, 200x200x20 voxels): B=1 first with periodic stack dumps (a fresh box spends
# minutes in MIOpen's first-use work for new conv shapes), then the configured B=4.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/c5
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export VFD_BENCH_TRACEBACK=150
timeout -k 10 540 python bench.py --config 5 --batch 1 --steps 5 --warmup 2 --kernel-table --no-cpu-baseline \
  > $OUT/bench_c5_b1.json 2> $OUT/bench_c5_b1.err || exit $?
timeout -k 10 540 python bench.py --config 5 --steps 5 --warmup 2 --kernel-table --no-cpu-baseline \
  > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit $?

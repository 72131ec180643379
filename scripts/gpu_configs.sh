#!/bin/bash
# Full-size benches of configs 3 (B=2), 4 (NuScenes 352x640) and 5 (640x960, 4x voxels, B=4) on one
# GPU, each under its own time limit; stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/configs
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for c in 4 3 5; do
  timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 3 --kernel-table --no-cpu-baseline \
    > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || exit $?
done

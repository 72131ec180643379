#!/bin/bash
# Final-tree benches of configs 4, 3 (bf16 nets, B=2) and 5 (B=4), each under its own limit.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/configs2
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for c in 4 3 5; do
  timeout -k 10 660 python bench.py --config $c --steps 5 --warmup 2 --kernel-table --no-cpu-baseline \
    > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || exit $?
done

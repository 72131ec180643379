#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python tools_diag_grads.py > gpurun_out/diag.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 10 --warmup 4 --no-cpu-baseline --conv-autotune 1 --kernel-table > gpurun_out/bench_autotune.log 2> gpurun_out/bench_autotune.err

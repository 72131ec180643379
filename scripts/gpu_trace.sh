#!/bin/bash
# Steady-state kernel trace of the eager step (per-kernel breakdown: tools/kernel_breakdown.py).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/trace -o run --output-format csv -- python bench.py --graph 0 --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/trace_bench.log 2>&1
rc=$?
echo "rocprof rc=$rc" >> gpurun_out/trace_bench.log
exit $rc

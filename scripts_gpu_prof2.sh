#!/bin/bash
# GPU tests + steady-state kernel trace of the eager step (per-kernel breakdown of the last steps).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -k "graph or full_step" > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/trace -o run --output-format csv -- python bench.py --graph 0 --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/trace_bench.log 2>&1
rc=$?
echo "rocprof rc=$rc" >> gpurun_out/trace_bench.log
exit $rc

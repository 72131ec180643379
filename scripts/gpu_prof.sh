#!/bin/bash
# rocprofv3 kernel-trace summary of the default bench + a bench run with the CPU baseline.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
rc=$?
echo "rocprof rc=$rc" >> gpurun_out/prof_bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py --steps 20 --warmup 5 --kernel-table > gpurun_out/bench_full.log 2> gpurun_out/bench_full.err
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench_full.err
exit $rc

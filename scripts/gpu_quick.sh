#!/bin/bash
# Quick loop: GPU parity tests (optionally filtered by $1) + fusion micro-benchmark + short bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/micro
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests -m gpu -q -rf ${1:+-k "$1"} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/micro_fusion.py --iters 10 > gpurun_out/micro/times.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --kernel-table --no-cpu-baseline > gpurun_out/bench.log 2> gpurun_out/bench.err

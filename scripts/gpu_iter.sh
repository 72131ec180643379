#!/bin/bash
# Iteration run: selected GPU tests (-k expression $1), then a short bench (tag $2) -> gpurun_out/
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
K=${1:-.}; TAG=${2:-iter}; shift 2
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -k "$K" --timeout 240 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/iter_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --kernel-table --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench_$TAG.err
exit $rc

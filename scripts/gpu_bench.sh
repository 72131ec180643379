#!/bin/bash
# Bench runs: `scripts/gpu_bench.sh [tag] [bench args...]` -> gpurun_out/bench_<tag>.{json,err}.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-default}; shift
timeout -k 10 900 python bench.py --kernel-table "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench_$TAG.err
exit $rc

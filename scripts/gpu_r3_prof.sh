#!/bin/bash
# config-2 bench line (no CPU leg) and kernel-trace breakdowns of configs 2 and 3
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --kernel-table > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit $?
echo "bench ok"
bash scripts/gpu_profile.sh c3 --config 3 || exit $?
echo "prof c3 ok"
bash scripts/gpu_profile.sh c2 --config 2 || exit $?
echo "prof c2 ok"

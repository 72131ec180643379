#!/bin/bash
# config-2 bench line (no CPU leg, kernel table) and its kernel-trace breakdown
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --kernel-table > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit $?
echo "bench ok"; python -c "import json;d=json.load(open('gpurun_out/bench_c2.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['frac'])"
bash scripts/gpu_profile.sh c2 --config 2 || exit $?
echo "prof c2 ok"; head -45 gpurun_out/prof_c2/breakdown.txt

#!/bin/bash
# round-3 final measurement: the default bench line (CPU baseline + parity, kernel table), its
# kernel-trace profile, and config 3's PMC traffic
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python bench.py --kernel-table > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel'],round(d['roofline']['frac'],3),d['cpu_baseline'])"
bash scripts/gpu_profile.sh final || exit 1
head -3 gpurun_out/prof_final/breakdown.txt
bash scripts/gpu_traffic_cfg.sh 3 || exit 1

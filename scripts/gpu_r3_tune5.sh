#!/bin/bash
# MIOpen benchmark-mode solver search at config 5 (fp32, B=4, 640x960, 200x200x20 voxels)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/miopen_db_tuned5
export PYTHONUNBUFFERED=1
timeout -k 10 900 python bench.py --config 5 --no-cpu-baseline --no-parity --steps 3 --warmup 2 --conv-autotune 1 > gpurun_out/t5_a.json 2> gpurun_out/t5_a.err || exit $?
cp miopen_db/*.txt gpurun_out/miopen_db_tuned5/
timeout -k 10 400 python bench.py --config 5 --no-cpu-baseline --no-parity --steps 10 --warmup 3 > gpurun_out/bench_c5_tuned.json 2> gpurun_out/t5_b.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c5_tuned.json'));print('c5 tuned',d['value'],d['ms_per_step'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --steps 20 --warmup 5 > gpurun_out/bench_c2_db.json 2> gpurun_out/t5_c.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c2_db.json'));print('c2 with the merged db',d['value'],d['ms_per_step'])"
wc -l miopen_db/*

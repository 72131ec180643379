#!/bin/bash
# MIOpen benchmark-mode solver search: config 3 with NCHW encoders (to compare layouts on tuned
# dbs), then configs 4 and 5; immediate-mode lines after; the db is copied back after each stage
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/miopen_db_tuned4
export PYTHONUNBUFFERED=1
VFD_CHANNELS_LAST=0 timeout -k 10 900 python bench.py --config 3 --no-cpu-baseline --no-parity --steps 5 --warmup 2 --conv-autotune 1 > gpurun_out/t4_a.json 2> gpurun_out/t4_a.err || exit $?
cp miopen_db/*.txt gpurun_out/miopen_db_tuned4/
VFD_CHANNELS_LAST=0 timeout -k 10 400 python bench.py --config 3 --no-cpu-baseline --no-parity --steps 10 --warmup 3 > gpurun_out/bench_c3_nchw_tuned.json 2> gpurun_out/t4_b.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c3_nchw_tuned.json'));print('c3 nchw tuned',d['value'],d['ms_per_step'])"
timeout -k 10 400 python bench.py --config 3 --no-cpu-baseline --no-parity --steps 10 --warmup 3 > gpurun_out/bench_c3_cl_tuned.json 2> gpurun_out/t4_c.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c3_cl_tuned.json'));print('c3 channels-last tuned',d['value'],d['ms_per_step'])"
timeout -k 10 400 python bench.py --config 4 --no-cpu-baseline --no-parity --steps 10 --warmup 3 > gpurun_out/bench_c4_before.json 2> gpurun_out/t4_d.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c4_before.json'));print('c4 before',d['value'],d['ms_per_step'])"
timeout -k 10 900 python bench.py --config 4 --no-cpu-baseline --no-parity --steps 5 --warmup 2 --conv-autotune 1 > gpurun_out/t4_e.json 2> gpurun_out/t4_e.err || exit $?
cp miopen_db/*.txt gpurun_out/miopen_db_tuned4/
timeout -k 10 400 python bench.py --config 4 --no-cpu-baseline --no-parity --steps 10 --warmup 3 > gpurun_out/bench_c4_tuned.json 2> gpurun_out/t4_f.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c4_tuned.json'));print('c4 tuned',d['value'],d['ms_per_step'])"
wc -l miopen_db/*

#!/bin/bash
# MIOpen benchmark-mode solver search at config 3 (bf16 shapes have no find-db entries), then the
# immediate-mode step with the tuned user db; the db is copied back
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python bench.py --config 3 --no-cpu-baseline --no-parity --steps 10 --warmup 3 --conv-autotune 1 > gpurun_out/bench_c3_tuned.json 2> gpurun_out/bench_c3_tuned.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c3_tuned.json'));print('c3 benchmark mode',d['value'],d['ms_per_step'])"
mkdir -p gpurun_out/miopen_db_tuned3 && cp miopen_db/* gpurun_out/miopen_db_tuned3/
timeout -k 10 400 python bench.py --config 3 --no-cpu-baseline --no-parity --steps 10 --warmup 3 > gpurun_out/bench_c3_after.json 2> gpurun_out/bench_c3_after.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c3_after.json'));print('c3 immediate after tuning',d['value'],d['ms_per_step'])"
wc -l miopen_db/*

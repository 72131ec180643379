#!/bin/bash
# MIOpen benchmark-mode solver search (torch.backends.cudnn.benchmark) at configs 2 and 3 vs the
# immediate-mode picks; the resulting user find-db is copied back
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --steps 20 --warmup 5 > gpurun_out/bench_c2_base.json 2> gpurun_out/bench_c2_base.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c2_base.json'));print('c2 immediate',d['value'],d['ms_per_step'])"
timeout -k 10 600 python bench.py --no-cpu-baseline --no-parity --steps 20 --warmup 5 --conv-autotune 1 > gpurun_out/bench_c2_tuned.json 2> gpurun_out/bench_c2_tuned.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c2_tuned.json'));print('c2 benchmark mode',d['value'],d['ms_per_step'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --steps 20 --warmup 5 > gpurun_out/bench_c2_after.json 2> gpurun_out/bench_c2_after.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c2_after.json'));print('c2 immediate after tuning',d['value'],d['ms_per_step'])"
mkdir -p gpurun_out/miopen_db_tuned && cp miopen_db/* gpurun_out/miopen_db_tuned/
wc -l miopen_db/*

#!/bin/bash
# config-3 bench line (tuned find-db, channels-last encoders) and its steady-state kernel breakdown
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python bench.py --config 3 --no-cpu-baseline --steps 10 --warmup 3 --kernel-table > gpurun_out/bench_c3_final.json 2> gpurun_out/bench_c3_final.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c3_final.json'));print('c3',d['value'],d['ms_per_step'],d.get('parity'))"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_c3_cl -o run --output-format csv -- python bench.py --config 3 --no-cpu-baseline --no-parity --steps 4 --warmup 2 > gpurun_out/prof_c3_cl.log 2>&1 || exit $?
python tools/kernel_breakdown.py $(find gpurun_out/prof_c3_cl -name '*kernel_trace.csv' | head -1) --last 3 --top 70 > gpurun_out/kbd_c3_final.txt
rm -rf gpurun_out/prof_c3_cl
head -30 gpurun_out/kbd_c3_final.txt | cut -c1-140

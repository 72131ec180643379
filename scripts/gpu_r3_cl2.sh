#!/bin/bash
# config 2 (fp32) with channels-last encoders vs the default NCHW (Winograd) encoders
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
VFD_CHANNELS_LAST=all timeout -k 10 400 python bench.py --no-cpu-baseline --no-parity --steps 20 --warmup 5 > gpurun_out/bench_c2_cl.json 2> gpurun_out/bench_c2_cl.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c2_cl.json'));print('c2 channels-last',d['value'],d['ms_per_step'])"
timeout -k 10 400 python bench.py --no-cpu-baseline --no-parity --steps 20 --warmup 5 > gpurun_out/bench_c2_nchw.json 2> gpurun_out/bench_c2_nchw.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c2_nchw.json'));print('c2 nchw',d['value'],d['ms_per_step'])"
timeout -k 10 300 python -u tools/micro_wrw_layout.py > gpurun_out/micro_wrw_fp32.txt 2>&1 || exit $?
grep -v "Warn\|amdgpu.ids" gpurun_out/micro_wrw_fp32.txt | tail -6

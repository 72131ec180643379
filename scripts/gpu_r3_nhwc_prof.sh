#!/bin/bash
# config-3 kernel stats with and without channels-last encoders
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3_cl -o run --output-format csv -- python bench.py --config 3 --no-cpu-baseline --no-parity --steps 4 --warmup 2 > gpurun_out/prof_c3_cl.log 2>&1 || exit $?
VFD_CHANNELS_LAST=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3_nchw -o run --output-format csv -- python bench.py --config 3 --no-cpu-baseline --no-parity --steps 4 --warmup 2 > gpurun_out/prof_c3_nchw.log 2>&1 || exit $?
for v in cl nchw; do python tools/kernel_breakdown.py $(find gpurun_out/prof_c3_$v -name '*kernel_trace.csv' | head -1) --last 3 --top 70 > gpurun_out/kbd_c3_$v.txt; done
for v in cl nchw; do f=$(find gpurun_out/prof_c3_$v -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/kstats_c3_$v.csv; done
find gpurun_out/prof_c3_cl -type f | head -20
rm -rf gpurun_out/prof_c3_cl gpurun_out/prof_c3_nchw
du -sh gpurun_out
echo ok

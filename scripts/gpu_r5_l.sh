#!/bin/bash
# Round 5: the bench line + rocprofv3 kernel statistics on the new defaults (channels-last fp32
# encoders, benchmark mode, frame pairs batched), twice on one box, and the per-step kernel diff of
# the two runs (is the run-to-run spread a different solver pick or the same kernels running slower?)
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_r4_benchprof.sh r5_a || exit 1
bash scripts/gpu_r4_benchprof.sh r5_b --no-cpu-baseline || exit 1
A=$(ls gpurun_out/bp_r5_a/stats/*/run_kernel_trace.csv.gz gpurun_out/bp_r5_a/stats/run_kernel_trace.csv.gz 2>/dev/null | head -1)
B=$(ls gpurun_out/bp_r5_b/stats/*/run_kernel_trace.csv.gz gpurun_out/bp_r5_b/stats/run_kernel_trace.csv.gz 2>/dev/null | head -1)
python tools/kernel_diff.py $A $B --last 5 --skip-a 1 --skip-b 1 --labels run_a,run_b > gpurun_out/bp_r5_b/diff_a_b.txt 2>&1; head -40 gpurun_out/bp_r5_b/diff_a_b.txt

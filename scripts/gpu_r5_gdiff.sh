#!/bin/bash
# Round 5: kernel-name diff of the captured step vs the eager step in the SAME configuration (frame
# pairs one at a time, one stream — as the capture runs them), config 2, both under rocprofv3
cd "$GRAFT_REPO_ROOT" || exit 1
VFD_POSE_PAIRS=0 VFD_BRANCH_STREAMS=0 bash scripts/gpu_r4_benchprof.sh r5_eager1 --no-cpu-baseline || exit 1
bash scripts/gpu_r4_benchprof.sh r5_graph --no-cpu-baseline --graph 1 || exit 1
A=gpurun_out/bp_r5_eager1/stats/run_kernel_trace.csv.gz; B=gpurun_out/bp_r5_graph/stats/run_kernel_trace.csv.gz
python tools/kernel_diff.py $A $B --last 5 --skip-a 2 --skip-b 2 --labels eager,graph > gpurun_out/bp_r5_graph/diff_eager_graph.txt 2>&1
head -30 gpurun_out/bp_r5_graph/diff_eager_graph.txt

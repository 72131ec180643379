#!/bin/bash
# Round 5: phase timeline of the branch-stream step (HIP events on both streams)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5/kk
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/diag_phases.py > gpurun_out/r5/kk/phases.txt 2> gpurun_out/r5/kk/phases.err; echo rc=$?
cat gpurun_out/r5/kk/phases.txt
VFD_BRANCH_STREAMS=0 timeout -k 10 300 python tools/diag_phases.py > gpurun_out/r5/kk/phases_single.txt 2>> gpurun_out/r5/kk/phases.err; echo rc=$?
cat gpurun_out/r5/kk/phases_single.txt

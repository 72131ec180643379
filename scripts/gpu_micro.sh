#!/bin/bash
# One-off micro timings of the fused dense kernels (tools/micro_dense.py), plus a kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python tools/micro_dense.py > gpurun_out/micro_dense.txt 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/mdprof" -o md -- python3 "$GRAFT_REPO_ROOT/tools/micro_dense.py" > "$GRAFT_REPO_ROOT/gpurun_out/micro_dense_prof.txt" 2>&1 || exit 1

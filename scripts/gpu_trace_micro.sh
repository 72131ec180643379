#!/bin/bash
# Kernel trace (durations only) of the fusion micro-benchmark ($1 = ops).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/tm
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/micro_fusion.py --iters 5 --ops ${1:-pose} > $OUT/trace.log 2>&1

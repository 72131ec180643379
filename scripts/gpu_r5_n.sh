#!/bin/bash
# Round 5: capture-only checks of the graphed step (no replay): host<->device transfers inside the
# capture and autograd graphs kept alive into it (VFD_GRAPH_CHECK=1), at the graph test's config
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/n
mkdir -p $OUT
export PYTHONUNBUFFERED=1
VFD_GRAPH_CHECK=1 timeout -k 10 300 python tools/diag_graph_step.py --replays 0 > $OUT/check.txt 2> $OUT/check.err
echo "check rc=$?"; tail -30 $OUT/check.txt; grep -v Warning $OUT/check.err | tail -30

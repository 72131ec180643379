#!/bin/bash
# Round 5: the captured graph of the graph-test step as DOT (no replay) + the allocator's segments
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/o
mkdir -p $OUT
export PYTHONUNBUFFERED=1
VFD_GRAPH_DUMP=$OUT/graph.dot timeout -k 10 300 python tools/diag_graph_step.py --replays 0 > $OUT/dump.txt 2> $OUT/dump.err
echo "dump rc=$?"; tail -5 $OUT/dump.txt; ls -la $OUT; gzip -f $OUT/graph.dot

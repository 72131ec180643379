#!/bin/bash
# Round 6: graph replay vs eager, bit for bit (tests/graph_det_worker.py): deterministic mode plain /
# DDP, then the non-deterministic mode (VFD_GRAPH_DET_OFF=1: only replay-vs-replay orderings are exact).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/capture
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tests/graph_det_worker.py > $OUT/graphdet.log 2>&1; rc=$?; tail -1 $OUT/graphdet.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tests/graph_det_worker.py --ddp > $OUT/graphdet_ddp.log 2>&1; rc=$?; tail -1 $OUT/graphdet_ddp.log; exit $rc

#!/bin/bash
# Round 6: captured default step (pose branch stream) vs eager, per-net / per-parameter gradients:
# with the optimizer step in the graph, then without it (is the Adam step racing the branch?).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/capture
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/diag_capture.py --compare > $OUT/cmp_branch.log 2>&1 || exit $?
timeout -k 10 300 python tools/diag_capture.py --compare --no-opt > $OUT/cmp_branch_noopt.log 2>&1 || exit $?
for f in cmp_branch cmp_branch_noopt; do echo "== $f"; grep -A6 "losses graph\|_net:" $OUT/$f.log | head -16; done

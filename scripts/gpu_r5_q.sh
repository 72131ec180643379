#!/bin/bash
# Round 5: reference cycles holding a step's autograd graph (eager only)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/q
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/diag_cycles.py --config -1 --pairs 0 > $OUT/cycles0.txt 2> $OUT/cycles0.err; echo "rc=$?"
head -80 $OUT/cycles0.txt
timeout -k 10 300 python tools/diag_cycles.py --config -1 --pairs 1 > $OUT/cycles1.txt 2> $OUT/cycles1.err; echo "rc=$?"
head -30 $OUT/cycles1.txt

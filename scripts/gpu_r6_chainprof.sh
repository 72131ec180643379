#!/bin/bash
# Round 6: the full-resolution gradient dump for the stage-2 analysis (tools/diag_gradchain.py gpu;
# its cpu / nets halves run on the host).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/chain
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/diag_gradchain.py gpu $OUT/gradchain_full.npz > $OUT/gradchain.log 2>&1 || exit 1
tail -1 $OUT/gradchain.log

#!/bin/bash
# Round 5: which framework ops launch the remaining copies / adds / fills (config 2, defaults)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/cc
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/op_attribution.py --top 60 --match copy,add,Fill,transpose,Cat,reduce > $OUT/attr.txt 2> $OUT/attr.err || exit 1
head -3 $OUT/attr.txt

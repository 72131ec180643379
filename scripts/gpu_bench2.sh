#!/bin/bash
# Repeat the default bench (box-to-box / run-to-run variance check).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/bench2
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/a.json 2> $OUT/a.err || exit $?
timeout -k 10 400 python bench.py --kernel-table > $OUT/b.json 2> $OUT/b.err || exit $?

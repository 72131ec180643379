#!/bin/bash
# MIOpen benchmark-mode search at config 5 with the user db copied back every minute (the search
# ran past 15 minutes before: keep what it records even if the limit ends it)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/miopen_db_tuned5
export PYTHONUNBUFFERED=1
( while true; do cp miopen_db/*.txt gpurun_out/miopen_db_tuned5/ 2>/dev/null; sleep 60; done ) &
CP=$!
timeout -k 10 1080 python bench.py --config 5 --no-cpu-baseline --no-parity --steps 1 --warmup 1 --conv-autotune 1 > gpurun_out/t5b.json 2> gpurun_out/t5b.err
rc=$?
kill $CP
cp miopen_db/*.txt gpurun_out/miopen_db_tuned5/
wc -l miopen_db/*.txt
echo "search rc=$rc"

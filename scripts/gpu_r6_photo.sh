#!/bin/bash
# Round 6: photo_fwd_k occupancy experiment: K5 parity tests + the bench kernel table.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/photo
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests -k "photo or loss" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --kernel-table > $OUT/bench.json 2> $OUT/table.txt || exit 1
grep "photo\|hot-path" $OUT/table.txt

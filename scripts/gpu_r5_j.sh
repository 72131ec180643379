#!/bin/bash
# Round 5: does a bench right after the parity tests on the same box run slow (37 ms in step I vs
# 33 ms fresh)?  parity tests, bench, bench, then the bench in immediate mode for reference.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/j
mkdir -p $OUT
export PYTHONUNBUFFERED=1
B="--no-cpu-baseline --no-parity --steps 20 --warmup 5"
pr() { python -c "import json;d=json.load(open('$OUT/$1.json'));print('$1',d['value'],d['ms_per_step'])"; }
ls -la miopen_db > $OUT/db_before.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py > $OUT/parity.log 2>&1 || exit 1
tail -1 $OUT/parity.log
ls -la miopen_db > $OUT/db_after.txt; diff $OUT/db_before.txt $OUT/db_after.txt
timeout -k 10 400 python bench.py $B > $OUT/b1.json 2> $OUT/b1.err && pr b1 || exit 1
timeout -k 10 400 python bench.py $B > $OUT/b2.json 2> $OUT/b2.err && pr b2 || exit 1
ls -la ~/.config/miopen ~/.cache/miopen 2>/dev/null | head -20

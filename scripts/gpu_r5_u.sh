#!/bin/bash
# Round 5: K3C data-gradient address arithmetic (per-tile pixel geometry, uniform fold deltas,
# scalar prefetch offsets, compare-based epilogue rows): parity tests, then the bench profile
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/u
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "proj_conv or config3_step" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "full_step or full_resolution" > $OUT/tests2.log 2>&1
rc=$?; tail -3 $OUT/tests2.log; [ $rc = 0 ] || exit $rc
SKIP_MARKS=2 bash scripts/gpu_r4_benchprof.sh r5_c || exit 1
grep -n "pcdf_main\|pcv_main\|pcw_main" gpurun_out/bp_r5_c/breakdown.txt | head

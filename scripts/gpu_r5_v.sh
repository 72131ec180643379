#!/bin/bash
# Round 5: K2C forward per-tile geometry + loader row limit: parity tests, then the bench profile
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/v
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "pad_conv or pose_conv or fuse_pose" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "full_step" > $OUT/tests2.log 2>&1
rc=$?; tail -3 $OUT/tests2.log; [ $rc = 0 ] || exit $rc
bash scripts/gpu_r4_benchprof.sh r5_d || exit 1
grep -n "pcdf_main\|pcv_main\|pcw_main\|ppc_main" gpurun_out/bp_r5_d/breakdown.txt | head
timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > $OUT/bench.json 2> $OUT/bench.err && python -c "import json;d=json.load(open('$OUT/bench.json'));print('bench',d['value'],d['ms_per_step'])"

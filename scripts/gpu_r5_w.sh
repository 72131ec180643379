#!/bin/bash
# Round 5: K2C bf16 forward / data-gradient per-tile geometry + 32-bit loader offsets: parity tests,
# then the config-3 bench profile (bf16 nets) and the config-2 bench
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/w
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "pad_conv or pose_conv or config3 or fuse_pose" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || exit $rc
bash scripts/gpu_r4_benchprof.sh r5_c3 --config 3 || exit 1
grep -n "ppd_main\|ppcb_main\|pcvb\|pch_main\|pwb_main" gpurun_out/bp_r5_c3/breakdown.txt | head

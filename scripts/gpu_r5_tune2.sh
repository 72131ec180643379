#!/bin/bash
# Round 5: MIOpen find-db for config 2's new shapes — the pose net's stacked frame pairs (batch 12
# NCHW fp32, the K2C backward at B = 2 NHWC) and, for the channels-last fp32 A/B, the NHWC fp32
# encoder shapes — by one benchmark-mode run each; then immediate-mode bench lines of both layouts.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/tune2
mkdir -p $OUT
export PYTHONUNBUFFERED=1
B="--no-cpu-baseline --no-parity --steps 10 --warmup 3"
timeout -k 10 900 python bench.py $B --conv-autotune 1 > $OUT/nchw_tune.json 2> $OUT/nchw_tune.err || exit $?
mkdir -p $OUT/db_nchw && cp miopen_db/* $OUT/db_nchw/
VFD_CHANNELS_LAST=all timeout -k 10 900 python bench.py $B --conv-autotune 1 > $OUT/cl_tune.json 2> $OUT/cl_tune.err || exit $?
mkdir -p $OUT/db_all && cp miopen_db/* $OUT/db_all/
timeout -k 10 400 python bench.py $B > $OUT/nchw.json 2> $OUT/nchw.err || exit $?
VFD_CHANNELS_LAST=all timeout -k 10 400 python bench.py $B > $OUT/cl.json 2> $OUT/cl.err || exit $?
VFD_POSE_PAIRS=0 timeout -k 10 400 python bench.py $B > $OUT/nchw_nopairs.json 2> $OUT/nchw_nopairs.err || exit $?
for f in nchw_tune cl_tune nchw cl nchw_nopairs; do
  python -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',d['value'],d['ms_per_step'])"
done

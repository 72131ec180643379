#!/bin/bash
# Round 5: channels-last fp32 encoders at config 2 with a TUNED MIOpen find-db (round 3's 36.2 ms
# measurement ran its NHWC fp32 convs on immediate-mode heuristics: the db held 6 NHWC fp32 shapes).
# One benchmark-mode run records MIOpen's measured picks for the NHWC fp32 shapes, then immediate-
# mode bench lines of both layouts on the same box.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/tune2
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/miopen_db   # the tuning run writes the committed db
B="--no-cpu-baseline --no-parity --steps 10 --warmup 3"
VFD_CHANNELS_LAST=all timeout -k 10 900 python bench.py $B --conv-autotune 1 > $OUT/cl_tune.json 2> $OUT/cl_tune.err || exit $?
mkdir -p $OUT/db && cp miopen_db/* $OUT/db/
timeout -k 10 400 python bench.py $B > $OUT/nchw.json 2> $OUT/nchw.err || exit $?
VFD_CHANNELS_LAST=all timeout -k 10 400 python bench.py $B > $OUT/cl.json 2> $OUT/cl.err || exit $?
for f in cl_tune nchw cl; do
  python -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',d['value'],d['ms_per_step'])"
done

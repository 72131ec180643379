#!/bin/bash
# Round 5: the pose net's frame pairs as one batch (VFD_POSE_PAIRS=1) on the new defaults
# (channels-last fp32 encoders, MIOpen benchmark mode), same box, alternating.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/k
mkdir -p $OUT
export PYTHONUNBUFFERED=1
B="--no-cpu-baseline --no-parity --steps 20 --warmup 5"
pr() { python -c "import json;d=json.load(open('$OUT/$1.json'));print('$1',d['value'],d['ms_per_step'])"; }
for i in 1 2; do
  VFD_POSE_PAIRS=1 timeout -k 10 400 python bench.py $B > $OUT/pairs$i.json 2> $OUT/pairs$i.err && pr pairs$i || exit 1
  VFD_POSE_PAIRS=0 timeout -k 10 400 python bench.py $B > $OUT/single$i.json 2> $OUT/single$i.err && pr single$i || exit 1
done

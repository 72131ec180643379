#!/bin/bash
# Round 5: channels-last vs NCHW fp32 encoders at config 2, benchmark-mode vs immediate-mode MIOpen,
# on one box with the tuned find-db (miopen_db/, NHWC fp32 shapes added by gpu_r5_tune2.sh).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/cl
mkdir -p $OUT
export PYTHONUNBUFFERED=1
B="--no-cpu-baseline --no-parity --steps 20 --warmup 5"
for L in all 0; do for A in 1 0; do
  VFD_CHANNELS_LAST=$L timeout -k 10 400 python bench.py $B --conv-autotune $A > $OUT/cl${L}_a$A.json 2> $OUT/cl${L}_a$A.err || exit $?
  python -c "import json;d=json.load(open('$OUT/cl${L}_a$A.json'));print('CL=$L autotune=$A',d['value'],d['ms_per_step'])"
done; done

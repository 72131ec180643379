#!/bin/bash
# round 4: MIOpen benchmark-mode search for the channels-last bf16 decoder shapes (VFD_DEC_CL=1) at
# config 3, the db copied back, then the immediate-mode step with each decoder layout
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4
mkdir -p $OUT
export PYTHONUNBUFFERED=1
VFD_DEC_CL=1 timeout -k 10 900 python bench.py --config 3 --no-cpu-baseline --no-parity --steps 5 --warmup 2 --conv-autotune 1 > $OUT/tune_deccl.json 2> $OUT/tune_deccl.err || { tail -5 $OUT/tune_deccl.err; exit 1; }
mkdir -p $OUT/miopen_db_deccl && cp miopen_db/* $OUT/miopen_db_deccl/
wc -l miopen_db/*
for v in 1 0 1; do
  VFD_DEC_CL=$v timeout -k 10 400 python bench.py --config 3 --no-cpu-baseline --no-parity --steps 10 --warmup 3 > $OUT/tdeccl_$v.json 2> $OUT/tdeccl_$v.err || { tail -5 $OUT/tdeccl_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/tdeccl_$v.json'));print('tuned VFD_DEC_CL=$v config 3', round(d['ms_per_step'],2), 'ms/step')"
done

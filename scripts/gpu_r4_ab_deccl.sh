#!/bin/bash
# round 4: config-3 A/B of the decoder layout (VFD_DEC_CL 0 / 1, alternating) on the committed find-db
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4
mkdir -p $OUT
export PYTHONUNBUFFERED=1
k=0
for v in ${ORDER:-0 1 0 1}; do
  k=$((k+1))
  VFD_DEC_CL=$v timeout -k 10 400 python bench.py --config ${CONFIG:-3} --no-cpu-baseline --no-parity --steps ${STEPS:-20} --warmup 3 > $OUT/ab_${k}_$v.json 2> $OUT/ab_${k}_$v.err || { tail -5 $OUT/ab_${k}_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab_${k}_$v.json'));print('run $k VFD_DEC_CL=$v', round(d['ms_per_step'],2), 'ms/step')"
done

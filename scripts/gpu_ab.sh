#!/bin/bash
# A/B of the side-stream planning (VFD_SIDE_PLANS=1) against in-order planning (0), eager bench.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/ab
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for v in 0 1 0 1; do
  VFD_SIDE_PLANS=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/side$v.json 2> $OUT/side$v.err || exit $?
  python -c "import json;d=json.load(open('$OUT/side$v.json'));print('side', $v, round(d['ms_per_step'],2))" >> $OUT/summary.txt
done

#!/bin/bash
# Round 5: issue the depth branch before the pose branch (VFD_DEPTH_FIRST=1) — bench A/B alternating
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/hh
mkdir -p $OUT
export PYTHONUNBUFFERED=1
B="--no-cpu-baseline --no-parity --steps 30 --warmup 5"
pr() { python -c "import json;d=json.load(open('$OUT/$1.json'));print('$1',d['value'],d['ms_per_step'])"; }
for i in 1 2; do
  VFD_DEPTH_FIRST=1 timeout -k 10 300 python bench.py $B > $OUT/df$i.json 2> $OUT/df$i.err && pr df$i || exit 1
  VFD_DEPTH_FIRST=0 timeout -k 10 300 python bench.py $B > $OUT/pf$i.json 2> $OUT/pf$i.err && pr pf$i || exit 1
done

#!/bin/bash
# Round 5: K3C forward gather with 6 positions' corner rows in flight (VFD_PCG_U=6) vs 4: kernel
# table + step time, alternating
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/gg
mkdir -p $OUT
export PYTHONUNBUFFERED=1
B="--no-cpu-baseline --no-parity --steps 30 --warmup 5 --kernel-table"
for i in 1 2; do
  VFD_LIB=variants/libvfd_pcg6.so timeout -k 10 300 python bench.py $B > $OUT/u6_$i.json 2> $OUT/u6_$i.err || exit 1
  timeout -k 10 300 python bench.py $B > $OUT/u4_$i.json 2> $OUT/u4_$i.err || exit 1
  for v in u6 u4; do python -c "import json;d=json.load(open('$OUT/${v}_$i.json'));print('$v',d['ms_per_step'])"; grep "proj_conv_fwd " $OUT/${v}_$i.err | head -1; done
done

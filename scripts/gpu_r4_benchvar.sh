#!/bin/bash
# round 4: bench kernel tables of variant builds at one config (VARIANTS, CONFIG)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4
mkdir -p $OUT
export PYTHONUNBUFFERED=1
C=${CONFIG:-3}
for v in ${VARIANTS:-main}; do
  if [ "$v" = main ]; then lib=vfdepth_amd/libvfd_hip.so; else lib=variants/libvfd_$v.so; fi
  VFD_LIB=$lib timeout -k 10 600 python bench.py --config $C --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-parity --kernel-table > $OUT/bv_${v}_c$C.json 2> $OUT/bv_${v}_c$C.err || { tail -5 $OUT/bv_${v}_c$C.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bv_${v}_c$C.json'));print('$v config $C', round(d['ms_per_step'],2), 'ms/step')"
  grep -E "${GREP:-proj_conv|pad_conv}" $OUT/bv_${v}_c$C.err
done

#!/bin/bash
# round 4: channels-last bf16 decoders — parity tests, then config-3 bench with VFD_DEC_CL off / on
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu -s tests/test_gpu_fullsize.py \
  -k "channels_last_decoder or elu_upsample or dense_maps_bf16 or decoder_conv_mfma" > $OUT/deccl_tests.log 2>&1 \
  || { tail -40 $OUT/deccl_tests.log; exit 1; }
grep -E "passed|failed|decoder " $OUT/deccl_tests.log
C=${CONFIG:-3}
for v in ${DECCL:-0 1}; do
  VFD_DEC_CL=$v timeout -k 10 600 python bench.py --config $C --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-parity --kernel-table > $OUT/deccl_${v}_c$C.json 2> $OUT/deccl_${v}_c$C.err || { tail -5 $OUT/deccl_${v}_c$C.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/deccl_${v}_c$C.json'));print('VFD_DEC_CL=$v config $C', round(d['ms_per_step'],2), 'ms/step')"
  grep -E "${GREP:-transpose|elu_pad|reflect_pad|igemm|naive|conv}" $OUT/deccl_${v}_c$C.err | head -30
done

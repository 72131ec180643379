#!/bin/bash
# Round 5: the encoder input converted to channels-last once, the weight swap without a contiguous
# copy: step tests + pad-conv tests, then two benches
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/dd
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "full_step or full_resolution or pad_conv or pose_conv or channels_last or config3" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || exit $rc
B="--no-cpu-baseline --no-parity --steps 30 --warmup 5"
for i in 1 2; do timeout -k 10 300 python bench.py $B > $OUT/b$i.json 2> $OUT/b$i.err || exit 1
python -c "import json;d=json.load(open('$OUT/b$i.json'));print('b$i',d['value'],d['ms_per_step'])"; done

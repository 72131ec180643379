#!/bin/bash
# Round 5 step A: full-resolution reference parity, the PadConvBF16 fallback, pose-batching micro, bench.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/a
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "full_resolution or full_step_against" tests/test_gpu_fullsize.py::test_pad_conv_bf16_wgrad_declined_falls_back \
  > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python tools/micro_pose_batch.py > $OUT/micro_pose_batch.txt 2>&1 || exit 1
cat $OUT/micro_pose_batch.txt
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['parity']['full_resolution'])"

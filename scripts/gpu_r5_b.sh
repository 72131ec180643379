#!/bin/bash
# Round 5 step B: grouped BN + the pose pairs as one batch — parity tests, then the bench.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/b
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py -k "groups_equal or batchnorm_act_matches or pose_conv or pad_conv_matches" \
  > $OUT/tests1.log 2>&1 || { tail -40 $OUT/tests1.log; exit 1; }
tail -2 $OUT/tests1.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_ddp.py tests/test_gpu_0_ddp_world2.py \
  > $OUT/tests2.log 2>&1 || { tail -40 $OUT/tests2.log; exit 1; }
tail -2 $OUT/tests2.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['parity']['full_resolution'])"

#!/bin/bash
# BN kernels: parity tests, then the config-2 kernel-trace breakdown (BN lines)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "batchnorm_act or residual_join or ddp" tests/test_gpu_fullsize.py tests/test_gpu_ddp.py tests/test_gpu_0_ddp_world2.py > gpurun_out/bn_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAIL" gpurun_out/bn_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_profile.sh c2 --config 2 || exit $?
grep -E "bn_|bn1_|ms/step, kernel" gpurun_out/prof_c2/breakdown.txt | cut -c1-110
python -c "import json;d=json.load(open('gpurun_out/prof_c2/bench.json'));print(d['value'],d['ms_per_step'])"

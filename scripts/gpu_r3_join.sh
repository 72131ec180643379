#!/bin/bash
# residual join: its own test, the BN tests and the full-step parity / determinism tests, then a bench line
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "residual_join or batchnorm_act or full_step or deterministic or config3_step" tests/test_gpu_fullsize.py tests/test_gpu_parity.py > gpurun_out/join_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error" gpurun_out/join_tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c2.json'));print(d['value'],d['ms_per_step'])"

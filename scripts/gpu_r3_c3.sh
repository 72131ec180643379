#!/bin/bash
# config-3 bench line and the config-3 step test
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python bench.py --config 3 --no-cpu-baseline --no-parity --steps 10 --warmup 3 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c3.json'));print('c3',d['value'],d['ms_per_step'])"
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -p no:cacheprovider \
  -k "config3_step or pad_conv_bf16 or bf16_nets" tests/test_gpu_fullsize.py tests/test_gpu_parity.py > gpurun_out/c3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAIL" gpurun_out/c3_tests.log | tail -5; exit $rc

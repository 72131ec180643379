#!/bin/bash
# K2C / K3C batch: micros, conv parity, the golden-fixture parity suite, step bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 180 python tools/micro_padconv.py > gpurun_out/micro_pp.log 2>&1 || exit 1
K="pad_conv or proj_conv" bash scripts/gpu_tests.sh tests/test_gpu_fullsize.py || exit 1
cp gpurun_out/tests/tests.log gpurun_out/tests_conv.log
bash scripts/gpu_tests.sh tests/test_gpu_parity.py || exit 1
bash scripts/gpu_bench.sh r2_pp --steps 10 --no-cpu-baseline --no-parity || exit 1

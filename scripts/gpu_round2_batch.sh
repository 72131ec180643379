#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
K="deterministic or reflect_pad or proj_conv or pad_conv" bash scripts/gpu_tests.sh tests/test_gpu_parity.py tests/test_gpu_fullsize.py || exit 1
cp gpurun_out/tests/tests.log gpurun_out/tests_det.log
bash scripts/gpu_bench.sh r2_det --steps 10 --no-cpu-baseline --no-parity || exit 1

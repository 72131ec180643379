#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
K="config3_step_b2 or full_step_gradient_chain" bash scripts/gpu_tests.sh tests/test_gpu_fullsize.py tests/test_gpu_parity.py || exit 1
cp gpurun_out/tests/tests.log gpurun_out/tests_fix.log
bash scripts/gpu_bench.sh r2_all --steps 20 --no-cpu-baseline || exit 1
bash scripts/gpu_profile.sh r2

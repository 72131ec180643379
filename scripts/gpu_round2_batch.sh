#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
K="max_pool or batchnorm or reflect_pad or full_step or deterministic or aggregat" bash scripts/gpu_tests.sh tests/test_gpu_parity.py tests/test_gpu_fullsize.py || exit 1
cp gpurun_out/tests/tests.log gpurun_out/tests_t.log
bash scripts/gpu_bench.sh r2_idx --steps 20 --no-cpu-baseline --no-parity || exit 1

#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
K="max_pool or reflect_pad or full_step or deterministic or plan or fuse" bash scripts/gpu_tests.sh tests/test_gpu_parity.py tests/test_gpu_fullsize.py || exit 1
cp gpurun_out/tests/tests.log gpurun_out/tests_t.log
bash scripts/gpu_bench.sh r2_mp2 --steps 20 --no-cpu-baseline --no-parity || exit 1
timeout -k 10 300 python tools/micro_dense.py > gpurun_out/micro_dense.txt 2>&1 || exit 1

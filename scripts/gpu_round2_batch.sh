#!/bin/bash
# K3C batch: micro (fused fwd / dgrad vs K3 + MIOpen), K3C full-size parity, step bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 180 python tools/micro_projconv.py > gpurun_out/micro_pc.log 2>&1 || exit 1
K="proj_conv or k3c" bash scripts/gpu_tests.sh tests/test_gpu_fullsize.py || exit 1
bash scripts/gpu_bench.sh r2_fused --steps 10 --no-cpu-baseline --no-parity || exit 1

#!/bin/bash
# K3C side-output batch: micro (fused vs K3 + MIOpen), K3C full-size parity, fused / unfused step bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash scripts/gpu_pcvar.sh || exit 1
K="proj_conv or k3c" bash scripts/gpu_tests.sh tests/test_gpu_fullsize.py || exit 1
bash scripts/gpu_bench.sh r2_fused --steps 10 --no-cpu-baseline --no-parity || exit 1
VFD_PROJ_CONV=0 bash scripts/gpu_bench.sh r2_unfused --steps 10 --no-cpu-baseline --no-parity || exit 1

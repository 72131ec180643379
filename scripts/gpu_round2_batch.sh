#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash scripts/gpu_bench.sh r2_bn --steps 10 --no-cpu-baseline --no-parity || exit 1
VFD_FUSED_BN=0 bash scripts/gpu_bench.sh r2_nobn --steps 10 --no-cpu-baseline --no-parity || exit 1
timeout -k 10 400 python tools/diag_ops.py > gpurun_out/ops.txt 2> gpurun_out/ops.err

#!/bin/bash
# Step bench under MIOpen solver switches / layouts: gpurun_out/bench_env_<tag>.{json,err}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
A="--steps 10 --no-cpu-baseline --no-parity"
bash scripts/gpu_bench.sh env_base $A || exit 1
MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 bash scripts/gpu_bench.sh env_nowrwnhwc $A || exit 1
MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 bash scripts/gpu_bench.sh env_nobwdnhwc $A || exit 1
MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0 bash scripts/gpu_bench.sh env_nofwdnhwc $A || exit 1
bash scripts/gpu_bench.sh env_cl $A --channels-last 1 || exit 1

#!/bin/bash
# which aten op / shapes launch the cast / copy / conv kernels of the config-3 (bf16, B=2) step
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python tools/op_attribution.py --config 3 --top 70 --match SubTensorOpWithCast,igemm,bfloat16,kernel_grouped,transpose > gpurun_out/op_attr_c3.txt 2>&1 || exit $?
grep -v Warning gpurun_out/op_attr_c3.txt | head -75 | cut -c1-250

#!/bin/bash
# which aten op / shapes launch MIOpen's conv kernels in the config-2 step
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/op_attribution.py --config 2 --top 120 --match igemm_bwd,igemm_wrw,SubTensorOpWithScalar > gpurun_out/op_attr_conv.txt 2>&1 || exit $?
grep -v Warning gpurun_out/op_attr_conv.txt | head -100 | cut -c1-230

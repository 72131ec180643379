#!/bin/bash
# Fusion-kernel micro-benchmark + PMC passes on it (one counter group per pass).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/micro
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 300 python tools/micro_fusion.py --iters 10 --ops ${1:-pose,vproj} > gpurun_out/micro/times.txt 2>&1 || exit $?
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctr -d gpurun_out/micro/pmc$i -o run --output-format csv -- python tools/micro_fusion.py --iters 3 --ops ${1:-pose,vproj} > gpurun_out/micro/pmc$i.log 2>&1 || exit $?
done

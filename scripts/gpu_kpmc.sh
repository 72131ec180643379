#!/bin/bash
# PMC passes (one counter group each) over the fusion micro-benchmark ($1 = ops) -> gpurun_out/kpmc.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/kpmc
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
cd /tmp
i=0
for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 90 rocprofv3 --pmc $ctr -d $OUT/p$i -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/micro_fusion.py --iters 3 --ops ${1:-vproj} > $OUT/p$i.log 2>&1 || exit $?
done

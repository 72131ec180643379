#!/bin/bash
# PMC passes of the K2C bf16 forward + data gradient (micro tool, config 3 shape)
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r4/pmc_k2c
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"
P2="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
for i in 1 2 3 4; do
  eval P=\$P$i
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- python $R/tools/micro_convbwd_capi.py --ops ${OPS:-pfwd_bf16,pdgrad_bf16} --shapes c3 --iters 3 > $OUT/p$i.log 2>&1) || exit $?
done
python tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1; grep -E "==|ppcb|ppd_|ppc_" $OUT/summary.txt | head -60

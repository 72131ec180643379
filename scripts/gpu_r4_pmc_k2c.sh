#!/bin/bash
# PMC passes of the K2C bf16 kernels (micro tool, config 3 shape): OPS, VARIANTS (main = in-tree build)
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"
P2="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD"
P3="SQ_INSTS_SMEM SQ_INSTS_MFMA SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_LDS"
for V in ${VARIANTS:-main}; do
  OUT=$R/gpurun_out/r4/pmc_k2c_$V
  mkdir -p $OUT
  if [ $V = main ]; then unset VFD_LIB; else export VFD_LIB=$R/variants/libvfd_$V.so; fi
  for i in 1 2 3; do
    eval P=\$P$i
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- python $R/tools/micro_convbwd_capi.py --ops ${OPS:-pdgrad_bf16} --shapes c3 --iters 3 > $OUT/p$i.log 2>&1) || exit $?
  done
  python tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1; echo "== $V"; grep -E "ppd_main|kIDF16bDF16b" $OUT/summary.txt | cut -c1-400
done

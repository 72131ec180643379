#!/bin/bash
# PMC comparison of the K3C data-gradient forms at config 2: pcg (main build) vs pcdf (variant pcd1)
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r4/pmc_dgrad
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"
P2="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD"
for V in main pcd1; do
  LIBENV=""
  [ $V = pcd1 ] && export VFD_LIB=$R/variants/libvfd_pcd1.so || unset VFD_LIB
  for i in 1 2; do
    eval P=\$P$i
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/${V}_$i -o run --output-format csv -- python $R/tools/micro_convbwd_capi.py --ops ${OPS:-dgrad} --shapes c2 --iters 3 > $OUT/${V}_$i.log 2>&1) || exit $?
  done
done
unset VFD_LIB
python tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt | head -80

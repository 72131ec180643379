#!/bin/bash
# PMC pass over the K3C kernels (micro_projconv): MFMA busy, waits, LDS conflicts
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_k3c
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $OUT/p1 -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/micro_projconv.py --iters 3 > $OUT/p1.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $OUT/p2 -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/micro_projconv.py --iters 3 > $OUT/p2.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
python tools/pmc_kernels.py $OUT pcd_main pcdf_main pcv_main pcw_main > gpurun_out/pmc_k3c.txt
cat gpurun_out/pmc_k3c.txt

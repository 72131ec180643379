#!/bin/bash
# PMC passes over the MFMA conv kernels (tools/micro_projconv.py, tools/micro_padconv.py):
# MFMA busy / wait / LDS conflicts, then L2 hit rates.  Each pass its own run and time limit.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_conv
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $OUT/p1 -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/micro_projconv.py --iters 3 > $OUT/p1.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/p2 -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/micro_projconv.py --iters 3 > $OUT/p2.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $OUT/p3 -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/micro_padconv.py --iters 3 > $OUT/p3.log 2>&1 || exit $?

#!/bin/bash
# Instruction-mix PMC pass over the fusion micro-benchmark ($1 = ops).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc2
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
OPS=${1:-pose}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/p4 -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/micro_fusion.py --iters 3 --ops $OPS > $OUT/p4.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE -d $OUT/p5 -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/micro_fusion.py --iters 3 --ops $OPS > $OUT/p5.log 2>&1

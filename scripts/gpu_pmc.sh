#!/bin/bash
# PMC passes over the fusion micro-benchmark ($1 = ops): kernel trace, HBM fetch + L2 hit, waits.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
OPS=${1:-pose}
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/micro_fusion.py --iters 5 --ops $OPS > $OUT/trace.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum -d $OUT/p1 -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/micro_fusion.py --iters 3 --ops $OPS > $OUT/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_MISS_sum -d $OUT/p2 -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/micro_fusion.py --iters 3 --ops $OPS > $OUT/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_BUSY_CYCLES -d $OUT/p3 -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/micro_fusion.py --iters 3 --ops $OPS > $OUT/p3.log 2>&1

#!/bin/bash
# Round 6: K3C data-gradient rewrite + row-parallel combine kernels: micro timing, the bench kernel
# table, and the full-resolution gradient-chain dump (tools/diag_gradchain.py gpu).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/k3c
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/micro_projconv.py --config 2 > $OUT/micro.log 2>&1 || exit 1
cat $OUT/micro.log
timeout -k 10 400 python bench.py --no-cpu-baseline --kernel-table > $OUT/bench.json 2> $OUT/bench_table.txt || exit 1
cat $OUT/bench.json
timeout -k 10 300 python tools/diag_gradchain.py gpu $OUT/gradchain_full.npz > $OUT/gradchain.log 2>&1 || exit 1
tail -2 $OUT/gradchain.log

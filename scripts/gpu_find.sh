#!/bin/bash
# (1) fusion micro-benchmark; (2) MIOpen find-mode warm-up of the default bench, continuing the
# committed user db (copied to gpurun_out/miopen_db, merged back afterwards).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/micro gpurun_out/miopen_db
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/micro_fusion.py --iters 10 > gpurun_out/micro/times.txt 2>&1 || exit $?
cp miopen_db/*.txt gpurun_out/miopen_db/
MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db timeout -k 10 1000 python bench.py --graph 0 --conv-autotune 1 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/find.log 2> gpurun_out/find.err
echo "find rc=$?" >> gpurun_out/find.err

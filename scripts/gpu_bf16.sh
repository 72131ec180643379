#!/bin/bash
# bf16-nets parity test, reduce_dim dgrad micro-benchmark, config-3 bench (bf16 nets, B=2).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/bf16
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -k bf16 > $OUT/test.log 2>&1 || exit $?
timeout -k 10 300 python tools/micro_dgrad.py > $OUT/micro_dgrad.log 2>&1 || exit $?
timeout -k 10 450 python bench.py --config 3 --steps 10 --warmup 3 --kernel-table --no-cpu-baseline \
  > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit $?

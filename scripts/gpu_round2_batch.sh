#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
K="voxel or proj or full_step or deterministic" bash scripts/gpu_tests.sh tests/test_gpu_parity.py tests/test_gpu_fullsize.py || exit 1
cp gpurun_out/tests/tests.log gpurun_out/tests_t.log
bash scripts/gpu_bench.sh r2_vpb --steps 20 --no-cpu-baseline --no-parity || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/traffic
mkdir -p $OUT
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $OUT/write.log 2>&1 || exit $?

#!/bin/bash
# Round-end validation: the whole -m gpu suite, smoke, the default bench (cpu baseline + parity),
# a kernel-trace profile and PMC traffic passes.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash scripts/gpu_tests.sh tests/test_gpu_ddp.py || exit 1
cp gpurun_out/tests/tests.log gpurun_out/tests_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --kernel-table > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
bash scripts/gpu_profile.sh r2final || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/traffic
mkdir -p $OUT
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $OUT/write.log 2>&1 || exit $?

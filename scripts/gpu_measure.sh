#!/bin/bash
# Round measurement: GPU parity tests, smoke, the default bench (with CPU baseline), a rocprofv3
# kernel-trace/stats pass of the bench and two PMC passes (FETCH_SIZE, WRITE_SIZE) for traffic.
# Every GPU step has its own time limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/measure
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --kernel-table > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 600 python bench.py --graph 1 --no-cpu-baseline > $OUT/bench_graph.json 2> $OUT/bench_graph.err || exit $?
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/stats -o bench --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/stats.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/$OUT/pmc_fetch -o bench --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/$OUT/pmc_write -o bench --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/pmc_write.log 2>&1 || exit $?

#!/bin/bash
# FETCH_SIZE calibration probe + per-op HBM traffic of the step (FETCH_SIZE and WRITE_SIZE passes).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/traffic
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/probe -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/probe_fetch.py > $OUT/probe.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $OUT/write.log 2>&1 || exit $?

#!/bin/bash
# Selected GPU parity tests ($1 = -k filter), then the default bench with the per-kernel table
# (no CPU baseline) -> gpurun_out/kb_*.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ${1:+-k "$1"} > gpurun_out/kb_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/kb_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --kernel-table ${2} > gpurun_out/kb_bench.json 2> gpurun_out/kb_bench.err

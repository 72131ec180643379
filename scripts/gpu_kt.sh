#!/bin/bash
# Kernel loop: selected GPU parity tests ($1 = -k filter), then a rocprofv3 kernel trace of the
# fusion micro-benchmark ($2 = ops) -> gpurun_out/tm.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/tm
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q -rf --timeout 200 --timeout-method thread ${1:+-k "$1"} > gpurun_out/k_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/k_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/tm -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/micro_fusion.py --iters 5 --ops ${2:-vproj} > $GRAFT_REPO_ROOT/gpurun_out/tm/trace.log 2>&1

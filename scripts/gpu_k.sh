#!/bin/bash
# Kernel loop: selected GPU parity tests ($1 = -k filter) + fusion micro-benchmark ($2 = ops).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -q -rf --timeout 200 --timeout-method thread ${1:+-k "$1"} > gpurun_out/k_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/k_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/micro_fusion.py --iters 20 ${2:+--ops $2} > gpurun_out/k_micro.txt 2>&1

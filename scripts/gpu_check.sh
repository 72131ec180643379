#!/bin/bash
# Focused check: selected GPU parity tests ($1 = -k filter) + full-step gradient diagnostic.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf -s --timeout 300 --timeout-method thread ${1:+-k "$1"} > gpurun_out/check_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/check_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python tools/diag_grads.py > gpurun_out/diag.log 2>&1

#!/bin/bash
# The whole GPU suite, as the driver runs it at round end.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/all_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/all_tests.log

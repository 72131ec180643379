#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python tools/diag_stages.py > gpurun_out/diag_stages.log 2>&1

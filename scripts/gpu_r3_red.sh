#!/bin/bash
# reduce kernels: K3C / K2C parity, then per-config PMC traffic
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "proj_conv or pad_conv or config3_step" tests/test_gpu_fullsize.py > gpurun_out/red_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAIL" gpurun_out/red_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_traffic_cfg.sh 2 3 5

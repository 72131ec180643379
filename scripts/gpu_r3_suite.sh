#!/bin/bash
# the whole -m gpu suite + smoke on the final tree
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash scripts/gpu_alltests.sh
tail -1 gpurun_out/all_tests.log | grep -q "rc=0" || { tail -30 gpurun_out/all_tests.log; exit 1; }
tail -3 gpurun_out/all_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log

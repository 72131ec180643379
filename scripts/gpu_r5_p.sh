#!/bin/bash
# Round 5: the ordered depth-synthesis backward's tests, then the graph DOT dump (capture only)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/p
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "depth_synthesis" > $OUT/ds.log 2>&1
rc=$?; tail -8 $OUT/ds.log; [ $rc = 0 ] || exit $rc
bash scripts/gpu_r5_o.sh

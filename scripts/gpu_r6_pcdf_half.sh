#!/bin/bash
# Round 6: the K3C data gradient with the half-width last n-tile as its own launch: parity
# (folded / padded / full-size K3C tests) and the micro timing at config 2.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/pcdf_half
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py -k "proj_conv" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/micro_projconv.py --config 2 > $OUT/micro.log 2>&1 || exit 1
grep dgrad $OUT/micro.log

#!/bin/bash
# Round 6: the K2 backward with the split-tile combine in its main kernel (last part sums the
# slots): K2 parity / determinism / graph tests, then the bench kernel table.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/posecombine
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests \
  -k "pose or fuse or deterministic or bit_identical" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --kernel-table > $OUT/bench.json 2> $OUT/table.txt || exit 1
grep "fuse_pose_bwd\|hot-path" $OUT/table.txt

#!/bin/bash
# Conv experiments with the committed MIOpen user db: immediate mode (default), find mode,
# channels-last.  Each run under its own limit; stop at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # name, limit, args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/$name.log 2> gpurun_out/$name.err
  local rc=$?
  echo "rc=$rc" >> gpurun_out/$name.err
  return $rc
}
run conv_db 400 --graph 0 || exit $?
run conv_db_find 400 --graph 0 --conv-autotune 1 || exit $?
run conv_cl 600 --graph 0 --channels-last 1 || exit $?
run conv_db_graph 400 --graph 1 || exit $?

#!/bin/bash
# Bench execution modes: default eager, HIP graph, channels-last nets.  Each under its own limit.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/modes
export PYTHONUNBUFFERED=1
run() {  # name, limit, args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python bench.py --steps 10 --warmup 3 --no-cpu-baseline --kernel-table "$@" > gpurun_out/modes/$name.json 2> gpurun_out/modes/$name.err
  local rc=$?
  echo "rc=$rc" >> gpurun_out/modes/$name.err
  return $rc
}
run eager 300 || exit $?
run graph 300 --graph 1 || exit $?
run cl 400 --channels-last 1 || exit $?

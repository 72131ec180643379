#!/bin/bash
# Round-end measurement: `scripts/gpu_round_end.sh tests` = the whole -m gpu suite + smoke;
# `scripts/gpu_round_end.sh bench TAG` = the default bench line (CPU baseline + parity) and a
# kernel-trace profile (gpurun_out/prof_TAG).  Every step has its own time limit; stop at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
if [ "$1" = tests ]; then
  bash scripts/gpu_alltests.sh
  tail -1 gpurun_out/all_tests.log | grep -q "rc=0" || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit 1
else
  TAG=${2:-final}
  timeout -k 10 600 python bench.py --kernel-table > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
  bash scripts/gpu_profile.sh $TAG || exit 1
fi

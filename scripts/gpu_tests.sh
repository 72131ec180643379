#!/bin/bash
# GPU tests: `scripts/gpu_tests.sh [pytest selection...]` (default: the whole -m gpu suite).
# Each step has its own time limit; the script stops at the first crash / timeout.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/tests
mkdir -p $OUT
export PYTHONUNBUFFERED=1
# optional: K='expr' selects tests by keyword
SEL=${@:-tests}
KARG=()
[ -n "$K" ] && KARG=(-k "$K")
timeout -k 10 1500 python -u -m pytest $SEL "${KARG[@]}" -m gpu -v -rf --timeout 900 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log
exit $rc

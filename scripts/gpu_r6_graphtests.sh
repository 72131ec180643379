#!/bin/bash
# Round 6: the graph-replay tests (plain default step, DDP world 1) on their own.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/capture
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_ddp.py -k "graph_replay" > $OUT/graphtests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|worst" $OUT/graphtests.log | cut -c1-600; exit $rc

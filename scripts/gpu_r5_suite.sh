#!/bin/bash
# Round 5: the whole -m gpu suite (stops at the first failure), then the DDP graph test on its own.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/suite
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests \
  --deselect tests/test_gpu_ddp.py::test_ddp_graphed_step_world1_matches_eager > $OUT/suite.log 2>&1
rc=$?; tail -3 $OUT/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_ddp.py::test_ddp_graphed_step_world1_matches_eager > $OUT/ddp_graph.log 2>&1
rc=$?; tail -3 $OUT/ddp_graph.log; exit $rc

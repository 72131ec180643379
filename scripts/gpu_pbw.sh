#!/bin/bash
# K2 backward loop: pose/fusion GPU parity tests, the per-task trace (VFD_PBW_TRACE variant), a
# kernel trace of the pose micro-benchmark and the bench kernel table -> gpurun_out/pbw_*.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pbw_tm
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q -rf --timeout 200 --timeout-method thread -k "${1:-pose or vfnet or full_step or graph}" > gpurun_out/pbw_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pbw_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
VFD_LIB=variants/libvfd_trace.so timeout -k 10 200 python tools/diag_pbw_trace.py > gpurun_out/pbw_trace.txt 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pbw_tm -o run --output-format csv -- python tools/micro_fusion.py --iters 5 --ops pose > gpurun_out/pbw_tm/trace.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --kernel-table > gpurun_out/pbw_bench.json 2> gpurun_out/pbw_bench.err
if [ -n "$PBW_DIAG_GRAPH" ]; then
  timeout -k 10 300 python tools/diag_graph.py 4 > gpurun_out/pbw_diag_graph.txt 2>&1
fi

#!/bin/bash
# GPU session: parity tests, smoke, short eager bench with kernel table.  Stops at any GPU fault /
# abort / timeout.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc" >> gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after smoke rc=$rc"; exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --kernel-table --no-cpu-baseline > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench.err
exit $rc

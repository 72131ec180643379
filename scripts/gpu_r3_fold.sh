#!/bin/bash
# folded K3C data gradient: parity (K3C at every config, step tests, determinism), then the bench line
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  -k "proj_conv_matches or full_step or deterministic or config3_step or batch4" tests/test_gpu_fullsize.py tests/test_gpu_parity.py > gpurun_out/fold_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/fold_tests.log | tail -16
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --kernel-table > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c2.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel'],round(d['roofline']['frac'],3))"
grep -E "proj_conv|voxel_project" gpurun_out/bench_c2.err

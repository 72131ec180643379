#!/bin/bash
# per-image K2C data gradient: pad-conv tests, config-3 step test, config-3 bench with and without the split
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 500 --timeout-method thread -p no:cacheprovider \
  -k "pad_conv or config3_step" tests/test_gpu_fullsize.py > gpurun_out/pose2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error" gpurun_out/pose2_tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --config 3 --no-cpu-baseline --no-parity --steps 10 --warmup 3 > gpurun_out/bench_c3_split.json 2> gpurun_out/bench_c3_split.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c3_split.json'));print('c3 split',d['value'],d['ms_per_step'])"
VFD_POSE_DGRAD_SPLIT=0 timeout -k 10 400 python bench.py --config 3 --no-cpu-baseline --no-parity --steps 10 --warmup 3 > gpurun_out/bench_c3_nosplit.json 2> gpurun_out/bench_c3_nosplit.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c3_nosplit.json'));print('c3 no split',d['value'],d['ms_per_step'])"
timeout -k 10 400 python bench.py --config 5 --no-cpu-baseline --no-parity --steps 10 --warmup 3 > gpurun_out/bench_c5_split.json 2> gpurun_out/bench_c5_split.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c5_split.json'));print('c5 split',d['value'],d['ms_per_step'])"
VFD_POSE_DGRAD_SPLIT=0 timeout -k 10 400 python bench.py --config 5 --no-cpu-baseline --no-parity --steps 10 --warmup 3 > gpurun_out/bench_c5_nosplit.json 2> gpurun_out/bench_c5_nosplit.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c5_nosplit.json'));print('c5 no split',d['value'],d['ms_per_step'])"

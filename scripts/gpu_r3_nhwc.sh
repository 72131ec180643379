#!/bin/bash
# channels-last bf16 encoders: NHWC BN / max-pool / encoder tests, then config-3 bench lines with and
# without channels-last, then the steady-state kernel breakdown of the channels-last step
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "channels_last or max_pool or batchnorm_act" tests/test_gpu_fullsize.py > gpurun_out/nhwc_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|fro |vs fp32" gpurun_out/nhwc_tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --config 3 --no-cpu-baseline --no-parity --steps 10 --warmup 3 > gpurun_out/bench_c3_cl.json 2> gpurun_out/bench_c3_cl.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c3_cl.json'));print('c3 channels-last',d['value'],d['ms_per_step'])"
VFD_CHANNELS_LAST=0 timeout -k 10 400 python bench.py --config 3 --no-cpu-baseline --no-parity --steps 10 --warmup 3 > gpurun_out/bench_c3_nchw.json 2> gpurun_out/bench_c3_nchw.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c3_nchw.json'));print('c3 nchw',d['value'],d['ms_per_step'])"
timeout -k 10 400 python bench.py --config 3 --no-cpu-baseline --no-parity --steps 10 --warmup 3 > gpurun_out/bench_c3_cl2.json 2> gpurun_out/bench_c3_cl2.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c3_cl2.json'));print('c3 channels-last again',d['value'],d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_c3_cl -o run --output-format csv -- python bench.py --config 3 --no-cpu-baseline --no-parity --steps 4 --warmup 2 > gpurun_out/prof_c3_cl.log 2>&1 || exit $?
python tools/kernel_breakdown.py $(find gpurun_out/prof_c3_cl -name '*kernel_trace.csv' | head -1) --last 3 --top 70 > gpurun_out/kbd_c3_cl.txt
rm -rf gpurun_out/prof_c3_cl
head -3 gpurun_out/kbd_c3_cl.txt

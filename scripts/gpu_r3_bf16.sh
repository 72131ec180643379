#!/bin/bash
# bf16 kernel tests, config-3 step tests, then a config-3 bench line
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -v --timeout 500 --timeout-method thread -p no:cacheprovider tests/test_gpu_fullsize.py -k "bf16 or config3_step_b2 or batchnorm or elu_upsample or stem_max_pool or reflect_pad" tests/test_gpu_parity.py::test_bf16_nets_step_tracks_fp32 > gpurun_out/gpu_bf16b.log 2>&1
echo "pytest rc=$?"
timeout -k 10 400 python bench.py --config 3 --steps 10 --warmup 4 --no-cpu-baseline --no-parity --kernel-table > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit $?
echo "bench c3 ok"

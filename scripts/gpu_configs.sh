cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit 1
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit 1
timeout -k 10 400 python bench.py --config 5 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || exit 1

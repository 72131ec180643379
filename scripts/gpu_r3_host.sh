#!/bin/bash
# host-boundness of the eager step (config 2) and the graphed step's bench line
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/diag_host.py --config 2 > gpurun_out/diag_host.txt 2>&1 || exit $?
tail -1 gpurun_out/diag_host.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --graph 1 > gpurun_out/bench_c2_graph.json 2> gpurun_out/bench_c2_graph.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_c2_graph.json'));print('graph',d['value'],d['ms_per_step'])"

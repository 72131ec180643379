#!/bin/bash
# whole-step HIP graph replay vs eager on the tuned find-db, configs 2 and 3
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for C in 2 3; do
  timeout -k 10 400 python bench.py --config $C --no-cpu-baseline --no-parity --steps 20 --warmup 5 --graph 1 > gpurun_out/bench_graph_c$C.json 2> gpurun_out/bench_graph_c$C.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bench_graph_c$C.json'));print('config $C graph',d['value'],d['ms_per_step'])"
done

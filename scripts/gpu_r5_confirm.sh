#!/bin/bash
# round 5 close: smoke + the default bench line on the committed tree
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5/confirm
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5/confirm/smoke.log 2>&1 || { tail -5 gpurun_out/r5/confirm/smoke.log; exit 1; }
tail -2 gpurun_out/r5/confirm/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r5/confirm/bench.json 2> gpurun_out/r5/confirm/bench.err || { tail -5 gpurun_out/r5/confirm/bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r5/confirm/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'])"

#!/bin/bash
# round-3 end: the whole -m gpu suite + smoke, then the default bench line and its kernel-trace profile
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash scripts/gpu_alltests.sh
tail -1 gpurun_out/all_tests.log | grep -q "rc=0" || { tail -30 gpurun_out/all_tests.log; exit 1; }
tail -3 gpurun_out/all_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --kernel-table > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel'],round(d['roofline']['frac'],3))"
bash scripts/gpu_profile.sh final || exit 1
head -2 gpurun_out/prof_final/breakdown.txt

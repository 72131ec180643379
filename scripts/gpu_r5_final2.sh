#!/bin/bash
# Round 5 final check (2): the parity file (graph test with its eager reference in the capture's
# configuration), smoke(), the default bench line
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/final2
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_ddp.py tests/test_gpu_0_ddp_world2.py tests/test_gpu_0_bench_world2.py > $OUT/parity.log 2>&1
rc=$?; tail -2 $OUT/parity.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['execution'],d['cpu_baseline']['value'])"

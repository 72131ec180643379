#!/bin/bash
# Round 6 check: the GPU suite (the driver's command), smoke(), the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/${1:-final}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests > $OUT/suite.log 2>&1
rc=$?; tail -3 $OUT/suite.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
python -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel'],r['frac'],r.get('frac_isolated'),d['roofline_aggregate']['frac'],d['execution'],d['cpu_baseline']['value'])"

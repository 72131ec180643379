#!/bin/bash
# Round 5: the whole GPU suite with the pose branch on its own stream by default (DDP tests
# included), then the default bench line
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/aa
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $OUT/suite.log 2>&1
rc=$?; tail -3 $OUT/suite.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['parity'].get('full_resolution'))"

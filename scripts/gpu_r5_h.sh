#!/bin/bash
# Round 5 step H: find-db entries for the fp32 NHWC shapes at batch 12 (the config-3-shape fp32 step
# test), then the -m gpu suite on the new defaults (channels-last fp32 encoders), then the bench.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/h
mkdir -p $OUT
export PYTHONUNBUFFERED=1
true \

mkdir -p $OUT/db && cp miopen_db/* $OUT/db/
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > $OUT/suite.log 2>&1
rc=$?; tail -3 $OUT/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['miopen'],d['encoder_layout'],d['parity']['full_resolution'])"

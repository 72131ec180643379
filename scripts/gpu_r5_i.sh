#!/bin/bash
# Round 5 step I: the parity file on the new defaults (channels-last fp32 encoders), then the bench.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/i
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py > $OUT/parity.log 2>&1
rc=$?; tail -3 $OUT/parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['miopen'],d['encoder_layout'],d['parity']['full_resolution'])"

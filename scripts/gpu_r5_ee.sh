#!/bin/bash
# Round 5 experiment: the depth branch on a high-priority stream (VFD_STREAM_PRIORITY=1): step
# tests with it on, then bench A/B alternating
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/ee
mkdir -p $OUT
export PYTHONUNBUFFERED=1
VFD_STREAM_PRIORITY=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "full_step or full_resolution or deterministic" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc = 0 ] || exit $rc
B="--no-cpu-baseline --no-parity --steps 30 --warmup 5"
pr() { python -c "import json;d=json.load(open('$OUT/$1.json'));print('$1',d['value'],d['ms_per_step'])"; }
for i in 1 2; do
  VFD_STREAM_PRIORITY=1 timeout -k 10 300 python bench.py $B > $OUT/prio$i.json 2> $OUT/prio$i.err && pr prio$i || exit 1
  VFD_STREAM_PRIORITY=0 timeout -k 10 300 python bench.py $B > $OUT/base$i.json 2> $OUT/base$i.err && pr base$i || exit 1
done

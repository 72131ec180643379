#!/bin/bash
# Round 5: the pose branch on a second stream (VFD_BRANCH_STREAMS=1): step parity tests with it on,
# then config-2 bench A/B on one box (alternating)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/z
mkdir -p $OUT
export PYTHONUNBUFFERED=1
VFD_BRANCH_STREAMS=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "full_step or full_resolution or deterministic or graph" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || exit $rc
B="--no-cpu-baseline --no-parity --steps 30 --warmup 5"
pr() { python -c "import json;d=json.load(open('$OUT/$1.json'));print('$1',d['value'],d['ms_per_step'])"; }
for i in 1 2; do
  VFD_BRANCH_STREAMS=1 timeout -k 10 300 python bench.py $B > $OUT/on$i.json 2> $OUT/on$i.err && pr on$i || exit 1
  VFD_BRANCH_STREAMS=0 timeout -k 10 300 python bench.py $B > $OUT/off$i.json 2> $OUT/off$i.err && pr off$i || exit 1
done

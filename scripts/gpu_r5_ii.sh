#!/bin/bash
# Round 5: the fusion plan's readiness as an event (the depth branch's K1 backward no longer waits
# for everything the pose stream queued before it): step tests, then two benches
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/ii
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "full_step or full_resolution or deterministic or graph or fuse" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc = 0 ] || exit $rc
B="--no-cpu-baseline --no-parity --steps 30 --warmup 5"
for i in 1 2 3; do timeout -k 10 300 python bench.py $B > $OUT/b$i.json 2> $OUT/b$i.err || exit 1
python -c "import json;d=json.load(open('$OUT/b$i.json'));print('b$i',d['value'],d['ms_per_step'])"; done

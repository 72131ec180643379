#!/bin/bash
# round 4: whole -m gpu suite, then bench lines at configs 3, 2 and 5 (kernel tables)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4
mkdir -p $OUT
export PYTHONUNBUFFERED=1
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 1500 python -u -m pytest tests -x -v -m gpu --timeout 900 --timeout-method thread > $OUT/suite.log 2>&1
rc=$?; tail -3 $OUT/suite.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/suite.log | head; exit $rc; }
fi
for C in ${CONFIGS:-3 2 5}; do
  ST=20; WU=5; [ $C = 5 ] && { ST=4; WU=2; }
  timeout -k 10 900 python bench.py --config $C --steps $ST --warmup $WU --no-cpu-baseline --no-parity --kernel-table > $OUT/bench_c$C.json 2> $OUT/bench_c$C.err || exit $?
  python -c "import json;d=json.load(open('$OUT/bench_c$C.json'));print('config $C', round(d['value'],3), 'it/s', round(d['ms_per_step'],2), 'ms/step', d['roofline']['kernel'], round(d['roofline']['frac'],3))"
done

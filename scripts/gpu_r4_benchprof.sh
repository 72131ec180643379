#!/bin/bash
# The bench line and its rocprofv3 kernel statistics from ONE run (same box, same tree, same
# process): `scripts/gpu_r4_benchprof.sh TAG [bench args...]` -> gpurun_out/bp_TAG/{bench.json,
# bench.err, stats/, breakdown.txt, roofline_check.json}
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-default}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/bp_$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd /tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
  python $GRAFT_REPO_ROOT/bench.py --kernel-table "$@" > $OUT/bench.json 2> $OUT/bench.err || exit $?
cd $GRAFT_REPO_ROOT
TRACE=$(ls $OUT/stats/*/run_kernel_trace.csv $OUT/stats/run_kernel_trace.csv 2>/dev/null | head -1)
STATS=$(ls $OUT/stats/*/run_kernel_stats.csv $OUT/stats/run_kernel_stats.csv 2>/dev/null | head -1)
python tools/kernel_breakdown.py $TRACE --last 5 --skip ${SKIP_MARKS:-2} --top 70 > $OUT/breakdown.txt   # --skip 1: the parity step after the timed ones
python tools/roofline_check.py $OUT/bench.json $STATS --trace $TRACE > $OUT/roofline_check.json
echo "roofline_check rc=$?"
gzip -f $TRACE
head -3 $OUT/breakdown.txt
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel'],round(d['roofline']['frac'],3))"

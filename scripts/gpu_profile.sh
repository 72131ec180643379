#!/bin/bash
# Kernel-trace profile of the step bench: `scripts/gpu_profile.sh TAG [bench args...]`
# -> gpurun_out/prof_TAG/ (rocprofv3 csv + stats) and gpurun_out/prof_TAG/breakdown.txt
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-default}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-parity "$@" > $OUT/bench.json 2> $OUT/bench.err || exit $?
cd $GRAFT_REPO_ROOT
python tools/kernel_breakdown.py $(ls $OUT/*/*kernel_trace.csv $OUT/*kernel_trace.csv 2>/dev/null | head -1) --last 6 --top 60 > $OUT/breakdown.txt

#!/bin/bash
# Round 5: kernel-name diff of config 2's HIP-graph step against the eager step (verdict: the
# "MIOpen picks different solvers for captured shapes" claim), from one rocprofv3 kernel trace each.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5/graphdiff
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
B="--no-cpu-baseline --no-parity --steps 10 --warmup 3"
cd /tmp
for G in 0 1; do
  timeout -k 10 600 rocprofv3 --kernel-trace -d $OUT/trace_g$G -o run --output-format csv -- \
    python $GRAFT_REPO_ROOT/bench.py $B --graph $G > $OUT/bench_g$G.json 2> $OUT/bench_g$G.err || exit $?
done
cd $GRAFT_REPO_ROOT
TA=$(ls $OUT/trace_g0/*/run_kernel_trace.csv $OUT/trace_g0/run_kernel_trace.csv 2>/dev/null | head -1)
TB=$(ls $OUT/trace_g1/*/run_kernel_trace.csv $OUT/trace_g1/run_kernel_trace.csv 2>/dev/null | head -1)
python tools/kernel_diff.py $TA $TB --skip-a 5 --skip-b 5 > $OUT/kernel_diff.txt
gzip -f $TA $TB
head -40 $OUT/kernel_diff.txt
for G in 0 1; do python -c "import json;d=json.load(open('$OUT/bench_g$G.json'));print('graph=$G',d['value'],d['ms_per_step'])"; done

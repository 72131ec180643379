#!/bin/bash
# Round 6: the DEFAULT step (batched pose pairs + pose branch stream) captured as a HIP graph, plain
# and under DDP (NCCL world 1), stage by stage; then the graph tests; then graph vs eager benches.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6/capture
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/diag_capture.py > $OUT/plain.log 2>&1; rc=$?
echo "plain rc=$rc"; grep "^ok\|segv_bt\|rror" $OUT/plain.log | head -20; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/diag_capture.py --ddp > $OUT/ddp.log 2>&1; rc=$?
echo "ddp rc=$rc"; grep "^ok\|segv_bt\|rror" $OUT/ddp.log | head -20; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_ddp.py -k "graph or ddp" > $OUT/tests.log 2>&1; rc=$?
tail -5 $OUT/tests.log; [ $rc = 0 ] || exit $rc
B="--no-cpu-baseline --no-parity --steps 30 --warmup 5"
for c in 2 3; do
  timeout -k 10 400 python bench.py $B --config $c --graph 1 > $OUT/graph_c$c.json 2> $OUT/graph_c$c.err || exit 1
  timeout -k 10 400 python bench.py $B --config $c > $OUT/eager_c$c.json 2> $OUT/eager_c$c.err || exit 1
done
for f in graph_c2 eager_c2 graph_c3 eager_c3; do python -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',round(d['value'],3),round(d['ms_per_step'],3))"; done

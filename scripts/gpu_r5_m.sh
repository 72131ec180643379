#!/bin/bash
# Round 5: (1) which framework ops launch the remaining transposes / fills / adds / copies of the
# config-2 step on the new defaults; (2) the uninitialised-read tracer on the graph test's config
# (eager step on NaN-poisoned allocator memory, large and small pools)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/m
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/op_attribution.py --top 70 > $OUT/attr.txt 2> $OUT/attr.err || exit 1
head -5 $OUT/attr.txt
timeout -k 10 300 python tools/diag_poison.py --config -1 --pairs 0 > $OUT/poison.txt 2> $OUT/poison.err
rc=$?; echo "poison rc=$rc"; tail -35 $OUT/poison.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/diag_poison.py --config -1 --pairs 1 > $OUT/poison1.txt 2> $OUT/poison1.err
echo "poison1 rc=$?"; tail -35 $OUT/poison1.txt

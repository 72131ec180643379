#!/bin/bash
# Round 5: op attribution of config 2's glue kernels + a plain bench line on the same box.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/${1:-attr}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/op_attribution.py --config 2 --top 150 > $OUT/op_attr_c2.txt 2> $OUT/op_attr_c2.err || exit $?
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
cat $OUT/bench.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['ms_per_step'])"

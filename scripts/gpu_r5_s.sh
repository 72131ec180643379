#!/bin/bash
# Round 5: which round-5 change broke the deterministic-steps test (bisect by switches)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/s
mkdir -p $OUT
export PYTHONUNBUFFERED=1
run() { tag=$1; shift; env "$@" timeout -k 10 200 python tests/det_worker.py > $OUT/$tag.json 2> $OUT/$tag.err;
  echo "$tag rc=$? $(python -c "import json;r=json.loads(open('$OUT/$tag.json').read().strip().splitlines()[-1]);print('grad_diff',len(r['grad_diff']),'depth',r['depth_equal'],'loss',r['loss_diff'],'d_disp',r['d_disp_equal'])" 2>&1 | tail -1)"; }
run base
run pairs0 VFD_POSE_PAIRS=0
run level0 VFD_LEVEL_CONV=0
run fold0 VFD_FOLD_WEIGHTS=0
run all0 VFD_POSE_PAIRS=0 VFD_LEVEL_CONV=0 VFD_FOLD_WEIGHTS=0

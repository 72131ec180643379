#!/bin/bash
# Round 5 final evidence: the default bench line under rocprofv3 (config 2) on the final tree
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_r4_benchprof.sh r5_final || exit 1

#!/bin/bash
# Round 6 final evidence on the final tree: per-op HBM traffic at config 2 (FETCH_SIZE / WRITE_SIZE
# passes), then the default bench line under rocprofv3 with tools/roofline_check.py.
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_traffic_cfg.sh 2 || exit 1
bash scripts/gpu_r4_benchprof.sh r6_final || exit 1

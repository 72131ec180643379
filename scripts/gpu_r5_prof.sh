#!/bin/bash
# Round 5 evidence: the default bench line + rocprofv3 kernel statistics (config 2), the same at
# config 3, and the PMC traffic tables (FETCH_SIZE / WRITE_SIZE passes) at configs 2 and 3
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_r4_benchprof.sh r5_c2 || exit 1
bash scripts/gpu_r4_benchprof.sh r5_c3b --config 3 || exit 1
bash scripts/gpu_traffic_cfg.sh 2 3 || exit 1
ls gpurun_out/traffic_config*.json

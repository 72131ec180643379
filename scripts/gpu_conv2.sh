#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/micro_conv.py > gpurun_out/micro_conv.txt 2>&1 || exit $?
mkdir -p gpurun_out/miopen_db2 && cp miopen_db/*.txt gpurun_out/miopen_db2/
MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db2 timeout -k 10 600 python tools/micro_conv.py --find 1 > gpurun_out/micro_conv_find.txt 2>&1

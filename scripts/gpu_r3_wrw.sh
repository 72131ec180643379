#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/micro_wrw_layout.py --bf16 > gpurun_out/micro_wrw.txt 2>&1; rc=$?
grep -v Warn gpurun_out/micro_wrw.txt | tail -6; exit $rc

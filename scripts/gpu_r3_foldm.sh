#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/micro_projconv.py --config 2 > gpurun_out/micro_fold.txt 2>&1 || exit $?
grep dgrad gpurun_out/micro_fold.txt
VFD_LIB=$GRAFT_REPO_ROOT/variants/libvfd_pf8.so timeout -k 10 300 python -u tools/micro_projconv.py --config 2 > gpurun_out/micro_fold_pf8.txt 2>&1 || exit $?
echo pf8; grep dgrad gpurun_out/micro_fold_pf8.txt

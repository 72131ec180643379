#!/bin/bash
# Round 6: HIP API log (AMD_LOG_LEVEL=3) of the default-step capture, filtered to the capture's
# stream / event calls and the reconstructed fork tree (tools/hiplog_capture.py).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6/capture
AMD_LOG_LEVEL=3 AMD_LOG_MASK=1 AMD_LOG_LEVEL_FILE=/tmp/hiplog.txt timeout -k 10 300 python tools/diag_capture.py ${1:-} > gpurun_out/r6/capture/plain_log${1:-}.log 2>&1
rc=$?
python tools/hiplog_capture.py /tmp/hiplog.txt* > gpurun_out/r6/capture/hiplog_summary${1:-}.txt 2>&1
exit $rc

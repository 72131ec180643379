#!/bin/bash
# pose conv data / weight gradient at config 3's batch: one call vs one call per image
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/micro_poseconv.py --batch 2 > gpurun_out/micro_pose_b2.txt 2>&1; rc=$?
grep -v "Warn\|amdgpu.ids" gpurun_out/micro_pose_b2.txt | tail -20; exit $rc

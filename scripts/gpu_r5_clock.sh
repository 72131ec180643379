#!/bin/bash
# round 5: effective clock of the K3C MFMA kernels (GRBM_GUI_ACTIVE / 8 / kernel duration, one pmc pass)
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5/clock
export PYTHONUNBUFFERED=1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE -d gpurun_out/r5/clock/w -o run --output-format csv \
  -- python3 tools/micro_pcw.py --config 2 --iters 10 > gpurun_out/r5/clock/w.log 2>&1 || { tail -5 gpurun_out/r5/clock/w.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE -d gpurun_out/r5/clock/p -o run --output-format csv \
  -- python3 tools/micro_projconv.py --config 2 --iters 10 > gpurun_out/r5/clock/p.log 2>&1 || { tail -5 gpurun_out/r5/clock/p.log; exit 1; }
python3 tools/clock_from_pmc.py gpurun_out/r5/clock/w gpurun_out/r5/clock/p | tee gpurun_out/r5/clock/summary.txt

#!/bin/bash
# Round-3 diagnostics: the config-5 view test, op attribution of the config-2 step's glue kernels,
# and a kernel-trace breakdown of the config-3 (B=2, bf16) step.  Each step under its own limit.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 560 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_fullsize.py::test_view_synthesis_and_losses_full_size[5]" > gpurun_out/view5.log 2>&1
echo "view5 rc=$?"
timeout -k 10 300 python tools/op_attribution.py --config 2 --top 80 > gpurun_out/op_attr_c2.txt 2>&1 || exit $?
echo "attr ok"
scripts/gpu_profile.sh c3 --config 3 || exit $?
echo "prof c3 ok"

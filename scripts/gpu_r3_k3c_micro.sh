#!/bin/bash
# K3C micro timings (forward / data / weight gradient vs MIOpen) at config 2 under a kernel trace,
# then the K3C parity tests.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof_micro
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_micro -o run --output-format csv -- python -u $R/tools/micro_projconv.py --config 2 > $R/gpurun_out/micro_projconv.txt 2>&1) || exit $?
cat gpurun_out/micro_projconv.txt | grep config
python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/prof_micro/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    n=r['Name']
    if 'pcw' in n or 'pcd' in n or 'pcv' in n or 'wrw' in n:
        print(f"{float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4}  {n[:90]}")
PY
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "proj_conv_matches" tests/test_gpu_fullsize.py > gpurun_out/k3c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/k3c_tests.log
exit $rc

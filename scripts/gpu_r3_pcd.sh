#!/bin/bash
# K3C data-gradient A/B: stream-K ranges (default) vs XCD-strided whole tiles (variant), kernel trace
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for V in base stride; do
  unset VFD_LIB; [ $V = stride ] && export VFD_LIB=$R/variants/libvfd_stride.so
  mkdir -p gpurun_out/prof_$V
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$V -o run --output-format csv -- python -u $R/tools/micro_projconv.py --config 2 > $R/gpurun_out/micro_$V.txt 2>&1) || exit $?
  grep dgrad gpurun_out/micro_$V.txt
  python - $V <<'PY'
import csv,glob,sys
f=glob.glob(f'gpurun_out/prof_{sys.argv[1]}/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    n=r['Name']
    if 'pc' in n and 'vfd' in n:
        print(f"{float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4}  {n[:60]}")
PY
done

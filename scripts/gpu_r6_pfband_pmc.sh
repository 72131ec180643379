#!/bin/bash
# Round 6: FETCH_SIZE of the K3C data gradient (pcdf_main_k) per tile-order variant, one pmc pass each
# over tools/micro_projconv.py (config 2).
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6/pfband_pmc
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for nb in 1 3 25; do
  (cd /tmp && VFD_LIB=$R/variants/libvfd_pfnb$nb.so timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/nb$nb -o run --output-format csv -- python $R/tools/micro_projconv.py --config 2 --iters 5 > $OUT/nb$nb.log 2>&1) || exit 1
  python - $OUT/nb$nb $nb <<'PY'
import csv, glob, sys
f = (glob.glob(sys.argv[1] + '/*/*counter_collection.csv') + glob.glob(sys.argv[1] + '/*counter_collection.csv'))[0]
v = [float(r['Counter_Value']) for r in csv.DictReader(open(f)) if 'pcdf_main_k' in r['Kernel_Name']]
print(f'nband {sys.argv[2]}: pcdf_main_k {len(v)} dispatches, FETCH_SIZE x2 per launch {2 * sum(v) / len(v) * 1024 / 1e9:.3f} GB')
PY
  rm -rf $OUT/nb$nb
done

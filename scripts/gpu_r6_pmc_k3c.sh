#!/bin/bash
# Round 6: one SQ counter pass over the K3C kernels (tools/micro_projconv.py, config 2): MFMA busy,
# wave stall buckets, LDS conflicts — where the data gradient's cycles go against the forward's and
# the weight gradient's.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6/pmc_k3c
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $OUT/p1 -o run --output-format csv -- python $R/tools/micro_projconv.py --config 2 --iters 5 > $OUT/p1.log 2>&1) || exit 1
python - $OUT/p1 <<'PY' | tee $OUT/summary.txt
import csv, glob, sys, collections
f = (glob.glob(sys.argv[1] + '/*/*counter_collection.csv') + glob.glob(sys.argv[1] + '/*counter_collection.csv'))[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name']
    if any(s in k for s in ('pcdf_main_k', 'pcv_main_k', 'pcw_main_k')):
        agg[k[:40]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f'   {c:28s} mean {sum(v) / len(v):18.1f}  n {len(v)}')
PY
rm -rf $OUT/p1

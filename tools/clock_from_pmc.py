"""Effective shader clock per kernel from a `rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE` run:
GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 / the dispatch's duration (MI355X_MICROARCH.md,
DVFS give-back).  Prints per kernel name: dispatches, mean duration, mean effective clock.

    python tools/clock_from_pmc.py DIR [DIR ...]     (DIR: rocprofv3 -d output, csv format)"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    cc = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    kt = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)
    dur = {}
    for f in kt:
        for r in csv.DictReader(open(f)):
            dur[r['Correlation_Id']] = (r['Kernel_Name'], int(r['End_Timestamp']) - int(r['Start_Timestamp']))
    out = defaultdict(list)
    for f in cc:
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] != 'GRBM_GUI_ACTIVE':
                continue
            cid = r['Correlation_Id']
            if cid not in dur:
                continue
            name, ns = dur[cid]
            out[name].append((ns, float(r['Counter_Value'])))
    return out


def main():
    rows = defaultdict(list)
    for d in sys.argv[1:]:
        for k, v in load(d).items():
            rows[k] += v
    for name, v in sorted(rows.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
        ns = sum(x[0] for x in v) / len(v)
        if ns < 300e3:          # the quotient reads high below ~0.3 ms
            continue
        ghz = sum(c / 8 / t for t, c in v) / len(v)
        print(f'{name[:70]:70s} n={len(v):3d} {ns / 1e3:9.1f} us  clock {ghz:.3f} GHz')


if __name__ == '__main__':
    main()

"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel (mean per dispatch).

    python tools/pmc_kernels.py <dir> [substring ...]
"""
import collections
import csv
import glob
import sys


def main():
    d, subs = sys.argv[1], sys.argv[2:]
    files = glob.glob(f'{d}/**/*counter_collection.csv', recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name']
            if subs and not any(s in k for s in subs):
                continue
            agg[k[:60]][r['Counter_Name']].append(float(r['Counter_Value']))
    for k, cs in agg.items():
        print(k)
        for c, v in sorted(cs.items()):
            # one row per dispatch per counter (summed over instances by rocprofv3)
            print(f'   {c:28s} mean {sum(v) / len(v):16.1f}  n {len(v)}')


if __name__ == '__main__':
    main()

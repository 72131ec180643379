"""Summarise rocprofv3 PMC / kernel-trace CSVs under a directory: mean per kernel (short name)."""
import collections
import csv
import glob
import sys


def short(name):
    n = name.split('(')[0]
    return n.replace('void ', '').split('<')[0][-40:]


def main(root):
    for path in sorted(glob.glob(f'{root}/**/*counter_collection.csv', recursive=True)):
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(path)):
            agg[short(r['Kernel_Name'])][r['Counter_Name']].append(float(r['Counter_Value']))
        print('==', path)
        for k, cs in agg.items():
            print(f'  {k:40s} ' + '  '.join(f'{c}={sum(v) / len(v):.4g}' for c, v in sorted(cs.items())))
    for path in sorted(glob.glob(f'{root}/**/*kernel_stats.csv', recursive=True)):
        print('==', path)
        for r in csv.DictReader(open(path)):
            print(f"  {short(r['Name']):40s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs']) / 1e3:9.1f}")


if __name__ == '__main__':
    main(sys.argv[1])

"""Print the top kernels of a rocprofv3 --stats CSV: python tools/kstat_top.py DIR [N]."""
import csv
import glob
import sys

path = glob.glob(f'{sys.argv[1]}/**/*kernel_stats.csv', recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
for r in list(csv.DictReader(open(path)))[:n]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e3:9.1f} us {float(r['Percentage']):6.2f}%")

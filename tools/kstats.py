"""Print the rocprofv3 kernel stats CSV (gpurun_out/tm by default) as a short table."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/tm/run_kernel_stats.csv'
for r in list(csv.DictReader(open(path)))[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{r['Name'][:72]:72s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e3:9.1f} us")

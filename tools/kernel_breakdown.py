"""Steady-state per-step kernel breakdown from a rocprofv3 --kernel-trace CSV.

    python tools/kernel_breakdown.py <kernel_trace.csv> [--marker mask_downsample_k] [--last 5]

Steps are delimited by the launches of a once-per-step marker kernel; the last N complete steps
are aggregated by kernel name (first-step MIOpen find/compile noise excluded)."""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('csv')
    ap.add_argument('--marker', default='mask_downsample_k')
    ap.add_argument('--last', type=int, default=5)
    ap.add_argument('--top', type=int, default=40)
    ap.add_argument('--skip', type=int, default=0, help='ignore the last N marker launches (the bench\'s parity step)')
    a = ap.parse_args()
    import gzip
    rows = list(csv.DictReader(gzip.open(a.csv, 'rt') if a.csv.endswith('.gz') else open(a.csv)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    marks = [i for i, r in enumerate(rows) if a.marker in r['Kernel_Name']]
    marks = marks[:len(marks) - a.skip] if a.skip else marks
    if len(marks) < a.last + 1:
        raise SystemExit(f'only {len(marks)} marker launches')
    lo, hi = marks[-a.last - 1], marks[-1]
    sel = rows[lo:hi]
    span = (int(rows[hi]['Start_Timestamp']) - int(rows[lo]['Start_Timestamp'])) / 1e6 / a.last
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in sel:
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        k = r['Kernel_Name']
        agg[k][0] += 1
        agg[k][1] += d
    busy = sum(v[1] for v in agg.values()) / 1e3 / a.last
    print(f'steps {a.last}: wall {span:.2f} ms/step, kernel busy {busy:.2f} ms/step, '
          f'{len(sel) / a.last:.0f} launches/step')
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f'{t / 1e3 / a.last:8.3f} ms/step {n // a.last:5d}x {t / n:9.1f} us  {k[:120]}')


if __name__ == '__main__':
    main()

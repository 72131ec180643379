"""Per-step kernel-name diff of two rocprofv3 --kernel-trace CSVs of the same step (e.g. the eager
bench and the HIP-graph bench): which kernels one run launches that the other does not, and the
per-step time of each, over the last N complete steps (delimited by a once-per-step marker kernel).

    python tools/kernel_diff.py eager_trace.csv[.gz] graph_trace.csv[.gz] [--last 5] [--skip-a 1] [--skip-b 1]
"""
import argparse
import collections
import csv
import gzip
import re


def per_step(path, marker, last, skip):
    rows = list(csv.DictReader(gzip.open(path, 'rt') if path.endswith('.gz') else open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    marks = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
    marks = marks[:len(marks) - skip] if skip else marks
    if len(marks) < last + 1:
        raise SystemExit(f'{path}: only {len(marks)} marker launches')
    lo, hi = marks[-last - 1], marks[-1]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in rows[lo:hi]:
        # one family per MIOpen solver kernel: drop template / argument lists
        name = re.sub(r'\(.*', '', r['Kernel_Name'])[:110]
        agg[name][0] += 1
        agg[name][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    span = (int(rows[hi]['Start_Timestamp']) - int(rows[lo]['Start_Timestamp'])) / 1e6 / last
    return {k: (n / last, t / last) for k, (n, t) in agg.items()}, span


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('a')
    ap.add_argument('b')
    ap.add_argument('--marker', default='mask_downsample_k')
    ap.add_argument('--last', type=int, default=5)
    ap.add_argument('--skip-a', type=int, default=0)
    ap.add_argument('--skip-b', type=int, default=0)
    ap.add_argument('--labels', default='eager,graph')
    x = ap.parse_args()
    la, lb = x.labels.split(',')
    A, sa = per_step(x.a, x.marker, x.last, x.skip_a)
    B, sb = per_step(x.b, x.marker, x.last, x.skip_b)
    ta, tb = sum(t for _, t in A.values()) / 1e3, sum(t for _, t in B.values()) / 1e3
    print(f'{la}: {sum(n for n, _ in A.values()):.0f} launches/step, kernel time {ta:.3f} ms/step, span {sa:.3f} ms/step')
    print(f'{lb}: {sum(n for n, _ in B.values()):.0f} launches/step, kernel time {tb:.3f} ms/step, span {sb:.3f} ms/step')
    rows = []
    for k in set(A) | set(B):
        na, ta_ = A.get(k, (0, 0.0))
        nb, tb_ = B.get(k, (0, 0.0))
        if abs(na - nb) > 0.01 or abs(ta_ - tb_) > 20.0:
            rows.append((tb_ - ta_, k, na, ta_, nb, tb_))
    rows.sort(key=lambda r: -abs(r[0]))
    print(f'{"d us/step":>10s} {la + " n":>8s} {la + " us":>10s} {lb + " n":>8s} {lb + " us":>10s}  kernel')
    for d, k, na, ta_, nb, tb_ in rows:
        print(f'{d:10.1f} {na:8.1f} {ta_:10.1f} {nb:8.1f} {tb_:10.1f}  {k}')


if __name__ == '__main__':
    main()

"""Recompute the bench line's roofline fraction from a rocprofv3 kernel-stats CSV of the SAME run.

    python tools/roofline_check.py <bench.json> <kernel_stats.csv> [--trace <kernel_trace.csv>]

The bench line's `roofline.avg_launch_us` is the HIP-event time of one op call (all of its
launches: main kernel + reduce); here the same op's time is rebuilt from rocprof's per-kernel
averages (sum over the op's kernels of calls-per-op x average duration) and, with --trace, from the
last --prof-calls calls of each kernel only (the bench's profiled steps are its last steady steps).  Prints
both fractions and their ratio; exit 1 if they differ by more than 2 %."""
import argparse
import csv
import gzip
import json
import sys

# op -> kernel-name prefixes of its launches (C-ABI scopes in csrc/*.hip)
OP_KERNELS = {
    'proj_conv_fwd': ('vfd::pcv_main_k', 'vfd::pcvb_main_k', 'void vfd::pcv_reduce_k'),
    'proj_conv_dgrad': ('vfd::pcdf_main_k', 'vfd::pcdf_reduce_k', 'vfd::pcd_main_k', 'vfd::pcd_reduce_k',
                        'vfd::pct_main_k', 'vfd::pct_reduce_k'),
    'proj_conv_wgrad': ('vfd::pcw_main_k', 'vfd::pcw_reduce_k', 'vfd::pcw_bias_k', 'vfd::pcw_bias_fin_k'),
    'pad_conv_fwd': ('vfd::ppc_main_k', 'vfd::ppcb_main_k', 'void vfd::ppc_reduce_k', '_ZN3vfd11ppcb_main_k'),
    'pad_conv_dgrad': ('_ZN3vfd10ppd_main_k', 'vfd::ppd_reduce_k'),
    'fuse_pose_fwd': ('void vfd::fuse_pose_fwd_k',),
    'voxel_project_bwd': ('void vfd::vpb_main_k', 'vfd::vpb_fold_k', 'vfd::vpb_split_k'),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('bench')
    ap.add_argument('stats')
    ap.add_argument('--trace', default=None)
    ap.add_argument('--key', default='roofline')
    ap.add_argument('--prof-calls', type=int, default=5, help="op calls in the bench's profiled steps")
    a = ap.parse_args()
    line = None
    with open(a.bench) as fh:
        for l in fh:
            l = l.strip()
            if l.startswith('{'):
                line = json.loads(l)
    if line is None:
        raise SystemExit('no JSON line in ' + a.bench)
    r = line[a.key]
    op, launches = r['kernel'], r['launches']
    prefixes = OP_KERNELS.get(op)
    if prefixes is None:
        raise SystemExit(f'no kernel map for {op}')
    rows = list(csv.DictReader(open(a.stats)))
    # kernels of the op that ran at least once per profiled call (a kernel of another form of the
    # op, e.g. the parity step's small shape, is not part of the measured calls)
    mine = [x for x in rows if x['Name'].startswith(prefixes) and int(x['Calls']) >= launches]
    if not mine:
        raise SystemExit(f'no kernel of {op} in {a.stats}')
    # every kernel of the op runs once per op call (reduce kernels included), so per-call time =
    # sum of the kernels' average durations
    per_call_avg = sum(float(x['AverageNs']) for x in mine) / 1e3
    per_call_min = sum(float(x['MinNs']) for x in mine) / 1e3
    work = r['achieved'] * r['avg_launch_us']            # TFLOP/s x us (or GB/s x us): per-call work
    out = {'op': op, 'bench_avg_launch_us': r['avg_launch_us'], 'bench_frac': r['frac'],
           'rocprof_kernels': {x['Name'][:60]: {'calls': int(x['Calls']), 'avg_us': float(x['AverageNs']) / 1e3,
                                                'min_us': float(x['MinNs']) / 1e3} for x in mine},
           'rocprof_per_call_avg_us': per_call_avg, 'rocprof_frac_avg': work / per_call_avg / r['peak'],
           'rocprof_per_call_min_us': per_call_min}
    if a.trace:
        names = {x['Name'] for x in mine}
        fh = gzip.open(a.trace, 'rt') if a.trace.endswith('.gz') else open(a.trace)
        tr = [x for x in csv.DictReader(fh) if x['Kernel_Name'] in names]
        by = {}
        for x in sorted(tr, key=lambda x: int(x['Start_Timestamp'])):
            by.setdefault(x['Kernel_Name'], []).append((int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e3)
        tail = {k: v[-a.prof_calls:] for k, v in by.items()}
        per_call_tail = sum(sum(v) / len(v) for v in tail.values())
        out['rocprof_last_calls'] = a.prof_calls
        out['rocprof_per_call_last_us'] = per_call_tail
        out['rocprof_frac_last'] = work / per_call_tail / r['peak']
    ref = out.get('rocprof_frac_last', out['rocprof_frac_avg'])
    out['ratio_bench_over_rocprof'] = r['frac'] / ref
    print(json.dumps(out, indent=1))
    return 0 if abs(out['ratio_bench_over_rocprof'] - 1) <= 0.02 else 1


if __name__ == '__main__':
    sys.exit(main())

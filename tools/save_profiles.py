"""Copy a gpu_measure.sh run (gpurun_out/measure) into the tracked profiles/<tag>/ directory.

    python tools/save_profiles.py r1
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, 'gpurun_out', 'measure')


def main(tag):
    dst = os.path.join(ROOT, 'profiles', tag)
    os.makedirs(dst, exist_ok=True)
    copies = {'bench.json': 'bench.json', 'bench_graph.json': 'bench_graph.json', 'gpu_tests.log': 'gpu_tests.log',
              'smoke.log': 'smoke.log', 'stats/bench_kernel_stats.csv': 'rocprof_kernel_stats.csv'}
    for s, d in copies.items():
        p = os.path.join(SRC, s)
        if os.path.isfile(p):
            shutil.copy(p, os.path.join(dst, d))
    err = os.path.join(SRC, 'bench.err')
    if os.path.isfile(err):
        with open(err) as fh, open(os.path.join(dst, 'bench_kernel_table.txt'), 'w') as out:
            out.writelines(l for l in fh if l.startswith('[bench]'))
    trace = os.path.join(SRC, 'stats', 'bench_kernel_trace.csv')
    if os.path.isfile(trace):
        with open(os.path.join(dst, 'step_breakdown.txt'), 'w') as out:
            subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'kernel_breakdown.py'), trace],
                           stdout=out, check=False)
    f = os.path.join(SRC, 'pmc_fetch', 'bench_counter_collection.csv')
    w = os.path.join(SRC, 'pmc_write', 'bench_counter_collection.csv')
    if os.path.isfile(f) and os.path.isfile(w):
        with open(os.path.join(ROOT, 'profiles', 'traffic_config2.json'), 'w') as out:
            subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'traffic_from_pmc.py'), f, w], stdout=out,
                           check=True)
    print('saved to', dst)


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'r1')

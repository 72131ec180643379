"""Which aten ops (and shapes) spend the step's device time: torch.profiler over a few eager bench
steps at config 2, grouped by op + input shapes, sorted by device time.

    python tools/diag_ops.py [--steps 3] [--top 70] > ops.txt
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.path.isdir(os.path.join(ROOT, 'miopen_db')):
    sys.path.insert(0, ROOT)
    from vfdepth_amd.miopen_db import use_private_copy  # noqa: E402
    use_private_copy()

import torch  # noqa: E402


def main():
    import bench
    from vfdepth_amd import _lib, synth
    from vfdepth_amd.vfdepth import VFDepthAlgo
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--top', type=int, default=70)
    ap.add_argument('--config', type=int, default=2)
    ap.add_argument('--stacks', default='', help='comma-separated aten ops to attribute by Python stack')
    ap.add_argument('--ops', default='', help='comma-separated aten ops to list by input shapes')
    a = ap.parse_args()
    torch.cuda.set_device(0)
    _lib.load()
    cfg, _ = bench.make_cfg(a.config, None)
    algo = VFDepthAlgo(cfg, 0)
    for m in algo.models.values():
        m.load_state_dict(bench.seeded_state_dict(m, seed=7))
    algo.set_train()
    batch = synth.make_batch(cfg, seed=1234, device='cuda:0')
    for _ in range(3):
        algo.train_step(dict(batch))
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=True, with_stack=bool(a.stacks)) as prof:
        for _ in range(a.steps):
            algo.train_step(dict(batch))
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_input_shape=True)
    print(ka.table(sort_by='self_cuda_time_total', row_limit=a.top, max_name_column_width=40,
                   max_shapes_column_width=90))
    print(prof.key_averages().table(sort_by='self_cuda_time_total', row_limit=40, max_name_column_width=50))
    if a.ops:
        want = set(a.ops.split(','))
        rows = [e for e in ka if e.key in want]
        rows.sort(key=lambda e: -e.self_device_time_total)
        for e in rows[:80]:
            print(f'{e.key:22s} calls {e.count / a.steps:6.1f}/step  dev {e.self_device_time_total / a.steps / 1e3:7.3f} '
                  f'ms/step  {str(e.input_shapes)[:160]}')
    if a.stacks:
        want = set(a.stacks.split(','))
        rows = [e for e in prof.key_averages(group_by_stack_n=8) if e.key in want]
        rows.sort(key=lambda e: -e.count)
        for e in rows[:60]:
            stack = ' <- '.join(s for s in e.stack if 'vfdepth_amd' in s or 'bench' in s)[:400]
            print(f'{e.key:22s} calls {e.count // a.steps:5d}/step  cpu {e.self_cpu_time_total / a.steps / 1e3:7.3f} ms/step  {stack}')


if __name__ == '__main__':
    main()

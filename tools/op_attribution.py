"""Which framework op launches each GPU kernel of a training step (torch.profiler on the GPU box).

Groups the device time of one eager config-2 step by (kernel name pattern, launching aten op,
input shapes), so MIOpen's layout transposes / zero fills / residual adds can be traced to the
convolutions and autograd nodes that cause them.

    python tools/op_attribution.py [--config 2] [--top 60] [--match transpose,SubTensor,add,copy]
"""
import argparse
import collections
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
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.vfdepth import VFDepthAlgo
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', type=int, default=2)
    ap.add_argument('--top', type=int, default=60)
    ap.add_argument('--match', default='transpose,SubTensor,add,copy,Fill,reduce')
    ap.add_argument('--autotune', type=int, default=1, help='MIOpen benchmark mode, as bench.py defaults')
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = bool(a.autotune)
    _lib.load()
    cfg, name = bench.make_cfg(a.config)
    algo = VFDepthAlgo(cfg, 0)
    for m in algo.models.values():
        m.load_state_dict(seeded_state_dict(m, seed=7))
    algo.set_train()
    batch = synth.make_batch(cfg, seed=1234, device='cuda:0')
    for _ in range(4):
        algo.train_step(dict(batch))
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        algo.train_step(dict(batch))
        torch.cuda.synchronize()
    events = prof.events()
    # every device kernel is attached (by correlation id) to the CPU op that launched it
    rows = collections.defaultdict(lambda: [0, 0.0])
    pats = [p for p in a.match.split(',') if p]
    total = 0.0
    for e in events:
        for k in getattr(e, 'kernels', []) or []:
            dur = float(getattr(k, 'duration', 0.0))
            total += dur
            if pats and not any(p in k.name for p in pats):
                continue
            names, shapes, p = [], '', e
            while p is not None and len(names) < 5:
                names.append(p.name)
                if not shapes and p.input_shapes:
                    shapes = str([tuple(s) for s in p.input_shapes if s][:3])
                p = p.cpu_parent
            key = (k.name[:70], ' < '.join(names[:4]), shapes[:90])
            rows[key][0] += 1
            rows[key][1] += dur
    print(f'{name}: step device time {total / 1e3:.2f} ms (all kernels)')
    for (k, chain, shp), (n, t) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f'{t / 1e3:7.3f} ms {n:4d}x  {k:70s} | {chain} | {shp}')


if __name__ == '__main__':
    main()

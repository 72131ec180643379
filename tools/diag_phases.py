"""Where a config-2 training step spends its wall time with the pose branch on its own stream:
HIP events on the two streams at the phase boundaries (fork, each branch's forward done, join,
losses done, each stream's backward done, optimizer done), averaged over steps.

    python tools/diag_phases.py [--config 2] [--steps 10]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vfdepth_amd.miopen_db import use_private_copy  # noqa: E402
use_private_copy()

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', type=int, default=2)
    ap.add_argument('--steps', type=int, default=10)
    a = ap.parse_args()
    import bench
    from vfdepth_amd import _lib, synth
    from vfdepth_amd import vfdepth as VD
    from vfdepth_amd.layers import seeded_state_dict
    torch.backends.cudnn.benchmark = True
    _lib.load()
    cfg, name = bench.make_cfg(a.config)
    algo = VD.VFDepthAlgo(cfg, 0)
    for m in algo.models.values():
        m.load_state_dict(seeded_state_dict(m, seed=7))
    algo.set_train()
    batch = synth.make_batch(cfg, seed=1234, device='cuda:0')
    marks = {}

    def mark(tag, stream):
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        marks.setdefault(tag, []).append(e)

    orig_pose, orig_depth = algo.predict_pose, algo.predict_depth

    def predict_pose(inputs):
        st = torch.cuda.current_stream()
        mark('pose fwd start', st)
        out = orig_pose(inputs)
        mark('pose fwd done', st)
        return out

    def predict_depth(inputs):
        st = torch.cuda.current_stream()
        mark('depth fwd start', st)
        out = orig_depth(inputs)
        mark('depth fwd done', st)
        return out
    algo.predict_pose, algo.predict_depth = predict_pose, predict_depth
    host = {'forward issue': 0.0, 'backward issue': 0.0, 'optimizer issue': 0.0}
    for i in range(3 + a.steps):
        if i == 3:
            marks.clear()
            for k in host:
                host[k] = 0.0
        torch.cuda.synchronize()
        main = torch.cuda.current_stream()
        mark('step start', main)
        t0 = time.perf_counter()
        algo.optimizer.zero_grad(set_to_none=True)
        _, losses = algo.process_batch(dict(batch), 0)
        t1 = time.perf_counter()
        mark('losses done (main)', main)
        losses['total_loss'].backward()
        t2 = time.perf_counter()
        if getattr(algo, '_bstream', None) is not None:
            mark('backward done (side)', algo._bstream)
        mark('backward done (main, joined)', main)
        algo.optimizer.step()
        t3 = time.perf_counter()
        mark('step end', main)
        host['forward issue'] += (t1 - t0) * 1e3
        host['backward issue'] += (t2 - t1) * 1e3
        host['optimizer issue'] += (t3 - t2) * 1e3
    torch.cuda.synchronize()
    n = len(marks['step start'])
    print(f'{name}: {n} steps, branch stream {"on" if getattr(algo, "_bstream", None) is not None else "off"}')
    for k, v in host.items():
        print(f'  host {k:27s} {v / n:8.2f} ms per step (host time to issue, GPU idle at the start)')
    for tag in marks:
        if tag == 'step start':
            continue
        t = sum(marks['step start'][k].elapsed_time(marks[tag][k]) for k in range(n)) / n
        print(f'  {tag:32s} {t:8.2f} ms after step start')


if __name__ == '__main__':
    main()

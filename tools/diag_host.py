"""Is the eager step host-bound?  Times, per step, the host's enqueue time (step() returns, no
sync) against the synchronised step time, and the device-idle gaps (kernel-free time) measured
by events at both ends of a step.

    python tools/diag_host.py [--config 2] [--steps 10]
"""
import argparse
import os
import sys
import time

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
    ap.add_argument('--config', type=int, default=2)
    ap.add_argument('--steps', type=int, default=10)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    _lib.load()
    cfg, name = bench.make_cfg(a.config, None)
    cfg['ddp'].update({'ddp_enable': False, 'world_size': 1, 'gpus': [0]})
    torch.manual_seed(42)
    algo = VFDepthAlgo(cfg, 0)
    for m in algo.models.values():
        m.load_state_dict(bench.seeded_state_dict(m, seed=7))
    algo.set_train()
    batch = synth.make_batch(cfg, seed=1234, device='cuda:0')
    for _ in range(4):
        algo.train_step(dict(batch))
    torch.cuda.synchronize()
    enq, tot = [], []
    for _ in range(a.steps):
        t0 = time.perf_counter()
        algo.train_step(dict(batch))
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        enq.append(t1 - t0)
        tot.append(t2 - t0)
    # back-to-back steps (as the bench times them)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        algo.train_step(dict(batch))
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    ms = lambda v: 1e3 * sum(v) / len(v)  # noqa: E731
    print(f'{name}: isolated step: host enqueue {ms(enq):.2f} ms, enqueue + drain {ms(tot):.2f} ms; '
          f'back-to-back: enqueue {1e3 * (t1 - t0) / a.steps:.2f} ms/step, wall {1e3 * (t2 - t0) / a.steps:.2f} ms/step',
          flush=True)


if __name__ == '__main__':
    main()

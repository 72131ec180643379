"""Time the two reduce_dim convolutions (config 2) in NCHW vs channels-last, fwd + bwd.

    python tools/micro_conv.py [--find 1]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if os.path.isdir(os.path.join(ROOT, 'miopen_db')):
    sys.path.insert(0, ROOT)
    from vfdepth_amd.miopen_db import use_private_copy  # noqa: E402
    use_private_copy()

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def bench(x, w, stride, iters=10):
    x = x.detach().requires_grad_(True)
    w = w.detach().requires_grad_(True)
    for _ in range(3):
        y = F.conv2d(x, w, stride=stride)
        y.backward(torch.ones_like(y))
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf = tb = 0.0
    for _ in range(iters):
        ev[0].record()
        y = F.conv2d(x, w, stride=stride)
        ev[1].record()
        y.backward(torch.ones_like(y))
        ev[2].record()
        torch.cuda.synchronize()
        tf += ev[0].elapsed_time(ev[1])
        tb += ev[1].elapsed_time(ev[2])
    return tf / iters, tb / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--find', type=int, default=0)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = bool(a.find)
    dev = 'cuda'
    cases = [('depth reduce 3200->256 s1', (6, 3200, 50, 82), (256, 3200, 3, 3), 1),
             ('pose reduce 5140->256 s2', (1, 5140, 102, 102), (256, 5140, 3, 3), 2)]
    for name, xs, ws, st in cases:
        x = torch.randn(xs, device=dev)
        w = torch.randn(ws, device=dev) * 0.01
        t0 = time.time()
        f, b = bench(x, w, st)
        print(f'{name:28s} NCHW          fwd {f:7.3f} ms  bwd {b:7.3f} ms  ({time.time() - t0:.0f} s)', flush=True)
        t0 = time.time()
        f, b = bench(x.to(memory_format=torch.channels_last), w.to(memory_format=torch.channels_last), st)
        print(f'{name:28s} channels_last fwd {f:7.3f} ms  bwd {b:7.3f} ms  ({time.time() - t0:.0f} s)', flush=True)


if __name__ == '__main__':
    main()

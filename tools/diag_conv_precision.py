"""Relative error of MIOpen's fp32 convolution passes (forward, data gradient, weight gradient)
against an fp64 evaluation of the same conv on the GPU (ATen's im2col + dgemm path), for the
step's dense convs around K3C: reduce_dim[3] (256 -> 128, 3x3 on the padded K3C output) and a
decoder conv.  Prints one line per (shape, pass, layout, autotune mode).

    python tools/diag_conv_precision.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vfdepth_amd.miopen_db import use_private_copy  # noqa: E402
use_private_copy()

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

SHAPES = {   # name: (N, Cin, H, W (input incl. padding), Cout)
    'reduce_dim3': (6, 256, 98, 162, 128),
    'dec_96x160': (6, 128, 98, 162, 64),
}


def rel(a, b):
    return float((a.double() - b).norm() / b.norm())


def main():
    dev = torch.device('cuda:0')
    g = torch.Generator(device=dev).manual_seed(0)
    for name, (N, C, H, W, O) in SHAPES.items():
        x = torch.randn(N, C, H, W, device=dev, generator=g)
        w = torch.randn(O, C, 3, 3, device=dev, generator=g) / (9 * C) ** 0.5
        b = torch.randn(O, device=dev, generator=g)
        gy = torch.randn(N, O, H - 2, W - 2, device=dev, generator=g)
        xd, wd, gd = x.double().requires_grad_(True), w.double().requires_grad_(True), gy.double()
        yd = F.conv2d(xd, wd, b.double())
        yd.backward(gd)
        for bench_mode in (False, True):
            torch.backends.cudnn.benchmark = bench_mode
            for cl in (False, True):
                mf = torch.channels_last if cl else torch.contiguous_format
                xs = x.detach().contiguous(memory_format=mf).requires_grad_(True)
                ws = w.detach().contiguous(memory_format=mf).requires_grad_(True)
                y = F.conv2d(xs, ws, b)
                y.backward(gy.contiguous(memory_format=mf))
                torch.cuda.synchronize()
                print(f'{name} benchmark={int(bench_mode)} channels_last={int(cl)}: fwd {rel(y, yd.detach()):.2e} '
                      f'dgrad {rel(xs.grad, xd.grad):.2e} wgrad {rel(ws.grad, wd.grad):.2e}', flush=True)


if __name__ == '__main__':
    main()

"""K2C (pose reduce_dim's first conv) vs MIOpen at config 2: C = 5140, 102x102 padded, stride 2.

    python tools/micro_padconv.py [--iters 10]
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
import torch.nn.functional as F  # noqa: E402

from micro_projconv import timed  # noqa: E402


def main():
    from vfdepth_amd import _lib
    from vfdepth_amd import kernels as KN
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=10)
    a = ap.parse_args()
    _lib.load()
    dev = torch.device('cuda:0')
    C, H, W, s, O = 5140, 102, 102, 2, 256
    x = torch.randn(1, C, H, W, device=dev).contiguous(memory_format=torch.channels_last)
    w = torch.randn(O, C, 3, 3, device=dev) * (C * 9) ** -0.5
    b = 0.1 * torch.randn(O, device=dev)
    flop = 2.0 * 50 * 50 * O * C * 9
    with torch.no_grad():
        t_k = timed(lambda: KN.PadConv.apply(x, w, b, s), a.iters)
        t_m = timed(lambda: F.pad(F.leaky_relu(F.conv2d(x, w, b, stride=s), 0.1), (1, 1, 1, 1), mode='reflect'),
                    a.iters)
        _lib.prof_enable('pad_conv_fwd')
        for _ in range(a.iters):
            KN.PadConv.apply(x, w, b, s)
        torch.cuda.synchronize()
        n, ms = _lib.prof_read().get('pad_conv_fwd', (1, float('nan')))
        _lib.prof_enable('off')
        y = KN.PadConv.apply(x, w, b, s)
        ref = F.pad(F.leaky_relu(F.conv2d(x, w, b, stride=s), 0.1), (1, 1, 1, 1), mode='reflect')
        err = float((y - ref).abs().max() / ref.abs().max())
    print(f'K2C {t_k:.3f} ms (kernel {ms / n:.3f} ms, {flop / (ms / n) / 1e9:.1f} TFLOP/s, weight copy incl. in '
          f'the first); MIOpen conv + lrelu + pad {t_m:.3f} ms; max rel err {err:.2e}', flush=True)


if __name__ == '__main__':
    main()

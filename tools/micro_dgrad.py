"""reduce_dim (config 2, depth: 3200->256 3x3, NHWC) input-gradient: MIOpen's backward-data
(what autograd runs) vs the same product as a forward conv with transposed, flipped weights
(dX = conv2d(dY, W^T flipped, padding=2)).  Also the bf16 forward/backward for config 3.

    python tools/micro_dgrad.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if os.path.isdir(os.path.join(ROOT, 'miopen_db')):
    sys.path.insert(0, ROOT)
    from vfdepth_amd.miopen_db import use_private_copy  # noqa: E402
    use_private_copy()

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def timed(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    cl = torch.channels_last
    for dt in (torch.float32, torch.bfloat16):
        x = torch.randn(6, 3200, 50, 82, device='cuda', dtype=dt).to(memory_format=cl)
        w = (torch.randn(256, 3200, 3, 3, device='cuda', dtype=dt) * 0.01).to(memory_format=cl)
        dy = torch.randn(6, 256, 48, 80, device='cuda', dtype=dt).to(memory_format=cl)
        wt = w.transpose(0, 1).flip(2, 3).contiguous(memory_format=cl)
        fl = 2 * 6 * 48 * 80 * 3200 * 256 * 9
        t_f = timed(lambda: F.conv2d(x, w))
        t_bd = timed(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [0, 0], [1, 1], False,
                                                                  [0, 0], 1, [True, False, False]))
        t_bw = timed(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [0, 0], [1, 1], False,
                                                                  [0, 0], 1, [False, True, False]))
        t_alt = timed(lambda: F.conv2d(dy, wt, padding=2))
        ref = torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                                  [True, False, False])[0]
        alt = F.conv2d(dy, wt, padding=2)
        err = float((ref.float() - alt.float()).abs().max() / ref.float().abs().max())
        print(f'{dt}: fwd {t_f:.3f} ms ({fl / t_f / 1e9:.0f} TF/s)  bwd-data {t_bd:.3f} ms ({fl / t_bd / 1e9:.0f})  '
              f'wgrad {t_bw:.3f} ms ({fl / t_bw / 1e9:.0f})  dgrad-as-fwd {t_alt:.3f} ms  rel err {err:.2e}',
              flush=True)


if __name__ == '__main__':
    sys.exit(main())

"""Times the decoder's MFMA convolutions (decconv.hip: forward, data gradient, weight gradient
separately) against MIOpen on the same problems (config-2 decoder shapes).

    python tools/micro_decconv.py
"""
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


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    from vfdepth_amd import _lib as L
    torch.cuda.set_device(0)
    lib = L.load()
    dev = 'cuda:0'
    for n, ci, co, h, w in ((6, 16, 16, 384, 640), (6, 32, 32, 192, 320), (6, 32, 16, 192, 320)):
        xp = torch.randn(n, ci, h + 2, w + 2, device=dev)
        wt = torch.randn(co, ci, 3, 3, device=dev)
        b = torch.randn(co, device=dev)
        y = torch.empty(n, co, h, w, device=dev)
        dy = torch.randn_like(y)
        dxp = torch.empty_like(xp)
        part = torch.empty(lib.vfd_dec_conv_wgrad_blocks(n, h, w), co, ci, 9, device=dev)
        st = L.stream()
        gf = 2 * n * h * w * co * ci * 9 / 1e9
        t_f = timeit(lambda: lib.vfd_dec_conv_fwd(xp.data_ptr(), wt.data_ptr(), b.data_ptr(), y.data_ptr(), n, ci, co, h, w, st))
        t_d = timeit(lambda: lib.vfd_dec_conv_bwd(dy.data_ptr(), xp.data_ptr(), wt.data_ptr(), dxp.data_ptr(), None, n, ci, co, h, w, st))
        t_w = timeit(lambda: lib.vfd_dec_conv_bwd(dy.data_ptr(), xp.data_ptr(), wt.data_ptr(), None, part.data_ptr(), n, ci, co, h, w, st))
        t_mf = timeit(lambda: F.conv2d(xp, wt, b))
        t_mb = timeit(lambda: torch.ops.aten.convolution_backward(dy, xp, wt, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, True, False]))
        print(f'{ci}->{co} @{h}x{w}: HIP fwd {t_f:7.1f} us ({gf / t_f * 1e3:6.1f} TF)  dgrad {t_d:7.1f}  wgrad {t_w:7.1f} | '
              f'MIOpen fwd {t_mf:7.1f}  bwd(d+w) {t_mb:7.1f}', flush=True)


if __name__ == '__main__':
    main()

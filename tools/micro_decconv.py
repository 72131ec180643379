"""Times the decoder's MFMA convolutions (decconv.hip: forward, data gradient, weight gradient
separately) against MIOpen on the same problems (config-2 decoder shapes).

    python tools/micro_decconv.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.path.isdir(os.path.join(ROOT, 'miopen_db')):
    os.environ.setdefault('MIOPEN_USER_DB_PATH', os.path.join(ROOT, 'miopen_db'))

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


def stem():
    from vfdepth_amd import _lib as L
    lib = L.load()
    dev = 'cuda:0'
    for c in (6, 3):
        img = torch.rand(6, c, 384, 640, device=dev)
        wt = torch.randn(64, c, 7, 7, device=dev)
        y = torch.empty(6, 64, 192, 320, device=dev)
        g = torch.randn_like(y)
        part = torch.empty(lib.vfd_stem_conv_wgrad_groups(), (lib.vfd_stem_conv_ktiles(c) + 3) // 4 * 4, 64, 16, device=dev)
        st = L.stream()
        gf = 2 * 6 * 192 * 320 * 64 * c * 49 / 1e9
        t_f = timeit(lambda: lib.vfd_stem_conv_fwd(img.data_ptr(), wt.data_ptr(), y.data_ptr(), 6, c, 384, 640, st))
        t_w = timeit(lambda: lib.vfd_stem_conv_wgrad(img.data_ptr(), g.data_ptr(), part.data_ptr(), 6, c, 384, 640, st))
        xn = (img - 0.45) / 0.225
        t_mf = timeit(lambda: F.conv2d((img - 0.45) / 0.225, wt, None, 2, 3))
        t_mw = timeit(lambda: torch.ops.aten.convolution_backward(g, xn, wt, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1, [False, True, False]))
        print(f'stem {c}->64 @384x640: HIP fwd (incl. normalise) {t_f:7.1f} us ({gf / t_f * 1e3:6.1f} TF)  wgrad {t_w:7.1f} | '
              f'MIOpen normalise+fwd {t_mf:7.1f}  wgrad {t_mw:7.1f}', flush=True)


if __name__ == '__main__':
    stem()
    main()

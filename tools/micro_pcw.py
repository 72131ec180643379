"""Time the fp32 K3C weight gradient (`vfd_proj_conv_wgrad`, pcw_main_k + reduce + bias) at a
bench config and check it against MIOpen's weight gradient of the same conv.

    VFD_LIB=variants/libvfd_X.so python tools/micro_pcw.py [--config 2] [--iters 20]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vfdepth_amd.miopen_db import use_private_copy  # noqa: E402
use_private_copy()

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', type=int, default=2)
    ap.add_argument('--iters', type=int, default=20)
    a = ap.parse_args()
    import bench
    from vfdepth_amd import _lib as L
    from vfdepth_amd import kernels as KN
    dev = torch.device('cuda:0')
    cfg, _ = bench.make_cfg(a.config, 1)
    space = KN.VoxelSpace(cfg, dev)
    lib = L.load()
    N, Cv, O, D, h, w = cfg['data']['num_cams'], 64, 256, space.D, space.h, space.w
    gen = torch.Generator(device=dev).manual_seed(5)
    g = torch.randn(N, O, h, w, device=dev, generator=gen).contiguous(memory_format=torch.channels_last)
    x = torch.randn(N, Cv * D, h + 2, w + 2, device=dev, generator=gen).contiguous(memory_format=torch.channels_last)
    dw = torch.empty(O, Cv * D, 3, 3, device=dev)
    db = torch.empty(O, device=dev)
    d = space.desc(1, N, Cv=Cv, pad_out=2)
    nb = lib.vfd_proj_conv_wgrad_workspace(ctypes.byref(d))
    assert nb, 'wgrad declined this shape'
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)

    def call():
        L.check(lib.vfd_proj_conv_wgrad(ctypes.byref(d), g.data_ptr(), x.data_ptr(), dw.data_ptr(), db.data_ptr(),
                                        ws.data_ptr(), nb, L.stream()), 'proj_conv_wgrad')

    for _ in range(3):
        call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        call()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    flop = 2.0 * N * h * w * O * Cv * D * 9
    # the kernel writes dW in channel order c*D + d; MIOpen's conv over x uses x's order d*Cv + c
    wm = torch.empty(O, Cv * D, 3, 3, device=dev)
    _, ref, rb = torch.ops.aten.convolution_backward(g, x, wm, [O], [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                                     [False, True, True])
    ref = ref.view(O, D, Cv, 3, 3).transpose(1, 2).reshape(O, Cv * D, 3, 3)
    err = float((dw - ref).abs().max() / ref.abs().max())
    berr = float((db - rb).abs().max() / rb.abs().max())
    print(f'config {a.config}: wgrad {ms:.3f} ms, {flop / ms / 1e9:.1f} TFLOP/s ({flop / ms / 1e9 / 157.3:.3f} of '
          f'fp32 peak); max rel err dW {err:.2e} db {berr:.2e}', flush=True)
    assert err < 1e-4 and berr < 1e-4


if __name__ == '__main__':
    main()

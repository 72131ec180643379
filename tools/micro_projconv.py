"""Time K3C (K3 fused into reduce_dim's first conv) against K3 + MIOpen conv at config 2.

    python tools/micro_projconv.py [--config 2] [--iters 20]
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


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    import bench
    from vfdepth_amd import _lib
    from vfdepth_amd import kernels as KN
    from vfdepth_amd import synth
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', type=int, default=2)
    ap.add_argument('--iters', type=int, default=20)
    a = ap.parse_args()
    _lib.load()
    cfg, _ = bench.make_cfg(a.config, 1)
    dev = torch.device('cuda:0')
    space = KN.VoxelSpace(cfg, dev)
    b = synth.make_batch(cfg, seed=71, device=dev)
    lvl = cfg['model']['fusion_level'] + 1
    invK, E = b['inv_K', lvl], b['extrinsics']
    B, N = E.shape[:2]
    Cv, D, O = 64, space.D, 256
    vox = torch.randn(B, space.V, Cv, device=dev)
    w0 = torch.randn(O, Cv * D, 3, 3, device=dev) * (Cv * D * 9) ** -0.5
    bias = 0.1 * torch.randn(O, device=dev)
    flop = 2.0 * B * N * space.h * space.w * O * Cv * D * 9
    with torch.no_grad():
        t_fused = timed(lambda: KN.ProjConv.apply(space, vox, invK, E, w0, bias), a.iters)
        wp = KN.proj_conv_weight(w0, Cv, D)
        t_k3 = timed(lambda: KN.VoxelProject.apply(space, vox, invK, E), a.iters)
        x = KN.VoxelProject.apply(space, vox, invK, E)
        t_conv = timed(lambda: F.leaky_relu(F.conv2d(x, wp, bias), 0.1), a.iters)
        _lib.prof_enable('proj_conv_fwd')
        for _ in range(a.iters):
            KN.ProjConv.apply(space, vox, invK, E, w0, bias)
        torch.cuda.synchronize()
        prof = _lib.prof_read()
        _lib.prof_enable('off')
        n, ms = prof.get('proj_conv_fwd', (1, float('nan')))
        y = KN.ProjConv.apply(space, vox, invK, E, w0, bias)
        ref = F.pad(F.leaky_relu(F.conv2d(x, wp, bias), 0.1), (1, 1, 1, 1), mode='reflect')
        err = float((y - ref).abs().max()) / float(ref.abs().max())
    # with a voxel gradient: the kernel also writes the frustum features (K3's output) as a side output
    vg = vox.clone().requires_grad_(True)
    t_side = timed(lambda: KN.ProjConv.apply(space, vg, invK, E, w0, bias), a.iters)
    y2 = KN.ProjConv.apply(space, vg, invK, E, w0, bias)
    xs = y2.grad_fn.saved_tensors[2]
    xerr = float((xs - x).abs().max())
    print(f'config {a.config}: K3C fused {t_fused:.3f} ms (kernel {ms / n:.3f} ms, {flop / (ms / n) / 1e9:.1f} TFLOP/s); '
          f'with side output {t_side:.3f} ms; '
          f'K3 {t_k3:.3f} ms + MIOpen conv {t_conv:.3f} ms = {t_k3 + t_conv:.3f} ms; max rel err {err:.2e}; '
          f'side output max |dx| {xerr:.2e}', flush=True)
    # data gradient: the MFMA kernel vs MIOpen's (channels-last) data gradient
    import ctypes
    lib = _lib.load()
    h, w = space.h, space.w
    g_pre = torch.randn(B * N, O, h, w, device=dev).contiguous(memory_format=torch.channels_last)
    d = space.desc(B, N, Cv=Cv)
    nbytes = lib.vfd_proj_conv_dgrad_workspace(ctypes.byref(d))
    if not nbytes:
        print('dgrad kernel: shape unsupported', flush=True)
        return
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dx = torch.empty(B * N, Cv * D, h + 2, w + 2, device=dev, memory_format=torch.channels_last)

    def dgrad():
        wd = KN.proj_conv_dgrad_weight(w0, Cv, D)
        _lib.check(lib.vfd_proj_conv_dgrad(ctypes.byref(d), g_pre.data_ptr(), wd.data_ptr(), dx.data_ptr(),
                                           ws.data_ptr(), nbytes, _lib.stream()), 'proj_conv_dgrad')
    xcl = x.contiguous(memory_format=torch.channels_last)
    cb = torch.ops.aten.convolution_backward
    args = ([O], [1, 1], [0, 0], [1, 1], False, [0, 0], 1)
    t_dg = timed(dgrad, a.iters)
    t_mi = timed(lambda: cb(g_pre, xcl, wp, *args, [True, False, False]), a.iters)
    t_wg = timed(lambda: cb(g_pre, xcl, wp, *args, [False, True, True]), a.iters)
    _lib.prof_enable('proj_conv_dgrad')
    for _ in range(a.iters):
        dgrad()
    torch.cuda.synchronize()
    prof = _lib.prof_read()
    _lib.prof_enable('off')
    n2, ms2 = prof.get('proj_conv_dgrad', (1, float('nan')))
    dgrad()
    ref = cb(g_pre, xcl, wp, *args, [True, False, False])[0]
    derr = float((dx - ref).abs().max()) / float(ref.abs().max())
    print(f'config {a.config}: dgrad kernel {t_dg:.3f} ms (kernel {ms2 / n2:.3f} ms, {flop / (ms2 / n2) / 1e9:.1f} TFLOP/s, '
          f'weight copy incl.); MIOpen dgrad {t_mi:.3f} ms, MIOpen wgrad {t_wg:.3f} ms; max rel err {derr:.2e}', flush=True)
    # the folded form (pad_out = 2): interior only, reflect copies folded in; check against the
    # padded result folded on the host side
    df = space.desc(B, N, Cv=Cv, pad_out=2)
    nbf = lib.vfd_proj_conv_dgrad_workspace(ctypes.byref(df))
    if nbf:
        wsf = torch.empty(nbf, dtype=torch.uint8, device=dev)
        dxf = torch.zeros_like(dx)

        def dgrad_f():
            wd = KN.proj_conv_dgrad_weight(w0, Cv, D)
            _lib.check(lib.vfd_proj_conv_dgrad(ctypes.byref(df), g_pre.data_ptr(), wd.data_ptr(), dxf.data_ptr(),
                                               wsf.data_ptr(), nbf, _lib.stream()), 'proj_conv_dgrad folded')
        _lib.prof_enable('proj_conv_dgrad')
        for _ in range(a.iters):
            dgrad_f()
        torch.cuda.synchronize()
        prof = _lib.prof_read()
        _lib.prof_enable('off')
        n4, ms4 = prof.get('proj_conv_dgrad', (1, float('nan')))
        dgrad()
        ref = dx.clone()                                   # padded, unfolded: fold it here
        ref[:, :, 2, :] += ref[:, :, 0, :]
        ref[:, :, h - 1, :] += ref[:, :, h + 1, :]
        ref[:, :, :, 2] += ref[:, :, :, 0]
        ref[:, :, :, w - 1] += ref[:, :, :, w + 1]
        inner = (slice(None), slice(None), slice(1, h + 1), slice(1, w + 1))
        ferr = float((dxf[inner] - ref[inner]).abs().max()) / float(ref[inner].abs().max())
        print(f'config {a.config}: folded dgrad kernel {ms4 / n4:.3f} ms ({flop / (ms4 / n4) / 1e9:.1f} TFLOP/s); '
              f'max rel err vs folded padded {ferr:.2e}', flush=True)
    # weight / bias gradient: the MFMA kernel (reference channel order) vs MIOpen's + the channel swap
    nbytes = lib.vfd_proj_conv_wgrad_workspace(ctypes.byref(d))
    ws2 = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dw = torch.empty(O, Cv * D, 3, 3, device=dev)
    db = torch.empty(O, device=dev)

    def wgrad():
        _lib.check(lib.vfd_proj_conv_wgrad(ctypes.byref(d), g_pre.data_ptr(), xcl.data_ptr(), dw.data_ptr(),
                                           db.data_ptr(), ws2.data_ptr(), nbytes, _lib.stream()), 'proj_conv_wgrad')
    t_wk = timed(wgrad, a.iters)
    _lib.prof_enable('proj_conv_wgrad')
    for _ in range(a.iters):
        wgrad()
    torch.cuda.synchronize()
    prof = _lib.prof_read()
    _lib.prof_enable('off')
    n3, ms3 = prof.get('proj_conv_wgrad', (1, float('nan')))
    _, dw_ref, db_ref = cb(g_pre, xcl, w0, *args, [False, True, True])
    dw_ref = KN.weight_swap(dw_ref, D, Cv)
    werr = float((dw - dw_ref).abs().max()) / float(dw_ref.abs().max())
    berr = float((db - db_ref).abs().max()) / float(db_ref.abs().max())
    print(f'config {a.config}: wgrad kernel {t_wk:.3f} ms (kernel {ms3 / n3:.3f} ms, {flop / (ms3 / n3) / 1e9:.1f} TFLOP/s, '
          f'bias incl.); max rel err dw {werr:.2e} db {berr:.2e}', flush=True)


if __name__ == '__main__':
    main()

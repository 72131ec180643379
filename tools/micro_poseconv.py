"""Pose reduce_dim first conv (Cin = (C+1)*Z = 5140, 3x3 stride 2 on the padded 102x102 BEV map,
-> 256) at config 2: MIOpen channels-last (the model's path) vs NCHW vs unfold + GEMM, fwd and bwd.

    python tools/micro_poseconv.py [--iters 10]
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
    for _ in range(2):
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
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--batch', type=int, default=1, help='>1: also the data gradient at that batch vs per image')
    a = ap.parse_args()
    dev = torch.device('cuda:0')
    C, Y, X, O = 5140, 100, 100, 256
    x_cl = torch.randn(1, C, Y + 2, X + 2, device=dev).contiguous(memory_format=torch.channels_last)
    x_nc = x_cl.contiguous()
    w = torch.randn(O, C, 3, 3, device=dev) * (C * 9) ** -0.5
    b = torch.randn(O, device=dev)
    flop = 2.0 * 50 * 50 * O * C * 9
    g = torch.randn(1, O, 50, 50, device=dev)
    res = {}
    res['fwd_cl'] = timed(lambda: F.conv2d(x_cl, w, b, stride=2), a.iters)
    res['fwd_nchw'] = timed(lambda: F.conv2d(x_nc, w, b, stride=2), a.iters)
    w2 = w.reshape(O, -1)

    def fwd_gemm():
        cols = F.unfold(x_nc, 3, stride=2)                     # [1, C*9, 2500]
        return torch.addmm(b[:, None], w2, cols[0])
    res['fwd_unfold_gemm'] = timed(fwd_gemm, a.iters)
    cols = F.unfold(x_nc, 3, stride=2)[0]
    res['gemm_only'] = timed(lambda: torch.addmm(b[:, None], w2, cols), a.iters)
    res['unfold_only'] = timed(lambda: F.unfold(x_nc, 3, stride=2), a.iters)
    cb = torch.ops.aten.convolution_backward
    args = ([O], [2, 2], [0, 0], [1, 1], False, [0, 0], 1)
    g_cl = g.contiguous(memory_format=torch.channels_last)
    res['dgrad_cl'] = timed(lambda: cb(g_cl, x_cl, w, *args, [True, False, False]), a.iters)
    res['wgrad_cl'] = timed(lambda: cb(g_cl, x_cl, w, *args, [False, True, True]), a.iters)
    res['dgrad_nchw'] = timed(lambda: cb(g, x_nc, w, *args, [True, False, False]), a.iters)
    res['wgrad_nchw'] = timed(lambda: cb(g, x_nc, w, *args, [False, True, True]), a.iters)
    res['wgrad_gemm'] = timed(lambda: torch.mm(g.reshape(O, -1), cols.t()), a.iters)

    def dgrad_gemm():
        dcols = torch.mm(w2.t(), g.reshape(O, -1))
        return F.fold(dcols[None], (Y + 2, X + 2), 3, stride=2)
    res['dgrad_gemm_fold'] = timed(dgrad_gemm, a.iters)
    if a.batch > 1:     # config 3 (B = 2): one call over the batch vs one call per image
        nb = a.batch
        xb = torch.randn(nb, C, Y + 2, X + 2, device=dev).contiguous(memory_format=torch.channels_last)
        gb = torch.randn(nb, O, 50, 50, device=dev).contiguous(memory_format=torch.channels_last)
        res[f'dgrad_cl_n{nb}'] = timed(lambda: cb(gb, xb, w, *args, [True, False, False]), a.iters) / nb
        res[f'dgrad_cl_per_image_n{nb}'] = timed(
            lambda: [cb(gb[i:i + 1], xb[i:i + 1], w, *args, [True, False, False]) for i in range(nb)], a.iters) / nb
        w16, xb16, gb16 = w.bfloat16(), xb.bfloat16(), gb.bfloat16()
        res[f'wgrad_cl_bf16_n{nb}'] = timed(lambda: cb(gb16, xb16, w16, *args, [False, True, True]), a.iters) / nb
        res[f'wgrad_cl_bf16_per_image_n{nb}'] = timed(
            lambda: [cb(gb16[i:i + 1], xb16[i:i + 1], w16, *args, [False, True, True]) for i in range(nb)], a.iters) / nb
        da = cb(gb, xb, w, *args, [True, False, False])[0]
        dp = torch.cat([cb(gb[i:i + 1], xb[i:i + 1], w, *args, [True, False, False])[0] for i in range(nb)])
        print(f'per-image vs batched dgrad max rel err {float((da - dp).abs().max() / da.abs().max()):.2e} '
              '(times per image below)', flush=True)
    ref = F.conv2d(x_cl, w, b, stride=2)
    err = float((fwd_gemm().reshape(1, O, 50, 50) - ref).abs().max() / ref.abs().max())
    for k, v in res.items():
        extra = f'  {flop / v / 1e9:.1f} TFLOP/s' if not k.startswith('unfold') else ''
        print(f'{k:18s} {v:8.3f} ms{extra}', flush=True)
    print(f'unfold+gemm vs conv max rel err {err:.2e}', flush=True)


if __name__ == '__main__':
    main()

"""Time the hand-written reduce_dim gradient kernels through the C ABI (HIP events on the launching
stream, the bench's own scopes), fp32 and bf16, at the step shapes.

    python tools/micro_convbwd_capi.py [--iters 10] [--ops dgrad,dgrad_bf16] [--shapes c2,c3,c5]
Run a variant build with VFD_LIB=/path/libvfd_X.so (tools/build_variant.py)."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

SHAPES = {'c2': (1, 48, 80, 50), 'c3': (2, 48, 80, 50), 'c4': (1, 44, 80, 50), 'c5': (4, 80, 120, 50)}
POSE = {'c2': (1, 102), 'c3': (2, 102), 'c4': (1, 102), 'c5': (4, 202)}     # (B, padded BEV side), C = 257 * 20
PEAK = {'fp32': 157.3, 'bf16': 2516.6}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--ops', default='dgrad,dgrad_bf16')
    ap.add_argument('--shapes', default='c2,c3,c5')
    a = ap.parse_args()
    from vfdepth_amd import _lib as L
    from vfdepth_amd import kernels as KN
    sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
    import common as G
    lib = L.load()
    dev = torch.device('cuda:0')
    space = KN.VoxelSpace(G.step_cfg(), dev)
    for sh in a.shapes.split(','):
        pose_ops = [o for o in a.ops.split(',') if o.startswith(('pdgrad', 'pwgrad', 'pfwd'))]
        if pose_ops:
            pose(lib, L, KN, dev, sh, pose_ops, a.iters)
        if all(o.startswith(('pdgrad', 'pwgrad', 'pfwd')) for o in a.ops.split(',')):
            continue
        B, h, w, D = SHAPES[sh]
        N, Cv, O = 6, 64, 256
        d = space.desc(B, N, Cv=Cv, pad_out=2)
        d.h, d.w, d.D = h, w, D
        g_pre = torch.randn(B * N, O, h, w, device=dev).contiguous(memory_format=torch.channels_last)
        w0 = torch.randn(O, Cv * D, 3, 3, device=dev) * (O * 9) ** -0.5
        dx = torch.empty(B * N, Cv * D, h + 2, w + 2, device=dev).contiguous(memory_format=torch.channels_last)
        flop = 2.0 * B * N * h * w * O * Cv * D * 9
        for op in a.ops.split(','):
            if op.startswith(('pdgrad', 'pwgrad', 'pfwd')):
                continue
            if op == 'dgrad':
                wd, gp, kind = KN.proj_conv_dgrad_weight(w0, Cv, D), g_pre, 'fp32'
                nb = lib.vfd_proj_conv_dgrad_workspace(ctypes.byref(d))
                fn = lib.vfd_proj_conv_dgrad
            elif op in ('wgrad_bf16', 'wgrad_bf16_miopen'):
                time_wgrad(lib, L, KN, dev, d, sh, B, N, h, w, D, op, a.iters)
                continue
            elif op == 'dgrad_bf16':
                wd, gp, kind = KN.proj_conv_dgrad_weight_bf16(w0, Cv, D), g_pre.to(torch.bfloat16), 'bf16'
                nb = lib.vfd_proj_conv_dgrad_bf16_workspace(ctypes.byref(d))
                fn = lib.vfd_proj_conv_dgrad_bf16
            else:
                raise SystemExit(f'unknown op {op}')
            if not nb:
                print(f'{sh} {op}: unsupported', flush=True)
                continue
            ws = torch.empty(nb, dtype=torch.uint8, device=dev)

            def call():
                L.check(fn(ctypes.byref(d), gp.data_ptr(), wd.data_ptr(), dx.data_ptr(), ws.data_ptr(), nb,
                           L.stream()), op)
            for _ in range(2):
                call()
            torch.cuda.synchronize()
            L.prof_enable('proj_conv_dgrad')
            for _ in range(a.iters):
                call()
            torch.cuda.synchronize()
            n, ms = L.prof_read()['proj_conv_dgrad']
            L.prof_enable('off')
            us = ms / n * 1e3
            tf = flop / (us * 1e-6) / 1e12
            print(f'{sh} {op:11s} {us:9.1f} us  {tf:7.1f} TF/s  {tf / PEAK[kind]:.3f} of {kind} peak', flush=True)


def _events(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def time_wgrad(lib, L, KN, dev, d, sh, B, N, h, w, D, op, iters):
    """K3C bf16 weight + bias gradient: the HIP kernel vs MIOpen's bf16 wrw of the same conv."""
    Cv, O = 64, 256
    gb = torch.randn(B * N, O, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xb = torch.randn(B * N, Cv * D, h + 2, w + 2, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    flop = 2.0 * B * N * h * w * O * Cv * D * 9
    if op == 'wgrad_bf16':
        nb = lib.vfd_proj_conv_wgrad_bf16_workspace(ctypes.byref(d))
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        dw = torch.empty(O, Cv * D, 3, 3, device=dev)
        db = torch.empty(O, device=dev)

        def call():
            L.check(lib.vfd_proj_conv_wgrad_bf16(ctypes.byref(d), gb.data_ptr(), xb.data_ptr(), dw.data_ptr(),
                                                 db.data_ptr(), ws.data_ptr(), nb, L.stream()), op)
    else:
        wb = torch.empty(O, Cv * D, 3, 3, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)

        def call():
            torch.ops.aten.convolution_backward(gb, xb, wb, [O], [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                                [False, True, True])
    us = _events(call, iters)
    tf = flop / (us * 1e-6) / 1e12
    print(f'{sh} {op:17s} {us:9.1f} us  {tf:7.1f} TF/s  {tf / PEAK["bf16"]:.3f} of bf16 peak', flush=True)


def pose(lib, L, KN, dev, sh, ops, iters):
    """K2C (pose reduce_dim[0], stride 2) data gradient: the HIP kernel (fp32 / bf16) vs MIOpen's
    backward-data of the same conv (fp32, torch events)."""
    import torch.nn.functional as F
    B, S = POSE[sh]
    C, C1, Z = 5140, 257, 20
    ho = (S - 3) // 2 + 1
    g = torch.randn(B, 256, ho, ho, device=dev).contiguous(memory_format=torch.channels_last)
    w = torch.randn(256, C, 3, 3, device=dev) * (256 * 9) ** -0.5
    x = torch.randn(B, C, S, S, device=dev).contiguous(memory_format=torch.channels_last)
    flop = 2.0 * B * ho * ho * 256 * C * 9
    for op in ops:
        if op in ('pfwd', 'pfwd_bf16', 'pfwd_bf16m'):
            bf = op != 'pfwd'
            xm = x.to(torch.bfloat16) if op == 'pfwd_bf16m' else x    # the bf16 map of PoseConvBF16
            d = KN.pad_conv_desc(x, 2, 256)
            bias = torch.randn(256, device=dev)
            wf = KN.pad_conv_weight_fragments_bf16(w, C1, Z) if bf else KN.pad_conv_weight_fragments(w, C1, Z)
            fn = lib.vfd_pad_conv_fwd_bf16 if bf else lib.vfd_pad_conv_fwd
            nb = (lib.vfd_pad_conv_fwd_bf16_workspace if bf else lib.vfd_pad_conv_fwd_workspace)(ctypes.byref(d))
            ws = torch.empty(nb, dtype=torch.uint8, device=dev)
            out = torch.empty(B, 256, ho + 2, ho + 2, device=dev, dtype=torch.bfloat16 if bf else torch.float32,
                              memory_format=torch.channels_last)

            def fcall():
                if op == 'pfwd_bf16m':
                    L.check(lib.vfd_pad_conv_fwd_bf16_t(ctypes.byref(d), xm.data_ptr(), 1, wf.data_ptr(), bias.data_ptr(),
                                                        out.data_ptr(), ws.data_ptr(), nb, L.stream()), op)
                    return
                L.check(fn(ctypes.byref(d), x.data_ptr(), wf.data_ptr(), bias.data_ptr(), out.data_ptr(),
                           ws.data_ptr(), nb, L.stream()), op)
            for _ in range(2):
                fcall()
            torch.cuda.synchronize()
            L.prof_enable('pad_conv_fwd')
            for _ in range(iters):
                fcall()
            torch.cuda.synchronize()
            n, ms = L.prof_read()['pad_conv_fwd']
            L.prof_enable('off')
            us = ms / n * 1e3
            kind = 'bf16' if bf else 'fp32'
            tf = flop / (us * 1e-6) / 1e12
            print(f'{sh} pose {op:14s} {us:9.1f} us  {tf:7.1f} TF/s  {tf / PEAK[kind]:.3f} of {kind} peak', flush=True)
            continue
        if op in ('pwgrad_bf16', 'pwgrad_bf16m', 'pwgrad_bf16_miopen'):
            gb = g.to(torch.bfloat16)
            if op == 'pwgrad_bf16':
                call = lambda: KN.pad_conv_wgrad_bf16(gb, x, w, 2)  # noqa: E731
            elif op == 'pwgrad_bf16m':
                xm = x.to(torch.bfloat16)
                call = lambda: KN.pad_conv_wgrad_bf16(gb, xm, w, 2)  # noqa: E731
            else:
                wm = KN.pose_conv_weight(w, C1, Z).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
                call = lambda: torch.ops.aten.convolution_backward(gb, x.to(torch.bfloat16), wm, [256], [2, 2], [0, 0],  # noqa: E731
                                                                   [1, 1], False, [0, 0], 1, [False, True, True])
            us = _events(call, iters)
            tf = flop / (us * 1e-6) / 1e12
            print(f'{sh} pose {op:18s} {us:9.1f} us  {tf:7.1f} TF/s  {tf / PEAK["bf16"]:.3f} of bf16 peak', flush=True)
            continue
        if op == 'pdgrad_miopen':
            wm = KN.pose_conv_weight(w, C1, Z).contiguous(memory_format=torch.channels_last)
            fn = lambda: torch.ops.aten.convolution_backward(g, x, wm, [256], [2, 2], [0, 0], [1, 1], False, [0, 0], 1,
                                                             [True, False, False])  # noqa: E731
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us, kind = e0.elapsed_time(e1) / iters * 1e3, 'fp32'
        else:
            gk = g.to(torch.bfloat16) if op == 'pdgrad_bf16' else g
            kind = 'bf16' if op == 'pdgrad_bf16' else 'fp32'
            for _ in range(2):
                KN.pad_conv_dgrad(gk, x.shape, w, 2, (C1, Z))
            torch.cuda.synchronize()
            L.prof_enable('pad_conv_dgrad')
            for _ in range(iters):
                KN.pad_conv_dgrad(gk, x.shape, w, 2, (C1, Z))
            torch.cuda.synchronize()
            n, ms = L.prof_read()['pad_conv_dgrad']
            L.prof_enable('off')
            us = ms / n * 1e3
        tf = flop / (us * 1e-6) / 1e12
        print(f'{sh} pose {op:14s} {us:9.1f} us  {tf:7.1f} TF/s  {tf / PEAK[kind]:.3f} of {kind} peak', flush=True)


if __name__ == '__main__':
    main()

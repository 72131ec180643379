"""Times the fused dense kernels against the ATen ops they replace, at the bench's shapes
(config 2: 6 cameras, 384x640): stem max pool fwd/bwd, reflect pad fwd/bwd, align-corners
upsample backward, BatchNorm+ReLU fwd/bwd.  Prints us/call and GB/s of the algorithmic bytes.

    python tools/micro_dense.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

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


def line(name, us, nbytes):
    print(f'{name:44s} {us:8.1f} us  {nbytes / us / 1e3:8.1f} GB/s', flush=True)


def main():
    from vfdepth_amd import _lib as L
    from vfdepth_amd import kernels as KN
    torch.cuda.set_device(0)
    lib = L.load()
    dev = 'cuda:0'
    x = torch.randn(6, 64, 192, 320, device=dev).relu_()
    y = KN.MaxPool3s2.apply(x)
    arg = torch.empty(y.shape, dtype=torch.uint8, device=dev)
    g = torch.randn_like(y)
    dx = torch.empty_like(x)
    nb = x.numel() * 4 + y.numel() * 5
    line('maxpool fwd (HIP)', timeit(lambda: lib.vfd_maxpool3s2_fwd(x.data_ptr(), y.data_ptr(), arg.data_ptr(), 384, 192, 320, 0, L.stream())), nb)
    line('maxpool bwd (HIP)', timeit(lambda: lib.vfd_maxpool3s2_bwd(g.data_ptr(), arg.data_ptr(), dx.data_ptr(), 384, 192, 320, 0, L.stream())), nb)
    yr, idx = F.max_pool2d(x, 3, 2, 1, return_indices=True)
    line('maxpool fwd (ATen)', timeit(lambda: F.max_pool2d(x, 3, 2, 1, return_indices=True)), x.numel() * 4 + y.numel() * 12)
    line('maxpool bwd (ATen)', timeit(lambda: torch.ops.aten.max_pool2d_with_indices_backward(g, x, [3, 3], [2, 2], [1, 1], [1, 1], False, idx)),
         x.numel() * 4 + y.numel() * 12)
    line('copy (reference stream)', timeit(lambda: dx.copy_(x)), x.numel() * 8)
    for shape in ((6, 64, 96, 160), (6, 256, 24, 40), (6, 32, 192, 320)):
        t = torch.randn(shape, device=dev)
        n, c, h, w = shape
        tp = torch.empty(n, c, h + 2, w + 2, device=dev)
        nbp = (t.numel() + tp.numel()) * 4
        line(f'reflect pad fwd {shape}', timeit(lambda: lib.vfd_reflect_pad1_fwd(t.data_ptr(), tp.data_ptr(), n * c, h, w, 0, L.stream())), nbp)
        line(f'reflect pad bwd {shape}', timeit(lambda: lib.vfd_reflect_pad1_bwd(tp.data_ptr(), t.data_ptr(), n * c, h, w, 0, L.stream())), nbp)
    # decoder ELU [+ nearest 2x] + reflect pad (config-2 decoder shapes) vs the ATen chain
    for shape, up in (((6, 16, 192, 320), 1), ((6, 16, 384, 640), 0), ((6, 32, 96, 160), 1), ((6, 64, 48, 80), 1)):
        n, c, h, w = shape
        yy = torch.randn(shape, device=dev)
        op = torch.empty(n, c, (h << up) + 2, (w << up) + 2, device=dev)
        dyy = torch.empty_like(yy)
        nbe = (yy.numel() + op.numel()) * 4
        line(f'elu_up_pad fwd {shape} up={up}', timeit(lambda: lib.vfd_elu_up_pad1_fwd(yy.data_ptr(), op.data_ptr(), n * c, h, w, up, 0, L.stream())), nbe)
        line(f'elu_up_pad bwd {shape} up={up}', timeit(lambda: lib.vfd_elu_up_pad1_bwd(op.data_ptr(), yy.data_ptr(), dyy.data_ptr(), n * c, h, w, up, None, 0, L.stream())), nbe + yy.numel() * 4)

        def aten_chain():
            a = F.elu(yy)
            if up:
                a = F.interpolate(a, scale_factor=2, mode='nearest')
            return F.pad(a, (1, 1, 1, 1), mode='reflect')
        line(f'  ATen elu->up->pad fwd {shape}', timeit(aten_chain), nbe)
    # decoder disparity head 16 -> 1 at full resolution vs MIOpen
    xpd = torch.randn(6, 16, 386, 642, device=dev, requires_grad=True)
    wd = (0.1 * torch.randn(1, 16, 3, 3, device=dev)).requires_grad_(True)
    bd = torch.zeros(1, device=dev, requires_grad=True)
    od = KN.DispConvSigmoid.apply(xpd, wd, bd)
    gd = torch.randn_like(od)
    line('disp conv fwd (HIP)', timeit(lambda: KN.DispConvSigmoid.apply(xpd, wd, bd)), xpd.numel() * 4)
    line('disp conv fwd+bwd (HIP)', timeit(lambda: torch.autograd.grad(KN.DispConvSigmoid.apply(xpd, wd, bd), (xpd, wd, bd), gd)), xpd.numel() * 12)
    line('disp conv fwd (MIOpen)', timeit(lambda: torch.sigmoid(F.conv2d(xpd, wd, bd))), xpd.numel() * 4)
    line('disp conv fwd+bwd (MIOpen)', timeit(lambda: torch.autograd.grad(torch.sigmoid(F.conv2d(xpd, wd, bd)), (xpd, wd, bd), gd)), xpd.numel() * 12)
    d = torch.randn(6, 256, 48, 80, device=dev)
    for hs, ws in ((24, 40), (12, 20), (6, 10)):
        dl = torch.empty(6, 256, hs, ws, device=dev)
        tmp = torch.empty(6 * 256 * 48 * ws, device=dev)
        line(f'upsample bwd {hs}x{ws}', timeit(lambda: lib.vfd_upsample_ac_bwd(d.data_ptr(), dl.data_ptr(), tmp.data_ptr(), 6 * 256, 48, 80, hs, ws, L.stream())),
             (d.numel() + dl.numel()) * 4)
    for shape in ((6, 64, 192, 320), (6, 64, 96, 160), (6, 512, 12, 20)):
        bn = torch.nn.BatchNorm2d(shape[1]).to(dev).train()
        t = torch.randn(shape, device=dev, requires_grad=True)
        from vfdepth_amd.layers import bn_act
        out = bn_act(bn, t)
        go = torch.randn_like(out)
        line(f'bn+relu fwd {shape}', timeit(lambda: bn_act(bn, t)), t.numel() * 12)
        line(f'bn+relu fwd+bwd {shape}', timeit(lambda: torch.autograd.grad(bn_act(bn, t), t, go)), t.numel() * 32)
    # per-step weight relayouts (weights.hip) at the config-2 reduce_dim weights
    wk = torch.randn(256, 64 * 50, 3, 3, device=dev)
    line('K3C fwd fragments 256x3200x9', timeit(lambda: KN.proj_conv_weight_fragments(wk, 64, 50)), wk.numel() * 8)
    line('K3C dgrad copy 256x3200x9', timeit(lambda: KN.proj_conv_dgrad_weight(wk, 64, 50)), wk.numel() * 8)
    wp = torch.randn(256, 256 * 20, 3, 3, device=dev)
    line('K2C pose fragments 256x5120x9', timeit(lambda: KN.pose_conv_fragments(wp, 256, 20)), wp.numel() * 8)
    line('pose swap -> channels-last', timeit(lambda: KN.weight_swap(wp, 256, 20, memory_format=torch.channels_last)), wp.numel() * 8)
    wpc = wp.contiguous(memory_format=torch.channels_last)
    line('pose swap channels-last -> NCHW', timeit(lambda: KN.weight_swap(wpc, 20, 256)), wp.numel() * 8)


if __name__ == '__main__':
    main()

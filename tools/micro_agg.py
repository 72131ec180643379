"""Time the fusion-level aggregation forward on channels-last bf16 products (config 3 shapes) and
its NCHW fp32 form: `python tools/micro_agg.py` (VFD_LIB selects a tools/build_variant.py build)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vfdepth_amd import kernels as KN  # noqa: E402


def timed(fn, iters=50):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    dev = 'cuda'
    g = torch.Generator(device=dev).manual_seed(1)
    BN, C, h, w = 12, 256, 48, 80
    lv = ((24, 40), (12, 20))
    cl = torch.channels_last
    base = torch.randn(BN, C, h, w, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    levels = [torch.randn(BN, C, a, b, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
              for a, b in lv]
    bias = torch.randn(C, device=dev, generator=g)
    with torch.no_grad():
        t_cl = timed(lambda: KN.AggregateUp.apply(base, bias, *levels))
        b32, l32 = base.float().contiguous(), [t.float().contiguous() for t in levels]
        t_nchw = timed(lambda: KN.AggregateUp.apply(b32, bias, *l32))
    print(f'aggregate fwd {BN}x{C}x{h}x{w} + {len(lv)} levels: channels-last bf16 {t_cl:.1f} us, NCHW fp32 {t_nchw:.1f} us')


if __name__ == '__main__':
    main()

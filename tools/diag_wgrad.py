"""Diagnose the bf16 weight-gradient kernel against MIOpen on small shapes: error by tap, by
channel block, by output-channel block (tools for development; not part of any test)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    from vfdepth_amd import kernels as KN
    dev = torch.device('cuda:0')
    for (B, C, H, W, s) in [(1, 40, 13, 11, 2), (1, 48, 9, 30, 1), (1, 64, 7, 7, 2), (1, 32, 35, 35, 2), (2, 5140, 102, 102, 2)]:
        gen = torch.Generator(device=dev).manual_seed(702)
        ho, wo = (H - 3) // s + 1, (W - 3) // s + 1
        gb = torch.randn(B, 256, ho, wo, device=dev, generator=gen).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x = torch.randn(B, C, H, W, device=dev, generator=gen).contiguous(memory_format=torch.channels_last)
        w = torch.empty(256, C, 3, 3, device=dev)
        dw, db = KN.pad_conv_wgrad_bf16(gb, x, w, s)
        gf, xf = gb.float(), x.to(torch.bfloat16).float()
        _, ref, rb = torch.ops.aten.convolution_backward(gf, xf, w, [256], [s, s], [0, 0], [1, 1], False, [0, 0], 1,
                                                         [False, True, True])
        e = (dw - ref).abs()
        sc = float(ref.abs().max())
        print(f'{(B, C, H, W, s)}: max rel {float(e.max()) / sc:.3g}; db max {float((db - rb).abs().max()):.3g}')
        print('  by tap', [round(float(e[:, :, k // 3, k % 3].max()) / sc, 3) for k in range(9)])
        print('  by c-block', [round(float(e[:, c:c + 32].max()) / sc, 3) for c in range(0, min(C, 256), 32)])
        print('  by o-block', [round(float(e[32 * o:32 * o + 32].max()) / sc, 3) for o in range(8)])


if __name__ == '__main__':
    main()

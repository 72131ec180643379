"""reduce_dim[0] backward (config 2: 3200 -> 256 3x3, 6 x 50x82 padded input) on MIOpen in the
layouts the step could hand it: data / weight gradients, NHWC vs NCHW, separately and together.

    python tools/micro_convbwd.py
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


def timed(fn, iters=10):
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
    dev = 'cuda'
    x = torch.randn(6, 3200, 50, 82, device=dev)
    w = torch.randn(256, 3200, 3, 3, device=dev) * 0.006
    g = torch.randn(6, 256, 48, 80, device=dev)
    flop = 2.0 * 6 * 48 * 80 * 256 * 3200 * 9
    cb = torch.ops.aten.convolution_backward
    for name, fmt in (('NCHW', torch.contiguous_format), ('NHWC', torch.channels_last)):
        xx, ww, gg = (t.contiguous(memory_format=fmt) for t in (x, w, g))
        for what, mask in (('dgrad', [True, False, False]), ('wgrad', [False, True, True]),
                           ('both', [True, True, True])):
            t = timed(lambda: cb(gg, xx, ww, [256], [1, 1], [0, 0], [1, 1], False, [0, 0], 1, mask))
            n = sum(mask[:2])
            print(f'{name} {what:5s} {t:7.3f} ms  ({n * flop / t / 1e9:6.1f} TFLOP/s)', flush=True)
    # mixed: NHWC grad/input, dgrad computed on NCHW copies (transposes included)
    xx, ww, gg = (t.contiguous(memory_format=torch.channels_last) for t in (x, w, g))

    def mixed():
        dx = cb(gg.contiguous(), xx, ww.contiguous(), [256], [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                [True, False, False])[0]
        return dx.contiguous(memory_format=torch.channels_last)
    print(f'mixed dgrad via NCHW (+transposes) {timed(mixed):7.3f} ms', flush=True)


if __name__ == '__main__':
    main()

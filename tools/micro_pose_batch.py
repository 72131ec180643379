"""Pose encoder + aggregation (fusion_posenet.py:42-67) forward+backward: the reference's two calls
per step (frame pairs (-1, 0) and (0, 1), 6 cameras each) against one call on both pairs stacked
(batch 12).  Times the device work per step with HIP events (config 2 shapes, fp32 nets).

    python tools/micro_pose_batch.py [--iters 10]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=10)
    a = ap.parse_args()
    import bench
    from vfdepth_amd import _lib, network
    _lib.load()
    cfg, _ = bench.make_cfg(2)
    net = network.FusedPoseNet(cfg).cuda().train()
    dev = 'cuda:0'
    imgs = [torch.rand(1, 6, 3, 384, 640, device=dev) for _ in range(3)]

    def two_calls():
        outs = []
        for p in ((0, 1), (1, 2)):
            x, normed = network._encoder_input([imgs[p[0]], imgs[p[1]]])
            _, agg = network._aggregate(net.encoder, net.conv1x1, x, net.fusion_level, 1, 6, normed)
            outs.append(agg)
        loss = sum(o.square().mean() for o in outs)
        loss.backward()

    def one_call():
        x0, n0 = network._encoder_input([imgs[0], imgs[1]])
        x1, _ = network._encoder_input([imgs[1], imgs[2]])
        x = torch.cat([x0, x1], 0)
        _, agg = network._aggregate(net.encoder, net.conv1x1, x, net.fusion_level, 2, 6, n0)
        loss = agg[0:1].square().mean() + agg[1:2].square().mean()
        loss.backward()

    for name, fn in (('two calls (B=6 each)', two_calls), ('one call (B=12)', one_call),
                     ('two calls (B=6 each)', two_calls), ('one call (B=12)', one_call)):
        for _ in range(3):
            net.zero_grad(set_to_none=True)
            fn()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(a.iters):
            net.zero_grad(set_to_none=True)
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        print(f'{name:24s} {ev[0].elapsed_time(ev[1]) / a.iters:8.3f} ms per step', flush=True)


if __name__ == '__main__':
    main()

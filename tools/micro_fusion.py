"""Micro-benchmark of the fusion kernels (K2 pose fwd/bwd, K3 fwd/bwd) at config-2 shapes.

    python tools/micro_fusion.py [--iters 20] [--ops pose,vproj]

Per-kernel device time from the C-ABI's HIP-event hooks; meant to run alone or under
rocprofv3 (--kernel-trace / --pmc) to study one kernel without the rest of the step."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from vfdepth_amd import _lib as L  # noqa: E402
from vfdepth_amd import config as C  # noqa: E402
from vfdepth_amd import kernels as KN  # noqa: E402
from vfdepth_amd import synth  # noqa: E402
from vfdepth_amd.geometry import inverse4x4  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--ops', default='pose,vproj')
    a = ap.parse_args()
    L.load()
    dev = torch.device('cuda:0')
    cfg = C.surround_fusion_cfg()
    space = KN.VoxelSpace(cfg, dev)
    b = synth.make_batch(cfg, seed=1, device=dev)
    Einv = inverse4x4(b['extrinsics'])
    lvl = cfg['model']['fusion_level'] + 1
    mask_lo = KN.mask_lowres(space, b['mask'])
    g = torch.Generator(device=dev).manual_seed(0)
    ops = a.ops.split(',')
    feats = torch.randn(1, 6, 256, space.h, space.w, device=dev, generator=g, requires_grad=True)
    vox = torch.randn(1, space.V, 64, device=dev, generator=g, requires_grad=True)
    gp = gv = None
    for it in range(a.iters + 2):
        if it == 2:
            torch.cuda.synchronize()
            L.prof_enable('all')
        if 'pose' in ops:
            plan = KN.FusionPlan(space, mask_lo, b['K', lvl], Einv)
            out = KN.FusePose.apply(space, plan, feats)
            if gp is None:
                gp = torch.randn(out.shape, device=dev, generator=g)
            out.backward(gp)
        if 'vproj' in ops:
            out = KN.VoxelProject.apply(space, vox, b['inv_K', lvl], b['extrinsics'])
            if gv is None:
                gv = torch.randn(out.shape, device=dev, generator=g)
            out.backward(gv)
    torch.cuda.synchronize()
    for k, (n, ms) in sorted(L.prof_read().items(), key=lambda kv: -kv[1][1]):
        if n:
            print(f'{k:20s} {n:4d} launches {1e3 * ms / n:9.1f} us/launch', flush=True)
    L.prof_enable('off')


if __name__ == '__main__':
    main()

"""Diagnostic: per-task timeline of the K2 backward (needs a VFD_PBW_TRACE variant library).

    python tools/build_variant.py trace -DVFD_PBW_TRACE
    VFD_LIB=variants/libvfd_trace.so python tools/diag_pbw_trace.py"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from vfdepth_amd import _lib as L  # noqa: E402
from vfdepth_amd import config as C  # noqa: E402
from vfdepth_amd import kernels as KN  # noqa: E402
from vfdepth_amd import synth  # noqa: E402
from vfdepth_amd.geometry import inverse4x4  # noqa: E402


def main():
    lib = L.load()
    dev = torch.device('cuda:0')
    cfg = C.surround_fusion_cfg()
    space = KN.VoxelSpace(cfg, dev)
    b = synth.make_batch(cfg, seed=1, device=dev)
    Einv = inverse4x4(b['extrinsics'])
    lvl = cfg['model']['fusion_level'] + 1
    mask_lo = KN.mask_lowres(space, b['mask'])
    g = torch.Generator(device=dev).manual_seed(0)
    feats = torch.randn(1, 6, 256, space.h, space.w, device=dev, generator=g, requires_grad=True)
    gp = None
    for it in range(4):
        plan = KN.FusionPlan(space, mask_lo, b['K', lvl], Einv)
        out = KN.FusePose.apply(space, plan, feats)
        if gp is None:
            gp = torch.randn(out.shape, device=dev, generator=g)
        out.backward(gp)
    torch.cuda.synchronize()
    raw = np.zeros(16384 * 4, dtype=np.uint64)
    fn = getattr(lib, 'vfd_pbw_trace_read')
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert fn(raw.ctypes.data, raw.nbytes) == 0
    r = raw.reshape(-1, 4)
    r = r[r[:, 1] > 0].astype(np.int64)
    t0 = r[:, 0].min()
    st, en = (r[:, 0] - t0) / 100.0, (r[:, 1] - t0) / 100.0     # us
    items, ng = r[:, 2] & 0xFFFFFF, r[:, 2] >> 24
    wg = r[:, 3] & 0xFFFF             # CU id
    dur = en - st
    print(f'tasks {len(r)}  span {en.max():.1f} us  items {items.sum()}')
    for k in (0, 1):                    # 1: a part of a split tile
        m = ng == k
        if m.any():
            rate = items[m] / dur[m]
            print(f'  S={k}: {m.sum():5d} tasks  items mean {items[m].mean():6.1f} max {items[m].max():5d}  '
                  f'dur mean {dur[m].mean():6.2f} max {dur[m].max():6.2f} us  items/us mean {rate.mean():6.1f}')
    ends = np.array([en[wg == w].max() for w in np.unique(wg)])
    busy = np.array([dur[wg == w].sum() for w in np.unique(wg)])
    print(f'  CUs {len(ends)}: end p50 {np.percentile(ends, 50):.1f} p90 {np.percentile(ends, 90):.1f} '
          f'max {ends.max():.1f} us; busy mean {busy.mean():.1f} us; first start max {st.max():.1f}')
    hist, edges = np.histogram(st, bins=10, range=(0, en.max()))
    print('  task starts per decile:', hist.tolist())
    order = np.argsort(-dur)[:10]
    for i in order:
        print(f'    slow task: items {items[i]} S {ng[i]} start {st[i]:.1f} dur {dur[i]:.2f} us')
    fit = np.polyfit(items, dur, 1)
    print(f'  dur ~ {fit[0] * 1e3:.2f} ns per item + {fit[1]:.2f} us')


if __name__ == '__main__':
    main()

"""Uninitialised-memory check of one eager training step: the caching allocator's memory is filled
with NaN bit patterns (0xFFFFFFFF) before the step, so any buffer a kernel reads before something
wrote it carries NaN.  Every autograd Function of vfdepth_amd.kernels is wrapped: after each
forward / backward the device is synchronised and the outputs are checked — the first op whose
inputs are NaN-free but whose outputs hold NaN names the kernel that reads (or leaves) uninitialised
memory.  ATen ops are checked the same way through a dispatch mode.

    python tools/diag_poison.py [--config 0] [--pairs 1]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
if os.path.isdir(os.path.join(ROOT, 'miopen_db')):
    sys.path.insert(0, ROOT)
    from vfdepth_amd.miopen_db import use_private_copy  # noqa: E402
    use_private_copy()

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

FIRST = []


def _nan(ts):
    bad = []
    for i, t in enumerate(ts):
        if torch.is_tensor(t) and t.is_cuda and t.is_floating_point() and t.numel():
            if bool(torch.isnan(t).any()):
                bad.append(i)
    return bad


def _flat(x):
    if isinstance(x, (list, tuple)):
        out = []
        for v in x:
            out += _flat(v)
        return out
    return [x]


def report(kind, name, ins, outs):
    torch.cuda.synchronize()
    if len(FIRST) >= 30:
        return
    bi, bo = _nan(_flat(ins)), _nan(_flat(outs))
    if bo and not bi:
        FIRST.append(f'{kind} {name}: NaN-free inputs, NaN in outputs {bo}')
        print('NaN PRODUCER:', FIRST[-1], flush=True)


def wrap_functions():
    from vfdepth_amd import kernels as KN
    for name in dir(KN):
        cls = getattr(KN, name)
        if not (isinstance(cls, type) and issubclass(cls, torch.autograd.Function) and cls is not torch.autograd.Function):
            continue
        for meth in ('forward', 'backward'):
            f = cls.__dict__.get(meth)
            if f is None:
                continue
            fn = f.__func__ if isinstance(f, staticmethod) else f

            def make(fn, nm):
                def wrapped(ctx, *a, **k):
                    out = fn(ctx, *a, **k)
                    report('fn', nm, a, out)
                    return out
                return staticmethod(wrapped)
            setattr(cls, meth, make(fn, f'{name}.{meth}'))


class AtenCheck(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        if len(FIRST) < 30 and 'fill' not in str(func) and 'empty' not in str(func):
            report('aten', str(func), list(args) + list((kwargs or {}).values()), out)
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', type=int, default=0)
    ap.add_argument('--pairs', type=int, default=1)
    ap.add_argument('--aten', type=int, default=1)
    a = ap.parse_args()
    os.environ['VFD_POSE_PAIRS'] = str(a.pairs)
    import bench
    from vfdepth_amd import _lib, synth
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.vfdepth import VFDepthAlgo
    _lib.load()
    if a.config < 0:                       # the graph-replay test's configuration
        import common as G
        cfg = G.step_cfg()
    else:
        cfg, name = bench.make_cfg(a.config)
    algo = VFDepthAlgo(cfg, 0)
    for m in algo.models.values():
        m.load_state_dict(seeded_state_dict(m, seed=7))
    algo.set_train()
    batch = synth.make_batch(cfg, seed=3, device='cuda:0')
    losses = algo.train_step(dict(batch))
    torch.cuda.synchronize()
    print('clean step', float(losses['total_loss']), flush=True)
    wrap_functions()
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info()
    poison = torch.empty(int(free * 0.7) // 4, dtype=torch.int32, device='cuda:0')
    poison.fill_(-1)
    # the small pool (blocks <= 1 MB, 2 MB segments) is separate: poison 4 GB of it too
    small = [torch.empty(256 * 1024, dtype=torch.int32, device='cuda:0') for _ in range(4096)]
    for t in small:
        t.fill_(-1)
    torch.cuda.synchronize()
    del poison, small
    algo.optimizer.zero_grad(set_to_none=True)
    if a.aten:
        with AtenCheck():
            _, losses = algo.process_batch(dict(batch), 0)
            losses['total_loss'].backward()
    else:
        _, losses = algo.process_batch(dict(batch), 0)
        losses['total_loss'].backward()
    torch.cuda.synchronize()
    bad = [n for n, p in ((n, p) for m in algo.models.values() for n, p in m.named_parameters())
           if p.grad is not None and bool(torch.isnan(p.grad).any())]
    print('poisoned step total_loss', float(losses['total_loss']), 'NaN grads in', len(bad), 'params', bad[:5], flush=True)
    print('NaN producers:', len(FIRST), flush=True)
    for f in FIRST:
        print('  ', f, flush=True)


if __name__ == '__main__':
    main()

"""Capture the DEFAULT training step (batched frame pairs, pose branch on its own stream) as a HIP
graph and replay it, with a device synchronisation and a line after every stage, so a crash or a
fault is attributed to its stage; a native stack is printed on SIGSEGV (tools/segv_bt.so).

    python tools/diag_capture.py [--ddp] [--config 0|2] [--replays 2]
"""
import argparse
import ctypes
import faulthandler
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
from vfdepth_amd.miopen_db import use_private_copy  # noqa: E402
use_private_copy()

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def stage(name):
    torch.cuda.synchronize()
    print(f'ok: {name}', flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--ddp', action='store_true')
    ap.add_argument('--config', type=int, default=0)
    ap.add_argument('--replays', type=int, default=2)
    ap.add_argument('--no-opt', action='store_true', help='capture without the optimizer step (race diagnostics)')
    ap.add_argument('--compare', action='store_true',
                    help='rewind to the initial state, one replay vs one eager step: per-net / per-parameter '
                         'gradient differences (and an eager-vs-eager pair)')
    a = ap.parse_args()
    import common as G
    import bench
    from vfdepth_amd import _lib, synth
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.vfdepth import VFDepthAlgo
    _lib.load()
    if a.ddp:
        with socket.socket() as s:
            s.bind(('127.0.0.1', 0))
            port = s.getsockname()[1]
        os.environ.setdefault('TORCH_NCCL_ASYNC_ERROR_HANDLING', '0')
        os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
        dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1)
    cfg = G.step_cfg() if a.config == 0 else bench.make_cfg(a.config)[0]
    cfg['ddp'].update({'ddp_enable': a.ddp, 'world_size': 1, 'gpus': [0], 'graph_capture': a.ddp})
    batch = synth.make_batch(cfg, seed=99, device='cuda:0')
    algo = VFDepthAlgo(cfg, 0)
    for m in algo.models.values():
        inner = getattr(m, 'module', m)
        inner.load_state_dict(seeded_state_dict(inner, seed=G.STEP_SEED))
    algo.set_train()
    algo.set_optimizer(capturable=True)
    algo.losses.device_seed = True
    if a.no_opt:
        algo.optimizer.step = lambda *args, **kw: None
    le = algo.train_step(dict(batch))
    # crash diagnostics installed after the runtimes set theirs: faulthandler prints the Python
    # stack, then re-raises into the native-stack handler (tools/segv_bt.so)
    bt = os.path.join(ROOT, 'tools', 'segv_bt.so')
    if os.path.isfile(bt):
        ctypes.CDLL(bt).segv_bt_install()
    faulthandler.enable()
    os.environ['VFD_GRAPH_TRACE'] = '1'
    stage(f'eager step: total_loss {float(le["total_loss"]):.6f}')
    graphed = algo.graphed_train_step(batch, warmup=2)
    stage(f'capture (branch stream used: {getattr(algo, "_bstream", None) is not None}, pairs batched: {algo.pose.batch_pairs})')
    for i in range(a.replays):
        losses = graphed()
        stage(f'replay {i}: total_loss {float(losses["total_loss"]):.6f}')
    if a.compare:     # before any eager step: that would replace the .grad tensors the graph writes
        compare(algo, graphed, batch, G, seeded_state_dict)
    le = algo.train_step(dict(batch))
    stage(f'eager step after replays: total_loss {float(le["total_loss"]):.6f}')
    if a.ddp:
        dist.destroy_process_group()


def compare(algo, graphed, batch, G, seeded_state_dict):
    def rewind():
        for m in algo.models.values():
            inner = getattr(m, 'module', m)
            inner.load_state_dict(seeded_state_dict(inner, seed=G.STEP_SEED))
        for st in algo.optimizer.state.values():
            for t in st.values():
                if torch.is_tensor(t):
                    t.zero_()
        algo.losses._counter.zero_()

    def grads():
        return {n: {k: p.grad.detach().clone() for k, p in getattr(m, 'module', m).named_parameters()
                    if p.grad is not None} for n, m in algo.models.items()}
    rewind()
    lg = {k: float(v) for k, v in graphed().items() if torch.is_tensor(v) and v.numel() == 1}
    torch.cuda.synchronize()
    gg = grads()
    res = []
    for i in range(2):
        rewind()
        algo.optimizer.zero_grad(set_to_none=True)
        _, le = algo.process_batch(dict(batch), 0)
        le['total_loss'].backward()
        torch.cuda.synchronize()
        res.append(({k: float(v) for k, v in le.items() if torch.is_tensor(v) and v.numel() == 1}, grads()))
    (le1, ge1), (le2, ge2) = res
    print('losses graph / eager / eager2:', {k: (round(lg[k], 7), round(le1[k], 7), round(le2[k], 7))
                                            for k in ('total_loss', 'reproj_loss', 'smooth')}, flush=True)
    for net in gg:
        def rel(a, b):
            num = sum(float((a[k].double() - b[k].double()).pow(2).sum()) for k in b)
            den = sum(float(b[k].double().pow(2).sum()) for k in b)
            return (num / max(den, 1e-300)) ** 0.5
        print(f'{net}: graph vs eager {rel(gg[net], ge1[net]):.3g}, eager vs eager {rel(ge2[net], ge1[net]):.3g}',
              flush=True)
        worst = sorted(((float((gg[net][k] - ge1[net][k]).norm() / max(float(ge1[net][k].norm()), 1e-30)), k)
                        for k in ge1[net]), reverse=True)[:8]
        for r, k in worst:
            print(f'    {k}: rel {r:.3g} |g| {float(ge1[net][k].norm()):.3g} graph {float(gg[net][k].norm()):.3g}'
                  f' eager2 {float((ge2[net][k] - ge1[net][k]).norm() / max(float(ge1[net][k].norm()), 1e-30)):.3g}')


if __name__ == '__main__':
    main()

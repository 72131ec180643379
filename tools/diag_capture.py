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
        dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1)
    cfg = G.step_cfg() if a.config == 0 else bench.make_cfg(a.config)[0]
    cfg['ddp'].update({'ddp_enable': a.ddp, 'world_size': 1, 'gpus': [0]})
    batch = synth.make_batch(cfg, seed=99, device='cuda:0')
    algo = VFDepthAlgo(cfg, 0)
    for m in algo.models.values():
        inner = getattr(m, 'module', m)
        inner.load_state_dict(seeded_state_dict(inner, seed=G.STEP_SEED))
    algo.set_train()
    algo.set_optimizer(capturable=True)
    algo.losses.device_seed = True
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
    stage(f'capture (branch stream used: {algo._bstream is not None}, pairs batched: {algo.pose.batch_pairs})')
    for i in range(a.replays):
        losses = graphed()
        stage(f'replay {i}: total_loss {float(losses["total_loss"]):.6f}')
    le = algo.train_step(dict(batch))
    stage(f'eager step after replays: total_loss {float(le["total_loss"]):.6f}')
    if a.ddp:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()

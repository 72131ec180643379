"""Multi-process (world_size 2, gloo, CPU) rehearsal of the data-parallel path.

The hot-path kernels need the MI355X, so these tests cover what the N>1 path adds around them:
the DDP + SyncBatchNorm wrapping of both nets (vfdepth.py:56-71 in the reference), DDP's gradient
all-reduce (the one collective of the step, RCCL on the GPU box, gloo here) on a net whose
forward runs on CPU, and the bench's max-over-ranks job time and whole-job throughput."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.set_num_threads(2)


def _ddp_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    try:
        _init(rank, world, port)
        from vfdepth_amd import config as C
        from vfdepth_amd.layers import seeded_state_dict
        from vfdepth_amd.vfdepth import VFDepthAlgo
        from torch.nn.parallel import DistributedDataParallel as DDP
        cfg = C.mono_cfg(batch_size=1, height=64, width=96)
        cfg['ddp'].update({'ddp_enable': True, 'world_size': world, 'gpus': list(range(world))})
        algo = VFDepthAlgo(cfg, 'cpu')
        nets = algo.models
        wrapped = {k: isinstance(v, DDP) for k, v in nets.items()}
        # CPU modules keep BatchNorm (torch's SyncBatchNorm is GPU-only); the GPU path converts
        sync_bn = {k: not any(isinstance(m, torch.nn.SyncBatchNorm) for m in v.modules()) and
                   any(isinstance(m, torch.nn.BatchNorm2d) for m in v.modules()) for k, v in nets.items()}
        depth = nets['depth_net']
        depth.module.load_state_dict(seeded_state_dict(depth.module, seed=3))
        depth.eval()                     # per-rank BN statistics out of the comparison
        x = torch.rand(1, 3, 64, 96, generator=torch.Generator().manual_seed(100 + rank))
        out = depth(x)
        loss = sum(v.float().mean() for v in out.values()) if isinstance(out, dict) else out.mean()
        loss.backward()
        g_ddp = torch.cat([p.grad.flatten() for p in depth.module.parameters() if p.grad is not None])
        # the same net without DDP on this rank's input: its local gradient
        ref = type(depth.module)(cfg)
        ref.load_state_dict(seeded_state_dict(ref, seed=3))
        ref.eval()
        out_r = ref(x)
        loss_r = sum(v.float().mean() for v in out_r.values()) if isinstance(out_r, dict) else out_r.mean()
        loss_r.backward()
        g_loc = torch.cat([p.grad.flatten() for p in ref.parameters() if p.grad is not None])
        g_all = [torch.zeros_like(g_loc) for _ in range(world)]
        dist.all_gather(g_all, g_loc)
        g_mean = torch.stack(g_all).mean(0)
        g_peer = [torch.zeros_like(g_ddp) for _ in range(world)]
        dist.all_gather(g_peer, g_ddp)
        q.put((rank, wrapped, sync_bn, float((g_ddp - g_mean).abs().max()), float(g_mean.abs().max()),
               float((g_peer[0] - g_peer[1]).abs().max())))
        dist.destroy_process_group()
    except Exception as e:                # surface the failure in the parent
        q.put((rank, 'error', repr(e)))
        raise


def _bench_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    _init(rank, world, port)
    import bench
    elapsed = 1.5 if rank == 1 else 1.0
    job = bench.max_over_ranks(elapsed, world, 'cpu')
    q.put((rank, job, bench.job_throughput(job, steps=20, world=world)))
    dist.destroy_process_group()


def _run(worker, world=2):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] != 'error', f'rank {r[0]} failed: {r[2]}'
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return sorted(res)


def test_ddp_gradient_allreduce_gloo_world2():
    for rank, wrapped, sync_bn, err, scale, peer in _run(_ddp_worker):
        assert all(wrapped.values()), wrapped          # both nets DDP-wrapped, as the reference does
        assert all(sync_bn.values()), sync_bn          # CPU rehearsal: plain BatchNorm kept
        assert err <= 1e-6 * max(scale, 1e-12) + 1e-9, (rank, err, scale)   # DDP grad == mean of local grads
        assert peer == 0.0, (rank, peer)               # every rank holds the same averaged gradient


def test_bench_job_time_is_max_over_ranks():
    for rank, job, thr in _run(_bench_worker):
        assert job == 1.5, (rank, job)
        assert abs(thr - 20 * 2 / 1.5) < 1e-9, (rank, thr)

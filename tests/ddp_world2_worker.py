"""One rank of the world-size-2 SyncBatchNorm / DDP check on ONE MI355X (tests/test_gpu_0_ddp_world2.py).

Both ranks run on cuda:0 over a gloo group (CUDA tensors; gloo stages them through the host, RCCL
does not run two ranks on one device).  What it checks (reference: models/vfdepth.py:56-71
convert_sync_batchnorm + DDP(broadcast_buffers=True), utils/ddp.py:10-29):

1. the fused BatchNorm(+residual)(+ReLU) kernels' synchronised branch (bnact.hip, one all-reduce per
   direction with the element count as an extra row): each rank's half of a 4-image batch gives the
   outputs, running statistics and input / residual gradients of nn.BatchNorm2d.train() on the
   whole batch (fp64 CPU), and the ranks' local d gamma / d beta sum to the whole batch's;
2. the fusion training step under DDP + SyncBatchNorm: DDP's gradients are identical on both ranks
   and equal the mean over ranks of the gradients the same SyncBatchNorm nets give without DDP;
   BatchNorm running statistics are identical on both ranks.

Usage: RANK=r WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=p python tests/ddp_world2_worker.py
Prints one line 'OK <summary>' and exits 0, or raises.
"""
import datetime
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests', 'golden')]
# deterministic mode (fixed-order sums in the fusion kernels; MIOpen without its split-K atomic
# solvers — read once, before the process's first convolution): the DDP and the local step then
# run bit-identical forwards, so their gradients differ only by DDP's averaging
os.environ['MIOPEN_DEBUG_CONVOLUTION_DETERMINISTIC'] = '1'
os.environ['VFD_DETERMINISTIC'] = '1'

import torch                       # noqa: E402
import torch.distributed as dist   # noqa: E402

DEV = torch.device('cuda:0')


def bn_layer_checks(rank, world):
    from vfdepth_amd.layers import bn_act
    worst = 0.0
    # (full batch shape, residual, relu): a layer1 tail, a downsample BN, a 1/32 layer (which the
    # local path would run as the one-launch kernel), HW % 4 != 0
    for shape, res, relu in (((4, 64, 24, 40), True, True), ((4, 128, 12, 20), False, False),
                             ((4, 256, 6, 10), True, True), ((4, 8, 5, 7), True, True)):
        C = shape[1]
        gen = torch.Generator().manual_seed(11 + C)
        x = 2.0 * torch.randn(shape, generator=gen, dtype=torch.float64) + 0.5
        r = torch.randn(shape, generator=gen, dtype=torch.float64) if res else None
        g = torch.randn(shape, generator=gen, dtype=torch.float64)
        gamma = 1 + 0.1 * torch.randn(C, generator=gen, dtype=torch.float64)
        beta = 0.1 * torch.randn(C, generator=gen, dtype=torch.float64)
        rmean = 0.2 * torch.randn(C, generator=gen, dtype=torch.float64)
        # reference: the whole batch through nn.BatchNorm2d.train() in fp64 on the CPU
        ref = torch.nn.BatchNorm2d(C).double().train()
        with torch.no_grad():
            ref.weight.copy_(gamma)
            ref.bias.copy_(beta)
            ref.running_mean.copy_(rmean)
        xr = x.clone().requires_grad_(True)
        rr = r.clone().requires_grad_(True) if res else None
        yr = ref(xr)
        if res:
            yr = yr + rr
        if relu:
            yr = torch.relu(yr)
        (yr * g).sum().backward()
        # this rank's half on the GPU through a SyncBatchNorm module (fused synchronised path), NCHW
        # and channels-last (bnact.hip's NHWC kernels), fp32 and — config 3's encoders — bf16
        # channels-last maps (fp32 statistics and arithmetic, outputs / input gradients rounded once)
        for fmt, dt in ((torch.contiguous_format, torch.float32), (torch.channels_last, torch.float32),
                        (torch.channels_last, torch.bfloat16)):
            bf = dt == torch.bfloat16
            half = slice(rank * shape[0] // world, (rank + 1) * shape[0] // world)
            bn = torch.nn.SyncBatchNorm(C).to(DEV).train()
            with torch.no_grad():
                bn.weight.copy_(gamma.float())
                bn.bias.copy_(beta.float())
                bn.running_mean.copy_(rmean.float())
            xh = x[half].to(dt).to(DEV).contiguous(memory_format=fmt).requires_grad_(True)
            rh = r[half].to(dt).to(DEV).contiguous(memory_format=fmt).requires_grad_(True) if res else None
            # bf16 maps take the fused path under config 3's bf16 autocast (layers._fused_dtype_ok)
            with torch.autocast('cuda', dtype=torch.bfloat16, enabled=bf):
                y = bn_act(bn, xh, rh, relu)
            assert y.grad_fn is not None and 'BatchNormAct' in type(y.grad_fn).__name__, type(y.grad_fn).__name__
            assert y.is_contiguous(memory_format=fmt) and y.dtype == dt
            (y.float() * g[half].to(dt).float().to(DEV)).sum().backward()
            torch.cuda.synchronize()
            if bf:
                # the bf16 check runs against the same fp64 reference on the bf16-rounded inputs
                # (statistics of the rounded maps), at bf16 output precision
                xb = x.to(dt).double().requires_grad_(True)
                rb = r.to(dt).double().requires_grad_(True) if res else None
                refb = torch.nn.BatchNorm2d(C).double().train()
                with torch.no_grad():
                    refb.weight.copy_(gamma.float().double())
                    refb.bias.copy_(beta.float().double())
                    refb.running_mean.copy_(rmean.float().double())
                yb = refb(xb)
                if res:
                    yb = yb + rb
                if relu:
                    yb = torch.relu(yb)
                (yb * g.to(dt).double()).sum().backward()

            def err(a, b, what, tol):
                nonlocal worst
                a, b = a.detach().double().cpu(), b.detach().double().cpu()
                e = float((a - b).abs().max()) / max(float(b.abs().max()), 1e-12)
                worst = max(worst, e)
                assert e <= tol, f'rank {rank} {shape} {fmt}: {what} rel err {e:.3g} > {tol}'
            if bf:
                e8 = 2.0 ** -7          # one bf16 rounding of the output / gradient (+ fp32 sums)
                err(y, yb[half], 'bf16 output', e8)
                err(bn.running_mean, refb.running_mean, 'bf16 running_mean', 1e-5)
                err(bn.running_var, refb.running_var, 'bf16 running_var', 1e-5)
                err(xh.grad, xb.grad[half], 'bf16 d input', 2 * e8)
                if res:
                    err(rh.grad, rb.grad[half], 'bf16 d residual', e8)
                dg, db = bn.weight.grad.clone(), bn.bias.grad.clone()
                dist.all_reduce(dg)
                dist.all_reduce(db)
                err(dg, refb.weight.grad, 'bf16 sum over ranks of d gamma', 1e-3)
                err(db, refb.bias.grad, 'bf16 sum over ranks of d beta', 1e-3)
                continue
            err(y, yr[half], 'output', 2e-6)
            err(bn.running_mean, ref.running_mean, 'running_mean', 1e-6)
            err(bn.running_var, ref.running_var, 'running_var', 1e-6)
            assert int(bn.num_batches_tracked) == 1
            err(xh.grad, xr.grad[half], 'd input', 2e-5)
            if res:
                err(rh.grad, rr.grad[half], 'd residual', 1e-6)
            # SyncBatchNorm's parameter gradients are this rank's local sums: they add up to the whole batch's
            dg, db = bn.weight.grad.clone(), bn.bias.grad.clone()
            dist.all_reduce(dg)
            dist.all_reduce(db)
            err(dg, ref.weight.grad, 'sum over ranks of d gamma', 2e-5)
            err(db, ref.bias.grad, 'sum over ranks of d beta', 2e-5)
    return worst


def _grads(models):
    out = {}
    for name, m in models.items():
        inner = m.module if hasattr(m, 'module') else m
        for k, p in inner.named_parameters():
            if p.grad is not None:
                out[f'{name}.{k}'] = p.grad.detach().clone()
    return out


def _bn_stats(models):
    out = {}
    for name, m in models.items():
        inner = m.module if hasattr(m, 'module') else m
        for k, b in inner.named_buffers():
            if 'running' in k:
                out[f'{name}.{k}'] = b.detach().clone()
    return out


def step_checks(rank, world, bf16=False):
    """bf16=True: config 3's precision — bf16 nets under autocast with channels-last encoders (the
    NHWC bf16 SyncBatchNorm branch inside a DDP step), B = 2 per rank."""
    import common as G
    from torch.nn.parallel import DistributedDataParallel as DDP
    from vfdepth_amd import kernels as KN
    from vfdepth_amd import synth
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.vfdepth import VFDepthAlgo

    def make_cfg():
        c = G.step_cfg()
        if bf16:
            c['training'].update(net_precision='bf16', batch_size=2)
        return c
    cfg = make_cfg()
    B = cfg['training']['batch_size']
    inputs = synth.make_batch(cfg, seed=50 + rank, device=DEV)        # each rank its own samples
    noise = 1e-5 * torch.randn(6, B, 2, cfg['training']['height'], cfg['training']['width'],
                               generator=torch.Generator().manual_seed(60 + rank)).to(DEV)

    def run(ddp):
        c = make_cfg()
        c['ddp'].update({'ddp_enable': ddp, 'world_size': world, 'gpus': list(range(world))})
        algo = VFDepthAlgo(c, DEV)
        for m in algo.models.values():
            inner = m.module if hasattr(m, 'module') else m
            inner.load_state_dict(seeded_state_dict(inner, seed=G.STEP_SEED))
        if not ddp:     # the same SyncBatchNorm nets without DDP: synchronised statistics, local gradients
            algo.models = {k: torch.nn.SyncBatchNorm.convert_sync_batchnorm(v) for k, v in algo.models.items()}
        algo.set_train()
        _, losses = algo.process_batch({k: v.clone() if torch.is_tensor(v) else v for k, v in inputs.items()},
                                       rank, noise=noise)
        losses['total_loss'].backward()
        torch.cuda.synchronize()
        return algo, losses
    run(False)                  # warm-up: MIOpen's solver picks on first use
    KN.syncbn_stats(reset=True)
    algo_d, loss_d = run(True)
    sbn = KN.syncbn_stats(reset=True)
    assert sbn['calls'] > 0, 'the DDP step issued no SyncBatchNorm collective'
    assert all(isinstance(m, DDP) for m in algo_d.models.values())
    if bf16:                    # the encoders really run channels-last bf16 (the NHWC SyncBN kernels)
        encs = [m.module.encoder for m in algo_d.models.values() if hasattr(m.module, 'encoder')]
        assert encs and all(e.channels_last for e in encs)
    for m in algo_d.models.values():
        assert any(isinstance(x, torch.nn.SyncBatchNorm) for x in m.module.modules())
        assert not any(type(x) is torch.nn.BatchNorm2d for x in m.module.modules())
    g_ddp, s_ddp = _grads(algo_d.models), _bn_stats(algo_d.models)
    algo_l, loss_l = run(False)
    g_loc, s_loc = _grads(algo_l.models), _bn_stats(algo_l.models)
    assert torch.equal(loss_d['total_loss'], loss_l['total_loss']), (float(loss_d['total_loss']), float(loss_l['total_loss']))
    keys = sorted(g_loc)
    assert keys == sorted(g_ddp), 'DDP and local steps produced gradients for different parameters'
    flat_d = torch.cat([g_ddp[k].flatten() for k in keys])
    flat_l = torch.cat([g_loc[k].flatten() for k in keys])
    peers = [torch.empty_like(flat_d) for _ in range(world)]
    dist.all_gather(peers, flat_d)
    assert torch.equal(peers[0], peers[1]), 'DDP gradients differ between ranks'
    locs = [torch.empty_like(flat_l) for _ in range(world)]
    dist.all_gather(locs, flat_l)
    assert not torch.equal(locs[0], locs[1]), 'the ranks saw identical local gradients (same data?)'
    mean = torch.stack(locs).mean(0)
    rel = float((flat_d - mean).double().norm() / mean.double().norm())
    # deterministic mode: the same local gradients on both paths; DDP's bucketed average rounds
    # differently from torch.stack(...).mean(0) only in the last bit
    assert rel <= 1e-6, f'DDP gradient vs mean of local gradients: rel {rel:.3g}'
    for k in sorted(s_ddp):
        peers = [torch.empty_like(s_ddp[k]) for _ in range(world)]
        dist.all_gather(peers, s_ddp[k])
        assert torch.equal(peers[0], peers[1]), f'{k} differs between ranks'
        e = float((s_ddp[k] - s_loc[k]).abs().max())
        assert e <= 1e-5 * max(float(s_loc[k].abs().max()), 1.0), f'{k}: DDP vs local-step statistics {e:.3g}'
    return rel, len(keys), sbn


def main():
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    torch.cuda.set_device(DEV)
    # a failed peer ends this rank within two minutes instead of gloo's 30-minute default
    dist.init_process_group('gloo', rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    from vfdepth_amd import _lib
    _lib.load()
    worst = bn_layer_checks(rank, world)
    rel, n, sbn = step_checks(rank, world)
    rel3, n3, sbn3 = step_checks(rank, world, bf16=True)
    dist.barrier()
    dist.destroy_process_group()
    print(f'OK rank {rank}: syncbn worst rel err {worst:.3g}; DDP step {n} gradients, rel vs mean of local {rel:.3g} '
          f'({sbn["calls"]} SyncBN all-reduces, {sbn["bytes"] / 1e3:.1f} KB, {sbn["host_s"] * 1e3:.1f} ms host); '
          f'bf16 channels-last B=2 DDP step {n3} gradients, rel {rel3:.3g} ({sbn3["calls"]} all-reduces, '
          f'{sbn3["host_s"] * 1e3:.1f} ms host)', flush=True)


if __name__ == '__main__':
    main()

#!/usr/bin/env python
"""VFDepth 6-camera training-step benchmark (BASELINE.json metric) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

One step = process_batch (pose nets x2, depth net, view synthesis, losses) + backward + Adam on
one synthetic DDAD-shaped batch that is already resident in HBM.  K timed steps between
barriers + device syncs, max over ranks; rank 0 prints ONE JSON line.  `value` = iterations
summed over ranks per second (batch per rank as configured; weak scaling).

roofline: the hot-path kernel with the largest device time in the timed steps, timed with HIP
events around each of its launches on its stream (C-ABI hook), against its algorithmic bytes
per launch ("Roofline accounting").  cpu_baseline: the CPU oracle (oracle/, a
restatement of the reference step) timed for a bounded sample on this host's cores (rank 0).
"""
import argparse
import faulthandler
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
# MIOpen's user find/perf database: a committed one (tuned on MI355X) makes conv-solver choice
# reproducible and skips the per-shape search on a fresh box.  Must be set before MIOpen loads; a
# private copy per process, so records other runs write never reach the committed picks
# (vfdepth_amd/miopen_db.py).
sys.path.insert(0, ROOT)
from vfdepth_amd.miopen_db import use_private_copy  # noqa: E402
use_private_copy()

import threading  # noqa: E402

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, ROOT)

from vfdepth_amd import _lib  # noqa: E402
from vfdepth_amd import config as C  # noqa: E402
from vfdepth_amd import synth  # noqa: E402
from vfdepth_amd.layers import seeded_state_dict  # noqa: E402

HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
MFMA_F32_PEAK_TFS = 157.3  # dense fp32-input MFMA (v_mfma_f32_32x32x2_f32), MI355X_MICROARCH.md
MFMA_BF16_PEAK_TFS = 2516.6  # dense bf16 MFMA (v_mfma_f32_32x32x16_bf16: 16x the fp32 rate, ~2.5 PF)


def max_over_ranks(elapsed, world, device):
    """The slowest rank's time (the job's time): all-reduce MAX over the process group."""
    if world <= 1:
        return elapsed
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t)


def job_throughput(elapsed, steps, world, batch_per_rank=1):
    """Whole-job iterations/s: every rank runs `steps` iterations of `batch_per_rank` samples
    (weak scaling); divided by the slowest rank's time."""
    return steps * world * batch_per_rank / elapsed


def make_cfg(config, batch=None):
    if config == 0:
        # the reduced 6-camera fusion step of the parity fixtures (tests/golden/common.step_cfg):
        # multi-rank plumbing rehearsals, not a bench line
        cfg = C.surround_fusion_cfg(height=96, width=160, batch_size=batch or 1, voxel_size=[40, 40, 10],
                                    voxel_unit_size=[2.5, 2.5, 3.0], voxel_str_p=[-50.0, -50.0, -15.0],
                                    proj_d_bins=16, focal_length_scale=30)
        name = 'reduced 6-cam 96x160 fusion, voxel 40x40x10, D=16, fp32 (rehearsal)'
    elif config == 2:
        cfg = C.surround_fusion_cfg(batch_size=batch or 1)
        name = '6-cam DDAD 384x640 fusion, voxel 100x100x20, D=50, fp32'
    elif config == 3:
        cfg = C.surround_fusion_cfg(batch_size=batch or 2, net_precision='bf16')
        name = '6-cam DDAD 384x640 fusion, B=2/GPU, bf16 nets, fp32 fusion/geometry/loss kernels'
    elif config == 4:
        cfg = C.surround_fusion_cfg(batch_size=batch or 1, height=352, width=640, max_depth=80.0,
                                    cameras=list(C.NUSC_CAMERAS))
        name = 'NuScenes 6-cam 352x640 fusion, fp32'
    elif config == 5:
        cfg = C.surround_fusion_cfg(batch_size=batch or 4, height=640, width=960, voxel_size=[200, 200, 20],
                                    voxel_unit_size=[0.5, 0.5, 1.5])
        name = f'6-cam 640x960, voxel 200x200x20 @0.5m, B={batch or 4}/GPU, fp32'
    else:
        raise SystemExit(f'unknown config {config}')
    return cfg, name


def shapes(cfg):
    m, t = cfg['model'], cfg['training']
    lvl = m['fusion_level']
    H, W = t['height'], t['width']
    X, Y, Z = m['voxel_size']
    return dict(B=t['batch_size'], N=cfg['data']['num_cams'], C=m['fusion_feat_in_dim'], Cv=m['voxel_pre_dim'][-1],
                H=H, W=W, h=H // 2 ** (lvl + 1), w=W // 2 ** (lvl + 1), X=X, Y=Y, Z=Z, V=X * Y * Z,
                D=m['proj_d_bins'], T=len(t['frame_ids']) - 1, F=len(t['frame_ids']))


def algorithmic_bytes(kernel, s):
    """Compulsory HBM bytes of ONE launch at the kernel's own boundary (fp32 = 4 B; the pose BEV
    map 2 B where K2 writes it in bf16, s['map_bytes']), with the unpadded tensor sizes of
    SURVEY.md §8(d) (the reflect-pad halos the K2/K3 kernels also write for the consumer convs are
    NOT counted: they are extra work, not algorithmic bytes)."""
    B, N, C, Cv, p, P = s['B'], s['N'], s['C'], s['Cv'], s['h'] * s['w'], s['H'] * s['W']
    V, D, T, F = s['V'], s['D'], s['T'], s['F']
    pose_out = B * (C + 1) * V                                    # [B, C+1, V] mean voxel features
    proj_out = B * N * Cv * D * p                                 # [B*N, Cv*D, h, w] frustum features
    h, w = s['h'], s['w']
    agg_levels = (h // 2) * (w // 2) + (h // 4) * (w // 4)
    planes = {
        'mask_downsample': B * N * (P + p),
        'fusion_plan': B * N * p + B * V * 8,                     # mask in, ~one 32-B entry per voxel out
        'aggregate': B * N * C * (2 * p + agg_levels),
        'fuse_depth_fwd': B * N * p * (2 * Cv + 1) + B * V * Cv,  # folded maps + 1/8 mask in, voxels out
        'fuse_depth_bwd': 2 * B * V * Cv + B * N * p + B * N * p * 2 * Cv,
        'fuse_pose_fwd': B * N * C * p + B * N * p + pose_out,    # SURVEY §8(d) K2 per call
        'fuse_pose_bwd': pose_out + B * N * C * p,
        'voxel_project_fwd': B * V * Cv + proj_out,
        'voxel_project_bwd': proj_out + B * V * Cv,
        'voxel_project_plan': 4 * B * N * p * D,                  # one 16-B sorted entry per frustum sample
        'view_stats': B * N * P * (1 + 3 * (T + 1) + 1),
        'view_apply': B * N * P * (1 + 3 * (T + 1) + 1) + B * N * P * (4 * T + 4 * F),
        'view_bwd': B * N * P * (1 + 3 * (T + 1) + 1) + B * N * P * 3 * (T + F) + B * N * P,
        'photo_fwd': B * N * P * (3 + 6 * T + 4 * F + 1) + B * N * P * 3 + B * N * P // 4,
        'photo_bwd': B * N * P * (3 + 3 * T + 4 * F + 1) + B * N * P // 4 + B * N * P * 3 * (T + F),
        'smooth_fwd': B * N * P * 4,
        'smooth_bwd': B * N * P * 5,
        'proj_conv_fwd': B * V * Cv + B * N * p * 256,            # voxels in, reduce_dim[0] output out
        'proj_conv_dgrad': B * N * p * 256 + proj_out,            # d pre-activation in, d frustum features out
        'pad_conv_fwd': pose_out + B * 256 * pose_hw(s),          # BEV map in, reduce_dim[0] out
        'depth_syn_fwd': B * N * P * 3 + 2 * B * N * 3 * P,        # depths + mask in, 3 sources x (depth, mask) out
        'depth_syn_bwd': B * N * P * 3 + B * N * 3 * P + 2 * B * N * P,
    }
    # K2C runs once over the stacked frame pairs (geometry.Pose's batched pairs): pose_pairs samples
    # of B per launch (K2 itself still launches per pair)
    k2c = s.get('pose_pairs', 1) if kernel == 'pad_conv_fwd' else 1
    if kernel in ('fuse_pose_fwd', 'pad_conv_fwd') and s.get('map_bytes', 4) != 4:
        return ((planes[kernel] - pose_out) * 4 + pose_out * s['map_bytes']) * k2c
    return planes[kernel] * 4 * k2c


def pose_hw(s):
    """Output pixels of the pose reduce_dim's first conv (3x3 stride 2 on the padded Y x X map)."""
    return ((s['Y'] - 1) // 2 + 1) * ((s['X'] - 1) // 2 + 1)


def mfma_flops(kernel, s):
    """Dense fp32 MFMA flops of one launch of the matrix-bound ops (None for the HBM-bound ones):
    K3C = reduce_dim's first conv, 2 * pixels * 256 * (Cv * D * 9); its data and weight gradients
    the same; K2C = the pose reduce_dim's first conv."""
    if kernel in ('proj_conv_fwd', 'proj_conv_dgrad', 'proj_conv_wgrad'):
        return 2.0 * s['B'] * s['N'] * s['h'] * s['w'] * 256 * s['Cv'] * s['D'] * 9
    if kernel in ('pad_conv_fwd', 'pad_conv_dgrad', 'pad_conv_wgrad'):   # K2C, pose reduce_dim[0]: K = (C+1)*Z*9
        # one launch over the stacked frame pairs (pose_pairs x B samples)
        return 2.0 * s['B'] * s.get('pose_pairs', 1) * pose_hw(s) * 256 * (s['C'] + 1) * s['Z'] * 9
    return None


def cpu_threads():
    """all cores of this process's affinity mask — capped by OMP_NUM_THREADS when
    the host sets it (the GPU pool gives each 1-GPU job a 16-thread CPU share and exports
    OMP_NUM_THREADS=16; `sched_getaffinity` there shows the whole machine)."""
    aff = len(os.sched_getaffinity(0))
    cap = os.environ.get('OMP_NUM_THREADS')
    return (min(aff, int(cap)) if cap and cap.isdigit() and int(cap) > 0 else aff), aff


def cpu_baseline(cfg, timed_steps=3, warmup_steps=1):
    """The CPU oracle's training step (forward + losses + backward + Adam; oracle/vfd_oracle.py,
    the reference's algorithm restated on torch CPU) at the per-GPU batch shape, B=1:
    `warmup_steps` untimed + `timed_steps` timed (1 + 3 for config 2)."""
    from oracle import vfd_oracle as O
    from vfdepth_amd.network import FusedDepthNet, FusedPoseNet
    threads, aff = cpu_threads()
    torch.set_num_threads(threads)
    dn, pn = FusedDepthNet(cfg), FusedPoseNet(cfg)
    dn.load_state_dict(seeded_state_dict(dn, seed=7))
    pn.load_state_dict(seeded_state_dict(pn, seed=7))
    nets = O.nets_from_modules(dn, pn)
    opt = torch.optim.Adam(list(dn.parameters()) + list(pn.parameters()), 1e-4)
    inputs = synth.make_batch(cfg, seed=1234, batch_size=1)
    N, T = cfg['data']['num_cams'], len(cfg['training']['frame_ids']) - 1
    H, W = cfg['training']['height'], cfg['training']['width']
    noise = [1e-5 * torch.randn(1, T, H, W) for _ in range(N)]
    times = []
    for i in range(warmup_steps + timed_steps):
        t0 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        _, losses = O.process_batch(nets, inputs, cfg, noise)
        losses['total_loss'].backward()
        opt.step()
        if i >= warmup_steps:
            times.append(time.perf_counter() - t0)
        print(f'[bench] cpu baseline step {i + 1}/{warmup_steps + timed_steps}: '
              f'{time.perf_counter() - t0:.1f} s', file=sys.stderr, flush=True)
    dt = sum(times) / len(times)
    cpu_model = ''
    try:
        with open('/proc/cpuinfo') as fh:
            cpu_model = next((l.split(':', 1)[1].strip() for l in fh if l.startswith('model name')), '')
    except OSError:
        pass
    return {'value': 1.0 / dt, 'unit': 'iters/s', 'cores': threads, 'kind': 'port',
            'cpu_model': cpu_model, 'torch_threads': torch.get_num_threads(), 'affinity_cores': aff,
            'step_s': [round(t, 2) for t in times],
            'sample': f'{warmup_steps} warm-up + {timed_steps} timed full steps (fwd+loss+bwd+Adam) of the '
                      f'CPU oracle at the same config, B=1, mean {dt:.1f} s/step on {threads} threads '
                      f'(torch CPU; affinity {aff} cores, capped by OMP_NUM_THREADS); the reference\'s '
                      f'train.py:17-20 pins OMP/MKL to 1 thread'}


def parity_check(device):
    """BASELINE.md §3 'Reported: parity': one training step of the reduced 6-camera fusion
    config (tests/golden/step_small.npz: the reference's own outputs on the same seeded weights,
    inputs and identity noise) through the HIP path, compared with the reference: max |Δ| of the
    depth maps and of every loss scalar, and the Abs.Rel / median-scaled metrics
    (Logger.compute_depth_losses) against tests/golden/depth_metrics.npz."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
    import common as G
    from vfdepth_amd.vfdepth import VFDepthAlgo
    gold = os.path.join(ROOT, 'tests', 'golden')
    fx = np.load(os.path.join(gold, 'step_small.npz'))
    fm = np.load(os.path.join(gold, 'depth_metrics.npz'))
    cfg = G.step_cfg()
    algo = VFDepthAlgo(cfg, device.index)
    for m in algo.models.values():
        m.load_state_dict(seeded_state_dict(m, seed=G.STEP_SEED))
    algo.set_train()
    inputs = synth.make_batch(cfg, seed=5, with_depth=True)
    N = cfg['data']['num_cams']
    noise = torch.stack([torch.tensor(fx[f'noise_c{c}']) for c in range(N)]).to(device)
    outputs, losses = algo.process_batch(inputs, device.index, noise=noise)
    losses['total_loss'].backward()
    torch.cuda.synchronize()
    d_depth = max(float((outputs[('cam', c)][('depth', 0)].cpu() - torch.tensor(fx[f'depth_c{c}'])).abs().max())
                  for c in range(N))
    rel_depth = max(float(((outputs[('cam', c)][('depth', 0)].cpu() - torch.tensor(fx[f'depth_c{c}'])).abs()
                           / torch.tensor(fx[f'depth_c{c}']).abs()).max()) for c in range(N))
    d_loss = {k[5:]: abs(float(losses[k[5:]]) - float(fx[k])) for k in fx.files if k.startswith('loss_')}
    metric, median = algo.compute_depth_metrics(inputs, outputs)
    absrel = {'metric': float(metric['abs_rel']), 'median': float(median['abs_rel']),
              'ref_metric': float(fm['step_metric_abs_rel']), 'ref_median': float(fm['step_median_abs_rel'])}
    full = parity_full(device)
    return {'config': 'reduced 6-cam fusion step (96x160, voxels 40x40x10, D=16) vs the reference\'s outputs',
            'full_resolution': full,
            'max_abs_diff_depth': d_depth, 'max_rel_diff_depth': rel_depth,
            'max_abs_diff_loss': max(d_loss.values()), 'loss_keys': len(d_loss),
            'abs_rel': absrel,
            'abs_rel_equal_1e-4': abs(absrel['metric'] - absrel['ref_metric']) <= 1e-4 * absrel['ref_metric']
            and abs(absrel['median'] - absrel['ref_median']) <= 1e-4 * absrel['ref_median']}


def parity_full(device):
    """The same check at config 2's full shape (6 x 384 x 640, 100 x 100 x 20 voxels, D = 50)
    against the reference's own CPU step there (tests/golden/step_full.npz): max |Δ| of the depth
    maps (every 4th pixel) and of every loss scalar, and the 1e-4 per-pixel north_star verdict."""
    import numpy as np
    import common as G
    from vfdepth_amd.vfdepth import VFDepthAlgo
    fx = np.load(os.path.join(ROOT, 'tests', 'golden', 'step_full.npz'))
    cfg = G.full_cfg()
    algo = VFDepthAlgo(cfg, device.index)
    for m in algo.models.values():
        m.load_state_dict(seeded_state_dict(m, seed=G.STEP_SEED))
    algo.set_train()
    inputs = synth.make_batch(cfg, seed=G.FULL_SEED, with_depth=True)
    t = cfg['training']
    noise = torch.stack(G.full_noise(fx, (t['batch_size'], len(t['frame_ids']) - 1, t['height'], t['width'])))
    outputs, losses = algo.process_batch(inputs, device.index, noise=noise.to(device))
    losses['total_loss'].backward()
    torch.cuda.synchronize()
    s, N = G.FULL_SUB, cfg['data']['num_cams']
    dd = [(outputs[('cam', c)][('depth', 0)][..., ::s, ::s].cpu().double(), torch.tensor(fx[f'depth_sub_c{c}']).double())
          for c in range(N)]
    d_depth = max(float((a - b).abs().max()) for a, b in dd)
    within = all(bool(((a - b).abs() <= 1e-4 + 1e-4 * b.abs()).all()) for a, b in dd)
    d_loss = {k[5:]: abs(float(losses[k[5:]]) - float(fx[k])) for k in fx.files if k.startswith('loss_')}
    within = within and all(v <= 1e-4 + 1e-4 * abs(float(fx['loss_' + k])) for k, v in d_loss.items())
    return {'config': '6-cam 384x640, voxels 100x100x20, D=50 (config 2) vs the reference\'s CPU step',
            'max_abs_diff_depth': d_depth, 'max_abs_diff_loss': max(d_loss.values()), 'loss_keys': len(d_loss),
            'within_1e-4': within}


def load_traffic(config):
    path = os.path.join(ROOT, 'profiles', f'traffic_config{config}.json')
    if os.path.isfile(path):
        with open(path) as fh:
            return json.load(fh)
    return {}


def launch_ranks(n):
    """Run this script on n ranks (torch.distributed.run, rendezvous on 127.0.0.1) as a child
    process; return its exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr', '127.0.0.1', '--master-port', str(port), os.path.abspath(__file__)] + sys.argv[1:]
    print(f'[bench] launching {n} ranks: {" ".join(cmd)}', file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--config', type=int, default=2)
    ap.add_argument('--batch', type=int, default=None)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--kernel-table', action='store_true', help='print per-kernel times to stderr')
    ap.add_argument('--graph', type=int, default=0, help='1: replay the step as a captured HIP graph (single GPU)')
    ap.add_argument('--conv-autotune', type=int, default=1,
                    help='1 (default): MIOpen picks each conv algorithm by measured time (torch.backends.cudnn.'
                         'benchmark; the committed find-db answers config 2 without a search); 0: immediate mode')
    ap.add_argument('--channels-last', type=int, default=0, help='1: NHWC memory format for the dense nets')
    ap.add_argument('--cpu-steps', type=int, default=3, help='timed CPU-baseline steps (after 1 warm-up)')
    ap.add_argument('--no-parity', action='store_true')
    args = ap.parse_args()
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        # `bench.py --gpus N` on its own: one rank per GPU, launched like the reference's
        # mp.spawn (train.py:59-61) — here torch.distributed.run as a CHILD process (this parent
        # has not touched the GPU; it never execs), and its exit code is ours
        return launch_ranks(args.gpus)
    faulthandler.enable()
    if os.environ.get('VFD_BENCH_TRACEBACK'):     # diagnostics: dump every thread's stack periodically
        faulthandler.dump_traceback_later(float(os.environ['VFD_BENCH_TRACEBACK']), repeat=True)
    t_start = time.time()
    done = threading.Event()

    def heartbeat():     # warm-up (MIOpen kernel compiles / solver search) can be silent for minutes
        while not done.wait(60):
            print(f'[bench] ... {time.time() - t_start:.0f} s', file=sys.stderr, flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        raise SystemExit(f'bench.py --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU')
    # test-only overrides (tests/test_gpu_0_bench_world2.py rehearses the multi-rank path on one
    # GPU): VFD_BENCH_BACKEND=gloo, VFD_BENCH_ONE_DEVICE=1 puts every rank on cuda:0 (RCCL does not
    # run two ranks on one device); the driver's runs set neither
    backend = os.environ.get('VFD_BENCH_BACKEND', 'nccl')
    if os.environ.get('VFD_BENCH_ONE_DEVICE') == '1':
        local = 0
    if world > 1:
        dist.init_process_group(backend, init_method='env://')
    torch.cuda.set_device(local)
    torch.backends.cudnn.benchmark = bool(args.conv_autotune)
    _lib.load()

    from vfdepth_amd.vfdepth import VFDepthAlgo
    cfg, name = make_cfg(args.config, args.batch)
    cfg['ddp'].update({'ddp_enable': world > 1, 'world_size': world, 'gpus': list(range(world))})
    torch.manual_seed(42 + rank)
    algo = VFDepthAlgo(cfg, local)
    for mname, m in algo.models.items():
        inner = m.module if hasattr(m, 'module') else m
        inner.load_state_dict(seeded_state_dict(inner, seed=7))
    algo.set_train()
    if args.channels_last:
        for m in algo.models.values():
            m.to(memory_format=torch.channels_last)
    batch = synth.make_batch(cfg, seed=1234 + rank, device=f'cuda:{local}')

    def eager_step():
        return algo.train_step(dict(batch))

    use_graph = bool(args.graph) and world == 1
    step = eager_step
    if use_graph:
        # warm-up runs inside graphed_train_step (side stream), then the capture, then replays
        algo.set_optimizer(capturable=True)
        step = algo.graphed_train_step(batch, warmup=max(args.warmup - 1, 1))
        print(f'[bench] captured the training step as a HIP graph ({name})', file=sys.stderr, flush=True)
        step()
    else:
        for i in range(args.warmup):
            eager_step()
            if rank == 0 and i == 0:
                print(f'[bench] first step done ({name})', file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        losses = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # per-kernel device times: HIP events around each hot-path launch on its stream, recorded in
    # a few eager steps right after the timed region (the timed steps carry no profiling hooks;
    # graph replays could not fire them).  Two sets: first one-stream steps (`frac_isolated`: a
    # kernel alone on the chip), then steps in the TIMED configuration (the pose branch on its own
    # stream, so an event pair also times the other branch's kernels sharing the CUs): the line's
    # `roofline` is the latter, which rocprofv3 of the same command reproduces (profiles/r6/)
    n_prof = min(args.steps, 5)
    torch.cuda.synchronize()
    from vfdepth_amd import kernels as KN

    def profiled(branch):
        algo.branch_streams = branch
        KN.syncbn_stats(reset=True)
        _lib.prof_enable('all')
        for _ in range(n_prof):
            last = eager_step()
        torch.cuda.synchronize()
        stats = KN.syncbn_stats(reset=True)
        pr = _lib.prof_read()
        dense = {k: v * args.steps / n_prof for k, v in _lib.ALG_BYTES.items()}
        _lib.prof_enable('off')
        pr = {k: (n * args.steps // n_prof, t * args.steps / n_prof) for k, (n, t) in pr.items()}
        return pr, dense, stats, last
    timed_branch = getattr(algo, '_bstream', None) is not None
    prof_iso, _, _, _ = profiled(False)
    prof, dense_bytes, sbn, losses = profiled(timed_branch)
    algo.branch_streams = True
    elapsed = max_over_ranks(elapsed, world, f'cuda:{local}')
    if rank != 0:
        dist.destroy_process_group()
        return 0

    s = shapes(cfg)
    from vfdepth_amd import geometry as GEO
    if cfg['model']['pose_model'] == 'fusion' and GEO._POSE_PAIRS and algo.pose.batch_pairs:
        s['pose_pairs'] = s['T']          # the frame pairs' K2C convs as one launch
    if cfg['training']['net_precision'] == 'bf16' and os.environ.get('VFD_POSE_BF16_MAP', '1') != '0':
        s['map_bytes'] = 2            # config 3: K2 writes the pose map in bf16 (kernels.PoseConvBF16)
    traffic_tab = load_traffic(args.config)

    def roofline_of(k, table=None):
        n_launch, ms = (table or prof)[k]
        avg_s = ms / 1e3 / n_launch
        fl = mfma_flops(k, s)
        if fl is not None:
            ach = fl / avg_s / 1e12
            # config 3 runs K3C / K2C (forward, data and weight gradients) on bf16 MFMA
            bf16 = cfg['training']['net_precision'] == 'bf16'
            if bf16 and os.environ.get('VFD_PC_BF16_BWD', '1') == '0':
                bf16 = k in ('proj_conv_fwd', 'pad_conv_fwd')
            peak = MFMA_BF16_PEAK_TFS if bf16 else MFMA_F32_PEAK_TFS
            return {'kernel': k, 'bound': 'mfma', 'mfma_dtype': 'bf16' if bf16 else 'fp32', 'achieved': ach,
                    'peak': peak, 'unit': 'TFLOP/s', 'frac': ach / peak, 'traffic': traffic_tab.get(k),
                    'flops_per_launch': fl, 'avg_launch_us': avg_s * 1e6, 'launches': n_launch}
        alg = dense_bytes[k] / n_launch if k in dense_bytes else algorithmic_bytes(k, s)
        ach = alg / avg_s / 1e9
        return {'kernel': k, 'bound': 'hbm', 'achieved': ach, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': ach / HBM_PEAK_GBS, 'traffic': traffic_tab.get(k), 'alg_bytes_per_launch': alg,
                'avg_launch_us': avg_s * 1e6, 'launches': n_launch}
    dense = {k: prof.pop(k) for k in list(prof) if k in dense_bytes}     # fused dense-net kernels (BN)
    dom = max(prof, key=lambda k: prof[k][1])
    hbm_ops = [k for k in prof if mfma_flops(k, s) is None]
    dom_hbm = max(hbm_ops, key=lambda k: prof[k][1])
    prof_all = dict(prof, **dense)

    def roofline_any(k):
        saved = prof.get(k)
        prof[k] = prof_all[k]
        try:
            return roofline_of(k)
        finally:
            if saved is None:
                del prof[k]
    if args.kernel_table:
        for k, (n, t) in sorted(prof_all.items(), key=lambda kv: -kv[1][1]):
            r = roofline_any(k)
            print(f'[bench] {k:20s} {n:4d} launches {t / n * 1e3:9.1f} us/launch  '
                  f'{r["achieved"]:8.1f} {r["unit"]} ({r["frac"]:.3f} of peak)', file=sys.stderr)
        print(f'[bench] hot-path kernels {sum(t for _, t in prof.values()) / args.steps:.2f} ms/step, fused dense '
              f'{sum(t for _, t in dense.values()) / args.steps:.2f} ms/step (BN, pads, upsample bwd), of '
              f'{elapsed / args.steps * 1e3:.2f} ms/step; loss {float(losses["total_loss"]):.5f}', file=sys.stderr)
    # aggregate over every HBM-bound hot-path op of the step (per-kernel and aggregate)
    agg_bytes = sum(algorithmic_bytes(k, s) * prof[k][0] for k in hbm_ops)
    agg_s = sum(prof[k][1] for k in hbm_ops) / 1e3
    iso_ops = [k for k in hbm_ops if k in prof_iso]     # the same ops in the one-stream profiling steps
    agg_iso = (sum(algorithmic_bytes(k, s) * prof_iso[k][0] for k in iso_ops)
               / (sum(prof_iso[k][1] for k in iso_ops) / 1e3) / 1e9) if iso_ops else None
    parity = None
    if not args.no_parity:
        # the parity steps run other shapes (96x160, the fixture's): immediate mode, no MIOpen search
        torch.backends.cudnn.benchmark = False
        parity = parity_check(torch.device(f'cuda:{local}'))
    base = None
    if world == 1 and not args.no_cpu_baseline:
        base = cpu_baseline(cfg, timed_steps=args.cpu_steps)
    out = {
        'metric': (f"6-cam {s['H']}x{s['W']} train iters/sec (" +
                   ('NuScenes-shaped' if args.config == 4 else 'DDAD-shaped') + ', volumetric fusion' +
                   (f", voxels {s['X']}x{s['Y']}x{s['Z']}" if args.config == 5 else '') + ')'),
        'value': job_throughput(elapsed, args.steps, world),
        'unit': 'iters/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': elapsed / args.steps * 1e3,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'fp32' if cfg['training']['net_precision'] == 'fp32' else
                 'bf16 nets (K3C / K2C forward, fused BN / pads / pool on bf16 maps), fp32 geometry, fusion and loss kernels',
        'data': 'synthetic DDAD-shaped batches (seeded), seeded random-init weights',
        'config': {'workload': name, 'config_id': args.config, 'batch_per_gpu': s['B'], 'cameras': s['N'],
                   'image': [s['H'], s['W']], 'voxels': [s['X'], s['Y'], s['Z']], 'depth_bins': s['D'],
                   'parallelism': f'dp{world}', 'net_precision': cfg['training']['net_precision']},
        'roofline': dict(roofline_of(dom), measured_in='the timed configuration (pose branch on its own stream)'
                         if timed_branch else 'one stream (the timed configuration)',
                         frac_isolated=roofline_of(dom, prof_iso)['frac'] if dom in prof_iso else None,
                         avg_launch_us_isolated=roofline_of(dom, prof_iso)['avg_launch_us'] if dom in prof_iso else None),
        'roofline_hbm_dominant': roofline_of(dom_hbm),
        'roofline_aggregate': {'bound': 'hbm', 'achieved': agg_bytes / agg_s / 1e9, 'peak': HBM_PEAK_GBS,
                               'unit': 'GB/s', 'frac': agg_bytes / agg_s / 1e9 / HBM_PEAK_GBS,
                               'alg_bytes_per_step': agg_bytes / args.steps,
                               'kernel_ms_per_step': agg_s * 1e3 / args.steps,
                               'measured_in': 'the timed configuration (each op timed on its stream while the '
                                              'other branch runs beside it)' if timed_branch else 'one stream',
                               'frac_isolated': agg_iso / HBM_PEAK_GBS if agg_iso else None,
                               'what': 'every HBM-bound hot-path op of the step (K1-K5, plans, aggregation)'},
        'hot_path_ms_per_step': sum(t for _, t in prof.values()) / args.steps,
        'dense_fused': {k: roofline_any(k) for k in dense},
        'execution': ('hip-graph replay of the whole step' if use_graph else
                      'eager, pose branch on a second stream' if getattr(algo, '_bstream', None) is not None else 'eager'),
        'miopen': ('benchmark mode (algorithm per shape by measured time, find-db miopen_db/)' if args.conv_autotune
                   else 'immediate mode (find-db miopen_db/)'),
        'encoder_layout': 'channels-last' if any(getattr(m, 'channels_last', False) for net in algo.models.values()
                                                  for m in (net.module if hasattr(net, 'module') else net).modules())
                          else 'NCHW',
        'syncbn': ({'backend': dist.get_backend(), 'allreduce_per_step': sbn['calls'] / n_prof,
                    'bytes_per_step': sbn['bytes'] / n_prof, 'host_ms_per_step': sbn['host_s'] * 1e3 / n_prof,
                    'what': 'the fused BN kernels\' SyncBatchNorm exchange: one all-reduce of [C+1][2] fp64 per '
                            'layer and direction (host time = enqueue for RCCL)'} if world > 1 else None),
        'parity': parity,
        'cpu_baseline': base,
    }
    done.set()
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == '__main__':
    sys.exit(main())

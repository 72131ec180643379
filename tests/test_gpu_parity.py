"""GPU parity: the HIP hot path against the reference's golden vectors (and the CPU oracle).

Every test calls the product through its C ABI (vfdepth_amd.kernels -> libvfd_hip.so).
Tolerance (BASELINE.json north_star): fp32 per-pixel 1e-4.  Values are compared with
|a - b| <= 1e-4 + 1e-4 |b|; gradients with max |a - b| <= 2e-4 x max |b| (they are sums of
many atomically accumulated fp32 terms in a different order than the reference's).
Discontinuities (nearest-mask lookups, OOB tests, argmin ties) are evaluated with the
reference's operation order, so no mismatch allowance is made for them.
"""
import math
import os

import numpy as np
import pytest
import torch

import common as G
from conftest import golden

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')
ATOL = RTOL = 1e-4


def close(a, b, what, atol=ATOL, rtol=RTOL):
    a = a.detach().float().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    b = b.detach().float().cpu().numpy() if torch.is_tensor(b) else np.asarray(b)
    assert a.shape == b.shape, f'{what}: shape {a.shape} vs {b.shape}'
    err = np.abs(a.astype(np.float64) - b)
    bad = err > atol + rtol * np.abs(b)
    assert not bad.any(), f'{what}: {int(bad.sum())}/{bad.size} off, max err {err.max():.3g}'


def gclose(a, b, what, rel=2e-4):
    a = a.detach().double().cpu().numpy()
    b = np.asarray(b.detach().cpu().numpy() if torch.is_tensor(b) else b, np.float64)
    assert a.shape == b.shape, f'{what}: shape {a.shape} vs {b.shape}'
    scale = max(np.abs(b).max(), 1e-12)
    err = np.abs(a - b).max() / scale
    assert err < rel, f'{what}: max rel err {err:.3g} (scale {scale:.3g})'


def to_dev(d):
    return {k: (v.to(DEV) if torch.is_tensor(v) else v) for k, v in d.items()}


@pytest.fixture(scope='module', autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    from vfdepth_amd import _lib
    _lib.load()


# ------------------------------------------------------------------------------------ fusion
def _fusion_net(model):
    from vfdepth_amd.fusion import VFNet
    cfg, d, seeds = G.fusion_case()
    fx = golden('fusion_small.npz')
    net = VFNet(cfg, d['feats'].shape[2], 32, model=model).to(DEV)
    if model == 'depth':
        with torch.no_grad():
            net.conv_non_overlap[0].weight.copy_(torch.tensor(fx['w_no']))
            net.conv_non_overlap[0].bias.copy_(torch.tensor(fx['b_no']))
            net.conv_overlap[0].weight.copy_(torch.tensor(fx['w_o']))
            net.conv_overlap[0].bias.copy_(torch.tensor(fx['b_o']))
    inputs = {('K', 3): d['K'].to(DEV), ('inv_K', 3): d['invK'].to(DEV), 'extrinsics': d['E'].to(DEV),
              'extrinsics_inv': d['Einv'].to(DEV), 'mask': d['mask'].to(DEV)}
    return cfg, d, seeds, fx, net, inputs


def test_mask_downsample():
    from oracle import vfd_oracle as O
    from vfdepth_amd import kernels as KN
    cfg, d, _ = G.fusion_case()
    space = KN.VoxelSpace(cfg, DEV)
    lo = KN.mask_lowres(space, d['mask'].to(DEV))
    ref = O.resize_bilinear_ac(d['mask'].flatten(0, 1), space.h, space.w).view_as(lo)
    close(lo, ref, 'mask 1/8', atol=1e-6, rtol=1e-6)


def test_fuse_depth_forward_backward():
    cfg, d, seeds, fx, net, inputs = _fusion_net('depth')
    feats = d['feats'].to(DEV).requires_grad_(True)
    vox = net.backproject_depth(inputs, feats)                               # [B, V, Cv]
    close(vox.permute(0, 2, 1), fx['vox'], 'K1 voxel features')
    g = G.seeded_randn(fx['vox'].shape, seeds['g_vox']).to(DEV)              # [B, Cv, V]
    (vox.permute(0, 2, 1) * g).sum().backward()
    gclose(feats.grad, fx['d_feats_depth'], 'K1 d feats')
    gclose(net.conv_non_overlap[0].weight.grad, fx['d_w_no'], 'K1 d W_no')
    gclose(net.conv_non_overlap[0].bias.grad, fx['d_b_no'], 'K1 d b_no')
    gclose(net.conv_overlap[0].weight.grad, fx['d_w_o'], 'K1 d W_o')
    gclose(net.conv_overlap[0].bias.grad, fx['d_b_o'], 'K1 d b_o')


def test_fuse_pose_forward_backward():
    from vfdepth_amd import kernels as KN
    cfg, d, seeds, fx, net, inputs = _fusion_net('pose')
    space = net.space(DEV)
    feats = d['feats'].to(DEV).requires_grad_(True)
    plan = KN.FusionPlan(space, KN.mask_lowres(space, inputs['mask']), inputs[('K', 3)], inputs['extrinsics_inv'])
    B, C1 = feats.shape[0], feats.shape[2] + 1
    out = KN.pose_to_reference(KN.FusePose.apply(space, plan, feats), C1, space.Z)
    inner = out[:, :, 1:-1, 1:-1].reshape(B, C1, space.Z, space.Y, space.X).reshape(B, C1, -1)
    close(inner, fx['vpose'], 'K2 pose voxels')
    # reflect halo holds the mirrored interior (what the stride-2 reflect conv reads)
    close(out[:, :, 0, 1:-1], out[:, :, 2, 1:-1], 'K2 top halo', atol=0, rtol=0)
    close(out[:, :, 1:-1, -1], out[:, :, 1:-1, -3], 'K2 right halo', atol=0, rtol=0)
    g = G.seeded_randn(fx['vpose'].shape, seeds['g_pose']).to(DEV)
    (inner * g).sum().backward()
    gclose(feats.grad, fx['d_feats_pose'], 'K2 d feats')


def test_voxel_project_forward_backward():
    from vfdepth_amd import kernels as KN
    cfg, d, seeds, fx, net, inputs = _fusion_net('depth')
    space = net.space(DEV)
    vleaf = G.seeded_randn(fx['vox'].shape, seeds['vleaf']).to(DEV)       # [B, Cv, V]
    v = vleaf.permute(0, 2, 1).contiguous().requires_grad_(True)
    out = KN.proj_to_reference(KN.VoxelProject.apply(space, v, inputs[('inv_K', 3)], inputs['extrinsics']),
                               v.shape[2], space.D)
    B, N = inputs['extrinsics'].shape[:2]
    inner = out[:, :, 1:-1, 1:-1].reshape(B, N, *out.shape[1:2], space.h, space.w)
    close(inner, fx['proj'], 'K3 frustum features')
    g = G.seeded_randn(fx['proj'].shape, seeds['g_proj']).to(DEV)
    (inner * g).sum().backward()
    gclose(v.grad.permute(0, 2, 1), fx['d_vleaf'], 'K3 d voxel')


def _k3_bwd_three_ways(deterministic):
    """K3 backward of one seeded gradient three ways: the op (split plan + planned backward), the
    one-call C entry (`vfd_voxel_project_bwd`: plan + backward) and that plan reused; plus the
    backward of |g| (every term non-negative: the per-voxel sum of |w g|)."""
    import ctypes
    from vfdepth_amd import _lib as L
    from vfdepth_amd import kernels as KN
    cfg, d, seeds, fx, net, inputs = _fusion_net('depth')
    space = net.space(DEV)
    lib = L.load()
    prev = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = deterministic
    try:
        v = G.seeded_randn(fx['vox'].shape, seeds['vleaf']).to(DEV).permute(0, 2, 1).contiguous().requires_grad_(True)
        invK, E = inputs[('inv_K', 3)].contiguous(), inputs['extrinsics'].contiguous()
        out = KN.VoxelProject.apply(space, v, invK, E)
        torch.manual_seed(0)
        g = torch.randn(out.shape, device=DEV).contiguous(memory_format=torch.channels_last)
        out.backward(g)
        ref = v.grad.clone()
        v.grad = None
        KN.VoxelProject.apply(space, v, invK, E).backward(g.abs())
        mag = v.grad.clone()
        B, V, Cv = v.shape
        desc = space.desc(B, E.shape[1], Cv=Cv)
        nbytes = lib.vfd_voxel_project_bwd_workspace(ctypes.byref(desc))
        ws = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
        one = torch.empty(B, V, Cv, device=DEV)
        L.check(lib.vfd_voxel_project_bwd(ctypes.byref(desc), g.data_ptr(), invK.data_ptr(), E.data_ptr(),
                                          one.data_ptr(), ws.data_ptr(), nbytes, L.stream()), 'voxel_project_bwd')
        again = torch.empty(B, V, Cv, device=DEV)
        L.check(lib.vfd_voxel_project_bwd_planned(ctypes.byref(desc), g.data_ptr(), ws.data_ptr(), nbytes,
                                                  again.data_ptr(), L.stream()), 'voxel_project_bwd_planned')
        torch.cuda.synchronize()
    finally:
        torch.backends.cudnn.deterministic = prev
    return ref, one, again, mag


def test_voxel_project_bwd_one_call_and_plan_reuse_deterministic():
    """Deterministic mode (no atomics: heavy tiles unsplit, per-cell lists in sample order): the
    one-call entry and the reused plan give the op's d voxels bit for bit."""
    ref, one, again, _ = _k3_bwd_three_ways(True)
    assert torch.equal(one, ref)
    assert torch.equal(again, ref)


def test_voxel_project_bwd_one_call_and_plan_reuse():
    """Default mode: the heavy tiles' parts (each summed in a fixed order) are added into the
    voxel rows with f32 atomics, so the three paths may differ by the reordering of those part
    sums.  Adding p part sums in two orders differs by at most 2 (p - 1) u sum|part| <= 2 (p - 1) u
    sum_s |w_s g_s| per element (u = 2^-24), and the backward of |g| is exactly sum_s |w_s g_s|.
    p <= 32 parts per tile (a part holds 1024 samples; no 8 x 4 x 2-voxel tile of these
    configs collects 32 768 samples): bound 64 u |.|-backward elementwise, + 1e-30 for zeros."""
    ref, one, again, mag = _k3_bwd_three_ways(False)
    bound = 64 * 2.0 ** -24 * mag + 1e-30
    assert bool(((one - ref).abs() <= bound).all()), float(((one - ref).abs() / (mag + 1e-30)).max())
    assert bool(((again - ref).abs() <= bound).all()), float(((again - ref).abs() / (mag + 1e-30)).max())


def test_voxel_project_padding_matches_reflect_conv():
    """Writing the reflect-padded layout then conv(padding=0) == reference conv(padding_mode='reflect')."""
    from vfdepth_amd import kernels as KN
    cfg, d, seeds, fx, net, inputs = _fusion_net('depth')
    space = net.space(DEV)
    v = G.seeded_randn(fx['vox'].shape, seeds['vleaf']).to(DEV).permute(0, 2, 1).contiguous()
    out = KN.VoxelProject.apply(space, v, inputs[('inv_K', 3)], inputs['extrinsics'])
    ref = torch.nn.functional.pad(out[:, :, 1:-1, 1:-1], (1, 1, 1, 1), mode='reflect')
    close(out, ref, 'reflect halo', atol=0, rtol=0)


@pytest.mark.parametrize('model', ['depth', 'pose'])
def test_vfnet_full_width_against_oracle(model):
    """VFNet at the real channel widths (C=256 features, Cv=64 voxel channels: the kernel template
    instances config 2 runs) on a reduced grid (40x40x10 voxels, D=16, 12x20 feature map), forward
    and backward, against the CPU oracle driving the same module's reduce_dim with the reference's
    reflect padding (volumetric_fusionnet.py:116-267, 289-343).  The golden fixture's Cv=8/C=8
    grid covers the narrow template instances."""
    from oracle import vfd_oracle as O
    from vfdepth_amd import synth
    from vfdepth_amd.fusion import VFNet
    from vfdepth_amd.layers import seeded_state_dict
    cfg = G.step_cfg()
    spec = O.VoxelSpec(cfg)
    C, out_dim = int(cfg['model']['fusion_feat_in_dim']), 128 if model == 'depth' else 256
    batch = synth.make_batch(cfg, seed=21)
    B, N = batch['extrinsics'].shape[:2]
    lvl = int(cfg['model']['fusion_level']) + 1
    feats = G.seeded_randn((B, N, C, spec.h, spec.w), 301)
    net = VFNet(cfg, C, out_dim, model=model)
    net.load_state_dict(seeded_state_dict(net, seed=302))
    Einv = torch.inverse(batch['extrinsics'])
    K, invK, E, mask = batch[('K', lvl)], batch[('inv_K', lvl)], batch['extrinsics'], batch['mask']
    # reference path on the CPU (fp32, autograd through the oracle)
    fr = feats.clone().requires_grad_(True)
    if model == 'depth':
        c_no, c_o = net.conv_non_overlap[0], net.conv_overlap[0]
        vox = O.fuse_depth(spec, fr, mask, K, Einv, c_no.weight, c_no.bias, c_o.weight, c_o.bias)
        ref = torch.stack([net.reduce_dim(p) for p in O.project_voxels(spec, vox, invK, E)], 1).flatten(0, 1)
    else:
        vox = O.fuse_pose(spec, fr, mask, K, Einv)
        ref = net.reduce_dim(vox.reshape(B, -1, spec.Y, spec.X))
    g = G.seeded_randn(ref.shape, 303)
    (ref * g).sum().backward()
    ref_grads = {k: p.grad.clone() for k, p in net.named_parameters()}
    net.zero_grad(set_to_none=True)
    # the product: the same module on the GPU through the C ABI
    gnet = net.to(DEV)
    inputs = {('K', lvl): K.to(DEV), ('inv_K', lvl): invK.to(DEV), 'extrinsics': E.to(DEV),
              'extrinsics_inv': Einv.to(DEV), 'mask': mask.to(DEV)}
    fg = feats.to(DEV).requires_grad_(True)
    out = gnet(inputs, fg)
    out = out['proj_feat'] if model == 'depth' else out
    close(out, ref, f'VFNet[{model}] output')
    (out * g.to(DEV)).sum().backward()
    gclose(fg.grad, fr.grad, f'VFNet[{model}] d feats')
    for k, p in gnet.named_parameters():
        gclose(p.grad, ref_grads[k], f'VFNet[{model}] d {k}')


# ------------------------------------------------------------------------------------ view synthesis
@pytest.mark.parametrize('name,skip', [('view_small.npz', False), ('view_skip.npz', True)])
def test_view_synthesis(name, skip):
    from vfdepth_amd.geometry import Pose, ViewRendering
    fx = golden(name)
    cfg, batch, depth, poses = G.view_case(skip)
    batch = to_dev(batch)
    vr, pose = ViewRendering(cfg, 0), Pose(cfg)
    d = depth.to(DEV).requires_grad_(True)
    outputs = {('cam', c): {} for c in range(6)}
    Ts = {}
    for c in range(6):
        for f in (-1, 1):
            Ts[(c, f)] = poses[(c, f)].to(DEV).requires_grad_(True)
            outputs[('cam', c)][('cam_T_cam', 0, f)] = Ts[(c, f)]
        outputs[('cam', c)][('depth', 0)] = d[:, c]
    rel = {c: pose.compute_relative_cam_poses(batch, outputs, c) for c in range(6)}
    vr.render_all(batch, outputs, rel, {0: d[:, :, 0]})
    loss = 0
    for c in range(6):
        out = outputs[('cam', c)]
        for i, k in enumerate(G.VIEW_IMG_KEYS):
            close(out[k], fx[f'{G.key_name(k)}_c{c}'], f'{k} cam {c}')
            loss = loss + (out[k] * G.seeded_randn(out[k].shape, 500 + 10 * c + i).to(DEV)).sum()
        for k in G.VIEW_MSK_KEYS:
            close(out[k], fx[f'{G.key_name(k)}_c{c}'], f'{k} cam {c}', atol=0, rtol=0)
    loss.backward()
    for c in range(6):
        gclose(d.grad[:, c], fx[f'd_depth_c{c}'], f'd depth cam {c}')
        for f in (-1, 1):
            gclose(Ts[(c, f)].grad, fx[f'd_T_{f}_c{c}'], f'd T{f} cam {c}')


def test_view_synthesis_per_camera_api():
    """ViewRendering.forward(inputs, outputs, cam, rel) (reference per-camera API) == batched path."""
    from vfdepth_amd.geometry import Pose, ViewRendering
    fx = golden('view_small.npz')
    cfg, batch, depth, poses = G.view_case(False)
    batch = to_dev(batch)
    vr, pose = ViewRendering(cfg, 0), Pose(cfg)
    for c in (0, 3):
        out = {('depth', 0): depth[:, c].to(DEV)}
        for f in (-1, 1):
            out[('cam_T_cam', 0, f)] = poses[(c, f)].to(DEV)
        outputs = {('cam', c): out}
        vr(batch, outputs, c, pose.compute_relative_cam_poses(batch, outputs, c))
        for k in G.VIEW_IMG_KEYS:
            close(out[k], fx[f'{G.key_name(k)}_c{c}'], f'{k} cam {c} (per-camera API)')


# ------------------------------------------------------------------------------------ losses
def _loss_inputs():
    cfg, batch, planes = G.loss_case()
    batch = to_dev(batch)
    return cfg, batch, planes


def test_losses_per_camera_api():
    from vfdepth_amd.losses import MultiCamLoss
    fx = golden('loss_small.npz')
    cfg, batch, planes = _loss_inputs()
    batch['extrinsics_inv'] = torch.inverse(batch['extrinsics'])
    loss_fn = MultiCamLoss(cfg, 0)
    for c in range(6):
        out, leaves = {}, {}
        for k in G.VIEW_IMG_KEYS:
            leaves[k] = planes[(c,) + k].to(DEV).requires_grad_(True)
            out[k] = leaves[k]
        for f in (0, -1, 1):
            out[('overlap_mask', f, 0)] = planes[(c, 'overlap_mask', f, 0)].to(DEV)
        disp = planes[(c, 'disp', 0)].to(DEV).requires_grad_(True)
        out[('disp', 0)] = disp
        out[('depth', 0)] = 1.0 / disp.detach()
        noise = torch.tensor(fx[f'noise_c{c}']).to(DEV).unsqueeze(0)
        cl, ld = loss_fn(batch, {('cam', c): out}, c, noise=noise)
        close(cl, fx[f'cam_loss_c{c}'], f'cam loss {c}')
        for k in ('reproj_loss', 'spatio_loss', 'spatio_tempo_loss', 'smooth'):
            close(ld[k], fx[f'{k}_c{c}'], f'{k} cam {c}')
        close(out[('reproj_loss', 0)], fx[f'reproj_plane_c{c}'], 'reproj plane')
        close(out[('reproj_mask', 0)], fx[f'reproj_mask_c{c}'], 'reproj mask', atol=0, rtol=0)
        close(out[('overlap_mask', 0, 0)], fx[f'spatio_mask_c{c}'], 'spatio mask', atol=0, rtol=0)
        cl.backward()
        for k in G.VIEW_IMG_KEYS:
            gclose(leaves[k].grad, fx[f'd_{G.key_name(k)}_c{c}'], f'd {k} cam {c}')
        gclose(disp.grad, fx[f'd_disp_c{c}'], f'd disp cam {c}')


def test_losses_all_cameras():
    """Batched forward_all over the six cameras == per-camera reference values."""
    from vfdepth_amd.losses import MultiCamLoss
    fx = golden('loss_small.npz')
    cfg, batch, planes = _loss_inputs()
    loss_fn = MultiCamLoss(cfg, 0)
    T, F = 2, 3
    color = torch.stack([torch.stack([planes[(c,) + k] for k in G.VIEW_IMG_KEYS[:T]], 1) for c in range(6)], 1)
    ovl = torch.stack([torch.stack([planes[(c,) + k] for k in G.VIEW_IMG_KEYS[T:]], 1) for c in range(6)], 1)
    omask = torch.stack([torch.stack([planes[(c, 'overlap_mask', f, 0)][:, 0] for f in (0, -1, 1)], 1)
                         for c in range(6)], 1)
    disp = torch.stack([planes[(c, 'disp', 0)][:, 0] for c in range(6)], 1)
    color, ovl, disp = (t.to(DEV).requires_grad_(True) for t in (color, ovl, disp))
    omask = omask.to(DEV)
    noise = torch.stack([torch.tensor(fx[f'noise_c{c}']) for c in range(6)]).to(DEV)
    outputs = {('cam', c): {} for c in range(6)}
    total, logs = loss_fn.forward_all(batch, outputs, {0: (color, None, ovl, omask)}, {0: disp},
                                      {0: 1.0 / disp.detach()}, noise=noise)
    ref_total = np.mean([float(fx[f'cam_loss_c{c}']) for c in range(6)])
    close(total, np.float32(ref_total), 'total loss')
    for k in ('reproj_loss', 'spatio_loss', 'spatio_tempo_loss', 'smooth'):
        close(logs[k], np.float32(np.mean([float(fx[f'{k}_c{c}']) for c in range(6)])), k)
    total.backward()
    for c in range(6):
        for i, k in enumerate(G.VIEW_IMG_KEYS):
            grad = color.grad[:, c, i] if i < T else ovl.grad[:, c, i - T]
            gclose(grad * 6, fx[f'd_{G.key_name(k)}_c{c}'], f'd {k} cam {c} (batched)')
        gclose(disp.grad[:, c].unsqueeze(1) * 6, fx[f'd_disp_c{c}'], f'd disp cam {c} (batched)')


# ------------------------------------------------------------------------------------ full step
def _step(cfg_fn, fixture, seed_inputs):
    from vfdepth_amd import synth
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.vfdepth import VFDepthAlgo
    fx = golden(fixture)
    cfg = cfg_fn()
    algo = VFDepthAlgo(cfg, 0)
    for m in algo.models.values():
        m.load_state_dict(seeded_state_dict(m, seed=G.STEP_SEED))
    algo.set_train()
    inputs = synth.make_batch(cfg, seed=seed_inputs, with_depth=True)
    np.testing.assert_array_equal(G.checksum(inputs[('color', 0, 0)]), fx['cs_color'])
    N = cfg['data']['num_cams']
    noise = torch.stack([torch.tensor(fx[f'noise_c{c}']) for c in range(N)]).to(DEV)
    outputs, losses = algo.process_batch(inputs, 0, noise=noise)     # moves `inputs` to the device in place
    losses['total_loss'].backward()
    return cfg, fx, algo, inputs, outputs, losses


def automask_flips(cfg, inputs, outputs, fx):
    """Pixels of camera 0 whose auto-mask decision differs from the reference's.

    The auto-mask is argmin([min reprojection, min identity + 1e-5 noise]) — a discontinuous
    function of the depth.  A decision may legitimately flip where the two candidates are within
    fp32 resolution of the upstream (conv-network) computation.  Each flip must therefore be
    explained by a margin |reprojection - identity| below the 1e-4 tolerance (recomputed with
    the CPU oracle from this run's warped images), and flips must stay rare (<= 1e-3 of pixels).
    """
    from oracle import vfd_oracle as O
    ref_mask_plane = torch.tensor(fx['c0_reproj_mask_0'])
    got = outputs[('cam', 0)][('reproj_mask', 0)].detach().cpu()
    ref_bin = (ref_mask_plane != 0)
    got_bin = (got != 0)
    flips = ref_bin != got_bin
    n = int(flips.sum())
    if n == 0:
        return flips.to(DEV)
    assert n <= 1e-3 * flips.numel(), f'{n} auto-mask flips'
    frames = cfg['training']['frame_ids']
    target = inputs[('color', 0, 0)][:, 0].cpu()
    rep = torch.cat([O.photometric(outputs[('cam', 0)][('color', f, 0)].detach().cpu(), target) for f in frames[1:]], 1)
    idn = torch.cat([O.photometric(inputs[('color', f, 0)][:, 0].cpu(), target) for f in frames[1:]], 1)
    idn = idn + torch.tensor(fx['noise_c0'])
    margin = (rep.min(1, keepdim=True).values - idn.min(1, keepdim=True).values).abs()
    worst = float(margin[flips].max())
    assert worst <= 1e-4, f'auto-mask flip with margin {worst:.3g} > 1e-4'
    return flips.to(DEV)


@pytest.mark.parametrize('which', ['fusion', 'mono'])
def test_full_step_against_reference(which):
    cfg_fn, fixture, seed = (G.step_cfg, 'step_small.npz', 5) if which == 'fusion' else (G.mono_cfg, 'mono_small.npz', 6)
    cfg, fx, algo, inputs, outputs, losses = _step(cfg_fn, fixture, seed)
    for k in [k for k in fx.files if k.startswith('loss_')]:
        close(losses[k[5:]], fx[k], k)
    for c in range(cfg['data']['num_cams']):
        close(outputs[('cam', c)][('depth', 0)], fx[f'depth_c{c}'], f'depth cam {c}')
        for f in cfg['training']['frame_ids'][1:]:
            close(outputs[('cam', c)][('cam_T_cam', 0, f)], fx[f'cam_T_cam_{f}_c{c}'], f'T{f} cam {c}', atol=1e-5)
    flips = automask_flips(cfg, inputs, outputs, fx)
    for key in [k for k in fx.files if k.startswith('c0_')]:
        parts = key[3:].split('_')
        name = '_'.join(p for p in parts if not p.lstrip('-').isdigit())
        nums = tuple(int(p) for p in parts if p.lstrip('-').isdigit())
        got = outputs[('cam', 0)][(name,) + nums]
        if name in ('reproj_loss', 'reproj_mask'):
            keep = ~flips
            got, ref = got[keep], torch.tensor(fx[key])[keep.cpu()]
            close(got, ref, key + ' (outside explained auto-mask flips)')
        else:
            close(got, fx[key], key)
    named = {}
    for mname, m in algo.models.items():
        for pname, p in m.named_parameters():
            named[f'{mname}.{pname}'] = p
    # End-to-end parameter gradients vs the reference's: a sanity bound only.  The step has
    # discrete per-pixel decisions (temporal min, spatio-temporal min/max, nearest-mask / OOB
    # tests) whose near-ties flip under 1e-7-relative forward differences (the disparities agree to
    # 6e-7 of max); a flipped pixel reroutes its gradient, and the ~40 dense layers above spread
    # that over every weight (measured: up to 4e-3 relative in the depth net, 2e-5 in the pose
    # net; tools/diag_stages.py).  The decision-free gradient parity of every stage is asserted
    # by test_full_step_gradient_chain.
    for key in [k for k in fx.files if k.startswith('grad__')]:
        a, b = named[key[6:]].grad.detach().double().cpu(), torch.tensor(fx[key]).double()
        rel = float((a - b).norm() / b.norm())
        assert rel < 1e-2, f'{key}: gradient rel diff {rel:.3g} vs the reference'


def test_full_resolution_step_against_reference():
    """BASELINE config 2's full shape (6 x 384 x 640, 100 x 100 x 20 voxels, D = 50, fp32) against
    the reference's own CPU step there (tests/golden/step_full.npz, same seeded weights, inputs
    and identity noise): every loss scalar, the 12 poses, the depth maps at every 4th pixel at
    the north_star tolerance (1e-4 abs + 1e-4 rel per pixel) and their full-map checksums; the
    small parameter gradients within the end-to-end sanity bound of
    test_full_step_against_reference (models/vfdepth.py:191-313)."""
    from vfdepth_amd import synth
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.vfdepth import VFDepthAlgo
    fx = golden('step_full.npz')
    cfg = G.full_cfg()
    algo = VFDepthAlgo(cfg, 0)
    for m in algo.models.values():
        m.load_state_dict(seeded_state_dict(m, seed=G.STEP_SEED))
    algo.set_train()
    inputs = synth.make_batch(cfg, seed=G.FULL_SEED, with_depth=True)
    # full-size double sums: the host's SIMD width changes the last bit (inputs drift would be gross)
    np.testing.assert_allclose(G.checksum(inputs[('color', 0, 0)]), fx['cs_color'], rtol=1e-12)
    t = cfg['training']
    noise = torch.stack(G.full_noise(fx, (t['batch_size'], len(t['frame_ids']) - 1, t['height'], t['width']))).to(DEV)
    outputs, losses = algo.process_batch(inputs, 0, noise=noise)
    losses['total_loss'].backward()
    torch.cuda.synchronize()
    for k in [k for k in fx.files if k.startswith('loss_')]:
        close(losses[k[5:]], fx[k], k)
    s = G.FULL_SUB
    for c in range(cfg['data']['num_cams']):
        d = outputs[('cam', c)][('depth', 0)]
        close(d[..., ::s, ::s], fx[f'depth_sub_c{c}'], f'depth cam {c} (every {s}th pixel)')
        cs, ref = G.checksum(d.cpu()), fx[f'cs_depth_c{c}']
        assert abs(cs[0] - ref[0]) <= 1e-5 * abs(ref[0]) and abs(cs[1] - ref[1]) <= 1e-5 * abs(ref[1]), \
            f'depth cam {c}: full-map checksum {cs[:2]} vs reference {ref[:2]}'
        for f in cfg['training']['frame_ids'][1:]:
            close(outputs[('cam', c)][('cam_T_cam', 0, f)], fx[f'cam_T_cam_{f}_c{c}'], f'T{f} cam {c}', atol=1e-5)
    named = {}
    for mname, m in algo.models.items():
        for pname, p in m.named_parameters():
            named[f'{mname}.{pname}'] = p
    # end-to-end sanity bound only (see test_full_step_against_reference): at 384x640 six times as
    # many auto-mask / min-selection decisions sit near a tie, and a flipped pixel reroutes its
    # gradient through every layer above it (measured 1.06e-2 on conv_overlap's weight with the
    # channels-last MIOpen algorithms); the decision-free stage-by-stage gradient parity is
    # test_full_step_gradient_chain's
    for key in [k for k in fx.files if k.startswith('grad__')]:
        a, b = named[key[6:]].grad.detach().double().cpu(), torch.tensor(fx[key]).double()
        rel = float((a - b).norm() / b.norm())
        assert rel < 3e-2, f'{key}: gradient rel diff {rel:.3g} vs the reference (full resolution)'


def test_step_depth_metrics_against_reference_logger():
    """A24 on the GPU: the fusion step's depth maps scored by `compute_depth_metrics` (all 7
    metrics, plain and median-scaled; reference utils/logger.py:193-247 + utils/misc.py:85-98)
    against the reference Logger's values on the reference step's own depths
    (tests/golden/depth_metrics.npz 'step_*'), at 1e-4 relative."""
    from vfdepth_amd.metrics import METRIC_NAMES
    cfg, fx, algo, inputs, outputs, losses = _step(G.step_cfg, 'step_small.npz', 5)
    torch.cuda.synchronize()
    fm = golden('depth_metrics.npz')
    metric, median = algo.compute_depth_metrics(inputs, outputs)
    assert METRIC_NAMES == ['abs_rel', 'sq_rel', 'rms', 'log_rms', 'a1', 'a2', 'a3']
    for k in METRIC_NAMES:
        for what, got in (('metric', metric[k]), ('median', median[k])):
            ref = float(fm[f'step_{what}_{k}'])
            assert abs(float(got) - ref) <= 1e-4 * abs(ref) + 1e-7, f'{what} {k}: GPU step {float(got):.8g} vs reference {ref:.8g}'


def _fro(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu().reshape(a.shape)
    return float((a - b).norm() / max(float(b.norm()), 1e-30)), float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


def _near_decisions(O, ci, co, go, c, frames, noise, rel_poses=None, margin=1e-4, cell_margin=3e-4):
    """Pixels of camera c within `margin` of a discrete loss decision (temporal min, auto-mask,
    spatio-temporal min), whose warp masks differ between GPU and oracle, or — with `rel_poses` —
    whose bilinear sample point in any warp (temporal, spatial, spatio-temporal) lies within
    `cell_margin` px of a texel grid line, dilated by the SSIM window (a decision at q moves the
    gradient of q's 3x3 neighbourhood).

    The grid-line decision: the warp's value is continuous there but its derivative in the sample
    coordinate jumps from one texel difference to the next (grid_sample's floor, ATen
    GridSampler.h), so a coordinate one fp32 ulp to either side (6.1e-5 px at x in [512, 1024))
    picks a different d loss / d disp.  At 384x640 this is 1.1% of the pixels, and every
    GPU / oracle difference above 6e-5 of the gradient scale sat on one (round 6,
    tools/diag_gradchain.py)."""
    target = ci[('color', 0, 0)][:, c]
    rep = torch.cat([O.photometric(co[('color', f, 0)], target) for f in frames[1:]], 1).detach()
    idn = torch.cat([O.photometric(ci[('color', f, 0)][:, c], target) for f in frames[1:]], 1) + noise

    def tie(m):     # exact ties resolve identically on both sides (equal inputs, first index wins)
        return (m > 0) & (m < margin)
    near = tie(rep.max(1, keepdim=True).values - rep.min(1, keepdim=True).values)
    near |= tie((rep.min(1, keepdim=True).values - idn.min(1, keepdim=True).values).abs())
    if ('overlap', frames[1], 0) in co:
        st = torch.cat([O.photometric(co[('overlap', f, 0)], target) for f in frames[1:]], 1).detach()
        near |= tie(st.max(1, keepdim=True).values - st.min(1, keepdim=True).values)
    for key in [('color_mask', f, 0) for f in frames[1:]] + [('overlap_mask', f, 0) for f in frames]:
        if key in co and key in go:
            near |= (go[key].detach().cpu() != co[key].detach())
    if rel_poses is not None:
        depth = co[('depth', 0)].detach()
        B, _, H, W = depth.shape
        pts = O.backproject(ci[('inv_K', 0)][:, c], depth)
        warps = [(ci[('K', 0)][:, c], co[('cam_T_cam', 0, f)].detach()) for f in frames[1:]]
        warps += [(ci[('K', 0)][:, src], T) for (f, src), T in rel_poses.items()]
        for K, T in warps:
            gx, gy = O.reproject(K, T, pts, H, W)
            ix, iy = O._unnorm(gx, W), O._unnorm(gy, H)
            inside = (ix > -1) & (ix < W) & (iy > -1) & (iy < H)
            grid = torch.minimum((ix - ix.round()).abs(), (iy - iy.round()).abs()) < cell_margin
            near |= (inside & grid).view(B, 1, H, W)
    return torch.nn.functional.max_pool2d(near.float(), 3, 1, 1) > 0


class _FusionDecisions:
    """Records the GPU step's LeakyReLU decisions on both nets' fusion paths as sign masks in the
    oracle's layouts while the step's forward runs: the fused aggregation conv (conv1x1) of each
    net, K1's folded 1x1 convs (conv_non_overlap / conv_overlap), K3C (the depth reduce_dim[0])
    and K2C (the pose reduce_dim[0]).  The pose masks are in call order, pairs stacked pair-major
    (the batched-pairs layout; one call per pair gives the same order).  Also reduce_dim's second
    activation (both nets) and the pose decoder's ReLUs."""

    def __init__(self, algo):
        inner = {k: getattr(m, 'module', m) for k, m in algo.models.items()}
        self.conv = {'depth': inner['depth_net'].conv1x1, 'pose': inner['pose_net'].conv1x1}
        self.relu = inner['pose_net'].pose_decoder.relu
        self.agg, self.vox, self.y0, self.y1, self.dec = {}, None, {}, {}, []

    def __enter__(self):
        from vfdepth_amd import kernels as KN
        from vfdepth_amd import network as NW
        from vfdepth_amd.fusion import VFNet
        self._orig = (NW._aggregate, KN.FuseDepth.apply, KN.ProjConv.apply, KN.PadConv.apply,
                      VFNet.project_voxel_into_image, VFNet._reduce)
        agg_fn, fuse_fn, proj_fn, pad_fn, pvi_fn, red_fn = self._orig
        # reduce_dim's second activation: the depth net's projected features, the pose net's BEV
        # (the returned maps are the LeakyReLU outputs: their signs are the decisions)

        def project_voxel_into_image(net, *a):
            out = pvi_fn(net, *a)
            self.y1.setdefault('depth', []).append((out.detach() > 0).cpu())
            return out

        def reduce(net, *a):
            out = red_fn(net, *a)
            if net.model == 'pose':
                self.y1.setdefault('pose', []).append((out.detach() > 0).cpu())
            return out
        VFNet.project_voxel_into_image, VFNet._reduce = project_voxel_into_image, reduce
        # the pose decoder's ReLU (one module, three calls per forward)
        self._hook = self.relu.register_forward_hook(lambda m, i, o: self.dec.append((o.detach() > 0).cpu()))

        def aggregate(encoder, conv1x1, *a, **kw):
            feats, agg = agg_fn(encoder, conv1x1, *a, **kw)
            for net, conv in self.conv.items():
                if conv1x1 is conv:                             # [B', N, C, h, w]
                    self.agg.setdefault(net, []).append((agg.detach() > 0).flatten(0, 1).cpu())
            return feats, agg

        def fuse(*a):
            vox = fuse_fn(*a)                                   # [B, V, Cv]
            self.vox = (vox.detach() > 0).permute(0, 2, 1).cpu()
            return vox

        def interior(y0):                                      # reflect-padded by one pixel
            return (y0.detach()[:, :, 1:-1, 1:-1] > 0).cpu()

        def proj(*a):
            y0 = proj_fn(*a)
            self.y0.setdefault('depth', []).append(interior(y0))
            return y0

        def pad(*a):
            y0 = pad_fn(*a)
            self.y0.setdefault('pose', []).append(interior(y0))
            return y0
        NW._aggregate, KN.FuseDepth.apply, KN.ProjConv.apply, KN.PadConv.apply = aggregate, fuse, proj, pad
        return self

    def __exit__(self, *exc):
        from vfdepth_amd import kernels as KN
        from vfdepth_amd import network as NW
        from vfdepth_amd.fusion import VFNet
        (NW._aggregate, KN.FuseDepth.apply, KN.ProjConv.apply, KN.PadConv.apply,
         VFNet.project_voxel_into_image, VFNet._reduce) = self._orig
        self._hook.remove()
        self.agg = {k: torch.cat(v, 0) for k, v in self.agg.items()}
        self.y0 = {k: torch.cat(v, 0) for k, v in self.y0.items()}
        self.y1 = {k: torch.cat(v, 0) for k, v in self.y1.items()}
        # the decoder's calls in order, three per forward: regroup as [squeeze, pose 0, pose 1]
        # masks over all of the forwards' batches (pair-major)
        self.dec = [torch.cat(self.dec[j::3], 0) for j in range(3)] if self.dec else []


class _MaskedLReLU(torch.nn.Module):
    """LeakyReLU(slope) — ReLU for slope 0 — whose slope choice follows given masks (one per call,
    in call order): the value differs from the activation only where a mask disagrees with the
    sign, i.e. within fp32 rounding of zero; the gradient takes the recorded decisions."""

    def __init__(self, masks, slope=0.1):
        super().__init__()
        self.masks, self.calls, self.slope = masks, 0, slope

    def forward(self, x):
        m = self.masks[self.calls]
        self.calls += 1
        assert m.shape == x.shape, (m.shape, x.shape)
        return torch.where(m, x, x * self.slope)


class _HoldFusionDecisions:
    """Runs the oracle step with the fusion-path LeakyReLU decisions of the GPU step
    (_FusionDecisions): each net's conv1x1 activation (the depth net's called once on B*N images,
    the pose net's once per frame pair), the oracle's K1 1x1-conv activation
    (vfd_oracle._conv1x1_lrelu), reduce_dim's two activations (depth: once per camera; pose: once
    per frame pair) and the pose decoder's ReLU (three calls per frame pair; its maps are small, so
    one flipped ReLU there visibly moves its weight gradients)."""

    def __init__(self, O, dn, pn, dec, B, N):
        self.O, self.dn, self.pn, self.dec, self.B, self.N = O, dn, pn, dec, B, N

    def __enter__(self):
        O, dn, pn, dec, B, N = self.O, self.dn, self.pn, self.dec, self.B, self.N
        self._orig = (dn.conv1x1[2], dn.fusion_net.reduce_dim[2], pn.conv1x1[2], pn.fusion_net.reduce_dim[2],
                      dn.fusion_net.reduce_dim[5], pn.fusion_net.reduce_dim[5], pn.pose_decoder.relu,
                      O._conv1x1_lrelu)
        if 'depth' in dec.y1:
            y1 = dec.y1['depth'].view(B, N, *dec.y1['depth'].shape[1:])
            dn.fusion_net.reduce_dim[5] = _MaskedLReLU([y1[:, c] for c in range(N)])
        if 'pose' in dec.y1:
            pn.fusion_net.reduce_dim[5] = _MaskedLReLU(list(dec.y1['pose'].split(B)))
        if dec.dec:                              # per pair: squeeze, pose 0, pose 1
            P = dec.dec[0].shape[0] // B
            pn.pose_decoder.relu = _MaskedLReLU([dec.dec[j][p * B:(p + 1) * B] for p in range(P) for j in range(3)],
                                                slope=0.0)
        dn.conv1x1[2] = _MaskedLReLU([dec.agg['depth']])
        pn.conv1x1[2] = _MaskedLReLU(list(dec.agg['pose'].split(B * N)))
        if 'depth' in dec.y0:                    # K3C ran (fp32, 64 voxel channels, D <= 64)
            y0 = dec.y0['depth'].view(B, N, *dec.y0['depth'].shape[1:])
            dn.fusion_net.reduce_dim[2] = _MaskedLReLU([y0[:, c] for c in range(N)])
        if 'pose' in dec.y0:                     # K2C ran (fp32)
            pn.fusion_net.reduce_dim[2] = _MaskedLReLU(list(dec.y0['pose'].split(B)))

        def conv1x1_lrelu(x, weight, bias):      # the no- and the ov-branch: one K1 output sign
            y = torch.einsum('oc,bcv->bov', weight[:, :, 0], x) + bias.view(1, -1, 1)
            return torch.where(dec.vox, y, y * O.LRELU)
        O._conv1x1_lrelu = conv1x1_lrelu
        return self

    def __exit__(self, *exc):
        (self.dn.conv1x1[2], self.dn.fusion_net.reduce_dim[2], self.pn.conv1x1[2], self.pn.fusion_net.reduce_dim[2],
         self.dn.fusion_net.reduce_dim[5], self.pn.fusion_net.reduce_dim[5], self.pn.pose_decoder.relu,
         self.O._conv1x1_lrelu) = self._orig


@pytest.mark.parametrize('shape', ['small', 'full'])
def test_full_step_gradient_chain(shape):
    """Full fusion step, gradient parity stage by stage with the decisions held fixed, at the
    fixtures' reduced shape (96x160, 40x40x10 voxels, D=16) and at BASELINE config 2's full shape
    (6 x 384x640, 100x100x20 voxels, D=50 — the shape the bench measures):

    1. loss path: d total / d disp and d total / d cam_T_cam of the GPU step against the CPU
       oracle's view synthesis + losses (view_rendering.py, multi_cam_loss.py) evaluated on the GPU's
       own disparities and poses (same decisions up to the near-ties of this one evaluation);
    2. nets: the GPU's upstream gradients injected into the CPU oracle step's disparity and pose
       outputs (same modules, weights and inputs, evaluated in fp64) must give the GPU's parameter gradients — the
       backward of K1/K2/K3, the fused aggregation and the dense layers — with the nets'
       fusion-path LeakyReLU decisions (conv1x1, K1's 1x1 convs, K3C, K2C) taken from the GPU step: at
       384x640, 7 of K3C's 5.9M pre-activations sit within 4e-6 of zero and flip between fp32
       evaluations; with them flipped, d reduce_dim[0].bias (a sum with heavy cancellation) moves
       by 3.8e-4 relative and the gradients upstream of it by up to 1.4e-3 (round 6,
       tools/diag_gradchain.py nets --fp64: the GPU's decisions in an fp64 oracle leave 1.2e-5).
    (models/vfdepth.py:191-313; network/volumetric_fusionnet.py:197-230)
    """
    from oracle import vfd_oracle as O
    from vfdepth_amd import synth
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.network import FusedDepthNet, FusedPoseNet
    from vfdepth_amd.vfdepth import VFDepthAlgo
    if shape == 'small':
        fx = golden('step_small.npz')
        cfg = G.step_cfg()
        N = cfg['data']['num_cams']
        noise = torch.stack([torch.tensor(fx[f'noise_c{c}']) for c in range(N)])
        inputs = synth.make_batch(cfg, seed=5, with_depth=True)
    else:
        fx = golden('step_full.npz')
        cfg = G.full_cfg()
        N, t = cfg['data']['num_cams'], cfg['training']
        noise = torch.stack(G.full_noise(fx, (t['batch_size'], len(t['frame_ids']) - 1, t['height'], t['width'])))
        inputs = synth.make_batch(cfg, seed=G.FULL_SEED, with_depth=True)
        torch.set_num_threads(max(1, min(16, len(os.sched_getaffinity(0)))))   # the CPU oracle's step
    frames = cfg['training']['frame_ids']
    cpu_inputs = {k: v.clone() if torch.is_tensor(v) else v for k, v in inputs.items()}
    algo = VFDepthAlgo(cfg, 0)
    for m in algo.models.values():
        m.load_state_dict(seeded_state_dict(m, seed=G.STEP_SEED))
    algo.set_train()
    with _FusionDecisions(algo) as dec:
        outputs, losses = algo.process_batch(inputs, 0, noise=noise.to(DEV))
    assert set(dec.agg) == {'depth', 'pose'} and dec.vox is not None, 'a fusion-path kernel did not run'
    disp = outputs['_disp_all'][0]
    disp.retain_grad()
    Ts = {(c, f): outputs[('cam', c)][('cam_T_cam', 0, f)] for c in range(N) for f in frames[1:]}
    # the fusion pose model's per-camera poses are views of one [B, N, 4, 4] tensor per frame,
    # which the batched warp path consumes: the gradient lands there
    P_all = outputs.get('_cam_T_cam')
    for t in (P_all.values() if P_all is not None else Ts.values()):
        t.retain_grad()

    def t_grad(k):
        return P_all[k[1]].grad[:, k[0]] if P_all is not None else Ts[k].grad
    losses['total_loss'].backward()
    # 1. loss path on the GPU's disparities / poses
    ci = dict(cpu_inputs)
    ci['extrinsics_inv'] = torch.inverse(ci['extrinsics'])
    d_leaf = disp.detach().cpu().clone().requires_grad_(True)
    T_leaf = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in Ts.items()}
    total = 0.0
    near = torch.zeros_like(d_leaf, dtype=torch.bool)
    for c in range(N):
        co = {('disp', 0): d_leaf[:, c:c + 1]}
        co[('depth', 0)] = O.to_depth(co[('disp', 0)], ci[('K', 0)][:, c], cfg)
        for f in frames[1:]:
            co[('cam_T_cam', 0, f)] = T_leaf[(c, f)]
        rp = O.relative_poses(ci, co, c, cfg)
        O.view_rendering(ci, co, c, rp, cfg)
        total = total + O.cam_loss(ci, co, c, cfg, noise[c])[0]
        near[:, c] = _near_decisions(O, ci, co, outputs[('cam', c)], c, frames, noise[c], rp)[:, 0]
    (total / N).backward()
    keep = ~near
    frac_near = float(near.float().mean())
    assert frac_near < 0.5, f'{frac_near:.3f} of the pixels near a decision'
    print(f'loss path ({shape}): {int(near.sum())} of {near.numel()} px near a decision')
    fro, mx = _fro(disp.grad[keep.to(DEV)], d_leaf.grad[keep])
    assert fro < 1e-3 and mx < 1e-2, f'd loss / d disp (outside {int(near.sum())} near-tie px): fro {fro:.3g}, max {mx:.3g}'
    for k in Ts:
        fro, mx = _fro(t_grad(k), T_leaf[k].grad)
        assert fro < 5e-3, f'd loss / d cam_T_cam{k}: fro {fro:.3g}'
    # 2. nets: inject the GPU's upstream gradients into the oracle step
    # (in fp64: the fp32 oracle is itself up to 1e-3 from the exact gradient of the pose net's
    # aggregation conv — tools/diag_gradchain.py nets vs nets --fp64 — as far as the GPU is)
    f64 = torch.float64
    dn, pn = FusedDepthNet(cfg), FusedPoseNet(cfg)
    dn.load_state_dict(seeded_state_dict(dn, seed=G.STEP_SEED))
    pn.load_state_dict(seeded_state_dict(pn, seed=G.STEP_SEED))
    dn.train().to(f64)
    pn.train().to(f64)
    cpu_inputs = {k: v.to(f64) if torch.is_tensor(v) and v.is_floating_point() else v for k, v in cpu_inputs.items()}
    held = {}
    hook = dn.decoder.register_forward_hook(lambda m, i, o: held.__setitem__('disp', o[('disp', 0)]))
    with _HoldFusionDecisions(O, dn, pn, dec, cfg['training']['batch_size'], N):
        o_out, _ = O.process_batch(O.nets_from_modules(dn, pn), cpu_inputs, cfg, [n.to(f64) for n in noise])
    hook.remove()
    tensors = [held['disp']] + [o_out[('cam', c)][('cam_T_cam', 0, f)] for (c, f) in Ts]
    grads = [disp.grad.detach().cpu().reshape(held['disp'].shape).to(f64)] + [t_grad(k).detach().cpu().to(f64) for k in Ts]
    torch.autograd.backward(tensors, grads)
    # The ResNet encoders' train-mode BatchNorm backward cancels (dx = (g - mean g - x̂·mean g x̂)/σ):
    # on the CPU alone a 1e-7 relative input perturbation moves encoder gradients by up to 4e-3
    # (fp64 vs fp32: 6e-3), so encoder parameters get 1e-2; every layer on the hot-path side of the
    # chain (aggregation conv, VFNet, decoders) has no BatchNorm in its backward and gets 2e-4.
    bad, margins = [], []
    for mname, ref_net in (('depth_net', dn), ('pose_net', pn)):
        got = dict(algo.models[mname].named_parameters())
        for pname, p in ref_net.named_parameters():
            fro, mx = _fro(got[pname].grad, p.grad)
            if not pname.startswith('encoder.'):
                margins.append((fro, f'{mname}.{pname}'))
            # (encoder: norm only — at the fixture's 96x160 the deep layers see 60 positions per
            # camera, so one ReLU / max-pool kink crossing moves single weight-gradient entries)
            # (hot-path side: 2e-4 — with the decisions held, 2.9e-5 at most at 384x640, round 6)
            tol = (1e-2, float('inf')) if pname.startswith('encoder.') else (2e-4, 1e-2)
            if not (fro < tol[0] and mx < tol[1]):
                bad.append(f'{mname}.{pname}: fro {fro:.3g}, max {mx:.3g}')
    print(f'nets ({shape}): largest non-encoder gradient differences (fro): '
          + ', '.join(f'{n} {f:.2g}' for f, n in sorted(margins, reverse=True)[:4]))
    assert not bad, f'{len(bad)} parameter gradients off: ' + '; '.join(bad[:8])


@pytest.mark.skipif(os.environ.get('VFD_TEST_GRAPHS') == '0', reason='VFD_TEST_GRAPHS=0')
def test_graph_replay_matches_eager():
    """A captured HIP-graph training step (forward, losses, backward, Adam) computes the same step
    as the eager path: after capture, both models are reset to the same initial state (weights,
    BN buffers, Adam moments, device noise counter), one replay and one eager step run from it,
    and their losses and parameter gradients must agree (up to fp32 atomic-order noise)."""
    from vfdepth_amd import synth
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.vfdepth import VFDepthAlgo
    cfg = G.step_cfg()
    # a moving scene: the auto-masked reprojection loss averages over most pixels, so an
    # auto-mask decision that flips between the runs (a near-tie; the captured and the eager
    # MIOpen launches round differently, and the non-deterministic mode sums some gradient terms
    # in atomic order) moves the loss by ~1/pixels.  (A static scene masks nearly every pixel: the loss is
    # then a mean over a handful of pixels and one flip moves it by percents.)
    batch = synth.make_batch(cfg, seed=99, device=DEV)
    algos, init = [], {}
    for _ in range(2):
        a = VFDepthAlgo(cfg, 0)
        for name, m in a.models.items():
            init[name] = seeded_state_dict(m, seed=G.STEP_SEED)
            m.load_state_dict(init[name])
        a.set_train()
        a.set_optimizer(capturable=True)
        a.losses.device_seed = True
        algos.append(a)
    # both run the DEFAULT step: frame pairs as one batch, the pose branch on its own stream (the
    # capture forks and joins it); the eager side is the bench's eager step
    assert algos[0].pose.batch_pairs and algos[1].pose.batch_pairs
    # an eager branch-stream step first: the capture must not depend on streams an earlier eager
    # step used (its branch stream is joined only when the step itself forked it)
    algos[0].train_step(dict(batch))
    graphed = algos[0].graphed_train_step(batch, warmup=2)
    assert algos[0]._bstream is not None, 'the captured step did not use the pose branch stream'
    assert algos[0].pose.batch_pairs, 'graphed_train_step changed the pose-pair setting'
    # rewind the graphed model to the initial state, in place (the graph holds these buffers)
    for name, m in algos[0].models.items():
        m.load_state_dict(init[name])
    for st in algos[0].optimizer.state.values():
        for t in st.values():
            if torch.is_tensor(t):
                t.zero_()
    algos[0].losses._counter.zero_()
    lg = {k: v.clone() for k, v in graphed().items()}
    # two eager steps of the twin model from the same state: outside the deterministic mode some
    # sums run in atomic order (K3's split tiles, the fusion plan's bucket order, MIOpen's split-K
    # forward and weight-gradient solvers), so eager steps differ among themselves and near-tie
    # auto-mask decisions flip; the replay must agree with eager as closely as eager agrees with
    # itself (bit-identity under the deterministic flag is test_deterministic_steps_*)
    runs = []
    for _ in range(2):
        algos[1].optimizer.zero_grad(set_to_none=True)
        if getattr(algos[1].losses, '_counter', None) is not None:
            algos[1].losses._counter.zero_()       # the same identity noise as the replay's
        out_i, le_i = algos[1].process_batch(dict(batch), 0)
        le_i['total_loss'].backward()
        torch.cuda.synchronize()
        runs.append((out_i, {k: v.detach().clone() for k, v in le_i.items()},
                     {net: {n: p.grad.detach().clone() for n, p in algos[1].models[net].named_parameters()}
                      for net in ('depth_net', 'pose_net')}))
    (out_e, le, g_e1), (out_e2, le2, g_e2) = runs
    for c in range(cfg['data']['num_cams']):
        close(graphed.outputs[('cam', c)][('depth', 0)], out_e[('cam', c)][('depth', 0)], f'depth cam {c}',
              atol=1e-5, rtol=1e-5)

    def nflips(oa, ob):
        return sum(int((oa[('cam', c)][('reproj_mask', 0)] != ob[('cam', c)][('reproj_mask', 0)]).sum())
                   for c in range(cfg['data']['num_cams']))
    flips, flips_ee = nflips(graphed.outputs, out_e), nflips(out_e2, out_e)
    npix = sum(out_e[('cam', c)][('reproj_mask', 0)].numel() for c in range(cfg['data']['num_cams']))
    assert flips <= max(16, npix // 1000), f'{flips} auto-mask flips between graph replay and eager'
    for k in ('total_loss', 'reproj_loss', 'spatio_loss', 'spatio_tempo_loss', 'smooth'):
        a_, b_, c_ = float(lg[k]), float(le[k]), float(le2[k])
        # 4e-4 relative: a handful of flipped auto-mask pixels in the spatio-temporal overlap terms
        # (means over a few thousand pixels) moves them by ~1e-4 (graph vs eager 5.6e-5 on 0.247
        # with 17 flips, round 6); the bitwise check is test_graph_replay_bit_identical
        tol = max(1e-5 + 1e-4 * abs(b_), 4.0 * abs(c_ - b_), 4e-4 * abs(b_))
        assert abs(a_ - b_) <= tol, (f'graph vs eager {k}: {a_:.7g} vs {b_:.7g} (eager vs eager {c_:.7g}; '
                                     f'{flips} / {flips_ee} auto-mask flips graph / eager vs eager)')

    def rel_diff(ga, gb):
        diff = ref = 0.0
        for name, g in gb.items():
            diff += float((ga[name].double() - g.double()).pow(2).sum())
            ref += float(g.double().pow(2).sum())
        return diff, ref

    for net in ('depth_net', 'pose_net'):
        pg = {n: p.grad for n, p in algos[0].models[net].named_parameters()}
        diff, ref = rel_diff(pg, g_e1[net])
        if ref == 0.0:
            # static scene: the identity term wins every auto-mask decision, so no temporal warp
            # (the pose net's only path into the loss) contributes — both runs must agree on that
            assert diff == 0.0, f'{net}: eager gradient is zero but the replay\'s is not ({diff:.3g})'
            continue
        rel = (diff / ref) ** 0.5
        d2, r2 = rel_diff(g_e2[net], g_e1[net])
        spread = (d2 / r2) ** 0.5
        worst = sorted(((float((pg[k] - g_e1[net][k]).norm()) / max(float(g_e1[net][k].norm()), 1e-30), k)
                        for k in g_e1[net]), reverse=True)[:5]
        # 1e-2: auto-mask flips alone move eager-vs-eager gradients by 1e-4 .. 3e-2 (measured over
        # round-6 runs); a missing dependency in the graph moved them by 0.1 .. 10 (the K1 / K2
        # backwards sharing the plan's split-tile pool, fixed).  Bit-for-bit equality of the replay
        # and the eager step is test_graph_replay_bit_identical's (deterministic mode, no flips).
        assert rel < max(1e-2, 4.0 * spread), \
            (f'{net}: gradient rel diff {rel:.3g} (eager-vs-eager {spread:.3g}, {flips} auto-mask flips); worst: '
             + ', '.join(f'{k} {r:.3g}' for r, k in worst))
    # a second replay draws fresh identity noise and keeps training
    l2 = graphed()
    assert torch.isfinite(l2['total_loss']).item()


@pytest.mark.parametrize('ddp', [False, True], ids=['plain', 'ddp_world1'])
def test_graph_replay_bit_identical(ddp):
    """The captured DEFAULT step (batched pose pairs, pose branch forked / joined inside the capture;
    under DDP the wrappers built on the capture stream, DDP's RCCL all-reduce captured) replays bit
    for bit what the eager step computes — losses, depth maps, every parameter gradient — under the
    deterministic flag, where two eager steps are bit-identical; three replays agree with each other,
    and two replays back to back (no host synchronisation between them) with two synchronised ones.
    A fresh process (tests/graph_det_worker.py): MIOpen reads its determinism switch once.
    (trainer/vfdepth_trainer.py:61-66, models/vfdepth.py:56-71)"""
    import json
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    res = subprocess.run([sys.executable, os.path.join(here, 'graph_det_worker.py')] + (['--ddp'] if ddp else []),
                         capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stderr[-3000:]
    r = json.loads(res.stdout.strip().splitlines()[-1])
    assert r['branch_stream'] and r['pairs_batched'] and r['ddp'] == ddp, r
    assert not r['eager_vs_eager'], f"eager steps differ in deterministic mode: {r['eager_vs_eager']}"
    assert not r['replay_vs_replay'], f"replays differ: {r['replay_vs_replay']}"
    assert not r['replay_vs_eager'], f"replay differs from the eager step: {r['replay_vs_eager']}"
    assert not r['back_to_back_vs_synced'], f"back-to-back replays differ: {r['back_to_back_vs_synced']}"


def test_bf16_nets_step_tracks_fp32():
    """Config 3's mixed precision (`net_precision='bf16'`): the dense nets run under bf16 autocast,
    the HIP fusion / geometry / loss kernels stay fp32.  Same weights and inputs as the fp32 step:
    the HIP ops must still receive fp32 tensors, the nets must hand back fp32 depths and poses, and
    the losses / gradients must track the fp32 step within bf16 resolution (8 mantissa bits
    through ~40 layers: 5e-2 relative on the losses, gradient cosine > 0.9 per net)."""
    from vfdepth_amd import synth
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.vfdepth import VFDepthAlgo
    runs = {}
    for prec in ('fp32', 'bf16'):
        cfg = G.step_cfg()
        cfg['training']['net_precision'] = prec
        algo = VFDepthAlgo(cfg, 0)
        for m in algo.models.values():
            m.load_state_dict(seeded_state_dict(m, seed=G.STEP_SEED))
        algo.set_train()
        inputs = synth.make_batch(cfg, seed=5)
        noise = torch.zeros(6, 1, 2, cfg['training']['height'], cfg['training']['width'], device=DEV)
        outputs, losses = algo.process_batch(inputs, 0, noise=noise)
        losses['total_loss'].backward()
        torch.cuda.synchronize()
        assert outputs[('cam', 0)][('depth', 0)].dtype == torch.float32
        assert outputs[('cam', 0)][('cam_T_cam', 0, -1)].dtype == torch.float32
        grads = {n: torch.cat([p.grad.flatten() for p in m.parameters() if p.grad is not None])
                 for n, m in algo.models.items()}
        runs[prec] = ({k: float(v) for k, v in losses.items() if torch.is_tensor(v) and v.numel() == 1}, grads)
    (l32, g32), (l16, g16) = runs['fp32'], runs['bf16']
    for k in ('total_loss', 'reproj_loss', 'spatio_loss', 'spatio_tempo_loss'):
        assert math.isfinite(l16[k]), k
        assert abs(l16[k] - l32[k]) <= 5e-2 * abs(l32[k]) + 1e-6, f'{k}: bf16 {l16[k]} vs fp32 {l32[k]}'
    for n in g32:
        assert torch.isfinite(g16[n]).all(), n
        cos = float(torch.nn.functional.cosine_similarity(g16[n].double(), g32[n].double(), dim=0))
        assert cos > 0.9, f'{n}: gradient cosine {cos:.3f} between the bf16 and fp32 steps'


@pytest.mark.parametrize('config', [2, 4, 5])
def test_fusion_adjoint_at_full_size(config):
    """Size-independent property at BASELINE.json's full sizes (configs 2 and 4 at B=1, config 5 at
    its per-GPU batch B=4), where the oracle is too slow: K2 (pose fusion, affine in the features) and K3 (voxel -> frustum, linear)
    backward kernels are the exact adjoints of their forward kernels,
    <fwd(x) - fwd(0), g> == <x, bwd(g)>, reflect-pad copies and zero padding included.  Inner
    products in fp64 over fp32 values; tolerance 1e-5 of sum |fwd(x) * g| (fp32 rounding of the
    per-element sums in the two kernels)."""
    import bench
    from vfdepth_amd import kernels as KN
    from vfdepth_amd import synth
    from vfdepth_amd.geometry import inverse4x4
    B = 4 if config == 5 else 1
    cfg, _ = bench.make_cfg(config, B)
    space = KN.VoxelSpace(cfg, DEV)
    b = synth.make_batch(cfg, seed=3, device=DEV)
    if B > 1:                      # per-element geometry (common.perturb_rig)
        b = {k: (v.to(DEV) if torch.is_tensor(v) else v) for k, v in G.perturb_rig(synth.make_batch(cfg, seed=3), 4).items()}
    lvl = cfg['model']['fusion_level'] + 1
    Einv = inverse4x4(b['extrinsics'])
    mask_lo = KN.mask_lowres(space, b['mask'])
    gen = torch.Generator(device=DEV).manual_seed(config)
    C, Cv = cfg['model']['fusion_feat_in_dim'], cfg['model']['voxel_pre_dim'][-1]

    def check(lhs_terms, rhs, what):
        lhs = float(lhs_terms.double().sum())
        scale = float(lhs_terms.double().abs().sum())
        assert abs(lhs - rhs) <= 1e-5 * scale, f'{what}: <Ax, g> {lhs} vs <x, A^T g> {rhs} (scale {scale})'

    # K2: features [B, N, C, h, w] -> padded pose volume (affine: the depth channel is constant)
    plan = KN.FusionPlan(space, mask_lo, b['K', lvl], Einv)
    feats = torch.randn(B, 6, C, space.h, space.w, device=DEV, generator=gen, requires_grad=True)
    out = KN.FusePose.apply(space, plan, feats)
    with torch.no_grad():
        out0 = KN.FusePose.apply(space, plan, torch.zeros_like(feats))
    g = torch.randn(out.shape, device=DEV, generator=gen)
    out.backward(g)
    check((out.detach() - out0) * g, float((feats.detach().double() * feats.grad.double()).sum()), 'K2')
    del out, out0, g, feats
    # K3: voxels [B, V, Cv] -> frustum features (linear)
    vox = torch.randn(B, space.V, Cv, device=DEV, generator=gen, requires_grad=True)
    out = KN.VoxelProject.apply(space, vox, b['inv_K', lvl], b['extrinsics'])
    g = torch.randn(out.shape, device=DEV, generator=gen).contiguous(memory_format=torch.channels_last)
    out.backward(g)
    check(out.detach() * g, float((vox.detach().double() * vox.grad.double()).sum()), 'K3')


# ------------------------------------------------------------------------------------ depth synthesis
def test_depth_synthesis_kernel_against_reference():
    """get_virtual_depth (view_rendering.py:84-116) through the C ABI (vfd_depth_syn_fwd/bwd)
    against the reference's fixture: warped depth, mask (exact), d source depth, d target depth."""
    from vfdepth_amd import kernels as KN
    fx = golden('virtual_depth.npz')
    c = G.virtual_depth_case()
    B = c['src_depth'].shape[0]
    T = c['T'].to(DEV)
    M = (c['src_K'].to(DEV) @ torch.inverse(T))[:, :3, :].reshape(B, 1, 1, 3, 4).contiguous()
    zrow = T[:, 2, :].reshape(B, 1, 1, 4).contiguous()
    tab = torch.zeros(1, 1, dtype=torch.int32, device=DEV)
    sd = c['src_depth'].to(DEV).requires_grad_(True)           # [B,1,H,W]: camera 0 as the source
    td = c['tar_depth'].to(DEV).requires_grad_(True)           # camera 0's augmented view
    invK = c['tar_invK'].to(DEV).reshape(B, 1, 4, 4)
    d, m = KN.DepthSynthesis.apply(tab, c['min_depth'], c['max_depth'], td, sd, c['src_mask'].to(DEV)[:, 0:1],
                                   invK, M, zrow)
    close(d[:, :, 0], fx['depth'], 'warped depth')
    close(m[:, :, 0], fx['mask'], 'warped mask', atol=0, rtol=0)
    (d[:, :, 0] * G.seeded_randn(fx['depth'].shape, 61).to(DEV)).sum().backward()
    gclose(sd.grad, fx['d_src_depth'], 'd source depth')
    gclose(td.grad, fx['d_tar_depth'], 'd augmented-view depth')


def test_depth_synthesis_ordered_backward(monkeypatch):
    """The deterministic mode's depth-synthesis backward (vfd_depth_syn_bwd_ordered: the scattered
    source-depth gradient summed in 128-bit fixed point) against the reference fixture, bitwise
    equal over repeated runs, and within fp32 summation error of the atomic form."""
    from vfdepth_amd import kernels as KN
    fx = golden('virtual_depth.npz')
    c = G.virtual_depth_case()
    B = c['src_depth'].shape[0]
    T = c['T'].to(DEV)
    M = (c['src_K'].to(DEV) @ torch.inverse(T))[:, :3, :].reshape(B, 1, 1, 3, 4).contiguous()
    zrow = T[:, 2, :].reshape(B, 1, 1, 4).contiguous()
    tab = torch.zeros(1, 1, dtype=torch.int32, device=DEV)
    invK = c['tar_invK'].to(DEV).reshape(B, 1, 4, 4)
    gout = G.seeded_randn(fx['depth'].shape, 61).to(DEV)

    def grads(det, scale=1.0):
        monkeypatch.setenv('VFD_DETERMINISTIC', '1' if det else '0')
        sd = c['src_depth'].to(DEV).requires_grad_(True)
        td = c['tar_depth'].to(DEV).requires_grad_(True)
        d, _ = KN.DepthSynthesis.apply(tab, c['min_depth'], c['max_depth'], td, sd,
                                       c['src_mask'].to(DEV)[:, 0:1], invK, M, zrow)
        (d[:, :, 0] * (gout * scale)).sum().backward()
        return sd.grad.clone(), td.grad.clone()

    ref_s, ref_t = grads(False)
    runs = [grads(True) for _ in range(3)]
    for s_, t_ in runs[1:]:
        assert torch.equal(s_, runs[0][0]) and torch.equal(t_, runs[0][1]), 'ordered backward not reproducible'
    gclose(runs[0][0], fx['d_src_depth'], 'd source depth (ordered)')
    gclose(runs[0][1], fx['d_tar_depth'], 'd augmented-view depth (ordered)')
    assert torch.equal(runs[0][1], ref_t)             # the per-pixel gradient has no scatter
    torch.testing.assert_close(runs[0][0], ref_s, rtol=1e-5, atol=1e-7)
    # contributions of magnitude >= 2^25 would overflow the pair's integer part: they take the
    # float atomic instead (depthsyn.hip ds_fixed_ok), so the result stays the atomic form's
    big_s, _ = grads(True, scale=2.0 ** 40)
    big_ref, _ = grads(False, scale=2.0 ** 40)
    assert float(big_ref.abs().max()) >= 2.0 ** 25, 'the scaled case must leave the fixed-point range'
    assert bool(torch.isfinite(big_s).all())
    torch.testing.assert_close(big_s, big_ref, rtol=1e-5, atol=1e-7 * 2.0 ** 40)


def test_full_step_depth_synthesis_against_reference():
    """The aug_depth step (ddad_surround_fusion_augdepth.yaml: augment_extrinsics, second K3C +
    decoder pass, depth synthesis, DepthSynLoss) against the reference's step fixture: every loss
    key, the augmented depths and every camera's warped source depths / masks."""
    from vfdepth_amd import synth
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.vfdepth import VFDepthAlgo
    fx = golden('step_aug_small.npz')
    cfg = G.step_aug_cfg()
    algo = VFDepthAlgo(cfg, 0)
    for m in algo.models.values():
        m.load_state_dict(seeded_state_dict(m, seed=G.STEP_SEED))
    algo.set_train()
    inputs = synth.make_batch(cfg, seed=5, with_depth=True)
    noise = torch.stack([torch.tensor(fx[f'noise_c{c}']) for c in range(6)]).to(DEV)
    torch.manual_seed(1234)               # the augmentation angles: the reference's CPU draw
    outputs, losses = algo.process_batch(inputs, 0, noise=noise)
    losses['total_loss'].backward()
    close(inputs['extrinsics_aug'], fx['extrinsics_aug'], 'extrinsics_aug', atol=1e-5, rtol=1e-5)
    for k in [k for k in fx.files if k.startswith('loss_')]:
        close(losses[k[5:]], fx[k], k)
    for c in range(6):
        o = outputs[('cam', c)]
        close(o[('depth', 0)], fx[f'depth_c{c}'], f'depth cam {c}')
        close(o[('depth', 0, 'aug')], fx[f'depth_aug_c{c}'], f'aug depth cam {c}')
        for j, (dd, mm) in enumerate(zip(o[('tform_depth', 0)], o[('tform_depth_mask', 0)])):
            ref_d, ref_m = fx[f'tform_depth_c{c}_{j}'], fx[f'tform_mask_c{c}_{j}']
            err = (dd.detach().cpu().double() - torch.tensor(ref_d).double()).abs()
            off = err > 1e-4 + 1e-4 * torch.tensor(ref_d).double().abs()
            # samples across a depth discontinuity move with fp32 coordinate rounding: rare
            assert float(off.float().mean()) <= 1e-3, f'tform depth cam {c} src {j}: {int(off.sum())} off'
            assert float((mm.detach().cpu() != torch.tensor(ref_m)).float().mean()) <= 1e-3, f'tform mask {c} {j}'


def test_deterministic_steps_bit_identical():
    """Under torch.backends.cudnn.deterministic (set by the reference's train.py:23-24) two eager
    training steps from the same state give bit-identical losses, depth maps and parameter
    gradients, and so does a third with the pose branch on the main stream instead of its own: the fusion plan's buckets and K3's cell lists are ordered by voxel / sample, K1's
    backward is the plan gather, K3's heavy tiles are not split, every other hot-path reduction
    already sums in a fixed order, and MIOpen runs its deterministic solvers.  In a fresh process
    (tests/det_worker.py): MIOpen reads its determinism switch once, at its first convolution."""
    import json
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    res = subprocess.run([sys.executable, os.path.join(here, 'det_worker.py')], capture_output=True, text=True,
                         timeout=600)
    assert res.returncode == 0, res.stderr[-3000:]
    r = json.loads(res.stdout.strip().splitlines()[-1])
    assert r['depth_equal'] and not r['loss_diff'] and r['d_disp_equal'], r
    assert not r['grad_diff'], f"{len(r['grad_diff'])} of {r['n_grads']} parameter gradients differ: {r['grad_diff']}"
    # the pose branch on its own stream (the default) computes exactly what one stream does
    assert r['single_stream_equal'], 'branch-stream step differs from the single-stream step'

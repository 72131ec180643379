"""Pin the CPU oracle against golden vectors produced by the real reference (CPU only).

The oracle (`oracle/vfd_oracle.py`) restates the hot path with explicit index arithmetic; here it
must reproduce the reference's own outputs and gradients (fixtures from
`tests/golden/gen_golden.py`).  Tolerances: fp32 math in a different operation order, so
1e-5 absolute / 1e-4 relative on values; gradients 1e-4 relative to their scale.
"""
import numpy as np
import pytest
import torch

import common as G
from conftest import golden
from oracle import vfd_oracle as O


def close(a, b, rtol=1e-4, atol=1e-5, what=''):
    a = a.detach().cpu().double().numpy() if torch.is_tensor(a) else np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape, f'{what}: shape {a.shape} vs {b.shape}'
    err = np.abs(a - b)
    tol = atol + rtol * np.abs(b)
    bad = err > tol
    assert not bad.any(), f'{what}: {bad.sum()} / {bad.size} off, max err {err.max():.3g}'


def close_most(a, b, what='', frac=1e-3, rtol=1e-4, atol=1e-5, outlier_rtol=1e-2):
    """`close`, except for at most `frac` of the elements, which may differ by `outlier_rtol`:
    bilinear samples across a depth discontinuity move by (far - near) x (coordinate change), so
    fp32-rounding differences of the sample coordinate show there."""
    a = a.detach().cpu().double().numpy() if torch.is_tensor(a) else np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape, f'{what}: shape {a.shape} vs {b.shape}'
    err = np.abs(a - b)
    bad = err > atol + rtol * np.abs(b)
    assert bad.mean() <= frac, f'{what}: {bad.sum()} / {bad.size} off'
    assert not (err > atol + outlier_rtol * np.abs(b)).any(), f'{what}: max err {err.max():.3g}'


def grad_close(a, b, what='', rel=1e-4):
    a = a.detach().double().numpy()
    b = np.asarray(b, np.float64)
    scale = max(np.abs(b).max(), 1e-12)
    err = np.abs(a - b).max() / scale
    assert err < rel, f'{what}: max err {err:.3g} of scale {scale:.3g}'


def test_fusion_inputs_reproducible():
    fx = golden('fusion_small.npz')
    _, d, _ = G.fusion_case()
    for k, t in (('feats', d['feats']), ('mask', d['mask']), ('K', d['K']), ('E', d['E'])):
        np.testing.assert_array_equal(G.checksum(t), fx['cs_' + k])


def test_fusion_depth_mode():
    fx = golden('fusion_small.npz')
    cfg, d, seeds = G.fusion_case()
    spec = O.VoxelSpec(cfg)
    feats = d['feats'].clone().requires_grad_(True)
    w_no, b_no = [torch.tensor(fx[k]).requires_grad_(True) for k in ('w_no', 'b_no')]
    w_o, b_o = [torch.tensor(fx[k]).requires_grad_(True) for k in ('w_o', 'b_o')]
    vox = O.fuse_depth(spec, feats, d['mask'], d['K'], d['Einv'], w_no, b_no, w_o, b_o)
    close(vox, fx['vox'], what='voxel features')
    (vox * G.seeded_randn(vox.shape, seeds['g_vox'])).sum().backward()
    grad_close(feats.grad, fx['d_feats_depth'], 'd feats')
    for t, k in ((w_no, 'd_w_no'), (b_no, 'd_b_no'), (w_o, 'd_w_o'), (b_o, 'd_b_o')):
        grad_close(t.grad, fx[k], k)
    cnt = np.stack([(np.abs(fx['vox']) > 0).any(1)])
    assert cnt.mean() > 0.05  # fixture exercises non-empty fusion


def test_fusion_pose_mode():
    fx = golden('fusion_small.npz')
    cfg, d, seeds = G.fusion_case()
    spec = O.VoxelSpec(cfg)
    feats = d['feats'].clone().requires_grad_(True)
    v = O.fuse_pose(spec, feats, d['mask'], d['K'], d['Einv'])
    close(v, fx['vpose'], what='pose voxels')
    (v * G.seeded_randn(v.shape, seeds['g_pose'])).sum().backward()
    grad_close(feats.grad, fx['d_feats_pose'], 'd feats (pose)')


def test_voxel_projection():
    fx = golden('fusion_small.npz')
    cfg, d, seeds = G.fusion_case()
    spec = O.VoxelSpec(cfg)
    vleaf = G.seeded_randn(fx['vox'].shape, seeds['vleaf']).requires_grad_(True)
    proj = torch.stack(O.project_voxels(spec, vleaf, d['invK'], d['E']), 1)
    close(proj, fx['proj'], what='frustum features')
    (proj * G.seeded_randn(proj.shape, seeds['g_proj'])).sum().backward()
    grad_close(vleaf.grad, fx['d_vleaf'], 'd voxel')


@pytest.mark.parametrize('name,skip', [('view_small.npz', False), ('view_skip.npz', True)])
def test_view_rendering(name, skip):
    fx = golden(name)
    cfg, batch, depth, poses = G.view_case(skip)
    np.testing.assert_array_equal(G.checksum(depth), fx['cs_depth'])
    for c in range(6):
        d = depth[:, c].clone().requires_grad_(True)
        Ts = {f: poses[(c, f)].clone().requires_grad_(True) for f in (-1, 1)}
        out = {('depth', 0): d, ('cam_T_cam', 0, -1): Ts[-1], ('cam_T_cam', 0, 1): Ts[1]}
        O.view_rendering(batch, out, c, O.relative_poses(batch, out, c, cfg), cfg)
        loss = 0
        for i, k in enumerate(G.VIEW_IMG_KEYS):
            close(out[k], fx[f'{G.key_name(k)}_c{c}'], what=f'{k} cam {c}')
            loss = loss + (out[k] * G.seeded_randn(out[k].shape, 500 + 10 * c + i)).sum()
        for k in G.VIEW_MSK_KEYS:
            close(out[k], fx[f'{G.key_name(k)}_c{c}'], what=f'{k} cam {c}')
        loss.backward()
        grad_close(d.grad, fx[f'd_depth_c{c}'], f'd depth cam {c}', rel=2e-4)
        for f in (-1, 1):
            grad_close(Ts[f].grad, fx[f'd_T_{f}_c{c}'], f'd T{f} cam {c}', rel=2e-4)


def test_losses():
    fx = golden('loss_small.npz')
    cfg, batch, planes = G.loss_case()
    for c in range(6):
        out, leaves = {}, {}
        for k in G.VIEW_IMG_KEYS:
            leaves[k] = planes[(c,) + k].clone().requires_grad_(True)
            out[k] = leaves[k]
        for f in (0, -1, 1):
            out[('overlap_mask', f, 0)] = planes[(c, 'overlap_mask', f, 0)].clone()
        disp = planes[(c, 'disp', 0)].clone().requires_grad_(True)
        out[('disp', 0)] = disp
        cl, terms = O.cam_loss(batch, out, c, cfg, torch.tensor(fx[f'noise_c{c}']))
        close(cl, fx[f'cam_loss_c{c}'], what=f'cam loss {c}')
        for k in ('reproj_loss', 'spatio_loss', 'spatio_tempo_loss', 'smooth'):
            close(terms[k], fx[f'{k}_c{c}'], what=f'{k} {c}')
        close(out[('reproj_loss', 0)], fx[f'reproj_plane_c{c}'], what='reproj plane')
        close(out[('reproj_mask', 0)], fx[f'reproj_mask_c{c}'], what='reproj mask')
        close(out[('overlap_mask', 0, 0)], fx[f'spatio_mask_c{c}'], what='spatio mask')
        cl.backward()
        for k in G.VIEW_IMG_KEYS:
            grad_close(leaves[k].grad, fx[f'd_{G.key_name(k)}_c{c}'], f'd {k} cam {c}')
        grad_close(disp.grad, fx[f'd_disp_c{c}'], f'd disp cam {c}')


def test_depth_metrics():
    fx = golden('metrics.npz')
    errs = O.depth_errors(torch.tensor(fx['pred']), torch.tensor(fx['gt']))
    close(torch.stack([e.double() for e in errs]), fx['errs'], rtol=1e-5, atol=1e-7, what='depth errors')


def test_virtual_depth():
    """A17: ViewRendering.get_virtual_depth (view_rendering.py:84-116), values, masks, gradients."""
    fx = golden('virtual_depth.npz')
    c = G.virtual_depth_case()
    np.testing.assert_array_equal(G.checksum(c['src_depth']), fx['cs_src'])
    sd = c['src_depth'].clone().requires_grad_(True)
    td = c['tar_depth'].clone().requires_grad_(True)
    d, m = O.virtual_depth(sd, c['src_mask'], c['src_invK'], td, c['tar_invK'], c['src_K'], c['T'],
                           c['min_depth'], c['max_depth'])
    close(d, fx['depth'], what='warped depth')
    close(m, fx['mask'], rtol=0, atol=0, what='warped mask')
    assert 0.05 < float(m.mean()) < 0.95
    (d * G.seeded_randn(d.shape, 61)).sum().backward()
    grad_close(sd.grad, fx['d_src_depth'], 'd src depth')
    grad_close(td.grad, fx['d_tar_depth'], 'd tar depth')


def _oracle_step(cfg, fx, aug):
    from vfdepth_amd import synth
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.network import FusedDepthNet, FusedPoseNet
    torch.set_num_threads(8)
    inputs = synth.make_batch(cfg, seed=5, with_depth=True)
    np.testing.assert_array_equal(G.checksum(inputs[('color', 0, 0)]), fx['cs_color'])
    dn, pn = FusedDepthNet(cfg), FusedPoseNet(cfg)
    dn.load_state_dict(seeded_state_dict(dn, seed=G.STEP_SEED))
    pn.load_state_dict(seeded_state_dict(pn, seed=G.STEP_SEED))
    noise = [torch.tensor(fx[f'noise_c{c}']) for c in range(6)]
    angles = torch.tensor(fx['aug_angles']) if aug else None
    with torch.no_grad():
        return inputs, O.process_batch(O.nets_from_modules(dn, pn), inputs, cfg, noise, aug_angles=angles)


@pytest.mark.parametrize('aug', [False, True])
def test_step_oracle(aug):
    """The oracle's whole step (process_batch: pose nets, K2, depth net, K1, K3, decoder, K4, K5
    and, with aug_depth, the depth-synthesis branch) against the reference's step fixture."""
    fx = golden('step_aug_small.npz' if aug else 'step_small.npz')
    cfg = G.step_aug_cfg() if aug else G.step_cfg()
    inputs, (out, losses) = _oracle_step(cfg, fx, aug)
    for k in [k for k in fx.files if k.startswith('loss_')]:
        close(losses[k[5:]], fx[k], what=k)
    for c in range(6):
        close(out[('cam', c)][('depth', 0)], fx[f'depth_c{c}'], what=f'depth cam {c}')
    if aug:
        E_aug = O.augment_extrinsics(inputs['extrinsics'], cfg['training']['aug_angle'], torch.tensor(fx['aug_angles']))
        close(E_aug, fx['extrinsics_aug'], rtol=1e-5, atol=1e-6, what='extrinsics_aug')
        for c in range(6):
            o = out[('cam', c)]
            close(o[('depth', 0, 'aug')], fx[f'depth_aug_c{c}'], what=f'aug depth cam {c}')
            for j, (d, m) in enumerate(zip(o[('tform_depth', 0)], o[('tform_depth_mask', 0)])):
                close_most(d, fx[f'tform_depth_c{c}_{j}'], what=f'tform depth cam {c} src {j}')
                close(m, fx[f'tform_mask_c{c}_{j}'], rtol=0, atol=0, what=f'tform mask cam {c} src {j}')


def test_step_oracle_full_resolution():
    """The oracle's whole step at BASELINE config 2's full shape (6 x 384 x 640, 100 x 100 x 20
    voxels, D = 50) against the reference's own CPU step there (tests/golden/step_full.npz):
    every loss scalar, the 12 poses and the depth maps (every 4th pixel, plus full-map checksums)
    at the north_star tolerance 1e-4 (models/vfdepth.py:191-313)."""
    from vfdepth_amd import synth
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.network import FusedDepthNet, FusedPoseNet
    torch.set_num_threads(8)
    fx = golden('step_full.npz')
    cfg = G.full_cfg()
    inputs = synth.make_batch(cfg, seed=G.FULL_SEED, with_depth=True)
    # full-size double sums: the host's SIMD width changes the last bit (inputs drift would be gross)
    np.testing.assert_allclose(G.checksum(inputs[('color', 0, 0)]), fx['cs_color'], rtol=1e-12)
    t = cfg['training']
    noise = G.full_noise(fx, (t['batch_size'], len(t['frame_ids']) - 1, t['height'], t['width']))
    dn, pn = FusedDepthNet(cfg), FusedPoseNet(cfg)
    dn.load_state_dict(seeded_state_dict(dn, seed=G.STEP_SEED))
    pn.load_state_dict(seeded_state_dict(pn, seed=G.STEP_SEED))
    with torch.no_grad():
        out, losses = O.process_batch(O.nets_from_modules(dn, pn), inputs, cfg, noise)
    for k in [k for k in fx.files if k.startswith('loss_')]:
        close(losses[k[5:]], fx[k], what=k)
    s = G.FULL_SUB
    for c in range(6):
        d = out[('cam', c)][('depth', 0)]
        close(d[..., ::s, ::s], fx[f'depth_sub_c{c}'], what=f'depth cam {c}')
        cs = G.checksum(d)
        close(cs[:2], fx[f'cs_depth_c{c}'][:2], rtol=1e-5, atol=0, what=f'depth checksum cam {c}')
        for f in cfg['training']['frame_ids'][1:]:
            close(out[('cam', c)][('cam_T_cam', 0, f)], fx[f'cam_T_cam_{f}_c{c}'], what=f'T{f} cam {c}')

"""Host-side (non-kernel) pieces of the product on CPU: depth metrics, 4x4 inverse, config."""
import os
import numpy as np
import torch

from conftest import golden


def test_cal_depth_error_matches_reference_fixture():
    from vfdepth_amd.metrics import cal_depth_error
    fx = golden('metrics.npz')
    errs = cal_depth_error(torch.tensor(fx['pred']), torch.tensor(fx['gt']))
    np.testing.assert_allclose([float(e) for e in errs], fx['errs'], rtol=1e-6, atol=1e-7)


def test_compute_depth_losses_median_scaling():
    """A prediction that is the GT times a constant has zero median-scaled error (logger.py:227-231)
    and the metric error of that constant."""
    from vfdepth_amd.metrics import compute_depth_losses
    g = torch.Generator().manual_seed(0)
    B, N, H, W = 1, 2, 8, 12
    gt = 1.0 + 50 * torch.rand(B, N, 1, H, W, generator=g)
    mask = torch.ones(B, N, 1, H, W)
    mask[..., :2, :] = 0
    outputs = {('cam', c): {('depth', 0): gt[:, c] * 0.5} for c in range(N)}
    metric, median, scales = compute_depth_losses({'depth': gt, 'mask': mask}, outputs, N, 0.0, 200.0,
                                                  return_scales=True)
    assert scales == [2.0, 2.0]
    assert abs(float(metric['abs_rel']) - 0.5) < 1e-6
    assert float(median['abs_rel']) < 1e-6 and float(median['a1']) == 1.0


def _metric_fixture(fx, prefix):
    names = ['abs_rel', 'sq_rel', 'rms', 'log_rms', 'a1', 'a2', 'a3']
    return ({k: float(fx[f'{prefix}_metric_{k}']) for k in names},
            {k: float(fx[f'{prefix}_median_{k}']) for k in names})


def test_compute_depth_losses_matches_reference_logger():
    """Logger.compute_depth_losses (logger.py:193-247) of the reference, run on the same inputs
    (tests/golden/depth_metrics.npz): resize of a 2x prediction, clamping, lidar holes, fractional
    mask, median scaling, two eval ranges; and the reference step's own depth maps vs the
    synthetic ground-plane GT (the Abs.Rel half of BASELINE.json's metric)."""
    import common as G
    from vfdepth_amd import synth
    from vfdepth_amd.metrics import METRIC_NAMES, compute_depth_losses
    fx = golden('depth_metrics.npz')
    assert METRIC_NAMES == ['abs_rel', 'sq_rel', 'rms', 'log_rms', 'a1', 'a2', 'a3']
    for case, (lo, hi) in (('unit', (0.0, 200.0)), ('unit_nusc', (1.5, 80.0))):
        cfg, inputs, outputs = G.depth_metric_case()
        np.testing.assert_allclose(G.checksum(inputs['depth']), fx['cs_unit_gt'], rtol=1e-12)
        metric, median = compute_depth_losses(inputs, outputs, 6, lo, hi)
        ref_metric, ref_median = _metric_fixture(fx, case)
        for k in METRIC_NAMES:
            np.testing.assert_allclose(float(metric[k]), ref_metric[k], rtol=1e-6, atol=1e-7, err_msg=f'{case} {k}')
            np.testing.assert_allclose(float(median[k]), ref_median[k], rtol=1e-6, atol=1e-7, err_msg=f'{case} {k}')
    cfg = G.step_cfg()
    inputs = synth.make_batch(cfg, seed=5, with_depth=True)
    outputs = {('cam', c): {('depth', 0): torch.tensor(fx[f'step_depth_c{c}'])} for c in range(6)}
    metric, median = compute_depth_losses(inputs, outputs, 6, 0.0, 200.0)
    ref_metric, ref_median = _metric_fixture(fx, 'step')
    for k in METRIC_NAMES:
        np.testing.assert_allclose(float(metric[k]), ref_metric[k], rtol=1e-6, atol=1e-7, err_msg=f'step {k}')
        np.testing.assert_allclose(float(median[k]), ref_median[k], rtol=1e-6, atol=1e-7, err_msg=f'step {k}')


def test_inverse4x4_matches_lu_inverse():
    from vfdepth_amd import synth
    from vfdepth_amd.geometry import inverse4x4
    E = torch.from_numpy(synth.rig_extrinsics(6)).float()[None].repeat(2, 1, 1, 1)
    np.testing.assert_allclose(inverse4x4(E).numpy(), torch.inverse(E).numpy(), atol=1e-6)
    A = torch.randn(64, 4, 4, dtype=torch.float64) + 3 * torch.eye(4, dtype=torch.float64)
    np.testing.assert_allclose((inverse4x4(A) @ A).numpy(), np.broadcast_to(np.eye(4), (64, 4, 4)), atol=1e-10)


def test_net_precision_flag():
    """`net_precision` (config 3's bf16 nets) is validated at construction; fp32 is the default."""
    import pytest
    from vfdepth_amd import config as C
    from vfdepth_amd.network import FusedDepthNet, FusedPoseNet
    assert C.surround_fusion_cfg()['training']['net_precision'] == 'fp32'
    cfg = C.surround_fusion_cfg(net_precision='bf16')
    assert FusedDepthNet(cfg).bf16 and FusedPoseNet(cfg).bf16
    from vfdepth_amd.vfdepth import VFDepthAlgo
    with pytest.raises(ValueError):
        VFDepthAlgo(C.surround_fusion_cfg(net_precision='fp16'), 'cpu')


def test_channels_last_encoder_switch():
    """The bf16 nets always, and the fp32 nets when MIOpen picks algorithms by measured time
    (torch.backends.cudnn.benchmark), build channels-last encoders (NHWC conv weights: MIOpen then
    runs their convs without layout transposes, the fused BN / max pool take their NHWC kernels;
    VFD_CHANNELS_LAST='auto'); `training.channels_last` overrides either way.  Same values either
    way: the state dict round-trips between the layouts."""
    from vfdepth_amd import config as C
    from vfdepth_amd.network import FusedDepthNet, FusedPoseNet
    cl = torch.channels_last

    def is_cl(net):
        w = net.encoder.encoder.layer1[0].conv1.weight
        return w.is_contiguous(memory_format=cl) and not w.is_contiguous()
    fp32, bf16 = C.surround_fusion_cfg(), C.surround_fusion_cfg(net_precision='bf16')
    bench = torch.backends.cudnn.benchmark
    try:
        torch.backends.cudnn.benchmark = False      # immediate mode: fp32 encoders stay NCHW
        assert not is_cl(FusedDepthNet(fp32)) and not is_cl(FusedPoseNet(fp32))
        torch.backends.cudnn.benchmark = True       # measured algorithm choice: channels-last
        assert is_cl(FusedDepthNet(fp32)) and is_cl(FusedPoseNet(fp32))
    finally:
        torch.backends.cudnn.benchmark = bench
    assert is_cl(FusedDepthNet(bf16)) and is_cl(FusedPoseNet(bf16))
    bf16['training']['channels_last'] = False
    assert not is_cl(FusedPoseNet(bf16))
    fp32['training']['channels_last'] = True
    a = FusedPoseNet(fp32)
    assert is_cl(a)
    nchw = C.surround_fusion_cfg()
    nchw['training']['channels_last'] = False
    b = FusedPoseNet(nchw)
    assert not is_cl(b)
    b.load_state_dict(a.state_dict())
    for (k, va), vb in zip(a.state_dict().items(), b.state_dict().values()):
        assert torch.equal(va, vb), k


def test_batched_pose_and_warp_matrices_match_per_camera():
    """The batched pose distribution + warp-matrix chain (one gather + batched products) equals the
    per-camera reference formulation (pose.py:66-96, view_rendering.py:118-198) bit for bit."""
    import copy
    import common as G
    from vfdepth_amd.geometry import Pose, ViewRendering, inverse4x4
    from vfdepth_amd.rotation import axis_angle_to_matrix
    cfg = G.step_cfg()
    N = cfg['data']['num_cams']
    B = 2
    gen = torch.Generator().manual_seed(5)
    R = axis_angle_to_matrix(0.3 * torch.randn(B, N, 3, generator=gen))
    E = torch.eye(4).repeat(B, N, 1, 1)
    E[:, :, :3, :3] = R
    E[:, :, :3, 3] = torch.randn(B, N, 3, generator=gen)
    K = torch.eye(4).repeat(B, N, 1, 1)
    K[:, :, 0, 0], K[:, :, 1, 1] = 200.0, 210.0
    K[:, :, 0, 2], K[:, :, 1, 2] = 80.0, 48.0
    inputs = {('K', 0): K, 'extrinsics': E, 'extrinsics_inv': inverse4x4(E)}
    pose = Pose(cfg)
    T = {}
    for f in cfg['training']['frame_ids'][1:]:
        Tf = torch.eye(4).repeat(B, 1, 1)
        Tf[:, :3, :3] = axis_angle_to_matrix(0.05 * torch.randn(B, 3, generator=gen))
        Tf[:, :3, 3] = 0.5 * torch.randn(B, 3, generator=gen)
        T[('cam_T_cam', 0, f)] = Tf
    out = pose.distribute_pose(T, E, inputs['extrinsics_inv'])
    for f in cfg['training']['frame_ids'][1:]:
        for c in range(N):
            ref = inputs['extrinsics_inv'][:, c] @ E[:, 0] @ T['cam_T_cam', 0, f] @ inputs['extrinsics_inv'][:, 0] @ E[:, c]
            assert torch.equal(out[('cam', c)][('cam_T_cam', 0, f)], ref)
    outputs = copy.copy(out)
    vr = ViewRendering(cfg, 0)
    rel = {c: pose.compute_relative_cam_poses(inputs, outputs, c) for c in range(N)}
    per_cam = vr.warp_matrices(inputs, outputs, rel, list(range(N)))
    batched = vr.warp_matrices(inputs, outputs, None, list(range(N)))
    assert batched.shape == per_cam.shape
    assert torch.equal(batched, per_cam)


def test_fold_weights_backward_matches_autograd_slices():
    """kernels.FoldWeights (K1's folded 1x1 columns, one direct backward) against autograd through
    VFNet.folded_weights' slice / cat / stack form, on the CPU in float64."""
    from vfdepth_amd import kernels as KN
    torch.manual_seed(0)
    Cv, C = 5, 7
    groups = KN.overlap_group_table(6)
    w_no = torch.randn(Cv, C + 1, 1, dtype=torch.float64, requires_grad=True)
    w_o = torch.randn(Cv, 2 * C + 2, 1, dtype=torch.float64, requires_grad=True)
    gf = torch.randn(6, 2 * Cv, C, dtype=torch.float64)
    gz = torch.randn(3, Cv, dtype=torch.float64)
    wf, wz = KN.FoldWeights.apply(w_no, w_o, groups)
    ((wf * gf).sum() + (wz * gz).sum()).backward()
    a_no, a_o = w_no.grad.clone(), w_o.grad.clone()
    w_no.grad = w_o.grad = None
    wn, wo = w_no[:, :, 0], w_o[:, :, 0]
    halves = [wo[:, :C], wo[:, C + 1:2 * C + 1]]
    rf = torch.stack([torch.cat([wn[:, :C], halves[g]], 0) for g in groups], 0)
    rz = torch.stack([wn[:, C], wo[:, C], wo[:, 2 * C + 1]], 0)
    assert torch.equal(wf, rf) and torch.equal(wz, rz)
    ((rf * gf).sum() + (rz * gz).sum()).backward()
    torch.testing.assert_close(a_no, w_no.grad, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(a_o, w_o.grad, rtol=1e-12, atol=1e-12)


def test_miopen_private_db_copy(tmp_path, monkeypatch):
    """vfdepth_amd.miopen_db.use_private_copy: a process works on its own copy of the committed
    find-db (its writes cannot reach miopen_db/); an exported MIOPEN_USER_DB_PATH is kept."""
    from vfdepth_amd import miopen_db
    src = tmp_path / 'db'
    src.mkdir()
    (src / 'gfx950.ufdb.txt').write_text('record')
    monkeypatch.delenv('MIOPEN_USER_DB_PATH', raising=False)
    dst = miopen_db.use_private_copy(str(src))
    assert dst != str(src) and os.environ['MIOPEN_USER_DB_PATH'] == dst
    assert open(os.path.join(dst, 'gfx950.ufdb.txt')).read() == 'record'
    with open(os.path.join(dst, 'gfx950.ufdb.txt'), 'a') as fh:      # MIOpen appending a record
        fh.write('+new')
    assert (src / 'gfx950.ufdb.txt').read_text() == 'record'
    monkeypatch.setenv('MIOPEN_USER_DB_PATH', '/some/where')
    assert miopen_db.use_private_copy(str(src)) == '/some/where'

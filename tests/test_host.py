"""Host-side (non-kernel) pieces of the product on CPU: depth metrics, 4x4 inverse, config."""
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

"""Data path on the GPU: batches read from an on-disk DDAD-layout dataset, moved by
the pinned-memory `DevicePrefetcher` (side-stream H2D), drive the fusion step; the step's losses
and depth are BIT-IDENTICAL to those of the same batch handed to `process_batch` as host tensors
(its own `.to(device)` path): the prefetcher's on-device float64 -> fp32 cast rounds exactly like
the host cast, and the forward has no order-dependent sums.  (Round 2 saw a 1e-6 relative
`reproj_loss` difference here: the first step of the process ran before MIOpen had settled its
solver choice for each conv problem, so the two compared steps ran different conv algorithms; the
untimed warm-up step below fixes the picks.)"""
import pytest
import torch

import common as G
import data_fake

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')


def test_reader_prefetcher_drives_step(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    from vfdepth_amd import _lib
    from vfdepth_amd import data as D
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.vfdepth import VFDepthAlgo
    _lib.load()
    cfg = G.step_cfg()                               # 96x160, reduced voxels
    path, _, _ = data_fake.write_ddad(str(tmp_path), h=192, w=320, n_samples=5)
    cfg['data']['data_path'] = path
    cfg['data']['mask_path'] = D.ALL_ONES_MASK
    algo = VFDepthAlgo(cfg, 0)
    for m in algo.models.values():
        m.load_state_dict(seeded_state_dict(m, seed=G.STEP_SEED))
    algo.set_train()
    loader = torch.utils.data.DataLoader(D.construct_dataset(cfg, 'val', **D.augmentation(cfg, 'val')),
                                         batch_size=1, shuffle=False, pin_memory=True)
    host = [dict(b) for b in loader]
    assert len(host) == 3
    noise = torch.zeros(6, 1, 2, 96, 160, device=DEV)
    with torch.no_grad():                            # MIOpen picks its solvers on first use
        algo.process_batch(dict(host[0]), 0, noise=noise)
    for i, dev_batch in enumerate(D.DevicePrefetcher(loader, DEV)):
        assert dev_batch[('color', 0, 0)].is_cuda and dev_batch[('K', 0)].dtype == torch.float32
        for k, v in host[i].items():        # the resident inputs equal the host path's casts
            if torch.is_tensor(v) and v.is_floating_point():
                assert torch.equal(dev_batch[k].cpu(), v.float()), k
        with torch.no_grad():
            # alternate which path runs first: any state carried between steps would show up
            if i % 2:
                out_h, loss_h = algo.process_batch(dict(host[i]), 0, noise=noise)
                out_d, loss_d = algo.process_batch(dev_batch, 0, noise=noise)
            else:
                out_d, loss_d = algo.process_batch(dev_batch, 0, noise=noise)
                out_h, loss_h = algo.process_batch(dict(host[i]), 0, noise=noise)
        diff = [k for k in loss_h if not torch.equal(loss_d[k], loss_h[k])]
        assert not diff, {k: (float(loss_d[k]), float(loss_h[k])) for k in diff}
        for c in range(6):
            assert torch.equal(out_d[('cam', c)][('depth', 0)], out_h[('cam', c)][('depth', 0)]), f'depth cam {c}'
        assert torch.isfinite(loss_d['total_loss'])

"""Data path on the GPU: batches read from an on-disk DDAD-layout dataset, moved by
the pinned-memory `DevicePrefetcher` (side-stream H2D), drive the fusion step; the step's losses
and depth equal those of the same batch handed to `process_batch` as host tensors (its own
`.to(device)` path)."""
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
        with torch.no_grad():
            out_d, loss_d = algo.process_batch(dev_batch, 0, noise=noise)
            out_h, loss_h = algo.process_batch(dict(host[i]), 0, noise=noise)
        for k in loss_h:
            torch.testing.assert_close(loss_d[k], loss_h[k], rtol=1e-4, atol=1e-6, msg=k)
        torch.testing.assert_close(out_d[('cam', 0)][('depth', 0)], out_h[('cam', 0)][('depth', 0)], rtol=1e-4, atol=1e-4)
        assert torch.isfinite(loss_d['total_loss'])

"""Data path: align_dataset / transform_mask_sample against the reference's own
functions (fixture `golden/data_align.npz`), the DDAD (dgp JSON) and NuScenes (devkit tables)
readers on tiny on-disk datasets with a known rig, collation, the trainer integration and the
device prefetcher.  CPU only."""
import os

import numpy as np
import PIL.Image as pil
import pytest
import torch

from vfdepth_amd import config as C
from vfdepth_amd import data as D
from vfdepth_amd import synth

import data_fake

HERE = os.path.dirname(os.path.abspath(__file__))


def _fixture():
    return np.load(os.path.join(HERE, 'golden', 'data_align.npz'))


def test_align_dataset_matches_reference():
    z = _fixture()
    sample = {'rgb': torch.from_numpy(z['in_rgb']), 'rgb_original': torch.from_numpy(z['in_rgb_original']),
              'rgb_context': [torch.from_numpy(a) for a in z['in_rgb_context']],
              'rgb_context_original': [torch.from_numpy(a) for a in z['in_rgb_context_original']],
              'intrinsics': z['in_intrinsics'], 'extrinsics': z['out_extrinsics'], 'contexts': [-1, 1],
              'splitname': 'x'}
    out = D.align_dataset(sample, np.arange(4), [-1, 1])
    names = {k for k in z.files if k.startswith('out_') and k != 'out_mask'}
    got = {'out_' + ('_'.join(str(x) for x in k) if isinstance(k, tuple) else k): v for k, v in out.items()}
    assert set(got) == names
    for k in names:
        g = got[k].numpy() if torch.is_tensor(got[k]) else got[k]
        np.testing.assert_array_equal(g, z[k], err_msg=k)


def test_transform_mask_sample_matches_reference():
    z = _fixture()
    tf = D.get_transforms('train', image_shape=(40, 64), jittering=(0.0, 0.0, 0.0, 0.0))
    m = D.transform_mask_sample({'mask': pil.fromarray(z['in_mask'], 'L')}, tf)['mask']
    np.testing.assert_array_equal(m.numpy(), z['out_mask'])


def _cfg(path, dataset='ddad', h=40, w=64, **data):
    cfg = C.surround_fusion_cfg(height=h, width=w)
    cfg['data'].update({'data_path': path, 'dataset': dataset, 'mask_path': D.ALL_ONES_MASK, **data})
    return cfg


def _check_schema(s, N, h, w, scales=4):
    for sc in range(scales):
        assert s[('K', sc)].shape == (N, 4, 4) and s[('inv_K', sc)].shape == (N, 4, 4)
        assert s[('color', 0, sc)].shape == (N, 3, h >> sc, w >> sc)
        assert s[('color_aug', 0, sc)].shape == (N, 3, h >> sc, w >> sc)
        np.testing.assert_allclose(s[('inv_K', sc)], np.linalg.pinv(s[('K', sc)]), atol=1e-12)
    for f in (-1, 1):
        assert s[('color', f, 0)].shape == (N, 3, h, w)
    assert s['mask'].shape == (N, 1, h, w)
    for k in ('rgb', 'rgb_context', 'intrinsics', 'contexts', 'splitname'):
        assert k not in s


def _resized(arr, h, w):
    return D.to_tensor(pil.fromarray(arr).resize((w, h), pil.LANCZOS))


@pytest.mark.parametrize('mode', ['train', 'val'])
def test_ddad_reader(tmp_path, mode):
    path, K, E = data_fake.write_ddad(str(tmp_path), h=80, w=128, n_samples=4)
    cfg = _cfg(path)
    ds = D.construct_dataset(cfg, mode, **D.augmentation(cfg, mode))
    assert len(ds) == 2                                    # samples 1, 2 have both contexts
    s = ds[0]
    _check_schema(s, 6, 40, 64)
    K0 = K.copy()
    K0[:, :2] *= 0.5                                       # 128x80 source -> 64x40
    np.testing.assert_allclose(s[('K', 0)], K0, rtol=1e-6)
    np.testing.assert_allclose(s[('K', 2)][:, :2], K0[:, :2] / 4, rtol=1e-6)
    np.testing.assert_allclose(s['extrinsics'], E, atol=1e-6)
    for c in range(6):                                     # original frames: exact LANCZOS + ToTensor
        for f, t in ((0, 1), (-1, 0), (1, 2)):
            ref = _resized(data_fake.frame_image(c, t, 80, 128), 40, 64)
            torch.testing.assert_close(s[('color', f, 0)][c], ref, rtol=0, atol=0)
    if mode == 'train':                                    # jittered copies differ, shapes equal
        assert not torch.equal(s[('color_aug', 0, 0)], s[('color', 0, 0)])
    else:
        torch.testing.assert_close(s[('color_aug', 0, 0)], s[('color', 0, 0)], rtol=0, atol=0)
        assert s['depth'].shape == (6, 1, 40, 64)
        cfg1 = _cfg(path, h=80, w=128)                     # depth at the source resolution
        d = D.construct_dataset(cfg1, mode, **D.augmentation(cfg1, mode))[0]['depth']
        gp = synth.ground_plane_depth(K, E, 80, 128).numpy()
        hit = d.numpy() > 0
        assert hit.sum() > 100
        rel = np.abs(d.numpy()[hit] - gp[hit]) / gp[hit]
        assert np.median(rel) < 0.05                       # lidar ground points land on the ground plane


def test_ddad_depth_cache_is_read(tmp_path):
    path, K, E = data_fake.write_ddad(str(tmp_path), h=80, w=128, n_samples=3)
    cached = np.full((80, 128), 7.0)
    cdir = os.path.join(str(tmp_path), '000000', 'depth', 'lidar', 'CAMERA_01')
    os.makedirs(cdir)
    np.savez_compressed(os.path.join(cdir, '1.npz'), depth=cached)
    cfg = _cfg(path)
    ds = D.construct_dataset(cfg, 'val', **D.augmentation(cfg, 'val'))
    d = ds[0]['depth'][0, 0]
    assert torch.all(d == 7.0)


@pytest.mark.parametrize('mode', ['train', 'val'])
def test_nuscenes_reader(tmp_path, mode):
    root, K, E = data_fake.write_nuscenes(str(tmp_path), h=80, w=128, n_samples=4)
    cfg = _cfg(root, 'nuscenes', nusc_version='v1.0-mini', cameras=[c.lower() for c in data_fake.NUSC_CAMERAS])
    ds = D.construct_dataset(cfg, mode, **D.augmentation(cfg, mode))
    assert len(ds) == (2 if mode == 'train' else 4)
    s = ds[0]
    _check_schema(s, 6, 40, 64)
    K0 = K.copy()
    K0[:, :2] *= 0.5
    np.testing.assert_allclose(s[('K', 0)][:, :3, :3], K0[:, :3, :3], rtol=1e-6)
    np.testing.assert_allclose(s['extrinsics'], E, atol=1e-6)
    t = 1 if mode == 'train' else 0
    for c in range(6):
        for f, tt in ((0, t), (-1, t - 1 if mode == 'train' else t), (1, t + 1 if mode == 'train' else t)):
            ref = _resized(data_fake.frame_image(c, tt, 80, 128), 40, 64)
            torch.testing.assert_close(s[('color', f, 0)][c], ref, rtol=0, atol=0)
    if mode == 'val':
        cfg1 = _cfg(root, 'nuscenes', h=80, w=128, nusc_version='v1.0-mini',
                    cameras=[c.lower() for c in data_fake.NUSC_CAMERAS])
        d = D.construct_dataset(cfg1, mode, **D.augmentation(cfg1, mode))[0]['depth'].numpy()
        gp = synth.ground_plane_depth(K, E, 80, 128).numpy()
        hit = d > 0
        assert hit.sum() > 100
        assert np.median(np.abs(d[hit] - gp[hit]) / gp[hit]) < 0.05


def test_quaternion_round_trip():
    rng = np.random.default_rng(0)
    for _ in range(20):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        R = D.quat_to_matrix(*q)
        np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-12)
        assert np.linalg.det(R) == pytest.approx(1.0)
        q2 = data_fake._quat_of(R)
        np.testing.assert_allclose(D.quat_to_matrix(*q2), R, atol=1e-12)


def test_trainer_uses_reader_and_prefetcher(tmp_path):
    """VFDepthAlgo builds its loaders over the on-disk reader when data_path names a dataset; the
    collated batch has the synthetic generator's schema (so process_batch is unchanged); the
    prefetcher passes batches through on a CPU device."""
    from vfdepth_amd.vfdepth import VFDepthAlgo
    path, _, _ = data_fake.write_ddad(str(tmp_path), h=80, w=128, n_samples=4)
    cfg = _cfg(path)
    algo = VFDepthAlgo(cfg, 'cpu')
    batch = next(iter(algo.train_dataloader()))
    ref = synth.make_batch(cfg, seed=0)
    for k, v in ref.items():
        if torch.is_tensor(v) and k != 'idx':
            assert k in batch and tuple(batch[k].shape) == tuple(v.shape), k
    pf = D.DevicePrefetcher(algo.train_dataloader(), 'cpu')
    got = list(pf)
    assert len(got) == len(algo.train_dataloader()) == 2
    assert got[0][('K', 0)].dtype == torch.float32


def test_threaded_loader(tmp_path):
    path, _, _ = data_fake.write_ddad(str(tmp_path), h=80, w=128, n_samples=4)
    cfg = _cfg(path)
    ds = D.construct_dataset(cfg, 'val', **D.augmentation(cfg, 'val'))
    batches = list(D.ThreadedLoader(ds, batch_size=2))
    assert len(batches) == 1 and batches[0][('color', 0, 0)].shape == (2, 6, 3, 40, 64)
    torch.testing.assert_close(batches[0][('color', 0, 0)][1], ds[1][('color', 0, 0)])


def _write_masks(root, cams, sets):
    """<root>/<set>/<CAM>_mask.png, set k filled with value 10 * (k + 1) (distinguishable)."""
    for k in sets:
        os.makedirs(os.path.join(root, str(k)), exist_ok=True)
        for cam in cams:
            pil.new('L', (128, 80), 10 * (k + 1)).save(os.path.join(root, str(k), cam.upper() + '_mask.png'))


def test_ddad_mask_set_lookup(tmp_path):
    """The scene directory '000000' is looked up as int('000000') -> '0' in the JSON dump of the
    reference's mask_idx_dict (ddad_dataset_sf.py:102); a mapping without the scene is an error;
    no mask_path at all is an error unless 'all_ones' asks for the all-255 mask."""
    import json
    from vfdepth_amd.config import DDAD_CAMERAS
    path, _, _ = data_fake.write_ddad(str(tmp_path / 'ddad'), h=80, w=128, n_samples=4)
    masks = str(tmp_path / 'masks')
    _write_masks(masks, DDAD_CAMERAS, (0, 2))
    mj = str(tmp_path / 'mask_idx.json')
    with open(mj, 'w') as f:
        json.dump({'0': 2, '150': 0}, f)
    cfg = _cfg(path, mask_path=masks, mask_idx_json=mj, h=80, w=128)
    s = D.construct_dataset(cfg, 'val', **D.augmentation(cfg, 'val'))[0]
    np.testing.assert_allclose(s['mask'].numpy(), 30 / 255.0, rtol=1e-6)        # set 2, not set 0
    with open(mj, 'w') as f:
        json.dump({'150': 0}, f)
    with pytest.raises(KeyError):
        D.construct_dataset(cfg, 'val', **D.augmentation(cfg, 'val'))[0]
    cfg = _cfg(path)
    del cfg['data']['mask_path']
    with pytest.raises(ValueError, match='mask_path'):
        D.construct_dataset(cfg, 'val', **D.augmentation(cfg, 'val'))


def test_nuscenes_depth_cache_is_read(tmp_path):
    """nuscenes_dataset.py:108-116: the cached map <dirname(path)>/samples/DEPTH_MAP/<CAM>/<file>.npz
    is read (arrays only) instead of re-projecting the lidar sweep."""
    root, _, _ = data_fake.write_nuscenes(str(tmp_path / 'nusc'), h=80, w=128, n_samples=4)
    cam = data_fake.NUSC_CAMERAS[0]
    cdir = os.path.join(str(tmp_path), 'samples', 'DEPTH_MAP', cam, 'samples', cam)
    os.makedirs(cdir)
    np.savez_compressed(os.path.join(cdir, '0.png.npz'), depth=np.full((80, 128), 9.0))
    cfg = _cfg(root, 'nuscenes', h=80, w=128, nusc_version='v1.0-mini',
               cameras=[c.lower() for c in data_fake.NUSC_CAMERAS])
    s = D.construct_dataset(cfg, 'val', **D.augmentation(cfg, 'val'))[0]
    assert torch.all(s['depth'][0] == 9.0)
    assert not torch.all(s['depth'][1] == 9.0)                # other cameras: projected lidar


def test_threaded_loader_propagates_errors():
    class Bad(torch.utils.data.Dataset):
        def __len__(self):
            return 4

        def __getitem__(self, i):
            if i == 2:
                raise RuntimeError('corrupt sample 2')
            return {'x': torch.full((2,), float(i))}
    it = iter(D.ThreadedLoader(Bad(), batch_size=1, pin=False))
    assert float(next(it)['x'][0, 0]) == 0.0
    assert float(next(it)['x'][0, 0]) == 1.0
    with pytest.raises(RuntimeError, match='corrupt sample 2'):
        next(it)

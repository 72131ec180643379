"""Deterministic synthetic surround-view batches in the reference's input schema.

The reference's loaders (`/root/reference/dataset/ddad_dataset_sf.py:85-155` →
`align_dataset` `/root/reference/dataset/data_util.py:46-91`) need DDAD/NuScenes on disk; this
generator reproduces the *schema* of what they emit after collation:

* `('color', f, s)`, `('color_aug', f, s)`  [B, N, 3, H/2^s, W/2^s]  (f=0 for every scale,
  context frames f=±1 at scale 0 only; scales 0..fusion_level+1)
* `('K', s)`, `('inv_K', s)`  [B, N, 4, 4]   (K rows 0-1 divided by 2^s, inv_K = pinv(K))
* `'mask'` [B, N, 1, H, W], `'extrinsics'` [B, N, 4, 4] (camera→vehicle), optional `'depth'`

Rig: yaw 0/+60/-60/+120/-120/180 deg in DDAD axes (x fwd, y left, z up),
camera axes right/down/forward, position (1.5cosψ, 0.5sinψ, 1.5) m; front/rear focal 1.12·W,
side cameras 0.56·W, principal point at the image centre.  Images are low-passed uniform noise,
masks invalidate the bottom 15 % rows, ground-truth depth is the analytic ground-plane depth.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

YAWS_DEG = [0.0, 60.0, -60.0, 120.0, -120.0, 180.0]


def rig_extrinsics(n_cams):
    """Camera→vehicle 4×4 transforms for rig positions 0..n_cams-1 (float64)."""
    axes = np.array([[0.0, 0.0, 1.0],     # camera x (right)  -> vehicle -y ; columns below
                     [-1.0, 0.0, 0.0],
                     [0.0, -1.0, 0.0]])
    out = []
    for c in range(n_cams):
        psi = math.radians(YAWS_DEG[c])
        rz = np.array([[math.cos(psi), -math.sin(psi), 0.0],
                       [math.sin(psi), math.cos(psi), 0.0],
                       [0.0, 0.0, 1.0]])
        T = np.eye(4)
        T[:3, :3] = rz @ axes
        T[:3, 3] = [1.5 * math.cos(psi), 0.5 * math.sin(psi), 1.5]
        out.append(T)
    return np.stack(out)


def rig_intrinsics(n_cams, height, width):
    out = []
    for c in range(n_cams):
        f = (1.12 if c in (0, 5) else 0.56) * width
        K = np.eye(4)
        K[0, 0] = K[1, 1] = f
        K[0, 2] = width / 2.0
        K[1, 2] = height / 2.0
        out.append(K)
    return np.stack(out)


def _lowpass_noise(gen, shape):
    x = torch.rand(shape, generator=gen, dtype=torch.float32)
    lead = x.shape[:-3]
    x = x.reshape(-1, *x.shape[-3:])
    for _ in range(2):
        x = F.avg_pool2d(F.pad(x, (1, 1, 1, 1), mode='replicate'), 3, 1)
    return x.reshape(*lead, *x.shape[-3:])


def ground_plane_depth(K, E, height, width, min_d=1.5, max_d=200.0):
    """Camera-z depth of the vehicle ground plane z=0 for every pixel ([N,1,H,W], float32)."""
    n = K.shape[0]
    ys, xs = np.meshgrid(np.arange(height), np.arange(width), indexing='ij')
    pix = np.stack([xs, ys, np.ones_like(xs)], 0).reshape(3, -1).astype(np.float64)
    out = []
    for c in range(n):
        ray = np.linalg.inv(K[c, :3, :3]) @ pix               # camera frame, z = 1
        d_w = E[c, :3, :3] @ ray                               # vehicle frame direction
        h = E[c, 2, 3]
        with np.errstate(divide='ignore', invalid='ignore'):
            t = np.where(d_w[2] < -1e-9, -h / d_w[2], max_d)
        out.append(np.clip(t, min_d, max_d).reshape(1, height, width))
    return torch.from_numpy(np.stack(out)).float()


def make_batch(cfg, seed=0, batch_size=None, with_depth=False, device='cpu'):
    """One collated training batch for `cfg` (the dict returned by `config.get_config`)."""
    tr, md, dt = cfg['training'], cfg['model'], cfg['data']
    B = int(batch_size or tr['batch_size'])
    N = int(dt['num_cams'])
    H, W = int(tr['height']), int(tr['width'])
    fusion_level = int(md.get('fusion_level', 2))
    scales = range(fusion_level + 2)
    gen = torch.Generator().manual_seed(int(seed))
    frames = tr['frame_ids']

    E = rig_extrinsics(6)[:N]
    K0 = rig_intrinsics(6, H, W)[:N]
    inputs = {}
    base = {f: _lowpass_noise(gen, (B, N, 3, H, W)) for f in frames}
    for s in scales:
        Ks = K0.copy()
        Ks[:, :2, :] /= 2 ** s
        inputs[('K', s)] = torch.from_numpy(np.broadcast_to(Ks, (B, N, 4, 4)).copy()).float()
        inputs[('inv_K', s)] = torch.from_numpy(np.broadcast_to(np.linalg.pinv(Ks), (B, N, 4, 4)).copy()).float()
        if s == 0:
            img = base[0]
        else:
            img = F.interpolate(base[0].reshape(B * N, 3, H, W), size=(H // 2 ** s, W // 2 ** s),
                                mode='bilinear', align_corners=False).reshape(B, N, 3, H // 2 ** s, W // 2 ** s)
        inputs[('color', 0, s)] = img
        inputs[('color_aug', 0, s)] = img.clone()
    for f in frames[1:]:
        inputs[('color', f, 0)] = base[f]
        inputs[('color_aug', f, 0)] = base[f].clone()
    mask = torch.ones(B, N, 1, H, W)
    mask[..., int(round(H * 0.85)):, :] = 0.0
    inputs['mask'] = mask
    inputs['extrinsics'] = torch.from_numpy(np.broadcast_to(E, (B, N, 4, 4)).copy()).float()
    if with_depth:
        gt = ground_plane_depth(K0, E, H, W, tr['min_depth'], tr['max_depth'])
        inputs['depth'] = gt.unsqueeze(0).expand(B, -1, -1, -1, -1).contiguous()
    inputs['idx'] = torch.arange(B)
    if device != 'cpu':
        inputs = {k: (v.to(device) if torch.is_tensor(v) else v) for k, v in inputs.items()}
    return inputs


class SyntheticSurroundDataset(torch.utils.data.Dataset):
    """Map-style dataset of per-sample dicts (collates to `make_batch`'s schema)."""

    def __init__(self, cfg, length=64, seed=0, with_depth=False):
        self.cfg, self.length, self.seed, self.with_depth = cfg, length, seed, with_depth

    def __len__(self):
        return self.length

    def __getitem__(self, idx):
        b = make_batch(self.cfg, seed=self.seed * 100003 + idx, batch_size=1, with_depth=self.with_depth)
        return {k: (v[0] if torch.is_tensor(v) else v) for k, v in b.items()}

"""Input builders shared by the golden generator and the tests.

Large inputs and upstream gradients are NOT stored in the fixtures: they are regenerated
bit-identically from CPU `torch.Generator` seeds here (same torch build in the build container
and on the GPU box), and every fixture stores a checksum of them so that drift is detected.
"""
import math

import numpy as np
import torch

from vfdepth_amd import config as C
from vfdepth_amd import synth
from vfdepth_amd.rotation import axis_angle_to_matrix


def seeded_randn(shape, seed):
    return torch.randn(tuple(shape), generator=torch.Generator().manual_seed(int(seed)))


def checksum(t):
    t = t.detach().double()
    return np.array([t.sum().item(), (t * t).sum().item(), float(t.numel())])


def random_mask(gen, shape):
    """Binary self-occlusion mask (bottom 15 % invalid) with one fractional, antialiased row."""
    m = torch.ones(shape)
    H = shape[-2]
    cut = int(round(H * 0.85))
    m[..., cut:, :] = 0.0
    m[..., cut - 1, :] = torch.rand(tuple(shape[:-2]) + (shape[-1],), generator=gen)
    return m


# ------------------------------------------------------------------------------------ fusion
def fusion_cfg():
    return C.surround_fusion_cfg(height=96, width=160, batch_size=2, fusion_feat_in_dim=8,
                                 voxel_size=[16, 16, 6], voxel_unit_size=[6.0, 6.0, 5.0],
                                 voxel_str_p=[-45.0, -45.0, -12.5], voxel_pre_dim=[8],
                                 proj_d_bins=6)


def fusion_case():
    cfg = fusion_cfg()
    gen = torch.Generator().manual_seed(11)
    B, N, Cf = 2, 6, 8
    batch = synth.make_batch(cfg, seed=3)
    d = {'K': batch[('K', 3)], 'invK': batch[('inv_K', 3)], 'E': batch['extrinsics']}
    d['Einv'] = torch.inverse(d['E'])
    d['mask'] = random_mask(gen, (B, N, 1, 96, 160))
    d['feats'] = torch.randn(B, N, Cf, 12, 20, generator=gen)
    seeds = {'g_vox': 101, 'g_pose': 102, 'vleaf': 103, 'g_proj': 104}
    return cfg, d, seeds


# ------------------------------------------------------------------------------------ view synthesis
VIEW_B, VIEW_H, VIEW_W = 2, 24, 40


def view_case(skip_sample=False):
    B, H, W = VIEW_B, VIEW_H, VIEW_W
    seed = 22 if skip_sample else 21
    cfg = C.surround_fusion_cfg(height=H, width=W, batch_size=B)
    gen = torch.Generator().manual_seed(seed)
    batch = synth.make_batch(cfg, seed=seed)
    batch['extrinsics_inv'] = torch.inverse(batch['extrinsics'])
    K0 = synth.rig_intrinsics(6, H, W)
    gt = synth.ground_plane_depth(K0, synth.rig_extrinsics(6), H, W, 1.5, 60.0)
    depth = gt.unsqueeze(0).repeat(B, 1, 1, 1, 1) * (0.8 + 0.4 * torch.rand(B, 6, 1, H, W, generator=gen))
    batch['mask'] = random_mask(gen, (B, 6, 1, H, W))
    poses = {}
    for f in (-1, 1):
        aa = 0.02 * torch.randn(B, 1, 3, generator=gen)
        tr = 0.5 * torch.randn(B, 1, 3, generator=gen)
        if skip_sample:
            tr[1] = 500.0            # sample 1: temporal warps leave the image -> empty overlap
        T = torch.eye(4).repeat(B, 1, 1)
        T[:, :3, :3] = axis_angle_to_matrix(aa)[:, 0]
        T[:, :3, 3] = tr[:, 0]
        for c in range(6):
            # per-camera variation, as distribute_pose would produce
            Tc = T.clone()
            Tc[:, :3, 3] += 0.05 * c
            poses[(c, f)] = Tc
    if skip_sample:
        depth[1] = 0.02              # sample 1: spatial warps fall outside the neighbours
    return cfg, batch, depth, poses


def view_case_cfg(cfg, seed):
    """view_case at any configuration (full BASELINE sizes): batch with a fractional mask row,
    ground-plane depth x U(0.8, 1.2), small random per-camera motions."""
    t = cfg['training']
    B, N, H, W = t['batch_size'], cfg['data']['num_cams'], t['height'], t['width']
    gen = torch.Generator().manual_seed(seed)
    batch = synth.make_batch(cfg, seed=seed)
    batch['extrinsics_inv'] = torch.inverse(batch['extrinsics'])
    gt = synth.ground_plane_depth(synth.rig_intrinsics(N, H, W), synth.rig_extrinsics(N), H, W, 1.5, 60.0)
    depth = gt.unsqueeze(0).repeat(B, 1, 1, 1, 1) * (0.8 + 0.4 * torch.rand(B, N, 1, H, W, generator=gen))
    batch['mask'] = random_mask(gen, (B, N, 1, H, W))
    poses = {}
    for f in t['frame_ids'][1:]:
        aa = 0.02 * torch.randn(B, 1, 3, generator=gen)
        tr = 0.5 * torch.randn(B, 1, 3, generator=gen)
        T = torch.eye(4).repeat(B, 1, 1)
        T[:, :3, :3] = axis_angle_to_matrix(aa)[:, 0]
        T[:, :3, 3] = tr[:, 0]
        for c in range(N):
            Tc = T.clone()
            Tc[:, :3, 3] += 0.05 * c
            poses[(c, f)] = Tc
    return batch, depth, poses


VIEW_IMG_KEYS = [('color', -1, 0), ('color', 1, 0), ('overlap', 0, 0), ('overlap', -1, 0), ('overlap', 1, 0)]
VIEW_MSK_KEYS = [('color_mask', -1, 0), ('color_mask', 1, 0), ('overlap_mask', 0, 0),
                 ('overlap_mask', -1, 0), ('overlap_mask', 1, 0)]


def key_name(k):
    return '_'.join(str(x) for x in k)


# ------------------------------------------------------------------------------------ losses
def loss_case():
    """Synthetic warped planes around the target so every loss branch is exercised."""
    B, H, W = VIEW_B, VIEW_H, VIEW_W
    cfg = C.surround_fusion_cfg(height=H, width=W, batch_size=B)
    gen = torch.Generator().manual_seed(31)
    batch = synth.make_batch(cfg, seed=31)
    batch['mask'] = random_mask(gen, (B, 6, 1, H, W))
    planes = {}
    for c in range(6):
        tgt = batch[('color', 0, 0)][:, c]
        for k in VIEW_IMG_KEYS:
            noise = torch.rand(B, 3, H, W, generator=gen) - 0.5
            amp = 0.05 + 0.3 * torch.rand(B, 1, 1, 1, generator=gen)
            img = (tgt + amp * noise).clamp(0, 1)
            # a block of exact zeros (out-of-image warp) and of NaN-filled 2.0
            img[:, :, :3, :5] = 0.0
            img[:, :, -2:, -4:] = 2.0
            planes[(c,) + k] = img
        for f in (0, -1, 1):
            m = (torch.rand(B, 1, H, W, generator=gen) > 0.3).float()
            m = m + (torch.rand(B, 1, H, W, generator=gen) > 0.7).float()     # overlap masks reach 2
            planes[(c, 'overlap_mask', f, 0)] = m
        planes[(c, 'disp', 0)] = 0.2 + 0.6 * torch.rand(B, 1, H, W, generator=gen)
    return cfg, batch, planes


# ------------------------------------------------------------------------------------ depth metrics
def depth_metric_case():
    """(cfg, inputs, outputs) for Logger.compute_depth_losses: 6 cameras, B=2, GT 48x80 with
    lidar holes (0) and far returns, fractional mask, predictions at 96x160."""
    B, N, h, w = 2, 6, 48, 80
    cfg = C.surround_fusion_cfg(height=2 * h, width=2 * w, batch_size=B)
    gen = torch.Generator().manual_seed(41)
    K0 = synth.rig_intrinsics(N, h, w)
    gt = synth.ground_plane_depth(K0, synth.rig_extrinsics(N), h, w, 1.5, 250.0)
    gt = gt.unsqueeze(0).repeat(B, 1, 1, 1, 1)
    gt = gt * (torch.rand(B, N, 1, h, w, generator=gen) > 0.1).float()          # lidar holes
    mask = torch.ones(B, N, 1, h, w)
    mask[..., int(h * 0.85):, :] = 0.0
    mask[..., int(h * 0.85) - 1, :] = torch.rand(B, N, 1, w, generator=gen)      # antialiased row
    pred = torch.nn.functional.interpolate(gt.clamp(min=1.0).flatten(0, 1), [2 * h, 2 * w], mode='nearest')
    pred = pred.view(B, N, 1, 2 * h, 2 * w) * (0.6 + 0.8 * torch.rand(B, N, 1, 2 * h, 2 * w, generator=gen))
    inputs = {'depth': gt, 'mask': mask}
    outputs = {('cam', c): {('depth', 0): pred[:, c].contiguous()} for c in range(N)}
    return cfg, inputs, outputs


# ------------------------------------------------------------------------------------ full step
STEP_SEED = 7

# ------------------------------------------------------------------------------------ full resolution
# config 2 of BASELINE.json (6-cam DDAD 384x640, B=1, 100x100x20 voxels, D=50, fp32): the headline
# shape, pinned against the reference's own CPU step (tests/golden/step_full.npz)
FULL_SEED = 15            # synth.make_batch seed of the inputs
FULL_NOISE_SEED = 1234    # the reference step's torch.manual_seed before its identity-noise draws
FULL_SUB = 4              # depth maps stored at every FULL_SUB-th pixel (plus full-map checksums)


def full_cfg():
    return C.surround_fusion_cfg(batch_size=1)


def full_noise(fx, shape, n_cams=6):
    """The identity-loss noise of the full-resolution fixture, rebuilt bit-identically: the
    reference's raw torch.randn draws (one [B, T, H, W] block per camera, in camera order, from a
    CPU generator seeded FULL_NOISE_SEED, checked against the stored checksums) plus the sparse
    tie-breaking nudges of gen_golden._untie_noise, times the reference's 1e-5."""
    gen = torch.Generator().manual_seed(FULL_NOISE_SEED)
    out = []
    for c in range(n_cams):
        raw = torch.randn(tuple(shape), generator=gen)
        np.testing.assert_allclose(checksum(raw), fx[f'cs_noise_raw_c{c}'], rtol=1e-12)   # host SIMD: last bit
        flat = raw.flatten().clone()
        idx = torch.from_numpy(fx[f'noise_idx_c{c}'].astype(np.int64))
        flat[idx] += torch.from_numpy(fx[f'noise_add_c{c}'])
        out.append(flat.view(raw.shape) * 1e-5)
    return out


def step_cfg():
    return C.surround_fusion_cfg(height=96, width=160, batch_size=1, voxel_size=[40, 40, 10],
                                 voxel_unit_size=[2.5, 2.5, 3.0], voxel_str_p=[-50.0, -50.0, -15.0],
                                 proj_d_bins=16, focal_length_scale=30)


def step_aug_cfg():
    """The reduced step config with the depth-synthesis branch (ddad_surround_fusion_augdepth.yaml:
    aug_depth, aug_angle [15, 15, 40], depth_con_coeff 0.03, depth_sm_coeff 0.05)."""
    cfg = step_cfg()
    cfg['training']['aug_depth'] = True
    cfg['loss'].update({'depth_con_coeff': 0.03, 'depth_sm_coeff': 0.05})
    return cfg


def virtual_depth_case():
    """Inputs of ViewRendering.get_virtual_depth (view_rendering.py:84-116): B=2, 24x40, a source
    camera warped into a rotated novel view of a neighbouring camera; depth ranges that exercise
    the [min, max] clamps and the OOB / mask rules."""
    B, H, W = 2, 24, 40
    gen = torch.Generator().manual_seed(51)
    K = torch.from_numpy(synth.rig_intrinsics(6, H, W)).float()
    E = torch.from_numpy(synth.rig_extrinsics(6)).float()
    gt = synth.ground_plane_depth(K.double().numpy(), E.double().numpy(), H, W, 1.5, 60.0)
    src, tar = 0, 0                  # the `[cam]` source of view_rendering.py:210 (neighbours: step fixture)
    src_depth = gt[src].unsqueeze(0).repeat(B, 1, 1, 1) * (0.7 + 0.6 * torch.rand(B, 1, H, W, generator=gen))
    tar_depth = gt[tar].unsqueeze(0).repeat(B, 1, 1, 1) * (0.7 + 0.6 * torch.rand(B, 1, H, W, generator=gen))
    src_mask = random_mask(gen, (B, 1, H, W))
    aa = 0.3 * (torch.rand(B, 1, 3, generator=gen) - 0.5)
    Rm = torch.eye(4).repeat(B, 1, 1)
    Rm[:, :3, :3] = axis_angle_to_matrix(aa)[:, 0]
    E_aug = Rm @ E[tar]
    T = torch.inverse(E_aug) @ E[src]
    return {'src_depth': src_depth, 'src_mask': src_mask, 'src_invK': torch.inverse(K[src]).repeat(B, 1, 1),
            'tar_depth': tar_depth, 'tar_invK': torch.inverse(K[tar]).repeat(B, 1, 1),
            'src_K': K[src].repeat(B, 1, 1), 'T': T, 'min_depth': 1.5, 'max_depth': 40.0}


def mono_cfg():
    return C.mono_cfg(batch_size=1)


PARAM_GRADS = ['depth_net.decoder.decoder.0.0.weight', 'depth_net.fusion_net.conv_overlap.0.weight',
               'depth_net.fusion_net.conv_non_overlap.0.bias', 'depth_net.fusion_net.reduce_dim.0.bias',
               'depth_net.conv1x1.0.bias', 'pose_net.pose_decoder.net.3.weight',
               'pose_net.fusion_net.reduce_dim.0.bias', 'pose_net.conv1x1.0.bias',
               'depth_net.depth_decoder.decoder.10.conv.conv.weight', 'pose_net.pose_decoder.net.3.bias']


# ------------------------------------------------------------------------------------ data path
def data_align_case():
    """A stacked 6-camera sample as the reference's DDAD/NuScenes readers hand it to
    `align_dataset` (after the per-camera transforms and `stack_sample`): seeded images 40x64
    (augmented + original, contexts -1 / +1), intrinsics [6,3,3] float64 with a skew term and
    an off-centre principal point, extrinsics; plus a 97x151 'L' mask image for
    `transform_mask_sample`."""
    import numpy as np
    import PIL.Image as pil
    gen = torch.Generator().manual_seed(77)
    N, H, W = 6, 40, 64
    rgb = torch.rand(N, 3, H, W, generator=gen)
    org = torch.rand(N, 3, H, W, generator=gen)
    ctx = [torch.rand(N, 3, H, W, generator=gen) for _ in range(2)]
    ctx_o = [torch.rand(N, 3, H, W, generator=gen) for _ in range(2)]
    K = np.zeros((N, 3, 3))
    for c in range(N):
        K[c] = [[50.0 + 3 * c, 0.25 * c, 31.5 + c], [0.0, 48.0 + 2 * c, 19.25 - c], [0.0, 0.0, 1.0]]
    sample = {'rgb': rgb, 'rgb_original': org, 'rgb_context': ctx, 'rgb_context_original': ctx_o,
              'intrinsics': K, 'extrinsics': np.stack([np.eye(4)] * N), 'contexts': [-1, 1],
              'splitname': 'train_0000000000'}
    m = (torch.rand(97, 151, generator=gen) * 255).to(torch.uint8).numpy()
    return sample, pil.fromarray(m, 'L'), [-1, 1], np.arange(4)


def perturb_rig(batch, seed):
    """Per-batch-element geometry.  The synthetic rig is the same for every element, which would
    hide a kernel that reads element 0's K / E for all of them: element b gets its focal lengths
    scaled by 1 + 0.03 b (K, inv_K at every scale) and its whole rig turned by 2b degrees about
    the vertical axis and shifted by (0.1 b, -0.05 b, 0) m (extrinsics, extrinsics_inv)."""
    B = batch['extrinsics'].shape[0]
    gen = torch.Generator().manual_seed(seed)
    for b in range(B):
        a = math.radians(2.0 * b)
        R = torch.eye(4)
        R[0, 0], R[0, 1], R[1, 0], R[1, 1] = math.cos(a), -math.sin(a), math.sin(a), math.cos(a)
        R[:3, 3] = torch.tensor([0.1 * b, -0.05 * b, 0.0]) + 0.01 * torch.randn(3, generator=gen)
        batch['extrinsics'][b] = R @ batch['extrinsics'][b]
        for k in [k for k in batch if isinstance(k, tuple) and k[0] == 'K']:
            batch[k][b, :, 0, 0] *= 1 + 0.03 * b
            batch[k][b, :, 1, 1] *= 1 + 0.03 * b
    for k in [k for k in batch if isinstance(k, tuple) and k[0] == 'K']:
        batch[('inv_K', k[1])] = torch.inverse(batch[k].double()).float()
    batch['extrinsics_inv'] = torch.inverse(batch['extrinsics'])
    return batch

"""VFDepth hot-path ORACLE — test infrastructure only.

CPU restatement (PyTorch CPU tensors, fp32 or fp64, autograd-capable) of the reference's hot
path, written from the reference's semantics with explicit index arithmetic — no
`F.grid_sample` / `avg_pool2d` / `interpolate` — so that it pins those ATen semantics
independently.  It is pinned itself by golden vectors produced by the real reference
(`tests/golden/gen_golden.py`, fixtures `tests/golden/*.npz`).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
module, and only as the checker / CPU baseline.  The product (`vfdepth_amd`) never does.

Reference citations are `/root/reference/<file>:<line>`.
"""
import math

import torch

LRELU = 0.1


# =============================================================================================
# ATen sampling semantics (restated)
# =============================================================================================
def _unnorm(g, size):
    """align_corners=True unnormalisation ((g + 1) / 2) * (size - 1) (ATen GridSampler.h:27-31)."""
    return ((g + 1) / 2) * (size - 1)


def sample2d(img, gx, gy, mode='bilinear'):
    """`F.grid_sample(img, grid, mode, padding_mode='zeros', align_corners=True)` restated.

    img [B, C, H, W]; gx, gy [B, P] normalised coords -> [B, C, P].
    Bilinear: four corners weighted by opposite areas, out-of-range corners contribute 0, a
    non-finite coordinate gives NaN.  Nearest: round-half-to-even, out of range -> 0, non-finite -> 0.
    """
    B, C, H, W = img.shape
    flat = img.reshape(B, C, H * W)
    ix = _unnorm(gx, W)
    iy = _unnorm(gy, H)
    finite = torch.isfinite(ix) & torch.isfinite(iy)
    ixs = torch.where(finite, ix, torch.zeros_like(ix))
    iys = torch.where(finite, iy, torch.zeros_like(iy))

    def tap(xi, yi):
        ok = (xi >= 0) & (xi <= W - 1) & (yi >= 0) & (yi <= H - 1) & finite
        idx = (yi.clamp(0, H - 1) * W + xi.clamp(0, W - 1)).long()
        v = torch.gather(flat, 2, idx.unsqueeze(1).expand(B, C, idx.shape[-1]))
        return v * ok.unsqueeze(1).to(img.dtype)

    if mode == 'nearest':
        xn = torch.round(ixs)          # torch.round = round-half-to-even
        yn = torch.round(iys)
        return tap(xn, yn)
    x0 = torch.floor(ixs)
    y0 = torch.floor(iys)
    x1, y1 = x0 + 1, y0 + 1
    w_nw = (x1 - ixs) * (y1 - iys)
    w_ne = (ixs - x0) * (y1 - iys)
    w_sw = (x1 - ixs) * (iys - y0)
    w_se = (ixs - x0) * (iys - y0)
    out = (tap(x0, y0) * w_nw.unsqueeze(1) + tap(x1, y0) * w_ne.unsqueeze(1)
           + tap(x0, y1) * w_sw.unsqueeze(1) + tap(x1, y1) * w_se.unsqueeze(1))
    nan = torch.full_like(out, float('nan'))
    return torch.where(finite.unsqueeze(1), out, nan)


def sample3d(vol, gx, gy, gz):
    """5-D `F.grid_sample(vol, grid(x,y,z), 'bilinear', 'zeros', align_corners=True)` restated.

    vol [B, C, D, H, W]; grid x ↦ W, y ↦ H, z ↦ D; gx, gy, gz [B, P] -> [B, C, P].
    """
    B, C, D, H, W = vol.shape
    flat = vol.reshape(B, C, D * H * W)
    ix, iy, iz = _unnorm(gx, W), _unnorm(gy, H), _unnorm(gz, D)
    x0, y0, z0 = torch.floor(ix), torch.floor(iy), torch.floor(iz)
    out = 0
    for dz in (0, 1):
        zc = z0 + dz
        wz = (iz - z0) if dz else (z0 + 1 - iz)
        for dy in (0, 1):
            yc = y0 + dy
            wy = (iy - y0) if dy else (y0 + 1 - iy)
            for dx in (0, 1):
                xc = x0 + dx
                wx = (ix - x0) if dx else (x0 + 1 - ix)
                ok = (xc >= 0) & (xc <= W - 1) & (yc >= 0) & (yc <= H - 1) & (zc >= 0) & (zc <= D - 1)
                idx = ((zc.clamp(0, D - 1) * H + yc.clamp(0, H - 1)) * W + xc.clamp(0, W - 1)).long()
                v = torch.gather(flat, 2, idx.unsqueeze(1).expand(B, C, idx.shape[-1]))
                w = (wx * wy * wz) * ok.to(vol.dtype)
                out = out + v * w.unsqueeze(1)
    return out


def resize_bilinear_ac(x, h, w):
    """`F.interpolate(x, [h, w], mode='bilinear', align_corners=True)` restated (ATen UpSample.h)."""
    B, C, H, W = x.shape

    def axis(n_in, n_out):
        if n_out == n_in:
            i0 = torch.arange(n_out)
            return i0, i0, torch.zeros(n_out, dtype=x.dtype)
        scale = (n_in - 1) / (n_out - 1) if n_out > 1 else 0.0
        scale = torch.tensor(scale, dtype=torch.float32).to(x.dtype)
        src = scale * torch.arange(n_out, dtype=x.dtype)
        i0 = torch.clamp(torch.floor(src).long(), max=n_in - 1)
        lam = torch.clamp(src - i0.to(x.dtype), 0, 1)
        i1 = torch.where(i0 < n_in - 1, i0 + 1, i0)
        return i0, i1, lam

    y0, y1, ly = axis(H, h)
    x0, x1, lx = axis(W, w)
    top = x[:, :, y0][:, :, :, x0] * (1 - lx) + x[:, :, y0][:, :, :, x1] * lx
    bot = x[:, :, y1][:, :, :, x0] * (1 - lx) + x[:, :, y1][:, :, :, x1] * lx
    return top * (1 - ly)[:, None] + bot * ly[:, None]


def reflect_pad1(x):
    """ReflectionPad2d(1) on the last two dims."""
    x = torch.cat([x[..., 1:2, :], x, x[..., -2:-1, :]], dim=-2)
    return torch.cat([x[..., :, 1:2], x, x[..., :, -2:-1]], dim=-1)


def box3_mean(x):
    """avg_pool2d(kernel 3, stride 1) on an already padded map: window sum / 9."""
    H, W = x.shape[-2] - 2, x.shape[-1] - 2
    s = 0
    for dy in range(3):
        for dx in range(3):
            s = s + x[..., dy:dy + H, dx:dx + W]
    return s / 9


def linspace_f32(start, end, steps):
    """torch.linspace in fp32 (used by the reference for every constant grid)."""
    return torch.linspace(start, end, steps)


# =============================================================================================
# Volumetric fusion (reference network/volumetric_fusionnet.py)
# =============================================================================================
class VoxelSpec:
    """Constant grids of VFNet (volumetric_fusionnet.py:15-40, 67-103)."""

    def __init__(self, cfg):
        m, t = cfg['model'], cfg['training']
        self.size = [int(v) for v in m['voxel_size']]                # x, y, z counts
        self.unit = [float(v) for v in m['voxel_unit_size']]
        self.str_p = [float(v) for v in m['voxel_str_p']]
        self.end_p = [self.str_p[i] + self.unit[i] * (self.size[i] - 1) for i in range(3)]
        self.axes = [linspace_f32(self.str_p[i], self.end_p[i], self.size[i]) for i in range(3)]
        self.X, self.Y, self.Z = self.size
        self.V = self.X * self.Y * self.Z
        lvl = int(m['fusion_level'])
        self.h = int(t['height']) // 2 ** (lvl + 1)
        self.w = int(t['width']) // 2 ** (lvl + 1)
        self.D = int(m['proj_d_bins'])
        self.dbins = linspace_f32(m['proj_d_str'], m['proj_d_end'], self.D)
        self.z_scale = float(m['voxel_size'][0])

    def points(self, dtype=torch.float32):
        """[4, V] homogeneous voxel centres, x fastest then y then z."""
        zz, yy, xx = torch.meshgrid(self.axes[2], self.axes[1], self.axes[0], indexing='ij')
        return torch.stack([xx.reshape(-1), yy.reshape(-1), zz.reshape(-1),
                            torch.ones(self.V)]).to(dtype)

    def pixels(self, dtype=torch.float32):
        """[3, h*w] (x, y, 1), x fastest."""
        yy, xx = torch.meshgrid(torch.arange(self.h), torch.arange(self.w), indexing='ij')
        return torch.stack([xx.reshape(-1), yy.reshape(-1), torch.ones(self.h * self.w)]).to(dtype)


def voxel_camera_geometry(spec, K, Einv, mask_lo):
    """Per camera: normalised sample coords, validity and local depth of every voxel.

    A7 (volumetric_fusionnet.py:132-140, 166-195).  K [B,4,4] (fusion scale), Einv [B,4,4],
    mask_lo [B,1,h,w] -> gx, gy [B,V], valid [B,V] bool, z_local [B,V].
    """
    pts = spec.points(K.dtype)
    local = torch.matmul(Einv[:, :3, :], pts)                        # [B,3,V]
    cam = torch.matmul(K[:, :3, :3], local)
    uv = cam[:, :2, :] / (cam[:, 2:3, :] + 1e-8)
    if not bool(torch.isfinite(uv).all()):
        uv = torch.clamp(uv, -spec.w * 2, spec.w * 2)
    gx = (uv[:, 0] / (spec.w - 1) - 0.5) * 2
    gy = (uv[:, 1] / (spec.h - 1) - 0.5) * 2
    occ = sample2d(mask_lo, gx, gy, 'nearest')[:, 0] > 0.5
    front = local[:, 2] > 0
    oob = (gx > 1) | (gx < -1) | (gy > 1) | (gy < -1)
    return gx, gy, occ & front & ~oob, local[:, 2]


def camera_voxel_features(spec, feats, mask, K, Einv):
    """list over cameras of ([B, C+1, V] masked features, [B, V] valid) (fusionnet.py:116-149)."""
    B, N, C = feats.shape[:3]
    out = []
    for c in range(N):
        mlo = resize_bilinear_ac(mask[:, c], spec.h, spec.w)
        gx, gy, valid, z = voxel_camera_geometry(spec, K[:, c], Einv[:, c], mlo)
        f = sample2d(feats[:, c], gx, gy, 'bilinear')
        f = torch.cat([f, (z / spec.z_scale).unsqueeze(1)], 1)
        out.append((f * valid.unsqueeze(1).to(f.dtype), valid))
    return out


def _conv1x1_lrelu(x, weight, bias):
    y = torch.einsum('oc,bcv->bov', weight[:, :, 0], x) + bias.view(1, -1, 1)
    return torch.where(y > 0, y, y * LRELU)


def overlap_groups(n_cams):
    if n_cams == 3:
        return [0], [1, 2]
    if n_cams == 6:
        return [0, 3, 4], [1, 2, 5]
    raise NotImplementedError(f'overlap fusion needs 3 or 6 cameras, got {n_cams}')


def fuse_depth(spec, feats, mask, K, Einv, w_no, b_no, w_o, b_o):
    """K1 / A8: depth-mode fusion -> [B, Cv, V] (fusionnet.py:151-158, 197-230)."""
    per_cam = camera_voxel_features(spec, feats, mask, K, Einv)
    cnt = sum(v.to(feats.dtype) for _, v in per_cam).unsqueeze(1)
    one = (cnt == 1).to(feats.dtype)
    two = (cnt == 2).to(feats.dtype)
    s = sum(f for f, _ in per_cam) * one
    no = _conv1x1_lrelu(s, w_no, b_no) * one
    ga, gb = overlap_groups(len(per_cam))
    cat = torch.cat([sum(per_cam[i][0] for i in ga), sum(per_cam[i][0] for i in gb)], 1)
    ov = _conv1x1_lrelu(cat, w_o, b_o) * two
    return no + ov


def fuse_pose(spec, feats, mask, K, Einv):
    """K2 / A9: pose-mode fusion, mean over valid cameras -> [B, C+1, V] (fusionnet.py:160-162)."""
    per_cam = camera_voxel_features(spec, feats, mask, K, Einv)
    cnt = sum(v.to(feats.dtype) for _, v in per_cam).unsqueeze(1)
    return sum(f for f, _ in per_cam) / (cnt + 1e-7)


def project_voxels(spec, vox, invK, E):
    """K3 / A10: trilinear resampling of the voxel grid on each camera frustum.

    vox [B, Cv, V]; invK, E [B, N, 4, 4] -> list over cameras of [B, Cv*D, h, w]
    (channel = c*D + d) (fusionnet.py:232-262, before `reduce_dim`).
    """
    B, Cv, _ = vox.shape
    vol = vox.reshape(B, Cv, spec.Z, spec.Y, spec.X)
    pix = spec.pixels(vox.dtype)
    P = pix.shape[1]
    out = []
    for c in range(E.shape[1]):
        ray = torch.matmul(invK[:, c, :3, :3], pix)                          # [B,3,P]
        pts = spec.dbins.to(vox.dtype).view(1, 1, -1, 1) * ray.view(B, 3, 1, P)   # [B,3,D,P]
        pts = torch.cat([pts, torch.ones(B, 1, spec.D, P, dtype=vox.dtype)], 1).view(B, 4, -1)
        world = torch.matmul(E[:, c, :3, :], pts)                            # [B,3,D*P]
        g = [(world[:, i] - spec.str_p[i]) / (spec.end_p[i] - spec.str_p[i]) * 2.0 - 1.0 for i in range(3)]
        s = sample3d(vol, g[0], g[1], g[2])                                  # [B,Cv,D*P]
        out.append(s.view(B, Cv * spec.D, spec.h, spec.w))
    return out


# =============================================================================================
# Geometry / view synthesis (reference models/geometry/*)
# =============================================================================================
def backproject(invK, depth):
    """A13 (geometry_util.py:56-64): depth [B,1,H,W] -> homogeneous points [B,4,H*W]."""
    B, _, H, W = depth.shape
    yy, xx = torch.meshgrid(torch.arange(H), torch.arange(W), indexing='ij')
    pix = torch.stack([xx.reshape(-1), yy.reshape(-1), torch.ones(H * W)]).to(depth.dtype)
    pts = depth.reshape(B, 1, -1) * torch.matmul(invK[:, :3, :3], pix)
    return torch.cat([pts, torch.ones(B, 1, H * W, dtype=depth.dtype)], 1)


def reproject(K, T, pts, H, W):
    """A13 (geometry_util.py:66-81): -> normalised (gx, gy) [B, H*W]."""
    uvw = torch.matmul(torch.matmul(K, T)[:, :3, :], pts)
    uv = uvw[:, :2] / (uvw[:, 2:3] + 1e-7)
    return (uv[:, 0] / (W - 1) - 0.5) * 2, (uv[:, 1] / (H - 1) - 0.5) * 2


def virtual_image(src_img, src_mask, depth, invK, K, T):
    """A14 (view_rendering.py:61-82): warped image [B,3,H,W] and validity mask [B,1,H,W]."""
    B, _, H, W = depth.shape
    gx, gy = reproject(K, T, backproject(invK, depth), H, W)
    img = sample2d(src_img, gx, gy, 'bilinear')
    msk = sample2d(src_mask, gx, gy, 'nearest')
    img = torch.where(torch.isnan(img), torch.full_like(img, 2.0), img)
    msk = torch.where(torch.isnan(msk), torch.zeros_like(msk), msk)
    bad = ((gx > 1) | (gx < -1) | (gy > 1) | (gy < -1)).unsqueeze(1)
    return img.view(B, -1, H, W), ((~bad).to(img.dtype) * msk).view(B, 1, H, W)


def intensity_align(ref_img, ref_mask, warp_img, warp_mask):
    """A15 (view_rendering.py:30-59): match the warp's statistics to the target's."""
    warp_mask = warp_mask.detach()
    with torch.no_grad():
        m = (ref_mask * warp_mask) != 0
        m = m.expand(-1, 3, -1, -1).to(ref_img.dtype)
        if bool((m.sum(dim=(1, 2, 3)) == 0).any()):
            return warp_img
        n_all = m.shape[1] * m.shape[2] * m.shape[3]

        def stats(x):
            mu = (x * m).sum(dim=(1, 2, 3), keepdim=True) / (m.sum(dim=(1, 2, 3), keepdim=True) + 1e-8)
            var = ((x - mu) ** 2).sum(dim=(1, 2, 3), keepdim=True) / n_all
            return mu, torch.sqrt(var + 1e-16)

        s_mu, s_sd = stats(ref_img)
        w_mu, w_sd = stats(warp_img)
    return ((warp_img - w_mu) / (w_sd + 1e-8) * s_sd + s_mu) * warp_mask


def view_rendering(inputs, cam_out, cam, rel_poses, cfg):
    """A16 (view_rendering.py:118-198): fills cam_out with colour / overlap planes for scale 0."""
    t = cfg['training']
    frames = t['frame_ids']
    rel = cfg['data']['rel_cam_list'][cam]
    N = cfg['data']['num_cams']
    ref_color = inputs[('color', 0, 0)][:, cam]
    ref_mask = inputs['mask'][:, cam]
    ref_K = inputs[('K', 0)][:, cam]
    ref_invK = inputs[('inv_K', 0)][:, cam]
    for scale in t['scales']:
        depth = cam_out[('depth', scale)]
        for f in frames[1:]:
            img, msk = virtual_image(inputs[('color', f, 0)][:, cam], inputs['mask'][:, cam], depth,
                                     ref_invK, ref_K, cam_out[('cam_T_cam', 0, f)])
            if t['intensity_align']:
                img = intensity_align(ref_color, ref_mask, img, msk)
            cam_out[('color', f, scale)] = img
            cam_out[('color_mask', f, scale)] = msk
        if t['spatio'] or t['spatio_temporal']:
            for f in frames:
                acc_img = torch.zeros_like(ref_color)
                acc_msk = torch.zeros_like(ref_mask)
                for src in rel:
                    if src >= N:
                        continue
                    img, msk = virtual_image(inputs[('color', f, 0)][:, src], inputs['mask'][:, src], depth,
                                             ref_invK, inputs[('K', 0)][:, src], rel_poses[(f, src)])
                    if t['intensity_align']:
                        img = intensity_align(ref_color, ref_mask, img, msk)
                    acc_img = acc_img + img
                    acc_msk = acc_msk + msk
                cam_out[('overlap', f, scale)] = acc_img
                cam_out[('overlap_mask', f, scale)] = acc_msk


def relative_poses(inputs, cam_out, cam, cfg):
    """A12 (pose.py:66-96): spatial and spatio-temporal source←target transforms."""
    t = cfg['training']
    N = cfg['data']['num_cams']
    rel = cfg['data']['rel_cam_list'][cam]
    ref_ext = inputs['extrinsics'][:, cam]
    d = {}
    if t['spatio']:
        for src in rel:
            if src < N:
                d[(0, src)] = torch.matmul(inputs['extrinsics_inv'][:, src], ref_ext)
    if t['spatio_temporal']:
        for f in t['frame_ids'][1:]:
            for src in rel:
                if src < N:
                    d[(f, src)] = torch.matmul(d[(0, src)], cam_out[('cam_T_cam', 0, f)])
    return d


def axis_angle_to_matrix(aa):
    """pytorch3d formula (aa → quaternion → matrix), see vfdepth_amd/rotation.py for the cite."""
    ang = torch.norm(aa, dim=-1, keepdim=True)
    small = ang.abs() < 1e-6
    k = torch.where(small, 0.5 - ang * ang / 48, torch.sin(ang / 2) / torch.where(small, torch.ones_like(ang), ang))
    q = torch.cat([torch.cos(ang / 2), aa * k], -1)
    r, i, j, kk = q.unbind(-1)
    s = 2.0 / (q * q).sum(-1)
    return torch.stack([1 - s * (j * j + kk * kk), s * (i * j - kk * r), s * (i * kk + j * r),
                        s * (i * j + kk * r), 1 - s * (i * i + kk * kk), s * (j * kk - i * r),
                        s * (i * kk - j * r), s * (j * kk + i * r), 1 - s * (i * i + j * j)], -1).view(*aa.shape[:-1], 3, 3)


def vec_to_matrix(rot, trans, invert=False):
    """A12 (geometry_util.py:8-30): [B,1,3] axis-angle, [B,1,3] translation -> [B,4,4]."""
    B = rot.shape[0]
    R = torch.eye(4, dtype=rot.dtype).repeat(B, 1, 1)
    Tm = torch.eye(4, dtype=rot.dtype).repeat(B, 1, 1)
    R[:, :3, :3] = axis_angle_to_matrix(rot).squeeze(1)
    tv = trans.reshape(-1, 3, 1)
    if invert:
        R = R.transpose(1, 2)
        tv = -tv
    Tm[:, :3, 3:] = tv
    return torch.matmul(R, Tm) if invert else torch.matmul(Tm, R)


def distribute_pose(T, E, Einv, N):
    """A12 (pose.py:44-64): canonical pose -> per-camera poses."""
    return [Einv[:, c] @ E[:, 0] @ T @ Einv[:, 0] @ E[:, c] for c in range(N)]


def to_depth(disp, K0, cfg):
    """A3 (vfdepth.py:277-288); the resize to (H, W) is the identity at scale 0."""
    t = cfg['training']
    lo, hi = 1 / t['max_depth'], 1 / t['min_depth']
    d = 1 / (lo + (hi - lo) * disp)
    return d * K0[:, 0:1, 0:1].unsqueeze(2) / t['focal_length_scale']


def augment_extrinsics(E, aug_angle, angle):
    """A17 (volumetric_fusionnet.py:269-287): a random rotation applied in front of every camera's
    extrinsics.  `angle` [B, N, 3] stands for the reference's `torch.rand(b, cam, 3)` draw;
    (angle - 0.5) * aug_angle[i] is used as an axis-angle in RADIANS (the config's values are
    called degrees, the reference feeds them to axis_angle_to_matrix unchanged)."""
    a = (angle - 0.5) * torch.tensor([float(v) for v in aug_angle], dtype=angle.dtype)
    T = torch.eye(4, dtype=E.dtype).repeat(*E.shape[:2], 1, 1)
    T[:, :, :3, :3] = axis_angle_to_matrix(a).to(E.dtype)
    return T @ E


def virtual_depth(src_depth, src_mask, src_invK, tar_depth, tar_invK, src_K, T, min_depth, max_depth):
    """A17 (view_rendering.py:84-116): the source depth map, expressed in the novel view's camera
    (z of T @ backproject(src)), backward-warped into the novel view through the novel view's own
    depth; NaN -> 2.0, masks by nearest lookup, OOB and the [min, max] range (out-of-range values
    replaced by the bound: no gradient through them).  -> depth [B,1,H,W], mask [B,1,H,W]."""
    B, _, H, W = src_depth.shape
    z = torch.matmul(T[:, :3, :], backproject(src_invK, src_depth)).reshape(B, 3, H, W)[:, 2:3]
    gx, gy = reproject(src_K, torch.inverse(T), backproject(tar_invK, tar_depth), H, W)
    d = sample2d(z, gx, gy, 'bilinear')
    m = sample2d(src_mask, gx, gy, 'nearest')
    d = torch.where(torch.isnan(d), torch.full_like(d, 2.0), d)
    m = torch.where(torch.isnan(m), torch.zeros_like(m), m)
    bad = ((gx > 1) | (gx < -1) | (gy > 1) | (gy < -1)).unsqueeze(1)
    vmin = d > min_depth
    d = torch.where(vmin, d, torch.full_like(d, min_depth))
    vmax = d < max_depth
    d = torch.where(vmax, d, torch.full_like(d, max_depth))
    mask = (~bad).to(d.dtype) * m * vmin.to(d.dtype) * vmax.to(d.dtype)
    return d.view(B, 1, H, W), mask.view(B, 1, H, W)


def depth_synthesis(inputs, outputs, cam, cfg):
    """A17 (view_rendering.py:201-241): tform_depth / tform_depth_mask lists of camera `cam`
    (sources rel_cam_list[cam] + [cam], each warped into the augmented view of `cam`)."""
    t = cfg['training']
    N = cfg['data']['num_cams']
    aug_ext = inputs['extrinsics_aug'][:, cam]
    aug_inv = torch.inverse(aug_ext)
    ref_K, ref_invK = inputs[('K', 0)][:, cam], inputs[('inv_K', 0)][:, cam]
    view = outputs[('cam', cam)]
    depths, masks = [], []
    for src in list(cfg['data']['rel_cam_list'][cam]) + [cam]:
        if src >= N:
            continue
        rel = torch.matmul(aug_inv, inputs['extrinsics'][:, src])
        d, m = virtual_depth(outputs[('cam', src)][('depth', 0)], inputs['mask'][:, src],
                             inputs[('inv_K', 0)][:, src], view[('depth', 0, 'aug')], ref_invK,
                             inputs[('K', 0)][:, src], rel, t['min_depth'], t['max_depth'])
        depths.append(d)
        masks.append(m)
    view[('tform_depth', 0)] = depths
    view[('tform_depth_mask', 0)] = masks


def depth_synthesis_loss(view):
    """A17 (depth_synthesis_loss.py:15-45): consistency clamp(|a - t| / (a + t + 1e-8), 0, 1),
    masked mean pooled over all sources; plain gradient smoothness of disp_aug / mean."""
    aug = view[('depth', 0, 'aug')]
    pl = torch.cat([torch.clamp((aug - d).abs() / (aug + d + 1e-8), 0., 1.) for d in view[('tform_depth', 0)]], 0)
    pm = torch.cat(list(view[('tform_depth_mask', 0)]), 0)
    con = masked_mean(pl, pm)
    disp = view[('disp', 0, 'aug')]
    nd = disp / (disp.mean(2, True).mean(3, True) + 1e-8)
    sm = (nd[..., :-1] - nd[..., 1:]).abs().mean() + (nd[..., :-1, :] - nd[..., 1:, :]).abs().mean()
    return con, sm


# =============================================================================================
# Losses (reference models/losses/*)
# =============================================================================================
def ssim_loss(pred, target):
    """A18 (loss_util.py:43-67)."""
    p, t = reflect_pad1(pred), reflect_pad1(target)
    mu_p, mu_t = box3_mean(p), box3_mean(t)
    mp2, mt2, mpt = mu_p * mu_p, mu_t * mu_t, mu_p * mu_t
    s_p = box3_mean(p * p) - mp2
    s_t = box3_mean(t * t) - mt2
    s_pt = box3_mean(p * t) - mpt
    c1, c2 = 0.01 ** 2, 0.03 ** 2
    ssim = ((2 * mpt + c1) * (2 * s_pt + c2)) / ((mp2 + mt2 + c1) * (s_p + s_t + c2) + 1e-8)
    return torch.clamp((1 - ssim) / 2, 0, 1)


def photometric(pred, target):
    """A19 (loss_util.py:70-78): 0.85 SSIM + 0.15 L1, channel means -> [B,1,H,W]."""
    l1 = (target - pred).abs().mean(1, True)
    return 0.85 * ssim_loss(pred, target).mean(1, True) + 0.15 * l1


def masked_mean(loss, mask):
    """A20 (loss_util.py:21-25): batch-pooled masked mean."""
    return (loss * mask).sum() / (mask.sum() + 1e-8)


def edge_smoothness(rgb, disp):
    """A20 (loss_util.py:28-40)."""
    gix = (rgb[..., :-1] - rgb[..., 1:]).abs().mean(1, True)
    giy = (rgb[..., :-1, :] - rgb[..., 1:, :]).abs().mean(1, True)
    gdx = (disp[..., :-1] - disp[..., 1:]).abs() * torch.exp(-gix)
    gdy = (disp[..., :-1, :] - disp[..., 1:, :]).abs() * torch.exp(-giy)
    return gdx.mean() + gdy.mean()


def cam_loss(inputs, cam_out, cam, cfg, noise):
    """A21/A22 (single_cam_loss.py:17-65, multi_cam_loss.py:16-59, 94-121) for scale 0.

    `noise` [B, T, H, W] stands for `1e-5 * torch.randn(...)` of single_cam_loss.py:45-46.
    Returns (cam_loss, dict of the four scalar terms).
    """
    t, lc = cfg['training'], cfg['loss']
    frames = t['frame_ids']
    target = inputs[('color', 0, 0)][:, cam]
    ref_mask = inputs['mask'][:, cam]
    total = 0.0
    terms = {}
    for scale in t['scales']:
        rep = torch.cat([photometric(cam_out[('color', f, scale)], target) for f in frames[1:]], 1)
        rep_min, _ = torch.min(rep, 1, keepdim=True)
        idn = torch.cat([photometric(inputs[('color', f, 0)][:, cam], target) for f in frames[1:]], 1)
        idn = idn + noise
        idn_min, _ = torch.min(idn, 1, keepdim=True)
        auto = (torch.argmin(torch.cat([rep_min, idn_min], 1), 1, keepdim=True) == 0).to(rep.dtype)
        auto = auto * ref_mask
        cam_out[('reproj_loss', scale)] = auto * rep_min
        cam_out[('reproj_mask', scale)] = auto
        l_rep = masked_mean(rep_min, auto)
        disp = cam_out[('disp', scale)]
        mean_disp = disp.mean(2, True).mean(3, True)
        l_sm = edge_smoothness(inputs[('color', 0, scale)][:, cam], disp / (mean_disp + 1e-8))
        multi = t['spatio'] or t['spatio_temporal']
        if multi:
            sp_mask = ref_mask * cam_out[('overlap_mask', 0, scale)]
            l_sp = masked_mean(photometric(cam_out[('overlap', 0, scale)], target), sp_mask)
            cam_out[('overlap_mask', 0, scale)] = sp_mask
            st = torch.cat([photometric(cam_out[('overlap', f, scale)], target) for f in frames[1:]], 1)
            sm = torch.cat([ref_mask * cam_out[('overlap_mask', f, scale)] * auto for f in frames[1:]], 1)
            st_min, _ = torch.min(st, 1, keepdim=True)
            sm_max, _ = torch.max(sm, 1, keepdim=True)
            l_st = masked_mean(st_min, sm_max)
        total = total + l_rep
        total = total + lc['disparity_smoothness'] * l_sm / (2 ** scale)
        if multi:
            total = total + (lc['spatio_coeff'] * l_sp + lc['spatio_tempo_coeff'] * l_st)
        if scale == 0:
            terms = {'reproj_loss': l_rep, 'smooth': l_sm}
            if multi:
                terms.update({'spatio_loss': l_sp, 'spatio_tempo_loss': l_st})
    return total / len(t['scales']), terms


def depth_errors(pred, gt):
    """A24 (utils/misc.py:85-98): abs_rel, sq_rel, rmse, rmse_log, a1, a2, a3."""
    thresh = torch.max(gt / pred, pred / gt)
    return (torch.mean((pred - gt).abs() / gt), torch.mean((pred - gt) ** 2 / gt),
            torch.sqrt(torch.mean((pred - gt) ** 2)), torch.sqrt(torch.mean((torch.log(gt) - torch.log(pred)) ** 2)),
            (thresh < 1.25).float().mean(), (thresh < 1.25 ** 2).float().mean(), (thresh < 1.25 ** 3).float().mean())


# =============================================================================================
# Whole step (A1/A2/A4/A5 restated around caller-supplied dense layers)
# =============================================================================================
def process_batch(nets, inputs, cfg, noise, aug_angles=None):
    """Restated `VFDepthAlgo.process_batch` (vfdepth.py:191-313) for the fusion configs.

    `nets` supplies the dense (non-hot-path) layers as callables/tensors shared with the
    product via one state dict: pose_encoder, pose_conv1x1, pose_reduce_dim, pose_decoder,
    depth_encoder, depth_conv1x1, depth_reduce_dim, depth_decoder, w_no, b_no, w_o, b_o.
    `noise[cam]` is the identity-loss noise for camera `cam`; with training.aug_depth,
    `aug_angles` [B, N, 3] stands for augment_extrinsics' torch.rand draw (depth synthesis:
    volumetric_fusionnet.py:313-317, fusion_depthnet.py:79-86, depth_synthesis_loss.py).
    Returns (outputs, losses) in the reference schema.
    """
    t = cfg['training']
    N = cfg['data']['num_cams']
    B = inputs[('color', 0, 0)].shape[0]
    lvl = cfg['model']['fusion_level']
    spec = VoxelSpec(cfg)
    inputs = dict(inputs)
    inputs['extrinsics_inv'] = torch.inverse(inputs['extrinsics'])
    K_l, invK_l = inputs[('K', lvl + 1)], inputs[('inv_K', lvl + 1)]
    E, Einv = inputs['extrinsics'], inputs['extrinsics_inv']

    def aggregate(enc, conv1x1, images):
        feats = enc(images.reshape(B * N, *images.shape[2:]))
        hh, ww = feats[lvl].shape[-2:]
        up = [feats[lvl]] + [torch.nn.functional.interpolate(f, [hh, ww], mode='bilinear', align_corners=True)
                             for f in feats[lvl + 1:]]
        return feats, conv1x1(torch.cat(up, 1)).view(B, N, -1, hh, ww)

    outputs = {('cam', c): {} for c in range(N)}
    for f in t['frame_ids'][1:]:
        pair = [-1, 0] if f < 0 else [0, 1]
        imgs = torch.cat([inputs[('color_aug', pair[0], 0)], inputs[('color_aug', pair[1], 0)]], 2)
        _, agg = aggregate(nets.pose_encoder, nets.pose_conv1x1, imgs)
        vox = fuse_pose(spec, agg, inputs['mask'], K_l, Einv)
        bev = nets.pose_reduce_dim(vox.reshape(B, -1, spec.Y, spec.X))
        aa, tr = nets.pose_decoder([[bev]])
        T = vec_to_matrix(aa[:, 0], torch.clamp(tr, -4.0, 4.0)[:, 0], invert=(f < 0))
        for c, Tc in enumerate(distribute_pose(T, E, Einv, N)):
            outputs[('cam', c)][('cam_T_cam', 0, f)] = Tc

    feats, agg = aggregate(nets.depth_encoder, nets.depth_conv1x1, inputs[('color_aug', 0, 0)])
    vox = fuse_depth(spec, agg, inputs['mask'], K_l, Einv, nets.w_no, nets.b_no, nets.w_o, nets.b_o)
    proj = project_voxels(spec, vox, invK_l, E)
    proj = torch.stack([nets.depth_reduce_dim(p) for p in proj], 1).reshape(B * N, -1, spec.h, spec.w)
    disp = nets.depth_decoder(feats[:lvl] + [proj])
    aug = bool(t.get('aug_depth', False))
    if aug:
        inputs['extrinsics_aug'] = augment_extrinsics(E, t['aug_angle'], aug_angles)
        proj_aug = project_voxels(spec, vox, invK_l, inputs['extrinsics_aug'])
        proj_aug = torch.stack([nets.depth_reduce_dim(p) for p in proj_aug], 1).reshape(B * N, -1, spec.h, spec.w)
        disp_aug = nets.depth_decoder(feats[:lvl] + [proj_aug])
    for c in range(N):
        for k, v in disp.items():
            outputs[('cam', c)][k] = v.view(B, N, *v.shape[1:])[:, c]
        for s in t['scales']:
            outputs[('cam', c)][('depth', s)] = to_depth(outputs[('cam', c)][('disp', s)], inputs[('K', 0)][:, c], cfg)
        if aug:
            for k, v in disp_aug.items():
                outputs[('cam', c)][k + ('aug',)] = v.view(B, N, *v.shape[1:])[:, c]
            for s in t['scales']:
                outputs[('cam', c)][('depth', s, 'aug')] = to_depth(outputs[('cam', c)][('disp', s, 'aug')],
                                                                    inputs[('K', 0)][:, c], cfg)

    total = 0.0
    logs = {}
    for c in range(N):
        rp = relative_poses(inputs, outputs[('cam', c)], c, cfg)
        view_rendering(inputs, outputs[('cam', c)], c, rp, cfg)
        cl, terms = cam_loss(inputs, outputs[('cam', c)], c, cfg, noise[c])
        if aug:
            lc = cfg['loss']
            depth_synthesis(inputs, outputs, c, cfg)
            con, sm = depth_synthesis_loss(outputs[('cam', c)])
            syn = lc['depth_con_coeff'] * con + lc['depth_sm_coeff'] * sm
            cl = cl + syn
            terms.update({'depth_loss': syn, 'depth_sm_loss': sm, 'depth_con_loss': con, 'cam_loss': cl})
        total = total + cl
        d = outputs[('cam', c)][('depth', 0)].detach()
        terms.update({'depth/mean': d.mean(), 'depth/max': d.max(), 'depth/min': d.min()})
        if c == 0:
            pt = outputs[('cam', 0)][('cam_T_cam', 0, -1)].detach()
            terms.update({'pose/tx': pt[:, 0, 3].abs().mean(), 'pose/ty': pt[:, 1, 3].abs().mean(),
                          'pose/tz': pt[:, 2, 3].abs().mean()})
        for k, v in terms.items():
            logs.setdefault(k, []).append(v.detach() if torch.is_tensor(v) else v)
    losses = {k: sum(v) / len(v) for k, v in logs.items()}
    losses['total_loss'] = total / N
    return outputs, losses


class _Nets:
    pass


def nets_from_modules(depth_net, pose_net):
    """Adapter: dense layers of depth/pose networks that use the reference's attribute names
    (FusedDepthNet.encoder/conv1x1/fusion_net/decoder, FusedPoseNet.…/pose_decoder)."""
    n = _Nets()
    n.depth_encoder, n.depth_conv1x1 = depth_net.encoder, depth_net.conv1x1
    n.depth_reduce_dim, n.depth_decoder = depth_net.fusion_net.reduce_dim, depth_net.decoder
    n.pose_encoder, n.pose_conv1x1 = pose_net.encoder, pose_net.conv1x1
    n.pose_reduce_dim, n.pose_decoder = pose_net.fusion_net.reduce_dim, pose_net.pose_decoder
    fn = depth_net.fusion_net
    n.w_no, n.b_no = fn.conv_non_overlap[0].weight, fn.conv_non_overlap[0].bias
    n.w_o, n.b_o = fn.conv_overlap[0].weight, fn.conv_overlap[0].bias
    return n

"""Camera geometry and view synthesis (reference `/root/reference/models/geometry/`).

* `vec_to_matrix`, `Pose` — pose assembly (geometry_util.py:8-30, pose.py:7-96); tiny 4x4 math,
  stays in PyTorch (autograd carries the pose-net gradient).
* `ViewRendering` — the K4 kernels.  `forward(inputs, outputs, cam, rel_pose_dict)` keeps the
  reference's per-camera API; `render_all(inputs, outputs, rel_poses)` renders every camera's
  warps in one fused launch sequence and is what `VFDepthAlgo` uses.
"""
import os

import torch
import torch.nn as nn

from . import kernels as KN
from .rotation import axis_angle_to_matrix


def inverse4x4(m):
    """Batched general 4x4 inverse by cofactors (capturable in a HIP graph, no solver workspace).
    Replaces torch.inverse on the extrinsics (vfdepth.py:211); for the rigid camera transforms the
    two agree to fp32 rounding.  fp32 GPU tensors without a gradient run the one-launch HIP kernel
    (`vfd_inverse4x4`, the same operation order: bit-identical); otherwise the torch ops below."""
    if m.is_cuda and m.dtype == torch.float32 and not (m.requires_grad and torch.is_grad_enabled()):
        from . import _lib as L
        src = m.contiguous()
        out = torch.empty_like(src)
        L.check(L.load().vfd_inverse4x4(src.data_ptr(), out.data_ptr(), src.numel() // 16, L.stream()), 'inverse4x4')
        return out
    a = m.reshape(-1, 4, 4)
    a00, a01, a02, a03 = a[:, 0, 0], a[:, 0, 1], a[:, 0, 2], a[:, 0, 3]
    a10, a11, a12, a13 = a[:, 1, 0], a[:, 1, 1], a[:, 1, 2], a[:, 1, 3]
    a20, a21, a22, a23 = a[:, 2, 0], a[:, 2, 1], a[:, 2, 2], a[:, 2, 3]
    a30, a31, a32, a33 = a[:, 3, 0], a[:, 3, 1], a[:, 3, 2], a[:, 3, 3]
    s0, s1, s2 = a00 * a11 - a10 * a01, a00 * a12 - a10 * a02, a00 * a13 - a10 * a03
    s3, s4, s5 = a01 * a12 - a11 * a02, a01 * a13 - a11 * a03, a02 * a13 - a12 * a03
    c5, c4, c3 = a22 * a33 - a32 * a23, a21 * a33 - a31 * a23, a21 * a32 - a31 * a22
    c2, c1, c0 = a20 * a33 - a30 * a23, a20 * a32 - a30 * a22, a20 * a31 - a30 * a21
    det = s0 * c5 - s1 * c4 + s2 * c3 + s3 * c2 - s4 * c1 + s5 * c0
    inv = torch.stack([
        a11 * c5 - a12 * c4 + a13 * c3, -a01 * c5 + a02 * c4 - a03 * c3,
        a31 * s5 - a32 * s4 + a33 * s3, -a21 * s5 + a22 * s4 - a23 * s3,
        -a10 * c5 + a12 * c2 - a13 * c1, a00 * c5 - a02 * c2 + a03 * c1,
        -a30 * s5 + a32 * s2 - a33 * s1, a20 * s5 - a22 * s2 + a23 * s1,
        a10 * c4 - a11 * c2 + a13 * c0, -a00 * c4 + a01 * c2 - a03 * c0,
        a30 * s4 - a31 * s2 + a33 * s0, -a20 * s4 + a21 * s2 - a23 * s0,
        -a10 * c3 + a11 * c1 - a12 * c0, a00 * c3 - a01 * c1 + a02 * c0,
        -a30 * s3 + a31 * s1 - a32 * s0, a20 * s3 - a21 * s1 + a22 * s0], -1)
    return (inv / det.unsqueeze(-1)).reshape(m.shape)


def vec_to_matrix(rot_angle, trans_vec, invert=False):
    """Axis-angle [B,1,3] + translation [B,1,3] -> [B,4,4]; invert -> R^T @ T(-t)."""
    b = rot_angle.shape[0]
    R = torch.eye(4, device=rot_angle.device, dtype=rot_angle.dtype).repeat(b, 1, 1)
    Tm = torch.eye(4, device=rot_angle.device, dtype=rot_angle.dtype).repeat(b, 1, 1)
    R[:, :3, :3] = axis_angle_to_matrix(rot_angle).squeeze(1)
    t = trans_vec.clone().contiguous().view(-1, 3, 1)
    if invert:
        R = R.transpose(1, 2)
        t = -1 * t
    Tm[:, :3, 3:] = t
    return torch.matmul(R, Tm) if invert else torch.matmul(Tm, R)


# the fused pose net's frame pairs as one batch in eager steps (VFD_POSE_PAIRS=0 turns it off):
# config 2 31.3/32.2 vs 34.5/33.9 ms/step on one box, alternating runs (round 5)
_POSE_PAIRS = os.environ.get('VFD_POSE_PAIRS', '1') == '1'


class Pose:
    """Multi-camera pose handling (pose.py:7-96)."""

    def __init__(self, cfg):
        t, dt = cfg['training'], cfg['data']
        self.pose_model = cfg['model']['pose_model']
        self.frame_ids = list(t['frame_ids'])
        self.num_cams = int(dt['num_cams'])
        self.rel_cam_list = dt['rel_cam_list']
        self.spatio, self.spatio_temporal = bool(t['spatio']), bool(t['spatio_temporal'])
        # the frame pairs as one batch (eager steps and the captured step alike); False: one pose-net
        # call per pair, as the reference
        self.batch_pairs = True

    def compute_pose(self, net, inputs):
        if self.pose_model == 'fusion':
            pose = self.get_single_pose(net, inputs, None)
            return self.distribute_pose(pose, inputs['extrinsics'], inputs['extrinsics_inv'])
        return {('cam', c): self.get_single_pose(net, inputs, c) for c in range(self.num_cams)}

    def get_single_pose(self, net, inputs, cam):
        """pose.py:31-42: one net call per context frame (pairs in temporal order).  By default
        (VFD_POSE_PAIRS=1) the fused pose net takes all pairs in ONE call: its stacked-batch forward
        gives each pair exactly the reference call's BatchNorm statistics."""
        out = {}
        fids = self.frame_ids[1:]
        pairs = [[-1, 0] if f < 0 else [0, 1] for f in fids]
        if cam is None and self.pose_model == 'fusion' and len(pairs) > 1 and _POSE_PAIRS and self.batch_pairs:
            for f, (axisangle, translation) in zip(fids, net(inputs, pairs, cam)):
                out[('cam_T_cam', 0, f)] = vec_to_matrix(axisangle[:, 0], translation[:, 0], invert=(f < 0))
            return out
        for f, pair in zip(fids, pairs):
            axisangle, translation = net(inputs, pair, cam)
            out[('cam_T_cam', 0, f)] = vec_to_matrix(axisangle[:, 0], translation[:, 0], invert=(f < 0))
        return out

    def distribute_pose(self, poses, exts, exts_inv):
        """Canonical (camera 0) motion -> every camera: E_c^-1 E_0 T E_0^-1 E_c, all cameras in one
        batched chain (the reference's left-to-right association).  The per-camera entries are
        views of out['_cam_T_cam'][f] = [B, N, 4, 4], which the batched warp path consumes."""
        out = {('cam', c): {} for c in range(self.num_cams)}
        out['_cam_T_cam'] = {}
        ref_ext, ref_inv = exts[:, :1], exts_inv[:, :1]
        for f in self.frame_ids[1:]:
            T = poses['cam_T_cam', 0, f].float().unsqueeze(1)
            P = exts_inv @ ref_ext @ T @ ref_inv @ exts
            out['_cam_T_cam'][f] = P
            for c in range(self.num_cams):
                out[('cam', c)][('cam_T_cam', 0, f)] = P[:, c]
        return out

    def compute_relative_cam_poses(self, inputs, outputs, cam):
        ref_ext = inputs['extrinsics'][:, cam]
        view = outputs[('cam', cam)]
        rel = {}
        if self.spatio:
            for s in self.rel_cam_list[cam]:
                if s < self.num_cams:
                    rel[(0, s)] = torch.matmul(inputs['extrinsics_inv'][:, s], ref_ext)
        if self.spatio_temporal:
            for f in self.frame_ids[1:]:
                for s in self.rel_cam_list[cam]:
                    if s < self.num_cams:
                        rel[(f, s)] = torch.matmul(rel[(0, s)], view[('cam_T_cam', 0, f)])
        return rel


class ViewRendering(nn.Module):
    """Warped colour / overlap synthesis on the K4 kernels (view_rendering.py:9-243)."""

    def __init__(self, cfg, rank):
        super().__init__()
        t, dt = cfg['training'], cfg['data']
        self.cfg = cfg
        self.rank = rank
        self.scales = list(t['scales'])
        self.frame_ids = list(t['frame_ids'])
        self.num_cams = int(dt['num_cams'])
        self.aug_depth = bool(t.get('aug_depth', False))
        self._plan = None

    def plan(self, device):
        if self._plan is None or self._plan.tab.device != torch.device(device):
            self._plan = KN.ViewPlan(self.cfg, device)
        return self._plan

    def warp_matrices(self, inputs, outputs, rel_poses, cams):
        """(K_src @ T)[:3] per (target camera, warp) in the plan's order -> [B, len(cams), n_warp, 3, 4].
        T: the temporal pose cam_T_cam[c][f], or the relative pose (E_src^-1 E_c) [@ cam_T_cam[c][f]]
        (pose.py:66-96).  With the batched poses of the fusion pose model and rel_poses None,
        every warp of every camera is one gather + three batched products."""
        if rel_poses is None:
            return self._warp_matrices_all(inputs, outputs)[:, cams[0]:cams[-1] + 1]
        plan = self.plan(inputs[('K', 0)].device)
        K = inputs[('K', 0)]
        B = K.shape[0]
        eye = torch.eye(4, device=K.device, dtype=K.dtype).expand(B, 4, 4)
        rows = []
        for c in cams:
            mats = []
            for w in range(plan.n_warp):
                if w >= len(plan.entries[c]):
                    mats.append(eye[:, :3, :])
                    continue
                fslot, src, oslot = plan.entries[c][w]
                f = self.frame_ids[fslot]
                T = outputs[('cam', c)][('cam_T_cam', 0, f)] if oslot < 0 else rel_poses[c][(f, src)]
                mats.append(torch.matmul(K[:, src], T)[:, :3, :])
            rows.append(torch.stack(mats, 1))
        return torch.stack(rows, 1)

    def _warp_index(self, plan, device):
        """Per (camera, warp) of the plan: target, source, frame slot, and kind (0 temporal,
        1 spatial at frame 0, 2 spatio-temporal, 3 padding) as device index tensors."""
        key = (plan, str(device))
        if getattr(self, '_widx_key', None) != key:
            rows = []
            for c in range(plan.N):
                for w in range(plan.n_warp):
                    if w >= len(plan.entries[c]):
                        rows.append((c, c, 0, 3))
                        continue
                    fs, src, os_ = plan.entries[c][w]
                    rows.append((c, src, fs, 0 if os_ < 0 else (1 if fs == 0 else 2)))
            t = torch.tensor(rows, dtype=torch.long, device=device)
            self._widx = (t[:, 0], t[:, 1], t[:, 2], t[:, 3])
            self._widx_key = key
        return self._widx

    def _warp_matrices_all(self, inputs, outputs):
        plan = self.plan(inputs[('K', 0)].device)
        K, E, Einv = inputs[('K', 0)], inputs['extrinsics'], inputs['extrinsics_inv']
        B, N = K.shape[:2]
        tgt, src, fslot, kind = self._warp_index(plan, K.device)
        eye = torch.eye(4, device=K.device, dtype=K.dtype)
        P_all = outputs['_cam_T_cam']
        Pst = torch.stack([eye.expand(B, N, 4, 4) if f == 0 else P_all[f] for f in self.frame_ids], 1)
        Pw = Pst[:, fslot, tgt]                                           # [B, n, 4, 4]
        R = Einv[:, src] @ E[:, tgt]                                      # rel pose (0, src)
        T = torch.where((kind == 0).view(-1, 1, 1), Pw, R @ Pw)           # R @ I == R exactly
        M = (K[:, src] @ T)[:, :, :3, :]
        M = torch.where((kind == 3).view(-1, 1, 1), eye[:3], M)
        return M.view(B, N, plan.n_warp, 3, 4)

    def _render(self, inputs, outputs, rel_poses, cam_begin, cam_count, depth_all=None):
        """Render cameras [cam_begin, +cam_count); returns {scale: (color, cmask, ovl, omask)}."""
        plan = self.plan(inputs[('K', 0)].device)
        cams = list(range(cam_begin, cam_begin + cam_count))
        colors = [inputs[('color', f, 0)] for f in self.frame_ids]
        mask = inputs['mask'][:, :, 0]
        invK = inputs[('inv_K', 0)][:, cam_begin:cam_begin + cam_count]
        packed = {}
        M = self.warp_matrices(inputs, outputs, rel_poses, cams)          # the same at every scale
        for scale in self.scales:
            if depth_all is not None and scale in depth_all:
                depth = depth_all[scale]
            else:
                depth = torch.stack([outputs[('cam', c)][('depth', scale)][:, 0] for c in cams], 1)
            color, cmask, ovl, omask = KN.ViewSynthesis.apply(plan, cam_begin, depth, invK, M, mask, *colors)
            for i, c in enumerate(cams):
                view = outputs[('cam', c)]
                for ti, f in enumerate(self.frame_ids[1:]):
                    view[('color', f, scale)] = color[:, i, ti]
                    view[('color_mask', f, scale)] = cmask[:, i, ti].unsqueeze(1)
                for fi, f in enumerate(self.frame_ids[:plan.F]):
                    view[('overlap', f, scale)] = ovl[:, i, fi]
                    view[('overlap_mask', f, scale)] = omask[:, i, fi].unsqueeze(1)
            packed[scale] = (color, cmask, ovl, omask)
        return packed

    def render_all(self, inputs, outputs, rel_poses, depth_all=None):
        """Every camera in one launch sequence; rel_poses[c] = compute_relative_cam_poses(.., c).
        depth_all: optional {scale: [B, N, H, W]} depth (avoids re-stacking the per-camera views)."""
        return self._render(inputs, outputs, rel_poses, 0, self.num_cams, depth_all)

    # ------------------------------------------------------------------ depth synthesis
    def depth_sources(self, device):
        """[N, S] source cameras of each target's augmented view: rel_cam_list[c] + [c], present
        cameras only (view_rendering.py:210-213), padded with -1."""
        key = ('_ds_tab', str(device))
        if getattr(self, '_ds_key', None) != key:
            rel = self.cfg['data']['rel_cam_list']
            lists = [[s for s in list(rel[c]) + [c] if s < self.num_cams] for c in range(self.num_cams)]
            S = max(len(x) for x in lists)
            tab = torch.full((self.num_cams, S), -1, dtype=torch.int32)
            for c, x in enumerate(lists):
                tab[c, :len(x)] = torch.tensor(x, dtype=torch.int32)
            self._ds_lists, self._ds_tab, self._ds_key = lists, tab.to(device), key
        return self._ds_lists, self._ds_tab

    def render_depth_synthesis(self, inputs, outputs, depth, aug_depth, cams=None):
        """Depth of every source camera warped into the augmented view of each target camera
        (view_rendering.py:200-241): depth, aug_depth [B, N, H, W] (scale 0) -> the packed
        (tform_depth, tform_mask) [B, N, S, H, W]; the per-camera lists go to
        outputs[('cam', c)][('tform_depth', 0)] / [('tform_depth_mask', 0)]."""
        t = self.cfg['training']
        lists, tab = self.depth_sources(depth.device)
        E, E_aug, K = inputs['extrinsics'], inputs['extrinsics_aug'], inputs[('K', 0)]
        aug_inv = inverse4x4(E_aug)
        B, N = E.shape[:2]
        S = tab.shape[1]
        eye = torch.eye(4, device=E.device, dtype=E.dtype).expand(B, 4, 4)
        Ms, zs = [], []
        for c in range(N):
            for j in range(S):
                src = lists[c][j] if j < len(lists[c]) else c
                T = aug_inv[:, c] @ E[:, src] if j < len(lists[c]) else eye
                Ms.append((K[:, src] @ inverse4x4(T))[:, :3, :])
                zs.append(T[:, 2, :])
        M = torch.stack(Ms, 1).view(B, N, S, 3, 4)
        zrow = torch.stack(zs, 1).view(B, N, S, 4)
        tform, tmask = KN.DepthSynthesis.apply(tab, t['min_depth'], t['max_depth'], aug_depth, depth,
                                               inputs['mask'][:, :, 0], inputs[('inv_K', 0)], M, zrow)
        for c in (range(N) if cams is None else cams):
            view = outputs[('cam', c)]
            view[('tform_depth', 0)] = [tform[:, c, j:j + 1] for j in range(len(lists[c]))]
            view[('tform_depth_mask', 0)] = [tmask[:, c, j:j + 1] for j in range(len(lists[c]))]
        return tform, tmask

    def forward(self, inputs, outputs, cam, rel_pose_dict):
        """Reference per-camera API (view_rendering.py:118)."""
        self._render(inputs, outputs, {cam: rel_pose_dict}, cam, 1)
        if self.aug_depth:
            N = self.num_cams
            depth = torch.stack([outputs[('cam', c)][('depth', 0)][:, 0] for c in range(N)], 1)
            aug = torch.stack([outputs[('cam', c)][('depth', 0, 'aug')][:, 0] for c in range(N)], 1)
            self.render_depth_synthesis(inputs, outputs, depth, aug, cams=[cam])

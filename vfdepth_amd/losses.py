"""Self-supervised losses on the K5 kernels (reference `/root/reference/models/losses/`).

`SingleCamLoss` / `MultiCamLoss` keep the reference's per-camera API
`loss(inputs, outputs, cam) -> (cam_loss, loss_dict)` (single_cam_loss.py:67-95,
multi_cam_loss.py:94-138).  `forward_all` evaluates every camera in one launch sequence on the
packed view-synthesis tensors and is what `VFDepthAlgo` uses.  Scalars in `loss_dict` are 0-d
device tensors (no host synchronisation); `float()` them for printing.
"""
import torch
import torch.nn as nn

from . import kernels as KN
from .rotation import matrix_to_euler_angles

IDENTITY_NOISE = 1e-5     # single_cam_loss.py:8


class SingleCamLoss(nn.Module):
    multi = False

    def __init__(self, cfg, rank):
        super().__init__()
        t, lc = cfg['training'], cfg['loss']
        self.cfg = cfg
        self.rank = rank
        self.scales = list(t['scales'])
        self.frame_ids = list(t['frame_ids'])
        self.pose_model = cfg['model']['pose_model']
        self.num_cams = int(cfg['data']['num_cams'])
        for k, v in lc.items():
            setattr(self, k, v)
        self._plan = None
        self.noise_mode = 'device'     # 'device': in-kernel counter RNG; 'cpu_global': reference RNG stream
        self.device_seed = False       # True: seed counter on the device (required under graph capture)
        self._seed = int(torch.initial_seed()) & 0xFFFFFFFF
        self._calls = 0

    # ------------------------------------------------------------------ plumbing
    def plan(self, device):
        if self._plan is None or self._plan.tab.device != torch.device(device):
            self._plan = KN.ViewPlan(self.cfg, device)
        return self._plan

    def next_seed(self, device=None):
        """Identity-noise seed of the next call: a host counter in eager mode; with a device the
        counter lives on the device and is advanced by a kernel (so a captured graph draws fresh
        noise on every replay)."""
        self._calls += 1
        if device is None:
            return (self._seed << 20) ^ self._calls
        if getattr(self, '_counter', None) is None or self._counter.device != torch.device(device):
            self._counter = torch.zeros(1, dtype=torch.int64, device=device)
        self._counter += 1
        return (self._seed << 20, self._counter)

    def draw_noise(self, B, H, W, cams, device):
        """Identity-loss noise exactly as the reference draws it: CPU global RNG, camera by camera
        (single_cam_loss.py:45-46).  Only used in noise_mode 'cpu_global'."""
        T = len(self.frame_ids) - 1
        n = [IDENTITY_NOISE * torch.randn([B, T, H, W]) for _ in cams]
        return torch.stack(n, 0).to(device)

    def _noise(self, B, H, W, cams, device, noise):
        if noise is not None:
            return noise
        if self.noise_mode == 'cpu_global':
            return self.draw_noise(B, H, W, cams, device)
        return None

    @staticmethod
    def get_logs(loss_dict, depth_all, cam0_T):
        """depth statistics (mean over cameras of per-camera stats) and camera-0 translation
        magnitudes (base_loss.py:27-43)."""
        d = depth_all.detach()
        per_cam = d.transpose(0, 1).reshape(d.shape[1], -1)
        # two-stage reductions (a camera's pixels in k rows first): ATen reduces a [6, 245760]
        # tensor with one workgroup per camera (~50 us each); max / min are exact either way, the
        # mean is the mean of k equal-sized row means
        M = per_cam.shape[1]
        k = next((c for c in (256, 128, 64, 32, 16, 8, 4, 2) if M % c == 0), 1)
        rows = per_cam.view(per_cam.shape[0], k, M // k)
        loss_dict['depth/mean'] = rows.mean(2).mean(1).mean()
        loss_dict['depth/max'] = rows.amax(2).amax(1).mean()
        loss_dict['depth/min'] = rows.amin(2).amin(1).mean()
        if cam0_T is not None:
            t = cam0_T.detach()
            loss_dict['pose/tx'] = t[:, 0, 3].abs().mean()
            loss_dict['pose/ty'] = t[:, 1, 3].abs().mean()
            loss_dict['pose/tz'] = t[:, 2, 3].abs().mean()
        return loss_dict

    def compute_pose_con_loss(self, inputs, outputs, cam):
        """fsm pose consistency (multi_cam_loss.py:61-92); torch (4x4 math)."""
        ref_ext, ref_inv = inputs['extrinsics'][:, 0], inputs['extrinsics_inv'][:, 0]
        cur_ext, cur_inv = inputs['extrinsics'][:, cam], inputs['extrinsics_inv'][:, cam]
        tl = al = 0.0
        for f in self.frame_ids[1:]:
            ref_T = outputs[('cam', 0)][('cam_T_cam', 0, f)]
            cur_T = outputs[('cam', cam)][('cam_T_cam', 0, f)]
            aligned = ref_inv @ cur_ext @ cur_T @ cur_inv @ ref_ext
            ang = torch.norm(matrix_to_euler_angles(ref_T[:, :3, :3]) - matrix_to_euler_angles(aligned[:, :3, :3]), p=2, dim=1).mean()
            tr = torch.norm(ref_T[:, :3, 3] - aligned[:, :3, 3], p=2, dim=1).mean()
            tl, al = tl + tr, al + ang
        return (tl + 10 * al) / len(self.frame_ids[1:])

    # ------------------------------------------------------------------ batched path
    def forward_all(self, inputs, outputs, packed, disp_all, depth_all, noise=None):
        """All cameras at once.  packed[scale] = ViewRendering.render_all output;
        disp_all / depth_all[scale] = [B, N, H, W].  Returns (total_loss, mean loss dict)."""
        plan = self.plan(disp_all[self.scales[0]].device)
        N = self.num_cams
        target = inputs[('color', 0, 0)]
        ref_mask = inputs['mask'][:, :, 0]
        idents = [inputs[('color', f, 0)] for f in self.frame_ids[1:]]
        cam_loss = 0.0
        logs = {}
        for scale in self.scales:
            color, _, ovl, omask = packed[scale]
            B, _, _, _, H, W = color.shape
            nz = self._noise(B, H, W, range(N), color.device, noise)
            seed = self.next_seed(color.device) if self.device_seed else self.next_seed()
            losses, reproj, automask, spatio = KN.PhotoLoss.apply(plan, 0, seed, nz, target, ref_mask,
                                                                  color, ovl, omask, *idents)
            smooth = KN.Smoothness.apply(disp_all[scale], inputs[('color', 0, scale)])
            per_cam = losses[:, 0] + self.disparity_smoothness * smooth / (2 ** scale)
            if self.multi:
                per_cam = per_cam + (self.spatio_coeff * losses[:, 1] + self.spatio_tempo_coeff * losses[:, 2])
                if self.pose_model == 'fsm':
                    pose = torch.stack([torch.zeros((), device=color.device)] +
                                       [self.compute_pose_con_loss(inputs, outputs, c) for c in range(1, N)])
                    per_cam = per_cam + self.pose_loss_coeff * pose
                    if scale == 0 and N > 1:
                        logs['pose'] = pose[1:].detach().mean()
            cam_loss = cam_loss + per_cam
            for c in range(N):
                view = outputs[('cam', c)]
                view[('reproj_loss', scale)] = reproj[:, c].unsqueeze(1)
                view[('reproj_mask', scale)] = automask[:, c].unsqueeze(1)
                if self.multi:
                    view[('overlap_mask', 0, scale)] = spatio[:, c].unsqueeze(1)
            if scale == 0:
                logs['reproj_loss'] = losses[:, 0].detach().mean()
                if self.multi:
                    logs['spatio_loss'] = losses[:, 1].detach().mean()
                    logs['spatio_tempo_loss'] = losses[:, 2].detach().mean()
                logs['smooth'] = smooth.detach().mean()
                cam0_T = outputs[('cam', 0)].get(('cam_T_cam', 0, -1))
                self.get_logs(logs, depth_all[0], cam0_T)
        cam_loss = cam_loss / len(self.scales)
        return cam_loss.sum() / N, logs

    # ------------------------------------------------------------------ per-camera reference API
    def forward(self, inputs, outputs, cam, noise=None):
        plan = self.plan(inputs[('color', 0, 0)].device)
        view = outputs[('cam', cam)]
        frames = self.frame_ids
        ref_mask = inputs['mask'][:, :, 0]
        target = inputs[('color', 0, 0)]
        idents = [inputs[('color', f, 0)] for f in frames[1:]]
        cam_loss = 0.0
        loss_dict = {}
        for scale in self.scales:
            color = torch.stack([view[('color', f, scale)] for f in frames[1:]], 1).unsqueeze(1)
            if self.multi:
                ovl = torch.stack([view[('overlap', f, scale)] for f in frames], 1).unsqueeze(1)
                omask = torch.stack([view[('overlap_mask', f, scale)][:, 0] for f in frames], 1).unsqueeze(1)
            else:
                ovl = color[:, :, :0]
                omask = color[:, :, :0, 0]
            B, _, _, _, H, W = color.shape
            nz = self._noise(B, H, W, [cam], color.device, noise)
            losses, reproj, automask, spatio = KN.PhotoLoss.apply(plan, cam, self.next_seed(), nz, target, ref_mask,
                                                                  color, ovl, omask, *idents)
            disp = view[('disp', scale)][:, 0].unsqueeze(1)
            smooth = KN.Smoothness.apply(disp, inputs[('color', 0, scale)][:, cam].unsqueeze(1))[0]
            l_rep, l_sp, l_st = losses[0, 0], losses[0, 1], losses[0, 2]
            cam_loss = cam_loss + l_rep
            cam_loss = cam_loss + self.disparity_smoothness * smooth / (2 ** scale)
            pose = 0.0
            if self.multi:
                cam_loss = cam_loss + (self.spatio_coeff * l_sp + self.spatio_tempo_coeff * l_st)
                if self.pose_model == 'fsm' and cam != 0:
                    pose = self.compute_pose_con_loss(inputs, outputs, cam)
                cam_loss = cam_loss + self.pose_loss_coeff * pose
            view[('reproj_loss', scale)] = reproj[:, 0].unsqueeze(1)
            view[('reproj_mask', scale)] = automask[:, 0].unsqueeze(1)
            if self.multi:
                view[('overlap_mask', 0, scale)] = spatio[:, 0].unsqueeze(1)
            if scale == 0:
                loss_dict['reproj_loss'] = l_rep.detach()
                if self.multi:
                    loss_dict['spatio_loss'] = l_sp.detach()
                    loss_dict['spatio_tempo_loss'] = l_st.detach()
                    if self.pose_model == 'fsm' and cam != 0:
                        loss_dict['pose'] = pose.detach()
                loss_dict['smooth'] = smooth.detach()
                depth = view[('depth', 0)]
                self.get_logs(loss_dict, depth.unsqueeze(1)[:, :, 0] if depth.dim() == 4 else depth,
                              view.get(('cam_T_cam', 0, -1)) if cam == 0 else None)
        return cam_loss / len(self.scales), loss_dict


class MultiCamLoss(SingleCamLoss):
    """Spatial + spatio-temporal terms on top of the temporal loss (multi_cam_loss.py:9-138)."""
    multi = True


class DepthSynLoss(MultiCamLoss):
    """MultiCamLoss + the depth-synthesis terms (depth_synthesis_loss.py:8-91): consistency between
    each camera's augmented-view depth and the source depths warped into that view,
    clamp(|a - t| / (a + t + 1e-8), 0, 1) as one masked mean over all sources, and plain-gradient
    smoothness of disp_aug / mean; weighted by depth_con_coeff / depth_sm_coeff."""

    def __init__(self, cfg, rank):
        super().__init__(cfg, rank)
        if list(self.scales) != [0]:
            # the reference adds the depth-synthesis terms of every scale before dividing by the
            # scale count (depth_synthesis_loss.py:66-89); this build renders the augmented view
            # at scale 0 only (every shipped config uses scales [0]), so refuse rather than
            # silently weight the terms differently
            raise NotImplementedError(f'aug_depth supports scales [0] only, got {list(self.scales)}')

    @staticmethod
    def syn_terms(aug_depth, tform, tmask, disp_aug):
        """aug_depth, disp_aug [B, N, H, W]; tform, tmask [B, N, S, H, W] -> (con [N], sm [N])."""
        a = aug_depth.unsqueeze(2)
        pl = torch.clamp((a - tform).abs() / (a + tform + 1e-8), 0., 1.)
        con = (pl * tmask).sum((0, 2, 3, 4)) / (tmask.sum((0, 2, 3, 4)) + 1e-8)
        nd = disp_aug / (disp_aug.mean((2, 3), keepdim=True) + 1e-8)
        sm = (nd[..., :-1] - nd[..., 1:]).abs().mean((0, 2, 3)) + (nd[..., :-1, :] - nd[..., 1:, :]).abs().mean((0, 2, 3))
        return con, sm

    def forward_all(self, inputs, outputs, packed, disp_all, depth_all, noise=None):
        total, logs = super().forward_all(inputs, outputs, packed, disp_all, depth_all, noise)
        tform, tmask = outputs['_tform']
        con, sm = self.syn_terms(outputs['_depth_aug_all'][0], tform, tmask, outputs['_disp_aug_all'][0])
        syn = self.depth_con_coeff * con + self.depth_sm_coeff * sm
        total = total + syn.sum() / self.num_cams
        logs['depth_loss'] = syn.detach().mean()
        logs['depth_sm_loss'] = sm.detach().mean()
        logs['depth_con_loss'] = con.detach().mean()
        logs['cam_loss'] = total.detach()
        return total, logs

    def forward(self, inputs, outputs, cam, noise=None):
        cam_loss, loss_dict = super().forward(inputs, outputs, cam, noise)
        view = outputs[('cam', cam)]
        aug = view[('depth', 0, 'aug')]
        tform = torch.stack(view[('tform_depth', 0)], 1)[:, :, 0].unsqueeze(1)
        tmask = torch.stack(view[('tform_depth_mask', 0)], 1)[:, :, 0].unsqueeze(1)
        con, sm = self.syn_terms(aug, tform, tmask, view[('disp', 0, 'aug')])
        syn = self.depth_con_coeff * con[0] + self.depth_sm_coeff * sm[0]
        cam_loss = cam_loss + syn / len(self.scales)
        loss_dict.update({'depth_loss': syn.detach(), 'depth_sm_loss': sm[0].detach(),
                          'depth_con_loss': con[0].detach(), 'cam_loss': cam_loss.detach()})
        return cam_loss, loss_dict


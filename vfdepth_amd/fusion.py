"""`VFNet` — surround-view volumetric fusion on the gfx950 kernels.

Drop-in for `/root/reference/network/volumetric_fusionnet.py:11-343`: same constructor
(`VFNet(cfg, feat_in_dim, feat_out_dim, model='depth'|'pose')`), same parameters and
state-dict keys (`conv_overlap.0.*`, `conv_non_overlap.0.*`, `reduce_dim.{0,3}.*`), same
`forward(inputs, feats_agg)` contract (depth: dict with 'proj_feat' [B*N, out, h, w];
pose: BEV feature map).  What changes is how it is computed:

* depth mode: the 1x1 convs' feature columns are folded into the per-camera maps by one
  batched GEMM (W·bilinear(F) = bilinear(W·F)), K1 gathers 64 folded channels per valid
  (voxel, camera) pair and applies depth column, bias, LeakyReLU and the count masks in
  registers — no [B,6,257,V] intermediates;
* K3 resamples the voxel grid on all camera frustums in one launch and writes the
  reflect-padded, channels-last (NHWC) layout `reduce_dim`'s first conv reads (no F.pad pass,
  no layout transposes); the six cameras' `reduce_dim` runs as one batched NHWC conv;
* pose mode: K2 writes the camera-mean voxel features straight into the reflect-padded NHWC
  [B, Y+2, X+2, Z(C+1)] map of the stride-2 conv.
The two kernels order their channels voxel-row-major (z*(C+1)+c, d*Cv+c) so that every gather
and store is a contiguous row; `_reduce` permutes the conv weight's input channels to match,
which leaves the convolution (and the parameters / state dict) exactly the reference's.
"""
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels as KN
from .layers import conv1d_block, conv2d_block, pack_cam_feat
from .rotation import axis_angle_to_matrix


class _GeometryCache:
    """Step-scoped products (1/8 mask, K2 fusion plan, K2C weight copy) shared by the three VFNet calls
    of a step (two pose calls, one depth call).

    Keyed on the IDENTITY and version of the input tensors they derive from, not on the
    `inputs` dict: DDP re-packs a module's positional inputs into a fresh dict every call
    (`torch.distributed.utils._recursive_to`), so anything cached inside `inputs` would be lost
    and rebuilt per call.  One entry per tag holds strong references to its key tensors (their
    addresses cannot be reused while cached); the next step's tensors replace it."""

    def __init__(self):
        self.entries = {}

    def get(self, tag, tensors, build):
        e = self.entries.get(tag)
        vers = tuple(t._version for t in tensors)
        if e is not None and len(e[0]) == len(tensors) and all(a is b for a, b in zip(e[0], tensors)) \
                and e[1] == vers:
            return e[2]
        self.entries.pop(tag, None)
        val = build()
        self.entries[tag] = (tuple(tensors), vers, val)
        return val

    def clear(self):
        self.entries.clear()


_GEOMETRY_CACHE = _GeometryCache()


def begin_step():
    """Drop the previous step's geometry products (VFDepthAlgo.process_batch calls this first, so
    every step builds its own 1/8 mask and fusion plan even when a batch tensor is reused)."""
    _GEOMETRY_CACHE.clear()


class VFNet(nn.Module):
    def __init__(self, cfg, feat_in_dim, feat_out_dim, model='depth'):
        super().__init__()
        self.cfg = cfg
        m, t = cfg['model'], cfg['training']
        self.model = model
        self.num_cams = int(cfg['data']['num_cams'])
        self.fusion_level = int(m['fusion_level'])
        self.feat_in_dim = int(feat_in_dim)
        self.voxel_size = [int(v) for v in m['voxel_size']]
        self.proj_d_bins = int(m['proj_d_bins'])
        self.aug_depth = bool(t.get('aug_depth', False))
        self.aug_angle = [float(v) for v in t.get('aug_angle', [15, 15, 40])]
        self.syn_visualize = bool(cfg.get('eval', {}).get('syn_visualize', False))
        x_dim, y_dim, z_dim = self.voxel_size
        self.z_dim, self.y_dim, self.x_dim = z_dim, y_dim, x_dim
        self.n_voxels = x_dim * y_dim * z_dim
        if model == 'depth':
            pre = list(m['voxel_pre_dim'])
            self.v_dim_o = [(feat_in_dim + 1) * 2] + pre
            self.v_dim_no = [feat_in_dim + 1] + pre
            self.conv_overlap = conv1d_block(self.v_dim_o[0], self.v_dim_o[1], kernel_size=1)
            self.conv_non_overlap = conv1d_block(self.v_dim_no[0], self.v_dim_no[1], kernel_size=1)
            enc_dims, stride = self.proj_d_bins * self.v_dim_o[-1], 1
            if KN.overlap_group_table(self.num_cams) is None:
                raise NotImplementedError(f'overlap fusion needs 3 or 6 cameras, got {self.num_cams}')
        else:
            enc_dims, stride = (feat_in_dim + 1) * z_dim, 2
            if feat_in_dim % 4 or not 0 < feat_in_dim <= 256:
                # K2's backward moves channel quads (fusion.hip, vfd_fuse_pose_bwd): refuse at
                # construction instead of failing mid-step
                raise ValueError(f'pose fusion needs fusion_feat_in_dim % 4 == 0 and <= 256, got {feat_in_dim}')
        self.stride = stride
        self.reduce_dim = nn.Sequential(*conv2d_block(enc_dims, 256, kernel_size=3, stride=stride).children(),
                                        *conv2d_block(256, feat_out_dim, kernel_size=3, stride=stride).children())
        self._space = None

    # ------------------------------------------------------------------ helpers
    def space(self, device):
        if self._space is None or self._space.device != torch.device(device):
            self._space = KN.VoxelSpace(self.cfg, device)
        return self._space

    def _mask_lowres(self, inputs, space):
        return _GEOMETRY_CACHE.get(('mask_lo', space.h, space.w), (inputs['mask'],),
                                   lambda: KN.mask_lowres(space, inputs['mask']))

    def _plan(self, inputs, space):
        K, Einv = inputs['K', self.fusion_level + 1], inputs['extrinsics_inv']
        mask_lo = self._mask_lowres(inputs, space)
        # buffers built by the first forward that needs a gradient (FusePose), shared by both
        # pose calls of the step
        return _GEOMETRY_CACHE.get(('plan', space.h, space.w, tuple(self.voxel_size)), (mask_lo, K, Einv),
                                   lambda: KN.FusionPlan(space, mask_lo, K, Einv, build=False))

    def _reduce(self, x_padded):
        """reduce_dim with the first conv reading the kernel's channels-last, reflect-padded output
        (padding 0; its weight's input channels permuted to the kernel's channel order).  Both
        convs run channels-last (MIOpen NHWC implicit GEMM, no layout transposes); the result is
        handed on in the usual contiguous NCHW layout."""
        c0, c1 = self.reduce_dim[0], self.reduce_dim[3]
        if self.model == 'depth':
            w0 = KN.proj_conv_weight(c0.weight, self.v_dim_o[-1], self.proj_d_bins)
        else:
            C1, Z = self.feat_in_dim + 1, self.z_dim
            if self.pad_conv_bf16(x_padded):
                # K2C's bf16 form under config 3's autocast (padconv.hip ppcb_main_k); fragments from
                # the fp32 mode-0 copy, shared by the step's pose calls
                wf = _GEOMETRY_CACHE.get(('pose_wf_bf16', id(c0.weight)), (c0.weight,),
                                         lambda: KN.pad_conv_weight_fragments_bf16(c0.weight.detach(), C1, Z))
                y0 = KN.PadConvBF16.apply(x_padded, c0.weight, c0.bias, self.stride, wf, (C1, Z))
                return F.leaky_relu(F.conv2d(y0, c1.weight, c1.bias, stride=self.stride), 0.1,
                                    inplace=True).contiguous()
            if self.pad_conv(x_padded):
                # K2C: the first conv on MFMA (padconv.hip), written reflect-padded for the second;
                # it takes the weight in the reference channel order (relayouts in weights.hip);
                # the fragment copy is shared by the step's pose calls (same version)
                wf = _GEOMETRY_CACHE.get(('pose_wf', id(c0.weight)), (c0.weight,),
                                         lambda: KN.pose_conv_fragments(c0.weight, C1, Z))
                y0 = KN.PadConv.apply(x_padded, c0.weight, c0.bias, self.stride, wf, (C1, Z))
                return F.leaky_relu(F.conv2d(y0, c1.weight, c1.bias, stride=self.stride), 0.1,
                                    inplace=True).contiguous()
            w0 = KN.pose_conv_weight(c0.weight, C1, Z)
        x = F.leaky_relu(F.conv2d(x_padded, w0, c0.bias, stride=self.stride), 0.1, inplace=True)
        return F.leaky_relu(c1(x), 0.1, inplace=True).contiguous()

    def pad_conv_bf16(self, x_padded):
        """K2C's bf16 form applies: 256 outputs, bf16 autocast (config 3), a supported shape, not
        disabled by VFD_PAD_CONV=0 / VFD_PAD_CONV_BF16=0."""
        return (os.environ.get('VFD_PAD_CONV', '1') != '0' and os.environ.get('VFD_PAD_CONV_BF16', '1') != '0'
                and self.reduce_dim[0].out_channels == 256 and torch.is_autocast_enabled('cuda')
                and torch.get_autocast_dtype('cuda') == torch.bfloat16
                and KN.pad_conv_bf16_supported(x_padded, self.stride, 256))

    def pad_conv(self, x_padded):
        """K2C (the pose reduce_dim's first conv as an fp32 MFMA kernel) applies: 256 outputs, fp32
        nets (under bf16 autocast MIOpen's bf16 path runs instead), a supported shape, not
        disabled by VFD_PAD_CONV=0."""
        return (os.environ.get('VFD_PAD_CONV', '1') != '0' and self.reduce_dim[0].out_channels == 256
                and not torch.is_autocast_enabled('cuda') and x_padded.dtype == torch.float32
                and KN.pad_conv_supported(x_padded, self.stride, 256))

    def folded_weights(self):
        """Per-camera [N, 2Cv, C] feature columns of (W_no, W_o[group]) and the [3, Cv] depth columns."""
        C = self.feat_in_dim
        groups = KN.overlap_group_table(self.num_cams)
        w_no, w_o = self.conv_non_overlap[0].weight, self.conv_overlap[0].weight
        if w_no.is_cuda and os.environ.get('VFD_FOLD_WEIGHTS', '1') != '0':
            return KN.FoldWeights.apply(w_no, w_o, groups)
        w_no, w_o = w_no[:, :, 0], w_o[:, :, 0]
        halves = [w_o[:, :C], w_o[:, C + 1:2 * C + 1]]
        wf = torch.stack([torch.cat([w_no[:, :C], halves[g]], 0) for g in groups], 0)
        wz = torch.stack([w_no[:, C], w_o[:, C], w_o[:, 2 * C + 1]], 0)
        return wf, wz

    # ------------------------------------------------------------------ forward
    def backproject_depth(self, inputs, feats_agg):
        """K1: [B,N,C,h,w] -> voxel features [B, V, Cv] (channels-last)."""
        space = self.space(feats_agg.device)
        B, N, C, h, w = feats_agg.shape
        wf, wz = self.folded_weights()
        # the fold is part of K1's algebra (it replaces the reference's fp32 1x1 convs after the
        # gather): fp32 even when the dense nets run under bf16 autocast (config 3)
        with torch.autocast(device_type='cuda', enabled=False):
            P = torch.einsum('bncp,nkc->bnpk', feats_agg.float().reshape(B, N, C, h * w), wf.float()).contiguous()
        K = inputs['K', self.fusion_level + 1]
        # the step's fusion plan (shared with the pose calls) indexes K1's atomic-free backward
        return KN.FuseDepth.apply(space, P, self._mask_lowres(inputs, space), K, inputs['extrinsics_inv'],
                                  wz, self.conv_non_overlap[0].bias, self.conv_overlap[0].bias,
                                  self._plan(inputs, space))

    def fused_projection(self, voxel_feat):
        """K3C (K3 fused into reduce_dim's first conv, fp32 MFMA) applies: 64 voxel channels, 256
        conv outputs, <= 64 depth bins, fp32 nets (under bf16 autocast the conv runs on MIOpen's
        bf16 path instead), not disabled by VFD_PROJ_CONV=0."""
        c0 = self.reduce_dim[0]
        return (os.environ.get('VFD_PROJ_CONV', '1') != '0' and voxel_feat.shape[-1] == 64
                and c0.out_channels == 256 and self.proj_d_bins <= 64
                and not torch.is_autocast_enabled('cuda'))

    def fused_projection_bf16(self, voxel_feat):
        """K3C's bf16 form applies: as fused_projection, under bf16 autocast (config 3), not
        disabled by VFD_PROJ_CONV_BF16=0."""
        c0 = self.reduce_dim[0]
        return (os.environ.get('VFD_PROJ_CONV', '1') != '0' and os.environ.get('VFD_PROJ_CONV_BF16', '1') != '0'
                and voxel_feat.shape[-1] == 64 and c0.out_channels == 256 and self.proj_d_bins <= 64
                and torch.is_autocast_enabled('cuda') and torch.get_autocast_dtype('cuda') == torch.bfloat16)

    def project_voxel_into_image(self, voxel_feat, inv_K, extrinsics):
        """K3 + reduce_dim: voxel features [B,V,Cv] -> [B*N, feat_out, h, w]."""
        space = self.space(voxel_feat.device)
        if self.fused_projection(voxel_feat) or self.fused_projection_bf16(voxel_feat):
            c0, c1 = self.reduce_dim[0], self.reduce_dim[3]
            fn = KN.ProjConv if self.fused_projection(voxel_feat) else KN.ProjConvBF16
            y0 = fn.apply(space, voxel_feat.float(), inv_K, extrinsics, c0.weight, c0.bias)
            return F.leaky_relu(F.conv2d(y0, c1.weight, c1.bias), 0.1, inplace=True).contiguous()
        return self._reduce(KN.VoxelProject.apply(space, voxel_feat, inv_K, extrinsics))

    def augment_extrinsics(self, ext):
        """Random rotation in front of every camera (volumetric_fusionnet.py:269-287): the angles
        are the reference's `torch.rand(b, cam, 3)` draw on the CPU global generator, scaled by
        `aug_angle` (used as radians, as the reference does); no gradient.  Under HIP-graph
        capture the draw is on the device generator instead (a CPU draw and its host->device copy
        would be frozen into the graph: every replay would reuse the capture step's rotation)."""
        with torch.no_grad():
            b, cam = ext.shape[:2]
            capturing = ext.is_cuda and torch.cuda.is_current_stream_capturing()
            angle = torch.rand(b, cam, 3, device=ext.device if capturing else 'cpu')
            for i in range(3):
                angle[:, :, i] = (angle[:, :, i] - 0.5) * self.aug_angle[i]
            tform = torch.eye(4, device=angle.device).repeat(b, cam, 1, 1)
            tform[:, :, :3, :3] = axis_angle_to_matrix(angle)
            return tform.to(device=ext.device, dtype=ext.dtype) @ ext

    def forward(self, inputs, feats_agg):
        if self.syn_visualize:
            raise NotImplementedError('synthesis visualisation (eval.syn_visualize) is out of scope of this build')
        space = self.space(feats_agg.device)
        fusion_dict = {('cam', c): {} for c in range(self.num_cams)}
        if self.model == 'depth':
            vox = self.backproject_depth(inputs, feats_agg)
            inv_K = inputs['inv_K', self.fusion_level + 1]
            fusion_dict['proj_feat'] = self.project_voxel_into_image(vox, inv_K, inputs['extrinsics'])
            if self.aug_depth:
                # depth synthesis at a novel view (volumetric_fusionnet.py:313-317); the augmented
                # extrinsics also travel in the returned dict (DDP re-packs `inputs` per call)
                ext_aug = self.augment_extrinsics(inputs['extrinsics'])
                inputs['extrinsics_aug'] = fusion_dict['extrinsics_aug'] = ext_aug
                fusion_dict['proj_feat_aug'] = self.project_voxel_into_image(vox, inv_K, ext_aug)
            return fusion_dict
        if self.pose_conv_bf16(space, feats_agg):
            # config 3: K2 writes the map in bf16 for the bf16 K2C, one autograd node (kernels.py)
            c0, c1 = self.reduce_dim[0], self.reduce_dim[3]
            C1, Z = self.feat_in_dim + 1, self.z_dim
            wf = _GEOMETRY_CACHE.get(('pose_wf_bf16', id(c0.weight)), (c0.weight,),
                                     lambda: KN.pad_conv_weight_fragments_bf16(c0.weight.detach(), C1, Z))
            y0 = KN.PoseConvBF16.apply(space, self._plan(inputs, space), feats_agg, c0.weight, c0.bias,
                                       self.stride, wf, (C1, Z))
            return F.leaky_relu(F.conv2d(y0, c1.weight, c1.bias, stride=self.stride), 0.1,
                                inplace=True).contiguous()
        vox = KN.FusePose.apply(space, self._plan(inputs, space), feats_agg)
        return self._reduce(vox)

    def pose_conv_bf16(self, space, feats_agg):
        """K2 + K2C on the bf16 map (PoseConvBF16) applies: K2C's bf16 form would run (bf16
        autocast, 256 outputs), its three kernels accept the map, not disabled by
        VFD_POSE_BF16_MAP=0 (or VFD_PAD_CONV / VFD_PAD_CONV_BF16 = 0)."""
        return (os.environ.get('VFD_POSE_BF16_MAP', '1') != '0' and os.environ.get('VFD_PAD_CONV', '1') != '0'
                and os.environ.get('VFD_PAD_CONV_BF16', '1') != '0' and self.reduce_dim[0].out_channels == 256
                and torch.is_autocast_enabled('cuda') and torch.get_autocast_dtype('cuda') == torch.bfloat16
                and KN.pose_conv_bf16_supported(space, feats_agg.shape[0], feats_agg.shape[2], self.stride, 256))


__all__ = ['VFNet', 'pack_cam_feat']

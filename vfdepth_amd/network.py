"""Depth / pose networks around VFNet (dense layers on MIOpen, fusion on the HIP kernels).

Mirrors `/root/reference/network/{fusion_depthnet,fusion_posenet,mono_depthnet,mono_posenet}.py`
module-for-module (attribute names and state-dict keys included) so reference checkpoints load.
"""
import os
from collections import OrderedDict

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels as KN
from .fusion import VFNet
from .layers import (MonoDepthDecoder, PoseDecoder, ResnetEncoder, conv2d_block, pack_cam_feat,
                     unpack_cam_feat, upsample)


# channels-last encoders: training.channels_last when set, else VFD_CHANNELS_LAST — 'auto' (default):
# the bf16 nets always, the fp32 nets when MIOpen picks its algorithms by measured time
# (torch.backends.cudnn.benchmark at construction); 'all': always, '1': the bf16 nets only, '0':
# never.  With the find-db tuned for the NHWC fp32 shapes (miopen_db/, round 5) MIOpen's
# channels-last fp32 convolutions in benchmark mode beat its NCHW Winograd + transposed implicit
# GEMMs at config 2 (33.2 vs 34.3 ms/step; NCHW immediate mode 35.5), but its immediate-mode picks
# for them do not (37.1, profiles/r5/ab/); round 3's NCHW-wins result ran them untuned
_CL_ENV = os.environ.get('VFD_CHANNELS_LAST', 'auto')


def _use_channels_last(training, bf16):
    cl = training.get('channels_last')
    if cl is None:
        cl = (_CL_ENV == 'all' or (bf16 and _CL_ENV != '0')
              or (_CL_ENV == 'auto' and bool(torch.backends.cudnn.benchmark)))
    return bool(cl)


def _encoder_input(frames, pairs=None):
    """cat(frames, channels) of [B, N, 3, H, W] batches, packed to [B*N, ...]: the fused nets' encoder
    input.  On the GPU (fp32, no gradient, H*W % 4 == 0) it comes normalised from one HIP pass
    (`kernels.normalize_cat`, bit-identical to cat + (x - 0.45) / 0.225); returns (x, normalized).
    pairs: a list of frame lists, stacked along the batch ([P*B*N, ...], pair-major)."""
    groups = pairs if pairs is not None else [frames]
    fs = [[pack_cam_feat(t) for t in fr] for fr in groups]
    if (all(len(f) <= 2 for f in fs) and all(t.is_cuda and t.dtype == torch.float32 and not t.requires_grad
                                             for f in fs for t in f)
            and (fs[0][0].shape[-1] * fs[0][0].shape[-2]) % 4 == 0 and os.environ.get('VFD_NORM_CAT', '1') != '0'):
        if len(fs) == 1:
            return KN.normalize_cat(*fs[0]), True
        n, _, h, w = fs[0][0].shape
        out = torch.empty(len(fs) * n, sum(t.shape[1] for t in fs[0]), h, w, device=fs[0][0].device)
        for p, f in enumerate(fs):
            KN.normalize_cat(*f, out=out[p * n:(p + 1) * n])
        return out, True
    cat = [torch.cat(f, 1) if len(f) > 1 else f[0] for f in fs]
    return (torch.cat(cat, 0) if len(cat) > 1 else cat[0]), False


def _aggregate(encoder, conv1x1, images, lvl, B, N, normalized=False, groups=1):
    """Encoder pyramid -> fusion-level aggregate [B,N,C,h,w] (fusion_depthnet.py:53-65,
    fusion_posenet.py:55-67): LReLU(conv1x1(cat(f_lvl, up(f_lvl+1), ...))) evaluated as
    LReLU(W_lvl f_lvl + sum up(W_k f_k) + b) — each slice of the 1x1 conv at its own resolution,
    one fused upsample-add-bias-LReLU kernel (same parameters, same result up to fp32 rounding)."""
    feats = encoder(images, normalized, groups)
    conv = conv1x1[0]
    if images.is_cuda and os.environ.get('VFD_LEVEL_CONV', '1') != '0':
        parts = KN.LevelConv1x1.apply(conv.weight, *feats[lvl:])
    else:
        off, parts = 0, []
        for f in feats[lvl:]:
            c = f.shape[1]
            parts.append(F.conv2d(f, conv.weight[:, off:off + c]))
            off += c
    agg = KN.AggregateUp.apply(parts[0], conv.bias, *parts[1:])
    return feats, unpack_cam_feat(agg, B, N)


def net_autocast(module, x):
    """bf16 autocast around a fusion net's body when `net_precision == 'bf16'` (config 3): the
    MIOpen convs run in bf16, the HIP ops cast their inputs back to fp32
    (`custom_fwd(cast_inputs=float32)`), and the nets return fp32 disparities / poses, so the
    geometry and losses always run in fp32."""
    return torch.autocast(device_type='cuda', dtype=torch.bfloat16, enabled=module.bf16 and x.is_cuda)


class FusionDepthDecoder(nn.Module):
    """Decoder from the fusion level up to full resolution (fusion_depthnet.py:97-145)."""

    def __init__(self, level_in, num_ch_enc, num_ch_dec, scales=range(2), use_skips=False):
        super().__init__()
        self.num_output_channels = 1
        self.scales = scales
        self.use_skips = use_skips
        self.level_in = level_in
        self.num_ch_enc = num_ch_enc
        self.num_ch_dec = num_ch_dec
        self.convs = OrderedDict()
        for i in range(level_in, -1, -1):
            cin = num_ch_enc[-1] if i == level_in else num_ch_dec[i + 1]
            self.convs[('upconv', i, 0)] = conv2d_block(int(cin), num_ch_dec[i], kernel_size=3, nonlin='ELU')
            cin = num_ch_dec[i] + (num_ch_enc[i - 1] if (use_skips and i > 0) else 0)
            self.convs[('upconv', i, 1)] = conv2d_block(int(cin), num_ch_dec[i], kernel_size=3, nonlin='ELU')
        for s in scales:
            self.convs[('dispconv', s)] = conv2d_block(num_ch_dec[s], self.num_output_channels, 3, nonlin=None)
        self.decoder = nn.ModuleList(list(self.convs.values()))
        self.sigmoid = nn.Sigmoid()

    def _fused_ok(self, x):
        """The HIP chain applies: GPU maps (fp32, or bf16 under config 3's bf16 autocast), no skip
        concatenation, and the blocks are the stock (reflect conv 3x3, Identity, ELU(1.0)) —
        VFD_ELU_PAD=0 disables it."""
        from .layers import _fused_dtype_ok
        if not (x.is_cuda and _fused_dtype_ok(x) and not self.use_skips and os.environ.get('VFD_ELU_PAD', '1') != '0'):
            return False
        for k, blk in self.convs.items():
            conv, norm, act = blk
            if not (isinstance(norm, nn.Identity) and conv.padding_mode == 'reflect' and conv.kernel_size == (3, 3)
                    and conv.stride == (1, 1) and conv.padding == (1, 1) and conv.dilation == (1, 1)
                    and conv.groups == 1):
                return False
            if k[0] == 'upconv' and not (isinstance(act, nn.ELU) and act.alpha == 1.0):
                return False
            if k[0] == 'dispconv' and not isinstance(act, nn.Identity):
                return False
        return True

    def _forward_fused(self, input_features):
        """The same decoder with each block's ELU, the nearest upsample and the next conv's reflect
        pad done by one HIP kernel (`KN.EluUpPad`): every conv reads a padded map that the
        previous block's kernel wrote (padding 0), the ELU / upsample / pad intermediates never
        exist."""
        out = {}
        x = input_features[-1]
        if KN.decoder_channels_last(x):
            x = x.contiguous(memory_format=torch.channels_last)
        xp = KN.ReflectPad1.apply(x)
        for i in range(self.level_in, -1, -1):
            c0 = self.convs[('upconv', i, 0)][0]
            xp = KN.ConvEluUpPad.apply(xp, c0.weight, c0.bias, True)
            c1 = self.convs[('upconv', i, 1)][0]
            xp = KN.ConvEluUpPad.apply(xp, c1.weight, c1.bias, False)
            if i in self.scales:
                cd = self.convs[('dispconv', i)][0]
                if KN.DispConvSigmoid.supported(xp, cd.weight) and cd.bias is not None:
                    out[('disp', i)] = KN.DispConvSigmoid.apply(xp, cd.weight, cd.bias)
                else:
                    out[('disp', i)] = self.sigmoid(F.conv2d(xp, cd.weight, cd.bias))
        return out

    def forward(self, input_features):
        if self._fused_ok(input_features[-1]):
            return self._forward_fused(input_features)
        out = {}
        x = input_features[-1]
        for i in range(self.level_in, -1, -1):
            x = upsample(self.convs[('upconv', i, 0)](x))
            if self.use_skips and i > 0:
                x = torch.cat([x, input_features[i - 1]], 1)
            x = self.convs[('upconv', i, 1)](x)
            if i in self.scales:
                out[('disp', i)] = self.sigmoid(self.convs[('dispconv', i)](x))
        return out


class FusedDepthNet(nn.Module):
    """ResNet encoder -> 1/8 aggregation -> VFNet(depth) -> decoder (fusion_depthnet.py:12-94)."""

    def __init__(self, cfg):
        super().__init__()
        m, t = cfg['model'], cfg['training']
        self.num_cams = int(cfg['data']['num_cams'])
        self.fusion_level = lvl = int(m['fusion_level'])
        self.scales = list(t['scales'])
        self.encoder = ResnetEncoder(int(m['num_layers']), bool(m['weights_init']), 1)
        del self.encoder.encoder.fc
        enc_dim = int(sum(self.encoder.num_ch_enc[lvl:]))
        self.conv1x1 = conv2d_block(enc_dim, int(m['fusion_feat_in_dim']), kernel_size=1, padding_mode='reflect')
        out_dim = int(self.encoder.num_ch_enc[lvl])
        self.fusion_net = VFNet(cfg, int(m['fusion_feat_in_dim']), out_dim, model='depth')
        self.decoder = FusionDepthDecoder(lvl, self.encoder.num_ch_enc[:lvl + 1], [16, 32, 64, 128, 256],
                                          self.scales, use_skips=bool(m['use_skips']))
        self.bf16 = t.get('net_precision', 'fp32') == 'bf16'
        if _use_channels_last(t, self.bf16):
            self.encoder.use_channels_last()

    def forward(self, inputs):
        outputs = {('cam', c): {} for c in range(self.num_cams)}
        imgs = inputs[('color_aug', 0, 0)]
        B, N = imgs.shape[:2]
        with net_autocast(self, imgs):
            x, normed = _encoder_input([imgs])          # fp32, normalised (the stem conv casts under autocast)
            feats, agg = _aggregate(self.encoder, self.conv1x1, x, self.fusion_level, B, N, normed)
            fusion = self.fusion_net(inputs, agg)
            disp = self.decoder(feats[:self.fusion_level] + [fusion['proj_feat']])
            # depth synthesis: a second decoder pass on the augmented view (fusion_depthnet.py:79-86)
            disp_aug = (self.decoder(feats[:self.fusion_level] + [fusion['proj_feat_aug']])
                        if 'proj_feat_aug' in fusion else None)
        for tag, dd, suffix in (('_packed', disp, ()), ('_packed_aug', disp_aug, ('aug',))):
            if dd is None:
                continue
            dd = {k: v.float() for k, v in dd.items()}
            for k, v in dd.items():
                v = v.view(B, N, *v.shape[1:])
                for c in range(N):
                    outputs[('cam', c)][k + suffix] = v[:, c]
            outputs[tag] = dd
        if 'extrinsics_aug' in fusion:
            outputs['_extrinsics_aug'] = fusion['extrinsics_aug']
        return outputs


class FusedPoseNet(nn.Module):
    """Canonical motion from the fused BEV volume (fusion_posenet.py:10-72)."""

    def __init__(self, cfg):
        super().__init__()
        m = cfg['model']
        self.num_cams = int(cfg['data']['num_cams'])
        self.fusion_level = lvl = int(m['fusion_level'])
        self.encoder = ResnetEncoder(int(m['num_layers']), bool(m['weights_init']), 2)
        del self.encoder.encoder.fc
        enc_dim = int(sum(self.encoder.num_ch_enc[lvl:]))
        self.conv1x1 = conv2d_block(enc_dim, int(m['fusion_feat_in_dim']), kernel_size=1, padding_mode='reflect')
        out_dim = int(self.encoder.num_ch_enc[lvl])
        self.fusion_net = VFNet(cfg, int(m['fusion_feat_in_dim']), out_dim, model='pose')
        self.pose_decoder = PoseDecoder(num_ch_enc=[out_dim], num_input_features=1,
                                        num_frames_to_predict_for=1, stride=2)
        self.bf16 = cfg['training'].get('net_precision', 'fp32') == 'bf16'
        if _use_channels_last(cfg['training'], self.bf16):
            self.encoder.use_channels_last()

    def forward(self, inputs, frame_ids, _cam=None):
        """frame_ids: one pair [f0, f1] -> (axis_angle, translation), the reference's call; or a list
        of pairs -> one (axis_angle, translation) per pair, computed as ONE batch: the pairs are
        stacked along the batch (pair-major), every encoder BatchNorm normalises each pair's part on
        its own (`layers.bn_groups`: the statistics, running-statistics updates and parameter
        gradients of one call per pair), K2 fuses each pair with the step's geometry, and the
        convolutions / K2C / decoder run once on the stacked batch."""
        batched = isinstance(frame_ids[0], (list, tuple))
        pairs = [list(p) for p in frame_ids] if batched else [list(frame_ids)]
        P = len(pairs)
        frames = [[inputs[('color_aug', f, 0)] for f in p] for p in pairs]
        B, N = frames[0][0].shape[:2]
        with net_autocast(self, frames[0][0]):
            x, normed = _encoder_input(None, frames)
            _, agg = _aggregate(self.encoder, self.conv1x1, x, self.fusion_level, P * B, N, normed, groups=P)
            bev = self.fusion_net(inputs, agg)
            axis_angle, translation = self.pose_decoder([[bev]])
        axis_angle, translation = axis_angle.float(), torch.clamp(translation.float(), -4.0, 4.0)
        if not batched:
            return axis_angle, translation
        return [(axis_angle[p * B:(p + 1) * B], translation[p * B:(p + 1) * B]) for p in range(P)]


class MonoDepthNet(nn.Module):
    """fsm baseline depth net (mono_depthnet.py:7-25)."""

    def __init__(self, cfg):
        super().__init__()
        self.depth_encoder = ResnetEncoder(cfg['model']['num_layers'], cfg['model']['weights_init'], 1)
        del self.depth_encoder.encoder.fc
        self.depth_decoder = MonoDepthDecoder(self.depth_encoder.num_ch_enc, cfg['training']['scales'])

    def forward(self, images):
        return self.depth_decoder(self.depth_encoder(images))


class MonoPoseNet(nn.Module):
    """fsm baseline pose net (mono_posenet.py:8-29)."""

    def __init__(self, cfg):
        super().__init__()
        self.pose_encoder = ResnetEncoder(cfg['model']['num_layers'], cfg['model']['weights_init'], num_input_images=2)
        del self.pose_encoder.encoder.fc
        self.pose_decoder = PoseDecoder(self.pose_encoder.num_ch_enc, num_input_features=1,
                                        num_frames_to_predict_for=1)

    def forward(self, inputs, frame_ids, cam):
        x = torch.cat([inputs['color_aug', f, 0][:, cam] for f in frame_ids], 1)
        axis_angle, translation = self.pose_decoder([self.pose_encoder(x)])
        return axis_angle, torch.clamp(translation, -4.0, 4.0)

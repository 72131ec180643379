"""Dense CNN layers around the hot path (they stay on MIOpen / hipBLASLt via PyTorch-ROCm).

* `conv2d_block` / `conv1d_block`: the reference's conv + (BN|Identity) + act Sequential builders
  (`/root/reference/network/blocks.py:41-84`); kept as `nn.Sequential(conv, norm, act)` so
  state-dict keys (`….0.weight`) line up with reference checkpoints.
* `pack_cam_feat` / `unpack_cam_feat` / `upsample` (`blocks.py:6-38`).
* `ResnetEncoder`, `PoseDecoder`, `MonoDepthDecoder`: the third-party packnet-sfm / monodepth2
  layers that the reference imports from an un-vendored submodule
  (`/root/reference/external/layers/__init__.py:2-4`).  Restated from their published
  architecture (ResNet-18/34/50 with an n-image first conv, input normalised
  `(x-0.45)/0.225`; squeeze → two 3×3 → 1×1 pose head scaled ×0.01; 5-level
  reflect-padded ELU decoder).  Parameter names follow torchvision's ResNet so an
  ImageNet or reference-trained state dict loads unchanged.
"""
import os
from collections import OrderedDict

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


# ----------------------------------------------------------------------------- reference blocks
def _activation(nonlin):
    if nonlin == 'LRU':
        return nn.LeakyReLU(0.1, inplace=True)
    if nonlin == 'ELU':
        return nn.ELU(inplace=True)
    return nn.Identity()


def _fused_dtype_ok(x):
    """fp32 outside autocast, or the bf16 activations of config 3's bf16 autocast."""
    if torch.is_autocast_enabled('cuda'):
        return x.dtype == torch.bfloat16 and torch.get_autocast_dtype('cuda') == torch.bfloat16
    return x.dtype == torch.float32


class ReflectConv2d(nn.Conv2d):
    """nn.Conv2d(padding_mode='reflect') (same parameters and state-dict keys) whose one-pixel
    reflect padding runs on the HIP pad kernels for GPU maps (fp32, or bf16 under config 3's
    autocast): a deterministic backward (ATen's reflection_pad2d backward scatters with atomics)
    and one launch each way."""

    def _conv_forward(self, x, weight, bias):
        if (self.padding_mode == 'reflect' and tuple(self.padding) == (1, 1) and x.is_cuda and x.dim() == 4
                and _fused_dtype_ok(x) and x.shape[-1] >= 2 and x.shape[-2] >= 2
                and os.environ.get('VFD_REFLECT_PAD', '1') != '0'):
            from . import kernels as KN
            return F.conv2d(KN.ReflectPad1.apply(x), weight, bias, self.stride, 0, self.dilation, self.groups)
        return super()._conv_forward(x, weight, bias)


def conv2d_block(cin, cout, kernel_size=3, stride=1, dilation=1, nonlin='LRU',
                 padding_mode='reflect', norm=False):
    pad = ((kernel_size - 1) * dilation) // 2
    conv = ReflectConv2d(cin, cout, kernel_size, stride=stride, dilation=dilation, padding=pad,
                         bias=not norm, padding_mode=padding_mode)
    return nn.Sequential(conv, nn.BatchNorm2d(cout) if norm else nn.Identity(), _activation(nonlin))


def conv1d_block(cin, cout, kernel_size=3, stride=1, dilation=1, nonlin='LRU',
                 padding_mode='reflect', norm=False):
    pad = ((kernel_size - 1) * dilation) // 2
    conv = nn.Conv1d(cin, cout, kernel_size, stride=stride, dilation=dilation, padding=pad,
                     bias=not norm, padding_mode=padding_mode)
    return nn.Sequential(conv, nn.BatchNorm1d(cout) if norm else nn.Identity(), _activation(nonlin))


def pack_cam_feat(x):
    """[B, N, ...] -> [B*N, ...] (dicts are packed in place)."""
    if isinstance(x, dict):
        for k in list(x.keys()):
            v = x[k]
            x[k] = v.reshape(v.shape[0] * v.shape[1], *v.shape[2:])
        return x
    return x.reshape(x.shape[0] * x.shape[1], *x.shape[2:])


def unpack_cam_feat(x, b, n_cam):
    """[B*N, ...] -> [B, N, ...] (dicts are unpacked in place)."""
    if isinstance(x, dict):
        for k in list(x.keys()):
            v = x[k]
            x[k] = v.view(b, n_cam, *v.shape[1:])
        return x
    return x.view(b, n_cam, *x.shape[1:])


def upsample(x):
    return F.interpolate(x, scale_factor=2, mode='nearest')


# ----------------------------------------------------------------------------- ResNet encoder
_BN_GROUPS = [1]


class bn_groups:
    """Inside the block every training-mode BatchNorm of `bn_act` treats its batch as G consecutive
    groups with their own statistics — exactly G separate calls of the layer (running statistics
    updated G times in order).  The fused pose net runs its two frame pairs as one batch this way
    (models/geometry/pose.py:33-42 calls it once per pair)."""

    def __init__(self, groups):
        self.groups = int(groups)

    def __enter__(self):
        _BN_GROUPS.append(self.groups)
        return self

    def __exit__(self, *exc):
        _BN_GROUPS.pop()


def bn_act(bn, x, residual=None, relu=True, join=False):
    """relu(bn(x) [+ residual]): one fused HIP kernel pair (bnact.hip, SyncBatchNorm-aware) for a
    training-mode BatchNorm2d on the GPU, fp32 activations or (under bf16 autocast) bf16 ones with
    fp32 statistics; the module + torch ops otherwise (eval mode, CPU).  VFD_FUSED_BN=0 disables
    the fused path.  join: the residual is this block's input and also feeds its first conv (an
    identity block): its gradient is summed inside the producing BN's backward kernels."""
    G = _BN_GROUPS[-1]
    if (bn.training and bn.track_running_stats and bn.affine and bn.momentum is not None and x.is_cuda
            and x.dim() == 4 and _fused_dtype_ok(x) and os.environ.get('VFD_FUSED_BN', '1') != '0'
            and (residual is None or residual.shape == x.shape)):
        from . import kernels as KN
        return KN.BatchNormAct.apply(x, bn.weight, bn.bias, residual, bn.running_mean, bn.running_var,
                                     bn.eps, bn.momentum, relu, KN._bn_group(bn),
                                     bn.num_batches_tracked, join, G)   # += G inside the apply kernel
    if G > 1 and bn.training:
        y = torch.cat([bn(xc) for xc in x.chunk(G)])        # G calls, in group order
    else:
        y = bn(x)
    if residual is not None:
        y = y + residual
    return F.relu(y, inplace=True) if relu else y


def max_pool_stem(pool, x):
    """The stem's MaxPool2d(3, 2, 1): the HIP kernel pair for GPU maps, fp32 or bf16 under bf16
    autocast (one-byte argmax, gather backward), the module otherwise."""
    if (x.is_cuda and x.dim() == 4 and _fused_dtype_ok(x) and pool.kernel_size in (3, (3, 3))
            and pool.stride in (2, (2, 2)) and pool.padding in (1, (1, 1)) and pool.dilation in (1, (1, 1))
            and not pool.ceil_mode and os.environ.get('VFD_MAXPOOL', '1') != '0'):
        from . import kernels as KN
        return KN.MaxPool3s2.apply(x)
    return pool(x)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else bn_act(self.downsample[1], self.downsample[0](x), relu=False)
        y = bn_act(self.bn1, self.conv1(x))
        return bn_act(self.bn2, self.conv2(y), residual=idt, join=self.downsample is None)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else bn_act(self.downsample[1], self.downsample[0](x), relu=False)
        y = bn_act(self.bn1, self.conv1(x))
        y = bn_act(self.bn2, self.conv2(y))
        return bn_act(self.bn3, self.conv3(y), residual=idt, join=self.downsample is None)


_RESNET_SPECS = {18: (BasicBlock, [2, 2, 2, 2]), 34: (BasicBlock, [3, 4, 6, 3]),
                 50: (Bottleneck, [3, 4, 6, 3])}


class ResNetTrunk(nn.Module):
    """torchvision-named ResNet trunk with a `3*num_input_images`-channel stem."""

    def __init__(self, num_layers, num_input_images=1):
        super().__init__()
        block, counts = _RESNET_SPECS[num_layers]
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3 * num_input_images, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._stage(block, 64, counts[0], 1)
        self.layer2 = self._stage(block, 128, counts[1], 2)
        self.layer3 = self._stage(block, 256, counts[2], 2)
        self.layer4 = self._stage(block, 512, counts[3], 2)
        self.fc = nn.Linear(512 * block.expansion, 1000)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode='fan_out', nonlinearity='relu')
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def _stage(self, block, planes, n, stride):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes * block.expansion, 1, stride, bias=False),
                                 nn.BatchNorm2d(planes * block.expansion))
        blocks = [block(self.inplanes, planes, stride, down)]
        self.inplanes = planes * block.expansion
        blocks += [block(self.inplanes, planes) for _ in range(1, n)]
        return nn.Sequential(*blocks)


class ResnetEncoder(nn.Module):
    """Five-level ResNet feature pyramid (1/2 … 1/32) — packnet/monodepth2 `ResnetEncoder`."""

    def __init__(self, num_layers, pretrained=False, num_input_images=1):
        super().__init__()
        if num_layers not in _RESNET_SPECS:
            raise ValueError(f'{num_layers} is not a valid number of resnet layers')
        if pretrained:
            # no network access: ImageNet weights cannot be fetched; callers load their own.
            import warnings
            warnings.warn('weights_init=True requested but pretrained ImageNet weights are not '
                          'available offline; using seeded random init')
        self.num_ch_enc = np.array([64, 64, 128, 256, 512])
        if num_layers > 34:
            self.num_ch_enc[1:] *= 4
        self.encoder = ResNetTrunk(num_layers, num_input_images)
        self.channels_last = False

    def use_channels_last(self):
        """Config 3's bf16 encoders run channels-last: the conv weights (and through them every map:
        ATen's MIOpen convs take the channels-last layout when input or weight has it) live NHWC,
        so MIOpen's bf16 convs skip their NCHW <-> NHWC transposes and the fused BN kernels take
        the maps as they are (bnact.hip, d.nhwc).  The returned pyramid is channels-last; its
        consumers (1x1 aggregation slices, HIP ops via .contiguous()) accept either layout."""
        self.channels_last = True
        self.to(memory_format=torch.channels_last)
        return self

    def forward(self, image, normalized=False, groups=1):
        """image: [n, 3*num_input_images, H, W] in [0, 1]; normalized=True: already (x - 0.45) / 0.225
        (the fused nets normalise while concatenating frames: kernels.normalize_cat).  groups G: the
        batch is G stacked calls' batches, each BatchNorm'd on its own (`bn_groups`)."""
        e = self.encoder
        x = image if normalized else (image - 0.45) / 0.225
        if self.channels_last:
            # the first conv's input in its layout once: MIOpen's NHWC forward and weight gradient
            # would each make their own channels-last copy of it
            x = x.contiguous(memory_format=torch.channels_last)
        with bn_groups(groups):
            f0 = bn_act(e.bn1, e.conv1(x))
            f1 = e.layer1(max_pool_stem(e.maxpool, f0))
            f2 = e.layer2(f1)
            f3 = e.layer3(f2)
            f4 = e.layer4(f3)
        # returned, not kept as a module attribute (monodepth2's encoder stores `self.features`):
        # a kept pyramid would hold this step's autograd graph — and its AccumulateGrad nodes, with
        # the stream they were created on — alive into the next step (a captured HIP-graph step
        # after eager warm-up steps on a side stream then accumulates on that stream)
        return [f0, f1, f2, f3, f4]


# ----------------------------------------------------------------------------- decoders
class PoseDecoder(nn.Module):
    """squeeze(1×1, ReLU) → 3×3 → 3×3 → 1×1 → spatial mean × 0.01 → (axis-angle, translation)."""

    def __init__(self, num_ch_enc, num_input_features, num_frames_to_predict_for=None, stride=1):
        super().__init__()
        self.num_ch_enc = num_ch_enc
        self.num_input_features = num_input_features
        if num_frames_to_predict_for is None:
            num_frames_to_predict_for = num_input_features - 1
        self.num_frames_to_predict_for = num_frames_to_predict_for
        self.convs = OrderedDict()
        self.convs['squeeze'] = nn.Conv2d(int(num_ch_enc[-1]), 256, 1)
        self.convs[('pose', 0)] = nn.Conv2d(num_input_features * 256, 256, 3, stride, 1)
        self.convs[('pose', 1)] = nn.Conv2d(256, 256, 3, stride, 1)
        self.convs[('pose', 2)] = nn.Conv2d(256, 6 * num_frames_to_predict_for, 1)
        self.relu = nn.ReLU()
        self.net = nn.ModuleList(list(self.convs.values()))

    def forward(self, input_features):
        last = [feats[-1] for feats in input_features]
        x = torch.cat([self.relu(self.convs['squeeze'](f)) for f in last], 1)
        for i in range(3):
            x = self.convs[('pose', i)](x)
            if i < 2:
                x = self.relu(x)
        x = 0.01 * x.mean(3).mean(2).view(-1, self.num_frames_to_predict_for, 1, 6)
        return x[..., :3], x[..., 3:]


class _Conv3x3(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.pad = nn.ReflectionPad2d(1)
        self.conv = nn.Conv2d(int(cin), int(cout), 3)

    def forward(self, x):
        return self.conv(self.pad(x))


class _ConvBlock(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.conv = _Conv3x3(cin, cout)
        self.nonlin = nn.ELU(inplace=True)

    def forward(self, x):
        return self.nonlin(self.conv(x))


class MonoDepthDecoder(nn.Module):
    """Five-level monodepth2 decoder used by the fsm baseline (`network/mono_depthnet.py:19`)."""

    def __init__(self, num_ch_enc, scales=range(4), num_output_channels=1, use_skips=True):
        super().__init__()
        self.num_output_channels = num_output_channels
        self.use_skips = use_skips
        self.scales = scales
        self.num_ch_enc = num_ch_enc
        self.num_ch_dec = np.array([16, 32, 64, 128, 256])
        self.convs = OrderedDict()
        for i in range(4, -1, -1):
            cin = num_ch_enc[-1] if i == 4 else self.num_ch_dec[i + 1]
            self.convs[('upconv', i, 0)] = _ConvBlock(cin, self.num_ch_dec[i])
            cin = self.num_ch_dec[i] + (num_ch_enc[i - 1] if (use_skips and i > 0) else 0)
            self.convs[('upconv', i, 1)] = _ConvBlock(cin, self.num_ch_dec[i])
        for s in scales:
            self.convs[('dispconv', s)] = _Conv3x3(self.num_ch_dec[s], num_output_channels)
        self.decoder = nn.ModuleList(list(self.convs.values()))
        self.sigmoid = nn.Sigmoid()

    def forward(self, input_features):
        out = {}
        x = input_features[-1]
        for i in range(4, -1, -1):
            x = upsample(self.convs[('upconv', i, 0)](x))
            if self.use_skips and i > 0:
                x = torch.cat([x, input_features[i - 1]], 1)
            x = self.convs[('upconv', i, 1)](x)
            if i in self.scales:
                out[('disp', i)] = self.sigmoid(self.convs[('dispconv', i)](x))
        return out


def seeded_state_dict(module, seed=0):
    """Deterministic, machine-independent weights for parity runs (no checkpoint download).

    Conv/linear weights ~ U(-a, a) with a = sqrt(3 / fan_in) (unit-variance pre-activations),
    biases ~ U(-0.05, 0.05), BatchNorm affine (1, 0) and running stats (0, 1).  Values are drawn
    from one CPU `torch.Generator` in sorted-key order, so any model with the same parameter
    names and shapes (this package's or the reference's) receives identical tensors.
    """
    gen = torch.Generator().manual_seed(int(seed))
    sd = module.state_dict()
    out = OrderedDict()
    for key in sorted(sd.keys()):
        t = sd[key]
        if key.endswith('num_batches_tracked'):
            out[key] = torch.zeros_like(t)
        elif key.endswith('running_mean'):
            out[key] = torch.zeros_like(t)
        elif key.endswith('running_var'):
            out[key] = torch.ones_like(t)
        elif t.dim() == 1 and ('bn' in key or 'downsample.1' in key):
            out[key] = torch.ones_like(t) if key.endswith('weight') else torch.zeros_like(t)
        elif t.dim() >= 2:
            fan_in = int(np.prod(t.shape[1:]))
            a = (3.0 / fan_in) ** 0.5
            out[key] = (torch.rand(t.shape, generator=gen, dtype=torch.float64) * 2 - 1).mul_(a).to(t.dtype)
        else:
            out[key] = ((torch.rand(t.shape, generator=gen, dtype=torch.float64) * 2 - 1) * 0.05).to(t.dtype)
    return out

"""Autograd wrappers of the gfx950 hot-path kernels (C ABI in include/vfd_capi.h).

Each op is a `torch.autograd.Function` whose forward and backward are single C-ABI calls on the
current HIP stream.  Inputs must be fp32 HIP tensors; there is no CPU or ATen fallback — a
missing library or a non-HIP tensor raises.
"""
import ctypes
import math
import os
import weakref

import torch
import torch.nn.functional as F

from . import _lib as L


def _check_device(t, what):
    if not torch.is_tensor(t) or not t.is_cuda:
        raise RuntimeError(f'{what}: the VFDepth hot path runs only on a HIP device (got '
                           f'{"non-tensor" if not torch.is_tensor(t) else t.device})')
    if t.device.index is not None and t.device.index != torch.cuda.current_device():
        # every launch goes on the current device's stream (_lib.stream): a tensor of another
        # device would be read through the wrong context
        raise RuntimeError(f'{what}: tensor on {t.device} but the current HIP device is '
                           f'cuda:{torch.cuda.current_device()} (torch.cuda.set_device first)')


def _dev(t, what):
    _check_device(t, what)
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


# Under bf16 autocast (net_precision='bf16', config 3) the fusion ops take fp32 inputs and run
# with autocast off; their gradients are cast back to the callers' dtypes by autograd.
_amp_fwd = torch.amp.custom_fwd(device_type='cuda', cast_inputs=torch.float32)
_amp_bwd = torch.amp.custom_bwd(device_type='cuda')
_amp_keep = torch.amp.custom_fwd(device_type='cuda')     # autocast-aware, inputs as given


def _dt(t):
    """C-ABI activation dtype code of a dense-net map: 0 fp32, 1 bf16."""
    if t.dtype == torch.float32:
        return 0
    if t.dtype == torch.bfloat16:
        return 1
    raise RuntimeError(f'dense-net kernels take fp32 or bf16 maps, got {t.dtype}')


def _ws(nbytes, device):
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


# =============================================================================================
# Voxel space (constant grids of VFNet, volumetric_fusionnet.py:15-40, 67-103)
# =============================================================================================
def overlap_group_table(n_cams):
    """Camera -> overlap group (volumetric_fusionnet.py:217-225); None if overlap is undefined."""
    if n_cams == 6:
        return [0, 1, 1, 0, 0, 1]
    if n_cams == 3:
        return [0, 1, 1]
    return None


class VoxelSpace:
    """Device-resident voxel axes / depth bins / camera groups + descriptor factory."""

    def __init__(self, cfg, device):
        m, t = cfg['model'], cfg['training']
        self.size = [int(v) for v in m['voxel_size']]
        unit = [float(v) for v in m['voxel_unit_size']]
        self.str_p = [float(v) for v in m['voxel_str_p']]
        self.end_p = [self.str_p[i] + unit[i] * (self.size[i] - 1) for i in range(3)]
        self.X, self.Y, self.Z = self.size
        self.V = self.X * self.Y * self.Z
        lvl = int(m['fusion_level'])
        self.H, self.W = int(t['height']), int(t['width'])
        self.h, self.w = self.H // 2 ** (lvl + 1), self.W // 2 ** (lvl + 1)
        self.D = int(m['proj_d_bins'])
        self.z_scale = float(m['voxel_size'][0])
        self.n_cams = int(cfg['data']['num_cams'])
        self.device = torch.device(device)
        axes = [torch.linspace(self.str_p[i], self.end_p[i], self.size[i]) for i in range(3)]
        self.axes = [a.to(self.device) for a in axes]
        self.dbins = torch.linspace(m['proj_d_str'], m['proj_d_end'], self.D).to(self.device)
        grp = overlap_group_table(self.n_cams) or [0] * self.n_cams
        self.group = torch.tensor(grp, dtype=torch.int32, device=self.device)
        self._pose_order = None

    def pose_order(self):
        """K2's voxel order by azimuth sector (fusion.hip fuse_pose_fwd_k's `order`): [8, cap] int32
        voxel indices, sector k = the voxel columns whose centre azimuth atan2(y, x) falls in
        [-pi + k pi/4, -pi + (k+1) pi/4), index order inside a sector, -1 padding to a common cap
        (a multiple of 32).  Not used by the step (measured 193 vs 186 us per call at config 3,
        102 vs 100 at config 2: the gather is not bound by the cross-XCD feature re-reads); kept for
        the C ABI's `order` argument, which test_pose_conv_bf16_map_matches_two_nodes covers."""
        if self._pose_order is None:
            v = torch.arange(self.V)
            ax, ay = (a.cpu().double() for a in self.axes[:2])
            theta = torch.atan2(ay[(v // self.X) % self.Y], ax[v % self.X])
            sec = ((theta + math.pi) / (math.pi / 4)).floor().long().clamp(0, 7)
            parts = [v[sec == k] for k in range(8)]
            cap = (max(len(p) for p in parts) + 31) // 32 * 32
            order = torch.full((8, cap), -1, dtype=torch.int32)
            for k, p in enumerate(parts):
                order[k, :len(p)] = p.to(torch.int32)
            self._pose_order = order.to(self.device)
        return self._pose_order

    def desc(self, B, N, C=0, Cv=0, pad_out=1):
        d = L.VoxelDesc()
        d.B, d.N, d.C, d.Cv = B, N, C, Cv
        d.h, d.w, d.H, d.W = self.h, self.w, self.H, self.W
        d.X, d.Y, d.Z, d.D = self.X, self.Y, self.Z, self.D
        for i in range(3):
            d.str[i] = self.str_p[i]
            d.len[i] = self.end_p[i] - self.str_p[i]
        d.z_scale = self.z_scale
        d.pad_out = pad_out
        d.axis_x, d.axis_y, d.axis_z = (a.data_ptr() for a in self.axes)
        d.dbins = self.dbins.data_ptr()
        d.group = self.group.data_ptr()
        d.deterministic = int(deterministic())
        return d


def deterministic():
    """Fixed-order gradient sums in the fusion kernels: on when torch.backends.cudnn.deterministic
    is set (the reference's train.py:23-24 sets it, with benchmark off) or VFD_DETERMINISTIC=1."""
    return bool(torch.backends.cudnn.deterministic) or os.environ.get('VFD_DETERMINISTIC', '0') == '1'


def mask_lowres(space, mask):
    """mask [B,N,1,H,W] -> [B,N,h,w] (bilinear, align_corners=True); no gradient."""
    lib = L.load()
    mask = _dev(mask, 'mask')
    B, N = mask.shape[:2]
    out = torch.empty(B, N, space.h, space.w, device=mask.device)
    d = space.desc(B, N)
    L.check(lib.vfd_mask_downsample(ctypes.byref(d), mask.data_ptr(), out.data_ptr(), L.stream()), 'mask_downsample')
    return out


_K1_GATHER = os.environ.get('VFD_K1_GATHER', '1') != '0'


class FuseDepth(torch.autograd.Function):
    """K1: P [B,N,hw,2Cv] (folded 1x1-conv maps) -> voxel features [B,V,Cv] (channels-last).

    Backward: with the step's FusionPlan (`plan`, the K2 backward's tile index of the same
    geometry) and Cv = 64, d P is an atomic-free gather over the plan's tile buckets
    (`vfd_fuse_depth_bwd_planned`); otherwise the voxel-walk scatter with f32 atomics."""

    @staticmethod
    @_amp_fwd
    def forward(ctx, space, P, mask_lo, K, Einv, wz, b_no, b_o, plan=None):
        lib = L.load()
        P, mask_lo, K, Einv = (_dev(t, n) for t, n in ((P, 'P'), (mask_lo, 'mask'), (K, 'K'), (Einv, 'Einv')))
        wz, b_no, b_o = (_dev(t, 'fusion params') for t in (wz, b_no, b_o))
        B, N, hw, two_cv = P.shape
        Cv = two_cv // 2
        if hw != space.h * space.w:
            raise ValueError(f'feature map {hw} px does not match voxel space {space.h}x{space.w}')
        vox = torch.empty(B, space.V, Cv, device=P.device)
        d = space.desc(B, N, Cv=Cv)
        L.check(lib.vfd_fuse_depth_fwd(ctypes.byref(d), P.data_ptr(), mask_lo.data_ptr(), K.data_ptr(),
                                       Einv.data_ptr(), wz.data_ptr(), b_no.data_ptr(), b_o.data_ptr(),
                                       vox.data_ptr(), L.stream()), 'fuse_depth_fwd')
        ctx.space, ctx.shape = space, (B, N, hw, Cv)
        ctx.plan = plan if (plan is not None and Cv == 64 and _K1_GATHER) else None
        if ctx.plan is None and deterministic() and torch.is_grad_enabled():
            raise RuntimeError('deterministic mode: the K1 backward needs the fusion plan gather (Cv = 64, '
                               'VFD_K1_GATHER=1); the atomic scatter sums in arrival order')
        ctx.save_for_backward(vox, mask_lo, K, Einv)
        return vox

    @staticmethod
    @_amp_bwd
    def backward(ctx, g):
        lib = L.load()
        vox, mask_lo, K, Einv = ctx.saved_tensors
        B, N, hw, Cv = ctx.shape
        g = _dev(g, 'grad')
        d = ctx.space.desc(B, N, Cv=Cv)
        dP = torch.empty(B, N, hw, 2 * Cv, device=g.device)
        dwzb = torch.empty(5, Cv, device=g.device)
        nbytes = (lib.vfd_fuse_depth_bwd_planned_workspace if ctx.plan is not None
                  else lib.vfd_fuse_depth_bwd_workspace)(ctypes.byref(d))
        ws = _ws(nbytes, g.device)
        if ctx.plan is not None:
            plan, ctx.plan = ctx.plan.build(), None
            plan.wait()
            L.check(lib.vfd_fuse_depth_bwd_planned(ctypes.byref(d), plan.buf.data_ptr(), g.data_ptr(), vox.data_ptr(),
                                                   mask_lo.data_ptr(), K.data_ptr(), Einv.data_ptr(), dP.data_ptr(),
                                                   dwzb.data_ptr(), ws.data_ptr(), nbytes, L.stream()),
                    'fuse_depth_bwd_planned')
        else:
            L.check(lib.vfd_fuse_depth_bwd(ctypes.byref(d), g.data_ptr(), vox.data_ptr(), mask_lo.data_ptr(),
                                           K.data_ptr(), Einv.data_ptr(), dP.data_ptr(), dwzb.data_ptr(),
                                           ws.data_ptr(), nbytes, L.stream()), 'fuse_depth_bwd')
        return None, dP, None, None, None, dwzb[:3], dwzb[3], dwzb[4], None


def _wait_stream(dst, src):
    """dst waits for the work queued on src so far — skipped when they are one stream.  A stream
    waiting on its own event is a no-op on the device, but under HIP-graph capture this HIP runtime
    (ROCm 7.x) files a non-origin capture stream that waits on an event of ITSELF (or of another
    non-origin stream that joined through it) as its own parallel-capture child; hipStreamEndCapture
    then recurses through that cycle until the host stack overflows (round 6: a SIGSEGV inside
    libamdhip64 with ~170k identical frames; tools/diag_capture_patterns.py, tools/hiplog_capture.py)."""
    if dst != src:
        dst.wait_stream(src)


class FusionPlan:
    """Per-(batch, camera) compacted list of visible voxels with their tap data (device buffers).

    Built once per step from K (fusion scale), E^-1 and the 1/8 mask; every pose-mode fusion call
    of the step reuses it (the geometry does not depend on features).  Only the backward reads the
    buffers, so they are built on demand (`build()`: by the first forward that needs a gradient;
    a no-grad evaluation step never allocates them), on the current stream; `wait()` joins that
    stream from another (the depth branch's K1 backward reads the plan the pose branch built)."""

    def __init__(self, space, mask_lo, K, Einv, build=True):
        mask_lo, K, Einv = (_dev(t, n) for t, n in ((mask_lo, 'mask'), (K, 'K'), (Einv, 'Einv')))
        self.B, self.N = mask_lo.shape[:2]
        self.mask_lo, self.K, self.Einv = mask_lo, K, Einv
        self.space = space
        self.buf = None
        if build:
            self.build()

    def build(self):
        if self.buf is not None:
            return self
        lib = L.load()
        mask_lo, K, Einv = self.mask_lo, self.K, self.Einv
        d = self.space.desc(self.B, self.N)
        nbytes = lib.vfd_fusion_plan_bytes(ctypes.byref(d))
        # built on the current stream (round 2: a side stream overlapping the dense layers measured
        # slower at config 2, 44.2-44.4 vs 41.9-42.1 ms/step — the plan kernels co-running with
        # MIOpen's implicit-GEMM convs cost those more than the plans take)
        self.side = torch.cuda.current_stream(mask_lo.device)
        self.buf = torch.empty(nbytes, dtype=torch.uint8, device=mask_lo.device)
        self.counts = torch.empty(self.B * self.N, dtype=torch.int32, device=mask_lo.device)
        L.check(lib.vfd_fusion_plan(ctypes.byref(d), mask_lo.data_ptr(), K.data_ptr(), Einv.data_ptr(),
                                    self.buf.data_ptr(), self.counts.data_ptr(), L.stream()), 'fusion_plan')
        # the point right after the plan kernels: a consumer on another stream waits for this, not
        # for everything queued on the building stream later (the pose branch's stream builds the
        # plan in its forward; the depth branch's K1 backward reads it while the pose backward runs)
        self.ready = torch.cuda.Event()
        self.ready.record(self.side)
        return self

    def wait(self):
        """Make the current stream wait for the plan (before any kernel that reads its buffers)."""
        cur = torch.cuda.current_stream(self.buf.device)
        if cur != self.side:
            cur.wait_event(self.ready)


def _channels_last(t, what):
    """Device fp32 tensor in channels-last (NHWC) memory order (no copy when it already is)."""
    _check_device(t, what)
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous(memory_format=torch.channels_last)


def _nhwc(t, what):
    """Device tensor in channels-last (NHWC) memory order, its dtype kept (no copy when it already is)."""
    _check_device(t, what)
    return t.contiguous(memory_format=torch.channels_last)


def pose_conv_weight(w, C1, Z):
    """reduce_dim[0] weight [O, C1*Z, kh, kw] (reference channel c*Z + z) -> the z-major order
    z*C1 + c of FusePose's output; differentiable (a view + one gather)."""
    O = w.shape[0]
    return w.view(O, C1, Z, *w.shape[2:]).transpose(1, 2).reshape(O, Z * C1, *w.shape[2:])


def proj_conv_weight(w, Cv, D):
    """reduce_dim[0] weight [O, Cv*D, kh, kw] (reference channel c*D + d) -> the depth-major
    order d*Cv + c of VoxelProject's output."""
    O = w.shape[0]
    return w.view(O, Cv, D, *w.shape[2:]).transpose(1, 2).reshape(O, D * Cv, *w.shape[2:])


def pose_to_reference(out, C1, Z):
    """FusePose output -> the reference's [B, C1*Z, Y+2, X+2] channel order (tests, tools)."""
    B, _, H, W = out.shape
    return out.reshape(B, Z, C1, H, W).transpose(1, 2).reshape(B, C1 * Z, H, W)


def proj_to_reference(out, Cv, D):
    """VoxelProject output -> the reference's [B*N, Cv*D, h+2, w+2] channel order."""
    BN, _, H, W = out.shape
    return out.reshape(BN, D, Cv, H, W).transpose(1, 2).reshape(BN, Cv * D, H, W)


class FusePose(torch.autograd.Function):
    """K2: feats [B,N,C,h,w] -> mean voxel features as the channels-last, reflect-padded input of
    reduce_dim's stride-2 conv: logical [B, Z*(C+1), Y+2, X+2], channel z*(C+1) + c."""

    @staticmethod
    @_amp_fwd
    def forward(ctx, space, plan, feats):
        out = _pose_fuse_t(space, plan, feats, torch.float32)
        ctx.space, ctx.plan, ctx.shape = space, plan, tuple(feats.shape)
        if ctx.needs_input_grad[2]:
            plan.build()            # the backward's index (kept in the order the step issued it)
        return out

    @staticmethod
    @_amp_bwd
    def backward(ctx, g):
        return None, None, _pose_unfuse(ctx.space, ctx.plan, ctx.shape, _channels_last(g, 'grad'))


class VoxelProject(torch.autograd.Function):
    """K3: voxel features [B,V,Cv] -> frustum features as the channels-last, reflect-padded input
    of reduce_dim's first conv: logical [B*N, D*Cv, h+2, w+2], channel d*Cv + c.

    When the voxels need a gradient, the forward also builds the backward's geometry-only plan
    (`vfd_voxel_project_plan`: the frustum samples sorted by voxel cell, on the forward's stream);
    the backward joins that stream and runs only the d_out-dependent part
    (`vfd_voxel_project_bwd_planned`)."""

    @staticmethod
    @_amp_fwd
    def forward(ctx, space, vox, invK, E):
        lib = L.load()
        vox, invK, E = (_dev(t, n) for t, n in ((vox, 'voxel'), (invK, 'inv_K'), (E, 'extrinsics')))
        B, V, Cv = vox.shape
        N = E.shape[1]
        out = torch.empty(B * N, Cv * space.D, space.h + 2, space.w + 2, device=vox.device,
                          memory_format=torch.channels_last)
        d = space.desc(B, N, Cv=Cv)
        L.check(lib.vfd_voxel_project_fwd(ctypes.byref(d), vox.data_ptr(), invK.data_ptr(), E.data_ptr(),
                                          out.data_ptr(), L.stream()), 'voxel_project_fwd')
        ctx.space, ctx.shape = space, (B, N, V, Cv)
        ctx.plan = ctx.side = None
        if ctx.needs_input_grad[1]:
            nbytes = lib.vfd_voxel_project_plan_bytes(ctypes.byref(d))
            plan = torch.empty(nbytes, dtype=torch.uint8, device=vox.device)
            L.check(lib.vfd_voxel_project_plan(ctypes.byref(d), invK.data_ptr(), E.data_ptr(), plan.data_ptr(),
                                               nbytes, L.stream()), 'voxel_project_plan')
            ctx.plan, ctx.side = plan, torch.cuda.current_stream(vox.device)
        return out

    @staticmethod
    @_amp_bwd
    def backward(ctx, g):
        lib = L.load()
        B, N, V, Cv = ctx.shape
        g = _channels_last(g, 'grad')
        dvox = torch.empty(B, V, Cv, device=g.device)
        d = ctx.space.desc(B, N, Cv=Cv)
        _wait_stream(torch.cuda.current_stream(g.device), ctx.side)
        L.check(lib.vfd_voxel_project_bwd_planned(ctypes.byref(d), g.data_ptr(), ctx.plan.data_ptr(),
                                                  ctx.plan.numel(), dvox.data_ptr(), L.stream()), 'voxel_project_bwd')
        ctx.plan = None
        return None, dvox, None, None




def _weight_fragments(mode, w, shape, C1=0, Z=0, Cv=0, D=0):
    """One relayout launch (weights.hip) of a conv weight [O, C, 3, 3] into an MFMA kernel's copy."""
    lib = L.load()
    w = _dev(w.detach(), 'conv weight')
    out = torch.empty(shape, device=w.device)
    O, C = w.shape[:2]
    L.check(lib.vfd_weight_fragments(mode, w.data_ptr(), out.data_ptr(), O, C, C1, Z, Cv, D, L.stream()),
            'weight_fragments')
    return out


def proj_conv_weight_fragments(w, Cv, D):
    """reduce_dim[0] weight [O, Cv*D, 3, 3] (reference channel c*D + d) -> the fused kernel's
    fragment-ordered copy [D, 3, 3, Cv/4, O, 2, 2] (c = 4q + 2h + s; projconv.hip, pcv_main_k)."""
    O = w.shape[0]
    return _weight_fragments(1, w, (D, 3, 3, Cv // 4, O, 2, 2), Cv=Cv, D=D)


def proj_conv_dgrad_weight(w, Cv, D):
    """reduce_dim[0] weight [O, Cv*D, 3, 3] (reference channel c*D + d) -> the data-gradient
    kernel's copy [9 flipped taps, O/4, np, 2, 2] (o = 4q + 2h + s; n = d*Cv + c zero-padded to a
    multiple of 256; projconv.hip, pcd_main_k)."""
    O = w.shape[0]
    npad = (Cv * D + 255) // 256 * 256
    return _weight_fragments(2, w, (9, O // 4, npad, 2, 2), Cv=Cv, D=D)


_PC_DGRAD = os.environ.get('VFD_PC_DGRAD', '1') != '0'
_PC_WGRAD = os.environ.get('VFD_PC_WGRAD', '1') != '0'
_PC_FOLD = os.environ.get('VFD_PC_FOLD', '1') != '0'    # K3C data gradient with the reflect fold inside
_PC_BF16_BWD = os.environ.get('VFD_PC_BF16_BWD', '1') != '0'   # hand-written bf16 K3C / K2C backward (config 3)


def pad_conv_weight_fragments(w, C1=0, Z=0):
    """Conv weight [O, C, 3, 3] -> K2C's copy [9 taps, Cpad/4, O, 2, 2] (c = 4q + 2h + s over the
    input map's channel order, Cpad = C rounded up to 16, zero-padded; padconv.hip, ppc_main_k).
    C1, Z > 0: w is in the reference order c*Z + z and the map is K2's z-major z*C1 + c."""
    O, C = w.shape[:2]
    cpad = (C + 15) // 16 * 16
    return _weight_fragments(0, w, (9, cpad // 4, O, 2, 2), C1=C1, Z=Z)


def pose_conv_fragments(w, C1, Z):
    """The pose reduce_dim[0] weight [O, C1*Z, 3, 3] (reference channel c*Z + z) straight to K2C's
    fragment copy over FusePose's channel order z*C1 + c; no gradient."""
    return pad_conv_weight_fragments(w, C1, Z)


_SWAP_CACHE = {}


def weight_swap(w, A, B, cache=False, memory_format=torch.contiguous_format):
    """w [O, A*B, kh, kw] (any layout) with channel a*B + b -> channel b*A + a, written in
    `memory_format` (weights.hip, one launch; NCHW and channels-last on either side, so MIOpen's
    channels-last convolutions get their weight without a conversion copy).  cache: reuse the last
    result for the same tensor, version and format (the pose weight, swapped once per step for both
    pose calls' backward)."""
    key = (w.data_ptr(), w._version, tuple(w.shape), A, B, memory_format) if cache else None
    hit = _SWAP_CACHE.get('entry')
    if key is not None and hit is not None and hit[1] == key:
        return hit[2]
    out = _weight_permute_swap(w, A, B, memory_format)
    if key is not None:     # the entry holds the source, so its address cannot be reused meanwhile
        _SWAP_CACHE['entry'] = (w, key, out)
    return out


def _weight_permute_swap(w, A, B, memory_format):
    lib = L.load()
    _check_device(w, 'conv weight')
    if w.dtype != torch.float32:
        w = w.float()
    # any layout whose taps are evenly strided (NCHW, channels-last: MIOpen's NHWC weight gradient)
    # goes in as it is — no contiguous copy of the 47-MB pose weight gradient
    O, C, kh, kw = w.shape
    T = kh * kw
    out = torch.empty(O, C, kh, kw, device=w.device, memory_format=memory_format)
    so, sc, sy, sx = w.stride()
    if sy != kw * sx:
        w = w.contiguous()
        so, sc, sy, sx = w.stride()
    do, dc, dy_, dx_ = out.stride()
    # element (o, a, b, t): source channel a*B + b, destination channel b*A + a, tap t = y*kw + x
    src = (ctypes.c_longlong * 4)(so, B * sc, sc, sx)
    dst = (ctypes.c_longlong * 4)(do, dc, A * dc, dx_)
    L.check(lib.vfd_weight_permute(w.data_ptr(), out.data_ptr(), O, A, B, T, src, dst, L.stream()), 'weight_permute')
    return out


def pad_conv_desc(x, stride, out_channels):
    B, C, H, W = x.shape
    return L.ConvDesc(B, H, W, C, stride, out_channels)


def pad_conv_supported(x, stride, out_channels):
    """K2C applies: fp32 NHWC-able map, C % 4 == 0, 256 outputs, rows of a tile fit in LDS."""
    return bool(L.load().vfd_pad_conv_fwd_workspace(ctypes.byref(pad_conv_desc(x, stride, out_channels))))


# K2C data gradient on the HIP path: '1' (default) the bf16 form (config 3: 0.71 vs MIOpen's fp32
# 1.91 ms per call at B = 2), 'all' the fp32 form too (slower than MIOpen's at configs 2 / 5: 1.09 vs
# 0.91 ms, 15.9 vs 9.3 ms — profiles/r4/pdgrad_micro.txt), '0' never
_PAD_DGRAD_ENV = os.environ.get('VFD_PAD_DGRAD', '1')
_PAD_DGRAD = _PAD_DGRAD_ENV != '0'
_PAD_DGRAD_FP32 = _PAD_DGRAD_ENV == 'all'
_PDW_CACHE = {}


def pad_conv_dgrad_weight(w, perm=None, bf16=False, cache=True):
    """K2C weight [O, C, 3, 3] -> the data-gradient kernel's copy over the MAP's channel order:
    mode 2 [9 flipped taps, O/4, np, 2, 2] with Cv = C1, D = Z (perm = (C1, Z): reference channel
    c*Z + z at map channel z*C1 + c) or Cv = C, D = 1; bf16: mode 5 of it.  Cached per (tensor,
    version): the step's two pose calls share one copy (padconv.hip ppd_main_k)."""
    lib = L.load()
    w = _dev(w.detach(), 'pad_conv weight')
    O, C = w.shape[:2]
    Cv, D = perm if perm else (C, 1)
    # the entry holds the source tensor (so its storage stays alive and no other weight can be
    # handed the same address while the key is live) next to (address, version, shape)
    key = (w.data_ptr(), w._version, tuple(w.shape), Cv, D, bf16)
    hit = _PDW_CACHE.get('entry')
    if cache and hit is not None and hit[1] == key:
        return hit[2]
    npad = (C + 255) // 256 * 256
    f2 = torch.empty(9, O // 4, npad, 2, 2, device=w.device)
    L.check(lib.vfd_weight_fragments(2, w.data_ptr(), f2.data_ptr(), O, 0, 0, 0, Cv, D, L.stream()),
            'weight_fragments')
    out = f2
    if bf16:
        out = torch.empty(9, O // 16, npad // 32, 64, 8, dtype=torch.bfloat16, device=w.device)
        L.check(lib.vfd_weight_fragments_bf16(5, f2.data_ptr(), out.data_ptr(), O, 0, 0, 0, Cv, D, L.stream()),
                'weight_fragments_bf16')
    if cache:
        _PDW_CACHE['entry'] = (w, key, out)
    return out


_PD_DX_BF16 = os.environ.get('VFD_PD_DX_BF16', '0') == '1'   # opt-in: slower K2 backward  # bf16 K2C: d map rounded to bf16 (autocast's)


def pad_conv_dgrad(g_pre, x_shape, w, stride, perm=None, out_dtype=torch.float32):
    """K2C's data gradient through the C ABI: g_pre [B, 256, Ho, Wo] channels-last (fp32 or bf16) ->
    d x [B, C, H, W] channels-last (every padded position written), fp32 or — bf16 g_pre only —
    bf16 (the fp32 sums rounded once, as a bf16 convolution's input gradient is); None when
    unsupported."""
    lib = L.load()
    B, C, H, W = x_shape
    d = L.ConvDesc(B, H, W, C, stride, g_pre.shape[1])
    bf16 = g_pre.dtype == torch.bfloat16
    nbytes = (lib.vfd_pad_conv_dgrad_bf16_workspace if bf16 else lib.vfd_pad_conv_dgrad_workspace)(ctypes.byref(d))
    if not nbytes:
        return None
    wd = pad_conv_dgrad_weight(w, perm, bf16)
    out_dtype = out_dtype if bf16 else torch.float32
    dx = torch.empty(B, C, H, W, device=g_pre.device, dtype=out_dtype, memory_format=torch.channels_last)
    ws = _ws(nbytes, g_pre.device)
    if bf16:
        L.check(lib.vfd_pad_conv_dgrad_bf16_t(ctypes.byref(d), g_pre.data_ptr(), wd.data_ptr(), dx.data_ptr(),
                                              _DT[out_dtype], ws.data_ptr(), nbytes, L.stream()), 'pad_conv_dgrad')
    else:
        L.check(lib.vfd_pad_conv_dgrad(ctypes.byref(d), g_pre.data_ptr(), wd.data_ptr(), dx.data_ptr(), ws.data_ptr(),
                                       nbytes, L.stream()), 'pad_conv_dgrad')
    return dx


_PAD_WGRAD = os.environ.get('VFD_PAD_WGRAD', '1') != '0'    # bf16 K2C weight gradient on the HIP path


def pad_conv_wgrad_bf16(gb, x, w, stride, need_w=True, need_b=True):
    """K2C's bf16 weight / bias gradient through the C ABI: gb [B, 256, Ho, Wo] bf16 channels-last
    (d pre-activation), x the channels-last map [B, C, H, W] (fp32, or the bf16 map of PoseConvBF16)
    -> (d w in the MAP's channel order [256, C, 3, 3] fp32, d b [256] fp32); (None, None) parts not
    asked for."""
    lib = L.load()
    B, C, H, W = x.shape
    d = L.ConvDesc(B, H, W, C, stride, gb.shape[1])
    nbytes = lib.vfd_pad_conv_wgrad_bf16_workspace(ctypes.byref(d))
    if not nbytes:
        raise RuntimeError(f'pad_conv_wgrad_bf16: unsupported shape {tuple(x.shape)}, stride {stride}')
    dw = torch.empty(gb.shape[1], C, 3, 3, device=gb.device) if need_w else None
    db = torch.empty(gb.shape[1], device=gb.device) if need_b else None
    ws = _ws(nbytes, gb.device)
    gb = _nhwc(gb.to(torch.bfloat16), 'grad')
    x = _nhwc(x if x.dtype == torch.bfloat16 else x.float(), 'map')
    L.check(lib.vfd_pad_conv_wgrad_bf16_t(ctypes.byref(d), gb.data_ptr(), x.data_ptr(), _DT[x.dtype], L.ptr(dw),
                                          L.ptr(db), ws.data_ptr(), nbytes, L.stream()), 'pad_conv_wgrad_bf16')
    return dw, db


class PadConv(torch.autograd.Function):
    """K2C: reflect-padded channels-last map x [B, C, H, W] -> LeakyReLU(conv3x3_stride(x) + bias)
    as the reflect-padded channels-last input of the next reflect conv, logical
    [B, 256, Ho+2, Wo+2] (fp32 MFMA, padconv.hip).  Backward: MIOpen's data / weight gradients of
    the conv on the pre-activation gradient (pad adjoint + LeakyReLU slope from the output)."""

    @staticmethod
    @_amp_fwd
    def forward(ctx, x, w, bias, stride, wf=None, perm=None):
        lib = L.load()
        x = _channels_last(x, 'pad_conv input')
        w, bias = _dev(w, 'pad_conv weight'), _dev(bias, 'pad_conv bias')
        O = w.shape[0]
        d = pad_conv_desc(x, stride, O)
        nbytes = lib.vfd_pad_conv_fwd_workspace(ctypes.byref(d))
        if not nbytes:
            raise RuntimeError(f'pad_conv_fwd: unsupported shape {tuple(x.shape)}, stride {stride}, {O} outputs')
        ho, wo = (x.shape[2] - 3) // stride + 1, (x.shape[3] - 3) // stride + 1
        out = torch.empty(x.shape[0], O, ho + 2, wo + 2, device=x.device, memory_format=torch.channels_last)
        if wf is None:
            wf = pad_conv_weight_fragments(w, *(perm or (0, 0)))
        ws = _ws(nbytes, x.device)
        L.check(lib.vfd_pad_conv_fwd(ctypes.byref(d), x.data_ptr(), wf.data_ptr(), bias.data_ptr(), out.data_ptr(),
                                     ws.data_ptr(), nbytes, L.stream()), 'pad_conv_fwd')
        ctx.stride, ctx.perm = stride, perm
        ctx.save_for_backward(x, w, out)
        return out

    @staticmethod
    @_amp_bwd
    def backward(ctx, g):
        x, w, out = ctx.saved_tensors
        g_pre = lrelu_pad_backward(g, out)
        mask = [ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2]]
        s = ctx.stride
        dx = None
        if mask[0] and _PAD_DGRAD_FP32:
            # the data gradient on fp32 MFMA (padconv.hip ppd_main_k), straight from the
            # reference-order weight (opt-in: MIOpen's is faster at these shapes)
            dx = pad_conv_dgrad(g_pre, x.shape, w, s, ctx.perm)
            mask[0] = dx is None
        if ctx.perm:        # MIOpen works in the map's channel order (channels-last like x): swap
            C1, Z = ctx.perm  # in, and the gradient back to the reference order (NCHW)
            w = weight_swap(w, C1, Z, cache=True, memory_format=torch.channels_last)
        dx2, dw, db = torch.ops.aten.convolution_backward(g_pre, x, w, [w.shape[0]], [s, s], [0, 0], [1, 1],
                                                          False, [0, 0], 1, mask) if any(mask) else (None,) * 3
        if dx is None:
            dx = dx2
        if ctx.perm and dw is not None:
            dw = weight_swap(dw, Z, C1)
        return dx, dw, db, None, None, None


def pad_conv_weight_fragments_bf16(w, C1=0, Z=0, f0=None):
    """Conv weight [O, C, 3, 3] -> the bf16 K2C kernel's copy [9, ceil32(C)/16, O/32, 64, 8] over the
    map's channel order (padconv.hip ppcb_main_k), through the fp32 mode-0 fragments `f0` (built
    here unless given)."""
    lib = L.load()
    O, C = w.shape[:2]
    if f0 is None:
        f0 = pad_conv_weight_fragments(w, C1, Z)
    out = torch.empty(9, (C + 31) // 32 * 2, O // 32, 64, 8, dtype=torch.bfloat16, device=w.device)
    L.check(lib.vfd_weight_fragments_bf16(4, f0.data_ptr(), out.data_ptr(), O, C, C1, Z, 0, 0, L.stream()),
            'weight_fragments_bf16')
    return out


def pad_conv_bf16_supported(x, stride, out_channels):
    return bool(L.load().vfd_pad_conv_fwd_bf16_workspace(ctypes.byref(pad_conv_desc(x, stride, out_channels))))


def pad_conv_wgrad_bf16_supported(x, stride, out_channels):
    """The bf16 K2C weight gradient (pwb_main_k) accepts this map: its workspace query is non-zero (it
    depends on the channel tiles and the device's CU count); PadConvBF16 takes MIOpen's otherwise."""
    return bool(L.load().vfd_pad_conv_wgrad_bf16_workspace(ctypes.byref(pad_conv_desc(x, stride, out_channels))))


class PadConvBF16(torch.autograd.Function):
    """K2C in bf16 (config 3): the fp32 reflect-padded channels-last map rounded to bf16 as it is
    staged, bf16 weights, v_mfma_f32_32x32x16_bf16 with fp32 accumulation, bias + LeakyReLU in fp32,
    output bf16 (reflect-padded channels-last, the input of the next conv, which autocast runs in
    bf16).  Backward (default): the d pre-activation (LeakyReLU + pad adjoint in fp32) rounded once
    to bf16 is the operand of both hand-written bf16 MFMA gradients — the data gradient
    (padconv.hip ppd_main_k: bf16 weight fragments, fp32 accumulation, fp32 d map, or bf16 with
    VFD_PD_DX_BF16=1) and the weight / bias gradient (projconv.hip pwb_main_k: the map rounded to
    bf16 as it is staged, fp32 accumulation); gradients returned in fp32 (the map, the master
    weight, the bias).  VFD_PC_BF16_BWD=0 (both), VFD_PAD_DGRAD=0 / VFD_PAD_WGRAD=0 (one) restore
    MIOpen's: its fp32 data gradient of the fp32 map and its bf16 weight gradient on bf16 copies;
    shapes the HIP kernels decline (zero workspace) take MIOpen's as well."""

    @staticmethod
    def forward(ctx, x, w, bias, stride, wf=None, perm=None):
        lib = L.load()
        x = _channels_last(x, 'pad_conv input')
        bias = _dev(bias, 'pad_conv bias')
        O = w.shape[0]
        d = pad_conv_desc(x, stride, O)
        nbytes = lib.vfd_pad_conv_fwd_bf16_workspace(ctypes.byref(d))
        if not nbytes:
            raise RuntimeError(f'pad_conv_fwd_bf16: unsupported shape {tuple(x.shape)}, stride {stride}, {O} outputs')
        ho, wo = (x.shape[2] - 3) // stride + 1, (x.shape[3] - 3) // stride + 1
        out = torch.empty(x.shape[0], O, ho + 2, wo + 2, dtype=torch.bfloat16, device=x.device,
                          memory_format=torch.channels_last)
        if wf is None:
            wf = pad_conv_weight_fragments_bf16(_dev(w.detach(), 'pad_conv weight'), *(perm or (0, 0)))
        ws = _ws(nbytes, x.device)
        L.check(lib.vfd_pad_conv_fwd_bf16(ctypes.byref(d), x.data_ptr(), wf.data_ptr(), bias.data_ptr(), out.data_ptr(),
                                          ws.data_ptr(), nbytes, L.stream()), 'pad_conv_fwd_bf16')
        ctx.stride, ctx.perm = stride, perm
        ctx.save_for_backward(x, w, out)
        return out

    @staticmethod
    def backward(ctx, g):
        x, w, out = ctx.saved_tensors
        mask = [ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2]]
        s = ctx.stride
        # d pre-activation (LeakyReLU + pad adjoint in fp32, sign from the bf16 output) rounded once
        # to bf16: the operand of both gradients
        gb = lrelu_pad_backward(g.to(torch.bfloat16), out, dtype=torch.bfloat16)
        cb = torch.ops.aten.convolution_backward
        args = ([w.shape[0]], [s, s], [0, 0], [1, 1], False, [0, 0], 1)
        dx = dw = db = None
        if mask[0] and _PC_BF16_BWD and _PAD_DGRAD:
            # the bf16 data gradient (padconv.hip ppd_main_k<bf16>: bf16 operands, fp32 accumulation,
            # rounded to bf16 as autocast's bf16 conv gradient is, then cast back for an fp32 map)
            dx = pad_conv_dgrad(gb, x.shape, w, s, ctx.perm, torch.bfloat16 if _PD_DX_BF16 else torch.float32)
            if dx is not None:
                dx = dx.to(x.dtype)
        wd = None
        hip_wgrad = _PC_BF16_BWD and _PAD_WGRAD and pad_conv_wgrad_bf16_supported(x, s, w.shape[0])
        if (mask[0] and dx is None) or ((mask[1] or mask[2]) and not hip_wgrad):
            wd = w.detach()
            if ctx.perm:    # MIOpen works in the map's channel order (channels-last like x)
                C1, Z = ctx.perm
                wd = weight_swap(wd, C1, Z, cache=True, memory_format=torch.channels_last)
        if mask[0] and dx is None:
            # MIOpen's data gradient in fp32 from the fp32 pre-activation gradient (its bf16 data
            # gradient of this shape accumulates in an fp32 workspace and then casts to bf16, which
            # the fp32 map's gradient would cast back)
            g32 = lrelu_pad_backward(g.float(), out.float())
            dx = cb(g32, x, wd, *args, [True, False, False])[0]
        if (mask[1] or mask[2]) and hip_wgrad:
            # the bf16 weight / bias gradient on MFMA (projconv.hip pwb_main_k: the fp32 map rounded
            # to bf16 as it is staged), d weight in the map's channel order, then the pose swap
            dw, db = pad_conv_wgrad_bf16(gb, x, w, s, mask[1], mask[2])
            if dw is not None and ctx.perm:
                dw = weight_swap(dw, ctx.perm[1], ctx.perm[0])
            return dx, dw, db, None, None, None
        if mask[1] or mask[2]:
            if wd is None:
                wd = w.detach()
                if ctx.perm:
                    wd = weight_swap(wd, ctx.perm[0], ctx.perm[1], cache=True, memory_format=torch.channels_last)
            _, dw, db = cb(gb, x.to(torch.bfloat16), wd.to(torch.bfloat16), *args, [False, mask[1], mask[2]])
        if dw is not None:
            dw = dw.float()
            if ctx.perm:
                dw = weight_swap(dw, ctx.perm[1], ctx.perm[0])
        return dx, dw, (db.float() if db is not None else None), None, None, None


_DT = {torch.float32: 0, torch.bfloat16: 1}


def _pose_pairs(plan, B, N=None):
    """Frame pairs stacked in a pose batch of B elements over a plan (geometry) of plan.B elements.
    The per-pair slices below are raw pointer offsets into one buffer: the counts are checked here,
    before any launch (the kernels index [plan.B, N] geometry and a pair's slice only)."""
    if B % plan.B:
        raise RuntimeError(f'pose fusion: batch {B} is not a multiple of the geometry batch {plan.B}')
    if N is not None and N != plan.N:
        raise RuntimeError(f'pose fusion: {N} cameras against a plan of {plan.N}')
    return B // plan.B


def _pose_fuse_t(space, plan, feats, dtype, order=None):
    """K2 forward into a fresh map of `dtype` (fusion.hip fuse_pose_fwd_k) -> (map, desc shape).
    feats may stack P frame pairs over the plan's geometry batch ([P * plan.B, N, C, h, w], the
    pose net's pairs in one batch): K2 runs once per pair on its slice with the plan's geometry.
    `order`: an optional voxel order (VoxelSpace.pose_order), index order when None."""
    lib = L.load()
    feats = _dev(feats, 'feats')
    B, N, C = feats.shape[:3]
    P, Bg = _pose_pairs(plan, B, N), plan.B
    hw = feats.shape[3] * feats.shape[4]
    if hw != space.h * space.w:
        raise RuntimeError(f'pose fusion: feature map {tuple(feats.shape[3:])} is not {space.h}x{space.w}')
    feats_cl = torch.empty(B, N, hw, C, device=feats.device)          # [B, N, h*w, C]: one tiled pass
    L.check(lib.vfd_nchw_to_nhwc(feats.data_ptr(), feats_cl.data_ptr(), B * N, C, hw, 0, L.stream()), 'nchw_to_nhwc')
    if L.PROF_ON:                            # timed under its own layout_copy scope (vfd_nchw_to_nhwc)
        L.ALG_BYTES['layout_copy'] += 2 * feats.numel() * 4
    out = torch.empty(B, (C + 1) * space.Z, space.Y + 2, space.X + 2, device=feats.device, dtype=dtype,
                      memory_format=torch.channels_last)
    d = space.desc(Bg, N, C=C)
    fstep, ostep = Bg * N * hw * C * 4, Bg * out[0].numel() * out.element_size()     # bytes per pair
    for p in range(P):
        L.check(lib.vfd_fuse_pose_fwd_t(ctypes.byref(d), plan.mask_lo.data_ptr(), plan.K.data_ptr(),
                                        plan.Einv.data_ptr(), feats_cl.data_ptr() + p * fstep,
                                        out.data_ptr() + p * ostep, _DT[dtype],
                                        L.ptr(order), order.shape[1] if order is not None else 0, L.stream()),
                'fuse_pose_fwd')
    return out


def _pose_unfuse(space, plan, shape, g):
    """K2 backward: d map (fp32 or bf16, channels-last) -> d feats [B, N, C, h, w] fp32 (fuse_pose_bwd_k);
    once per stacked frame pair, as the forward."""
    lib = L.load()
    B, N, C = shape[:3]
    P, Bg = _pose_pairs(plan, B, N), plan.B
    want = (B, (C + 1) * space.Z, space.Y + 2, space.X + 2)
    if tuple(g.shape) != want or tuple(shape[3:]) != (space.h, space.w):
        raise RuntimeError(f'pose fusion backward: map gradient {tuple(g.shape)} / features {tuple(shape)} '
                           f'do not match the map {want}')
    g = _nhwc(g, 'grad') if g.dtype in _DT else _channels_last(g, 'grad')
    dfeats = torch.empty(shape, device=g.device)
    d = space.desc(Bg, N, C=C)
    plan.build().wait()
    gstep, fstep = Bg * g[0].numel() * g.element_size(), Bg * dfeats[0].numel() * 4       # bytes per pair
    for p in range(P):
        L.check(lib.vfd_fuse_pose_bwd_t(ctypes.byref(d), plan.buf.data_ptr(), plan.counts.data_ptr(),
                                        g.data_ptr() + p * gstep, _DT[g.dtype], dfeats.data_ptr() + p * fstep,
                                        L.stream()), 'fuse_pose_bwd')
    return dfeats


def pose_conv_bf16_supported(space, B, C, stride, out_channels):
    """PoseConvBF16 applies: the bf16 map's K2C forward / weight gradient accept its shape."""
    shape = (B, (C + 1) * space.Z, space.Y + 2, space.X + 2)
    d = L.ConvDesc(shape[0], shape[2], shape[3], shape[1], stride, out_channels)
    lib = L.load()
    return bool(_PC_BF16_BWD and _PAD_DGRAD and _PAD_WGRAD and lib.vfd_pad_conv_fwd_bf16_workspace(ctypes.byref(d))
                and lib.vfd_pad_conv_wgrad_bf16_workspace(ctypes.byref(d))
                and lib.vfd_pad_conv_dgrad_bf16_workspace(ctypes.byref(d)))


class PoseConvBF16(torch.autograd.Function):
    """K2 + K2C under config 3 as one autograd node: the pose gather writes the BEV map in bf16 —
    exactly the values the bf16 K2C stages from the fp32 map (rounded to nearest even), so the conv,
    its weight gradient and the map's gradient are those of FusePose -> PadConvBF16 — at half the
    map's bytes (written by K2, read by the conv's forward and weight gradient).  The map stays
    inside this node, so its gradient (the K2C data gradient, fp32) goes straight into K2's
    backward with no dtype round trip.  Output: LeakyReLU(conv + bias) bf16, reflect-padded
    channels-last [B, 256, Ho+2, Wo+2] (as PadConvBF16)."""

    @staticmethod
    def forward(ctx, space, plan, feats, w, bias, stride, wf, perm):
        lib = L.load()
        feats = feats.float()
        x = _pose_fuse_t(space, plan, feats, torch.bfloat16)
        if ctx.needs_input_grad[2]:
            plan.build()            # the backward's index (kept in the order the step issued it)
        bias = _dev(bias, 'pad_conv bias').float()
        O = w.shape[0]
        d = pad_conv_desc(x, stride, O)
        nbytes = lib.vfd_pad_conv_fwd_bf16_workspace(ctypes.byref(d))
        if not nbytes:
            raise RuntimeError(f'pad_conv_fwd_bf16: unsupported shape {tuple(x.shape)}, stride {stride}, {O} outputs')
        ho, wo = (x.shape[2] - 3) // stride + 1, (x.shape[3] - 3) // stride + 1
        out = torch.empty(x.shape[0], O, ho + 2, wo + 2, dtype=torch.bfloat16, device=x.device,
                          memory_format=torch.channels_last)
        ws = _ws(nbytes, x.device)
        L.check(lib.vfd_pad_conv_fwd_bf16_t(ctypes.byref(d), x.data_ptr(), 1, wf.data_ptr(), bias.data_ptr(),
                                            out.data_ptr(), ws.data_ptr(), nbytes, L.stream()), 'pad_conv_fwd_bf16')
        ctx.space, ctx.plan, ctx.shape, ctx.stride, ctx.perm = space, plan, tuple(feats.shape), stride, perm
        ctx.save_for_backward(x, w, out)
        return out

    @staticmethod
    def backward(ctx, g):
        x, w, out = ctx.saved_tensors
        s = ctx.stride
        gb = lrelu_pad_backward(g.to(torch.bfloat16), out, dtype=torch.bfloat16)
        dfeats = dw = db = None
        if ctx.needs_input_grad[2]:
            # the bf16 data gradient (ppd_main_k: fp32 sums rounded to bf16 as autocast's conv gradient
            # is, VFD_PD_DX_BF16=0 keeps them fp32) straight into K2's backward
            dmap = pad_conv_dgrad(gb, x.shape, w, s, ctx.perm, torch.bfloat16 if _PD_DX_BF16 else torch.float32)
            dfeats = _pose_unfuse(ctx.space, ctx.plan, ctx.shape, dmap)
        if ctx.needs_input_grad[3] or ctx.needs_input_grad[4]:
            dw, db = pad_conv_wgrad_bf16(gb, x, w, s, ctx.needs_input_grad[3], ctx.needs_input_grad[4])
            if dw is not None and ctx.perm:
                dw = weight_swap(dw, ctx.perm[1], ctx.perm[0])
        return None, None, dfeats, dw, db, None, None, None


def lrelu_pad_backward(g, out, slope=0.1, dtype=None):
    """d pre-activation of LeakyReLU(slope) + reflect pad(1) from the channels-last gradient of the
    padded output g and that output (fused, deterministic: reflectpad.hip) -> NHWC [n, C, h, w].
    g and out fp32 or bf16 (the same type); the result in `dtype` (default g's), computed in fp32."""
    lib = L.load()
    if g.dtype not in _DT:
        g = g.float()
    g = _nhwc(g, 'grad')
    out = _nhwc(out.to(g.dtype), 'output')
    dtype = dtype or g.dtype
    n, C, hp, wp = g.shape
    gp = torch.empty(n, C, hp - 2, wp - 2, device=g.device, dtype=dtype, memory_format=torch.channels_last)
    L.check(lib.vfd_lrelu_pad1_bwd_nhwc_t(g.data_ptr(), out.data_ptr(), gp.data_ptr(), n, hp - 2, wp - 2, C, slope,
                                          _DT[g.dtype], _DT[dtype], L.stream()), 'lrelu_pad1_bwd_nhwc')
    if L.PROF_ON:                            # g in, the output's interior in, gp out
        L.ALG_BYTES['reflect_pad'] += (g.numel() + gp.numel()) * g.element_size() + gp.numel() * gp.element_size()
    return gp


class ProjConv(torch.autograd.Function):
    """K3C: voxel features [B,V,Cv] -> LeakyReLU(conv3x3_reflect(frustum samples) + bias): K3's
    trilinear resampling fused into reduce_dim's first conv (fp32 MFMA implicit GEMM; the
    [B*N, Cv*D, h, w] frustum features never reach HBM).  Output: the reflect-padded
    channels-last input of reduce_dim's second conv, logical [B*N, O, h+2, w+2].

    When a gradient is needed the kernel also writes the frustum features themselves (K3's padded
    channels-last layout) as a side output.  Backward: the LeakyReLU + pad adjoint, the data
    gradient (`vfd_proj_conv_dgrad`) into K3's planned backward (d voxel), and the weight / bias
    gradient (`vfd_proj_conv_wgrad`, over the side output); all fp32 MFMA, fixed summation order."""

    @staticmethod
    @_amp_fwd
    def forward(ctx, space, vox, invK, E, w0, bias):
        lib = L.load()
        vox, invK, E = (_dev(t, n) for t, n in ((vox, 'voxel'), (invK, 'inv_K'), (E, 'extrinsics')))
        w0, bias = _dev(w0, 'reduce_dim weight'), _dev(bias, 'reduce_dim bias')
        B, V, Cv = vox.shape
        N, O = E.shape[1], w0.shape[0]
        wq = proj_conv_weight_fragments(w0, Cv, space.D)
        out = torch.empty(B * N, O, space.h + 2, space.w + 2, device=vox.device, memory_format=torch.channels_last)
        need_x = ctx.needs_input_grad[1] or ctx.needs_input_grad[4]
        x = (torch.empty(B * N, Cv * space.D, space.h + 2, space.w + 2, device=vox.device,
                         memory_format=torch.channels_last) if need_x else None)
        d = space.desc(B, N, Cv=Cv)
        nbytes = lib.vfd_proj_conv_fwd_workspace(ctypes.byref(d))
        ws = _ws(nbytes, vox.device)
        L.check(lib.vfd_proj_conv_fwd(ctypes.byref(d), vox.data_ptr(), invK.data_ptr(), E.data_ptr(), wq.data_ptr(),
                                      bias.data_ptr(), O, out.data_ptr(), x.data_ptr() if need_x else None,
                                      ws.data_ptr(), nbytes, L.stream()),
                'proj_conv_fwd')
        # the data gradient's folded form (reflect-pad adjoint inside the GEMM, interior only) when
        # it applies; K3's plan is then built for a folded d_out (pad_out = 2)
        d.pad_out = 2 if (_PC_DGRAD and _PC_FOLD and lib.vfd_proj_conv_dgrad_workspace(ctypes.byref(
            space.desc(B, N, Cv=Cv, pad_out=2)))) else 1
        ctx.pad_out = d.pad_out
        ctx.space, ctx.shape = space, (B, N, V, Cv, O)
        ctx.plan = None
        if ctx.needs_input_grad[1]:
            nbytes = lib.vfd_voxel_project_plan_bytes(ctypes.byref(d))
            ctx.plan = torch.empty(nbytes, dtype=torch.uint8, device=vox.device)
            L.check(lib.vfd_voxel_project_plan(ctypes.byref(d), invK.data_ptr(), E.data_ptr(), ctx.plan.data_ptr(),
                                               nbytes, L.stream()), 'voxel_project_plan')
        ctx.save_for_backward(w0, out, x)
        return out

    @staticmethod
    @_amp_bwd
    def backward(ctx, g):
        lib = L.load()
        w0, out, x = ctx.saved_tensors
        space = ctx.space
        B, N, V, Cv, O = ctx.shape
        d = space.desc(B, N, Cv=Cv, pad_out=ctx.pad_out)
        # adjoint of the reflect padding, then of the LeakyReLU (its sign from the output): one kernel
        g_pre = lrelu_pad_backward(g, out)
        if x is None:   # only the bias gradient was asked for
            x = torch.empty(B * N, Cv * space.D, space.h + 2, space.w + 2, device=g.device,
                            memory_format=torch.channels_last)
        mask = (ctx.needs_input_grad[1], ctx.needs_input_grad[4], ctx.needs_input_grad[5])
        cb = torch.ops.aten.convolution_backward
        args = ([O], [1, 1], [0, 0], [1, 1], False, [0, 0], 1)
        dx = None
        if mask[0] and _PC_DGRAD:
            nbytes = lib.vfd_proj_conv_dgrad_workspace(ctypes.byref(d))
            if nbytes:
                # the fused data gradient (fp32 MFMA, projconv.hip)
                wd = proj_conv_dgrad_weight(w0, Cv, space.D)
                dx = torch.empty(B * N, Cv * space.D, space.h + 2, space.w + 2, device=g.device,
                                 memory_format=torch.channels_last)
                ws = _ws(nbytes, g.device)
                L.check(lib.vfd_proj_conv_dgrad(ctypes.byref(d), g_pre.data_ptr(), wd.data_ptr(), dx.data_ptr(),
                                                ws.data_ptr(), nbytes, L.stream()), 'proj_conv_dgrad')
        dw0 = db0 = None
        wmask = [mask[1], mask[2]]          # what MIOpen still has to compute
        if (mask[1] or mask[2]) and _PC_WGRAD:
            nbytes = lib.vfd_proj_conv_wgrad_workspace(ctypes.byref(d))
            if nbytes:
                # the fused weight / bias gradient (fp32 MFMA, projconv.hip), straight into the
                # reference's channel order c*D + d (no swap)
                dw0 = torch.empty(w0.shape, device=g.device) if mask[1] else None
                db0 = torch.empty(O, device=g.device) if mask[2] else None
                ws = _ws(nbytes, g.device)
                L.check(lib.vfd_proj_conv_wgrad(ctypes.byref(d), g_pre.data_ptr(), x.data_ptr(),
                                                dw0.data_ptr() if mask[1] else None,
                                                db0.data_ptr() if mask[2] else None, ws.data_ptr(), nbytes,
                                                L.stream()), 'proj_conv_wgrad')
                wmask = [False, False]
        dw = db = None
        if dx is not None:
            if any(wmask):
                # the weight gradient reads only the weight's shape: w0 has it (no permuted copy)
                _, dw, db = cb(g_pre, x, w0, *args, [False] + wmask)
        elif mask[0] or any(wmask):
            dx, dw, db = cb(g_pre, x, proj_conv_weight(w0, Cv, space.D), *args, [mask[0]] + wmask)
        dvox = None
        if mask[0]:
            dx = _channels_last(dx, 'd frustum features')
            dvox = torch.empty(B, V, Cv, device=g.device)
            L.check(lib.vfd_voxel_project_bwd_planned(ctypes.byref(d), dx.data_ptr(), ctx.plan.data_ptr(),
                                                      ctx.plan.numel(), dvox.data_ptr(), L.stream()),
                    'voxel_project_bwd')
        if dw is not None:
            dw0 = weight_swap(dw, space.D, Cv)      # d*Cv + c -> the reference's c*D + d
        if db is not None:
            db0 = db
        ctx.plan = None
        return None, dvox, None, None, dw0, db0


def proj_conv_dgrad_weight_bf16(w, Cv, D):
    """reduce_dim[0] weight -> the bf16 data-gradient kernel's copy [9 flipped taps, O/16, np/32, 64, 8]
    (projconv.hip pcg_main_k<bf16>; through the fp32 mode-2 copy), rounded to nearest even."""
    lib = L.load()
    w = _dev(w.detach(), 'conv weight')
    O = w.shape[0]
    f2 = proj_conv_dgrad_weight(w, Cv, D)
    npad = f2.shape[2]
    out = torch.empty(9, O // 16, npad // 32, 64, 8, dtype=torch.bfloat16, device=w.device)
    L.check(lib.vfd_weight_fragments_bf16(5, f2.data_ptr(), out.data_ptr(), O, 0, 0, 0, Cv, D, L.stream()),
            'weight_fragments_bf16')
    return out


def proj_conv_weight_fragments_bf16(w, Cv, D):
    """reduce_dim[0] weight [O, Cv*D, 3, 3] (reference channel c*D + d) -> the bf16 K3C kernel's
    fragment copy [D, 9, Cv/16, O/32, 64, 8] (projconv.hip pcvb_main_k), rounded to nearest even."""
    lib = L.load()
    w = _dev(w.detach(), 'conv weight')
    O = w.shape[0]
    out = torch.empty(D, 9, Cv // 16, O // 32, 64, 8, dtype=torch.bfloat16, device=w.device)
    L.check(lib.vfd_weight_fragments_bf16(3, w.data_ptr(), out.data_ptr(), O, Cv * D, 0, 0, Cv, D, L.stream()),
            'weight_fragments_bf16')
    return out


class ProjConvBF16(torch.autograd.Function):
    """K3C in bf16 (config 3: the reference autocasts the fusion features to bf16,
    volumetric_fusionnet.py:105-114): the fp32 trilinear samples of the fp32 voxel grid rounded to
    bf16 in LDS, bf16 weights, v_mfma_f32_32x32x16_bf16 with fp32 accumulation, bias + LeakyReLU
    in fp32, output bf16 (the reflect-padded channels-last input of reduce_dim's second conv,
    which autocast runs in bf16).  Backward (default): the d pre-activation (LeakyReLU + pad
    adjoint in fp32) rounded once to bf16 feeds the hand-written bf16 MFMA gradients — the data
    gradient (projconv.hip pch_main_k, folded reflect-pad adjoint, bf16 weight fragments, fp32
    accumulation, fp32 d frustum features) into K3's fp32 planned backward, and the weight / bias
    gradient (pwb_main_k over the bf16 frustum features the forward writes as its side output, fp32
    accumulation, d weight straight in the reference channel order).  VFD_PC_BF16_BWD=0 (or
    VFD_PC_DGRAD=0 for the data gradient) restores MIOpen's bf16 gradients; shapes the HIP kernels
    decline (zero workspace) take MIOpen's as well.  Gradients to the fp32 voxels / master weight /
    bias come back in fp32."""

    @staticmethod
    def forward(ctx, space, vox, invK, E, w0, bias):
        lib = L.load()
        vox, invK, E = (_dev(t, n) for t, n in ((vox, 'voxel'), (invK, 'inv_K'), (E, 'extrinsics')))
        bias = _dev(bias, 'reduce_dim bias')
        B, V, Cv = vox.shape
        N, O = E.shape[1], w0.shape[0]
        wq = proj_conv_weight_fragments_bf16(w0, Cv, space.D)
        cl = torch.channels_last
        out = torch.empty(B * N, O, space.h + 2, space.w + 2, dtype=torch.bfloat16, device=vox.device, memory_format=cl)
        need_x = ctx.needs_input_grad[1] or ctx.needs_input_grad[4]
        x = (torch.empty(B * N, Cv * space.D, space.h + 2, space.w + 2, dtype=torch.bfloat16, device=vox.device,
                         memory_format=cl) if need_x else None)
        d = space.desc(B, N, Cv=Cv)
        nbytes = lib.vfd_proj_conv_fwd_workspace(ctypes.byref(d))
        ws = _ws(nbytes, vox.device)
        # the bf16 data gradient is the folded form: K3's plan built for a folded d_out (pad_out = 2)
        ctx.pad_out = 2 if (_PC_DGRAD and _PC_BF16_BWD and lib.vfd_proj_conv_dgrad_bf16_workspace(ctypes.byref(
            space.desc(B, N, Cv=Cv, pad_out=2)))) else 1
        L.check(lib.vfd_proj_conv_fwd_bf16(ctypes.byref(d), vox.data_ptr(), invK.data_ptr(), E.data_ptr(),
                                           wq.data_ptr(), bias.data_ptr(), O, out.data_ptr(),
                                           x.data_ptr() if need_x else None, ws.data_ptr(), nbytes, L.stream()),
                'proj_conv_fwd_bf16')
        ctx.space, ctx.shape = space, (B, N, V, Cv, O)
        ctx.plan = None
        if ctx.needs_input_grad[1]:
            d.pad_out = ctx.pad_out
            nbytes = lib.vfd_voxel_project_plan_bytes(ctypes.byref(d))
            ctx.plan = torch.empty(nbytes, dtype=torch.uint8, device=vox.device)
            L.check(lib.vfd_voxel_project_plan(ctypes.byref(d), invK.data_ptr(), E.data_ptr(), ctx.plan.data_ptr(),
                                               nbytes, L.stream()), 'voxel_project_plan')
        ctx.save_for_backward(w0, out, x)
        return out

    @staticmethod
    def backward(ctx, g):
        lib = L.load()
        w0, out, x = ctx.saved_tensors
        space = ctx.space
        B, N, V, Cv, O = ctx.shape
        d = space.desc(B, N, Cv=Cv, pad_out=ctx.pad_out)
        # adjoint of the reflect padding and the LeakyReLU (fp32 arithmetic, sign from the bf16
        # output), one bf16 rounding: the bf16 operand of the gradients
        g_pre = lrelu_pad_backward(g.to(torch.bfloat16), out, dtype=torch.bfloat16)
        mask = (ctx.needs_input_grad[1], ctx.needs_input_grad[4], ctx.needs_input_grad[5])
        dx = dw = db = None
        if mask[0] and ctx.pad_out == 2:
            # the folded bf16 data gradient (bf16 MFMA, fp32 accumulation, projconv.hip pcg_main_k)
            wd = proj_conv_dgrad_weight_bf16(w0, Cv, space.D)
            nbytes = lib.vfd_proj_conv_dgrad_bf16_workspace(ctypes.byref(d))
            dx = torch.empty(B * N, Cv * space.D, space.h + 2, space.w + 2, device=g.device,
                             memory_format=torch.channels_last)
            ws = _ws(nbytes, g.device)
            L.check(lib.vfd_proj_conv_dgrad_bf16(ctypes.byref(d), g_pre.data_ptr(), wd.data_ptr(), dx.data_ptr(),
                                                 ws.data_ptr(), nbytes, L.stream()), 'proj_conv_dgrad_bf16')
        need_dx = mask[0] and dx is None
        dw0 = None
        if (mask[1] or mask[2]) and _PC_BF16_BWD and x is not None:
            # the bf16 weight / bias gradient on MFMA (projconv.hip pwb_main_k), d weight straight
            # into the reference channel order c*D + d
            nbytes = lib.vfd_proj_conv_wgrad_bf16_workspace(ctypes.byref(d))
            if nbytes:
                dw0 = torch.empty(w0.shape, device=g.device) if mask[1] else None
                db = torch.empty(O, device=g.device) if mask[2] else None
                ws = _ws(nbytes, g.device)
                L.check(lib.vfd_proj_conv_wgrad_bf16(ctypes.byref(d), g_pre.data_ptr(), x.data_ptr(), L.ptr(dw0),
                                                     L.ptr(db), ws.data_ptr(), nbytes, L.stream()),
                        'proj_conv_wgrad_bf16')
                mask = (mask[0], False, False)
        if x is None:   # only the bias gradient was asked for (the forward wrote no side output)
            db = g_pre.float().sum((0, 2, 3))
        elif need_dx or mask[1] or mask[2]:
            wb = proj_conv_weight(w0.detach(), Cv, space.D).to(torch.bfloat16)
            dx2, dw, db = torch.ops.aten.convolution_backward(g_pre, x, wb, [O], [1, 1], [0, 0], [1, 1], False, [0, 0],
                                                              1, [need_dx, mask[1], mask[2]])
            if need_dx:
                dx = dx2
        dvox = None
        if ctx.needs_input_grad[1]:
            dxf = dx.float().contiguous(memory_format=torch.channels_last)
            dvox = torch.empty(B, V, Cv, device=g.device)
            L.check(lib.vfd_voxel_project_bwd_planned(ctypes.byref(d), dxf.data_ptr(), ctx.plan.data_ptr(),
                                                      ctx.plan.numel(), dvox.data_ptr(), L.stream()),
                    'voxel_project_bwd')
        if mask[1]:         # MIOpen's d weight: d*Cv + c -> the reference's c*D + d
            dw0 = weight_swap(dw.float(), space.D, Cv)
        ctx.plan = None
        return None, dvox, None, None, dw0, (db.float() if ctx.needs_input_grad[5] and db is not None else None)


# =============================================================================================
# View synthesis (K4)
# =============================================================================================
class ViewPlan:
    """Warp table of every target camera (view_rendering.py:118-198 enumeration order).

    Warps of camera c: first the temporal warps (frame_ids[1:], source = c), then — when the
    spatial terms are on — for every frame slot of frame_ids the neighbours rel_cam_list[c] that
    exist (< num_cams).  Each entry: (frame slot, source camera, overlap slot or -1).
    """

    def __init__(self, cfg, device):
        t, dt = cfg['training'], cfg['data']
        self.frames = list(t['frame_ids'])
        self.N = int(dt['num_cams'])
        self.T = len(self.frames) - 1
        spatial = bool(t['spatio'] or t['spatio_temporal'])
        if spatial and not (t['spatio'] and t['spatio_temporal']):
            raise KeyError('the reference needs spatio and spatio_temporal together '
                           '(pose.py:66-96 builds (0, cam) before the temporal entries)')
        self.F = len(self.frames) if spatial else 0
        self.intensity_align = bool(t['intensity_align'])
        rel = dt['rel_cam_list']
        self.entries = []
        for c in range(self.N):
            ent = [(1 + i, c, -1) for i in range(self.T)]
            if spatial:
                for fs in range(len(self.frames)):
                    for s in rel[c]:
                        if s < self.N:
                            ent.append((fs, s, fs))
            self.entries.append(ent)
        self.n_warp = max(len(e) for e in self.entries)
        tab = torch.full((self.N, self.n_warp, 3), -1, dtype=torch.int32)
        for c, ent in enumerate(self.entries):
            for w, e in enumerate(ent):
                tab[c, w] = torch.tensor(e, dtype=torch.int32)
        self.tab = tab.to(device)

    def desc(self, B, H, W, colors, cam_begin=0, cam_count=None):
        d = L.ViewDesc()
        d.B, d.N, d.H, d.W = B, self.N, H, W
        d.n_warp, d.n_temporal, d.n_overlap = self.n_warp, self.T, self.F
        d.intensity_align = int(self.intensity_align)
        d.cam_begin = cam_begin
        d.cam_count = self.N - cam_begin if cam_count is None else cam_count
        for i, c in enumerate(colors):
            d.color[i] = c.data_ptr()
        d.warp_tab = self.tab.data_ptr()
        return d


class ViewSynthesis(torch.autograd.Function):
    """K4: every warp of cameras [cam_begin, cam_begin+Nt) -> (color, color_mask, overlap, overlap_mask).

    depth [B,Nt,H,W], invK [B,Nt,4,4], M [B,Nt,n_warp,3,4] = (K_src @ T)[:3], mask [B,N,H,W],
    colors: one [B,N,3,H,W] tensor per frame slot.  Gradients flow to depth and M.
    """

    @staticmethod
    def forward(ctx, plan, cam_begin, depth, invK, M, mask, *colors):
        lib = L.load()
        depth, invK, M, mask = (_dev(t, n) for t, n in ((depth, 'depth'), (invK, 'inv_K'), (M, 'KT'), (mask, 'mask')))
        colors = [_dev(c, 'color') for c in colors]
        B, Nt, H, W = depth.shape
        d = plan.desc(B, H, W, colors, cam_begin, Nt)
        dev = depth.device
        color = torch.empty(B, Nt, plan.T, 3, H, W, device=dev)
        cmask = torch.empty(B, Nt, plan.T, H, W, device=dev)
        ovl = torch.empty(B, Nt, max(plan.F, 1), 3, H, W, device=dev)
        omask = torch.empty(B, Nt, max(plan.F, 1), H, W, device=dev)
        coef = torch.empty(B, Nt, plan.n_warp, 4, device=dev)
        nbytes = lib.vfd_view_workspace_bytes(ctypes.byref(d))
        ws = _ws(nbytes, dev)
        L.check(lib.vfd_view_fwd(ctypes.byref(d), depth.data_ptr(), invK.data_ptr(), M.data_ptr(), mask.data_ptr(),
                                 color.data_ptr(), cmask.data_ptr(), ovl.data_ptr(), omask.data_ptr(),
                                 coef.data_ptr(), ws.data_ptr(), nbytes, L.stream()), 'view_fwd')
        ctx.plan, ctx.cam_begin = plan, cam_begin
        ctx.save_for_backward(depth, invK, M, mask, coef, *colors)
        ctx.mark_non_differentiable(cmask, omask)
        if plan.F == 0:
            ovl, omask = ovl[:, :, :0], omask[:, :, :0]
        return color, cmask, ovl, omask

    @staticmethod
    def backward(ctx, g_color, g_cmask, g_ovl, g_omask):
        lib = L.load()
        depth, invK, M, mask, coef, *colors = ctx.saved_tensors
        plan = ctx.plan
        B, Nt, H, W = depth.shape
        d = plan.desc(B, H, W, colors, ctx.cam_begin, Nt)
        g_color = _dev(g_color, 'grad') if g_color is not None else None
        g_ovl = _dev(g_ovl, 'grad') if (g_ovl is not None and plan.F > 0) else None
        d_depth = torch.empty_like(depth)
        d_M = torch.empty_like(M)
        nbytes = lib.vfd_view_workspace_bytes(ctypes.byref(d))
        ws = _ws(nbytes, depth.device)
        L.check(lib.vfd_view_bwd(ctypes.byref(d), depth.data_ptr(), invK.data_ptr(), M.data_ptr(), mask.data_ptr(),
                                 coef.data_ptr(), L.ptr(g_color), L.ptr(g_ovl), d_depth.data_ptr(), d_M.data_ptr(),
                                 ws.data_ptr(), nbytes, L.stream()), 'view_bwd')
        return (None, None, d_depth, None, d_M, None) + (None,) * len(colors)


class DepthSynthesis(torch.autograd.Function):
    """get_virtual_depth of every (target camera, source slot) (view_rendering.py:84-116,
    201-241) in one launch: aug_depth, depth, mask [B,N,H,W], invK [B,N,4,4], M [B,N,S,3,4] =
    (K_src @ T^-1)[:3], zrow [B,N,S,4] = T[2] -> (tform_depth, tform_mask) [B,N,S,H,W].
    Gradients flow to aug_depth (sample coordinates) and depth (sampled values)."""

    @staticmethod
    def forward(ctx, src_tab, min_depth, max_depth, aug_depth, depth, mask, invK, M, zrow):
        lib = L.load()
        aug_depth, depth, mask, invK, M, zrow = (_dev(t, n) for t, n in (
            (aug_depth, 'aug depth'), (depth, 'depth'), (mask, 'mask'), (invK, 'inv_K'), (M, 'KT'), (zrow, 'T')))
        B, N, H, W = depth.shape
        S = src_tab.shape[1]
        d = DepthSynthesis.desc(src_tab, min_depth, max_depth, B, N, H, W)
        out_d = torch.empty(B, N, S, H, W, device=depth.device)
        out_m = torch.empty_like(out_d)
        L.check(lib.vfd_depth_syn_fwd(ctypes.byref(d), aug_depth.data_ptr(), depth.data_ptr(), mask.data_ptr(),
                                      invK.data_ptr(), M.data_ptr(), zrow.data_ptr(), out_d.data_ptr(),
                                      out_m.data_ptr(), L.stream()), 'depth_syn_fwd')
        ctx.src_tab, ctx.range = src_tab, (min_depth, max_depth)
        ctx.save_for_backward(aug_depth, depth, mask, invK, M, zrow)
        ctx.mark_non_differentiable(out_m)
        return out_d, out_m

    @staticmethod
    def desc(src_tab, min_depth, max_depth, B, N, H, W):
        d = L.DepthSynDesc()
        d.B, d.N, d.H, d.W, d.S = B, N, H, W, src_tab.shape[1]
        d.min_depth, d.max_depth = float(min_depth), float(max_depth)
        d.src_tab = src_tab.data_ptr()
        return d

    @staticmethod
    def backward(ctx, g, _g_mask):
        lib = L.load()
        aug_depth, depth, mask, invK, M, zrow = ctx.saved_tensors
        B, N, H, W = depth.shape
        d = DepthSynthesis.desc(ctx.src_tab, *ctx.range, B, N, H, W)
        g = _dev(g, 'grad')
        d_aug = torch.empty_like(aug_depth)
        d_depth = torch.empty_like(depth)
        if deterministic():          # exact fixed-point sums of the scattered source-depth gradient
            nbytes = lib.vfd_depth_syn_bwd_ordered_workspace(ctypes.byref(d))
            ws = _ws(nbytes, depth.device)
            L.check(lib.vfd_depth_syn_bwd_ordered(ctypes.byref(d), aug_depth.data_ptr(), depth.data_ptr(),
                                                  mask.data_ptr(), invK.data_ptr(), M.data_ptr(), zrow.data_ptr(),
                                                  g.data_ptr(), d_aug.data_ptr(), d_depth.data_ptr(), ws.data_ptr(),
                                                  nbytes, L.stream()), 'depth_syn_bwd_ordered')
        else:
            L.check(lib.vfd_depth_syn_bwd(ctypes.byref(d), aug_depth.data_ptr(), depth.data_ptr(), mask.data_ptr(),
                                          invK.data_ptr(), M.data_ptr(), zrow.data_ptr(), g.data_ptr(),
                                          d_aug.data_ptr(), d_depth.data_ptr(), L.stream()), 'depth_syn_bwd')
        return None, None, None, d_aug, d_depth, None, None, None, None


# =============================================================================================
# Photometric losses (K5) and smoothness
# =============================================================================================
class PhotoLoss(torch.autograd.Function):
    """K5: masked reprojection / spatial / spatio-temporal losses of cameras [cam_begin, +Nt).

    Returns (losses [Nt,3] (differentiable), reproj plane, auto-mask, spatial mask) with planes
    [B,Nt,H,W].  `noise` ([Nt,B,T,H,W], already scaled like `1e-5 * randn`) or None for the
    in-kernel counter RNG seeded by `seed`.
    """

    @staticmethod
    def forward(ctx, plan, cam_begin, seed, noise, target, ref_mask, color, ovl, omask, *idents):
        # seed: int, or (int, int64 device counter) — the counter is read by the kernel (graph replay)
        lib = L.load()
        target, ref_mask, color = (_dev(t, n) for t, n in ((target, 'target'), (ref_mask, 'mask'), (color, 'color')))
        ovl, omask = _dev(ovl, 'overlap'), _dev(omask, 'overlap mask')
        idents = [_dev(t, 'identity source') for t in idents]
        if noise is not None:
            noise = _dev(noise, 'noise')
        B, Nt, T, _, H, W = color.shape
        dev = color.device
        d = PhotoLoss.desc(plan, B, H, W, cam_begin, Nt, seed, noise is not None, idents)
        reproj = torch.empty(B, Nt, H, W, device=dev)
        automask = torch.empty_like(reproj)
        spatio = torch.zeros_like(reproj) if plan.F > 0 else torch.empty(0, device=dev)
        sel = torch.empty(B, Nt, H, W, dtype=torch.uint8, device=dev)
        sums = torch.empty(Nt, 6, dtype=torch.float64, device=dev)
        losses = torch.empty(Nt, 3, device=dev)
        nbytes = lib.vfd_photo_workspace_bytes(ctypes.byref(d))
        ws = _ws(nbytes, dev)
        L.check(lib.vfd_photo_fwd(ctypes.byref(d), target.data_ptr(), color.data_ptr(), L.ptr(ovl),
                                  ref_mask.data_ptr(), L.ptr(omask), L.ptr(noise), reproj.data_ptr(),
                                  automask.data_ptr(), L.ptr(spatio) if plan.F > 0 else None, sel.data_ptr(),
                                  sums.data_ptr(), losses.data_ptr(), ws.data_ptr(), nbytes, L.stream()), 'photo_fwd')
        ctx.plan, ctx.cam_begin, ctx.seed, ctx.n_id = plan, cam_begin, seed, len(idents)
        ctx.save_for_backward(target, ref_mask, color, ovl, omask, sel, sums, *idents)
        ctx.mark_non_differentiable(reproj, automask, spatio)
        return losses, reproj, automask, spatio

    @staticmethod
    def desc(plan, B, H, W, cam_begin, Nt, seed, has_noise, idents):
        d = L.PhotoDesc()
        d.B, d.N, d.H, d.W = B, plan.N, H, W
        d.T, d.F = plan.T, plan.F
        d.cam_begin, d.cam_count = cam_begin, Nt
        if isinstance(seed, tuple):
            seed, counter = seed
            d.step = counter.data_ptr()
        d.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        d.noise_scale = 1.0 if has_noise else 1e-5
        for i, t in enumerate(idents):
            d.ident[i] = t.data_ptr()
        return d

    @staticmethod
    def backward(ctx, g_losses, g_reproj, g_auto, g_spatio):
        lib = L.load()
        target, ref_mask, color, ovl, omask, sel, sums, *idents = ctx.saved_tensors
        plan = ctx.plan
        B, Nt, T, _, H, W = color.shape
        d = PhotoLoss.desc(plan, B, H, W, ctx.cam_begin, Nt, ctx.seed, True, idents)
        msum = sums[:, 1::2].float()                                   # M_reproj, M_spatio, M_st
        gcoef = (_dev(g_losses, 'grad') / (msum + 1e-8)).contiguous()
        d_color = torch.empty_like(color)
        d_ovl = torch.empty_like(ovl)
        L.check(lib.vfd_photo_bwd(ctypes.byref(d), target.data_ptr(), color.data_ptr(), L.ptr(ovl),
                                  ref_mask.data_ptr(), L.ptr(omask), sel.data_ptr(), gcoef.data_ptr(),
                                  d_color.data_ptr(), L.ptr(d_ovl), L.stream()), 'photo_bwd')
        return (None, None, None, None, None, None, d_color, d_ovl if plan.F > 0 else None, None) + (None,) * ctx.n_id


class Smoothness(torch.autograd.Function):
    """Edge-aware smoothness of disp / mean(disp): disp [B,Nt,H,W], color [B,Nt,3,H,W] -> [Nt]."""

    @staticmethod
    def forward(ctx, disp, color):
        lib = L.load()
        disp, color = _dev(disp, 'disp'), _dev(color, 'color')
        B, Nt, H, W = disp.shape
        sums = torch.empty(B * Nt, 3, dtype=torch.float64, device=disp.device)
        loss = torch.empty(Nt, device=disp.device)
        nbytes = lib.vfd_smooth_workspace_bytes(B, Nt, H, W)
        ws = _ws(nbytes, disp.device)
        L.check(lib.vfd_smooth_fwd(B, Nt, H, W, disp.data_ptr(), color.data_ptr(), sums.data_ptr(), loss.data_ptr(),
                                   ws.data_ptr(), nbytes, L.stream()), 'smooth_fwd')
        ctx.save_for_backward(disp, color, sums)
        return loss

    @staticmethod
    def backward(ctx, g):
        lib = L.load()
        disp, color, sums = ctx.saved_tensors
        B, Nt, H, W = disp.shape
        g = _dev(g, 'grad')
        d_disp = torch.empty_like(disp)
        L.check(lib.vfd_smooth_bwd(B, Nt, H, W, disp.data_ptr(), color.data_ptr(), sums.data_ptr(), g.data_ptr(),
                                   d_disp.data_ptr(), L.stream()), 'smooth_bwd')
        return d_disp, None


# =============================================================================================
# Fusion-level feature aggregation (fusion_depthnet.py:53-63)
# =============================================================================================
_AGG_CL = os.environ.get('VFD_AGG_CL', '1') != '0'     # channels-last products read in place
_AGG_CL_GRAD = os.environ.get('VFD_AGG_CL_GRAD', '1') != '0'   # their gradients handed back channels-last


def _agg_cl_ok(base, levels):
    """AggregateUp reads its inputs in place (vfd_aggregate_fwd_cl): all channels-last (and not also
    NCHW-contiguous) maps of one dtype, fp32 or bf16."""
    return _AGG_CL and all(t.is_cuda and t.dim() == 4 and t.dtype == base.dtype and t.dtype in _DT
                           and not t.is_contiguous() and t.is_contiguous(memory_format=torch.channels_last)
                           for t in (base,) + tuple(levels))


def _to_nhwc(x, dtype):
    """NCHW fp32 x -> channels-last `dtype` copy in one pass (vfd_nchw_to_nhwc)."""
    lib = L.load()
    n, C, h, w = x.shape
    y = torch.empty(n, C, h, w, device=x.device, dtype=dtype, memory_format=torch.channels_last)
    L.check(lib.vfd_nchw_to_nhwc(x.data_ptr(), y.data_ptr(), n, C, h * w, _DT[dtype], L.stream()), 'nchw_to_nhwc')
    if L.PROF_ON:                            # timed under the layout_copy scope (vfd_nchw_to_nhwc)
        L.ALG_BYTES['layout_copy'] += x.numel() * 4 + y.numel() * y.element_size()
    return y


_GROUP_CAMS = {}


def _group_cams(groups, g, device):
    """Device index of the cameras in overlap group g, made once per (groups, device): the first
    (eager) step builds it, so a captured step holds no host->device copy."""
    key = (tuple(groups), g, str(device))
    if key not in _GROUP_CAMS:
        cams = [n for n, gg in enumerate(groups) if gg == g]
        _GROUP_CAMS[key] = torch.tensor(cams, dtype=torch.long, device=device) if cams else None
    return _GROUP_CAMS[key]


class FoldWeights(torch.autograd.Function):
    """K1's folded 1x1-conv columns (VFNet.folded_weights): from conv_non_overlap's weight W_no
    [Cv, C+1, 1] and conv_overlap's W_o [Cv, 2C+2, 1] (volumetric_fusionnet.py:197-230) ->
    wf [N, 2Cv, C] (per camera: W_no's feature columns over W_o's half of the camera's overlap
    group) and wz [3, Cv] (the depth-feature columns).  The forward is the slices / cat / stack of
    VFNet.folded_weights; the backward writes both weight gradients directly (column sums over the
    cameras of each group, one copy per depth column) instead of autograd's zero fill + copy + add
    per slice and camera."""

    @staticmethod
    def forward(ctx, w_no, w_o, groups):
        Cv, C1 = w_no.shape[:2]
        C = C1 - 1
        wn, wo = w_no[:, :, 0], w_o[:, :, 0]
        halves = [wo[:, :C], wo[:, C + 1:2 * C + 1]]
        wf = torch.stack([torch.cat([wn[:, :C], halves[g]], 0) for g in groups], 0)
        wz = torch.stack([wn[:, C], wo[:, C], wo[:, 2 * C + 1]], 0)
        ctx.groups, ctx.shapes = tuple(groups), (tuple(w_no.shape), tuple(w_o.shape))
        return wf, wz

    @staticmethod
    def backward(ctx, dwf, dwz):
        (Cv, C1, _), so = ctx.shapes
        C = C1 - 1
        dev, dt = (dwf if dwf is not None else dwz).device, (dwf if dwf is not None else dwz).dtype
        dno = torch.zeros(Cv, C1, device=dev, dtype=dt)
        do = torch.zeros(so[0], so[1], device=dev, dtype=dt)
        if dwf is not None:
            torch.sum(dwf[:, :Cv, :], 0, out=dno[:, :C])
            for g, lo in ((0, 0), (1, C + 1)):
                cams = _group_cams(ctx.groups, g, dev)
                if cams is not None:
                    torch.sum(dwf.index_select(0, cams)[:, Cv:, :], 0, out=do[:, lo:lo + C])
        if dwz is not None:
            dno[:, C] = dwz[0]
            do[:, C] = dwz[1]
            do[:, 2 * C + 1] = dwz[2]
        return dno.unsqueeze(-1), do.unsqueeze(-1), None


class LevelConv1x1(torch.autograd.Function):
    """The aggregation's 1x1 conv (fusion_depthnet.py:57-63, fusion_posenet.py:58-66: conv1x1 over the
    channel concatenation of the upsampled levels) evaluated per pyramid level at its own
    resolution with the level's input-channel slice of ONE weight [O, sum C_k, 1, 1] (MIOpen, as
    F.conv2d on each slice).  Backward: each level's data and weight gradient from one
    convolution_backward, and the weight gradient as the concatenation of the slices' gradients —
    autograd's per-slice chain (a zero fill of the whole weight, a copy into the slice, an add of
    the slices: eight launches per call) becomes one concatenation.  Under bf16 autocast the slices
    run in bf16 as autocast casts them; their gradients come back fp32 (the master weight's)."""

    @staticmethod
    def forward(ctx, w, *feats):
        outs, off = [], 0
        for f in feats:
            c = f.shape[1]
            outs.append(F.conv2d(f, w[:, off:off + c]))
            off += c
        ctx.save_for_backward(w, *feats)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        w, *feats = ctx.saved_tensors
        dws, dfs, off = [], [], 0
        for i, (f, g) in enumerate(zip(feats, gs)):
            c = f.shape[1]
            wk = w[:, off:off + c].to(f.dtype)
            off += c
            if g is None:
                g = torch.zeros(f.shape[0], w.shape[0], *f.shape[2:], device=f.device, dtype=f.dtype)
            mask = [ctx.needs_input_grad[1 + i], ctx.needs_input_grad[0], False]
            df, dw, _ = torch.ops.aten.convolution_backward(g.to(f.dtype), f, wk, None, [1, 1], [0, 0], [1, 1],
                                                            False, [0, 0], 1, mask)
            dfs.append(df)
            dws.append(dw)
        dW = torch.cat([t.to(w.dtype) for t in dws], 1) if ctx.needs_input_grad[0] else None
        return (dW, *dfs)


class AggregateUp(torch.autograd.Function):
    """LReLU_0.1(base + sum_k up_align_corners(level_k) + bias) -> NCHW fp32; levels are upsampled to
    base's size.  NCHW inputs are taken in fp32 (the cast autocast's custom_fwd(cast_inputs=float32)
    did); channels-last fp32 / bf16 inputs (config 3's bf16 1x1-conv products) are read in place —
    the same fp32 values and arithmetic, without the cast and NCHW copies."""

    @staticmethod
    @_amp_keep
    def forward(ctx, base, bias, *levels):
        lib = L.load()
        BN, C, h, w = base.shape
        hw = (L.c_int * max(2 * len(levels), 1))(*[v for t in levels for v in t.shape[-2:]])
        if _agg_cl_ok(base, levels):
            for t in (base,) + tuple(levels):
                _check_device(t, 'aggregate input')
            bias = _dev(bias, 'bias')
            out = torch.empty(BN, C, h, w, device=base.device)
            ptrs = (L.c_fp * max(len(levels), 1))(*[t.data_ptr() for t in levels])
            L.check(lib.vfd_aggregate_fwd_cl(BN, C, h, w, base.data_ptr(), len(levels), ptrs, hw, bias.data_ptr(),
                                             out.data_ptr(), _DT[base.dtype], L.stream()), 'aggregate_fwd_cl')
            ctx.save_for_backward(out)
            ctx.level_shapes = [tuple(t.shape) for t in levels]
            ctx.cl_dtype = base.dtype if _AGG_CL_GRAD else None
            return out
        ctx.cl_dtype = None
        base, bias = _dev(base, 'aggregate base'), _dev(bias, 'bias')
        levels = [_dev(t, 'aggregate level') for t in levels]
        out = torch.empty_like(base)
        ptrs = (L.c_fp * max(len(levels), 1))(*[t.data_ptr() for t in levels])
        L.check(lib.vfd_aggregate_fwd(BN, C, h, w, base.data_ptr(), len(levels), ptrs, hw, bias.data_ptr(),
                                      out.data_ptr(), L.stream()), 'aggregate_fwd')
        ctx.save_for_backward(out)
        ctx.level_shapes = [tuple(t.shape) for t in levels]
        return out

    @staticmethod
    @_amp_bwd
    def backward(ctx, g):
        lib = L.load()
        out, = ctx.saved_tensors
        g = g.contiguous()
        BN, C, h, w = g.shape
        wsmax = max([shp[-1] for shp in ctx.level_shapes] + [0])
        if (h * w + h * wsmax + 5 * (h + w)) * 4 <= 64 * 1024:     # one launch: d, its plane sums, every level
            d = torch.empty_like(g)
            psum = torch.empty(BN * C, device=g.device)
            grads = [torch.empty(shp, device=g.device) for shp in ctx.level_shapes]
            n = len(grads)
            ptrs = (L.c_fp * max(n, 1))(*[t.data_ptr() for t in grads])
            hw = (L.c_int * max(2 * n, 1))(*[v for shp in ctx.level_shapes for v in shp[-2:]])
            L.check(lib.vfd_aggregate_bwd(BN, C, h, w, g.data_ptr(), out.data_ptr(), d.data_ptr(), n, ptrs, hw,
                                          psum.data_ptr(), L.stream()), 'aggregate_bwd')
            if L.PROF_ON:
                L.ALG_BYTES['upsample_bwd'] += (3 * g.numel() + sum(t.numel() for t in grads)) * 4
            if ctx.cl_dtype is not None:       # channels-last inputs: their gradients in their layout / dtype
                d, grads = _to_nhwc(d, ctx.cl_dtype), [_to_nhwc(t, ctx.cl_dtype) for t in grads]
            return (d, psum.view(BN, C).sum(0)) + tuple(grads)
        d = (g * torch.where(out > 0, 1.0, 0.1)).contiguous()
        grads = []
        for shp in ctx.level_shapes:          # the upsample's adjoint as a gather (deterministic)
            dl = torch.empty(shp, device=d.device)
            tmp = torch.empty(BN * C * h * shp[-1], device=d.device)
            L.check(lib.vfd_upsample_ac_bwd(d.data_ptr(), dl.data_ptr(), tmp.data_ptr(), BN * C, h, w, shp[-2], shp[-1],
                                            L.stream()), 'upsample_ac_bwd')
            if L.PROF_ON:
                L.ALG_BYTES['upsample_bwd'] += (d.numel() + dl.numel()) * 4
            grads.append(dl)
        db = d.sum((0, 2, 3))
        if ctx.cl_dtype is not None:
            d, grads = _to_nhwc(d, ctx.cl_dtype), [_to_nhwc(t, ctx.cl_dtype) for t in grads]
        return (d, db) + tuple(grads)


# =============================================================================================
# Fused training-mode BatchNorm (+ residual) (+ ReLU) of the ResNet encoders (bnact.hip)
# =============================================================================================
_BN_ONE = os.environ.get('VFD_BN_ONE', '1') != '0'      # one-launch BN for small layers
_BN_JOIN = os.environ.get('VFD_BN_JOIN', '1') != '0'    # residual join (BatchNormAct.forward)
_BN_NHWC = os.environ.get('VFD_BN_NHWC', '1') != '0'    # channels-last maps stay channels-last
_DEC_CONV = os.environ.get('VFD_DEC_CONV', '1') != '0'   # decoder's narrow convs on MFMA (decconv.hip)


def _bn_group(bn):
    """SyncBatchNorm under an initialised process group of > 1 ranks -> that group, else None
    (nn.SyncBatchNorm itself falls back to the local batch norm at world size 1)."""
    import torch.distributed as dist
    if not isinstance(bn, torch.nn.SyncBatchNorm) or not (dist.is_available() and dist.is_initialized()):
        return None
    pg = bn.process_group or dist.group.WORLD
    return pg if dist.get_world_size(pg) > 1 else None


def _bn_sync(lib, d, partial, pg, count, what, invstd=None, dgamma=None, dbeta=None):
    """SyncBatchNorm exchange: the per-channel fp64 sums [C, 2] plus the local element count as row
    C, reduced over the group in ONE all-reduce (ranks may hold different batch sizes, as
    SyncBatchNorm allows; the apply kernels read the global count from row C on the device, so
    nothing waits on the host).  Backward (invstd given): d gamma / d beta from this rank's LOCAL
    sums first, as torch's SyncBatchNorm returns them (DDP then averages them over ranks)."""
    import time
    import torch.distributed as dist
    sums = torch.empty(max(d.groups, 1), d.C + 1, 2, dtype=torch.float64, device=partial.device)
    L.check(lib.vfd_bn_sum(ctypes.byref(d), partial.data_ptr(), float(count), sums.data_ptr(), L.ptr(invstd),
                           L.ptr(dgamma), L.ptr(dbeta), L.stream()), what)
    t0 = time.perf_counter()
    dist.all_reduce(sums, group=pg)
    SYNCBN_STATS['calls'] += 1
    SYNCBN_STATS['bytes'] += sums.numel() * sums.element_size()
    SYNCBN_STATS['host_s'] += time.perf_counter() - t0
    return sums


# SyncBatchNorm collectives issued by the fused BN (one all-reduce of [C+1][2] fp64 per layer and
# direction): count, payload and the host time spent in dist.all_reduce (for RCCL the enqueue, for
# gloo the whole exchange).  syncbn_stats(reset=True) reads them.
SYNCBN_STATS = {'calls': 0, 'bytes': 0, 'host_s': 0.0}


def syncbn_stats(reset=True):
    out = dict(SYNCBN_STATS)
    if reset:
        SYNCBN_STATS.update(calls=0, bytes=0, host_s=0.0)
    return out


def _bn_reduce(lib, d, partial, count, what, invstd=None, dgamma=None, dbeta=None):
    """The [G][C][S][2] partials reduced to [G][C + 1][2] sums (row C = the element count) on this rank."""
    sums = torch.empty(max(d.groups, 1), d.C + 1, 2, dtype=torch.float64, device=partial.device)
    L.check(lib.vfd_bn_sum(ctypes.byref(d), partial.data_ptr(), float(count), sums.data_ptr(), L.ptr(invstd),
                           L.ptr(dgamma), L.ptr(dbeta), L.stream()), what)
    return sums


def _bn_nhwc(x):
    """x is a channels-last map the NHWC kernels take (C/4 a power of two, C <= 2048)."""
    C = x.shape[1]
    return (_BN_NHWC and x.dim() == 4 and not x.is_contiguous() and x.is_contiguous(memory_format=torch.channels_last)
            and C % 4 == 0 and C <= 2048 and ((C >> 2) & ((C >> 2) - 1)) == 0)


def _bn_fields(d):
    return (d.N, d.C, d.HW, d.S, d.relu, d.eps, d.momentum, d.dtype, None, None, d.nhwc, d.groups)


def _observed(t):
    """Something reads t's gradient outside the autograd graph: a tensor hook or retain_grad."""
    return bool(t.retains_grad or getattr(t, '_backward_hooks', None))


class BatchNormAct(torch.autograd.Function):
    """y = relu(batch_norm_train(x) [+ r]) for NCHW fp32 x (one statistics + one apply pass each
    way; running statistics updated like nn.BatchNorm2d.train()).  `pg`: the SyncBatchNorm group
    (None = local statistics).  `groups` G > 1: x holds G consecutive batches normalised with their
    own statistics, exactly G train-mode calls of the layer (running statistics updated G times in
    order, num_batches_tracked += G, parameter gradients summed) in the launches of one
    (bnact.hip, vfd_bn_desc.groups)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, residual, running_mean, running_var, eps, momentum, relu, pg, nbt=None,
                join=False, groups=1):
        lib = L.load()
        _check_device(x, 'batch norm input')
        if x.dtype not in (torch.float32, torch.bfloat16):
            raise RuntimeError(f'fused batch norm: fp32 or bf16 activations, got {x.dtype}')
        N, C, H, W = x.shape
        G = int(groups)
        if G < 1 or N % G:
            raise RuntimeError(f'fused batch norm: {N} images do not split into {G} groups')
        # channels-last maps (config 3's bf16 encoders, layers.ResnetEncoder) stay channels-last
        fmt = torch.channels_last if _bn_nhwc(x) else torch.contiguous_format
        x = x.contiguous(memory_format=fmt)
        # bf16 activations (config 3's autocast: the conv outputs are bf16), fp32 parameters / stats
        d = L.BnDesc(N // G, C, H * W, 0, int(relu), float(eps), float(momentum), int(x.dtype == torch.bfloat16))
        d.nhwc = int(fmt is torch.channels_last)
        d.groups = G
        d.S = lib.vfd_bn_splits(ctypes.byref(d))
        ctx.fmt = fmt
        r = residual.to(x.dtype).contiguous(memory_format=fmt) if residual is not None else None
        # residual join: when the residual is the output of the previous block's fused BN (an
        # identity block), this layer's d residual (= g masked by its ReLU) is handed to that BN's
        # backward, which sums it into its own incoming gradient on load — no d residual tensor and
        # no autograd add of the two branches (the sum is the same fp32 add autograd performs)
        # The join bypasses autograd's delivery of d residual to the residual tensor, so it is only
        # taken when nothing observes that gradient: no tensor hooks and no retain_grad, checked
        # here and again at backward time (through a weak reference).  A partial autograd.grad(...,
        # inputs=[block output]) cannot be detected: set VFD_BN_JOIN=0 to inspect gradients of
        # intermediate encoder tensors.
        ctx.pending = []
        ctx.res_node = None
        ctx.res_ref = None
        if (join and _BN_JOIN and r is residual and residual.requires_grad
                and type(residual.grad_fn).__name__ == 'BatchNormActBackward' and not _observed(residual)):
            ctx.res_node = residual.grad_fn
            ctx.res_ref = weakref.ref(residual)
        ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        # with ReLU the forward also stores [y > 0] as one byte per element: the backward reads
        # that mask instead of y (d.relu == 2 there), a quarter of the bytes
        mk = torch.empty_like(x, dtype=torch.uint8) if relu else None
        ctx.one = pg is None and _BN_ONE and bool(lib.vfd_bn1_fits(ctypes.byref(d)))
        if ctx.one:       # small layer, local statistics: one launch (bnact.hip bn1_fwd_k)
            y = torch.empty_like(x)
            mean = torch.empty(G, C, device=x.device)
            invstd = torch.empty(G, C, device=x.device)
            L.check(lib.vfd_bn1_fwd(ctypes.byref(d), x.data_ptr(), ptr(r), gamma.data_ptr(), beta.data_ptr(),
                                    y.data_ptr(), mean.data_ptr(), invstd.data_ptr(), ptr(running_mean),
                                    ptr(running_var), ptr(nbt), ptr(mk), L.stream()), 'bn1_fwd')
            ctx.d, ctx.pg, ctx.count, ctx.has_res = _bn_fields(d), pg, float(N // G * H * W), r is not None
            if L.PROF_ON:
                L.ALG_BYTES['bn_fwd'] += x.numel() * (2 * x.element_size() + x.element_size() * (r is not None)
                                                      + (mk is not None))
            ctx.save_for_backward(x, mk, gamma, mean, invstd)
            return y
        partial = torch.empty(G, C, d.S, 2, dtype=torch.float64, device=x.device)
        L.check(lib.vfd_bn_fwd_stats(ctypes.byref(d), x.data_ptr(), partial.data_ptr(), L.stream()), 'bn_fwd_stats')
        count, sums, ns = float(N // G * H * W), partial, d.S
        if pg is not None:          # global sums and count from the group; count 0 = read on device
            sums, ns = _bn_sync(lib, d, partial, pg, count, 'bn_sum'), 1
            count = 0.0
        elif d.nhwc:                # channels-last apply passes take reduced sums
            sums, ns = _bn_reduce(lib, d, partial, count, 'bn_sum'), 1
        y = torch.empty_like(x)
        mean = torch.empty(G, C, device=x.device)
        invstd = torch.empty(G, C, device=x.device)
        L.check(lib.vfd_bn_fwd_apply(ctypes.byref(d), x.data_ptr(), r.data_ptr() if r is not None else None,
                                     sums.data_ptr(), ns, count, gamma.data_ptr(), beta.data_ptr(), y.data_ptr(),
                                     mean.data_ptr(), invstd.data_ptr(),
                                     running_mean.data_ptr() if running_mean is not None else None,
                                     running_var.data_ptr() if running_var is not None else None,
                                     nbt.data_ptr() if nbt is not None else None, ptr(mk), L.stream()),
                'bn_fwd_apply')
        ctx.d, ctx.pg, ctx.count, ctx.has_res = _bn_fields(d), pg, count, r is not None
        if L.PROF_ON:                        # compulsory: x (+ r) in, y (+ the ReLU byte mask) out
            L.ALG_BYTES['bn_fwd'] += x.numel() * (2 * x.element_size() + x.element_size() * (r is not None)
                                                  + (mk is not None))
        ctx.save_for_backward(x, mk, gamma, mean, invstd)
        return y

    @staticmethod
    def backward(ctx, g):
        lib = L.load()
        x, mk, gamma, mean, invstd = ctx.saved_tensors
        d = L.BnDesc(*ctx.d)
        if d.relu:
            d.relu = 2                       # the ReLU mask is the forward's byte mask
        g = g.to(x.dtype).contiguous(memory_format=ctx.fmt)
        need = ctx.needs_input_grad
        ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        # the next block's identity-branch gradient, deposited by its backward (residual join)
        pending, ctx.pending = ctx.pending, []
        res = ctx.res_ref() if ctx.res_ref is not None else None
        joined = ctx.res_node is not None and need[3] and not (res is not None and _observed(res))
        ctx.res_ref = None
        # a join chain (this block both receives and hands on an identity-branch gradient, deeper
        # ResNets) and extra deposits fold with autograd's own adds; one deposit rides in the kernel
        for g2, m2 in (pending if joined else pending[1:]):
            g = g + (g2 * m2 if m2 is not None else g2)
        if pending and not joined:
            d.g2, d.m2 = pending[0][0].data_ptr(), ptr(pending[0][1])
        if joined:      # hand d residual = g (ReLU-masked on load) to the block that produced r
            ctx.res_node.pending.append((g, mk if d.relu else None))
        ctx.res_node = None
        want_dr = ctx.has_res and need[3] and not joined
        if ctx.one:
            dx = torch.empty_like(x) if need[0] else None
            dr = torch.empty_like(x) if want_dr else None
            dgamma = torch.empty_like(gamma) if need[1] else None
            dbeta = torch.empty_like(gamma) if need[2] else None
            if L.PROF_ON:
                es = x.element_size()
                L.ALG_BYTES['bn_bwd'] += x.numel() * (2 * es + (d.relu != 0) + es * ((dx is not None) + (dr is not None))
                                                      + (es + (d.m2 is not None)) * (d.g2 is not None))
            L.check(lib.vfd_bn1_bwd(ctypes.byref(d), g.data_ptr(), mk.data_ptr() if d.relu else None, x.data_ptr(),
                                    gamma.data_ptr(), mean.data_ptr(), invstd.data_ptr(), ptr(dx), ptr(dr),
                                    ptr(dgamma), ptr(dbeta), L.stream()), 'bn1_bwd')
            return dx, dgamma, dbeta, dr, None, None, None, None, None, None, None, None, None
        partial = torch.empty(max(d.groups, 1), d.C, d.S, 2, dtype=torch.float64, device=g.device)
        yp = mk.data_ptr() if d.relu else None
        L.check(lib.vfd_bn_bwd_stats(ctypes.byref(d), g.data_ptr(), yp, x.data_ptr(), mean.data_ptr(),
                                     partial.data_ptr(), L.stream()), 'bn_bwd_stats')
        dx = torch.empty_like(x) if need[0] else None
        dr = torch.empty_like(x) if want_dr else None
        dgamma = torch.empty_like(gamma) if need[1] else None
        dbeta = torch.empty_like(gamma) if need[2] else None
        ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        sums, ns, count = partial, d.S, ctx.count
        pg_dgamma, pg_dbeta = dgamma, dbeta
        if ctx.pg is not None:      # local d gamma / d beta, then the global sums (+ count row)
            sums, ns = _bn_sync(lib, d, partial, ctx.pg, d.N * d.HW, 'bn_sum', invstd, dgamma, dbeta), 1
            count, pg_dgamma, pg_dbeta = 0.0, None, None
        elif d.nhwc:                # channels-last: reduced sums (d gamma / d beta written there)
            sums, ns = _bn_reduce(lib, d, partial, count, 'bn_sum', invstd, dgamma, dbeta), 1
            pg_dgamma, pg_dbeta = None, None
        if L.PROF_ON:                        # compulsory: g, x (, the mask) in, dx (, dr) out
            es = x.element_size()
            L.ALG_BYTES['bn_bwd'] += x.numel() * (2 * es + (d.relu != 0) + es * ((dx is not None) + (dr is not None))
                                                  + (es + (d.m2 is not None)) * (d.g2 is not None))
        L.check(lib.vfd_bn_bwd_apply(ctypes.byref(d), g.data_ptr(), yp, x.data_ptr(), sums.data_ptr(), ns, count,
                                     gamma.data_ptr(), mean.data_ptr(), invstd.data_ptr(), ptr(dx), ptr(dr),
                                     ptr(pg_dgamma), ptr(pg_dbeta), L.stream()), 'bn_bwd_apply')
        return dx, dgamma, dbeta, dr, None, None, None, None, None, None, None, None, None


# =============================================================================================
# Reflect padding by one pixel (the decoders' reflect 3x3 convs), deterministic backward
# =============================================================================================
_DEC_CL = os.environ.get('VFD_DEC_CL', '1') != '0'       # bf16 decoders keep their maps channels-last


def _nhwc_ok(t):
    """The channels-last reflectpad.hip kernels apply: a 4-d channels-last (not also NCHW-contiguous)
    map whose channel count is a multiple of 4 with C / 4 dividing 256 (the bias partials' blocks
    cover whole pixels)."""
    if t.dim() != 4 or t.is_contiguous() or not t.is_contiguous(memory_format=torch.channels_last):
        return False
    q, r = divmod(t.shape[1], 4)
    return r == 0 and 256 % q == 0 and t.data_ptr() % 16 == 0


def _as_nhwc(t, like):
    """t in the layout of `like` (channels-last), 16-B aligned, for the NHWC kernels."""
    t = t.to(like.dtype).contiguous(memory_format=torch.channels_last)
    return t if t.data_ptr() % 16 == 0 else t.clone(memory_format=torch.channels_last)


def decoder_channels_last(x):
    """Whether a bf16 decoder input goes channels-last (VFD_DEC_CL, default on): MIOpen's bf16
    convs then read / write NHWC directly instead of transposing every NCHW map around an NHWC
    solver (config 3's batched_transpose_* kernels)."""
    return _DEC_CL and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 4 == 0 and \
        256 % (x.shape[1] // 4) == 0


class ReflectPad1(torch.autograd.Function):
    """F.pad(x, (1, 1, 1, 1), mode='reflect') for NCHW or channels-last fp32 or bf16 x
    (reflectpad.hip); the backward gathers each pixel's copies in a fixed order in fp32 (ATen's
    scatters with atomics, in bf16 under autocast: 0.5 ms per decoder pad at config 3)."""

    @staticmethod
    def forward(ctx, x):
        lib = L.load()
        _check_device(x, 'reflect pad input')
        ctx.nhwc = _nhwc_ok(x)
        if ctx.nhwc:
            n, c, h, w = x.shape
            y = torch.empty(n, c, h + 2, w + 2, dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
            L.check(lib.vfd_elu_up_pad1_nhwc_fwd(x.data_ptr(), y.data_ptr(), n, h, w, c, 0, 0, _dt(x), L.stream()),
                    'elu_up_pad1_nhwc_fwd')
            if L.PROF_ON:
                L.ALG_BYTES['reflect_pad'] += (x.numel() + y.numel()) * x.element_size()
            ctx.shape, ctx.dtype = tuple(x.shape), x.dtype
            return y
        x = x.contiguous()
        *lead, h, w = x.shape
        y = torch.empty(*lead, h + 2, w + 2, dtype=x.dtype, device=x.device)
        planes = x.numel() // (h * w)
        L.check(lib.vfd_reflect_pad1_fwd(x.data_ptr(), y.data_ptr(), planes, h, w, _dt(x), L.stream()), 'reflect_pad1_fwd')
        if L.PROF_ON:
            L.ALG_BYTES['reflect_pad'] += (x.numel() + y.numel()) * x.element_size()
        ctx.shape, ctx.dtype = tuple(x.shape), x.dtype
        return y

    @staticmethod
    def backward(ctx, g):
        lib = L.load()
        if ctx.nhwc:
            n, c, h, w = ctx.shape
            dx = torch.empty(ctx.shape, dtype=ctx.dtype, device=g.device, memory_format=torch.channels_last)
            g = _as_nhwc(g, dx)
            L.check(lib.vfd_elu_up_pad1_nhwc_bwd(g.data_ptr(), None, dx.data_ptr(), n, h, w, c, 0, 0, None, _dt(dx),
                                                 L.stream()), 'elu_up_pad1_nhwc_bwd')
            if L.PROF_ON:
                L.ALG_BYTES['reflect_pad'] += (g.numel() + dx.numel()) * dx.element_size()
            return dx
        g = g.to(ctx.dtype).contiguous()
        h, w = ctx.shape[-2:]
        dx = torch.empty(ctx.shape, dtype=ctx.dtype, device=g.device)
        planes = dx.numel() // (h * w)
        L.check(lib.vfd_reflect_pad1_bwd(g.data_ptr(), dx.data_ptr(), planes, h, w, _dt(dx), L.stream()), 'reflect_pad1_bwd')
        if L.PROF_ON:
            L.ALG_BYTES['reflect_pad'] += (g.numel() + dx.numel()) * dx.element_size()
        return dx


class EluUpPad(torch.autograd.Function):
    """F.pad(upsample2x_nearest(elu(y)) if up else elu(y), (1, 1, 1, 1), mode='reflect') for NCHW
    fp32 y in one pass (reflectpad.hip): the decoders' ELU -> upsample -> next reflect conv chain
    without the ELU / upsample / cat / pad intermediates; backward is one gather kernel."""

    @staticmethod
    def forward(ctx, y, up):
        ctx.u = 1 if up else 0
        ctx.save_for_backward(y)
        return _elu_up_pad_fwd(y, ctx.u)

    @staticmethod
    def backward(ctx, g):
        y, = ctx.saved_tensors
        return _elu_up_pad_bwd(g, y, ctx.u)[0], None


def _elu_up_pad_fwd(y, u):
    lib = L.load()
    _check_device(y, 'elu_up_pad input')
    if _nhwc_ok(y):
        n, c, h, w = y.shape
        out = torch.empty(n, c, (h << u) + 2, (w << u) + 2, dtype=y.dtype, device=y.device,
                          memory_format=torch.channels_last)
        L.check(lib.vfd_elu_up_pad1_nhwc_fwd(y.data_ptr(), out.data_ptr(), n, h, w, c, u, 1, _dt(y), L.stream()),
                'elu_up_pad1_nhwc_fwd')
        if L.PROF_ON:
            L.ALG_BYTES['elu_pad'] += (y.numel() + out.numel()) * y.element_size()
        return out
    y = y.contiguous()
    *lead, h, w = y.shape
    out = torch.empty(*lead, (h << u) + 2, (w << u) + 2, dtype=y.dtype, device=y.device)
    planes = y.numel() // (h * w)
    L.check(lib.vfd_elu_up_pad1_fwd(y.data_ptr(), out.data_ptr(), planes, h, w, u, _dt(y), L.stream()),
            'elu_up_pad1_fwd')
    if L.PROF_ON:
        L.ALG_BYTES['elu_pad'] += (y.numel() + out.numel()) * y.element_size()
    return out


def _elu_up_pad_bwd(g, y, u, bias_grad=False):
    """d y of the fused ELU [+ up] + pad, and (bias_grad) its per-channel sum [C] in fp32 (the
    producing conv's bias gradient: fixed-order block partials from the kernel, then one sum)."""
    lib = L.load()
    if _nhwc_ok(y):
        n, c, h, w = y.shape
        dy = torch.empty_like(y, memory_format=torch.channels_last)
        g = _as_nhwc(g, y)
        part = (torch.empty(lib.vfd_elu_up_pad1_nhwc_bwd_blocks(n, h, w, c), c, device=y.device)
                if bias_grad else None)
        L.check(lib.vfd_elu_up_pad1_nhwc_bwd(g.data_ptr(), y.data_ptr(), dy.data_ptr(), n, h, w, c, u, 1,
                                             part.data_ptr() if part is not None else None, _dt(y), L.stream()),
                'elu_up_pad1_nhwc_bwd')
        if L.PROF_ON:
            L.ALG_BYTES['elu_pad'] += (g.numel() + 2 * y.numel()) * y.element_size()
        return dy, (part.sum(0) if part is not None else None)
    g = g.to(y.dtype).contiguous()
    h, w = y.shape[-2:]
    dy = torch.empty_like(y)
    planes = y.numel() // (h * w)
    psum = torch.empty(planes, lib.vfd_elu_up_pad1_bwd_blocks(h, w), device=y.device) if bias_grad else None
    L.check(lib.vfd_elu_up_pad1_bwd(g.data_ptr(), y.data_ptr(), dy.data_ptr(), planes, h, w, u,
                                    psum.data_ptr() if psum is not None else None, _dt(y), L.stream()),
            'elu_up_pad1_bwd')
    if L.PROF_ON:
        L.ALG_BYTES['elu_pad'] += (g.numel() + 2 * y.numel()) * y.element_size()
    return dy, (psum.view(y.shape[0], y.shape[1], -1).sum((0, 2)) if psum is not None else None)


class ConvEluUpPad(torch.autograd.Function):
    """One decoder block (fusion_depthnet.py:97-145): the reflect conv 3x3 on an already padded
    map xp (MIOpen, padding 0), then ELU [+ nearest 2x] + the next conv's reflect pad (HIP).  The
    backward takes the conv's bias gradient from the ELU kernel's per-block sums (fixed order)
    instead of an ATen reduction over d y, and asks MIOpen for the data / weight gradients only."""

    @staticmethod
    def forward(ctx, xp, weight, bias, up):
        lib = L.load()
        N, CI, Hp, Wp = xp.shape
        CO = weight.shape[0]
        ctx.mfma = (_DEC_CONV and bias is not None and xp.is_contiguous() and xp.dtype == torch.float32
                    and bool(lib.vfd_dec_conv_supported(N, CI, CO, Hp - 2, Wp - 2)))
        if ctx.mfma:      # decconv.hip: the narrow conv on fp32 MFMA
            w = weight.detach().contiguous()
            y = torch.empty(N, CO, Hp - 2, Wp - 2, device=xp.device)
            L.check(lib.vfd_dec_conv_fwd(xp.data_ptr(), w.data_ptr(), bias.data_ptr(), y.data_ptr(), N, CI, CO,
                                         Hp - 2, Wp - 2, L.stream()), 'dec_conv_fwd')
            if L.PROF_ON:
                L.ALG_BYTES['dec_conv'] += (xp.numel() + y.numel()) * 4
        else:
            # MIOpen; a bf16 map (config 3's autocast) takes the weight / bias in bf16, as autocast's
            # conv2d would
            with torch.no_grad():
                y = F.conv2d(xp, weight.to(xp.dtype), bias.to(xp.dtype) if bias is not None else None)
        ctx.u = 1 if up else 0
        ctx.save_for_backward(xp, weight, y)
        return _elu_up_pad_fwd(y, ctx.u)

    @staticmethod
    def backward(ctx, g):
        xp, weight, y = ctx.saved_tensors
        need = ctx.needs_input_grad
        dy, db = _elu_up_pad_bwd(g, y, ctx.u, bias_grad=need[2])
        dx = dw = None
        N, CI, Hp, Wp = xp.shape
        CO = weight.shape[0]
        # tools/micro_decconv.py: d x + d w at 16->16 / 384x640 152 + 129 us vs MIOpen's 509,
        # 32->32 / 192x320 108 + 139 vs 262, 32->16 54 + 82 vs 193
        if ctx.mfma and (need[0] or need[1]):
            lib = L.load()
            w = weight.detach().contiguous()
            dx = torch.empty_like(xp) if need[0] else None
            part = (torch.empty(lib.vfd_dec_conv_wgrad_blocks(N, Hp - 2, Wp - 2), CO, CI, 9, device=xp.device)
                    if need[1] else None)
            L.check(lib.vfd_dec_conv_bwd(dy.data_ptr(), xp.data_ptr(), w.data_ptr(),
                                         dx.data_ptr() if dx is not None else None,
                                         part.data_ptr() if part is not None else None, N, CI, CO, Hp - 2, Wp - 2,
                                         L.stream()), 'dec_conv_bwd')
            if L.PROF_ON:
                L.ALG_BYTES['dec_conv'] += (dy.numel() + (dx is not None) * xp.numel()
                                            + (part is not None) * (dy.numel() + xp.numel())) * 4
            dw = part.sum(0).view(CO, CI, 3, 3) if part is not None else None
        elif need[0] or need[1]:
            dx, dw, _ = torch.ops.aten.convolution_backward(dy, xp, weight.to(xp.dtype), None, [1, 1], [0, 0], [1, 1],
                                                            False, [0, 0], 1, [need[0], need[1], False])
            if dw is not None:
                dw = dw.to(weight.dtype)
        return dx, dw, db, None


class DispConvSigmoid(torch.autograd.Function):
    """sigmoid(conv3x3(xp) + b) for the decoder's full-resolution disparity head (16 -> 1 channels,
    xp already reflect-padded): one HIP sweep forward, one data-gradient and one weight/bias
    gradient sweep backward (dispconv.hip) instead of MIOpen's one-output-channel solvers."""

    @staticmethod
    def supported(xp, weight):
        N, C, Hp, Wp = xp.shape
        return (xp.is_cuda and xp.dtype == torch.float32 and tuple(weight.shape) == (1, C, 3, 3)
                and bool(L.load().vfd_disp_conv_supported(N, C, Hp - 2, Wp - 2)))

    @staticmethod
    def forward(ctx, xp, weight, bias):
        lib = L.load()
        xp = _dev(xp, 'disp conv input')
        w = weight.contiguous()
        N, C, Hp, Wp = xp.shape
        H, W = Hp - 2, Wp - 2
        out = torch.empty(N, 1, H, W, device=xp.device)
        L.check(lib.vfd_disp_conv_fwd(xp.data_ptr(), w.data_ptr(), bias.data_ptr(), out.data_ptr(), N, C, H, W,
                                      L.stream()), 'disp_conv_fwd')
        if L.PROF_ON:
            L.ALG_BYTES['disp_conv'] += (xp.numel() + out.numel()) * 4
        ctx.save_for_backward(xp, w, out)
        return out

    @staticmethod
    def backward(ctx, g):
        lib = L.load()
        xp, w, out = ctx.saved_tensors
        g = g.contiguous()
        N, C, Hp, Wp = xp.shape
        H, W = Hp - 2, Wp - 2
        need = ctx.needs_input_grad
        dxp = torch.empty_like(xp) if need[0] else None
        part = (torch.empty(lib.vfd_disp_conv_wgrad_blocks(N, H, W), C * 9 + 1, device=xp.device)
                if need[1] or need[2] else None)
        L.check(lib.vfd_disp_conv_bwd(g.data_ptr(), out.data_ptr(), xp.data_ptr(), w.data_ptr(),
                                      dxp.data_ptr() if dxp is not None else None,
                                      part.data_ptr() if part is not None else None, N, C, H, W, L.stream()),
                'disp_conv_bwd')
        if L.PROF_ON:
            L.ALG_BYTES['disp_conv'] += (2 * out.numel() + (dxp is not None) * xp.numel()
                                         + (part is not None) * xp.numel()) * 4
        dw = db = None
        if part is not None:
            tot = part.sum(0)
            dw = tot[:C * 9].view(1, C, 3, 3) if need[1] else None
            db = tot[C * 9:] if need[2] else None
        return dxp, dw, db


def normalize_cat(a, b=None, out=None):
    """(cat([a, b], dim=1) - 0.45) / 0.225 for image batches [n, c, h, w] without gradient, in one
    HIP pass (maxpool.hip norm_cat_k; the encoders' input normalisation, bit-identical).  `out`: a
    contiguous [n, ca + cb, h, w] slot to write (one frame pair's part of a stacked batch)."""
    lib = L.load()
    a = _dev(a, 'image').contiguous()
    b = _dev(b, 'image').contiguous() if b is not None else None
    n, ca, h, w = a.shape
    cb = b.shape[1] if b is not None else 0
    if out is None:
        out = torch.empty(n, ca + cb, h, w, device=a.device)
    elif tuple(out.shape) != (n, ca + cb, h, w) or not out.is_contiguous() or out.dtype != torch.float32:
        raise RuntimeError(f'normalize_cat: out {tuple(out.shape)} does not fit {(n, ca + cb, h, w)}')
    L.check(lib.vfd_normalize_cat(a.data_ptr(), b.data_ptr() if b is not None else None, out.data_ptr(), n, ca, cb,
                                  h * w, L.stream()), 'normalize_cat')
    return out


# =============================================================================================
# ResNet stem max pool (3x3, stride 2, padding 1) with a one-byte argmax and a gather backward
# =============================================================================================
class MaxPool3s2(torch.autograd.Function):
    """F.max_pool2d(x, 3, 2, 1) for NCHW fp32 or bf16 x (maxpool.hip): one byte of window index
    per output instead of ATen's int64 indices; deterministic gather backward.  A channels-last x
    (config 3's bf16 encoders, C % 4 == 0) takes the NHWC kernels and gives a channels-last y."""

    @staticmethod
    def forward(ctx, x):
        lib = L.load()
        _check_device(x, 'max pool input')
        cl = (x.dim() == 4 and x.shape[1] % 4 == 0 and not x.is_contiguous()
              and x.is_contiguous(memory_format=torch.channels_last))
        fmt = torch.channels_last if cl else torch.contiguous_format
        x = x.contiguous(memory_format=fmt)
        *lead, h, w = x.shape
        ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        y = torch.empty(*lead, ho, wo, dtype=x.dtype, device=x.device, memory_format=fmt)
        arg = torch.empty(*lead, ho, wo, dtype=torch.uint8, device=x.device, memory_format=fmt)
        if cl:
            L.check(lib.vfd_maxpool3s2_nhwc_fwd(x.data_ptr(), y.data_ptr(), arg.data_ptr(), x.shape[0], x.shape[1],
                                                h, w, _dt(x), L.stream()), 'maxpool3s2_nhwc_fwd')
        else:
            planes = x.numel() // (h * w)
            L.check(lib.vfd_maxpool3s2_fwd(x.data_ptr(), y.data_ptr(), arg.data_ptr(), planes, h, w, _dt(x),
                                           L.stream()), 'maxpool3s2_fwd')
        if L.PROF_ON:
            L.ALG_BYTES['maxpool'] += (x.numel() + y.numel()) * x.element_size() + arg.numel()
        ctx.shape, ctx.dtype, ctx.fmt = tuple(x.shape), x.dtype, fmt
        ctx.save_for_backward(arg)
        return y

    @staticmethod
    def backward(ctx, g):
        lib = L.load()
        arg, = ctx.saved_tensors
        g = g.to(ctx.dtype).contiguous(memory_format=ctx.fmt)
        h, w = ctx.shape[-2:]
        dx = torch.empty(ctx.shape, dtype=ctx.dtype, device=g.device, memory_format=ctx.fmt)
        if ctx.fmt is torch.channels_last:
            L.check(lib.vfd_maxpool3s2_nhwc_bwd(g.data_ptr(), arg.data_ptr(), dx.data_ptr(), ctx.shape[0],
                                                ctx.shape[1], h, w, _dt(dx), L.stream()), 'maxpool3s2_nhwc_bwd')
        else:
            planes = dx.numel() // (h * w)
            L.check(lib.vfd_maxpool3s2_bwd(g.data_ptr(), arg.data_ptr(), dx.data_ptr(), planes, h, w, _dt(dx),
                                           L.stream()), 'maxpool3s2_bwd')
        if L.PROF_ON:
            L.ALG_BYTES['maxpool'] += (g.numel() + dx.numel()) * dx.element_size() + arg.numel()
        return dx

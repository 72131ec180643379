"""ctypes binding of `libvfd_hip.so` (C ABI declared in include/vfd_capi.h).

The library is loaded after `torch` so that it binds to the HIP runtime PyTorch-ROCm already
loaded (same SONAME, one device context).  There is no fallback: if the library is missing or
fails to load, every hot-path op raises.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL: shares torch's libamdhip64)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('VFD_LIB', os.path.join(_HERE, 'libvfd_hip.so'))

c_int, c_float, c_double, c_size_t, c_void_p = ctypes.c_int32, ctypes.c_float, ctypes.c_double, ctypes.c_size_t, ctypes.c_void_p
c_fp = ctypes.c_void_p      # device pointers are passed as integers


class VoxelDesc(ctypes.Structure):
    _fields_ = [('B', c_int), ('N', c_int), ('C', c_int), ('Cv', c_int), ('h', c_int), ('w', c_int),
                ('H', c_int), ('W', c_int), ('X', c_int), ('Y', c_int), ('Z', c_int), ('D', c_int),
                ('str', c_float * 3), ('len', c_float * 3), ('z_scale', c_float), ('pad_out', c_int),
                ('axis_x', c_fp), ('axis_y', c_fp), ('axis_z', c_fp), ('dbins', c_fp), ('group', c_fp),
                ('deterministic', c_int)]


class ViewDesc(ctypes.Structure):
    _fields_ = [('B', c_int), ('N', c_int), ('H', c_int), ('W', c_int), ('n_warp', c_int),
                ('n_temporal', c_int), ('n_overlap', c_int), ('intensity_align', c_int),
                ('cam_begin', c_int), ('cam_count', c_int), ('color', c_fp * 4), ('warp_tab', c_fp)]


class PhotoDesc(ctypes.Structure):
    _fields_ = [('B', c_int), ('N', c_int), ('H', c_int), ('W', c_int), ('T', c_int), ('F', c_int),
                ('cam_begin', c_int), ('cam_count', c_int), ('seed', ctypes.c_uint64), ('step', c_fp),
                ('noise_scale', c_float), ('ident', c_fp * 4)]


class DepthSynDesc(ctypes.Structure):
    _fields_ = [('B', c_int), ('N', c_int), ('H', c_int), ('W', c_int), ('S', c_int),
                ('min_depth', c_float), ('max_depth', c_float), ('src_tab', c_fp)]


class ConvDesc(ctypes.Structure):
    _fields_ = [('B', c_int), ('H', c_int), ('W', c_int), ('C', c_int), ('stride', c_int),
                ('out_channels', c_int)]


class BnDesc(ctypes.Structure):
    _fields_ = [('N', c_int), ('C', c_int), ('HW', c_int), ('S', c_int), ('relu', c_int),
                ('eps', c_float), ('momentum', c_float), ('dtype', c_int), ('g2', c_void_p), ('m2', c_void_p),
                ('nhwc', c_int), ('groups', c_int)]


_SIGS = {
    'vfd_version': (c_int, []),
    'vfd_last_error': (ctypes.c_char_p, []),
    'vfd_kernel_name': (ctypes.c_char_p, [c_int]),
    'vfd_prof_enable': (c_int, [c_int]),
    'vfd_prof_read': (c_int, [ctypes.POINTER(c_int), ctypes.POINTER(c_double)]),
    'vfd_prof_read_kernels': (c_int, [c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_double)]),
    'vfd_mask_downsample': (c_int, [ctypes.POINTER(VoxelDesc), c_fp, c_fp, c_void_p]),
    'vfd_fuse_depth_fwd': (c_int, [ctypes.POINTER(VoxelDesc)] + [c_fp] * 8 + [c_void_p]),
    'vfd_fuse_depth_bwd_workspace': (c_size_t, [ctypes.POINTER(VoxelDesc)]),
    'vfd_fuse_depth_bwd_planned_workspace': (c_size_t, [ctypes.POINTER(VoxelDesc)]),
    'vfd_fuse_depth_bwd': (c_int, [ctypes.POINTER(VoxelDesc)] + [c_fp] * 8 + [c_size_t, c_void_p]),
    'vfd_fuse_depth_bwd_planned': (c_int, [ctypes.POINTER(VoxelDesc)] + [c_fp] * 9 + [c_size_t, c_void_p]),
    'vfd_fusion_plan_bytes': (c_size_t, [ctypes.POINTER(VoxelDesc)]),
    'vfd_fusion_plan': (c_int, [ctypes.POINTER(VoxelDesc)] + [c_fp] * 5 + [c_void_p]),
    'vfd_fuse_pose_fwd': (c_int, [ctypes.POINTER(VoxelDesc)] + [c_fp] * 5 + [c_void_p]),
    'vfd_fuse_pose_fwd_t': (c_int, [ctypes.POINTER(VoxelDesc)] + [c_fp] * 5 + [c_int, c_fp, c_int, c_void_p]),
    'vfd_fuse_pose_bwd': (c_int, [ctypes.POINTER(VoxelDesc)] + [c_fp] * 4 + [c_void_p]),
    'vfd_fuse_pose_bwd_t': (c_int, [ctypes.POINTER(VoxelDesc)] + [c_fp] * 3 + [c_int, c_fp, c_void_p]),
    'vfd_voxel_project_fwd': (c_int, [ctypes.POINTER(VoxelDesc)] + [c_fp] * 4 + [c_void_p]),
    'vfd_voxel_project_plan_bytes': (c_size_t, [ctypes.POINTER(VoxelDesc)]),
    'vfd_voxel_project_plan': (c_int, [ctypes.POINTER(VoxelDesc)] + [c_fp] * 2 + [c_void_p, c_size_t, c_void_p]),
    'vfd_voxel_project_bwd_planned': (c_int, [ctypes.POINTER(VoxelDesc), c_fp, c_void_p, c_size_t, c_fp, c_void_p]),
    'vfd_voxel_project_bwd_workspace': (c_size_t, [ctypes.POINTER(VoxelDesc)]),
    'vfd_voxel_project_bwd': (c_int, [ctypes.POINTER(VoxelDesc)] + [c_fp] * 4 + [c_void_p, c_size_t, c_void_p]),
    'vfd_view_workspace_bytes': (c_size_t, [ctypes.POINTER(ViewDesc)]),
    'vfd_view_fwd': (c_int, [ctypes.POINTER(ViewDesc)] + [c_fp] * 10 + [c_size_t, c_void_p]),
    'vfd_view_bwd': (c_int, [ctypes.POINTER(ViewDesc)] + [c_fp] * 10 + [c_size_t, c_void_p]),
    'vfd_photo_workspace_bytes': (c_size_t, [ctypes.POINTER(PhotoDesc)]),
    'vfd_photo_fwd': (c_int, [ctypes.POINTER(PhotoDesc)] + [c_fp] * 13 + [c_size_t, c_void_p]),
    'vfd_photo_bwd': (c_int, [ctypes.POINTER(PhotoDesc)] + [c_fp] * 9 + [c_void_p]),
    'vfd_aggregate_fwd': (c_int, [c_int] * 4 + [c_fp, c_int, ctypes.POINTER(c_fp), ctypes.POINTER(c_int), c_fp, c_fp, c_void_p]),
    'vfd_nchw_to_nhwc': (c_int, [c_fp, c_fp, ctypes.c_longlong, c_int, c_int, c_int, c_void_p]),
    'vfd_aggregate_fwd_cl': (c_int, [c_int] * 4 + [c_fp, c_int, ctypes.POINTER(c_fp), ctypes.POINTER(c_int), c_fp, c_fp,
                                                   c_int, c_void_p]),
    'vfd_proj_conv_fwd_workspace': (c_size_t, [ctypes.POINTER(VoxelDesc)]),
    'vfd_proj_conv_fwd': (c_int, [ctypes.POINTER(VoxelDesc)] + [c_fp] * 5 + [c_int, c_fp, c_fp, c_fp, c_size_t, c_void_p]),
    'vfd_proj_conv_fwd_bf16': (c_int, [ctypes.POINTER(VoxelDesc)] + [c_fp] * 5 + [c_int, c_fp, c_fp, c_fp, c_size_t, c_void_p]),
    'vfd_proj_conv_dgrad_workspace': (c_size_t, [ctypes.POINTER(VoxelDesc)]),
    'vfd_proj_conv_dgrad': (c_int, [ctypes.POINTER(VoxelDesc)] + [c_fp] * 4 + [c_size_t, c_void_p]),
    'vfd_proj_conv_dgrad_bf16_workspace': (c_size_t, [ctypes.POINTER(VoxelDesc)]),
    'vfd_proj_conv_dgrad_bf16': (c_int, [ctypes.POINTER(VoxelDesc)] + [c_fp] * 4 + [c_size_t, c_void_p]),
    'vfd_proj_conv_wgrad_bf16_workspace': (c_size_t, [ctypes.POINTER(VoxelDesc)]),
    'vfd_proj_conv_wgrad_bf16': (c_int, [ctypes.POINTER(VoxelDesc)] + [c_fp] * 5 + [c_size_t, c_void_p]),
    'vfd_pad_conv_wgrad_bf16_workspace': (c_size_t, [ctypes.POINTER(ConvDesc)]),
    'vfd_pad_conv_wgrad_bf16': (c_int, [ctypes.POINTER(ConvDesc)] + [c_fp] * 5 + [c_size_t, c_void_p]),
    'vfd_pad_conv_wgrad_bf16_t': (c_int, [ctypes.POINTER(ConvDesc)] + [c_fp] * 2 + [c_int] + [c_fp] * 3
                                  + [c_size_t, c_void_p]),
    'vfd_proj_conv_wgrad_workspace': (c_size_t, [ctypes.POINTER(VoxelDesc)]),
    'vfd_proj_conv_wgrad': (c_int, [ctypes.POINTER(VoxelDesc)] + [c_fp] * 5 + [c_size_t, c_void_p]),
    'vfd_bn_splits': (c_int, [ctypes.POINTER(BnDesc)]),
    'vfd_bn_fwd_stats': (c_int, [ctypes.POINTER(BnDesc), c_fp, c_fp, c_void_p]),
    'vfd_bn_sum': (c_int, [ctypes.POINTER(BnDesc), c_fp, c_double, c_fp, c_fp, c_fp, c_fp, c_void_p]),
    'vfd_bn_fwd_apply': (c_int, [ctypes.POINTER(BnDesc), c_fp, c_fp, c_fp, c_int, c_double] + [c_fp] * 9 + [c_void_p]),
    'vfd_bn_bwd_stats': (c_int, [ctypes.POINTER(BnDesc)] + [c_fp] * 5 + [c_void_p]),
    'vfd_bn_bwd_apply': (c_int, [ctypes.POINTER(BnDesc), c_fp, c_fp, c_fp, c_fp, c_int, c_double] + [c_fp] * 7
                         + [c_void_p]),
    'vfd_inverse4x4': (c_int, [c_fp, c_fp, c_int, c_void_p]),
    'vfd_maxpool3s2_fwd': (c_int, [c_fp, c_fp, c_fp, ctypes.c_longlong, c_int, c_int, c_int, c_void_p]),
    'vfd_normalize_cat': (c_int, [c_fp, c_fp, c_fp, ctypes.c_longlong, c_int, c_int, c_int, c_void_p]),
    'vfd_maxpool3s2_bwd': (c_int, [c_fp, c_fp, c_fp, ctypes.c_longlong, c_int, c_int, c_int, c_void_p]),
    'vfd_maxpool3s2_nhwc_fwd': (c_int, [c_fp, c_fp, c_fp, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    'vfd_maxpool3s2_nhwc_bwd': (c_int, [c_fp, c_fp, c_fp, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    'vfd_aggregate_bwd': (c_int, [c_int] * 4 + [c_fp, c_fp, c_fp, c_int, ctypes.POINTER(c_fp), ctypes.POINTER(c_int), c_fp, c_void_p]),
    'vfd_upsample_ac_bwd': (c_int, [c_fp, c_fp, c_fp, ctypes.c_longlong] + [c_int] * 4 + [c_void_p]),
    'vfd_reflect_pad1_fwd': (c_int, [c_fp, c_fp, ctypes.c_longlong, c_int, c_int, c_int, c_void_p]),
    'vfd_reflect_pad1_bwd': (c_int, [c_fp, c_fp, ctypes.c_longlong, c_int, c_int, c_int, c_void_p]),
    'vfd_bn1_fits': (c_int, [ctypes.POINTER(BnDesc)]),
    'vfd_bn1_fwd': (c_int, [ctypes.POINTER(BnDesc)] + [c_fp] * 11 + [c_void_p]),
    'vfd_bn1_bwd': (c_int, [ctypes.POINTER(BnDesc)] + [c_fp] * 10 + [c_void_p]),
    'vfd_disp_conv_supported': (c_int, [c_int] * 4),
    'vfd_disp_conv_wgrad_blocks': (c_int, [c_int] * 3),
    'vfd_disp_conv_fwd': (c_int, [c_fp] * 4 + [c_int] * 4 + [c_void_p]),
    'vfd_disp_conv_bwd': (c_int, [c_fp] * 6 + [c_int] * 4 + [c_void_p]),
    'vfd_dec_conv_supported': (c_int, [c_int] * 5),
    'vfd_dec_conv_wgrad_blocks': (c_int, [c_int] * 3),
    'vfd_dec_conv_fwd': (c_int, [c_fp] * 4 + [c_int] * 5 + [c_void_p]),
    'vfd_dec_conv_bwd': (c_int, [c_fp] * 5 + [c_int] * 5 + [c_void_p]),
    'vfd_weight_fragments': (c_int, [c_int, c_fp, c_fp] + [c_int] * 6 + [c_void_p]),
    'vfd_weight_fragments_bf16': (c_int, [c_int, c_fp, c_fp] + [c_int] * 6 + [c_void_p]),
    'vfd_weight_swap': (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_void_p]),
    'vfd_weight_permute': (c_int, [c_fp, c_fp] + [c_int] * 4 + [ctypes.POINTER(ctypes.c_longlong)] * 2 + [c_void_p]),
    'vfd_elu_up_pad1_fwd': (c_int, [c_fp, c_fp, ctypes.c_longlong, c_int, c_int, c_int, c_int, c_void_p]),
    'vfd_elu_up_pad1_bwd': (c_int, [c_fp, c_fp, c_fp, ctypes.c_longlong, c_int, c_int, c_int, c_fp, c_int, c_void_p]),
    'vfd_elu_up_pad1_bwd_blocks': (c_int, [c_int, c_int]),
    'vfd_elu_up_pad1_nhwc_fwd': (c_int, [c_fp, c_fp, ctypes.c_longlong, c_int, c_int, c_int, c_int, c_int, c_int,
                                         c_void_p]),
    'vfd_elu_up_pad1_nhwc_bwd': (c_int, [c_fp, c_fp, c_fp, ctypes.c_longlong, c_int, c_int, c_int, c_int, c_int, c_fp,
                                         c_int, c_void_p]),
    'vfd_elu_up_pad1_nhwc_bwd_blocks': (c_int, [ctypes.c_longlong, c_int, c_int, c_int]),
    'vfd_lrelu_pad1_bwd_nhwc': (c_int, [c_fp, c_fp, c_fp, ctypes.c_longlong, c_int, c_int, c_int, c_float, c_void_p]),
    'vfd_lrelu_pad1_bwd_nhwc_t': (c_int, [c_fp, c_fp, c_fp, ctypes.c_longlong, c_int, c_int, c_int, c_float, c_int, c_int,
                                          c_void_p]),
    'vfd_pad_conv_fwd_workspace': (c_size_t, [ctypes.POINTER(ConvDesc)]),
    'vfd_pad_conv_fwd': (c_int, [ctypes.POINTER(ConvDesc)] + [c_fp] * 5 + [c_size_t, c_void_p]),
    'vfd_pad_conv_fwd_bf16_workspace': (c_size_t, [ctypes.POINTER(ConvDesc)]),
    'vfd_pad_conv_fwd_bf16': (c_int, [ctypes.POINTER(ConvDesc)] + [c_fp] * 5 + [c_size_t, c_void_p]),
    'vfd_pad_conv_fwd_bf16_t': (c_int, [ctypes.POINTER(ConvDesc), c_fp, c_int] + [c_fp] * 4 + [c_size_t, c_void_p]),
    'vfd_pad_conv_dgrad_workspace': (c_size_t, [ctypes.POINTER(ConvDesc)]),
    'vfd_pad_conv_dgrad': (c_int, [ctypes.POINTER(ConvDesc)] + [c_fp] * 4 + [c_size_t, c_void_p]),
    'vfd_pad_conv_dgrad_bf16_workspace': (c_size_t, [ctypes.POINTER(ConvDesc)]),
    'vfd_pad_conv_dgrad_bf16': (c_int, [ctypes.POINTER(ConvDesc)] + [c_fp] * 4 + [c_size_t, c_void_p]),
    'vfd_pad_conv_dgrad_bf16_t': (c_int, [ctypes.POINTER(ConvDesc)] + [c_fp] * 3 + [c_int, c_fp, c_size_t, c_void_p]),
    'vfd_depth_syn_fwd': (c_int, [ctypes.POINTER(DepthSynDesc)] + [c_fp] * 8 + [c_void_p]),
    'vfd_depth_syn_bwd': (c_int, [ctypes.POINTER(DepthSynDesc)] + [c_fp] * 9 + [c_void_p]),
    'vfd_depth_syn_bwd_ordered_workspace': (ctypes.c_size_t, [ctypes.POINTER(DepthSynDesc)]),
    'vfd_depth_syn_bwd_ordered': (c_int, [ctypes.POINTER(DepthSynDesc)] + [c_fp] * 10 + [ctypes.c_size_t, c_void_p]),
    'vfd_smooth_workspace_bytes': (c_size_t, [c_int] * 4),
    'vfd_smooth_fwd': (c_int, [c_int] * 4 + [c_fp] * 5 + [c_size_t, c_void_p]),
    'vfd_smooth_bwd': (c_int, [c_int] * 4 + [c_fp] * 5 + [c_void_p]),
}

EXPORTED = sorted(_SIGS)
_lib = None
_load_error = None


def load():
    """Load (once) and return the library; raise with the reason if unavailable."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f'{LIB_PATH} not built: run `python -m vfdepth_amd.build` (hipcc, gfx950)')
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status, what):
    if status != 0:
        msg = load().vfd_last_error().decode(errors='replace')
        raise RuntimeError(f'{what} failed ({status}): {msg}')


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


KERNEL_IDS = {
    'mask_downsample': 0, 'fuse_depth_fwd': 1, 'fuse_depth_bwd': 2, 'fuse_pose_fwd': 3, 'fuse_pose_bwd': 4,
    'voxel_project_fwd': 5, 'voxel_project_bwd': 6, 'view_stats': 7, 'view_apply': 8, 'view_bwd': 9,
    'photo_fwd': 10, 'photo_bwd': 11, 'smooth_fwd': 12, 'smooth_bwd': 13, 'fusion_plan': 14,
    'aggregate': 15, 'voxel_project_plan': 16, 'proj_conv_fwd': 17,
    'depth_syn_fwd': 18, 'depth_syn_bwd': 19, 'proj_conv_dgrad': 20, 'pad_conv_fwd': 21, 'bn_fwd': 22, 'bn_bwd': 23, 'reflect_pad': 24, 'upsample_bwd': 25, 'maxpool': 26, 'elu_pad': 27, 'disp_conv': 28, 'dec_conv': 29, 'proj_conv_wgrad': 30, 'pad_conv_dgrad': 31, 'pad_conv_wgrad': 32, 'layout_copy': 33,
}


def prof_enable(kernel='all'):
    """Time launches of `kernel` (name, id, 'all' or 'off') with HIP events on their stream."""
    if kernel == 'all':
        kid = -1
    elif kernel == 'off':
        kid = -2
    else:
        kid = KERNEL_IDS[kernel] if isinstance(kernel, str) else int(kernel)
    load().vfd_prof_enable(kid)
    global PROF_ON
    PROF_ON = kid != -2
    if PROF_ON:
        for k in ALG_BYTES:
            ALG_BYTES[k] = 0


# Algorithmic bytes of the shape-varying dense-net kernels (fused BN, reflect pads, upsample
# backward), accumulated by their Python wrappers while profiling is on (bench.py's rooflines).
PROF_ON = False
ALG_BYTES = {'bn_fwd': 0, 'bn_bwd': 0, 'reflect_pad': 0, 'upsample_bwd': 0, 'maxpool': 0, 'elu_pad': 0, 'disp_conv': 0, 'dec_conv': 0, 'layout_copy': 0}


def prof_read():
    """{kernel name: (launches, total ms)} of everything recorded since prof_enable; resets."""
    n = len(KERNEL_IDS)
    cnt = (c_int * n)()
    ms = (c_double * n)()
    load().vfd_prof_read_kernels(n, cnt, ms)
    names = {v: k for k, v in KERNEL_IDS.items()}
    return {names[i]: (cnt[i], ms[i]) for i in range(n) if cnt[i]}

"""C-ABI boundary checks that need no GPU: the library loads and exports exactly what
include/vfd_capi.h declares; descriptor layouts agree between C and ctypes."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'vfd_capi.h')


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    return sorted(set(re.findall(r'\b(vfd_[a-z0-9_]+)\s*\(', text)))


def test_header_declares_the_bound_functions():
    from vfdepth_amd import _lib
    assert declared_functions() == _lib.EXPORTED


def test_library_exports_every_declared_symbol():
    from vfdepth_amd import _lib
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.vfd_version() >= 1
    assert lib.vfd_kernel_name(0) == b'mask_downsample'


def test_descriptor_layouts_match_c(tmp_path):
    from vfdepth_amd import _lib
    src = tmp_path / 'sz.c'
    src.write_text('#include "vfd_capi.h"\n#include <stdio.h>\n#include <stddef.h>\n'
                   'int main(){printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(vfd_voxel_desc), sizeof(vfd_view_desc),'
                   ' sizeof(vfd_photo_desc), offsetof(vfd_voxel_desc, axis_x), offsetof(vfd_view_desc, color),'
                   ' offsetof(vfd_photo_desc, ident), sizeof(vfd_depthsyn_desc), offsetof(vfd_depthsyn_desc, src_tab),'
                   ' sizeof(vfd_bn_desc), offsetof(vfd_bn_desc, dtype), offsetof(vfd_bn_desc, groups));'
                   'return 0;}\n')
    exe = tmp_path / 'sz'
    subprocess.check_call(['gcc', '-I', os.path.dirname(HEADER), str(src), '-o', str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    want = [ctypes.sizeof(_lib.VoxelDesc), ctypes.sizeof(_lib.ViewDesc), ctypes.sizeof(_lib.PhotoDesc),
            _lib.VoxelDesc.axis_x.offset, _lib.ViewDesc.color.offset, _lib.PhotoDesc.ident.offset,
            ctypes.sizeof(_lib.DepthSynDesc), _lib.DepthSynDesc.src_tab.offset,
            ctypes.sizeof(_lib.BnDesc), _lib.BnDesc.dtype.offset, _lib.BnDesc.groups.offset]
    assert got == want


def test_bad_descriptor_is_rejected_without_gpu():
    """Argument validation happens before any HIP call, so it is testable on the CPU."""
    from vfdepth_amd import _lib
    lib = _lib.load()
    d = _lib.VoxelDesc()          # all zero -> invalid sizes
    st = lib.vfd_fuse_pose_fwd(ctypes.byref(d), None, None, None, None, None, None)
    assert st == -1
    assert b'bad' in lib.vfd_last_error()


def test_hot_path_refuses_cpu_tensors():
    import torch
    from vfdepth_amd import kernels as KN
    from vfdepth_amd import config as C
    cfg = C.surround_fusion_cfg(height=96, width=160)
    with pytest.raises(RuntimeError, match='HIP device'):
        KN._dev(torch.zeros(2), 'x')

"""MI355X-native VFDepth training step (drop-in for tronglh241/VFDepth's `VFDepthAlgo`).

Hot path (volumetric fusion, view synthesis, photometric losses) runs as hand-written gfx950
HIP kernels behind the C ABI in `include/vfd_capi.h`; dense CNN layers run on MIOpen through
PyTorch-ROCm; DDP gradient all-reduce runs on RCCL.
"""
from .config import get_config, surround_fusion_cfg, mono_cfg  # noqa: F401

__all__ = ['get_config', 'surround_fusion_cfg', 'mono_cfg', 'VFDepthAlgo']


def __getattr__(name):
    if name == 'VFDepthAlgo':
        from .vfdepth import VFDepthAlgo
        return VFDepthAlgo
    raise AttributeError(name)

"""Load the reference VFDepth (read-only at /root/reference) on CPU for golden-vector generation.

Runs ONLY in the build container (the reference never travels to the GPU box).  The reference
package cannot be imported normally: `models/vfdepth.py` pulls `dataset` → `external.dataset`
→ the empty packnet-sfm / dgp submodules.  So every hot-path file is loaded by path under
synthetic package names, after registering small stand-ins for what is missing:

* `pytorch3d.transforms`   → `vfdepth_amd.rotation` (restated pytorch3d formula)
* `external.layers`        → `vfdepth_amd.layers` (restated packnet ResNet encoder / decoders)
* `dataset`                → `construct_dataset` returning a 1-element list (no loader needed)
* `utils`                  → `aug_depth_params` only (visualisation-only, never called here)

No reference source is copied; files are executed from their original location.
"""
import importlib.util
import os
import sys
import types

import torch
import torch.nn as nn

REF = os.environ.get('VFD_REFERENCE', '/root/reference')
_LOADED = {}


def _register(name, module):
    sys.modules[name] = module
    return module


def _pkg(name, path=None):
    m = types.ModuleType(name)
    m.__path__ = [path] if path else []
    return _register(name, m)


def _load(name, relpath):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, relpath))
    mod = importlib.util.module_from_spec(spec)
    _register(name, mod)
    spec.loader.exec_module(mod)
    return mod


def available():
    return os.path.isfile(os.path.join(REF, 'models', 'vfdepth.py'))


def load():
    """Return a namespace with the reference classes/functions needed for fixtures."""
    if 'ns' in _LOADED:
        return _LOADED['ns']
    from vfdepth_amd import layers as L
    from vfdepth_amd import rotation as R

    p3d = _pkg('pytorch3d')
    tr = _register('pytorch3d.transforms', types.ModuleType('pytorch3d.transforms'))
    tr.axis_angle_to_matrix = R.axis_angle_to_matrix
    tr.matrix_to_euler_angles = R.matrix_to_euler_angles
    p3d.transforms = tr

    ext = _pkg('external')
    el = _register('external.layers', types.ModuleType('external.layers'))
    el.ResnetEncoder = L.ResnetEncoder
    el.PoseDecoder = L.PoseDecoder
    el.DepthDecoder = L.MonoDepthDecoder
    ext.layers = el

    ds = _pkg('dataset')
    ds.construct_dataset = lambda cfg, mode, **kw: [0]

    ut = _pkg('utils')
    ut.aug_depth_params = lambda *a, **k: []

    _pkg('network', os.path.join(REF, 'network'))
    blocks = _load('network.blocks', 'network/blocks.py')
    vfn = _load('network.volumetric_fusionnet', 'network/volumetric_fusionnet.py')
    mono_d = _load('network.mono_depthnet', 'network/mono_depthnet.py')
    mono_p = _load('network.mono_posenet', 'network/mono_posenet.py')
    fus_p = _load('network.fusion_posenet', 'network/fusion_posenet.py')
    fus_d = _load('network.fusion_depthnet', 'network/fusion_depthnet.py')
    net = sys.modules['network']
    for cls_mod, cls in ((mono_p, 'MonoPoseNet'), (mono_d, 'MonoDepthNet'),
                         (fus_p, 'FusedPoseNet'), (fus_d, 'FusedDepthNet')):
        setattr(net, cls, getattr(cls_mod, cls))
    net.__all__ = ['MonoDepthNet', 'MonoPoseNet', 'FusedDepthNet', 'FusedPoseNet']

    _pkg('models', os.path.join(REF, 'models'))
    _pkg('models.geometry', os.path.join(REF, 'models', 'geometry'))
    gu = _load('models.geometry.geometry_util', 'models/geometry/geometry_util.py')
    pose = _load('models.geometry.pose', 'models/geometry/pose.py')
    vr = _load('models.geometry.view_rendering', 'models/geometry/view_rendering.py')
    g = sys.modules['models.geometry']
    g.Pose, g.ViewRendering = pose.Pose, vr.ViewRendering
    _pkg('models.losses', os.path.join(REF, 'models', 'losses'))
    lu = _load('models.losses.loss_util', 'models/losses/loss_util.py')
    bl = _load('models.losses.base_loss', 'models/losses/base_loss.py')
    scl = _load('models.losses.single_cam_loss', 'models/losses/single_cam_loss.py')
    mcl = _load('models.losses.multi_cam_loss', 'models/losses/multi_cam_loss.py')
    dsl = _load('models.losses.depth_synthesis_loss', 'models/losses/depth_synthesis_loss.py')
    lo = sys.modules['models.losses']
    lo.SingleCamLoss, lo.MultiCamLoss, lo.DepthSynLoss = scl.SingleCamLoss, mcl.MultiCamLoss, dsl.DepthSynLoss
    bm = _load('models.base_model', 'models/base_model.py')
    vfd = _load('models.vfdepth', 'models/vfdepth.py')
    misc = _load('ref_utils_misc', 'utils/misc.py')

    ns = types.SimpleNamespace(blocks=blocks, vfnet=vfn, geometry_util=gu, pose=pose,
                               view_rendering=vr, loss_util=lu, single_cam_loss=scl,
                               multi_cam_loss=mcl, vfdepth=vfd, misc=misc,
                               fusion_depthnet=fus_d, fusion_posenet=fus_p)
    _LOADED['ns'] = ns
    return ns


def load_logger():
    """The reference's `utils/logger.py` module (for `Logger.compute_depth_losses`, logger.py:193-247).

    Loaded under a synthetic package `ref_utils` rooted at the reference's `utils/` (its relative
    imports `.visualize` / `.misc` resolve there); `tensorboardX` is not installed, so a stand-in
    module with an inert `SummaryWriter` is registered first (no writer is ever constructed)."""
    if 'logger' in _LOADED:
        return _LOADED['logger']
    tbx = _register('tensorboardX', types.ModuleType('tensorboardX'))

    class SummaryWriter:            # never instantiated: compute_depth_losses does not log
        def __init__(self, *a, **k):
            raise RuntimeError('tensorboardX stand-in')
    tbx.SummaryWriter = SummaryWriter
    _pkg('ref_utils', os.path.join(REF, 'utils'))
    _load('ref_utils.misc', 'utils/misc.py')
    _load('ref_utils.visualize', 'utils/visualize.py')
    mod = _load('ref_utils.logger', 'utils/logger.py')
    _LOADED['logger'] = mod
    return mod


def load_data_util():
    """The reference's `dataset/data_util.py` (align_dataset, transform_mask_sample).

    Its module-level `import torchvision.transforms` names an absent package: a stand-in whose
    `Resize` / `ToTensor` are the plain PIL / numpy operations torchvision performs on PIL images,
    and Pillow >= 10 no longer has `ANTIALIAS` (it was always an alias of `LANCZOS`), so the alias
    is restored before the file runs.  `align_dataset` itself uses only numpy and F.interpolate."""
    if 'data_util' in _LOADED:
        return _LOADED['data_util']
    import numpy as np
    import PIL.Image as pil
    if not hasattr(pil, 'ANTIALIAS'):
        pil.ANTIALIAS = pil.LANCZOS
    tv = _pkg('torchvision')
    trm = _register('torchvision.transforms', types.ModuleType('torchvision.transforms'))

    class Resize:
        def __init__(self, size, interpolation=pil.BILINEAR):
            self.size, self.interpolation = size, interpolation

        def __call__(self, img):
            return img.resize((self.size[1], self.size[0]), self.interpolation)

    class ToTensor:
        def __call__(self, img):
            a = np.asarray(img)
            a = a[:, :, None] if a.ndim == 2 else a
            return torch.from_numpy(a.transpose(2, 0, 1).copy()).float().div(255.0)
    trm.Resize, trm.ToTensor = Resize, ToTensor
    tv.transforms = trm
    mod = _load('ref_dataset_data_util', 'dataset/data_util.py')
    _LOADED['data_util'] = mod
    return mod


def reference_depth_losses(cfg, inputs, outputs):
    """`Logger(cfg, use_tb=False).compute_depth_losses(inputs, outputs)` of the reference, with
    the log directory redirected to a temporary one (the constructor creates it)."""
    import copy
    import tempfile
    lg = load_logger()
    cfg = copy.deepcopy(cfg)
    with tempfile.TemporaryDirectory() as tmp:
        cfg['data']['log_path'] = tmp
        cfg['eval']['eval_visualize'] = False
        logger = lg.Logger(cfg, use_tb=False)
        return logger.compute_depth_losses(inputs, outputs)


def build_algo(cfg):
    """Reference `VFDepthAlgo(cfg, 'cpu')` with `.cuda()` neutralised."""
    ns = load()
    orig = nn.Module.cuda
    nn.Module.cuda = lambda self, *a, **k: self
    try:
        algo = ns.vfdepth.VFDepthAlgo(cfg, 'cpu')
    finally:
        nn.Module.cuda = orig
    return algo

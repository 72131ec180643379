"""Data path: DDAD / NuScenes readers producing the `align_dataset` schema, the
packnet-sfm sample transforms the reference trains with, and a pinned-memory device prefetcher.

Reference chain (`/root/reference/dataset/`):

* `base_dataset.py:5-50` `construct_dataset(cfg, mode, **augmentation)`  → `construct_dataset`
* `ddad_dataset_sf.py:13-155` `DDADdatasetSF` (over dgp's `SynchronizedSceneDataset`)  → `DDADDataset`
* `nuscenes_dataset.py:17-281` `NuScenesdataset` (over nuscenes-devkit)  → `NuScenesDataset`
* `data_util.py:13-91` `transform_mask_sample`, `img_loader`, `mask_loader_scene`, `align_dataset`
  → same names here
* packnet-sfm `datasets/transforms.py` / `augmentations.py` (`get_transforms`, `resize_sample`,
  `duplicate_sample`, `colorjitter_sample`, `to_tensor_sample`) and `dgp_dataset.py`
  (`stack_sample`), imported by the reference from its empty `external/packnet_sfm` submodule
  (`external/dataset/__init__.py:2-5`): restated from the published packnet-sfm code.

Third-party readers the reference depends on are absent offline, so their on-disk formats are
read directly: dgp's scene / calibration JSON (`scene_splits` dataset index, `samples` with
`datum_keys` + `calibration_key`, image datums, `calibration/<key>.json` with per-sensor pinhole
intrinsics and sensor→body extrinsics as translation + quaternion) and nuscenes-devkit's JSON tables
(`sample`, `sample_data`, `calibrated_sensor`, `ego_pose`); pyquaternion's quaternion → rotation
matrix is restated.  Parity: `align_dataset` is pinned by a fixture of the reference's own function
(`tests/golden/data_align.npz`); the PIL resizes, colour jitter and the format readers have no
reference-side vector ("parity unpinned") and are tested for schema and geometry round trips.

Not ported: the reference's `mask_idx_dict.pkl` (scene → DDAD self-occlusion mask set) is a pickle
and is never unpickled here; give the same mapping as JSON (`data.mask_idx_json`) or every scene uses
mask set 0.
"""
import functools
import json
import os
import random
import threading

import numpy as np
import PIL.Image as pil
from PIL import ImageEnhance
import torch
import torch.nn.functional as F
from torch.utils.data import Dataset

_DEL_KEYS = ['rgb', 'rgb_context', 'rgb_original', 'rgb_context_original', 'intrinsics', 'contexts', 'splitname']
_GLOBAL_KEYS = ['idx', 'dataset_idx', 'sensor_name', 'filename', 'token']
_LANCZOS = pil.LANCZOS          # PIL's ANTIALIAS (removed in Pillow 10) is this filter


# ----------------------------------------------------------------------------- loaders
def img_loader(path):
    """data_util.py:27-33: RGB PIL image."""
    with open(path, 'rb') as f:
        with pil.open(f) as img:
            return img.convert('RGB')


def mask_loader_scene(path, mask_idx, cam):
    """data_util.py:36-43: `<path>/<mask_idx>/<CAM>_mask.png` as an 'L' image."""
    fname = os.path.join(path, str(mask_idx), '{}_mask.png'.format(cam.upper()))
    with open(fname, 'rb') as f:
        with pil.open(f) as img:
            return img.convert('L')


def to_tensor(img):
    """torchvision ToTensor for PIL images: uint8 HWC -> float CHW / 255."""
    a = np.asarray(img)
    if a.ndim == 2:
        a = a[:, :, None]
    t = torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))
    return t.float().div(255.0) if a.dtype == np.uint8 else t.float()


def resize_pil(img, shape, interpolation=_LANCZOS):
    """torchvision Resize((h, w)) on a PIL image."""
    h, w = int(shape[0]), int(shape[1])
    return img.resize((w, h), interpolation)


# ----------------------------------------------------------------------------- packnet transforms
def _keys(sample, names):
    return [k for k in names if k in sample]


def resize_depth_preserve(depth, shape):
    """packnet `resize_depth_preserve`: re-grid a sparse depth map keeping every valid point
    (nearest target pixel of each source point; no interpolation across holes)."""
    if depth is None:
        return depth
    depth = np.asarray(depth)
    h, w = depth.shape[:2]
    out = np.zeros(tuple(shape), dtype=depth.dtype)
    ys, xs = np.nonzero(depth > 0)
    if len(ys):
        ty = (ys * shape[0] / h).astype(np.int64)
        tx = (xs * shape[1] / w).astype(np.int64)
        keep = (ty < shape[0]) & (tx < shape[1])
        out[ty[keep], tx[keep]] = depth[ys[keep], xs[keep]]
    return np.expand_dims(out, 2)


def resize_sample(sample, shape, image_interpolation=_LANCZOS):
    """packnet `resize_sample`: images (and contexts) to `shape`, intrinsics rows scaled by the
    size ratio, depth maps re-gridded preserving points."""
    orig_w, orig_h = sample['rgb'].size
    out_h, out_w = shape
    for key in _keys(sample, ['intrinsics']):
        K = np.copy(sample[key])
        K[0] *= out_w / orig_w
        K[1] *= out_h / orig_h
        sample[key] = K
    for key in _keys(sample, ['rgb', 'rgb_original']):
        sample[key] = resize_pil(sample[key], shape, image_interpolation)
    for key in _keys(sample, ['rgb_context', 'rgb_context_original']):
        sample[key] = [resize_pil(k, shape, image_interpolation) for k in sample[key]]
    for key in _keys(sample, ['depth', 'input_depth']):
        sample[key] = resize_depth_preserve(sample[key], shape)
    return sample


def duplicate_sample(sample):
    """packnet `duplicate_sample`: keep un-jittered copies as `*_original`."""
    for key in _keys(sample, ['rgb']):
        sample[key + '_original'] = sample[key].copy()
    for key in _keys(sample, ['rgb_context']):
        sample[key + '_original'] = [k.copy() for k in sample[key]]
    return sample


def _adjust_hue(img, factor):
    """torchvision adjust_hue on PIL: shift the H channel of HSV by factor * 255 (mod 256)."""
    if abs(factor) < 1e-12:
        return img
    h, s, v = img.convert('HSV').split()
    a = np.asarray(h, dtype=np.uint8)
    with np.errstate(over='ignore'):
        a = (a.astype(np.int16) + int(np.uint8(np.int8(round(factor * 255)))) % 256).astype(np.uint8)
    return pil.merge('HSV', (pil.fromarray(a, 'L'), s, v)).convert('RGB')


def color_jitter_fn(brightness, contrast, saturation, hue, rng=random):
    """torchvision ColorJitter.get_params (the pre-0.8 form packnet uses): factors drawn
    uniformly from [max(0, 1-x), 1+x] ([-hue, hue] for hue), applied in a random order."""
    ops = []
    if brightness > 0:
        f = rng.uniform(max(0.0, 1 - brightness), 1 + brightness)
        ops.append(lambda im, f=f: ImageEnhance.Brightness(im).enhance(f))
    if contrast > 0:
        f = rng.uniform(max(0.0, 1 - contrast), 1 + contrast)
        ops.append(lambda im, f=f: ImageEnhance.Contrast(im).enhance(f))
    if saturation > 0:
        f = rng.uniform(max(0.0, 1 - saturation), 1 + saturation)
        ops.append(lambda im, f=f: ImageEnhance.Color(im).enhance(f))
    if hue > 0:
        f = rng.uniform(-hue, hue)
        ops.append(lambda im, f=f: _adjust_hue(im, f))
    rng.shuffle(ops)

    def apply(im):
        for op in ops:
            im = op(im)
        return im
    return apply


def colorjitter_sample(sample, parameters, prob=1.0):
    """packnet `colorjitter_sample`: one jitter draw for the sample's image and its contexts."""
    if random.random() < prob:
        jit = color_jitter_fn(*parameters)
        for key in _keys(sample, ['rgb']):
            sample[key] = jit(sample[key])
        for key in _keys(sample, ['rgb_context']):
            sample[key] = [jit(k) for k in sample[key]]
    return sample


def to_tensor_sample(sample):
    """packnet `to_tensor_sample`."""
    for key in _keys(sample, ['rgb', 'rgb_original']):
        sample[key] = to_tensor(sample[key])
    for key in _keys(sample, ['depth', 'input_depth']):
        if sample[key] is not None:
            sample[key] = torch.from_numpy(np.ascontiguousarray(np.asarray(sample[key]).transpose(2, 0, 1))).float()
    for key in _keys(sample, ['rgb_context', 'rgb_context_original']):
        sample[key] = [to_tensor(k) for k in sample[key]]
    return sample


def train_transforms(sample, image_shape, jittering, crop_train_borders=()):
    if len(image_shape) > 0:
        sample = resize_sample(sample, image_shape)
    sample = duplicate_sample(sample)
    if len(jittering) > 0 and any(float(j) > 0 for j in jittering):
        sample = colorjitter_sample(sample, jittering)
    return to_tensor_sample(sample)


def validation_transforms(sample, image_shape, crop_eval_borders=()):
    if len(image_shape) > 0:
        sample['rgb'] = resize_pil(sample['rgb'], image_shape)
        if 'rgb_context' in sample:
            sample['rgb_context'] = [resize_pil(k, image_shape) for k in sample['rgb_context']]
        if 'intrinsics' in sample:
            pass        # packnet's eval path keeps K (the reference only uses 'train' transforms)
    return to_tensor_sample(sample)


def get_transforms(mode, image_shape, jittering=(), crop_train_borders=(), crop_eval_borders=(), **kwargs):
    """packnet `get_transforms`: a functools.partial whose `.keywords['image_shape']` the
    reference's `transform_mask_sample` reads (data_util.py:17)."""
    if mode == 'train':
        return functools.partial(train_transforms, image_shape=image_shape, jittering=jittering,
                                 crop_train_borders=crop_train_borders)
    if mode in ('validation', 'test', 'val'):
        return functools.partial(validation_transforms, image_shape=image_shape, crop_eval_borders=crop_eval_borders)
    raise ValueError('Unknown mode {}'.format(mode))


def transform_mask_sample(sample, data_transform):
    """data_util.py:13-24: mask resized (ANTIALIAS = LANCZOS) to the image shape, to tensor."""
    image_shape = data_transform.keywords['image_shape']
    sample['mask'] = to_tensor(resize_pil(sample['mask'], image_shape))
    return sample


def stack_sample(sample):
    """packnet `dgp_dataset.stack_sample`: per-camera dicts -> one dict, tensors / arrays stacked
    on a new camera axis, lists stacked per element, global keys taken from camera 0."""
    if len(sample) == 1:
        return sample[0]
    out = {}
    for key in sample[0]:
        v0 = sample[0][key]
        if key in _GLOBAL_KEYS:
            out[key] = v0
        elif torch.is_tensor(v0):
            out[key] = torch.stack([s[key] for s in sample], 0)
        elif isinstance(v0, np.ndarray):
            out[key] = np.stack([s[key] for s in sample], 0)
        elif isinstance(v0, list):
            out[key] = []
            if v0 and torch.is_tensor(v0[0]):
                out[key] = [torch.stack([s[key][i] for s in sample], 0) for i in range(len(v0))]
            elif v0 and isinstance(v0[0], np.ndarray):
                out[key] = [np.stack([s[key][i] for s in sample], 0) for i in range(len(v0))]
    return out


def align_dataset(sample, scales, contexts):
    """data_util.py:46-91: per-scale K / pinv(K) and bilinear (align_corners=False) image
    pyramids of the original and the augmented images, context frames under ('color', f, 0),
    the raw keys dropped."""
    K = sample['intrinsics']
    aug, aug_ctx = sample['rgb'], sample['rgb_context']
    org, org_ctx = sample['rgb_original'], sample['rgb_context_original']
    n_cam, _, h, w = aug.shape
    K4 = np.repeat(np.eye(4)[None], n_cam, axis=0)
    K4[:, :3, :3] = K
    for s in scales:
        Ks = K4.copy()
        Ks[:, :2, :] /= 2 ** s
        sample[('K', s)] = Ks.copy()
        sample[('inv_K', s)] = np.linalg.pinv(Ks).copy()
        size = (h // 2 ** s, w // 2 ** s)
        sample[('color', 0, s)] = F.interpolate(org, size=size, mode='bilinear', align_corners=False)
        sample[('color_aug', 0, s)] = F.interpolate(aug, size=size, mode='bilinear', align_corners=False)
    for i, f in enumerate(contexts):
        sample[('color', f, 0)] = org_ctx[i]
        sample[('color_aug', f, 0)] = aug_ctx[i]
    for key in list(sample.keys()):
        if key in _DEL_KEYS:
            del sample[key]
    return sample


# ----------------------------------------------------------------------------- geometry helpers
def quat_to_matrix(qw, qx, qy, qz):
    """Unit quaternion -> 3x3 rotation (pyquaternion's rotation_matrix; normalised first)."""
    q = np.array([qw, qx, qy, qz], dtype=np.float64)
    q = q / np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def pose_matrix(rotation, translation):
    T = np.eye(4)
    T[:3, :3] = rotation
    T[:3, 3] = np.asarray(translation, dtype=np.float64).reshape(3)
    return T


def project_depth_map(points_cam, K, height, width):
    """Sparse depth image of camera-frame points (z > 0, rounded pixel inside the image; a later
    point overwrites an earlier one at the same pixel, as the reference's fancy-index store)."""
    pts = np.asarray(points_cam, dtype=np.float64)
    pts = pts[pts[:, 2] > 0]
    uvw = pts @ np.asarray(K, dtype=np.float64)[:3, :3].T
    uv = uvw[:, :2] / uvw[:, 2:3]
    keep = (uv[:, 0] >= 0) & (uv[:, 0] <= width - 1) & (uv[:, 1] >= 0) & (uv[:, 1] <= height - 1)
    uv = np.round(uv[keep]).astype(np.int64)
    depth = np.zeros((height, width))
    depth[uv[:, 1], uv[:, 0]] = pts[keep, 2]
    return depth


def _load_depth_npz(path):
    with np.load(path, allow_pickle=False) as z:        # arrays only: never unpickle
        return z['depth']


def _contexts(bwd, fwd):
    return ([-1] if bwd else []) + ([1] if fwd else [])


# ----------------------------------------------------------------------------- DDAD (dgp format)
class DDADDataset(Dataset):
    """DDAD surround-view samples in the trainer's schema (ddad_dataset_sf.py:13-155).

    `path` is dgp's dataset JSON (`ddad.json`: `scene_splits` {"0": train, "1": val, "2": test}
    → scene JSON files relative to its directory).  A sample is one `samples[i]` of a scene whose
    `±context` neighbours exist (dgp SynchronizedSceneDataset's index); per camera it yields the
    image, pinhole K (fx, fy, cx, cy, skew), camera→vehicle extrinsics from the scene's
    calibration file, the self-occlusion mask and the context images (same camera, samples i∓1).
    Depth for val/eval: `<scene>/depth/<depth_type>/<CAMERA>/<stem>.npz` (key 'depth', as the
    reference caches it), else projected from the sample's lidar point cloud datum
    (`point_cloud.filename` npz, key 'data' = x, y, z in the lidar frame)."""

    _SPLITS = {'train': '0', 'val': '1', 'validation': '1', 'test': '2'}

    def __init__(self, path, split, cameras, back_context=0, forward_context=0, data_transform=None,
                 depth_type=None, scale_range=0, with_pose=True, with_mask=True, mask_path=None,
                 mask_idx=None):
        self.path, self.split = path, split
        self.cameras = [c.upper() for c in cameras]
        self.num_cameras = len(cameras)
        self.bwd, self.fwd = int(back_context), int(forward_context)
        self.has_context = self.bwd + self.fwd > 0
        self.data_transform = data_transform
        self.depth_type = depth_type
        self.with_depth = depth_type is not None
        self.with_pose, self.with_mask = with_pose, with_mask
        self.scales = np.arange(scale_range + 2)
        self.dataset_idx = 0
        self.mask_path = mask_path
        self.mask_idx = mask_idx or {}
        root = os.path.dirname(os.path.abspath(path))
        with open(path) as f:
            index = json.load(f)
        files = index['scene_splits'][self._SPLITS.get(split, split)]['filenames']
        self.scenes, self.items = [], []
        for fn in files:
            scene_file = os.path.join(root, fn)
            with open(scene_file) as f:
                scene = json.load(f)
            scene['_dir'] = os.path.dirname(scene_file)
            scene['_data'] = {d['key']: d for d in scene['data']}
            scene['_calib'] = {}
            si = len(self.scenes)
            self.scenes.append(scene)
            n = len(scene['samples'])
            self.items += [(si, i) for i in range(self.bwd, n - self.fwd)]

    def __len__(self):
        return len(self.items)

    def _calibration(self, scene, key):
        if key not in scene['_calib']:
            with open(os.path.join(scene['_dir'], 'calibration', key + '.json')) as f:
                cal = json.load(f)
            out = {}
            for name, intr, extr in zip(cal['names'], cal['intrinsics'], cal['extrinsics']):
                K = np.array([[intr['fx'], intr.get('skew', 0.0), intr['cx']],
                              [0.0, intr['fy'], intr['cy']],
                              [0.0, 0.0, 1.0]], dtype=np.float32)
                r, t = extr['rotation'], extr['translation']
                E = pose_matrix(quat_to_matrix(r['qw'], r['qx'], r['qy'], r['qz']), [t['x'], t['y'], t['z']])
                out[name.upper()] = (K, E)
            scene['_calib'][key] = out
        return scene['_calib'][key]

    def _datum(self, scene, sample_idx, name):
        smp = scene['samples'][sample_idx]
        for k in smp['datum_keys']:
            d = scene['_data'][k]
            if d['id']['name'].upper() == name:
                return d
        raise KeyError('datum {} missing in sample {}'.format(name, sample_idx))

    def _image(self, scene, sample_idx, cam):
        d = self._datum(scene, sample_idx, cam)
        return img_loader(os.path.join(scene['_dir'], d['datum']['image']['filename']))

    def _depth(self, scene, sample_idx, cam, K, E, size):
        d = self._datum(scene, sample_idx, cam)
        stem = os.path.splitext(d['datum']['image']['filename'])[0].replace('rgb', 'depth/' + self.depth_type, 1)
        cache = os.path.join(scene['_dir'], stem + '.npz')
        if os.path.exists(cache):
            return _load_depth_npz(cache)
        smp = scene['samples'][sample_idx]
        lidar = [scene['_data'][k] for k in smp['datum_keys']
                 if scene['_data'][k]['id']['name'].lower() == self.depth_type.lower()]
        if not lidar:
            raise FileNotFoundError('no cached depth {} and no {} datum'.format(cache, self.depth_type))
        pc = lidar[0]['datum']['point_cloud']
        with np.load(os.path.join(scene['_dir'], pc['filename']), allow_pickle=False) as z:
            pts = z['data'][:, :3].astype(np.float64)
        _, E_l = self._calibration(scene, smp['calibration_key'])[self.depth_type.upper()]
        hom = np.concatenate([pts, np.ones((len(pts), 1))], 1)
        cam_pts = (np.linalg.inv(E) @ E_l @ hom.T).T[:, :3]          # lidar -> vehicle -> camera
        return project_depth_map(cam_pts, K, size[1], size[0])

    def _mask_set(self, scene_name):
        """The scene's self-occlusion mask set: the reference looks up `mask_idx_dict[int(scene)]`
        (ddad_dataset_sf.py:102), so a JSON dump of its dict has keys like '150' for directory
        '000150'.  No mapping given: every scene uses set 0 (documented in the module header); a
        mapping that lacks the scene is an error, not a silent fallback."""
        if not self.mask_idx:
            return 0
        keys = [scene_name]
        if scene_name.isdigit():
            keys = [str(int(scene_name)), int(scene_name), scene_name]
        for k in keys:
            if k in self.mask_idx:
                return self.mask_idx[k]
        raise KeyError(f'scene {scene_name!r} is not in the mask-set mapping (tried {keys})')

    def __getitem__(self, idx):
        si, i = self.items[idx]
        scene = self.scenes[si]
        contexts = _contexts(self.bwd, self.fwd)
        calib = self._calibration(scene, scene['samples'][i]['calibration_key'])
        scene_name = os.path.basename(scene['_dir'])
        mask_idx = self._mask_set(scene_name)
        sample = []
        for cam in self.cameras:
            K, E = calib[cam]
            rgb = self._image(scene, i, cam)
            d = self._datum(scene, i, cam)
            data = {'idx': idx, 'dataset_idx': self.dataset_idx, 'sensor_name': cam, 'contexts': contexts,
                    'filename': os.path.join(scene_name, os.path.splitext(d['datum']['image']['filename'])[0]),
                    'splitname': '%s_%010d' % (self.split, idx), 'rgb': rgb, 'intrinsics': K.copy()}
            if self.with_depth:
                data['depth'] = self._depth(scene, i, cam, K, E, rgb.size)
            if self.with_pose:
                data['extrinsics'] = E.astype(np.float32)
            if self.with_mask:
                data['mask'] = (pil.new('L', rgb.size, 255) if self.mask_path == ALL_ONES_MASK
                                else mask_loader_scene(self.mask_path, mask_idx, cam))
            if self.has_context:
                data['rgb_context'] = ([self._image(scene, i - 1, cam)] if self.bwd else []) + \
                                      ([self._image(scene, i + 1, cam)] if self.fwd else [])
            sample.append(data)
        return _finish(sample, self, contexts)


def _finish(sample, ds, contexts):
    """ddad_dataset_sf.py:147-155 / nuscenes_dataset.py:272-280: per-camera transforms, stack,
    align."""
    if ds.data_transform:
        sample = [ds.data_transform(s) for s in sample]
        if ds.with_mask:
            sample = [transform_mask_sample(s, ds.data_transform) for s in sample]
    if ds.with_depth:
        for s in sample:
            if not torch.is_tensor(s['depth']):
                s['depth'] = torch.from_numpy(np.asarray(s['depth'], dtype=np.float32))[None]
    sample = stack_sample(sample)
    return align_dataset(sample, ds.scales, contexts)


# ----------------------------------------------------------------------------- NuScenes
class NuScenesDataset(Dataset):
    """NuScenes samples in the trainer's schema (nuscenes_dataset.py:17-281) over the devkit's
    JSON tables in `<path>/<version>/`; the split file `<split_dir>/<split>.txt` lists one sample
    token per line (the reference reads `dataset/nuscenes/<split>.txt`).  Contexts follow the
    camera's `prev` / `next` sample_data (the current frame itself for 'val', as the reference);
    extrinsics = calibrated_sensor rotation (quaternion w, x, y, z) + translation; depth = the
    LIDAR_TOP sweep projected through lidar→ego→world→ego(cam time)→camera."""

    _TABLES = ('sample', 'sample_data', 'calibrated_sensor', 'ego_pose')

    def __init__(self, path, split, cameras, back_context=0, forward_context=0, data_transform=None,
                 depth_type=None, scale_range=0, with_pose=True, with_mask=True, version='v1.0-trainval',
                 split_dir=None, mask_path=None):
        self.path, self.split = path, split
        self.cameras = [c.upper() for c in cameras]
        self.num_cameras = len(cameras)
        self.bwd, self.fwd = int(back_context), int(forward_context)
        self.has_context = self.bwd + self.fwd > 0
        self.data_transform = data_transform
        self.with_depth = depth_type is not None
        self.with_pose, self.with_mask = with_pose, with_mask
        self.scales = np.arange(scale_range + 2)
        self.dataset_idx = 0
        self.mask_path = mask_path
        self.tables = {}
        for t in self._TABLES:
            with open(os.path.join(path, version, t + '.json')) as f:
                self.tables[t] = {r['token']: r for r in json.load(f)}
        with open(os.path.join(split_dir or os.path.join(path, 'splits'), split + '.txt')) as f:
            self.filenames = [ln.strip().split()[0] for ln in f if ln.strip()]

    def get(self, table, token):
        return self.tables[table][token]

    def __len__(self):
        return len(self.filenames)

    def _extrinsics(self, cs):
        r = cs['rotation']
        return pose_matrix(quat_to_matrix(*r), cs['translation']).astype(np.float32)

    def _depth(self, sample, cam_sd):
        """nuscenes_dataset.py:103-210: the cached map `<dirname(path)>/samples/DEPTH_MAP/<CAM>/
        <image file>.npz` when it exists (read with allow_pickle=False: arrays only), else the
        LIDAR_TOP sweep projected; the homogeneous ego-frame points are rounded to fp32 before the
        lidar -> camera transform, as the reference's `torch.from_numpy(...).float()` does."""
        cam = cam_sd['filename'].split('/')[-2] if '/' in cam_sd['filename'] else ''
        cache = os.path.join(os.path.dirname(self.path), 'samples', 'DEPTH_MAP', cam, cam_sd['filename'] + '.npz')
        if os.path.exists(cache):
            return _load_depth_npz(cache)
        lid = self.get('sample_data', sample['data']['LIDAR_TOP'])
        pts = np.fromfile(os.path.join(self.path, lid['filename']), dtype=np.float32).reshape(-1, 5)[:, :3]
        lp = self.get('ego_pose', lid['ego_pose_token'])
        lidar_to_world = pose_matrix(quat_to_matrix(*lp['rotation']), lp['translation'])
        ls = self.get('calibrated_sensor', lid['calibrated_sensor_token'])
        ego_pts = pts.astype(np.float64) @ quat_to_matrix(*ls['rotation']).T + np.asarray(ls['translation'])
        hom = np.concatenate([ego_pts, np.ones((len(ego_pts), 1))], 1).astype(np.float32).astype(np.float64)
        ep = self.get('ego_pose', cam_sd['ego_pose_token'])
        world_to_ego = np.linalg.inv(pose_matrix(quat_to_matrix(*ep['rotation']), ep['translation']))
        cs = self.get('calibrated_sensor', cam_sd['calibrated_sensor_token'])
        ego_to_cam = np.linalg.inv(pose_matrix(quat_to_matrix(*cs['rotation']), cs['translation']))
        cam_pts = (ego_to_cam @ world_to_ego @ lidar_to_world @ hom.T).T[:, :3]
        with pil.open(os.path.join(self.path, cam_sd['filename'])) as im:
            w, h = im.size
        return project_depth_map(cam_pts, np.asarray(cs['camera_intrinsic']), h, w)

    def __getitem__(self, idx):
        sample_nusc = self.get('sample', self.filenames[idx])
        contexts = _contexts(self.bwd, self.fwd)
        sample = []
        for cam in self.cameras:
            sd = self.get('sample_data', sample_nusc['data'][cam])
            cs = self.get('calibrated_sensor', sd['calibrated_sensor_token'])
            data = {'idx': idx, 'sensor_name': cam, 'contexts': contexts, 'filename': sd['filename'],
                    'rgb': img_loader(os.path.join(self.path, sd['filename'])),
                    'intrinsics': np.array(cs['camera_intrinsic'], dtype=np.float32)}
            if self.with_depth:
                data['depth'] = self._depth(sample_nusc, sd)
            if self.with_pose:
                data['extrinsics'] = self._extrinsics(cs)
            if self.with_mask:
                data['mask'] = (pil.new('L', data['rgb'].size, 255) if self.mask_path == ALL_ONES_MASK
                                else mask_loader_scene(self.mask_path, '', cam))
            if self.has_context:
                ctx = []
                for k, on in (('prev', self.bwd), ('next', self.fwd)):
                    if on:
                        c_sd = sd if self.split == 'val' else self.get('sample_data', sd[k])
                        ctx.append(img_loader(os.path.join(self.path, c_sd['filename'])))
                data['rgb_context'] = ctx
            sample.append(data)
        return _finish(sample, self, contexts)


# ----------------------------------------------------------------------------- construction
def augmentation(cfg, mode):
    """models/vfdepth.py:98-103, 133-138: resize to (height, width); colour jitter for training."""
    tr = cfg['training']
    jit = (0.2, 0.2, 0.2, 0.05) if mode == 'train' else (0.0, 0.0, 0.0, 0.0)
    return {'image_shape': (int(tr['height']), int(tr['width'])), 'jittering': jit,
            'crop_train_borders': (), 'crop_eval_borders': ()}


ALL_ONES_MASK = 'all_ones'


def _mask_path(d, req):
    """`data.mask_path` when the requirements include 'mask'.  The reference always loads the
    self-occlusion masks (dataset/ddad_mask, dataset/nuscenes_mask); training without them changes
    the loss, so it must be asked for explicitly: `data.mask_path: 'all_ones'`."""
    path = d.get('mask_path')
    if 'mask' in req and not path:
        raise ValueError("data.mask_path is not set but the requirements include 'mask': point it at the "
                         "self-occlusion mask directory, or set it to 'all_ones' to train without masks")
    return path


def construct_dataset(cfg, mode, **kwargs):
    """base_dataset.py:5-50 (both modes use the 'train' transform, as the reference)."""
    d, m = cfg['data'], cfg['model']
    req = d['train_requirements'] if mode == 'train' else d['val_requirements']
    args = {'cameras': d['cameras'], 'back_context': d['back_context'], 'forward_context': d['forward_context'],
            'data_transform': get_transforms('train', **kwargs),
            'depth_type': d['depth_type'] if 'gt_depth' in req else None,
            'scale_range': m['fusion_level'] if 'fusion_level' in m else -1,
            'with_pose': 'gt_pose' in req, 'with_mask': 'mask' in req}
    if d['dataset'] == 'ddad':
        mask_idx = None
        if d.get('mask_idx_json'):
            with open(d['mask_idx_json']) as f:
                mask_idx = json.load(f)
        return DDADDataset(d['data_path'], mode, mask_path=_mask_path(d, req), mask_idx=mask_idx, **args)
    if d['dataset'] == 'nuscenes':
        return NuScenesDataset(d['data_path'], mode, version=d.get('nusc_version', 'v1.0-trainval'),
                               split_dir=d.get('split_dir'), mask_path=_mask_path(d, req), **args)
    raise ValueError('Unknown dataset: ' + d['dataset'])


def collate(batch):
    """DataLoader collate for the trainer schema: tensors / arrays stacked on a batch axis, the
    non-device keys kept as lists (vfdepth.py:17 `_NO_DEVICE_KEYS`)."""
    out = {}
    for key in batch[0]:
        v0 = batch[0][key]
        if torch.is_tensor(v0):
            out[key] = torch.stack([b[key] for b in batch], 0)
        elif isinstance(v0, np.ndarray):
            out[key] = torch.from_numpy(np.stack([b[key] for b in batch], 0))
        elif isinstance(v0, (int, float)):
            out[key] = torch.tensor([b[key] for b in batch])
        else:
            out[key] = [b[key] for b in batch]
    return out


# ----------------------------------------------------------------------------- device prefetch
class DevicePrefetcher:
    """Overlaps the next batch's host→device copy with the current step.

    Wraps a DataLoader built with `pin_memory=True`: while the caller runs step i, batch i+1's
    tensors are copied on a side stream (`non_blocking`, so the DMA engines move them while the
    compute queue runs); `next()` makes the current stream wait on that copy and marks the
    tensors as used by it (`record_stream`) so the caching allocator never recycles them early.
    float64 arrays (K, inv_K, extrinsics) are cast to fp32 on the device, as `process_batch`'s
    `.float()` would.  `VFDepthAlgo.process_batch` skips its own `.to(device)` for tensors already
    on the device, so the step sees resident inputs."""

    def __init__(self, loader, device):
        self.loader, self.device = loader, torch.device(device)
        self.stream = torch.cuda.Stream(self.device) if self.device.type == 'cuda' else None
        self._it, self._next = None, None

    def _copy(self, batch):
        def mv(v):
            if torch.is_tensor(v):
                return v.to(self.device, non_blocking=True).float() if v.is_floating_point() else v.to(self.device, non_blocking=True)
            if isinstance(v, list) and v and torch.is_tensor(v[0]):
                return [mv(t) for t in v]
            return v
        if self.stream is None:
            return {k: mv(v) for k, v in batch.items()}
        with torch.cuda.stream(self.stream):
            return {k: mv(v) for k, v in batch.items()}

    def _preload(self):
        try:
            self._next = self._copy(next(self._it))
        except StopIteration:
            self._next = None

    def __iter__(self):
        self._it = iter(self.loader)
        self._preload()
        return self

    def __next__(self):
        if self._next is None:
            raise StopIteration
        batch = self._next
        if self.stream is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_stream(self.stream)
            for v in batch.values():
                for t in (v if isinstance(v, list) else [v]):
                    if torch.is_tensor(t) and t.is_cuda:
                        t.record_stream(cur)
        self._preload()
        return batch

    def __len__(self):
        return len(self.loader)


class _LoaderError:
    def __init__(self, exc):
        self.exc = exc


class ThreadedLoader:
    """Background-thread batch producer (queue depth `depth`) for map-style datasets when
    DataLoader worker processes are unwanted (e.g. inside a process that already owns the GPU)."""

    def __init__(self, dataset, batch_size, indices=None, depth=2, collate_fn=collate, pin=True):
        import queue
        self.dataset, self.batch_size, self.collate = dataset, int(batch_size), collate_fn
        self.indices = list(range(len(dataset))) if indices is None else list(indices)
        self.depth, self.pin, self._queue = depth, pin, queue

    def __len__(self):
        return len(self.indices) // self.batch_size

    def __iter__(self):
        q = self._queue.Queue(maxsize=self.depth)
        n = len(self)

        def work():
            try:
                for b in range(n):
                    items = [self.dataset[i] for i in self.indices[b * self.batch_size:(b + 1) * self.batch_size]]
                    batch = self.collate(items)
                    if self.pin and torch.cuda.is_available():
                        batch = {k: (v.pin_memory() if torch.is_tensor(v) else v) for k, v in batch.items()}
                    q.put(batch)
            except BaseException as e:          # a bad sample fails the consumer, never hangs it
                q.put(_LoaderError(e))
            finally:
                q.put(None)
        threading.Thread(target=work, daemon=True).start()
        while True:
            b = q.get()
            if b is None:
                return
            if isinstance(b, _LoaderError):
                raise b.exc
            yield b

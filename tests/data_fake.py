"""Writes tiny on-disk datasets in the DDAD (dgp JSON) and NuScenes (devkit JSON tables) layouts
for the data-path tests: the synthetic rig of `vfdepth_amd.synth` (6 cameras, known K and
camera→vehicle E), PNG images (lossless, so pixel values survive the round trip), and a lidar
sweep of ground-plane points whose projected depth is known analytically."""
import json
import os

import numpy as np
import PIL.Image as pil

from vfdepth_amd import synth
from vfdepth_amd.config import DDAD_CAMERAS

NUSC_CAMERAS = ['CAM_FRONT', 'CAM_FRONT_LEFT', 'CAM_FRONT_RIGHT', 'CAM_BACK_LEFT', 'CAM_BACK_RIGHT', 'CAM_BACK']


def _quat_of(R):
    """Rotation matrix -> unit quaternion (w, x, y, z)."""
    m = np.asarray(R, dtype=np.float64)
    t = np.trace(m)
    if t > 0:
        s = 2.0 * np.sqrt(t + 1.0)
        return np.array([0.25 * s, (m[2, 1] - m[1, 2]) / s, (m[0, 2] - m[2, 0]) / s, (m[1, 0] - m[0, 1]) / s])
    i = int(np.argmax(np.diag(m)))
    j, k = (i + 1) % 3, (i + 2) % 3
    s = 2.0 * np.sqrt(1.0 + m[i, i] - m[j, j] - m[k, k])
    q = np.zeros(4)
    q[0] = (m[k, j] - m[j, k]) / s
    q[1 + i] = 0.25 * s
    q[1 + j] = (m[j, i] + m[i, j]) / s
    q[1 + k] = (m[k, i] + m[i, k]) / s
    return q


def frame_image(cam, t, h, w):
    """Deterministic RGB uint8 image of camera `cam` at frame `t`."""
    rng = np.random.default_rng(1000 * cam + t)
    return rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)


def lidar_points(n=4000, seed=3):
    """Points on the vehicle ground plane (z = 0) around the rig, in the vehicle frame."""
    rng = np.random.default_rng(seed)
    r = rng.uniform(3.0, 40.0, n)
    a = rng.uniform(-np.pi, np.pi, n)
    return np.stack([r * np.cos(a), r * np.sin(a), np.zeros(n)], 1)


def write_ddad(root, h=80, w=128, n_samples=4, n_scenes=1):
    """dgp layout: <root>/ddad.json -> <scene>/scene.json, calibration/<key>.json,
    rgb/<CAM>/<t>.png, point_cloud/LIDAR/<t>.npz (vehicle frame = lidar frame)."""
    K = synth.rig_intrinsics(6, h, w)
    E = synth.rig_extrinsics(6)
    files = []
    for sc in range(n_scenes):
        sdir = os.path.join(root, '%06d' % sc)
        os.makedirs(os.path.join(sdir, 'calibration'), exist_ok=True)
        names, intr, extr = [], [], []
        for c, cam in enumerate(DDAD_CAMERAS):
            q = _quat_of(E[c, :3, :3])
            names.append(cam.upper())
            intr.append({'fx': K[c, 0, 0], 'fy': K[c, 1, 1], 'cx': K[c, 0, 2], 'cy': K[c, 1, 2], 'skew': 0.0})
            extr.append({'translation': dict(zip('xyz', E[c, :3, 3].tolist())),
                         'rotation': {'qw': q[0], 'qx': q[1], 'qy': q[2], 'qz': q[3]}})
        names.append('LIDAR')
        intr.append({'fx': 0.0, 'fy': 0.0, 'cx': 0.0, 'cy': 0.0, 'skew': 0.0})
        extr.append({'translation': {'x': 0.0, 'y': 0.0, 'z': 0.0}, 'rotation': {'qw': 1.0, 'qx': 0.0, 'qy': 0.0, 'qz': 0.0}})
        with open(os.path.join(sdir, 'calibration', 'calib0.json'), 'w') as f:
            json.dump({'names': names, 'intrinsics': intr, 'extrinsics': extr}, f)
        samples, data = [], []
        os.makedirs(os.path.join(sdir, 'point_cloud', 'LIDAR'), exist_ok=True)
        for t in range(n_samples):
            keys = []
            for c, cam in enumerate(DDAD_CAMERAS):
                fn = 'rgb/%s/%d.png' % (cam.upper(), t)
                os.makedirs(os.path.join(sdir, os.path.dirname(fn)), exist_ok=True)
                pil.fromarray(frame_image(c, t + 10 * sc, h, w)).save(os.path.join(sdir, fn))
                key = 'k_%d_%s' % (t, cam)
                keys.append(key)
                data.append({'id': {'name': cam.upper(), 'index': str(t)}, 'key': key,
                             'datum': {'image': {'filename': fn, 'height': h, 'width': w, 'channels': 3}}})
            pfn = 'point_cloud/LIDAR/%d.npz' % t
            np.savez(os.path.join(sdir, pfn), data=lidar_points(seed=t).astype(np.float32))
            key = 'k_%d_lidar' % t
            keys.append(key)
            data.append({'id': {'name': 'LIDAR', 'index': str(t)}, 'key': key,
                         'datum': {'point_cloud': {'filename': pfn}}})
            samples.append({'id': {'index': str(t)}, 'datum_keys': keys, 'calibration_key': 'calib0'})
        with open(os.path.join(sdir, 'scene.json'), 'w') as f:
            json.dump({'name': 'scene%d' % sc, 'samples': samples, 'data': data}, f)
        files.append('%06d/scene.json' % sc)
    path = os.path.join(root, 'ddad.json')
    with open(path, 'w') as f:
        json.dump({'scene_splits': {'0': {'filenames': files}, '1': {'filenames': files}}}, f)
    return path, K, E


def write_nuscenes(root, h=80, w=128, n_samples=4):
    """devkit tables under <root>/v1.0-mini/, images samples/<CAM>/<t>.png, LIDAR_TOP .bin
    sweeps (x, y, z, intensity, ring; lidar frame = ego frame), ego poses translating along x."""
    K = synth.rig_intrinsics(6, h, w)
    E = synth.rig_extrinsics(6)
    tab = {'sample': [], 'sample_data': [], 'calibrated_sensor': [], 'ego_pose': []}
    for c, cam in enumerate(NUSC_CAMERAS):
        q = _quat_of(E[c, :3, :3])
        tab['calibrated_sensor'].append({'token': 'cs_' + cam, 'translation': E[c, :3, 3].tolist(),
                                         'rotation': q.tolist(), 'camera_intrinsic': K[c, :3, :3].tolist()})
    tab['calibrated_sensor'].append({'token': 'cs_LIDAR_TOP', 'translation': [0.0, 0.0, 0.0],
                                     'rotation': [1.0, 0.0, 0.0, 0.0], 'camera_intrinsic': []})
    for t in range(n_samples):
        tab['ego_pose'].append({'token': 'ep_%d' % t, 'translation': [2.0 * t, 0.0, 0.0], 'rotation': [1.0, 0.0, 0.0, 0.0]})
        data = {}
        for c, cam in enumerate(NUSC_CAMERAS + ['LIDAR_TOP']):
            tok = 'sd_%d_%s' % (t, cam)
            data[cam] = tok
            if cam == 'LIDAR_TOP':
                fn = 'samples/LIDAR_TOP/%d.bin' % t
                os.makedirs(os.path.join(root, os.path.dirname(fn)), exist_ok=True)
                pts = lidar_points(seed=t)
                pts = np.concatenate([pts, np.zeros((len(pts), 2))], 1).astype(np.float32)
                pts.tofile(os.path.join(root, fn))
            else:
                fn = 'samples/%s/%d.png' % (cam, t)
                os.makedirs(os.path.join(root, os.path.dirname(fn)), exist_ok=True)
                pil.fromarray(frame_image(c, t, h, w)).save(os.path.join(root, fn))
            tab['sample_data'].append({'token': tok, 'filename': fn, 'calibrated_sensor_token': 'cs_' + cam,
                                       'ego_pose_token': 'ep_%d' % t,
                                       'prev': 'sd_%d_%s' % (t - 1, cam) if t > 0 else '',
                                       'next': 'sd_%d_%s' % (t + 1, cam) if t + 1 < n_samples else ''})
        tab['sample'].append({'token': 's_%d' % t, 'data': data})
    os.makedirs(os.path.join(root, 'v1.0-mini'), exist_ok=True)
    for k, v in tab.items():
        with open(os.path.join(root, 'v1.0-mini', k + '.json'), 'w') as f:
            json.dump(v, f)
    os.makedirs(os.path.join(root, 'splits'), exist_ok=True)
    with open(os.path.join(root, 'splits', 'train.txt'), 'w') as f:
        f.write(''.join('s_%d\n' % t for t in range(1, n_samples - 1)))
    with open(os.path.join(root, 'splits', 'val.txt'), 'w') as f:
        f.write(''.join('s_%d\n' % t for t in range(n_samples)))
    return root, K, E

"""Axis-angle rotations (the pytorch3d functions the reference imports; pytorch3d is unpinned
in `/root/reference/requirements.txt:11` and absent here).

`axis_angle_to_matrix` restates pytorch3d's published algorithm: axis-angle → unit quaternion
(cos θ/2, sin(θ/2)/θ · a), with the Taylor form 1/2 − θ²/48 for θ < 1e-6, → rotation matrix.
Used by `vec_to_matrix` (`/root/reference/models/geometry/geometry_util.py:8-30`).
"""
import torch


def axis_angle_to_quaternion(axis_angle):
    angles = torch.norm(axis_angle, p=2, dim=-1, keepdim=True)
    half = angles * 0.5
    small = angles.abs() < 1e-6
    safe = torch.where(small, torch.ones_like(angles), angles)
    k = torch.where(small, 0.5 - (angles * angles) / 48, torch.sin(half) / safe)
    return torch.cat([torch.cos(half), axis_angle * k], dim=-1)


def quaternion_to_matrix(q):
    r, i, j, k = torch.unbind(q, -1)
    s = 2.0 / (q * q).sum(-1)
    m = torch.stack((
        1 - s * (j * j + k * k), s * (i * j - k * r), s * (i * k + j * r),
        s * (i * j + k * r), 1 - s * (i * i + k * k), s * (j * k - i * r),
        s * (i * k - j * r), s * (j * k + i * r), 1 - s * (i * i + j * j),
    ), -1)
    return m.reshape(q.shape[:-1] + (3, 3))


def axis_angle_to_matrix(axis_angle):
    return quaternion_to_matrix(axis_angle_to_quaternion(axis_angle))


def matrix_to_euler_angles(matrix, convention='XYZ'):
    """Euler angles for the fsm pose-consistency loss (`multi_cam_loss.py:82-83`), XYZ only."""
    if convention != 'XYZ':
        raise NotImplementedError(convention)
    m = matrix
    # intrinsic X-Y-Z: R = Rx(a) Ry(b) Rz(c)
    b = torch.asin(torch.clamp(m[..., 0, 2], -1.0, 1.0))
    a = torch.atan2(-m[..., 1, 2], m[..., 2, 2])
    c = torch.atan2(-m[..., 0, 1], m[..., 0, 0])
    return torch.stack([a, b, c], -1)

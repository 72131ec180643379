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


# pytorch3d's quaternion_to_matrix entries as (product a, product b, sign of b, sign of the s-term)
# over the 16 products q_x * q_y (x, y in r, i, j, k): m = [1|0] + sign_s * s * (P_a + sign_b * P_b)
# — the same products and sums in the same order, so the values are identical; as selections from
# one outer product it is ~10 kernels each way instead of ~30 scalar-shaped ones.
_QM_A = (10, 6, 7, 6, 5, 11, 7, 11, 5)          # jj, ij, ik, ij, ii, jk, ik, jk, ii
_QM_B = (15, 12, 8, 12, 15, 4, 8, 4, 10)        # kk, kr, jr, kr, kk, ir, jr, ir, jj
_QM_SB = (1., -1., 1., 1., 1., -1., -1., 1., 1.)
_QM_SS = (-1., 1., 1., 1., -1., 1., 1., 1., -1.)
_QM_BASE = (1., 0., 0., 0., 1., 0., 0., 0., 1.)
_QM_CACHE = {}


def _qm_consts(device, dtype):
    """0/1 selection matrices [16, 9] of the products (a matmul, not index_select: its backward is
    a plain GEMM, deterministic, where index_select's scatters with atomics)."""
    key = (str(device), dtype)
    if key not in _QM_CACHE:
        sa = torch.zeros(16, 9, dtype=dtype)
        sb = torch.zeros(16, 9, dtype=dtype)
        for k, (a, b) in enumerate(zip(_QM_A, _QM_B)):
            sa[a, k] = 1.0
            sb[b, k] = _QM_SB[k]
        mk = lambda v: torch.tensor(v, dtype=dtype, device=device)  # noqa: E731
        _QM_CACHE[key] = (sa.to(device), sb.to(device), mk(_QM_SS), mk(_QM_BASE))
    return _QM_CACHE[key]


def quaternion_to_matrix(q):
    sa, sb, ss, base = _qm_consts(q.device, q.dtype)
    s = 2.0 / (q * q).sum(-1, keepdim=True)
    P = (q.unsqueeze(-1) * q.unsqueeze(-2)).flatten(-2)
    t = P @ sa + P @ sb           # selections are exact (x * 1 + zeros); sb carries the sign of b
    m = base + ss * (s * t)
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

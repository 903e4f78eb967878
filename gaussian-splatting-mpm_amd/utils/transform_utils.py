"""World <-> grid transforms, covariance rotations and the orbit camera
(utils/transform_utils.py:8-216 of the reference).

Same arithmetic and dtypes as the reference (torch f32 for particle data,
numpy f64 for the camera), but device-agnostic: tensors stay on the device of
their input instead of a hard-coded ``.cuda()``.
"""
from __future__ import annotations

import os

import numpy as np
import torch


# ----------------------------------------------------------- world <-> grid --
def world2grid(means3D: torch.Tensor, sim_args):
    """transform_utils.py:8-15: centre on the bbox midpoint, scale the longest
    side to grid_extent/2, shift to the grid centre."""
    lo = means3D.min(dim=0)[0]
    hi = means3D.max(dim=0)[0]
    center = (lo + hi) / 2.0
    scale = sim_args.grid_extent / 2.0 / (hi - lo).max()
    half = torch.ones(3, device=means3D.device) * sim_args.grid_extent / 2.0
    return (means3D - center) * scale + half, center, scale


def grid2world(means3D: torch.Tensor, covs: torch.Tensor, scaling_modifier, pos_center, sim_args):
    """transform_utils.py:18-21."""
    half = torch.ones(3, device=means3D.device) * sim_args.grid_extent / 2.0
    means = (means3D - half) / scaling_modifier + pos_center
    return means, (covs / (scaling_modifier * scaling_modifier)).view(-1, 6)


# ---------------------------------------------------------------- rotations --
def generate_rotation_matrix(degree, axis, device="cuda"):
    c = torch.cos(degree / 180.0 * 3.1415926)  # the reference's pi literal
    s = torch.sin(degree / 180.0 * 3.1415926)
    if axis == 0:
        m = [[1, 0, 0], [0, c, -s], [0, s, c]]
    elif axis == 1:
        m = [[c, 0, s], [0, 1, 0], [-s, 0, c]]
    elif axis == 2:
        m = [[c, -s, 0], [s, c, 0], [0, 0, 1]]
    else:
        raise ValueError("Invalid axis selection")
    return torch.tensor(m).to(device)


def generate_rotation_matrices(degrees, axises, device="cuda"):
    assert len(degrees) == len(axises)
    return [generate_rotation_matrix(d, a, device) for d, a in zip(degrees, axises)]


def apply_rotation(position_tensor, rotation_matrix):
    return torch.mm(position_tensor, rotation_matrix.T)


def apply_cov_rotation(cov_tensor, rotation_matrix):
    return torch.matmul(rotation_matrix, torch.matmul(cov_tensor, rotation_matrix.T))


_UPPER_TO_FULL = [0, 1, 2, 1, 3, 4, 2, 4, 5]
_FULL_TO_UPPER = [0, 1, 2, 4, 5, 8]


def get_mat_from_upper(upper_mat):
    u = upper_mat.reshape(-1, 6)
    return u[:, _UPPER_TO_FULL].reshape(-1, 3, 3).to(torch.float32)


def get_upper_from_mat(mat):
    return mat.reshape(-1, 9)[:, _FULL_TO_UPPER].to(torch.float32)


def apply_rotations(position_tensor, rotation_matrices):
    for R in rotation_matrices:
        position_tensor = apply_rotation(position_tensor, R)
    return position_tensor


def apply_cov_rotations(upper_cov_tensor, rotation_matrices):
    cov = get_mat_from_upper(upper_cov_tensor)
    for R in rotation_matrices:
        cov = apply_cov_rotation(cov, R)
    return get_upper_from_mat(cov)


def undoshift2center111(position_tensor):
    return position_tensor - torch.tensor([1.0, 1.0, 1.0], device=position_tensor.device)


def apply_inverse_rotation(position_tensor, rotation_matrix):
    return torch.mm(position_tensor, rotation_matrix)


def apply_inverse_rotations(position_tensor, rotation_matrices):
    for R in reversed(rotation_matrices):
        position_tensor = apply_inverse_rotation(position_tensor, R)
    return position_tensor


def apply_inverse_cov_rotations(upper_cov_tensor, rotation_matrices):
    cov = get_mat_from_upper(upper_cov_tensor)
    for R in reversed(rotation_matrices):
        cov = apply_cov_rotation(cov, R.T)
    return get_upper_from_mat(cov)


def undotransform2origin(position_tensor, scale, original_mean_pos):
    return original_mean_pos + position_tensor / scale


def undo_all_transforms(x, rotation_matrices, scale_origin, original_mean_pos):
    return apply_inverse_rotations(undotransform2origin(undoshift2center111(x), scale_origin, original_mean_pos),
                                   rotation_matrices)


def rotate_covs(upper_cov_tensor, mats):
    cov = get_mat_from_upper(upper_cov_tensor)
    for m in mats:
        cov = torch.matmul(m, torch.matmul(cov, m.T))
    return get_upper_from_mat(cov)


def rotate(points, mats):
    for m in mats:
        points = torch.mm(points, m.T)
    return points


def get_rotation_matrix(degree, axis, device="cuda"):
    return generate_rotation_matrix(degree, axis if axis in (0, 1) else 2, device)


def get_rotation_matrices(degrees, device="cuda"):
    assert len(degrees) == 3
    return [get_rotation_matrix(degrees[i], i, device) for i in range(2)]


# -------------------------------------------------------------- orbit camera --
def generate_local_coord(vertical_vector):
    """transform_utils.py:136-148 (f64): up plus two Gram-Schmidt horizontals."""
    up = vertical_vector / np.linalg.norm(vertical_vector)
    h1 = np.array([1, 1, 1])
    if np.abs(np.dot(h1, up)) < 0.01:
        h1 = np.array([0.72, 0.37, -0.67])
    h1 = h1 - np.dot(h1, up) * up
    h1 = h1 / np.linalg.norm(h1)
    h2 = np.cross(h1, up)
    return up, h1, h2


def get_center_view_worldspace_and_observant_coordinate(mpm_space_viewpoint_center, mpm_space_vertical_upward_axis,
                                                        rotation_matrices, scale_origin, original_mean_pos):
    """transform_utils.py:150-173."""
    center_w = undo_all_transforms(mpm_space_viewpoint_center, rotation_matrices, scale_origin, original_mean_pos)
    up_w = undo_all_transforms(mpm_space_vertical_upward_axis + mpm_space_viewpoint_center, rotation_matrices,
                               scale_origin, original_mean_pos)
    axis_w = up_w - center_w
    center_np = np.squeeze(center_w.clone().detach().cpu().numpy(), 0)
    vertical, h1, h2 = generate_local_coord(np.squeeze(axis_w.clone().detach().cpu().numpy(), 0))
    return center_np, np.column_stack((h1, h2, vertical))


def get_point_on_sphere(azimuth, elevation, radius, center, observant_coordinates):
    """transform_utils.py:176-188."""
    a = azimuth / 180.0 * np.pi
    e = elevation / 180.0 * np.pi
    canonical = np.array([np.cos(a) * np.cos(e), np.sin(a) * np.cos(e), np.sin(e)]) * radius
    return center + observant_coordinates @ canonical


def generate_camera_rotation_matrix(camera_to_object, object_vertical_downward):
    """transform_utils.py:204-216: columns (y x z, y, z) with z toward the object."""
    z = camera_to_object / np.linalg.norm(camera_to_object)
    y = object_vertical_downward - np.dot(object_vertical_downward, z) * z
    y = y / np.linalg.norm(y)
    return np.column_stack((np.cross(y, z), y, z))


def get_camera_position_and_rotation(azimuth, elevation, radius, view_center, observant_coordinates):
    """transform_utils.py:191-202."""
    position = get_point_on_sphere(azimuth, elevation, radius, view_center, observant_coordinates)
    R = generate_camera_rotation_matrix(view_center - position, -observant_coordinates[:, 2])
    return position, R


def particle_position_tensor_to_ply(position_tensor, filename):
    """transform_utils.py:241-259: xyz-only binary PLY (debug output)."""
    if os.path.exists(filename):
        os.remove(filename)
    pos = position_tensor.clone().detach().cpu().numpy().astype(np.float32)
    header = ("ply\nformat binary_little_endian 1.0\n"
              f"element vertex {pos.shape[0]}\nproperty float x\nproperty float y\nproperty float z\nend_header\n")
    d = os.path.dirname(filename)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(filename, "wb") as f:
        f.write(header.encode())
        f.write(pos.tobytes())

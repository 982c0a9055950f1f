"""Camera math feeding GaussianRasterizationSettings.

``get_cam_info_gaussian`` restates threestudio.utils.ops.get_cam_info_gaussian (external to the
reference; called at renderer/gaussian_batch_renderer.py:24-26): OpenGL c2w -> flip the camera y/z
axes -> w2c -> transposed (row-vector) 4x4 matrices the rasterizer reads column-major.  The
projection matrix is the reference's getProjectionMatrix (utils/sugar_utils.py:809-829); the
world_view / full_proj / camera_center construction is the one at geometry/sugar.py:891-896.
Batched: every function accepts a leading view dimension, so a whole batch of cameras is built
with a handful of tensor ops instead of the reference's per-view Python loop.
"""
from __future__ import annotations

import math

import torch


def projection_matrix(znear: float, zfar: float, fovx, fovy) -> torch.Tensor:
    """getProjectionMatrix (utils/sugar_utils.py:809-829), batched over fov tensors -> (..., 4, 4)."""
    fovx = torch.as_tensor(fovx, dtype=torch.float32)
    fovy = torch.as_tensor(fovy, dtype=torch.float32)
    tan_y = torch.tan(fovy / 2)
    tan_x = torch.tan(fovx / 2)
    top = tan_y * znear
    bottom = -top
    right = tan_x * znear
    left = -right
    shape = torch.broadcast_shapes(fovx.shape, fovy.shape)
    P = torch.zeros(shape + (4, 4), dtype=torch.float32)
    z_sign = 1.0
    P[..., 0, 0] = 2.0 * znear / (right - left)
    P[..., 1, 1] = 2.0 * znear / (top - bottom)
    P[..., 0, 2] = (right + left) / (right - left)
    P[..., 1, 2] = (top + bottom) / (top - bottom)
    P[..., 3, 2] = z_sign
    P[..., 2, 2] = z_sign * zfar / (zfar - znear)
    P[..., 2, 3] = -(zfar * znear) / (zfar - znear)
    return P


def get_cam_info_gaussian(c2w: torch.Tensor, fovx, fovy, znear: float = 0.1, zfar: float = 100.0):
    """c2w (..., 4, 4) OpenGL camera-to-world -> (world_view_transform, full_proj_transform, camera_center).

    Unlike threestudio's helper this does not modify ``c2w`` in place.
    """
    c2w = c2w.clone().float()
    c2w[..., :3, 1:3] *= -1  # OpenGL -> COLMAP camera axes
    w2c = torch.linalg.inv(c2w)
    world_view = w2c.transpose(-1, -2).contiguous()
    proj = projection_matrix(znear, zfar, fovx, fovy).to(c2w.device).transpose(-1, -2)
    full_proj = world_view @ proj
    camera_center = torch.linalg.inv(world_view)[..., 3, :3].contiguous()
    return world_view, full_proj.contiguous(), camera_center


def orbit_c2w(distance, elevation_deg, azimuth_deg) -> torch.Tensor:
    """Look-at-origin cameras, z up — the recipe of data/uncond.py:305-315 (camera positions :150-200)."""
    distance = torch.as_tensor(distance, dtype=torch.float32)
    elev = torch.deg2rad(torch.as_tensor(elevation_deg, dtype=torch.float32))
    azim = torch.deg2rad(torch.as_tensor(azimuth_deg, dtype=torch.float32))
    distance, elev, azim = torch.broadcast_tensors(distance, elev, azim)
    pos = torch.stack([distance * torch.cos(elev) * torch.cos(azim),
                       distance * torch.cos(elev) * torch.sin(azim),
                       distance * torch.sin(elev)], dim=-1)
    center = torch.zeros_like(pos)
    up = torch.tensor([0.0, 0.0, 1.0]).expand_as(pos)
    lookat = torch.nn.functional.normalize(center - pos, dim=-1)
    right = torch.nn.functional.normalize(torch.cross(lookat, up, dim=-1), dim=-1)
    up = torch.nn.functional.normalize(torch.cross(right, lookat, dim=-1), dim=-1)
    c2w = torch.zeros(pos.shape[:-1] + (4, 4), dtype=torch.float32)
    c2w[..., :3, 0] = right
    c2w[..., :3, 1] = up
    c2w[..., :3, 2] = -lookat
    c2w[..., :3, 3] = pos
    c2w[..., 3, 3] = 1.0
    return c2w


def tan_half_fov(fov) -> float:
    return math.tan(float(fov) * 0.5)


def ray_bundle(c2w, fovy, height: int, width: int, normalize: bool = False):
    """Per-pixel rays of the batch (data/uncond.py:316-329 with threestudio's get_ray_directions /
    get_rays): unit-focal pixel-centre directions (x right, y up, -z), x/y divided by the focal length
    0.5 H / tan(fovy / 2), rotated by c2w; rays_o is the camera position.  ``rays_d_normalize`` is false
    in the MVDream config (configs/gaussian_splatting_mvdream.yaml:23), so rays are not normalised by
    default.  c2w (B, 4, 4) -> rays_o, rays_d (B, H, W, 3)."""
    c2w = torch.as_tensor(c2w, dtype=torch.float32)
    if c2w.dim() == 2:
        c2w = c2w[None]
    fovy = torch.as_tensor(fovy, dtype=torch.float32).reshape(-1).expand(c2w.shape[0])
    i, j = torch.meshgrid(torch.arange(width, dtype=torch.float32) + 0.5,
                          torch.arange(height, dtype=torch.float32) + 0.5, indexing="xy")
    unit = torch.stack([i - width / 2, -(j - height / 2), -torch.ones_like(i)], -1)
    focal = 0.5 * height / torch.tan(0.5 * fovy)
    dirs = unit[None].repeat(c2w.shape[0], 1, 1, 1)
    dirs[..., :2] = dirs[..., :2] / focal[:, None, None, None]
    rays_d = (dirs[:, :, :, None, :] * c2w[:, None, None, :3, :3]).sum(-1)
    if normalize:
        rays_d = torch.nn.functional.normalize(rays_d, dim=-1)
    rays_o = c2w[:, None, None, :3, 3].expand(rays_d.shape)
    return rays_o.contiguous(), rays_d


def light_positions_dreamfusion(c2w, distance: float = 2.0):
    """Light positions of the "dreamfusion" strategy without its random perturbation (data/uncond.py:258-267):
    the camera direction scaled to the light distance.  c2w (B, 4, 4) -> (B, 3)."""
    c2w = torch.as_tensor(c2w, dtype=torch.float32)
    return torch.nn.functional.normalize(c2w[..., :3, 3], dim=-1) * distance

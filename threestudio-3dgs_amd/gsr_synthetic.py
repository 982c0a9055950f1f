"""Synthetic Gaussian scenes and cameras for parity tests and the benchmark.

Recipes follow the reference so the shapes are realistic:
  positions   uniform in a ball of radius 0.8        geometry/gaussian_base.py:350-359
  scales      sqrt(mean squared 3-NN distance)        geometry/gaussian_base.py:434-438 (distCUDA2 recipe,
              clamp_min 1e-7, exp(log(.)) = the activated get_scaling value)
  rotations   random unit quaternions (w, x, y, z)    (identity at init, :439-440, is too easy)
  opacity     U(0.05, 0.95)
  SH          dc = RGB2SH(U(0,1)), rest ~ N(0, 0.05)  RGB2SH geometry/gaussian_base.py:35-36
  cameras     orbit, distance 2.5, fovy 60 deg, elevation 15 deg, azimuth i*360/V (data/uncond.py)
Data is synthetic (no datasets or checkpoints are available offline).
"""
from __future__ import annotations

import math

import numpy as np

C0 = 0.28209479177387814


def knn_scale(xyz: np.ndarray) -> np.ndarray:
    """sqrt(mean of the squared distances to the 3 nearest neighbours) per point (distCUDA2 recipe)."""
    from scipy.spatial import cKDTree

    tree = cKDTree(xyz)
    d, _ = tree.query(xyz, k=4, workers=-1)
    dist2 = np.mean(d[:, 1:] ** 2, axis=1)
    dist2 = np.maximum(dist2, 1e-7)
    return np.sqrt(dist2).astype(np.float32)


def make_scene(n: int, sh_degree: int = 3, seed: int = 0, radius: float = 0.8, scale_mult: float = 1.0,
               opacity_range=(0.05, 0.95)) -> dict:
    rng = np.random.default_rng(seed)
    phis = rng.random(n) * 2 * np.pi
    costheta = rng.random(n) * 2 - 1
    thetas = np.arccos(costheta)
    mu = rng.random(n)
    r = radius * np.cbrt(mu)
    xyz = np.stack([r * np.sin(thetas) * np.cos(phis), r * np.sin(thetas) * np.sin(phis), r * np.cos(thetas)],
                   axis=1).astype(np.float32)
    s = knn_scale(xyz) * scale_mult if n > 4 else np.full(n, 0.05, np.float32)
    scales = np.repeat(s[:, None], 3, axis=1).astype(np.float32)
    # mild anisotropy so EWA is exercised
    scales *= rng.uniform(0.5, 1.5, size=(n, 3)).astype(np.float32)
    q = rng.normal(size=(n, 4)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    opac = rng.uniform(opacity_range[0], opacity_range[1], size=(n, 1)).astype(np.float32)
    M = (sh_degree + 1) ** 2
    sh = np.zeros((n, M, 3), np.float32)
    sh[:, 0, :] = (rng.random((n, 3)) - 0.5) / C0
    if M > 1:
        sh[:, 1:, :] = rng.normal(0.0, 0.05, size=(n, M - 1, 3))
    return dict(means3D=xyz, scales=scales, rotations=q.astype(np.float32), opacities=opac, shs=sh,
                sh_degree=sh_degree)


def orbit_cameras(n_views: int, distance: float = 2.5, fovy_deg: float = 60.0, elevations=(15.0,),
                  azimuth0: float = 0.0):
    """(elevation, azimuth) grid: len(elevations) rows x n_views/len(elevations) azimuths."""
    n_el = len(elevations)
    per = max(1, n_views // n_el)
    cams = []
    for i in range(n_views):
        el = elevations[(i // per) % n_el]
        az = azimuth0 + (i % per) * 360.0 / per
        cams.append(dict(distance=distance, elevation=el, azimuth=az, fovy=math.radians(fovy_deg)))
    return cams


def camera_matrices(cam: dict, znear: float = 0.1, zfar: float = 100.0):
    """numpy (viewmatrix, projmatrix, campos, tanfov) for one orbit camera, via cameras.py."""
    import torch

    from diff_gaussian_rasterization.cameras import get_cam_info_gaussian, orbit_c2w

    c2w = orbit_c2w(cam["distance"], cam["elevation"], cam["azimuth"])
    wv, fp, cc = get_cam_info_gaussian(c2w, cam["fovy"], cam["fovy"], znear, zfar)
    tan = math.tan(cam["fovy"] * 0.5)
    return (wv.numpy().astype(np.float32), fp.numpy().astype(np.float32), cc.numpy().astype(np.float32), tan)


def upstream_grads(H: int, W: int, seed: int = 1):
    """Seeded dL/dcolor (3,H,W), dL/ddepth (1,H,W), dL/dalpha (1,H,W) ~ N(0,1)."""
    rng = np.random.default_rng(seed)
    return (rng.standard_normal((3, H, W)).astype(np.float32), rng.standard_normal((1, H, W)).astype(np.float32),
            rng.standard_normal((1, H, W)).astype(np.float32))

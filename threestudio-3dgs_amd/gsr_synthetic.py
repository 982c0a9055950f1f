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


def icosphere(subdiv: int, radius: float = 0.6, bump: float = 0.05):
    """Icosphere mesh (20 * 4^subdiv faces) with a smooth radial bump; vertices (V, 3), faces (F, 3)."""
    t = (1.0 + 5 ** 0.5) / 2
    v = np.array([[-1, t, 0], [1, t, 0], [-1, -t, 0], [1, -t, 0], [0, -1, t], [0, 1, t], [0, -1, -t], [0, 1, -t],
                  [t, 0, -1], [t, 0, 1], [-t, 0, -1], [-t, 0, 1]], np.float64)
    f = np.array([[0, 11, 5], [0, 5, 1], [0, 1, 7], [0, 7, 10], [0, 10, 11], [1, 5, 9], [5, 11, 4], [11, 10, 2],
                  [10, 7, 6], [7, 1, 8], [3, 9, 4], [3, 4, 2], [3, 2, 6], [3, 6, 8], [3, 8, 9], [4, 9, 5],
                  [2, 4, 11], [6, 2, 10], [8, 6, 7], [9, 8, 1]], np.int64)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    for _ in range(subdiv):
        e = np.concatenate([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]])
        e.sort(axis=1)
        uniq, inv = np.unique(e, axis=0, return_inverse=True)
        mid = v[uniq[:, 0]] + v[uniq[:, 1]]
        mid /= np.linalg.norm(mid, axis=1, keepdims=True)
        m = inv.reshape(3, -1) + len(v)
        v = np.concatenate([v, mid])
        a, b, c = f[:, 0], f[:, 1], f[:, 2]
        ab, bc, ca = m[0], m[1], m[2]
        f = np.concatenate([np.stack([a, ab, ca], 1), np.stack([b, bc, ab], 1), np.stack([c, ca, bc], 1),
                            np.stack([ab, bc, ca], 1)])
    r = radius * (1.0 + bump * np.sin(5 * v[:, 0]) * np.sin(4 * v[:, 1]) * np.sin(3 * v[:, 2] + 1.0))
    return (v * r[:, None]).astype(np.float64), f


def _matrix_to_quaternion(R: np.ndarray) -> np.ndarray:
    """(N, 3, 3) rotation matrices -> unit quaternions (w, x, y, z) with R = build_rotation(q)
    (the convention of pytorch3d's matrix_to_quaternion used at geometry/sugar.py:527)."""
    w = np.sqrt(np.maximum(0.0, 1.0 + R[:, 0, 0] + R[:, 1, 1] + R[:, 2, 2])) / 2
    x = np.sqrt(np.maximum(0.0, 1.0 + R[:, 0, 0] - R[:, 1, 1] - R[:, 2, 2])) / 2
    y = np.sqrt(np.maximum(0.0, 1.0 - R[:, 0, 0] + R[:, 1, 1] - R[:, 2, 2])) / 2
    z = np.sqrt(np.maximum(0.0, 1.0 - R[:, 0, 0] - R[:, 1, 1] + R[:, 2, 2])) / 2
    x = np.copysign(x, R[:, 2, 1] - R[:, 1, 2])
    y = np.copysign(y, R[:, 0, 2] - R[:, 2, 0])
    z = np.copysign(z, R[:, 1, 0] - R[:, 0, 1])
    q = np.stack([w, x, y, z], 1)
    return q / np.linalg.norm(q, axis=1, keepdims=True)


def make_sugar_scene(subdiv: int = 7, sh_degree: int = 3, seed: int = 0, thickness: float = 3.5e-6) -> dict:
    """Surface-aligned SuGaR Gaussians bound to a mesh: 6 Gaussians per face at the
    barycentres of geometry/sugar.py:275-286, in-plane scale = shortest edge / (4 + 2 sqrt 3) (:276,
    :319-323), normal-axis scale = the surface thickness (spatial extent / 1e6, :201), rotation columns
    (face normal, first edge, normal x edge) (:505-528), opacity U(0.6, 0.99), per-Gaussian face normals
    (get_gs_normals, :547-556).  subdiv 7 -> 327,680 faces -> 1,966,080 Gaussians (C5: ~2M)."""
    rng = np.random.default_rng(seed)
    v, f = icosphere(subdiv)
    fv = v[f]  # (F, 3, 3)
    bary = np.array([[2 / 3, 1 / 6, 1 / 6], [1 / 6, 2 / 3, 1 / 6], [1 / 6, 1 / 6, 2 / 3], [1 / 6, 5 / 12, 5 / 12],
                     [5 / 12, 1 / 6, 5 / 12], [5 / 12, 5 / 12, 1 / 6]])
    xyz = np.einsum("gk,fkc->fgc", bary, fv).reshape(-1, 3)
    edges = np.linalg.norm(fv - fv[:, [1, 2, 0]], axis=-1).min(-1) / (4.0 + 2.0 * np.sqrt(3.0))
    s = np.repeat(np.maximum(edges, 1e-7), 6)
    n = np.cross(fv[:, 1] - fv[:, 0], fv[:, 2] - fv[:, 0])
    n /= np.linalg.norm(n, axis=1, keepdims=True)
    e1 = fv[:, 0] - fv[:, 1]
    e1 /= np.linalg.norm(e1, axis=1, keepdims=True)
    e2 = np.cross(n, e1)
    e2 /= np.linalg.norm(e2, axis=1, keepdims=True)
    R = np.stack([n, e1, e2], axis=-1)  # columns
    q = np.repeat(_matrix_to_quaternion(R), 6, axis=0)
    P = xyz.shape[0]
    M = (sh_degree + 1) ** 2
    sh = np.zeros((P, M, 3), np.float32)
    sh[:, 0, :] = (rng.random((P, 3)) - 0.5) / C0
    if M > 1:
        sh[:, 1:, :] = rng.normal(0.0, 0.05, size=(P, M - 1, 3))
    return dict(means3D=xyz.astype(np.float32),
                scales=np.stack([np.full(P, thickness), s, s], 1).astype(np.float32),
                rotations=q.astype(np.float32),
                opacities=rng.uniform(0.6, 0.99, size=(P, 1)).astype(np.float32),
                shs=sh, sh_degree=sh_degree,
                normals=np.repeat(n, 6, axis=0).astype(np.float32))

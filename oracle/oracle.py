"""ctypes front-end of the CPU restatement (oracle/gsr_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
as the parity checker / CPU baseline.  Never used by the product path.  See gsr_oracle.c for what it
restates and how it is pinned (parity of the full rasterizer is unpinned by the reference; the SH,
covariance and projection pieces are pinned by tests/golden vectors lifted from the reference).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "build", "libgsr_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
    return _lib


def _p(a):
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.c_void_p)


def _f32(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float32)


def _dtype(prec):
    return np.float32 if prec in ("f32", "f32c") else np.float64


def _args(scene, cam, bg):
    view, proj, campos, tanx, tany, W, H = cam
    shs = _f32(scene.get("shs"))
    colors = _f32(scene.get("colors_precomp"))
    cov3 = _f32(scene.get("cov3D_precomp"))
    scales = None if cov3 is not None else _f32(scene["scales"])
    rots = None if cov3 is not None else _f32(scene["rotations"])
    if colors is not None:
        shs = None
    P = int(scene["means3D"].shape[0])
    M = int(shs.shape[1]) if shs is not None else 0
    keep = [_f32(scene["means3D"]), scales, rots, _f32(scene["opacities"]), shs, colors, cov3,
            _f32(view), _f32(proj), _f32(campos), _f32(bg)]
    return P, M, keep, (W, H, tanx, tany)


def forward(scene: dict, cam, bg, prec: str = "f32", mod: float = 1.0):
    """cam = (view(16), proj(16), campos(3), tanfovx, tanfovy, W, H).  Returns dict(color, depth, alpha, radii, K)."""
    P, M, k, (W, H, tanx, tany) = _args(scene, cam, bg)
    dt = _dtype(prec)
    color = np.zeros((3, H, W), dt)
    depth = np.zeros((1, H, W), dt)
    alpha = np.zeros((1, H, W), dt)
    radii = np.zeros((max(P, 1),), np.int32)
    fn = getattr(lib(), f"oracle_forward_{prec}")
    fn.restype = ctypes.c_long
    K = fn(ctypes.c_int(P), ctypes.c_int(int(scene.get("sh_degree", 0))), ctypes.c_int(M), _p(k[0]), _p(k[1]),
           ctypes.c_float(mod), _p(k[2]), _p(k[3]), _p(k[4]), _p(k[5]), _p(k[6]), _p(k[7]), _p(k[8]), _p(k[9]),
           ctypes.c_int(W), ctypes.c_int(H), ctypes.c_float(tanx), ctypes.c_float(tany), _p(k[10]),
           _p(color), _p(depth), _p(alpha), _p(radii))
    return dict(color=color, depth=depth, alpha=alpha, radii=radii[:P], K=int(K))


def backward(scene: dict, cam, bg, dL_dcolor, dL_ddepth=None, dL_dalpha=None, prec: str = "f32", mod: float = 1.0,
             order: int = 0):
    """order 1: the per-Gaussian sums add their per-pixel terms in the reverse pixel order (another run of the
    reference's atomic accumulation, whose order is unspecified); 0 = raster order."""
    P, M, k, (W, H, tanx, tany) = _args(scene, cam, bg)
    lib().oracle_set_order(ctypes.c_int(order))
    dt = _dtype(prec)
    n = max(P, 1)
    out = dict(means2D=np.zeros((n, 3), dt), colors=np.zeros((n, 3), dt), opacity=np.zeros((n, 1), dt),
               means3D=np.zeros((n, 3), dt), cov3D=np.zeros((n, 6), dt), sh=np.zeros((n, max(M, 1), 3), dt),
               scales=np.zeros((n, 3), dt), rotations=np.zeros((n, 4), dt))
    gc, gd, ga = _f32(dL_dcolor), _f32(dL_ddepth), _f32(dL_dalpha)
    fn = getattr(lib(), f"oracle_backward_{prec}")
    fn.restype = None
    fn(ctypes.c_int(P), ctypes.c_int(int(scene.get("sh_degree", 0))), ctypes.c_int(M), _p(k[0]), _p(k[1]),
       ctypes.c_float(mod), _p(k[2]), _p(k[3]), _p(k[4]), _p(k[5]), _p(k[6]), _p(k[7]), _p(k[8]), _p(k[9]),
       ctypes.c_int(W), ctypes.c_int(H), ctypes.c_float(tanx), ctypes.c_float(tany), _p(k[10]),
       _p(gc), _p(gd), _p(ga), _p(out["means2D"]), _p(out["colors"]), _p(out["opacity"]), _p(out["means3D"]),
       _p(out["cov3D"]), _p(out["sh"]) if M > 0 else None, _p(out["scales"]), _p(out["rotations"]))
    lib().oracle_set_order(ctypes.c_int(0))
    res = {key: v[:P] for key, v in out.items()}
    if M == 0:
        res["sh"] = np.zeros((P, 0, 3), dt)
    return res


def set_variant(v: int):
    """DIAGNOSTIC ONLY (gsr_oracle.c g_oracle_variant): evaluate pieces of the per-pixel arithmetic the way the
    HIP blends do.  Never used by a parity test."""
    lib().oracle_set_variant(ctypes.c_int(v))


def gauss_aux(scene: dict, cam, prec: str = "f64", mod: float = 1.0):
    """Per-Gaussian preprocess values (oracle_gauss_aux): dict(px, py, rad3 = 3 sqrt(max eigenvalue) before
    the ceil (-1 when culled before it), tiles = rectangle tiles of the oracle's radius, conic (P, 3),
    opacity, depth, rgb (P, 3), rect (P, 4) = tile xmin, ymin, xmax, ymax)."""
    P, M, k, (W, H, tanx, tany) = _args(scene, cam, np.zeros(3, np.float32))
    aux = np.zeros((max(P, 1), 16), np.float64)
    fn = getattr(lib(), f"oracle_gauss_aux_{prec}")
    fn.restype = None
    fn(ctypes.c_int(P), ctypes.c_int(int(scene.get("sh_degree", 0))), ctypes.c_int(M), _p(k[0]), _p(k[1]),
       ctypes.c_float(mod), _p(k[2]), _p(k[3]), _p(k[4]), _p(k[5]), _p(k[6]), _p(k[7]), _p(k[8]), _p(k[9]),
       ctypes.c_int(W), ctypes.c_int(H), ctypes.c_float(tanx), ctypes.c_float(tany), _p(aux))
    aux = aux[:P]
    return dict(px=aux[:, 0], py=aux[:, 1], rad3=aux[:, 2], tiles=aux[:, 3].astype(np.int64), conic=aux[:, 4:7],
                opacity=aux[:, 7], depth=aux[:, 8], rgb=aux[:, 9:12], rect=aux[:, 12:16].astype(np.int64))


def eval_sh(deg: int, sh: np.ndarray, pos: np.ndarray, campos: np.ndarray, prec: str = "f64") -> np.ndarray:
    """eval_sh of the reference (without +0.5/clamp) at normalize(pos - campos).  sh (n, M, 3)."""
    sh = np.ascontiguousarray(sh, np.float64)
    pos = np.ascontiguousarray(pos, np.float64)
    campos = np.ascontiguousarray(campos, np.float64)
    n, M = sh.shape[0], sh.shape[1]
    out = np.zeros((n, 3), np.float64)
    getattr(lib(), f"oracle_eval_sh_{prec}")(ctypes.c_int(n), ctypes.c_int(deg), ctypes.c_int(M), _p(sh), _p(pos),
                                             _p(campos), _p(out))
    return out


def cov3d(scales: np.ndarray, rots: np.ndarray, mod: float = 1.0, prec: str = "f64") -> np.ndarray:
    scales = np.ascontiguousarray(scales, np.float64)
    rots = np.ascontiguousarray(rots, np.float64)
    n = scales.shape[0]
    out = np.zeros((n, 6), np.float64)
    getattr(lib(), f"oracle_cov3d_{prec}")(ctypes.c_int(n), _p(scales), ctypes.c_double(mod), _p(rots), _p(out))
    return out


def knn_mean_dist(points: np.ndarray, prec: str = "f32", queries=None) -> np.ndarray:
    """simple_knn.distCUDA2 restated (oracle/gsr_oracle.c oracle_knn_mean_dist_*): mean squared distance to
    the 3 nearest other points, brute force; ``queries`` (indices) limits the points evaluated."""
    pts = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 3)
    q = None if queries is None else np.ascontiguousarray(queries, dtype=np.int32)
    nq = pts.shape[0] if q is None else q.shape[0]
    out = np.zeros(nq, np.float64)
    fn = getattr(lib(), f"oracle_knn_mean_dist_{prec}")
    fn(ctypes.c_int(pts.shape[0]), _p(pts), ctypes.c_int(nq), None if q is None else _p(q), _p(out))
    return out.astype(np.float32) if prec == "f32" else out

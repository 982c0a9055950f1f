"""Diagnostic: how many of a view's tile instances (3-sigma rectangle x tiles, the reference's
binning) can reach a pixel with alpha >= 1/255 (exact ellipse-vs-tile-box test, the blend's
quadrant test at tile size).  Reads the per-Gaussian records back from the geometry workspace
(csrc/gsr_common.h GaussRec: a = (px, py, conic a, b), b = (conic c, opacity, depth, .),
d = (xmin | ymin << 16, xmax | ymax << 16, ...)).  Usage (GPU box): python profiles/diag_cull.py"""
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "threestudio-3dgs_amd"))
import gsr_synthetic as gs  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402
from diff_gaussian_rasterization.cameras import get_cam_info_gaussian, orbit_c2w  # noqa: E402


def box_min(a, b, c, u0, u1, v0, v1):
    def qf(u, v):
        return a * u * u + 2 * b * u * v + c * v * v
    q0 = qf(u0, np.clip(-b * u0 / c, v0, v1))
    q1 = qf(u1, np.clip(-b * u1 / c, v0, v1))
    q2 = qf(np.clip(-b * v0 / a, u0, u1), v0)
    q3 = qf(np.clip(-b * v1 / a, u0, u1), v1)
    inside = (u0 <= 0) & (u1 >= 0) & (v0 <= 0) & (v1 >= 0)
    return np.where(inside, 0.0, np.minimum(np.minimum(q0, q1), np.minimum(q2, q3)))


res, n = 1024, 1_000_000
sc = gs.make_scene(n, sh_degree=3, seed=0)
dev = "cuda"
t = {k: torch.tensor(sc[k], device=dev) for k in ("means3D", "scales", "rotations", "opacities", "shs")}
fov = math.radians(60)
wv, fp, cc = get_cam_info_gaussian(orbit_c2w(2.5, 0.0, 0.0), fov, fov)
out = _C.rasterize_gaussians(torch.zeros(3, device=dev), t["means3D"], None, t["opacities"], t["scales"],
                             t["rotations"], 1.0, None, wv.to(dev), fp.to(dev), math.tan(fov / 2), math.tan(fov / 2),
                             res, res, t["shs"], 3, cc.to(dev), False, False)
K, geom = out[0], out[5]
rec = geom[: n * 64].view(torch.float32).view(n, 16).cpu().numpy()
rect = rec[:, 12:14].view(np.uint32)
xmin, ymin = (rect[:, 0] & 0xFFFF).astype(np.int64), (rect[:, 0] >> 16).astype(np.int64)
xmax, ymax = (rect[:, 1] & 0xFFFF).astype(np.int64), (rect[:, 1] >> 16).astype(np.int64)
cnt = np.maximum(xmax - xmin, 0) * np.maximum(ymax - ymin, 0)
print("K (kernel)", K, "K (rect sum)", int(cnt.sum()))
g = np.repeat(np.arange(n), cnt)
start = np.repeat(np.cumsum(cnt) - cnt, cnt)
k = np.arange(cnt.sum()) - start
w = (xmax - xmin)[g]
tx = xmin[g] + k % w
ty = ymin[g] + k // w
px, py, a, b, c, o = (rec[g, i].astype(np.float64) for i in (0, 1, 2, 3, 4, 5))
tau = np.log(np.maximum(255.0 * o, 1.0))
u1 = px - tx * 16.0
u0 = u1 - 15.0
v1 = py - ty * 16.0
v0 = v1 - 15.0
qmin = box_min(a, b, c, u0, u1, v0, v1)
keep = qmin <= 2 * tau
print("instances kept by the exact tile test: %d of %d (%.1f%%)" % (keep.sum(), len(keep), 100 * keep.mean()))
# 8x8 quadrant-level: average number of quadrants per kept instance
qs = 0
for dxq in (0, 8):
    for dyq in (0, 8):
        uu1 = px - (tx * 16.0 + dxq)
        vv1 = py - (ty * 16.0 + dyq)
        qs += (box_min(a, b, c, uu1 - 7.0, uu1, vv1 - 7.0, vv1) <= 2 * tau)
print("quadrant hits per rect instance %.3f, per kept instance %.3f" % (qs.mean(), qs[keep].mean()))

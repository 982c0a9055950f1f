"""Diagnostic: distribution of per-tile instance counts and per-quadrant blend depth (quad_maxc) for the
benchmark view, read back from the image workspace (layout: csrc/gsr_common.h ImageState)."""
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

res = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
sc = gs.make_scene(n, sh_degree=3, seed=0)
dev = "cuda"
t = {k: torch.tensor(sc[k], device=dev) for k in ("means3D", "scales", "rotations", "opacities", "shs")}
fov = math.radians(60)
wv, fp, cc = get_cam_info_gaussian(orbit_c2w(2.5, 0.0, 0.0), fov, fov)
out = _C.rasterize_gaussians(torch.zeros(3, device=dev), t["means3D"], None, t["opacities"], t["scales"],
                             t["rotations"], 1.0, None, wv.to(dev), fp.to(dev), math.tan(fov / 2), math.tan(fov / 2),
                             res, res, t["shs"], 3, cc.to(dev), False, False)
K, img = out[0], out[7]
tiles = ((res + 15) // 16) ** 2
al = lambda x: (x + 255) // 256 * 256
ranges = img[: tiles * 8].view(torch.int32).view(tiles, 2).cpu().numpy()
qoff = al(tiles * 8)
qmaxc = img[qoff: qoff + 16 * tiles].view(torch.int32).cpu().numpy()
cnt = ranges[:, 1] - ranges[:, 0]
print("K", K, "tiles", tiles, "non-empty", (cnt > 0).sum())
print("instances/tile  pct 50/90/99/max:", np.percentile(cnt[cnt > 0], [50, 90, 99]).astype(int), cnt.max())
q = qmaxc[qmaxc > 0]
print("quad_maxc (nonzero)", len(q), "pct 50/90/99/max:", np.percentile(q, [50, 90, 99]).astype(int), q.max(),
      "sum", q.sum())
tm = qmaxc.reshape(tiles, 4).max(1)
print("tile maxc sum", tm.sum(), "fraction of K", tm.sum() / K)

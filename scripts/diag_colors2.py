import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("threestudio-3dgs_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np, torch
from gsr_testutil import gs, make_camera
from test_gpu_configs import _settings
from diff_gaussian_rasterization.batched import rasterize_views
scene = gs.make_scene(15_000, sh_degree=1, seed=44)
rng = np.random.default_rng(4)
n = rng.normal(size=(15_000, 3)).astype(np.float32)
normals = torch.tensor(n / np.linalg.norm(n, axis=1, keepdims=True), device="cuda")
cams = [make_camera(144, 112, elevation=10.0 * i, azimuth=70.0 * i) for i in range(3)]
t = {k: torch.tensor(scene[k], device="cuda") for k in ("means3D", "scales", "rotations", "opacities", "shs")}
st = [_settings(c, [0.2, 0.4, 0.6], 1) for c in cams]
m2 = [torch.zeros((15_000, 3), device="cuda") for _ in cams]
common = dict(opacities=t["opacities"], scales=t["scales"], rotations=t["rotations"])
outs = []
for fused in (True, False, True, False):
    if fused:
        c, r, d, a, c2 = rasterize_views(st, t["means3D"], m2, shs=t["shs"], colors2=normals, **common)
    else:
        c, r, d, a = rasterize_views(st, t["means3D"], m2, shs=t["shs"], **common)
        c2, _, _, _ = rasterize_views(st, t["means3D"], m2, colors_precomp=normals, **common)
    outs.append([x.clone() for x in (c, d, a, c2)])
for i, name in enumerate(("c", "d", "a", "c2")):
    f1, s1, f2, s2 = (o[i] for o in outs)
    dd = (f1 - s1).abs()
    print(name, "fused==sep", torch.equal(f1, s1), "max", float(dd.max()), "n", int((dd > 0).sum()),
          "fused repeat", torch.equal(f1, f2), "sep repeat", torch.equal(s1, s2))
    if dd.max() > 0:
        idx = torch.nonzero(dd > 0)[:5].tolist()
        print("  at", idx, [float(f1[tuple(j)]) for j in idx], [float(s1[tuple(j)]) for j in idx])

"""Diagnostic: where the HIP forward and the fp32 oracle disagree (per-Gaussian preprocess state and
pixel misses beyond the fp64 bar).  Usage: python scripts/diag_parity.py N RES [bg]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("threestudio-3dgs_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np
import torch

import oracle
from gsr_testutil import gs, make_camera, oracle_cam, run_oracle, _pixels
from diff_gaussian_rasterization import _C

N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
R = int(sys.argv[2]) if len(sys.argv) > 2 else 512
bgv = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
scene = gs.make_scene(N, sh_degree=3, seed=0)
cam = make_camera(R, R)
dev = "cuda"
t = {k: torch.tensor(scene[k], device=dev) for k in ("means3D", "scales", "rotations", "opacities", "shs")}
bg = torch.full((3,), bgv, device=dev)
K, color, depth, alpha, radii, geom, binning, image = _C.rasterize_gaussians(
    bg, t["means3D"], None, t["opacities"], t["scales"], t["rotations"], 1.0, None, torch.tensor(cam["view"], device=dev),
    torch.tensor(cam["proj"], device=dev), cam["tanx"], cam["tany"], R, R, t["shs"], 3,
    torch.tensor(cam["campos"], device=dev), False, False)
rec, tiles = _C.gauss_state(geom, 1, N)
rec = rec[0].cpu().numpy()
tiles = tiles[0].cpu().numpy()
ref = run_oracle(scene, cam, [bgv] * 3)
a32 = ref["aux32"]
vis = a32["tiles"] > 0
print("K gpu", K, "oracle", ref["f32"]["K"], "visible", vis.sum(), "gpu visible", (tiles[:, 0] > 0).sum())
print("tiles mismatch", int((tiles[:, 0] != a32["tiles"]).sum()))
for name, g_, o_ in (("px", rec[vis, 0], a32["px"][vis]), ("py", rec[vis, 1], a32["py"][vis]),
                     ("ca", rec[vis, 2], a32["conic"][vis, 0]), ("cb", rec[vis, 3], a32["conic"][vis, 1]),
                     ("cc", rec[vis, 4], a32["conic"][vis, 2]), ("op", rec[vis, 5], a32["opacity"][vis]),
                     ("depth", rec[vis, 6], a32["depth"][vis]), ("r", rec[vis, 8], a32["rgb"][vis, 0])):
    d = np.abs(g_.astype(np.float64) - o_)
    rel = d / np.maximum(np.abs(o_), 1e-30)
    print(f"{name}: exact {np.mean(d == 0):.4f} max abs {d.max():.3g} max rel {rel.max():.3g}")
gpu = dict(color=color.cpu().numpy(), alpha=alpha.cpu().numpy(), depth=depth.cpu().numpy())
f32, f64 = ref["f32"], ref["f64"]
for k in ("color", "alpha", "depth"):
    g, o3, o6 = _pixels(gpu[k]).astype(np.float64), _pixels(f32[k]).astype(np.float64), _pixels(f64[k])
    bad_g = (np.abs(g - o6) > 1e-5 + (1e-5 * np.abs(o6) if k == "depth" else 0)).any(1)
    bad_3 = (np.abs(o3 - o6) > 1e-5 + (1e-5 * np.abs(o6) if k == "depth" else 0)).any(1)
    only = np.nonzero(bad_g & ~bad_3)[0]
    print(f"{k}: gpu miss {bad_g.sum()} f32 miss {bad_3.sum()} gpu-only {only.size}")
    if k == "color":
        for pid in only[:25]:
            y, x = divmod(int(pid), R)
            print(f"  px ({x},{y}) tile {(y // 16) * ((R + 15) // 16) + x // 16} gpu {g[pid]} f32 {o3[pid]} f64 {o6[pid]} "
                  f"alpha gpu {gpu['alpha'].reshape(-1)[pid]:.7f} f64 {f64['alpha'].reshape(-1)[pid]:.7f}")
        ys, xs = np.divmod(only, R)
        print("  gpu-only miss tiles:", np.unique((ys // 16) * ((R + 15) // 16) + xs // 16)[:40])
        print("  x mod 16 histogram", np.bincount(xs % 16, minlength=16), "y mod 16", np.bincount(ys % 16, minlength=16))
# the Gaussians whose colour differs most
d = np.abs(rec[:, 8:11].astype(np.float64) - a32["rgb"]).max(1)
d[~vis] = 0
a64 = oracle.gauss_aux(scene, oracle_cam(cam), "f64")
for i in np.argsort(-d)[:8]:
    m = scene["means3D"][i]
    dirv = m - cam["campos"]
    print(f"g {i}: |drgb| {d[i]:.3g} gpu {rec[i, 8:11]} f32 {a32['rgb'][i]} f64 {a64['rgb'][i]} block {i // 128} "
          f"lane {i % 128} mean {m} dir {dirv / np.linalg.norm(dirv)} clampflags {rec[i, 15].view(np.uint32)}")
print("count |drgb| > 1e-5:", int((d > 1e-5).sum()), " > 1e-6:", int((d > 1e-6).sum()))

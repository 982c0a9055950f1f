"""Delta-debug a colour mismatch between the HIP forward and the fp32 oracle: keep only the Gaussians
whose rectangle covers one tile, then drop chunks while the mismatch on that tile persists."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("threestudio-3dgs_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np

import oracle
from gsr_testutil import gpu_render, gs, make_camera, oracle_cam

N, R, TX, TY = 100_000, 512, 16, 11
scene = gs.make_scene(N, sh_degree=3, seed=0)
cam = make_camera(R, R)
bg = np.ones(3, np.float32)
aux = oracle.gauss_aux(scene, oracle_cam(cam), "f32")
rect = aux["rect"]
cover = np.nonzero((rect[:, 0] <= TX) & (TX < rect[:, 2]) & (rect[:, 1] <= TY) & (TY < rect[:, 3]) & (aux["tiles"] > 0))[0]
print("Gaussians covering tile", len(cover), flush=True)


def sub(idx):
    return {k: (v[idx] if isinstance(v, np.ndarray) and v.shape[0] == N else v) for k, v in scene.items()}


def err(idx):
    s = sub(idx)
    g = gpu_render(s, cam, bg)
    o = oracle.forward(s, oracle_cam(cam), bg, "f32")
    y0, x0 = TY * 16, TX * 16
    d = np.abs(g["color"][:, y0:y0 + 16, x0:x0 + 16] - o["color"][:, y0:y0 + 16, x0:x0 + 16])
    da = np.abs(g["alpha"][:, y0:y0 + 16, x0:x0 + 16] - o["alpha"][:, y0:y0 + 16, x0:x0 + 16])
    return float(d.max()), float(da.max())


full = err(np.arange(N))
e0 = err(cover)
print("full scene tile err", full, "subset err", e0, flush=True)
idx = cover
thr = 0.5 * e0[0]
if e0[0] > 2e-5:
    chunk = len(idx) // 2
    while chunk >= 1:
        i = 0
        changed = False
        while i < len(idx):
            trial = np.concatenate([idx[:i], idx[i + chunk:]])
            if len(trial) and err(trial)[0] > thr:
                idx = trial
                changed = True
            else:
                i += chunk
        print("chunk", chunk, "->", len(idx), "Gaussians, err", err(idx), flush=True)
        if not changed:
            chunk //= 2
    print("minimal set:", idx.tolist())
    s = sub(idx)
    a = oracle.gauss_aux(s, oracle_cam(cam), "f32")
    order = np.argsort(a["depth"], kind="stable")
    for j in order:
        print(f"  g {idx[j]} depth {a['depth'][j]:.7f} px {a['px'][j]:.3f} py {a['py'][j]:.3f} conic {a['conic'][j]} "
              f"op {a['opacity'][j]:.4f} rgb {a['rgb'][j]} rect {a['rect'][j]} rad3 {a['rad3'][j]:.3f}")
    g = gpu_render(s, cam, bg)
    o = oracle.forward(s, oracle_cam(cam), bg, "f32")
    y0, x0 = TY * 16, TX * 16
    d = np.abs(g["color"] - o["color"]).max(0)
    ys, xs = np.nonzero(d > 1e-5)
    print("bad pixels:", list(zip(xs.tolist(), ys.tolist()))[:40])
    np.savez("gpurun_out/r02_min_scene.npz", idx=idx, **{k: v for k, v in s.items() if isinstance(v, np.ndarray)})

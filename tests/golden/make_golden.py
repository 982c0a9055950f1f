"""Generate the golden vectors under tests/golden/ (run in the build container, where /root/reference exists).

Two kinds of fixtures:

1. reference_*.npz — outputs of the reference's OWN pure-torch functions, lifted from the source text
   with `ast` and executed on CPU (the reference package as a whole is not importable: it needs
   threestudio/plyfile/simple_knn, absent here; these functions need only torch/numpy/math):
     eval_sh, C0..C3                 geometry/sugar.py:743-830
     build_rotation, build_scaling_rotation, strip_lowerdiag/strip_symmetric
                                     geometry/gaussian_base.py:47-134   (device="cuda" rewritten to "cpu")
     getProjectionMatrix, getWorld2View2
                                     utils/sugar_utils.py:796-829
     camera construction             geometry/sugar.py:891-896 (world_view, full_proj, camera_center)
   They pin the CPU restatement's SH, covariance and projection pieces (tests/test_golden.py).
   Only inputs and outputs are written; no reference source is stored.

2. oracle_scene.npz — a small seeded scene + camera with the CPU restatement's fp64 forward outputs and
   gradients (oracle/gsr_oracle.c).  Regression fixture for the oracle and a committed target for the
   GPU parity tests.  (The reference has no rasterizer, so no reference-generated fixture exists for
   the full path: parity of the full rasterizer is unpinned by the reference)

Usage:  python tests/golden/make_golden.py [--reference /root/reference]
"""
from __future__ import annotations

import argparse
import ast
import math
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def lift(path: str, names: list[str], extra_globals: dict) -> dict:
    """Execute the top-level definitions `names` from a reference source file; return its namespace."""
    src = open(path).read()
    tree = ast.parse(src)
    keep = []
    for node in tree.body:
        if isinstance(node, (ast.FunctionDef, ast.ClassDef)) and node.name in names:
            keep.append(node)
        elif isinstance(node, ast.Assign) and any(isinstance(t, ast.Name) and t.id in names for t in node.targets):
            keep.append(node)
    code = ast.unparse(ast.Module(body=keep, type_ignores=[]))
    code = code.replace('device="cuda"', 'device="cpu"').replace("device='cuda'", "device='cpu'")
    ns = dict(extra_globals)
    exec(compile(code, path, "exec"), ns)  # noqa: S102 — reference pure functions, CPU only
    missing = [n for n in names if n not in ns]
    if missing:
        raise RuntimeError(f"could not lift {missing} from {path}")
    return ns


def make_reference(ref: str):
    g = {"torch": torch, "np": np, "math": math}
    sugar = lift(os.path.join(ref, "geometry/sugar.py"), ["C0", "C1", "C2", "C3", "C4", "eval_sh"], g)
    base = lift(os.path.join(ref, "geometry/gaussian_base.py"),
                ["C0", "RGB2SH", "SH2RGB", "strip_lowerdiag", "strip_symmetric", "build_rotation",
                 "build_scaling_rotation"], g)
    utils = lift(os.path.join(ref, "utils/sugar_utils.py"), ["getWorld2View2", "getProjectionMatrix", "fov2focal"], g)

    rng = np.random.default_rng(2024)
    # --- SH: eval_sh(deg, sh[..., C, coeff], dirs) at dirs = normalize(pos - campos)
    n = 64
    sh = rng.normal(0, 0.5, size=(n, 16, 3))
    pos = rng.normal(0, 1, size=(n, 3))
    campos = np.array([2.5, -0.3, 0.7])
    d = pos - campos
    d = d / np.linalg.norm(d, axis=1, keepdims=True)
    out = {"sh": sh, "pos": pos, "campos": campos}
    for deg in range(4):
        res = sugar["eval_sh"](deg, torch.tensor(sh).transpose(1, 2), torch.tensor(d))
        out[f"eval_sh_deg{deg}"] = res.numpy()
    rgb = rng.random((n, 3))
    out["rgb"] = rgb
    out["rgb2sh"] = base["RGB2SH"](torch.tensor(rgb)).numpy()
    np.savez_compressed(os.path.join(HERE, "reference_sh.npz"), **out)

    # --- covariance: L = R(q) S, Sigma = L L^T, upper triangle (strip_symmetric)
    scales = np.exp(rng.normal(-3, 1, size=(n, 3)))
    q = rng.normal(size=(n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    L = base["build_scaling_rotation"](torch.tensor(scales, dtype=torch.float32), torch.tensor(q, dtype=torch.float32))
    cov = base["strip_symmetric"](L @ L.transpose(1, 2))
    R = base["build_rotation"](torch.tensor(q, dtype=torch.float32))
    np.savez_compressed(os.path.join(HERE, "reference_cov.npz"), scales=scales, rotations=q,
                        cov3D=cov.double().numpy(), R=R.double().numpy())

    # --- projection + camera construction (geometry/sugar.py:891-896)
    cams = []
    for i in range(8):
        fovx = math.radians(rng.uniform(30, 90))
        fovy = math.radians(rng.uniform(30, 90))
        znear, zfar = 0.01 if i % 2 else 0.1, 100.0
        A = rng.normal(size=(3, 3))
        Qm, _ = np.linalg.qr(A)
        if np.linalg.det(Qm) < 0:
            Qm[:, 0] *= -1
        Rm, T = Qm, rng.normal(0, 2, size=3)
        P = utils["getProjectionMatrix"](znear=znear, zfar=zfar, fovX=fovx, fovY=fovy)
        wv = torch.tensor(utils["getWorld2View2"](Rm, T)).transpose(0, 1)
        full = (wv.unsqueeze(0).bmm(P.transpose(0, 1).unsqueeze(0))).squeeze(0)
        center = wv.inverse()[3, :3]
        # the same camera as an OpenGL camera-to-world (threestudio convention fed to get_cam_info_gaussian)
        c2w = np.linalg.inv(utils["getWorld2View2"](Rm, T).astype(np.float64))
        c2w[:3, 1:3] *= -1
        cams.append(dict(fovx=fovx, fovy=fovy, znear=znear, zfar=zfar, P=P.double().numpy(),
                         world_view=wv.double().numpy(), full_proj=full.double().numpy(),
                         center=center.double().numpy(), c2w_gl=c2w))
    np.savez_compressed(os.path.join(HERE, "reference_camera.npz"),
                        **{f"{k}_{i}": np.asarray(v) for i, c in enumerate(cams) for k, v in c.items()})


def make_oracle_scene():
    sys.path.insert(0, os.path.join(ROOT, "threestudio-3dgs_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle
    from gsr_testutil import make_camera, oracle_cam

    import gsr_synthetic as gs

    scene = gs.make_scene(600, sh_degree=3, seed=42)
    cam = make_camera(48, 40, fovy_deg=55.0, elevation=20.0, azimuth=35.0, distance=2.2)
    bg = np.array([0.3, 0.6, 0.9], np.float32)
    gc, gd, ga = gs.upstream_grads(40, 48, seed=5)
    f = oracle.forward(scene, oracle_cam(cam), bg, "f64")
    b = oracle.backward(scene, oracle_cam(cam), bg, gc, gd, ga, prec="f64")
    out = {f"scene_{k}": v for k, v in scene.items() if isinstance(v, np.ndarray)}
    out.update({f"cam_{k}": np.asarray(v) for k, v in cam.items()})
    out.update(bg=bg, dL_dcolor=gc, dL_ddepth=gd, dL_dalpha=ga, sh_degree=np.int64(scene["sh_degree"]))
    out.update({f"out_{k}": np.asarray(v) for k, v in f.items()})
    out.update({f"grad_{k}": v for k, v in b.items()})
    np.savez_compressed(os.path.join(HERE, "oracle_scene.npz"), **out)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--skip-reference", action="store_true")
    a = ap.parse_args()
    if not a.skip_reference:
        make_reference(a.reference)
    make_oracle_scene()
    print("golden vectors written to", HERE)

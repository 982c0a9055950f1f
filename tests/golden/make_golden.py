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
     Depth2Normal                    renderer/diff_gaussian_rasterizer_shading.py:22-51
     GaussianDiffuseWithPointLightMaterial.forward
                                     material/gaussian_material.py:41-104 (method body; threestudio's dot
                                     supplied), composed as the shading renderer does (:169-208)
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


def lift_method(path: str, cls: str, method: str, extra_globals: dict):
    """One method of a reference class as a plain function (annotations stripped: the class itself needs
    threestudio; the method body needs only torch)."""
    tree = ast.parse(open(path).read())
    node = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == cls)
    fn = next(n for n in node.body if isinstance(n, ast.FunctionDef) and n.name == method)
    fn.decorator_list = []
    fn.returns = None
    for a in fn.args.args + fn.args.kwonlyargs:
        a.annotation = None
    code = ast.unparse(ast.Module(body=[fn], type_ignores=[]))
    ns = dict(extra_globals)
    exec(compile(code, path, "exec"), ns)  # noqa: S102 — reference pure method body, CPU only
    return ns[method]


def make_shading_reference(ref: str):
    """The shading renderer's post-raster epilogue from the reference's own code: Depth2Normal
    (renderer/diff_gaussian_rasterizer_shading.py:22-51) and GaussianDiffuseWithPointLightMaterial.forward
    (material/gaussian_material.py:41-104), composed as the renderer does (:169-208); threestudio's
    dot(x, y) = sum(x * y, -1, keepdim=True) is supplied.  fp64, CPU; outputs and gradients for seeded
    upstream gradients."""
    from types import SimpleNamespace

    import random

    F = torch.nn.functional
    g = {"torch": torch, "F": F, "random": random, "dot": lambda x, y: torch.sum(x * y, -1, keepdim=True)}
    d2n = lift(os.path.join(ref, "renderer/diff_gaussian_rasterizer_shading.py"), ["Depth2Normal"], g)["Depth2Normal"]()
    # its stencil weights (0, +-1) as fp64 so the fixture is computed in fp64 (the values are exact)
    d2n.delzdelxkernel = d2n.delzdelxkernel.double()
    d2n.delzdelykernel = d2n.delzdelykernel.double()
    material_forward = lift_method(os.path.join(ref, "material/gaussian_material.py"),
                                   "GaussianDiffuseWithPointLightMaterial", "forward", g)
    rng = np.random.default_rng(77)
    out = {}
    H, W = 20, 28
    ys, xs = np.meshgrid(np.arange(H, dtype=np.float64), np.arange(W, dtype=np.float64), indexing="ij")
    depth = (2.0 + 0.3 * np.sin(xs / 5.0) * np.cos(ys / 4.0) + 0.01 * rng.random((H, W)))[None]
    f = 0.5 * H / math.tan(math.radians(30))
    rays_d = np.stack([(xs + 0.5 - W / 2) / f, -(ys + 0.5 - H / 2) / f, -np.ones_like(xs)], -1)
    Qm, _ = np.linalg.qr(rng.normal(size=(3, 3)))
    rays_d = rays_d @ Qm.T
    rays_o = np.broadcast_to(rng.normal(size=3), (H, W, 3)).copy()
    alpha = rng.random((1, H, W))
    alpha[:, : H // 2, : W // 2] = 1.0
    color = rng.random((3, H, W)) * alpha * 1.2 - 0.05
    bg = rng.random((H, W, 3))
    light = rng.normal(size=3) * 3
    ups = [rng.normal(size=(3, H, W)), rng.normal(size=(3, H, W)), rng.normal(size=(1, H, W))]
    out.update(color=color, depth=depth, alpha=alpha, rays_o=rays_o, rays_d=rays_d, bg=bg, light=light,
               up_render=ups[0], up_normal=ups[1], up_depth=ups[2])
    for shading in ("diffuse", "albedo", "textureless"):
        t = {k: torch.tensor(v, requires_grad=True) for k, v in (("color", color), ("depth", depth), ("alpha", alpha),
                                                                 ("bg", bg))}
        ro, rd = torch.tensor(rays_o), torch.tensor(rays_d)
        mat = SimpleNamespace(training=False, ambient_only=False,
                              cfg=SimpleNamespace(soft_shading=False, diffuse_prob=0.75, textureless_prob=0.5),
                              diffuse_light_color=torch.tensor([0.9, 0.8, 0.7], dtype=torch.float64),
                              ambient_light_color=torch.tensor([0.1, 0.2, 0.15], dtype=torch.float64))
        # renderer/diff_gaussian_rasterizer_shading.py:172-208 (pred_normal off, comp_rgb_bg = bg)
        rendered_depth = t["depth"].clone()
        xyz_map = ro + rendered_depth.permute(1, 2, 0) * rd
        normal_map = d2n(xyz_map.permute(2, 0, 1).unsqueeze(0))[0]
        normal_map = F.normalize(normal_map, dim=0)
        light_positions = torch.tensor(light)[None, None, :].expand(H, W, -1)
        shading_normal = normal_map.permute(1, 2, 0)
        rgb_fg = material_forward(mat, positions=xyz_map, shading_normal=shading_normal,
                                  albedo=(t["color"] / (t["alpha"] + 1e-6)).permute(1, 2, 0),
                                  light_positions=light_positions, shading=shading).permute(2, 0, 1)
        rendered_image = rgb_fg * t["alpha"] + (1 - t["alpha"]) * t["bg"].reshape(H, W, 3).permute(2, 0, 1)
        normal_map = normal_map * 0.5 * t["alpha"] + 0.5
        mask = t["alpha"] > 0.99
        normal_mask = mask.repeat(3, 1, 1)
        normal_map = torch.where(normal_mask, normal_map, normal_map.detach())
        rendered_depth = torch.where(mask, rendered_depth, rendered_depth.detach())
        render = rendered_image.clamp(0, 1)
        torch.autograd.backward([render, normal_map, rendered_depth],
                                [torch.tensor(ups[0]), torch.tensor(ups[1]), torch.tensor(ups[2])])
        out[f"{shading}_render"] = render.detach().numpy()
        out[f"{shading}_normal"] = normal_map.detach().numpy()
        out[f"{shading}_depth"] = rendered_depth.detach().numpy()
        for k, v in t.items():
            out[f"{shading}_grad_{k}"] = v.grad.numpy()
    out["ambient"] = np.array([0.1, 0.2, 0.15])
    out["diffuse"] = np.array([0.9, 0.8, 0.7])
    np.savez_compressed(os.path.join(HERE, "reference_shading.npz"), **out)


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
        make_shading_reference(a.reference)
    make_oracle_scene()
    print("golden vectors written to", HERE)

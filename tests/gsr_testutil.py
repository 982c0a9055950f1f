"""Shared helpers for the parity tests: run the HIP rasterizer through the public API and the CPU
oracle on identical float32 inputs, and compare with the tolerances stated in DESIGN.md §Parity."""
from __future__ import annotations

import math

import numpy as np

import gsr_synthetic as gs

# Parity bar (north_star): 1e-5 on RGB / alpha, 1e-4 on gradients (fp32).
RGB_ATOL = 1e-5
DEPTH_RTOL = 1e-5
GRAD_RTOL = 1e-4
# Discrete decisions (alpha >= 1/255, T (1 - alpha) >= 1e-4, ceil of the 3-sigma radius) can flip when
# two correct fp32 evaluations differ in the last ulp (exp implementations differ between the GPU and
# libm).  Such pixels / Gaussians are allowed up to this fraction; everything else must meet the bar.
FLIP_FRAC = 2e-4


def make_camera(W=256, H=256, fovy_deg=60.0, fovx_deg=None, elevation=15.0, azimuth=0.0, distance=2.5):
    import torch

    from diff_gaussian_rasterization.cameras import get_cam_info_gaussian, orbit_c2w

    fovy = math.radians(fovy_deg)
    fovx = math.radians(fovx_deg) if fovx_deg is not None else fovy
    c2w = orbit_c2w(distance, elevation, azimuth)
    wv, fp, cc = get_cam_info_gaussian(c2w, fovx, fovy, 0.1, 100.0)
    return dict(view=wv.numpy().astype(np.float32), proj=fp.numpy().astype(np.float32),
                campos=cc.numpy().astype(np.float32), tanx=math.tan(fovx / 2), tany=math.tan(fovy / 2), W=W, H=H)


def oracle_cam(cam):
    return (cam["view"].ravel(), cam["proj"].ravel(), cam["campos"], cam["tanx"], cam["tany"], cam["W"], cam["H"])


def to_torch(scene, device="cuda", requires_grad=True):
    import torch

    t = {}
    for k in ("means3D", "scales", "rotations", "opacities", "shs", "colors_precomp", "cov3D_precomp"):
        if scene.get(k) is not None:
            t[k] = torch.tensor(scene[k], device=device, requires_grad=requires_grad)
    return t


def gpu_render(scene, cam, bg, grads=None, mod=1.0, use=("shs",), cov3d=False, backward_twice=False):
    """Render through GaussianRasterizer; optionally backprop seeded upstream grads. Returns numpy dict."""
    import torch

    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer

    dev = "cuda"
    t = to_torch(scene, dev)
    P = scene["means3D"].shape[0]
    means2D = torch.zeros((P, 3), device=dev, requires_grad=True)
    settings = GaussianRasterizationSettings(
        image_height=cam["H"], image_width=cam["W"], tanfovx=cam["tanx"], tanfovy=cam["tany"],
        bg=torch.tensor(bg, device=dev, dtype=torch.float32), scale_modifier=mod,
        viewmatrix=torch.tensor(cam["view"], device=dev), projmatrix=torch.tensor(cam["proj"], device=dev),
        sh_degree=int(scene.get("sh_degree", 0)), campos=torch.tensor(cam["campos"], device=dev),
        prefiltered=False, debug=False)
    rast = GaussianRasterizer(raster_settings=settings)
    kw = dict(means3D=t["means3D"], means2D=means2D, opacities=t["opacities"])
    if "colors_precomp" in t:
        kw["colors_precomp"] = t["colors_precomp"]
    else:
        kw["shs"] = t["shs"]
    if cov3d:
        kw["cov3D_precomp"] = t["cov3D_precomp"]
    else:
        kw["scales"] = t["scales"]
        kw["rotations"] = t["rotations"]
    color, radii, depth, alpha = rast(**kw)
    out = dict(color=color.detach().cpu().numpy(), depth=depth.detach().cpu().numpy(),
               alpha=alpha.detach().cpu().numpy(), radii=radii.cpu().numpy())
    if grads is not None:
        gc, gd, ga = (torch.tensor(g, device=dev) for g in grads)
        loss = (color * gc).sum() + (depth * gd).sum() + (alpha * ga).sum()
        loss.backward(retain_graph=backward_twice)
        names = dict(means3D="means3D", scales="scales", rotations="rotations", opacities="opacity",
                     shs="sh", colors_precomp="colors", cov3D_precomp="cov3D")
        for k, v in t.items():
            if v.grad is not None:
                out["g_" + names[k]] = v.grad.detach().cpu().numpy().copy()
        out["g_means2D"] = means2D.grad.detach().cpu().numpy().copy()
        if backward_twice:
            for v in list(t.values()) + [means2D]:
                v.grad = None
            loss.backward()
            out["g2_means3D"] = t["means3D"].grad.detach().cpu().numpy().copy()
    return out


def flip_fraction(a, b, atol, rtol=0.0):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    bad = np.abs(a - b) > atol + rtol * np.abs(b)
    return float(bad.mean()) if bad.size else 0.0, bad


def assert_image_parity(gpu, ref, what=""):
    nflip_max = max(3, int(FLIP_FRAC * gpu["alpha"].size))
    _, bad_c = flip_fraction(gpu["color"], ref["color"], RGB_ATOL)
    _, bad_a = flip_fraction(gpu["alpha"], ref["alpha"], RGB_ATOL)
    _, bad_d = flip_fraction(gpu["depth"], ref["depth"], RGB_ATOL, DEPTH_RTOL)
    bad_px = bad_c.any(axis=0) | bad_a[0] | bad_d[0]
    assert bad_px.sum() <= nflip_max, (
        f"{what}: {bad_px.sum()} pixels outside tolerance (allowed {nflip_max}); "
        f"max |dC|={np.abs(gpu['color'] - ref['color']).max():.3g} |dA|={np.abs(gpu['alpha'] - ref['alpha']).max():.3g}")
    nr = max(3, int(FLIP_FRAC * max(1, gpu["radii"].size)))
    assert (gpu["radii"] != ref["radii"]).sum() <= nr, f"{what}: radii mismatch"
    return int(bad_px.sum())


def assert_grad_parity(gpu, ref, keys, what=""):
    """|g - g_ref| <= 1e-4 * max(1, max|g_ref|) per tensor, outside a FLIP_FRAC allowance of rows."""
    report = {}
    for k in keys:
        g, r = gpu["g_" + k], ref[k]
        g = g.reshape(r.shape)
        scale = max(1.0, float(np.abs(r).max()))
        bad = np.abs(g.astype(np.float64) - r) > GRAD_RTOL * scale
        rows = bad.reshape(bad.shape[0], -1).any(axis=1) if bad.ndim > 1 else bad
        nmax = max(3, int(FLIP_FRAC * 20 * rows.size))  # a pixel flip perturbs every Gaussian under it
        report[k] = (int(rows.sum()), float(np.abs(g - r).max()), scale)
        assert rows.sum() <= nmax, f"{what}: grad {k}: {rows.sum()} rows off (allowed {nmax}), {report[k]}"
    return report


def scene_subset(scene, **over):
    s = dict(scene)
    s.update(over)
    return s


__all__ = ["gs", "make_camera", "oracle_cam", "gpu_render", "assert_image_parity", "assert_grad_parity"]

"""The CPU restatement (oracle/gsr_oracle.c) checked three ways (no GPU needed):
  1. fp64 forward == a dense differentiable torch formulation of the same algorithm (tests/torch_reference.py);
  2. fp64 analytic backward == torch autograd of that formulation (the reference's gradient conventions are
     avoided in the scene: opacity <= 0.95 so the 0.99 clamp never binds, all means inside the 1.3 tan-fov
     guard; denom2inv's +1e-7 bounds the agreement to ~1e-5 relative);
  3. regression against the committed fixture tests/golden/oracle_scene.npz (see make_golden.py).
"""
import os

import numpy as np
import pytest
import torch

import oracle
import torch_reference as tr
from gsr_testutil import gs, make_camera, oracle_cam

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _torch_run(scene, cam, bg, grads, deg):
    dt = torch.float64
    t = {k: torch.tensor(scene[k], dtype=dt, requires_grad=True)
         for k in ("means3D", "scales", "rotations", "opacities", "shs")}
    m2d = torch.zeros(scene["means3D"].shape[0], 3, dtype=dt, requires_grad=True)
    view, proj, campos = tr.camera_tensors(cam)
    color, radii, depth, alpha = tr.render(t["means3D"], m2d, t["opacities"], view, proj, campos, cam["tanx"],
                                           cam["tany"], cam["W"], cam["H"], torch.tensor(bg, dtype=dt),
                                           sh=t["shs"], deg=deg, scales=t["scales"], rotations=t["rotations"])
    gc, gd, ga = (torch.tensor(g, dtype=dt) for g in grads)
    ((color * gc).sum() + (depth * gd).sum() + (alpha * ga).sum()).backward()
    out = dict(color=color.detach().numpy(), depth=depth.detach().numpy(), alpha=alpha.detach().numpy(),
               radii=radii.numpy())
    out.update({f"g_{k}": v.grad.numpy() for k, v in t.items()})
    out["g_means2D"] = m2d.grad.numpy()
    return out


@pytest.mark.parametrize("deg,W,H,bgv", [(0, 40, 32, 1.0), (3, 48, 40, 0.0), (1, 35, 29, 0.5)])
def test_oracle_matches_torch_autograd(deg, W, H, bgv):
    scene = gs.make_scene(150, sh_degree=deg, seed=10 + deg, radius=0.6)
    cam = make_camera(W, H, elevation=10.0 * deg, azimuth=25.0 * deg)
    bg = np.full(3, bgv, np.float32)
    grads = gs.upstream_grads(H, W, seed=deg)
    ref = _torch_run(scene, cam, bg, grads, deg)
    f = oracle.forward(scene, oracle_cam(cam), bg, "f64")
    np.testing.assert_array_equal(f["radii"], ref["radii"])
    for k in ("color", "depth", "alpha"):
        np.testing.assert_allclose(f[k], ref[k], rtol=1e-9, atol=1e-10, err_msg=k)
    b = oracle.backward(scene, oracle_cam(cam), bg, *grads, prec="f64")
    pairs = dict(means3D="means3D", scales="scales", rotations="rotations", opacities="opacity", shs="sh",
                 means2D="means2D")
    for tk, ok in pairs.items():
        g_ref, g_or = ref["g_" + tk], b[ok].reshape(ref["g_" + tk].shape)
        scale = max(1e-6, np.abs(g_ref).max())
        err = np.abs(g_or - g_ref).max() / scale
        assert err < 5e-5, f"{tk}: max rel err {err:.2e} (scale {scale:.3g})"


def test_oracle_fp32_vs_fp64():
    scene = gs.make_scene(3000, sh_degree=3, seed=4)
    cam = make_camera(128, 96, azimuth=70.0)
    bg = np.zeros(3, np.float32)
    a = oracle.forward(scene, oracle_cam(cam), bg, "f32")
    b = oracle.forward(scene, oracle_cam(cam), bg, "f64")
    bad = (np.abs(a["color"] - b["color"]) > 1e-5).any(0) | (np.abs(a["alpha"] - b["alpha"]) > 1e-5)[0]
    assert bad.sum() <= 3  # discrete fp32 decision flips only
    assert (a["radii"] != b["radii"]).sum() <= 3


def test_oracle_regression_fixture():
    z = np.load(os.path.join(GOLDEN, "oracle_scene.npz"))
    scene = {k[6:]: z[k] for k in z.files if k.startswith("scene_")}
    scene["sh_degree"] = int(z["sh_degree"])
    cam = {k[4:]: z[k] for k in z.files if k.startswith("cam_")}
    cam = dict(view=cam["view"], proj=cam["proj"], campos=cam["campos"], tanx=float(cam["tanx"]),
               tany=float(cam["tany"]), W=int(cam["W"]), H=int(cam["H"]))
    f = oracle.forward(scene, oracle_cam(cam), z["bg"], "f64")
    for k in ("color", "depth", "alpha", "radii"):
        np.testing.assert_allclose(f[k], z["out_" + k], rtol=1e-12, atol=1e-12, err_msg=k)
    b = oracle.backward(scene, oracle_cam(cam), z["bg"], z["dL_dcolor"], z["dL_ddepth"], z["dL_dalpha"], prec="f64")
    for k in ("means2D", "means3D", "opacity", "sh", "scales", "rotations", "cov3D", "colors"):
        np.testing.assert_allclose(b[k], z["grad_" + k], rtol=1e-10, atol=1e-10, err_msg=k)


def test_second_fp32_run_of_the_reference():
    """The null sample of the parity rule (tests/gsr_testutil.py): the fp32 restatement built with multiply-add
    contraction (as nvcc compiles the reference) and with the per-Gaussian sums in reverse pixel order is
    another faithful fp32 run: same radii, images within a few ulp, gradients within the bar of each other on
    a well-conditioned scene."""
    scene = gs.make_scene(2000, sh_degree=2, seed=21)
    cam = make_camera(72, 56)
    oc = oracle_cam(cam)
    bg = np.array([0.3, 0.2, 0.1], np.float32)
    grads = gs.upstream_grads(56, 72, seed=2)
    a, c = oracle.forward(scene, oc, bg, "f32"), oracle.forward(scene, oc, bg, "f32c")
    assert np.array_equal(a["radii"], c["radii"]) and a["K"] == c["K"]
    np.testing.assert_allclose(a["color"], c["color"], atol=2e-6)
    ga = oracle.backward(scene, oc, bg, *grads, prec="f32")
    gc = oracle.backward(scene, oc, bg, *grads, prec="f32c", order=1)
    for k in ("means3D", "means2D", "opacity", "scales", "rotations", "sh"):
        x, y = np.asarray(ga[k], np.float64), np.asarray(gc[k], np.float64)
        assert np.all(np.abs(x - y) <= 1e-4 * np.maximum(1.0, np.abs(x))), k
        assert not np.array_equal(x, y) or k == "sh", k  # a different evaluation, not the same bits

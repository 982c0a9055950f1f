"""HIP rasterizer vs the CPU restatement (oracle) on identical seeded inputs, through the public API.

Bars (north_star, tests/gsr_testutil.py): RGB / alpha 1e-5 abs, depth 1e-5 abs + rel, gradients
elementwise 1e-4 * max(1, |g|), all against the fp64 oracle; pixels / gradient rows beyond the bar are
adjudicated against the fp32 oracle's own misses (discrete fp32 decision flips).  Radii bit-exact except
fp64-verified ceil flips; num_rendered (K) exact up to those flips.
"""
import numpy as np
import pytest

from gsr_testutil import check_forward, check_grads, gpu_render, gs, make_camera, print_report, run_oracle

pytestmark = pytest.mark.gpu

GRAD_KEYS_SH = ["means3D", "means2D", "opacity", "sh", "scales", "rotations"]


@pytest.fixture(autouse=True)
def _parity_report():
    yield
    print_report()


def _run(scene, cam, bg, grads=True, mod=1.0, cov3d=False, keys=GRAD_KEYS_SH, what=""):
    g = gs.upstream_grads(cam["H"], cam["W"], seed=7) if grads else None
    gpu = gpu_render(scene, cam, bg, grads=g, mod=mod, cov3d=cov3d)
    ref = run_oracle(scene, cam, bg, grads=g, mod=mod)
    check_forward(gpu, ref, what, K_gpu=gpu["K"])
    if grads:
        check_grads(gpu, ref, keys, what)
    return gpu, ref


def test_c1_forward_backward_sh0():
    """C1: 10k Gaussians, 256^2, SH degree 0, white background."""
    scene = gs.make_scene(10_000, sh_degree=0, seed=0)
    cam = make_camera(256, 256)
    _run(scene, cam, [1.0, 1.0, 1.0], what="C1")


def test_c2_small_sh3_black_bg():
    """C2 shape at reduced N: SH degree 3, 512^2, zero background (background path)."""
    scene = gs.make_scene(30_000, sh_degree=3, seed=1)
    cam = make_camera(512, 512, elevation=30.0, azimuth=45.0)
    _run(scene, cam, [0.0, 0.0, 0.0], what="C2-small")


def test_ragged_image_and_aspect():
    """Image sizes not multiple of 16, fovx != fovy, coloured background."""
    scene = gs.make_scene(5_000, sh_degree=1, seed=2)
    cam = make_camera(200, 120, fovy_deg=50.0, fovx_deg=70.0, azimuth=100.0)
    _run(scene, cam, [0.2, 0.5, 0.9], what="ragged")


@pytest.mark.parametrize("deg", [1, 2])
def test_sh_degrees(deg):
    scene = gs.make_scene(4_000, sh_degree=deg, seed=3 + deg)
    cam = make_camera(128, 128, azimuth=30.0 * deg)
    _run(scene, cam, [1.0, 1.0, 1.0], what=f"deg{deg}")


def test_degree_larger_than_coefficients():
    """Pred-normal quirk: sh_degree > sqrt(M)-1 (renderer/diff_gaussian_rasterizer_shading.py:178-181)."""
    scene = gs.make_scene(3_000, sh_degree=0, seed=9)
    scene["sh_degree"] = 3
    cam = make_camera(128, 128)
    _run(scene, cam, [0.0, 0.0, 0.0], what="deg-quirk")


def test_colors_precomp_path():
    scene = gs.make_scene(6_000, sh_degree=0, seed=11)
    rng = np.random.default_rng(5)
    scene["colors_precomp"] = rng.random((6_000, 3)).astype(np.float32)
    scene.pop("shs")
    cam = make_camera(160, 160)
    _run(scene, cam, [1.0, 1.0, 1.0], keys=["means3D", "means2D", "opacity", "colors", "scales", "rotations"],
         what="colors_precomp")


def test_cov3d_precomp_path():
    scene = gs.make_scene(6_000, sh_degree=1, seed=12)
    import oracle

    scene["cov3D_precomp"] = oracle.cov3d(scene["scales"], scene["rotations"]).astype(np.float32)
    cam = make_camera(160, 160)
    _run(scene, cam, [1.0, 1.0, 1.0], cov3d=True, keys=["means3D", "means2D", "opacity", "sh", "cov3D"],
         what="cov3D_precomp")


def test_scale_modifier():
    scene = gs.make_scene(5_000, sh_degree=1, seed=13)
    cam = make_camera(128, 128)
    _run(scene, cam, [1.0, 1.0, 1.0], mod=0.7, what="scale_modifier")


def test_flat_surface_gaussians():
    """SuGaR-like: one axis 1e-6 thick (geometry/sugar.py:201,493-496) stresses the +0.3 dilation."""
    scene = gs.make_scene(6_000, sh_degree=0, seed=14)
    scene["scales"][:, 0] = 1e-6
    cam = make_camera(200, 200)
    _run(scene, cam, [0.0, 0.0, 0.0], what="flat")


@pytest.mark.parametrize("kind", ["needles_faint", "large_opaque"])
def test_tile_culling_edge_cases(kind):
    """The per-tile ellipse culling (csrc/gsr_common.h span_row) must never drop a tile with a
    contributing pixel: needle-like Gaussians with large off-diagonal conics and opacities just
    above / below 1/255, and large opaque Gaussians spanning many tiles, match the oracle (which
    bins every 3-sigma rectangle tile like the reference).  The needle scene is ill-conditioned
    (the fp32 oracle itself is ~4e-3 off its fp64 build on some scale gradients), so gradients are
    checked against the fp64 oracle with the fp32 oracle's own error as the yardstick: a dropped
    tile would remove whole pixel contributions, orders of magnitude above it."""
    if kind == "needles_faint":
        scene = gs.make_scene(3_000, sh_degree=0, seed=41, opacity_range=(0.9 / 255.0, 0.03))
        scene["scales"][:, 0] *= 6.0
        scene["scales"][:, 1] *= 0.15
    else:
        scene = gs.make_scene(400, sh_degree=0, seed=42, scale_mult=5.0, opacity_range=(0.5, 0.99))
    cam = make_camera(224, 176, azimuth=20.0)
    bg = np.array([0.3, 0.3, 0.3], np.float32)
    g = gs.upstream_grads(cam["H"], cam["W"], seed=7)
    gpu = gpu_render(scene, cam, bg, grads=g)
    ref = run_oracle(scene, cam, bg, grads=g)
    check_forward(gpu, ref, kind, K_gpu=gpu["K"])
    check_grads(gpu, ref, GRAD_KEYS_SH, kind)


def test_empty_and_culled():
    import torch

    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer

    cam = make_camera(64, 48)
    # P = 0: zero outputs, no launch (reference behaviour)
    scene = gs.make_scene(0, sh_degree=0, seed=0)
    out = gpu_render(scene, cam, [1.0, 1.0, 1.0])
    assert out["color"].shape == (3, 48, 64) and np.all(out["color"] == 0)
    # all behind the camera: background everywhere, radii 0, zero grads
    scene = gs.make_scene(500, sh_degree=0, seed=1)
    scene["means3D"] = scene["means3D"] * 0.1 + np.array([5.0, 0.0, 1.5], np.float32) * 2.0
    g = gs.upstream_grads(48, 64)
    out = gpu_render(scene, cam, [0.25, 0.5, 1.0], grads=g)
    ref = run_oracle(scene, cam, [0.25, 0.5, 1.0], grads=g)
    check_forward(out, ref, "culled", K_gpu=out["K"])
    assert np.all(out["radii"] == 0) and out["K"] == 0
    check_grads(out, ref, GRAD_KEYS_SH, "culled")
    del torch, GaussianRasterizationSettings, GaussianRasterizer


def test_single_gaussian_and_tile_edges():
    scene = gs.make_scene(1, sh_degree=0, seed=0)
    scene["means3D"][:] = 0.0
    scene["scales"][:] = 0.2
    cam = make_camera(100, 100)
    _run(scene, cam, [1.0, 1.0, 1.0], what="single")


def test_backward_is_repeatable():
    """retain_graph double backward (system/gaussian_splatting.py:129,138): bitwise-identical grads."""
    scene = gs.make_scene(8_000, sh_degree=2, seed=21)
    cam = make_camera(192, 192)
    g = gs.upstream_grads(192, 192, seed=3)
    out = gpu_render(scene, cam, [1.0, 1.0, 1.0], grads=g, backward_twice=True)
    assert np.array_equal(out["g_means3D"], out["g2_means3D"])


def test_forward_deterministic():
    scene = gs.make_scene(20_000, sh_degree=3, seed=22)
    cam = make_camera(256, 256)
    a = gpu_render(scene, cam, [0.0, 0.0, 0.0])
    b = gpu_render(scene, cam, [0.0, 0.0, 0.0])
    for k in ("color", "depth", "alpha", "radii"):
        assert np.array_equal(a[k], b[k]), k


def test_mark_visible():
    import torch

    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer

    scene = gs.make_scene(2_000, sh_degree=0, seed=3)
    scene["means3D"][:1000] += np.array([3.0, 0.0, 0.5], np.float32)  # some behind the camera
    cam = make_camera(64, 64)
    dev = "cuda"
    s = GaussianRasterizationSettings(64, 64, cam["tanx"], cam["tany"], torch.zeros(3, device=dev), 1.0,
                                      torch.tensor(cam["view"], device=dev), torch.tensor(cam["proj"], device=dev),
                                      0, torch.tensor(cam["campos"], device=dev), False, False)
    vis = GaussianRasterizer(s).markVisible(torch.tensor(scene["means3D"], device=dev)).cpu().numpy()
    v = cam["view"].reshape(-1)
    p = scene["means3D"]
    z = v[2] * p[:, 0] + v[6] * p[:, 1] + v[10] * p[:, 2] + v[14]
    assert np.array_equal(vis, z > 0.2)


def _settings(cam, bg, deg, dev="cuda", mod=1.0):
    import torch

    from diff_gaussian_rasterization import GaussianRasterizationSettings

    return GaussianRasterizationSettings(cam["H"], cam["W"], cam["tanx"], cam["tany"],
                                         torch.tensor(bg, device=dev, dtype=torch.float32), mod,
                                         torch.tensor(cam["view"], device=dev), torch.tensor(cam["proj"], device=dev),
                                         deg, torch.tensor(cam["campos"], device=dev), False, False)


@pytest.mark.parametrize("nviews", [1, 5, 19, 67])
def test_batched_views_match_per_view(nviews, monkeypatch):
    """rasterize_views (view sets: one launch per stage for up to 64 views; 67 = two sets) == per-view calls.
    Per-view calls and sets of <= 8 views split the backward (gsr_render.hip split_on), larger sets walk whole
    prefixes: the 19- and 67-view cases compare with the split disabled (tests/test_gpu_configs.py
    test_split_backward_* hold the split to the whole walk and the oracle)."""
    import torch

    if nviews > 8:
        monkeypatch.setenv("GSR_BWD_SPLIT", "0")

    from diff_gaussian_rasterization import GaussianRasterizer
    from diff_gaussian_rasterization.batched import rasterize_views

    scene = gs.make_scene(15_000, sh_degree=3, seed=31)
    cams = [make_camera(160, 128, elevation=10.0 * (i % 3), azimuth=360.0 * i / nviews) for i in range(nviews)]
    bg = [0.1, 0.2, 0.3]
    ups = [gs.upstream_grads(128, 160, seed=100 + i) for i in range(nviews)]
    dev = "cuda"
    keys = ("means3D", "scales", "rotations", "opacities", "shs")

    def leaves():
        return {k: torch.tensor(scene[k], device=dev, requires_grad=True) for k in keys}

    # per view
    t = leaves()
    per, m2_per = [], []
    for i, cam in enumerate(cams):
        m2 = torch.zeros((15_000, 3), device=dev, requires_grad=True)
        c, r, d, a = GaussianRasterizer(_settings(cam, bg, 3))(means3D=t["means3D"], means2D=m2, opacities=t["opacities"],
                                                               shs=t["shs"], scales=t["scales"], rotations=t["rotations"])
        gc, gd, ga = (torch.tensor(x, device=dev) for x in ups[i])
        ((c * gc).sum() + (d * gd).sum() + (a * ga).sum()).backward()
        per.append((c.detach(), r, d.detach(), a.detach()))
        m2_per.append(m2.grad.clone())
    g_per = {k: v.grad.clone() for k, v in t.items()}
    # batched
    t = leaves()
    m2s = [torch.zeros((15_000, 3), device=dev, requires_grad=True) for _ in cams]
    c, r, d, a = rasterize_views([_settings(cam, bg, 3) for cam in cams], t["means3D"], m2s, t["opacities"],
                                 shs=t["shs"], scales=t["scales"], rotations=t["rotations"])
    gc = torch.stack([torch.tensor(u[0], device=dev) for u in ups])
    gd = torch.stack([torch.tensor(u[1], device=dev) for u in ups])
    ga = torch.stack([torch.tensor(u[2], device=dev) for u in ups])
    ((c * gc).sum() + (d * gd).sum() + (a * ga).sum()).backward()
    for i in range(nviews):
        assert torch.equal(c[i], per[i][0]) and torch.equal(r[i], per[i][1])
        assert torch.equal(d[i], per[i][2]) and torch.equal(a[i], per[i][3])
        torch.testing.assert_close(m2s[i].grad, m2_per[i], rtol=0, atol=0)
    for k, v in t.items():
        ref = g_per[k]
        scale = max(1.0, float(ref.abs().max()))
        err = float((v.grad - ref).abs().max())
        assert err <= 1e-5 * scale, f"{k}: {err} vs scale {scale}"


def bitwise_case(kind, monkeypatch=None, fwd_kernel=None, between=None):
    """One 3-view rasterize_views forward + backward of the bitwise tests (every output, means2D and parameter
    gradient as numpy arrays).  ball_composite: 40k Gaussians, SH3, ragged 200 x 168 with the fused background
    composite; sugar_two_colors: a SuGaR scene with the second colour set (both calls in one backward)."""
    import torch

    from diff_gaussian_rasterization.batched import rasterize_views
    from test_gpu_configs import _settings

    if fwd_kernel is not None:
        monkeypatch.setenv("GSR_FWD_KERNEL", fwd_kernel)
        monkeypatch.setenv("GSR_BWD_SPLIT", "0")  # the tile-wave forward writes no split checkpoints
    dev = "cuda"
    if kind == "ball_composite":
        scene = gs.make_scene(40_000, sh_degree=3, seed=51)
        W_, H_ = 200, 168  # ragged: partial tiles and quadrants at the edges
    else:
        scene = gs.make_sugar_scene(5, sh_degree=0, seed=3)
        W_, H_ = 256, 256
    rng = np.random.default_rng(8)
    cams = [make_camera(W_, H_, elevation=12.0 * i, azimuth=55.0 * i + 5.0) for i in range(3)]
    ups = [torch.tensor(rng.standard_normal((3, 3, H_, W_)).astype(np.float32), device=dev) for _ in range(3)]
    bgimg = torch.tensor(rng.random((3, H_, W_, 3)).astype(np.float32), device=dev)
    P = scene["means3D"].shape[0]
    t = {k: torch.tensor(scene[k], device=dev, requires_grad=True)
         for k in ("means3D", "scales", "rotations", "opacities", "shs")}
    m2 = [torch.zeros((P, 3), device=dev, requires_grad=True) for _ in cams]
    st = [_settings(c, [0.1, 0.2, 0.3], int(scene["sh_degree"])) for c in cams]
    common = dict(opacities=t["opacities"], scales=t["scales"], rotations=t["rotations"])
    if kind == "ball_composite":
        outs = rasterize_views(st, t["means3D"], m2, shs=t["shs"], background=bgimg, **common)
    else:
        t["normals"] = torch.tensor(scene["normals"], device=dev, requires_grad=True)
        outs = rasterize_views(st, t["means3D"], m2, shs=t["shs"], colors2=t["normals"], **common)
    c, r, d, a = outs[:4]
    loss = (c * ups[0]).sum() + (d * ups[1][:, :1]).sum() + (a * ups[1][:, 1:2]).sum()
    if len(outs) > 4:
        loss = loss + (outs[4] * ups[2]).sum()
    if between is not None:  # (after the forward, before the backward)
        between()
    loss.backward()
    res = [x.detach() for x in outs] + [m.grad for m in m2] + [v.grad for v in t.values()]
    return [x.cpu().numpy() for x in res]


def _assert_bitwise(xs, ys, what):
    assert len(xs) == len(ys)
    for i, (x, y) in enumerate(zip(xs, ys)):
        assert x.dtype == y.dtype and np.array_equal(x, y), \
            f"{what}: output {i} differs: {float(np.abs(x.astype(np.float64) - y.astype(np.float64)).max())}"


@pytest.mark.parametrize("switch", ["fwd_kernel", "tile_keys", "mid_pass"])
@pytest.mark.parametrize("kind", ["ball_composite", "sugar_two_colors"])
def test_forward_kernels_bitwise(kind, switch, monkeypatch, tmp_path):
    """fwd_kernel: the one-wave-per-tile forward and the quadrant-wave forward (GSR_FWD_KERNEL) blend exactly
    the same candidates per pixel in the same order (the backward then culls from the tile-wave forward's
    quadrant masks or recomputes the cull); tile_keys: packed (tile, Gaussian) keys vs keys + values with the
    quadrant masks k_emit writes (the quadrant-wave forward then gathers only its quadrant's candidates) and
    without them (GSR_TILE_KEYS = unpacked | plain; large sets take the unpacked layout by themselves).  The
    layout override is read once per process (the backward derives the buffer layout from it on the host), so
    the forced layouts run in child processes.  Every output — colour, depth, alpha, the composite, the second
    colour set, radii — and every gradient (the backward reads the forward's per-pixel state) must be bitwise
    equal.  mid_pass: every switch changed between the forward and the backward to a value
    that differs from what the forward ran with (a child process sets GSR_TILE_KEYS=plain, GSR_FWD_KERNEL=tile
    and GSR_BWD_SPLIT=0 after a default forward: 3 views of 143 tiles take the quadrant-wave forward and split
    their backward) changes nothing: the backward follows the forward's recorded decisions on the device and
    the once-per-process layout latch."""
    if switch == "fwd_kernel":
        _assert_bitwise(bitwise_case(kind, monkeypatch, "tile"), bitwise_case(kind, monkeypatch, "quadrant"),
                        "tile-wave vs quadrant-wave forward")
        return
    import os
    import subprocess
    import sys

    base = bitwise_case(kind)
    if switch == "mid_pass":
        out = tmp_path / "mid.npz"
        code = ("import os, numpy as np, test_gpu_parity as t\n"
                "def flip():\n"
                "    os.environ.update(GSR_TILE_KEYS='plain', GSR_FWD_KERNEL='tile', GSR_BWD_SPLIT='0')\n"
                "np.savez(%r, *t.bitwise_case(%r, between=flip))\n" % (str(out), kind))
        env = dict(os.environ, PYTHONPATH=os.pathsep.join(p for p in sys.path if p))
        for k in ("GSR_TILE_KEYS", "GSR_FWD_KERNEL", "GSR_BWD_SPLIT"):
            env.pop(k, None)
        res = subprocess.run([sys.executable, "-c", code], cwd=os.path.dirname(os.path.abspath(__file__)), env=env,
                             capture_output=True, text=True, timeout=240)
        assert res.returncode == 0, res.stderr[-3000:]
        got = np.load(out)
        _assert_bitwise([got[f"arr_{i}"] for i in range(len(got.files))], base, "switches changed mid-pass")
        return
    for layout in ("unpacked", "plain"):
        out = tmp_path / f"{layout}.npz"
        code = "import numpy as np, test_gpu_parity as t; np.savez(%r, *t.bitwise_case(%r))" % (str(out), kind)
        env = dict(os.environ, GSR_TILE_KEYS=layout, PYTHONPATH=os.pathsep.join(p for p in sys.path if p))
        res = subprocess.run([sys.executable, "-c", code], cwd=os.path.dirname(os.path.abspath(__file__)), env=env,
                             capture_output=True, text=True, timeout=240)
        assert res.returncode == 0, res.stderr[-3000:]
        got = np.load(out)
        _assert_bitwise([got[f"arr_{i}"] for i in range(len(got.files))], base, f"{layout} keys vs packed")

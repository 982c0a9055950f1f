"""Fused background composite (include/gsr.h gsr_composite_*) against the reference's torch epilogue
(renderer/diff_gaussian_rasterizer_background.py:129-132, 139): forward bit-identical, gradients of
color / alpha / background equal to torch autograd of the same expression."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")


def _reference(color, alpha, bg_hwc):
    H, W = color.shape[-2:]
    return (color + (1 - alpha) * bg_hwc.reshape(-1, H, W, 3).permute(0, 3, 1, 2)).clamp(0, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(3, 64, 48), (5, 40, 36), (2, 30, 17)])
def test_composite_matches_torch(shape):
    from diff_gaussian_rasterization.composite import composite_background

    V, H, W = shape
    g = torch.Generator(device="cuda").manual_seed(V * 1000 + H)
    # values straddling the clamp bounds, incl. exact 0 / 1 pre-clamp values
    color = (torch.rand((V, 3, H, W), generator=g, device="cuda") * 1.4 - 0.2)
    color[:, 0, 0, 0] = 0.0
    alpha = torch.rand((V, 1, H, W), generator=g, device="cuda")
    alpha[:, 0, 0, :3] = 1.0
    bg = torch.rand((V, H, W, 3), generator=g, device="cuda")
    up = torch.randn((V, 3, H, W), generator=g, device="cuda")
    leaves = [t.clone().requires_grad_(True) for t in (color, alpha, bg)]
    ref = _reference(*leaves)
    ref.backward(up)
    mine = [t.clone().requires_grad_(True) for t in (color, alpha, bg)]
    out = composite_background(*mine)
    out.backward(up)
    assert torch.equal(out, ref)
    for a, b in zip(mine, leaves):
        np.testing.assert_allclose(a.grad.cpu().numpy(), b.grad.cpu().numpy(), rtol=1e-6, atol=1e-7)


@pytest.mark.gpu
def test_composite_single_view_and_constant_background():
    from diff_gaussian_rasterization.composite import composite_background

    H, W = 32, 24
    g = torch.Generator(device="cuda").manual_seed(3)
    color = torch.rand((3, H, W), generator=g, device="cuda").requires_grad_(True)
    alpha = torch.rand((1, H, W), generator=g, device="cuda").requires_grad_(True)
    bgc = torch.tensor([0.5, 0.25, 1.0], device="cuda")
    out = composite_background(color, alpha, bgc)
    ref = (color + (1 - alpha) * bgc[:, None, None]).clamp(0, 1)
    assert torch.equal(out, ref)
    up = torch.randn_like(ref)
    ga = torch.autograd.grad(out, (color, alpha), up)
    gr = torch.autograd.grad(ref, (color, alpha), up)
    for a, b in zip(ga, gr):
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-6, atol=1e-7)


def test_composite_symbols_exported():
    from diff_gaussian_rasterization import _C

    lib = _C.load_library()
    assert hasattr(lib, "gsr_composite_forward") and hasattr(lib, "gsr_composite_backward")


@pytest.mark.gpu
@pytest.mark.parametrize("V,H,W", [(3, 64, 48), (2, 40, 37)])
def test_fused_composite_matches_unfused(V, H, W):
    """rasterize_views(..., background=bg) == composite_background(rasterize_views(...)): forward bit-identical,
    gradients of every Gaussian parameter and of the background image identical."""
    import gsr_synthetic as gs
    from gsr_testutil import make_camera
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    from diff_gaussian_rasterization.batched import rasterize_views
    from diff_gaussian_rasterization.composite import composite_background

    scene = gs.make_scene(3000, sh_degree=3, seed=V)
    dev = "cuda"
    settings = []
    for v in range(V):
        cam = make_camera(W, H, azimuth=40.0 * v)
        settings.append(GaussianRasterizationSettings(
            image_height=H, image_width=W, tanfovx=cam["tanx"], tanfovy=cam["tany"],
            bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=torch.tensor(cam["view"], device=dev),
            projmatrix=torch.tensor(cam["proj"], device=dev), sh_degree=3,
            campos=torch.tensor(cam["campos"], device=dev), prefiltered=False, debug=False))
    g = torch.Generator(device=dev).manual_seed(7)
    bg = torch.rand((V, H, W, 3), generator=g, device=dev) * 1.2 - 0.1  # clamp bounds reached
    ups = [torch.randn((V, 3, H, W), generator=g, device=dev), torch.randn((V, 1, H, W), generator=g, device=dev),
           torch.randn((V, 1, H, W), generator=g, device=dev)]
    res = []
    for fused in (False, True):
        t = {k: torch.tensor(scene[k], device=dev, requires_grad=True)
             for k in ("means3D", "scales", "rotations", "opacities", "shs")}
        b = bg.clone().requires_grad_(True)
        m2 = [torch.zeros((3000, 3), device=dev, requires_grad=True) for _ in range(V)]
        kw = dict(shs=t["shs"], scales=t["scales"], rotations=t["rotations"])
        if fused:
            out, _, depth, alpha = rasterize_views(settings, t["means3D"], m2, t["opacities"], background=b, **kw)
        else:
            color, _, depth, alpha = rasterize_views(settings, t["means3D"], m2, t["opacities"], **kw)
            out = composite_background(color, alpha, b)
        torch.autograd.backward((out, depth, alpha), ups)
        res.append((out.detach(), {k: v.grad for k, v in t.items()}, b.grad, [m.grad for m in m2]))
    (o0, g0, b0, m0), (o1, g1, b1, m1) = res
    assert torch.equal(o0, o1)
    assert torch.equal(b0, b1)
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k
    for a, c in zip(m0, m1):
        assert torch.equal(a, c)


@pytest.mark.gpu
@pytest.mark.parametrize("V,H,W,two", [(3, 64, 48, False), (2, 40, 37, True)])
def test_fused_clamp_matches_torch_clamp(V, H, W, two):
    """rasterize_views(..., clamp=True) == rasterize_views(...)[0].clamp(0, 1) — the renderers' clamp of the
    colour output (renderer/diff_gaussian_rasterizer.py:141, renderer/diff_sugar_rasterizer_normal.py:212) formed
    in the blends: forward bit-identical, every gradient identical (the mask applied in the backward's per-pixel
    prologue), one colour set and two (the SuGaR normal renderer's calls)."""
    import gsr_synthetic as gs
    from gsr_testutil import make_camera
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    from diff_gaussian_rasterization.batched import rasterize_views

    P = 3000
    scene = gs.make_scene(P, sh_degree=3, seed=V + 10)
    dev = "cuda"
    settings = []
    for v in range(V):
        cam = make_camera(W, H, azimuth=40.0 * v)
        # backgrounds outside [0, 1]: the clamp bites on empty and thin pixels
        settings.append(GaussianRasterizationSettings(
            image_height=H, image_width=W, tanfovx=cam["tanx"], tanfovy=cam["tany"],
            bg=torch.tensor([1.3, -0.2, 0.5], device=dev), scale_modifier=1.0,
            viewmatrix=torch.tensor(cam["view"], device=dev), projmatrix=torch.tensor(cam["proj"], device=dev),
            sh_degree=3, campos=torch.tensor(cam["campos"], device=dev), prefiltered=False, debug=False))
    g = torch.Generator(device=dev).manual_seed(9)
    ups = [torch.randn((V, 3, H, W), generator=g, device=dev), torch.randn((V, 1, H, W), generator=g, device=dev),
           torch.randn((V, 1, H, W), generator=g, device=dev), torch.randn((V, 3, H, W), generator=g, device=dev)]
    n = torch.randn((P, 3), generator=g, device=dev)
    normals = n / n.norm(dim=1, keepdim=True)
    res = []
    for fused in (False, True):
        t = {k: torch.tensor(scene[k], device=dev, requires_grad=True)
             for k in ("means3D", "scales", "rotations", "opacities", "shs")}
        t["normals"] = normals.clone().requires_grad_(True)
        m2 = [torch.zeros((P, 3), device=dev, requires_grad=True) for _ in range(V)]
        kw = dict(shs=t["shs"], scales=t["scales"], rotations=t["rotations"])
        if two:
            kw["colors2"] = t["normals"]
        outs = rasterize_views(settings, t["means3D"], m2, t["opacities"], clamp=fused, **kw)
        out = outs[0] if fused else outs[0].clamp(0, 1)
        ts = [out, outs[2], outs[3]] + ([outs[4]] if two else [])
        torch.autograd.backward(ts, ups[:len(ts)])
        res.append(([x.detach() for x in ts], {k: v.grad for k, v in t.items()}, [m.grad for m in m2]))
    (o0, g0, m0), (o1, g1, m1) = res
    assert float((o0[0] == 0).float().mean() + (o0[0] == 1).float().mean()) > 0.01  # the clamp did bite
    for a, c in zip(o0, o1):
        assert torch.equal(a, c)
    for k in g0:
        if g0[k] is None:
            assert g1[k] is None, k
            continue
        assert torch.equal(g0[k], g1[k]), k
    for a, c in zip(m0, m1):
        assert torch.equal(a, c)

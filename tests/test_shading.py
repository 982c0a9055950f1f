"""Fused shading / depth-normal epilogue (include/gsr.h gsr_shade_*) against a torch restatement of the
reference's ops (tests/torch_reference.py: renderer/diff_gaussian_rasterizer_shading.py:22-51,169-208,
material/gaussian_material.py:86-104, renderer/diff_sugar_rasterizer_normal.py:170-197).

Floating-point kernel: the yardstick is torch fp64 on the CPU.  Bars: outputs within 1e-5 absolute
(render and normal maps live in [0, 1]); gradients within 1e-4 x max(1, max |g_ref|) per tensor, or 4x the
torch fp32 formulation's own error where that is larger (the normal is a normalised cross product of
central differences, so its conditioning depends on the surface)."""
import math

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import torch_reference as tr  # noqa: E402


def _scene(V, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    ys, xs = torch.meshgrid(torch.arange(H, dtype=torch.float64), torch.arange(W, dtype=torch.float64),
                            indexing="ij")
    out = []
    for v in range(V):
        ph = 0.7 * v
        depth = (2.0 + 0.3 * torch.sin(xs / 7.0 + ph) * torch.cos(ys / 5.0) + 0.002 * torch.rand((H, W), generator=g))
        # pinhole rays as threestudio builds them (x right, y up, -z forward; not normalised)
        f = 0.5 * H / math.tan(math.radians(30))
        d = torch.stack([(xs + 0.5 - W / 2) / f, -(ys + 0.5 - H / 2) / f, -torch.ones_like(xs)], -1)
        rot = torch.linalg.qr(torch.randn(3, 3, generator=g, dtype=torch.float64))[0]
        rays_d = d @ rot.T
        rays_o = torch.randn(3, generator=g, dtype=torch.float64).expand(H, W, 3).clone()
        alpha = torch.rand((1, H, W), generator=g, dtype=torch.float64)
        alpha[:, : H // 2, : W // 2] = 1.0                     # opaque block: normal / depth gradients kept
        alpha[:, H // 2:, : W // 3] = 0.995
        alpha[:, 0, :] = torch.where(torch.arange(W) % 2 == 0, 0.99, 0.9900001)  # the 0.99 boundary
        color = torch.rand((3, H, W), generator=g, dtype=torch.float64) * alpha * 1.2 - 0.05  # albedo clamp hits
        bg = torch.rand((H, W, 3), generator=g, dtype=torch.float64)
        light = torch.randn(3, generator=g, dtype=torch.float64) * 3
        pred = torch.rand((3, H, W), generator=g, dtype=torch.float64)
        ups = [torch.randn((3, H, W), generator=g, dtype=torch.float64),
               torch.randn((3, H, W), generator=g, dtype=torch.float64),
               torch.randn((1, H, W), generator=g, dtype=torch.float64)]
        out.append(dict(color=color, depth=depth[None], alpha=alpha, rays_o=rays_o, rays_d=rays_d, bg=bg,
                        light=light, pred=pred, ups=ups))
    return out


def _check(name, got, ref64, ref32, tol):
    got, ref64, ref32 = (x.detach().double().cpu().numpy() for x in (got, ref64, ref32))
    err = np.abs(got - ref64).max(initial=0.0)
    yard = np.abs(ref32 - ref64).max(initial=0.0)
    scale = max(1.0, float(np.abs(ref64).max(initial=0.0)))
    bar = max(tol * scale, 4.0 * yard)
    assert err <= bar, f"{name}: max err {err:.3g} > {bar:.3g} (torch fp32 yardstick {yard:.3g})"


def _reference(sc, dtype, shading, use_pred, ka, kd):
    leaves = {k: sc[k].to(dtype).clone().requires_grad_(True) for k in ("color", "depth", "alpha", "bg")}
    outs = tr.shading_epilogue(leaves["color"], leaves["depth"], leaves["alpha"], sc["rays_o"].to(dtype),
                               sc["rays_d"].to(dtype), leaves["bg"], sc["light"].to(dtype),
                               torch.tensor(ka, dtype=dtype), torch.tensor(kd, dtype=dtype), shading,
                               sc["pred"].to(dtype) if use_pred else None)
    torch.autograd.backward(outs, [u.to(dtype) for u in sc["ups"]])
    return outs, {k: v.grad for k, v in leaves.items()}


@pytest.mark.gpu
@pytest.mark.parametrize("shading,use_pred,V,H,W", [
    ("diffuse", False, 2, 40, 70),
    ("diffuse", True, 1, 33, 31),
    ("albedo", False, 1, 24, 64),
    ("textureless", False, 3, 17, 45),
])
def test_shade_views_match_torch(shading, use_pred, V, H, W):
    from diff_gaussian_rasterization.shading import shade_views

    ka, kd = (0.1, 0.2, 0.15), (0.9, 0.7, 0.8)
    scenes = _scene(V, H, W, seed=V * 100 + H)
    dev = "cuda"
    st = lambda k, dt=torch.float32: torch.stack([s[k] for s in scenes]).to(dev, dt)  # noqa: E731
    leaves = {k: st(k).requires_grad_(True) for k in ("color", "depth", "alpha", "bg")}
    render, nmap, depth = shade_views(leaves["color"], leaves["depth"], leaves["alpha"], st("rays_o"), st("rays_d"),
                                      leaves["bg"], st("light"), ka, kd, shading,
                                      st("pred") if use_pred else None)
    ups = [torch.stack([s["ups"][i] for s in scenes]).to(dev, torch.float32) for i in range(3)]
    torch.autograd.backward((render, nmap, depth), ups)
    for v, sc in enumerate(scenes):
        o64, g64 = _reference(sc, torch.float64, shading, use_pred, ka, kd)
        o32, g32 = _reference(sc, torch.float32, shading, use_pred, ka, kd)
        for name, got, r64, r32 in zip(("render", "normal", "depth"), (render[v], nmap[v], depth[v]), o64, o32):
            _check(f"view {v} {name}", got, r64, r32, 1e-5)
        for k in ("color", "depth", "alpha", "bg"):
            _check(f"view {v} d{k}", leaves[k].grad[v], g64[k], g32[k], 1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("V,H,W", [(3, 24, 40), (67, 9, 13)])
def test_shade_views_per_view_lights_and_modes(V, H, W):
    """Per-view (ka, kd, mode), as the material draws them once per view in training
    (material/gaussian_material.py:59-64,80-88); 67 views cross the 64-view launch chunk."""
    from diff_gaussian_rasterization.shading import shade_views

    modes = [("albedo", "textureless", "diffuse")[(7 * v + 1) % 3] for v in range(V)]
    kd = [(0.25 + 0.7 * ((v * 0.37) % 1.0),) * 3 for v in range(V)]  # soft shading: kd ~ U(0, 1), ka = 1 - kd
    ka = [(1.0 - d[0],) * 3 for d in kd]
    scenes = _scene(V, H, W, seed=11 + V)
    dev = "cuda"
    st = lambda k, dt=torch.float32: torch.stack([s[k] for s in scenes]).to(dev, dt)  # noqa: E731
    leaves = {k: st(k).requires_grad_(True) for k in ("color", "depth", "alpha", "bg")}
    render, nmap, depth = shade_views(leaves["color"], leaves["depth"], leaves["alpha"], st("rays_o"), st("rays_d"),
                                      leaves["bg"], st("light"), ka, kd, modes)
    ups = [torch.stack([s["ups"][i] for s in scenes]).to(dev, torch.float32) for i in range(3)]
    torch.autograd.backward((render, nmap, depth), ups)
    for v, sc in enumerate(scenes):
        o64, g64 = _reference(sc, torch.float64, modes[v], False, ka[v], kd[v])
        o32, g32 = _reference(sc, torch.float32, modes[v], False, ka[v], kd[v])
        for name, got, r64, r32 in zip(("render", "normal", "depth"), (render[v], nmap[v], depth[v]), o64, o32):
            _check(f"view {v} {name}", got, r64, r32, 1e-5)
        for k in ("color", "depth", "alpha", "bg"):
            _check(f"view {v} d{k}", leaves[k].grad[v], g64[k], g32[k], 1e-4)


def test_shade_tables_host_checks():
    from diff_gaussian_rasterization.shading import _light_table, _mode_table

    assert _light_table((0.1, 0.2, 0.3), 2) == (0.1, 0.2, 0.3, 0.1, 0.2, 0.3)
    assert _light_table([(0.1,) * 3, (0.5,) * 3], 2) == (0.1,) * 3 + (0.5,) * 3
    assert _mode_table("albedo", 2) == (1, 1)
    assert _mode_table(["diffuse", "textureless"], 2) == (0, 2)
    with pytest.raises(ValueError):
        _mode_table(["diffuse"], 2)
    with pytest.raises(ValueError):
        _mode_table("glossy", 1)
    with pytest.raises(ValueError):
        _light_table((0.1, 0.2), 1)


@pytest.mark.gpu
def test_shade_views_single_view_constant_background():
    from diff_gaussian_rasterization.shading import shade_views

    sc = _scene(1, 20, 36, seed=5)[0]
    ka, kd = (0.1, 0.1, 0.1), (0.9, 0.9, 0.9)
    bgc = torch.tensor([0.2, 0.5, 0.9], dtype=torch.float64)
    leaves = {k: sc[k].to("cuda", torch.float32).requires_grad_(True) for k in ("color", "depth", "alpha")}
    bg = bgc.to("cuda", torch.float32).requires_grad_(True)
    outs = shade_views(leaves["color"], leaves["depth"], leaves["alpha"], sc["rays_o"].float().cuda(),
                       sc["rays_d"].float().cuda(), bg, sc["light"].float().cuda(), ka, kd)
    torch.autograd.backward(outs, [u.float().cuda() for u in sc["ups"]])
    ref = {k: sc[k].clone().requires_grad_(True) for k in ("color", "depth", "alpha")}
    bref = bgc.clone().requires_grad_(True)
    H, W = 20, 36
    routs = tr.shading_epilogue(ref["color"], ref["depth"], ref["alpha"], sc["rays_o"], sc["rays_d"],
                                bref.expand(H, W, 3), sc["light"], torch.tensor(ka, dtype=torch.float64),
                                torch.tensor(kd, dtype=torch.float64))
    torch.autograd.backward(routs, sc["ups"])
    for a, b in zip(outs, routs):
        np.testing.assert_allclose(a.detach().cpu().double().numpy(), b.detach().numpy(), atol=1e-5)
    for k in ("color", "depth", "alpha"):
        g = ref[k].grad.numpy()
        np.testing.assert_allclose(leaves[k].grad.cpu().double().numpy(), g, atol=1e-4 * max(1, np.abs(g).max()))
    np.testing.assert_allclose(bg.grad.cpu().double().numpy(), bref.grad.numpy(), rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("V,H,W", [(1, 32, 32), (2, 27, 50)])
def test_depth_normal_views_match_torch(V, H, W):
    from diff_gaussian_rasterization.shading import depth_normal_views

    scenes = _scene(V, H, W, seed=7 + W)
    dev = "cuda"
    st = lambda k: torch.stack([s[k] for s in scenes]).to(dev, torch.float32)  # noqa: E731
    depth = st("depth").requires_grad_(True)
    alpha = st("alpha").requires_grad_(True)
    unit, nmap = depth_normal_views(depth, alpha, st("rays_o"), st("rays_d"))
    ups = [torch.stack([s["ups"][i] for s in scenes]).to(dev, torch.float32) for i in (0, 1)]
    torch.autograd.backward((unit, nmap), ups)
    for v, sc in enumerate(scenes):
        res = {}
        for dt in (torch.float64, torch.float32):
            d = sc["depth"].to(dt).clone().requires_grad_(True)
            a = sc["alpha"].to(dt).clone().requires_grad_(True)
            outs = tr.sugar_normal_from_dist(d, a, sc["rays_o"].to(dt), sc["rays_d"].to(dt))
            torch.autograd.backward(outs, [sc["ups"][i].to(dt) for i in (0, 1)])
            res[dt] = (outs, d.grad, a.grad)
        (o64, d64, a64), (o32, d32, a32) = res[torch.float64], res[torch.float32]
        _check("unit", unit[v], o64[0], o32[0], 1e-5)
        _check("nmap", nmap[v], o64[1], o32[1], 1e-5)
        _check("ddepth", depth.grad[v], d64, d32, 1e-4)
        _check("dalpha", alpha.grad[v], a64, a32, 1e-4)


def test_shading_has_no_cpu_path():
    from diff_gaussian_rasterization import _C
    from diff_gaussian_rasterization.shading import depth_normal_views

    sc = _scene(1, 8, 8, seed=1)[0]
    with pytest.raises(_C.GSRError):
        depth_normal_views(sc["depth"].float(), sc["alpha"].float(), sc["rays_o"].float(), sc["rays_d"].float())


def test_torch_restatement_gradients_finite_difference():
    """The torch restatement itself: the depth gradient through the normal stencil (incl. the zero-padded
    border) matches central finite differences in fp64."""
    sc = _scene(1, 9, 11, seed=2)[0]
    d = sc["depth"].clone().requires_grad_(True)
    up = sc["ups"][1]

    def f(dd):
        xyz = sc["rays_o"] + dd.permute(1, 2, 0) * sc["rays_d"]
        n = torch.nn.functional.normalize(tr.depth_to_normal(xyz.permute(2, 0, 1).unsqueeze(0))[0], dim=0)
        return (n * up).sum()

    (g,) = torch.autograd.grad(f(d), d)
    for (y, x) in [(0, 0), (0, 5), (4, 10), (8, 3), (2, 2)]:
        e = torch.zeros_like(d)
        e[0, y, x] = 1e-6
        fd = (f(sc["depth"] + e) - f(sc["depth"] - e)) / 2e-6
        assert abs(float(fd) - float(g[0, y, x])) < 1e-6 * max(1.0, abs(float(fd))) + 1e-7


@pytest.mark.gpu
def test_shade_saturated_masks_match_torch():
    """Pixels whose albedo col / (alpha + 1e-6) sits exactly on (or one ulp beside) the [0, 1] clamp edges
    and whose composited image saturates: the HIP backward must take every clamp-mask decision as the
    forward (and torch autograd in fp32 on the same inputs) does — a differing decision changes the
    gradient by O(1), far above the bar."""
    from diff_gaussian_rasterization.shading import shade_views

    H, W = 32, 48
    sc = _scene(1, H, W, seed=7)[0]
    dev = "cuda"
    al = sc["alpha"].float()
    ad = al + 1e-6
    g = torch.Generator().manual_seed(3)
    pick = torch.randint(0, 5, (3, H, W), generator=g)
    one = torch.ones_like(ad.expand(3, H, W))
    factor = torch.stack([one, torch.nextafter(one, 2 * one), torch.nextafter(one, 0 * one),
                          torch.full_like(one, 1.5), torch.zeros_like(one)])
    color = (ad * factor.gather(0, pick[None])[0]).float()  # alb exactly 1, 1 + ulp, 1 - ulp, 1.5, 0
    bg = torch.where(torch.rand((H, W, 3), generator=g) < 0.5, torch.ones(H, W, 3), torch.rand((H, W, 3), generator=g))
    ka, kd = (0.3, 0.3, 0.3), (0.9, 0.9, 0.9)  # tl up to 1.2: the image clamp at 1 saturates
    leaves = dict(color=color.to(dev), depth=sc["depth"].float().to(dev), alpha=al.to(dev), bg=bg.float().to(dev))
    ups = [u.float().to(dev) for u in sc["ups"]]
    ro, rd, light = sc["rays_o"].float().to(dev), sc["rays_d"].float().to(dev), sc["light"].float().to(dev)
    t = {k: v.clone().requires_grad_(True) for k, v in leaves.items()}
    outs = shade_views(t["color"], t["depth"], t["alpha"], ro, rd, t["bg"], light, ka, kd, "diffuse")
    torch.autograd.backward(outs, ups)
    r = {k: v.clone().requires_grad_(True) for k, v in leaves.items()}
    ref = tr.shading_epilogue(r["color"], r["depth"], r["alpha"], ro, rd, r["bg"], light,
                              torch.tensor(ka, device=dev), torch.tensor(kd, device=dev), "diffuse")
    torch.autograd.backward(ref, ups)
    for k in ("color", "bg", "alpha"):
        a, b = t[k].grad.double(), r[k].grad.double()
        err = ((a - b).abs() / b.abs().clamp(min=1.0)).max()
        assert float(err) <= 1e-4, f"grad {k}: {float(err)}"


def _normal_map_ref(normal, alpha):
    """renderer/diff_sugar_rasterizer_normal.py:192-197 for one view, in torch (the reference's lines)."""
    n = torch.nn.functional.normalize(normal, dim=0)
    n = torch.cat([-n[:2], n[2:]], 0)
    nmap = n * 0.5 * alpha + 0.5
    mask = (alpha > 0.99).repeat(3, 1, 1)
    return torch.where(mask, nmap, nmap.detach())


@pytest.mark.gpu
@pytest.mark.parametrize("V,H,W", [(1, 16, 16), (3, 27, 50)])
def test_sugar_normal_map_matches_torch(V, H, W):
    """The fused SuGaR normal map (normalize, axis flip, alpha-weighted map, alpha > 0.99 gradient mask) against
    the reference's torch lines in fp64 / fp32; a third of the pixels below the 0.99 mask and a few zero
    normals (the 1e-12 clamp)."""
    from diff_gaussian_rasterization.shading import sugar_normal_map

    g = torch.Generator().manual_seed(11 + W)
    normal = torch.randn((V, 3, H, W), generator=g, dtype=torch.float64)
    # (masks clear of 0.99, so fp32 and fp64 take the same side; the zero normals sit where alpha <= 0.99,
    # their clamped forward exercised, their gradient masked)
    alpha = torch.where(torch.rand((V, 1, H, W), generator=g) < 0.33, torch.rand((V, 1, H, W), generator=g) * 0.98,
                        0.995 + 0.005 * torch.rand((V, 1, H, W), generator=g)).double()
    normal[:, :, 0, :3] = 0.0
    alpha[:, :, 0, :3] = 0.5
    up = torch.randn((V, 3, H, W), generator=g, dtype=torch.float64)
    n_gpu = normal.float().cuda().requires_grad_(True)
    a_gpu = alpha.float().cuda().requires_grad_(True)
    out = sugar_normal_map(n_gpu, a_gpu)
    out.backward(up.float().cuda())
    for v in range(V):
        res = {}
        for dt in (torch.float64, torch.float32):
            n = normal[v].to(dt).clone().requires_grad_(True)
            a = alpha[v].to(dt).clone().requires_grad_(True)
            o = _normal_map_ref(n, a)
            o.backward(up[v].to(dt))
            res[dt] = (o, n.grad, a.grad)
        (o64, n64, a64), (o32, n32, a32) = res[torch.float64], res[torch.float32]
        _check("nmap", out[v], o64, o32, 1e-6)
        _check("dnormal", n_gpu.grad[v], n64, n32, 1e-5)
        _check("dalpha", a_gpu.grad[v], a64, a32, 1e-5)


def test_sugar_normal_map_has_no_cpu_path():
    from diff_gaussian_rasterization import _C
    from diff_gaussian_rasterization.shading import sugar_normal_map

    with pytest.raises(_C.GSRError):
        sugar_normal_map(torch.ones((1, 3, 4, 4)), torch.ones((1, 1, 4, 4)))

"""Parity at the BASELINE.json configurations and of the view-set path, against the oracle.

- C2 at full size (100k Gaussians, 512^2, SH3) through the per-view GaussianRasterizer;
- C3 (1M Gaussians, 1024^2, SH3, background path: bg = 0, then the composite with the background
  network's image + clamp of renderer/diff_gaussian_rasterizer_background.py:58,116-139) through
  rasterize_views with the composite fused into the blends, two views of the bench's orbit;
- rasterize_views compared directly with the oracle, view by view, on a 4-view set;
- equal-depth Gaussians keep the reference's (depth, index) order (stable sorts);
- the backward split into view groups (GSR_BWD_WORK_BYTES) and into view sets is bitwise invariant;
- C5: the SuGaR normal renderer (renderer/diff_sugar_rasterizer_normal.py:157-213) on ~2M
  surface-aligned Gaussians at 800^2: pass 1 with colors_precomp = get_points_rgb()
  (system/sugar_static.py:117-121, geometry/sugar.py:650-660: SH2RGB of the DC coefficients), the
  normal-from-distance maps, pass 2 with the face normals as colors_precomp and a zero means2D, the
  normal map and the alpha > 0.99 gradient masks; gradients of a loss over every output.

Bars as tests/gsr_testutil.py (fp64-oracle adjudication of fp32 decision flips).
"""
import math

import numpy as np
import pytest

import oracle
from gsr_testutil import (adjudicate, check_forward, check_grads, check_radii, flip_excuse, gs, make_camera, oracle_cam,
                          print_report, run_oracle)

pytestmark = pytest.mark.gpu

GRAD_KEYS = ["means3D", "opacity", "sh", "scales", "rotations"]
TORCH_NAMES = dict(means3D="means3D", scales="scales", rotations="rotations", opacities="opacity", shs="sh",
                   colors_precomp="colors")


@pytest.fixture(autouse=True)
def _parity_report():
    yield
    print_report()


def _settings(cam, bg, deg, mod=1.0):
    import torch

    from diff_gaussian_rasterization import GaussianRasterizationSettings

    dev = "cuda"
    return GaussianRasterizationSettings(cam["H"], cam["W"], cam["tanx"], cam["tany"],
                                         torch.tensor(bg, device=dev, dtype=torch.float32), mod,
                                         torch.tensor(cam["view"], device=dev), torch.tensor(cam["proj"], device=dev),
                                         deg, torch.tensor(cam["campos"], device=dev), False, False)


def _gpu_views(scene, cams, bgs, ups=None, background=None):
    """rasterize_views over `cams`; returns per-view numpy outputs, K, means2D grads and summed grads."""
    import torch

    from diff_gaussian_rasterization import _C
    from diff_gaussian_rasterization.batched import rasterize_views

    dev = "cuda"
    keys = [k for k in ("means3D", "scales", "rotations", "opacities", "shs", "colors_precomp") if scene.get(k) is not None]
    t = {k: torch.tensor(scene[k], device=dev, requires_grad=True) for k in keys}
    P = scene["means3D"].shape[0]
    V = len(cams)
    m2s = [torch.zeros((P, 3), device=dev, requires_grad=True) for _ in cams]
    bg_t = None if background is None else torch.tensor(background, device=dev, requires_grad=True)
    settings = [_settings(c, b, int(scene.get("sh_degree", 0))) for c, b in zip(cams, bgs)]
    c, r, d, a = rasterize_views(settings, t["means3D"], m2s, t["opacities"], shs=t.get("shs"),
                                 colors_precomp=t.get("colors_precomp"), scales=t["scales"],
                                 rotations=t["rotations"], background=bg_t)
    Ks = [k for k, _, _ in list(_C.RECENT_FORWARDS)[-V:]]
    out = dict(color=c.detach().cpu().numpy(), depth=d.detach().cpu().numpy(), alpha=a.detach().cpu().numpy(),
               radii=r.cpu().numpy(), K=Ks)
    if ups is not None:
        gc = torch.stack([torch.tensor(u[0], device=dev) for u in ups])
        gd = torch.stack([torch.tensor(u[1], device=dev) for u in ups])
        ga = torch.stack([torch.tensor(u[2], device=dev) for u in ups])
        ((c * gc).sum() + (d * gd).sum() + (a * ga).sum()).backward()
        for k, v in t.items():
            out["g_" + TORCH_NAMES[k]] = v.grad.cpu().numpy()
        out["g_means2D"] = [m.grad.cpu().numpy() for m in m2s]
        if bg_t is not None:
            out["g_background"] = bg_t.grad.cpu().numpy()
    return out


def _view(out, v):
    return dict(color=out["color"][v], depth=out["depth"][v], alpha=out["alpha"][v], radii=out["radii"][v])


def _sum_grads(refs, prec, keys):
    return {k: sum(np.asarray(r[prec][k], np.float64) for r in refs) for k in keys}


def _composite(color, alpha, bg_hwc):
    """renderer/diff_gaussian_rasterizer_background.py:129-132,139 in the arrays' precision, torch's op
    order: color + (1 - alpha) * bg, then clamp(0, 1).  Returns (render, pre-clamp value)."""
    one = color.dtype.type(1)
    pre = color + (one - alpha) * bg_hwc.transpose(2, 0, 1).astype(color.dtype)
    return np.clip(pre, 0, 1), pre


def _composite_upstream(g_render, g_alpha, pre, bg_hwc):
    """Gradients of the composite + clamp: dL/dcolor = g [0 <= pre <= 1], dL/dalpha += -sum_ch dL/dcolor bg,
    dL/dbg = dL/dcolor (1 - alpha) (torch's clamp passes the gradient on the closed interval)."""
    m = (pre >= 0) & (pre <= 1)
    gcol = np.where(m, g_render.astype(pre.dtype), 0)
    ga = g_alpha.astype(pre.dtype) - (gcol * bg_hwc.transpose(2, 0, 1).astype(pre.dtype)).sum(0, keepdims=True)
    return gcol, ga


# ------------------------------------------------------------------------------------------------

@pytest.mark.slow
def test_c2_full_100k_512_sh3():
    """C2 (BASELINE.json configs[1]): 100k Gaussians, 512^2, SH degree 3, fwd + bwd, white background."""
    from gsr_testutil import gpu_render

    scene = gs.make_scene(100_000, sh_degree=3, seed=0)
    cam = make_camera(512, 512)
    g = gs.upstream_grads(512, 512, seed=5)
    gpu = gpu_render(scene, cam, [1.0, 1.0, 1.0], grads=g)
    ref = run_oracle(scene, cam, [1.0, 1.0, 1.0], grads=g)
    check_forward(gpu, ref, "C2", K_gpu=gpu["K"])
    check_grads(gpu, ref, ["means3D", "means2D", "opacity", "sh", "scales", "rotations"], "C2")


@pytest.mark.slow
def test_c3_views_fused_background_composite():
    """C3 (configs[2]): 1M Gaussians, 1024^2, SH3, the background path with the composite fused into the
    blends, two views of the bench's 64-view orbit, forward + backward through rasterize_views."""
    scene = gs.make_scene(1_000_000, sh_degree=3, seed=0)
    cams = [make_camera(1024, 1024, elevation=0.0, azimuth=0.0), make_camera(1024, 1024, elevation=20.0, azimuth=202.5)]
    rng = np.random.default_rng(11)
    bg_img = rng.random((len(cams), 1024, 1024, 3)).astype(np.float32)
    ups = [gs.upstream_grads(1024, 1024, seed=40 + v) for v in range(len(cams))]
    zero = [0.0, 0.0, 0.0]
    gpu = _gpu_views(scene, cams, [zero] * len(cams), ups, background=bg_img)
    refs = []
    for v, cam in enumerate(cams):
        ref = run_oracle(scene, cam, zero)
        g_r, g_d, g_a = ups[v]
        b = {}
        for prec, dt in (("f32", np.float32), ("f64", np.float64)):
            f = ref[prec]
            render, pre = _composite(f["color"].astype(dt), f["alpha"].astype(dt), bg_img[v].astype(dt))
            f["color"] = render
            gcol, ga = _composite_upstream(g_r, g_a, pre, bg_img[v])
            b[prec] = oracle.backward(scene, oracle_cam(cam), np.zeros(3, np.float32), gcol, g_d, ga,
                                      prec=prec)
            if prec == "f32":  # another run of the reference's (unordered, atomic) accumulation
                b["f32r"] = oracle.backward(scene, oracle_cam(cam), np.zeros(3, np.float32), gcol, g_d, ga,
                                            prec="f32c", order=1)
            b["bg_" + prec] = (gcol * (dt(1) - f["alpha"].astype(dt))).transpose(1, 2, 0)
        check_forward(_view(gpu, v), ref, f"C3 view {v}", K_gpu=gpu["K"][v])
        adjudicate(gpu["g_means2D"][v], b["f32"]["means2D"], b["f64"]["means2D"],
                   1e-4 * np.maximum(1.0, np.abs(b["f64"]["means2D"])), f"C3 view {v}", "grad means2D", rowwise=True,
                   r32b=b["f32r"]["means2D"], excuse=flip_excuse([ref]))
        b["oracle_fwd"] = ref
        adjudicate(gpu["g_background"][v].reshape(-1, 3), b["bg_f32"].reshape(-1, 3), b["bg_f64"].reshape(-1, 3),
                   1e-4 * np.maximum(1.0, np.abs(b["bg_f64"].reshape(-1, 3))), f"C3 view {v}", "grad background",
                   rowwise=True)
        refs.append(b)
    tot = dict(b32=_sum_grads(refs, "f32", GRAD_KEYS), b64=_sum_grads(refs, "f64", GRAD_KEYS),
               b32r=_sum_grads(refs, "f32r", GRAD_KEYS))
    check_grads(gpu, tot, GRAD_KEYS, "C3 summed", excuse=flip_excuse([b["oracle_fwd"] for b in refs]))


def test_view_set_vs_oracle():
    """rasterize_views (one launch per stage for the set) vs the oracle per view: images, radii, K,
    per-view means2D gradients, and the parameter gradients summed over the views."""
    scene = gs.make_scene(30_000, sh_degree=3, seed=17)
    cams = [make_camera(320, 256, elevation=10.0 * i, azimuth=90.0 * i + 15.0) for i in range(4)]
    bgs = [[1.0, 1.0, 1.0], [0.0, 0.0, 0.0], [0.2, 0.5, 0.9], [0.7, 0.1, 0.3]]
    ups = [gs.upstream_grads(256, 320, seed=60 + v) for v in range(4)]
    gpu = _gpu_views(scene, cams, bgs, ups)
    refs = []
    for v, cam in enumerate(cams):
        ref = run_oracle(scene, cam, bgs[v], grads=ups[v])
        check_forward(_view(gpu, v), ref, f"set view {v}", K_gpu=gpu["K"][v])
        adjudicate(gpu["g_means2D"][v], ref["b32"]["means2D"], ref["b64"]["means2D"],
                   1e-4 * np.maximum(1.0, np.abs(ref["b64"]["means2D"])), f"set view {v}", "grad means2D",
                   rowwise=True, r32b=ref["b32r"]["means2D"], excuse=flip_excuse([ref]))
        refs.append(ref)
    tot = dict(b32=_sum_grads(refs, "b32", GRAD_KEYS), b64=_sum_grads(refs, "b64", GRAD_KEYS),
               b32r=_sum_grads(refs, "b32r", GRAD_KEYS))
    check_grads(gpu, tot, GRAD_KEYS, "set summed", excuse=flip_excuse(refs))


@pytest.mark.parametrize("layout", ["duplicates", "plane"])
def test_equal_depth_tie_order(layout):
    """Gaussians at exactly equal view depth blend in index order (the reference's stable radix sort of
    (tile | depth) keys over index-ordered instances).  duplicates: 3 copies of 300 means with different
    colours / opacities / footprints at indices i, i + 300, i + 600; plane: a camera looking straight
    along -x (elevation 0, azimuth 0: an exact axis-aligned view matrix) at Gaussians on three x = const
    planes (view depth depends on x only)."""
    from gsr_testutil import gpu_render

    rng = np.random.default_rng(3)
    if layout == "duplicates":
        base = gs.make_scene(300, sh_degree=0, seed=23)
        scene = {k: np.concatenate([base[k]] * 3, 0) for k in ("means3D", "scales", "rotations", "opacities")}
        scene["scales"] = scene["scales"] * rng.uniform(0.6, 1.6, size=(900, 1)).astype(np.float32)
        scene["opacities"] = rng.uniform(0.3, 0.95, size=(900, 1)).astype(np.float32)
        cam = make_camera(160, 144, azimuth=35.0)
    else:
        n = 900
        yz = rng.uniform(-0.5, 0.5, size=(n, 2)).astype(np.float32)
        x = np.float32(0.25) * rng.integers(0, 3, size=(n, 1)).astype(np.float32)
        scene = dict(means3D=np.concatenate([x, yz], 1), scales=np.full((n, 3), 0.04, np.float32),
                     rotations=np.tile(np.array([[1, 0, 0, 0]], np.float32), (n, 1)),
                     opacities=rng.uniform(0.3, 0.95, size=(n, 1)).astype(np.float32))
        cam = make_camera(160, 144, elevation=0.0, azimuth=0.0)  # exact axis-aligned view: depth = f(x)
        v = cam["view"].reshape(-1)
        depth = v[2] * scene["means3D"][:, 0] + v[6] * scene["means3D"][:, 1] + v[10] * scene["means3D"][:, 2] + v[14]
        assert len(np.unique(depth)) < n // 10, "plane layout should produce equal depths"
    P = scene["means3D"].shape[0]
    scene["colors_precomp"] = rng.random((P, 3)).astype(np.float32)
    scene["sh_degree"] = 0
    g = gs.upstream_grads(cam["H"], cam["W"], seed=9)
    gpu = gpu_render(scene, cam, [0.1, 0.1, 0.1], grads=g)
    ref = run_oracle(scene, cam, [0.1, 0.1, 0.1], grads=g)
    check_forward(gpu, ref, f"ties {layout}", K_gpu=gpu["K"])
    # a swapped pair of equal-depth Gaussians changes the colour by O(0.1): far beyond any flip allowance
    assert np.abs(gpu["color"] - ref["f32"]["color"]).max() < 1e-3
    check_grads(gpu, ref, ["means3D", "means2D", "opacity", "colors", "scales", "rotations"], f"ties {layout}")


def _batched_grads(scene, cams, ups, monkeypatch=None, budget=None, set_max=None):
    import torch

    from diff_gaussian_rasterization import batched

    if monkeypatch is not None:
        if budget is not None:
            monkeypatch.setattr(batched, "WORK_BUDGET", budget)
        if set_max is not None:
            monkeypatch.setattr(batched, "SET_MAX", set_max)
    out = _gpu_views(scene, cams, [[0.3, 0.3, 0.3]] * len(cams), ups)
    torch.cuda.synchronize()
    return out


def test_backward_view_groups_bitwise(monkeypatch):
    """gsr_set_backward walks the views in groups that fit the work buffer (GSR_BWD_WORK_BYTES);
    the per-Gaussian sums continue across groups in view order, so one view per group gives bitwise
    the gradients of one group for all views (include/gsr.h gsr_set_backward)."""
    from diff_gaussian_rasterization import _C

    scene = gs.make_scene(20_000, sh_degree=3, seed=29)
    cams = [make_camera(192, 160, elevation=5.0 * i, azimuth=60.0 * i) for i in range(6)]
    ups = [gs.upstream_grads(160, 192, seed=80 + v) for v in range(6)]
    one = _batched_grads(scene, cams, ups)
    lib = _C.load_library()
    import ctypes

    Ks = (ctypes.c_int * 6)(*one["K"])
    need = int(lib.gsr_set_backward_bytes(6, 20_000, Ks))
    largest = max(int(lib.gsr_backward_bytes(20_000, k)) for k in one["K"])
    assert largest * 3 <= need, "the split must produce at least 3 groups"
    split = _batched_grads(scene, cams, ups, monkeypatch, budget=1)  # work = one view's bytes: 6 groups
    for k in ("g_means3D", "g_opacity", "g_sh", "g_scales", "g_rotations"):
        assert np.array_equal(one[k], split[k]), k
    for v in range(6):
        assert np.array_equal(one["g_means2D"][v], split["g_means2D"][v])


@pytest.mark.parametrize("case", ["colors-one-group", "colors-six-groups", "colors-one-view"])
def test_gauss_fused_bitwise(case, monkeypatch):
    """The per-Gaussian backward fused into one kernel (k_gauss_fused: one thread per Gaussian walks the views,
    no per-(view, Gaussian) records; launches without SH — precomputed colours, the SuGaR renderers — as one
    group, as six groups of one view that continue the sums, and as one view) gives bitwise the gradients of
    the split kernels (GSR_GAUSS_FUSED=0: k_view_grad + k_gauss_accum)."""
    scene = gs.make_scene(20_000, sh_degree=0, seed=33)
    scene = dict(scene, colors_precomp=(scene["shs"][:, 0, :] * np.float32(gs.C0) +
                                        np.float32(0.5)).astype(np.float32))
    scene.pop("shs")
    nv = 1 if case == "colors-one-view" else 6
    cams = [make_camera(192, 160, elevation=5.0 * i, azimuth=60.0 * i) for i in range(nv)]
    ups = [gs.upstream_grads(160, 192, seed=90 + v) for v in range(nv)]
    budget = 1 if case.endswith("six-groups") else None
    fused = _batched_grads(scene, cams, ups, monkeypatch, budget=budget)
    monkeypatch.setenv("GSR_GAUSS_FUSED", "0")
    split = _batched_grads(scene, cams, ups, monkeypatch, budget=budget)
    keys = ["g_means3D", "g_opacity", "g_scales", "g_rotations", "g_colors"]
    for k in keys:
        assert np.array_equal(fused[k], split[k]), k
    for v in range(nv):
        assert np.array_equal(fused["g_means2D"][v], split["g_means2D"][v]), v


@pytest.mark.parametrize("split", ["off", "on"])
def test_view_sets_bitwise(split, monkeypatch):
    """20 views as one set vs four sets of 5 (later sets continue the sums: include/gsr.h accumulate with
    the running dL/dcov3D): identical images and bitwise identical gradients.  The split backward of sets of
    <= 8 views (gsr_render.hip split_on) replays other fp32 sums than the whole-prefix walk of a 20-view set:
    "off" compares 20 views against 4 x 5 with it disabled, "on" 8 views against 4 x 2 with it on in both."""
    scene = gs.make_scene(12_000, sh_degree=2, seed=31)
    nv = 20 if split == "off" else 8
    if split == "off":
        monkeypatch.setenv("GSR_BWD_SPLIT", "0")
    cams = [make_camera(128, 112, elevation=(i % 3) * 12.0, azimuth=18.0 * i) for i in range(nv)]
    ups = [gs.upstream_grads(112, 128, seed=120 + v) for v in range(nv)]
    one = _batched_grads(scene, cams, ups)
    sets = _batched_grads(scene, cams, ups, monkeypatch, set_max=5 if split == "off" else 2)
    for k in ("color", "depth", "alpha", "radii"):
        assert np.array_equal(one[k], sets[k]), k
    for k in ("g_means3D", "g_opacity", "g_sh", "g_scales", "g_rotations"):
        assert np.array_equal(one[k], sets[k]), k


def _deep_scene():
    """Many faint Gaussians in a small image: tiles blend well past GSR_SPLIT_NCK x GSR_SPLIT_CH candidates."""
    scene = gs.make_scene(80_000, sh_degree=1, seed=71, scale_mult=2.0, opacity_range=(0.005, 0.03))
    return scene, make_camera(80, 64, azimuth=25.0)


def _quad_maxc(scene, cam):
    """Per tile, the deepest blended list position of its quadrants (the image state's quad_maxc)."""
    import torch

    from diff_gaussian_rasterization import _C

    dev = "cuda"
    t = {k: torch.tensor(scene[k], device=dev) for k in ("means3D", "opacities", "scales", "rotations", "shs")}
    with torch.no_grad():
        out = _C.rasterize_gaussians(torch.zeros(3, device=dev), t["means3D"], None, t["opacities"], t["scales"],
                                     t["rotations"], 1.0, None, torch.tensor(cam["view"], device=dev),
                                     torch.tensor(cam["proj"], device=dev), cam["tanx"], cam["tany"], cam["H"],
                                     cam["W"], t["shs"], int(scene["sh_degree"]), torch.tensor(cam["campos"], device=dev),
                                     False, False)
    image = out[7].cpu().numpy()
    tiles = ((cam["W"] + 15) // 16) * ((cam["H"] + 15) // 16)
    # csrc/gsr_common.h ImageState: split_mode (one 256-byte unit), ranges, then quad_maxc
    off = 256 + (8 * tiles + 255) // 256 * 256
    return image[off:off + 16 * tiles].view(np.uint32).reshape(tiles, 4).max(1)


@pytest.mark.parametrize("size", ["listed", "overflow"])
def test_split_backward_matches_whole_walk(size, monkeypatch):
    """The split backward (sets of <= 8 views: GSR_SPLIT_NCK + 1 workgroups per tile, each replaying
    GSR_SPLIT_CH candidates from the forward's per-pixel checkpoint) against the whole-prefix walk
    (GSR_BWD_SPLIT=0): the same candidates and rows, other fp32 sums (the accumulated colour behind a chunk is
    suffix sums of the later chunks' own blends over T_chunk instead of the back-to-front recursion) — every
    gradient within the parity bar 1e-4 max(1, |g|) (lists here reach 20k candidates: both fp32 orders drift
    ~1e-5 from each other); and the scene does exercise every chunk.  "overflow": more later chunks than the
    GSR_SPLIT_EXTRA listed items, the tiles' own workgroups walk the rest (ImageState::split_cap)."""
    from gsr_testutil import gpu_render

    scene, cam = _deep_scene()
    if size == "overflow":
        cam = make_camera(448, 384, azimuth=25.0)
    maxc = _quad_maxc(scene, cam)
    later = int(np.minimum(15, np.maximum(maxc.astype(np.int64) - 1, 0) // 256).sum())
    print(f"later chunks {later}")
    assert (later > 1024) == (size == "overflow"), later
    print(f"split scene: tile maxc p50 {int(np.median(maxc))} max {int(maxc.max())} tiles > 256: {(maxc > 256).sum()}")
    assert (maxc > 256).sum() > 5 and maxc.max() > 1536, f"chunks not exercised: max {maxc.max()}"
    g = gs.upstream_grads(cam["H"], cam["W"], seed=17)
    split = gpu_render(scene, cam, [0.3, 0.2, 0.1], grads=g)
    monkeypatch.setenv("GSR_BWD_SPLIT", "0")
    whole = gpu_render(scene, cam, [0.3, 0.2, 0.1], grads=g)
    # the forward that writes the checkpoints keeps its running totals in list order: its outputs are bitwise
    # those of the launch without checkpoints (a view's bits do not depend on the launch size)
    for k in ("alpha", "radii", "color", "depth"):
        assert np.array_equal(split[k], whole[k]), k
    for k in ("g_means3D", "g_means2D", "g_opacity", "g_sh", "g_scales", "g_rotations"):
        ref = whole[k].astype(np.float64)
        err = float((np.abs(split[k] - ref) / np.maximum(1.0, np.abs(ref))).max())
        assert err <= 1e-4, f"{k}: {err}"


def test_split_backward_parity():
    """The split backward against the fp64 oracle with every parity test's bars (deep tiles: all chunks)."""
    from gsr_testutil import gpu_render

    scene, cam = _deep_scene()
    bg = [0.3, 0.2, 0.1]
    g = gs.upstream_grads(cam["H"], cam["W"], seed=17)
    gpu = gpu_render(scene, cam, bg, grads=g)
    ref = run_oracle(scene, cam, bg, grads=g)
    check_forward(gpu, ref, "split deep", K_gpu=gpu["K"])
    check_grads(gpu, ref, ["means3D", "means2D", "opacity", "sh", "scales", "rotations"], "split deep")


# ------------------------------------------------------------------------------------------------
# C5: the SuGaR normal renderer

def _sugar_epilogue(torch, color, depth, alpha, normal, rays_o, rays_d, depth_normal):
    """renderer/diff_sugar_rasterizer_normal.py:169-213 after the two rasterizer calls, one view (C,H,W).
    depth_normal(depth, alpha) -> (normal_from_dist, normal_map_from_dist) (both gradient masked)."""
    F = torch.nn.functional
    nfd, nmap_dist = depth_normal(depth, alpha)
    n = F.normalize(normal, dim=0)
    n = torch.cat([-n[:2], n[2:]], 0)
    nmap = n * 0.5 * alpha + 0.5
    mask = alpha > 0.99
    nmap = torch.where(mask.expand_as(nmap), nmap, nmap.detach())
    depth_m = torch.where(mask, depth, depth.detach())
    return dict(render=color.clamp(0, 1), normal=nmap, normal_from_dist=nmap_dist, mask=alpha, depth=depth_m,
                raw_normal_from_dist=nfd)


SUGAR_OUT = ("render", "normal", "normal_from_dist", "mask", "depth")


@pytest.mark.slow
def test_c5_sugar_normal_renderer():
    import torch

    import torch_reference as tr
    from diff_gaussian_rasterization.batched import rasterize_views
    from diff_gaussian_rasterization.cameras import orbit_c2w, ray_bundle
    from diff_gaussian_rasterization.shading import depth_normal_views

    S = 800
    scene = gs.make_sugar_scene(7, sh_degree=0, seed=0)
    P = scene["means3D"].shape[0]
    assert P > 1_900_000
    colors = (scene["shs"][:, 0, :] * np.float32(gs.C0) + np.float32(0.5)).astype(np.float32)  # SH2RGB(dc)
    normals = scene["normals"]
    cam = make_camera(S, S, elevation=15.0, azimuth=40.0)
    rays_o, rays_d = ray_bundle(orbit_c2w(2.5, 15.0, 40.0)[None], math.radians(60.0), S, S)
    rays_o, rays_d = rays_o[0].float(), rays_d[0].float()
    rng = np.random.default_rng(77)
    ups = {k: rng.standard_normal((1 if k in ("mask", "depth") else 3, S, S)).astype(np.float32) for k in SUGAR_OUT}

    def loss_of(out, tt):
        return sum((out[k] * tt(ups[k])).sum() for k in SUGAR_OUT)

    # ---- GPU: the two rasterize_views passes + the fused normal-from-depth epilogue ----
    dev = "cuda"
    leaf = lambda x: torch.tensor(x, device=dev, requires_grad=True)  # noqa: E731
    t = dict(means3D=leaf(scene["means3D"]), scales=leaf(scene["scales"]), rotations=leaf(scene["rotations"]),
             opacities=leaf(scene["opacities"]), colors=leaf(colors), normals=leaf(normals))
    s = _settings(cam, [0.0, 0.0, 0.0], 0)
    m2 = torch.zeros((P, 3), device=dev, requires_grad=True)
    # both rasterizer calls from one geometry / sort / blend (colors2 = the second call's colours)
    c, r, d, a, nrm = rasterize_views([s], t["means3D"], [m2], t["opacities"], colors_precomp=t["colors"],
                                      scales=t["scales"], rotations=t["rotations"], colors2=t["normals"])
    ro, rd = rays_o.to(dev), rays_d.to(dev)
    out = _sugar_epilogue(torch, c[0], d[0], a[0], nrm[0], ro, rd, lambda dd, aa: depth_normal_views(dd, aa, ro, rd))
    loss_of(out, lambda x: torch.tensor(x, device=dev)).backward()
    gpu_out = {k: out[k].detach().cpu().numpy() for k in SUGAR_OUT}
    gpu_grads = dict(g_means3D=t["means3D"].grad.cpu().numpy(), g_scales=t["scales"].grad.cpu().numpy(),
                     g_rotations=t["rotations"].grad.cpu().numpy(), g_opacity=t["opacities"].grad.cpu().numpy(),
                     g_colors=t["colors"].grad.cpu().numpy(), g_normals=t["normals"].grad.cpu().numpy(),
                     g_means2D=m2.grad.cpu().numpy())
    gpu_pass1 = dict(color=c[0].detach().cpu().numpy(), depth=d[0].detach().cpu().numpy(),
                     alpha=a[0].detach().cpu().numpy(), radii=r[0].cpu().numpy())
    del t, c, d, a, nrm, out
    torch.cuda.empty_cache()

    # ---- oracle: both passes in fp32 and fp64, the torch epilogue on CPU in the same precision ----
    sc1 = dict(scene, colors_precomp=colors)
    sc1.pop("shs")
    sc2 = dict(sc1, colors_precomp=normals)
    ref1 = run_oracle(sc1, cam, [0.0, 0.0, 0.0])
    ref2 = run_oracle(sc2, cam, [0.0, 0.0, 0.0])
    check_forward(gpu_pass1, ref1, "C5 pass 1")
    # The epilogue's upstream gradients into the rasterizer, from the torch restatement on the oracle's fp32 /
    # fp64 outputs (the normal-from-distance stencil is ill-conditioned: its fp32 and fp64 gradients differ
    # far more than the rasterizer's do, and the GPU's fused HIP epilogue — held to torch in
    # tests/test_shading.py — sees the GPU's depth)
    epi, ups_r = {}, {}
    for prec, dt in (("f32", torch.float32), ("f64", torch.float64)):
        f1, f2 = ref1[prec], ref2[prec]
        lc, ld, la, ln = (torch.tensor(x, dtype=dt, requires_grad=True)
                          for x in (f1["color"], f1["depth"], f1["alpha"], f2["color"]))
        o = _sugar_epilogue(torch, lc, ld, la, ln, rays_o.to(dt), rays_d.to(dt),
                            lambda dd, aa: tr.sugar_normal_from_dist(dd, aa, rays_o.to(dt), rays_d.to(dt)))
        loss_of(o, lambda x: torch.tensor(x, dtype=dt)).backward()
        epi[prec] = {k: o[k].detach().numpy() for k in SUGAR_OUT}
        # (the C ABI takes fp32 gradients)
        ups_r[prec] = [x.grad.numpy().astype(np.float32) for x in (lc, ld, la, ln)]

    def oracle_grads(prec, up, order=0):
        b1 = oracle.backward(sc1, oracle_cam(cam), np.zeros(3, np.float32), up[0], up[1], up[2], prec=prec,
                             order=order)
        b2 = oracle.backward(sc2, oracle_cam(cam), np.zeros(3, np.float32), up[3], None, None, prec=prec,
                             order=order)
        g = {k: np.asarray(b1[k], np.float64) + np.asarray(b2[k], np.float64)
             for k in ("means3D", "scales", "rotations", "opacity")}
        g.update(colors=b1["colors"], normals=b2["colors"], means2D=b1["means2D"])
        return g

    for k in SUGAR_OUT:
        a64 = epi["f64"][k]
        rows = lambda x: np.asarray(x).reshape(x.shape[0], -1).T  # noqa: E731
        adjudicate(rows(gpu_out[k]), rows(epi["f32"][k]), rows(a64), 1e-5 + 1e-5 * np.abs(rows(a64)), "C5", k,
                   cap=0.05 * max(1.0, float(np.abs(a64).max())))
    keys = ["means3D", "means2D", "opacity", "colors", "normals", "scales", "rotations"]
    # (1) the rasterizer (both calls' backward in one pass): the GPU backward with the fp32 epilogue's upstream
    # gradients, against the oracle's two backward passes with the same upstream gradients in fp32 / fp64 and
    # the fp32 one in reverse pixel order (another run of the reference's unordered atomic accumulation):
    # every row under the row rule
    up32 = ups_r["f32"]
    t = dict(means3D=leaf(scene["means3D"]), scales=leaf(scene["scales"]), rotations=leaf(scene["rotations"]),
             opacities=leaf(scene["opacities"]), colors=leaf(colors), normals=leaf(normals))
    m2 = torch.zeros((P, 3), device=dev, requires_grad=True)
    c, r, d, a, nrm = rasterize_views([s], t["means3D"], [m2], t["opacities"], colors_precomp=t["colors"],
                                      scales=t["scales"], rotations=t["rotations"], colors2=t["normals"])
    torch.autograd.backward((c[0], d[0], a[0], nrm[0]), [torch.tensor(x, device=dev) for x in up32])
    gpu_rast = dict(g_means3D=t["means3D"].grad.cpu().numpy(), g_scales=t["scales"].grad.cpu().numpy(),
                    g_rotations=t["rotations"].grad.cpu().numpy(), g_opacity=t["opacities"].grad.cpu().numpy(),
                    g_colors=t["colors"].grad.cpu().numpy(), g_normals=t["normals"].grad.cpu().numpy(),
                    g_means2D=m2.grad.cpu().numpy())
    del t, c, d, a, nrm
    torch.cuda.empty_cache()
    check_grads(gpu_rast, dict(b32=oracle_grads("f32", up32), b64=oracle_grads("f64", up32),
                               b32r=oracle_grads("f32c", up32, order=1)), keys, "C5 rasterizer",
                excuse=flip_excuse([ref1]))
    # (2) the renderer end to end (fused HIP epilogue + rasterizer) against the oracle's pipeline in fp32 / fp64:
    # the count rule (the epilogue's conditioning moves rows that no rasterizer difference explains)
    pipe32, pipe64 = oracle_grads("f32", up32), oracle_grads("f64", ups_r["f64"])
    for k in keys:
        r64 = np.asarray(pipe64[k], np.float64)
        adjudicate(gpu_grads["g_" + k], pipe32[k], r64, 1e-4 * np.maximum(1.0, np.abs(r64)), "C5 end to end",
                   "grad " + k, excuse=flip_excuse([ref1]))
    check_radii(gpu_pass1["radii"], ref1, "C5 pass 1")


@pytest.mark.parametrize("bwd", ["fused", "separate"])
def test_second_colors_match_separate_call(bwd, monkeypatch):
    """rasterize_views(colors2=...) — the SuGaR normal renderer's second rasterizer call from the first's
    geometry, sorts and blend — against the two separate calls (renderer/diff_sugar_rasterizer_normal.py:
    157-191): the second colour image bitwise equal, the first call's outputs and means2D gradient bitwise
    equal; parameter gradients (summed over both calls) within 1e-5 relative when the backward runs the two
    calls one after the other (two_color_backward="separate"), and then the first call's means2D gradient is
    bitwise the one-colour backward's.  The one-pass two-colour backward
    (gsr_set_backward_two_colors) adds both calls' dL/dalpha per pixel before the moments and the chain
    rule, an fp32 reassociation of the two-call sum (measured up to 1.6e-4 max(1, |g|) apart from the
    two-call sequence where the calls' gradients cancel): it is held to the fp64 oracle's two summed
    backward passes with the gradient bar of every parity test (check_grads); its sums come from hit lists
    (k_render_bwd_tw), the one-colour backward's from the matrix cores, so its means2D gradient matches the
    separate call's within that bar."""
    import torch

    # the two-colour backward never splits (its checkpoints hold the first colour only): compare it with
    # whole-prefix walks of the separate calls
    monkeypatch.setenv("GSR_BWD_SPLIT", "0")

    from diff_gaussian_rasterization.batched import rasterize_views

    scene = gs.make_scene(15_000, sh_degree=1, seed=44)
    rng = np.random.default_rng(4)
    n = rng.normal(size=(15_000, 3)).astype(np.float32)
    normals = n / np.linalg.norm(n, axis=1, keepdims=True)
    cams = [make_camera(144, 112, elevation=10.0 * i, azimuth=70.0 * i) for i in range(3)]
    ups = [torch.tensor(rng.standard_normal((3, 3, 112, 144)).astype(np.float32), device="cuda") for _ in range(3)]
    dev = "cuda"

    def run(fused, part=None):
        t = {k: torch.tensor(scene[k], device=dev, requires_grad=True)
             for k in ("means3D", "scales", "rotations", "opacities", "shs")}
        t["normals"] = torch.tensor(normals, device=dev, requires_grad=True)
        st = [_settings(c, [0.2, 0.4, 0.6], 1) for c in cams]
        m2 = [torch.zeros((15_000, 3), device=dev, requires_grad=True) for _ in cams]
        common = dict(opacities=t["opacities"], scales=t["scales"], rotations=t["rotations"])
        if fused:
            c, r, d, a, c2 = rasterize_views(st, t["means3D"], m2, shs=t["shs"], colors2=t["normals"],
                                             two_color_backward=bwd, **common)
        else:
            c, r, d, a = rasterize_views(st, t["means3D"], m2, shs=t["shs"], **common)
            z = [torch.zeros((15_000, 3), device=dev) for _ in cams]
            c2, _, _, _ = rasterize_views(st, t["means3D"], z, colors_precomp=t["normals"], **common)
        l1 = (c * ups[0]).sum() + (d * ups[1][:, :1]).sum() + (a * ups[1][:, 1:2]).sum()
        l2 = (c2 * ups[2]).sum()
        (l1 + l2 if part is None else l1 if part == 1 else l2).backward()
        grad = lambda v: v.grad.clone() if v.grad is not None else torch.zeros_like(v)  # noqa: E731
        return dict(c=c.detach(), c2=c2.detach(), d=d.detach(), a=a.detach(), r=r,
                    m2=[grad(m) for m in m2], g={k: grad(v) for k, v in t.items()})

    f, s_ = run(True), run(False)
    for k in ("c", "c2", "d", "a", "r"):
        assert torch.equal(f[k], s_[k]), k
    for v in range(3):
        if bwd == "separate":
            assert torch.equal(f["m2"][v], s_["m2"][v])
        else:
            ref = s_["m2"][v].double()
            err = float(((f["m2"][v].double() - ref).abs() / ref.abs().clamp(min=1.0)).max())
            assert err <= 1e-4, f"means2D view {v}: {err}"
    if bwd == "separate":
        for k in f["g"]:
            ref = s_["g"][k].double()
            err = float(((f["g"][k].double() - ref).abs() / ref.abs().clamp(min=1.0)).max())
            assert err <= 1e-5, f"grad {k}: {err}"
        return
    # the one-pass backward against the oracle's two backward passes, summed over the views (fp32 / fp64)
    bg = np.array([0.2, 0.4, 0.6], np.float32)
    sc2 = dict(scene, colors_precomp=normals)
    sc2.pop("shs")
    ref = {}
    for prec, order, key in (("f32", 0, "b32"), ("f64", 0, "b64"), ("f32c", 1, "b32r")):
        acc = {}
        for v, cam in enumerate(cams):
            u0, u1, u2 = (ups[i][v].cpu().numpy() for i in range(3))
            b1 = oracle.backward(scene, oracle_cam(cam), bg, u0, u1[:1], u1[1:2], prec=prec, order=order)
            b2 = oracle.backward(sc2, oracle_cam(cam), bg, u2, None, None, prec=prec, order=order)
            terms = {k: np.asarray(b1[k], np.float64) + np.asarray(b2[k], np.float64)
                     for k in ("means3D", "scales", "rotations", "opacity")}
            terms["sh"], terms["normals"] = np.asarray(b1["sh"], np.float64), np.asarray(b2["colors"], np.float64)
            for k, x in terms.items():
                acc[k] = acc.get(k, 0.0) + x
        ref[key] = acc
    gpu = {"g_" + k: f["g"][src].cpu().numpy() for k, src in (("means3D", "means3D"), ("scales", "scales"),
           ("rotations", "rotations"), ("opacity", "opacities"), ("sh", "shs"), ("normals", "normals"))}
    check_grads(gpu, ref, ["means3D", "scales", "rotations", "opacity", "sh", "normals"], "two-colour backward")
    print_report()


def test_two_color_backward_groups_and_sets_bitwise(monkeypatch):
    """The one-pass two-colour backward (gsr_set_backward_two_colors) walked in view groups that fit a small
    work buffer, and over several view sets (accumulate: dL/dcolors2 and the running dL/dcov3D continue in
    view order): bitwise the gradients of one group / one set.  And the second colours read from the records the
    preprocess embedded them in (gsr_set_preprocess_ex, the default) against gathered from colors2 apart: the same
    images and gradients, bit for bit."""
    import torch

    from diff_gaussian_rasterization import batched

    scene = gs.make_scene(12_000, sh_degree=1, seed=61)
    rng = np.random.default_rng(6)
    n = rng.normal(size=(12_000, 3)).astype(np.float32)
    normals = n / np.linalg.norm(n, axis=1, keepdims=True)
    cams = [make_camera(128, 96, elevation=8.0 * i, azimuth=50.0 * i) for i in range(6)]
    ups = [torch.tensor(rng.standard_normal((6, 3, 96, 128)).astype(np.float32), device="cuda") for _ in range(3)]

    def run():
        t = {k: torch.tensor(scene[k], device="cuda", requires_grad=True)
             for k in ("means3D", "scales", "rotations", "opacities", "shs")}
        t["normals"] = torch.tensor(normals, device="cuda", requires_grad=True)
        st = [_settings(c, [0.1, 0.2, 0.3], 1) for c in cams]
        m2 = [torch.zeros((12_000, 3), device="cuda", requires_grad=True) for _ in cams]
        c, _, d, a, c2 = batched.rasterize_views(st, t["means3D"], m2, t["opacities"], shs=t["shs"],
                                                 scales=t["scales"], rotations=t["rotations"], colors2=t["normals"])
        ((c * ups[0]).sum() + (d * ups[1][:, :1]).sum() + (a * ups[1][:, 1:2]).sum() + (c2 * ups[2]).sum()).backward()
        torch.cuda.synchronize()
        return [m.grad.clone() for m in m2], {k: v.grad.clone() for k, v in t.items()}, (c, d, a, c2)

    m2_one, g_one, o_one = run()
    with monkeypatch.context() as mp:
        mp.setattr(batched, "WORK_BUDGET", 1)  # one view per group
        m2_grp, g_grp, _ = run()
    with monkeypatch.context() as mp:
        mp.setattr(batched, "SET_MAX", 2)  # three sets of two views
        m2_set, g_set, _ = run()
    with monkeypatch.context() as mp:
        mp.setattr(batched, "EMBED_COLORS2", False)  # the blends gather colors2 apart
        m2_gat, g_gat, o_gat = run()
    for x, y in zip(o_one, o_gat):
        assert torch.equal(x, y), "embedded vs gathered second colours: images"
    for other, what in ((g_grp, "groups"), (g_set, "sets"), (g_gat, "gathered colors2")):
        for k in g_one:
            assert torch.equal(g_one[k], other[k]), f"{what}: grad {k}"
    for v in range(6):
        assert torch.equal(m2_one[v], m2_grp[v]) and torch.equal(m2_one[v], m2_set[v]), f"means2D {v}"
        assert torch.equal(m2_one[v], m2_gat[v]), f"means2D {v} (gathered colors2)"


def test_two_color_backward_with_fused_composite():
    """rasterize_views(background=..., colors2=...): the background renderer's fused composite on the first
    colour set and a second colour set in the same forward and the same one-pass backward
    (gsr_set_render_two_colors / gsr_set_backward_two_colors with bg_images): the parameter, background and
    colors2 gradients against the fp64 oracle's two backward passes with the composite's upstream gradients
    (renderer/diff_gaussian_rasterizer_background.py:129-132,139 restated in _composite_upstream)."""
    import torch

    from diff_gaussian_rasterization.batched import rasterize_views

    P = 15_000
    scene = gs.make_scene(P, sh_degree=1, seed=71)
    rng = np.random.default_rng(8)
    n = rng.normal(size=(P, 3)).astype(np.float32)
    normals = n / np.linalg.norm(n, axis=1, keepdims=True)
    cams = [make_camera(144, 112, elevation=12.0 * i, azimuth=80.0 * i) for i in range(2)]
    bg_img = rng.random((2, 112, 144, 3)).astype(np.float32)
    ups = [rng.standard_normal((2, 3, 112, 144)).astype(np.float32) for _ in range(3)]
    dev = "cuda"
    t = {k: torch.tensor(scene[k], device=dev, requires_grad=True)
         for k in ("means3D", "scales", "rotations", "opacities", "shs")}
    t["normals"] = torch.tensor(normals, device=dev, requires_grad=True)
    bg_t = torch.tensor(bg_img, device=dev, requires_grad=True)
    st = [_settings(c, [0.0, 0.0, 0.0], 1) for c in cams]
    m2 = [torch.zeros((P, 3), device=dev, requires_grad=True) for _ in cams]
    render, _, d, a, c2 = rasterize_views(st, t["means3D"], m2, t["opacities"], shs=t["shs"], scales=t["scales"],
                                          rotations=t["rotations"], background=bg_t, colors2=t["normals"])
    u = [torch.tensor(x, device=dev) for x in ups]
    ((render * u[0]).sum() + (d * u[1][:, :1]).sum() + (a * u[1][:, 1:2]).sum() + (c2 * u[2]).sum()).backward()

    sc2 = dict(scene, colors_precomp=normals)
    sc2.pop("shs")
    zero = np.zeros(3, np.float32)
    ref = {"b32": {}, "b64": {}, "b32r": {}}
    for v, cam in enumerate(cams):
        fw = run_oracle(scene, cam, [0.0, 0.0, 0.0])
        g_r, g_d, g_a = ups[0][v], ups[1][v][:1], ups[1][v][1:2]
        bgs = {}
        for prec, dt, order, key in (("f32", np.float32, 0, "b32"), ("f64", np.float64, 0, "b64"),
                                     ("f32c", np.float32, 1, "b32r")):
            f = fw["f32" if prec == "f32c" else prec]
            _, pre = _composite(f["color"].astype(dt), f["alpha"].astype(dt), bg_img[v].astype(dt))
            gcol, ga = _composite_upstream(g_r, g_a, pre, bg_img[v])
            b1 = oracle.backward(scene, oracle_cam(cam), zero, gcol, g_d, ga, prec=prec, order=order)
            b2 = oracle.backward(sc2, oracle_cam(cam), zero, ups[2][v], None, None, prec=prec, order=order)
            acc = ref[key]
            terms = {k: np.asarray(b1[k], np.float64) + np.asarray(b2[k], np.float64)
                     for k in ("means3D", "scales", "rotations", "opacity")}
            terms["sh"], terms["normals"] = np.asarray(b1["sh"], np.float64), np.asarray(b2["colors"], np.float64)
            for k, x in terms.items():
                acc[k] = acc.get(k, 0.0) + x
            if prec != "f32c":
                bgs[prec] = (gcol * (dt(1) - f["alpha"].astype(dt))).transpose(1, 2, 0).reshape(-1, 3)
                bgs["m2_" + prec] = b1["means2D"]
            else:
                bgs["m2_f32r"] = b1["means2D"]
        adjudicate(bg_t.grad[v].detach().cpu().numpy().reshape(-1, 3), bgs["f32"], bgs["f64"],
                   1e-4 * np.maximum(1.0, np.abs(bgs["f64"])), f"two colours + composite view {v}", "grad background",
                   rowwise=True)
        adjudicate(m2[v].grad.cpu().numpy(), bgs["m2_f32"], bgs["m2_f64"],
                   1e-4 * np.maximum(1.0, np.abs(bgs["m2_f64"])), f"two colours + composite view {v}", "grad means2D",
                   rowwise=True, r32b=bgs["m2_f32r"])
    gpu = {"g_" + k: t[src].grad.cpu().numpy() for k, src in (("means3D", "means3D"), ("scales", "scales"),
           ("rotations", "rotations"), ("opacity", "opacities"), ("sh", "shs"), ("normals", "normals"))}
    check_grads(gpu, ref, ["means3D", "scales", "rotations", "opacity", "sh", "normals"], "two colours + composite")
    print_report()

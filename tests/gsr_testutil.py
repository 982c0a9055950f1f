"""Shared helpers for the parity tests: run the HIP rasterizer through the public API and the CPU
oracle on identical float32 inputs, and compare with the tolerances stated in DESIGN.md §Parity."""
from __future__ import annotations

import math

import numpy as np

import gsr_synthetic as gs

# Parity bars (north_star): 1e-5 on RGB / alpha (depth 1e-5 abs + 1e-5 rel), and elementwise
# |g - g_ref| <= 1e-4 * max(1, |g_ref|) on gradients.  The reference values are the fp64 oracle's.
RGB_ATOL = 1e-5
DEPTH_RTOL = 1e-5
GRAD_TOL = 1e-4
# fp64 adjudication of discrete fp32 decisions (alpha >= 1/255, T (1 - alpha) >= 1e-4, the radius ceil):
# two correct fp32 evaluations (GPU exp2 vs libm expf, fma contraction) can land on different sides of a
# threshold and change a whole pixel contribution.  A pixel / gradient row may therefore miss the fp64
# result by more than the bar only as often as the fp32 oracle itself does (a faithful fp32
# implementation of the reference algorithm): at most FLIP_RATIO x its count + FLIP_SLACK, and image
# misses stay flip-sized.  Radii are compared bit-exactly with the fp32 oracle, excusing only Gaussians
# whose fp64 3 sqrt(lambda_max) lies within RAD_TIE of an integer (ceil flip), and num_rendered (K) must
# equal the oracle's up to exactly the rectangle-tile change of those excused Gaussians (and of Gaussians
# whose fp64 rectangle edge lies within RECT_TIE of a tile boundary).
FLIP_RATIO = 2
FLIP_SLACK = 3
# Gradients bind row by row on top of the count: a GPU element may miss the fp64 value by more than the bar
# only up to ROW_RATIO x the fp32 oracle's own miss of that element, |g - g64| <= max(bar, ROW_RATIO |g32 - g64|)
# (a faithful fp32 evaluation of an ill-conditioned row is allowed what the fp32 restatement needs, never
# more); at most ROW_SLACK rows (besides the excused flip dependents) may break that.
ROW_RATIO = 4.0
ROW_SLACK = 3
ROW_SLACK_PER_MILLION = 10  # the slack grows by 10 rows per million (C3 / C4: 1M rows)
# The reference's own fp32 results are not unique: nvcc contracts multiply-adds into FMAs by default and the
# per-Gaussian gradient sums are float atomics in an unspecified order.  A second fp32 oracle run built with
# contraction and visiting the pixels in reverse order (oracle.backward prec="f32c", order=1) is another faithful
# run of it; where it breaks the row rule against the first (either way) on `null` rows — the rows whose fp32
# result hinges on one rounding that an ill-conditioned step amplifies — the GPU may break it on up to
# slack + 2 null rows ("as far from the reference as the reference is from itself").  Measured: 0 rows at C1-C4
# and for SuGaR with unit upstream gradients; ~3 % of the bar-missing rows when the upstream depth gradient
# reaches ~1e3 (the normal-from-depth loss of the SuGaR renderer), e.g. 849 rows in 31.7k at 123k Gaussians.
RAD_TIE = 1e-5
RECT_TIE = 2e-5  # in tiles
REPORT = []  # (what, name, stats) of every adjudication, printed by the tests with -s


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
    from diff_gaussian_rasterization import _C

    out = dict(color=color.detach().cpu().numpy(), depth=depth.detach().cpu().numpy(),
               alpha=alpha.detach().cpu().numpy(), radii=radii.cpu().numpy(), K=_C.RECENT_FORWARDS[-1][0])
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


def run_oracle(scene, cam, bg, grads=None, mod=1.0):
    """fp32 + fp64 oracle forward (and backward when grads), plus the per-Gaussian aux values."""
    import oracle

    oc = oracle_cam(cam)
    bg = np.asarray(bg, np.float32)
    ref = dict(f32=oracle.forward(scene, oc, bg, "f32", mod=mod), f64=oracle.forward(scene, oc, bg, "f64", mod=mod),
               aux64=oracle.gauss_aux(scene, oc, "f64", mod=mod), aux32=oracle.gauss_aux(scene, oc, "f32", mod=mod),
               W=cam["W"], H=cam["H"])
    if grads is not None:
        ref["b32"] = oracle.backward(scene, oc, bg, *grads, prec="f32", mod=mod)
        ref["b32r"] = oracle.backward(scene, oc, bg, *grads, prec="f32c", mod=mod, order=1)
        ref["b64"] = oracle.backward(scene, oc, bg, *grads, prec="f64", mod=mod)
    return ref


def adjudicate(gpu, r32, r64, bar, what, name, cap=None, excuse=None, rowwise=False, r32b=None):
    """Rows (first axis) whose GPU value misses the fp64 value by more than `bar` (elementwise) may be at
    most FLIP_RATIO x the fp32 oracle's such rows + FLIP_SLACK; with `cap`, no GPU miss exceeds
    max(cap, 4 x the fp32 oracle's largest miss).  With `rowwise` (gradients) every element must also satisfy
    |g - g64| <= max(bar, ROW_RATIO |g32 - g64|), up to ROW_SLACK rows.  Returns the stats (incl.
    gpu_only_miss = rows the GPU misses where the fp32 oracle does not, and worst_ratio = the largest
    |g - g64| / max(bar, ROW_RATIO |g32 - g64|))."""
    gpu = np.asarray(gpu, np.float64).reshape(r64.shape)
    r32 = np.asarray(r32, np.float64)
    r64 = np.asarray(r64, np.float64)
    e_g = np.abs(gpu - r64)
    e_3 = np.abs(r32 - r64)
    n = r64.shape[0]
    bad_g = (e_g > bar).reshape(n, -1).any(1) if n else np.zeros(0, bool)
    bad_3 = (e_3 > bar).reshape(n, -1).any(1) if n else np.zeros(0, bool)
    ok_rows = ~bad_g
    n_excused = 0
    if excuse is not None and n:  # rows that depend on a pixel the GPU flipped where the fp32 oracle did not
        n_excused = int((bad_g & excuse).sum())
        bad_g = bad_g & ~excuse
        bad_3 = bad_3 & ~excuse
    lim = np.maximum(bar, ROW_RATIO * e_3)
    ratio = e_g / lim
    beyond = (ratio > 1.0).reshape(n, -1).any(1) if n else np.zeros(0, bool)
    if excuse is not None and n:
        beyond = beyond & ~excuse
    worst = ratio.reshape(n, -1).max(1) if n and ratio.size else np.zeros(0)
    worst_row = int(np.argmax(np.where(excuse, 0, worst))) if excuse is not None and n and worst.size else (
        int(np.argmax(worst)) if worst.size else -1)
    null = 0
    if r32b is not None and n:  # the reference against itself (another summation order)
        e_b = np.abs(np.asarray(r32b, np.float64).reshape(r64.shape) - r64)
        nb = (e_b > lim).reshape(n, -1).any(1) | (e_3 > np.maximum(bar, ROW_RATIO * e_b)).reshape(n, -1).any(1)
        if excuse is not None:
            nb = nb & ~excuse
        null = int(nb.sum())
    st = dict(rows=int(n), gpu_miss=int(bad_g.sum()), f32_miss=int(bad_3.sum()),
              gpu_only_miss=int((bad_g & ~bad_3).sum()), beyond_ratio=int(beyond.sum()),
              null_beyond=null if r32b is not None else None,
              worst_ratio=float(worst[worst_row]) if worst_row >= 0 else 0.0, worst_row=worst_row,
              max_err_gpu=float(e_g.max()) if e_g.size else 0.0, max_err_f32=float(e_3.max()) if e_3.size else 0.0,
              max_err_gpu_in_bar=float(e_g.reshape(n, -1)[ok_rows].max()) if ok_rows.any() and e_g.size else 0.0,
              max_diff_gpu_f32=float(np.abs(gpu - r32).max()) if e_g.size else 0.0, excused=n_excused)
    REPORT.append((what, name, st))
    allowed = FLIP_RATIO * st["f32_miss"] + FLIP_SLACK
    assert st["gpu_miss"] <= allowed, f"{what}: {name}: {st['gpu_miss']} rows miss the fp64 bar (allowed {allowed}): {st}"
    if cap is not None and st["gpu_miss"]:
        lim = max(cap, 4.0 * st["max_err_f32"])
        assert st["max_err_gpu"] <= lim, f"{what}: {name}: miss {st['max_err_gpu']} beyond flip size {lim}: {st}"
    if rowwise:
        allowed_rows = max(ROW_SLACK, (ROW_SLACK_PER_MILLION * n) // 1_000_000) + 2 * null
        assert st["beyond_ratio"] <= allowed_rows, (
            f"{what}: {name}: {st['beyond_ratio']} rows miss the fp64 value by more than max(bar, {ROW_RATIO} x the "
            f"fp32 oracle's miss) (allowed {allowed_rows}): {st}")
    return st


def _pixels(a):
    """(C, H, W) -> (H*W, C) rows of pixels."""
    a = np.asarray(a)
    return a.reshape(a.shape[0], -1).T


def rect_tiles(px, py, r, W, H):
    """getRect tile count of a radius r at pixel (px, py), in fp32 as the oracle / kernels compute it."""
    gx, gy = (W + 15) // 16, (H + 15) // 16
    f = np.float32
    px, py, rr = f(px), f(py), f(r)
    xmin = min(gx, max(0, int((px - rr) / f(16))))
    ymin = min(gy, max(0, int((py - rr) / f(16))))
    xmax = min(gx, max(0, int((px + rr + f(15)) / f(16))))
    ymax = min(gy, max(0, int((py + rr + f(15)) / f(16))))
    return (xmax - xmin) * (ymax - ymin)


def check_radii(r_gpu, ref, what, K_gpu=None):
    """Bit-exact radii vs the fp32 oracle except fp64-verified ceil flips; K exact up to those flips."""
    r32 = ref["f32"]["radii"]
    r_gpu = np.asarray(r_gpu).reshape(r32.shape)
    rad3 = ref["aux64"]["rad3"]
    diff = np.nonzero(r_gpu != r32)[0]
    excused_dk = 0
    for i in diff:
        t = rad3[i]
        n = float(np.round(t))
        tie = t > 0 and abs(t - n) <= RAD_TIE * max(1.0, t)
        cands = (int(n), int(n) + 1)
        assert tie and int(r_gpu[i]) in cands + (0,) and int(r32[i]) in cands + (0,) and r_gpu[i] + r32[i] > 0, (
            f"{what}: radius of Gaussian {i}: GPU {r_gpu[i]} vs oracle {r32[i]} (fp64 3 sqrt(lambda) = {t!r})")
        W, H = ref["W"], ref["H"]
        a = ref["aux32"]
        t_gpu = rect_tiles(a["px"][i], a["py"][i], int(r_gpu[i]), W, H) if r_gpu[i] > 0 else 0
        excused_dk += t_gpu - int(a["tiles"][i])
    REPORT.append((what, "radii", dict(rows=int(r32.size), gpu_miss=int(diff.size), excused_ceil_flips=int(diff.size))))
    if K_gpu is not None:
        K_ref = ref["f32"]["K"]
        # getRect boundary ties: a visible Gaussian whose fp64 (px - r) / 16, (px + r + 15) / 16 (or py) lies
        # within RECT_TIE of an integer may get one tile row / column more or less in fp32
        a64 = ref["aux64"]
        vis = r32 > 0
        r = r32[vis].astype(np.float64)
        vals = np.stack([(a64["px"][vis] - r) / 16, (a64["py"][vis] - r) / 16, (a64["px"][vis] + r + 15) / 16,
                         (a64["py"][vis] + r + 15) / 16], 1)
        tie = (np.abs(vals - np.round(vals)) <= RECT_TIE).any(1)
        rect = ref["aux32"]["rect"][vis]
        slack = int(((rect[:, 2] - rect[:, 0]) + (rect[:, 3] - rect[:, 1]) + 1)[tie].sum())
        dk = int(K_gpu) - (K_ref + excused_dk)
        REPORT.append((what, "num_rendered", dict(gpu=int(K_gpu), oracle=int(K_ref), ceil_flip_delta=int(excused_dk),
                                                  rect_ties=int(tie.sum()), rect_tie_slack=slack, residual=dk)))
        assert abs(dk) <= slack, (f"{what}: num_rendered {K_gpu} vs oracle {K_ref} (+{excused_dk} from ceil flips, "
                                  f"{int(tie.sum())} rect-boundary ties allow +-{slack})")


def check_forward(gpu, ref, what="", K_gpu=None, color_key="color"):
    """Colour / alpha (1e-5) and depth (1e-5 abs + rel) per pixel vs fp64 with fp32-oracle adjudication;
    radii and K as check_radii."""
    f32, f64 = ref["f32"], ref["f64"]
    scale_c = max(1.0, float(np.abs(f64["color"]).max()))
    d64 = _pixels(f64["depth"])
    scale_d = max(1.0, float(np.abs(d64).max()))
    gpu_only = np.zeros(d64.shape[0], bool)
    for key, bar, cap in ((color_key, RGB_ATOL, 0.02 * scale_c), ("alpha", RGB_ATOL, 0.02),
                          ("depth", RGB_ATOL + DEPTH_RTOL * np.abs(d64), 0.02 * scale_d)):
        rk = "color" if key == color_key else key
        g, o3, o6 = _pixels(gpu[key]).astype(np.float64), _pixels(f32[rk]).astype(np.float64), _pixels(f64[rk])
        adjudicate(g, o3, o6, bar, what, rk, cap=cap)
        gpu_only |= (np.abs(g - o6) > bar).any(1) & ~(np.abs(o3 - o6) > bar).any(1)
    # pixels where the GPU took a different discrete decision than both oracles (allowed above, as often
    # as the fp32 oracle does so): every Gaussian blended at such a pixel has a legitimately different
    # gradient; check_grads excuses those rows
    ref["gpu_only_px"] = np.nonzero(gpu_only)[0]
    if "radii" in gpu:
        check_radii(gpu["radii"], ref, what, K_gpu)


def flip_dependents(ref, pixels):
    """Gaussians that reach alpha >= 1/255 (fp64 preprocess values, 1 % margin) at any of `pixels`."""
    a = ref["aux64"]
    P = a["px"].shape[0]
    dep = np.zeros(P, bool)
    if len(pixels) == 0 or P == 0:
        return dep
    vis = a["tiles"] > 0
    W = ref["W"]
    for pid in pixels:
        y, x = divmod(int(pid), W)
        dx, dy = a["px"] - x, a["py"] - y
        power = -0.5 * (a["conic"][:, 0] * dx * dx + a["conic"][:, 2] * dy * dy) - a["conic"][:, 1] * dx * dy
        alpha = np.minimum(0.99, a["opacity"] * np.exp(np.minimum(power, 0.0)))
        dep |= vis & (power <= 0) & (alpha >= 0.99 / 255.0)
    return dep


def flip_excuse(refs):
    """Union over views (run_oracle dicts that went through check_forward) of the Gaussians blended at a pixel
    the GPU flipped on its own: their gradient rows legitimately differ (see check_forward)."""
    out = None
    for r in refs:
        if "aux64" not in r:
            continue
        d = flip_dependents(r, r.get("gpu_only_px", ()))
        out = d if out is None else (out | d)
    return out


def check_grads(gpu, ref, keys, what="", excuse=None):
    """Elementwise |g - g64| <= 1e-4 max(1, |g64|) with fp32-oracle adjudication of flip-affected rows;
    rows of Gaussians blended at a pixel the GPU flipped on its own (check_forward) are excused (`excuse`:
    the rows to excuse when `ref` is not a run_oracle dict, e.g. gradients summed over views: flip_excuse)."""
    b32, b64, b32r = ref["b32"], ref["b64"], ref.get("b32r")
    if excuse is None:
        excuse = flip_dependents(ref, ref.get("gpu_only_px", ())) if "aux64" in ref else None
    out, failed = {}, []
    for k in keys:  # every tensor is adjudicated (and reported) before the first failure is raised
        r64 = b64[k]
        bar = GRAD_TOL * np.maximum(1.0, np.abs(r64))
        ex = excuse if excuse is not None and excuse.shape[0] == r64.shape[0] else None
        try:
            out[k] = adjudicate(gpu["g_" + k], b32[k], r64, bar, what, "grad " + k, excuse=ex, rowwise=True,
                                r32b=b32r[k] if b32r is not None else None)
        except AssertionError as e:
            failed.append(str(e))
    assert not failed, "\n".join(failed)
    return out


def assert_image_parity(gpu, ref32, what="", scene=None, cam=None, bg=None, mod=1.0):
    """Back-compat wrapper: full fp64-adjudicated forward check (needs scene / cam / bg)."""
    ref = run_oracle(scene, cam, bg, mod=mod)
    check_forward(gpu, ref, what)
    return 0


def print_report(reset=True):
    for what, name, st in REPORT:
        print(f"PARITY {what} {name} {st}")
    if reset:
        REPORT.clear()


def last_num_rendered():
    from diff_gaussian_rasterization import _C

    return _C.RECENT_FORWARDS[-1][0]


def scene_subset(scene, **over):
    s = dict(scene)
    s.update(over)
    return s


__all__ = ["gs", "make_camera", "oracle_cam", "gpu_render", "run_oracle", "check_forward", "check_grads",
           "check_radii", "adjudicate", "print_report", "last_num_rendered", "flip_excuse", "flip_dependents"]

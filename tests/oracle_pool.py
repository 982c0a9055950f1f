"""Per-view oracle runs in a pool of spawned processes (TEST INFRASTRUCTURE: the checker side of the view-set
parity tests; never the thing measured or shipped).

The CPU oracle (oracle/gsr_oracle.c) runs serially and keeps process-global state (the backward's accumulation
order), so large view sets run one view per task in separate processes.  Spawned, not forked: the parent holds a
GPU context.  Each worker rebuilds the seeded scene from its spec (no scene pickling) and returns per view either
the forward results for the caller's per-view checks, or — for sets whose per-view gradient rows would not fit
in memory — its own partial sums of the parameter gradients and the Gaussians to excuse (blended at a pixel the
GPU flipped on its own, tests/gsr_testutil.py flip_dependents), so that only a few partial sums cross the pipe.
"""
from __future__ import annotations

import multiprocessing as mp
import os

import numpy as np

_SCENES = {}


def scene_of(spec):
    """spec = ("ball", n, sh_degree, seed) | ("sugar", subdiv, sh_degree, seed, colors): colors False keeps the
    SH, True = SH2RGB(dc) as colors_precomp (the SuGaR normal renderer's pass 1), "normals" = the face normals as
    colors_precomp (its pass 2)."""
    key = tuple(spec)
    if key not in _SCENES:
        import gsr_synthetic as gs

        if spec[0] == "ball":
            s = gs.make_scene(spec[1], sh_degree=spec[2], seed=spec[3])
        else:
            s = gs.make_sugar_scene(spec[1], sh_degree=spec[2], seed=spec[3])
            if spec[4] == "normals":
                s = dict(s, colors_precomp=np.ascontiguousarray(s["normals"], np.float32))
                s.pop("shs")
            elif spec[4]:  # pass 1 of the SuGaR normal renderer: colours = SH2RGB(dc) as colors_precomp
                s = dict(s, colors_precomp=(s["shs"][:, 0, :] * np.float32(gs.C0) + np.float32(0.5)).astype(np.float32))
                s.pop("shs")
        _SCENES.clear()
        _SCENES[key] = s
    return _SCENES[key]


def composite(color, alpha, bg_hwc):
    """renderer/diff_gaussian_rasterizer_background.py:129-132,139 in the arrays' precision."""
    one = color.dtype.type(1)
    pre = color + (one - alpha) * bg_hwc.transpose(2, 0, 1).astype(color.dtype)
    return np.clip(pre, 0, 1), pre


def composite_upstream(g_render, g_alpha, pre, bg_hwc):
    m = (pre >= 0) & (pre <= 1)
    gcol = np.where(m, g_render.astype(pre.dtype), 0)
    ga = g_alpha.astype(pre.dtype) - (gcol * bg_hwc.transpose(2, 0, 1).astype(pre.dtype)).sum(0, keepdims=True)
    return gcol, ga


GRAD_KEYS = ("means3D", "sh", "opacity", "scales", "rotations", "colors", "cov3D")


def _view_task(task):
    """One view: fp32 / fp64 forwards (+ the background composite when bg_img is given, in each precision) and
    the backwards of the upstream gradients `ups` = (dL/dcolour-or-render, dL/ddepth, dL/dalpha) in fp32 and fp64
    (and fp32 in the other accumulation order, tag "f32r", when `want` holds it; "cov32": the per-view fp32
    dL/dcov3D stays in the kept view results).  With `gpu_img` (the GPU's
    colour or render of the view): the pixels the GPU flipped on its own and the Gaussians to excuse there.
    Returns dict(f32, f64 forward dicts, aux64, W, H, b = {tag: backward dict}[, gpu_only_px, excuse])."""
    import oracle
    from gsr_testutil import flip_dependents, oracle_cam

    spec, cam, bg, ups, bg_img, gpu_img, want = task
    scene = scene_of(spec)
    oc = oracle_cam(cam)
    bg = np.asarray(bg, np.float32)
    out = dict(W=cam["W"], H=cam["H"])
    b = {}
    for prec, dt in (("f32", np.float32), ("f64", np.float64)):
        f = oracle.forward(scene, oc, bg, prec)
        g_c, g_d, g_a = ups
        if bg_img is not None:
            render, pre = composite(f["color"].astype(dt), f["alpha"].astype(dt), bg_img.astype(dt))
            f["color"] = render
            g_c, g_a = composite_upstream(ups[0], ups[2], pre, bg_img)
        out[prec] = f
        runs = [(prec, prec, 0)] + ([("f32r", "f32c", 1)] if prec == "f32" and "f32r" in want else [])
        for tag, p, order in runs:
            b[tag] = oracle.backward(scene, oc, bg, np.asarray(g_c, np.float32), g_d, np.asarray(g_a, np.float32),
                                     prec=p, order=order)
    out["aux64"] = oracle.gauss_aux(scene, oc, "f64")
    if "aux32" in want:  # (check_radii's rectangle test)
        out["aux32"] = oracle.gauss_aux(scene, oc, "f32")
    if gpu_img is not None:  # the GPU's own flips (check_forward's rule on the colour) -> the rows to excuse
        px = lambda a: np.asarray(a, np.float64).reshape(3, -1).T  # noqa: E731
        e_g = np.abs(px(gpu_img) - px(out["f64"]["color"])).max(1)
        e_3 = np.abs(px(out["f32"]["color"]) - px(out["f64"]["color"])).max(1)
        out["gpu_only_px"] = np.nonzero((e_g > 1e-5) & ~(e_3 > 1e-5))[0]
        out["excuse"] = flip_dependents(out, out["gpu_only_px"])
    out["b"] = b
    return out


def _chunk(args):
    """A chunk of views: their parameter gradients summed in float64 per precision, the union of their excused
    rows, and (keep_views) each view's forward results, aux64, flips and means2D gradients.  One result per chunk
    crosses the pipe; the per-view parameter gradients stay in the worker."""
    tasks, keep_views = args
    part, views = {}, []
    for task in tasks:
        r = _view_task(task)
        for tag, b in r["b"].items():
            acc = part.setdefault(tag, {})
            for k in GRAD_KEYS:
                if k in b:
                    acc[k] = acc.get(k, 0.0) + np.asarray(b[k], np.float64)
        ex = r.get("excuse")
        if ex is not None:
            part["excuse"] = ex if "excuse" not in part else (part["excuse"] | ex)
        if keep_views:
            want = task[6]
            r["b"] = {tag: dict({"means2D": b["means2D"]},
                                **({"cov3D": b["cov3D"]} if tag == "f32" and "cov32" in want else {}))
                      for tag, b in r["b"].items()}
            views.append(r)
    return views, part


def _pool(workers):
    return mp.get_context("spawn").Pool(workers)


def workers_for(n_tasks, cap=16):
    return max(1, min(n_tasks, cap, os.cpu_count() or 1))


def scale_rot_chain(dcov, scales, rots, mod=1.0, dt=np.float32):
    """The scale / rotation chain rule of oracle/gsr_oracle.c (oracle_backward, computeCov3D's backward) applied
    once to dL/dcov3D already summed over views and calls, in precision `dt` — the association the GPU's
    per-Gaussian backward uses (it sums dL/dcov3D over the set's views before the chain rule; the oracle applies
    it per view).  A null model for the summed scale / rotation gradients."""
    c = np.asarray(dcov, dt)
    q = np.asarray(rots, dt)
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    one, two = dt(1), dt(2)
    R = np.empty((q.shape[0], 3, 3), dt)
    R[:, 0, 0] = one - two * (y * y + z * z)
    R[:, 0, 1] = two * (x * y - r * z)
    R[:, 0, 2] = two * (x * z + r * y)
    R[:, 1, 0] = two * (x * y + r * z)
    R[:, 1, 1] = one - two * (x * x + z * z)
    R[:, 1, 2] = two * (y * z - r * x)
    R[:, 2, 0] = two * (x * z - r * y)
    R[:, 2, 1] = two * (y * z + r * x)
    R[:, 2, 2] = one - two * (x * x + y * y)
    s = dt(mod) * np.asarray(scales, dt)
    h = dt(0.5)
    G = np.stack([np.stack([c[:, 0], h * c[:, 1], h * c[:, 2]], 1),
                  np.stack([h * c[:, 1], c[:, 3], h * c[:, 4]], 1),
                  np.stack([h * c[:, 2], h * c[:, 4], c[:, 5]], 1)], 1)
    dE = np.empty_like(R)
    for a in range(3):
        for k in range(3):
            dE[:, a, k] = two * (G[:, a, 0] * s[:, k] * R[:, 0, k] + G[:, a, 1] * s[:, k] * R[:, 1, k]
                                 + G[:, a, 2] * s[:, k] * R[:, 2, k])
    dsc = np.stack([dE[:, 0, k] * R[:, 0, k] + dE[:, 1, k] * R[:, 1, k] + dE[:, 2, k] * R[:, 2, k]
                    for k in range(3)], 1)
    dR = dE * s[:, None, :]
    d = lambda a, k: dR[:, a, k]  # noqa: E731
    f4 = dt(4)
    drot = np.stack([
        -two * z * d(0, 1) + two * y * d(0, 2) + two * z * d(1, 0) - two * x * d(1, 2) - two * y * d(2, 0)
        + two * x * d(2, 1),
        two * y * d(0, 1) + two * z * d(0, 2) + two * y * d(1, 0) - f4 * x * d(1, 1) - two * r * d(1, 2)
        + two * z * d(2, 0) + two * r * d(2, 1) - f4 * x * d(2, 2),
        -f4 * y * d(0, 0) + two * x * d(0, 1) + two * r * d(0, 2) + two * x * d(1, 0) + two * z * d(1, 2)
        - two * r * d(2, 0) + two * z * d(2, 1) - f4 * y * d(2, 2),
        -f4 * z * d(0, 0) - two * r * d(0, 1) + two * x * d(0, 2) + two * r * d(1, 0) - f4 * z * d(1, 1)
        + two * y * d(1, 2) + two * x * d(2, 0) + two * y * d(2, 1)], 1)
    return dsc, drot


def views_and_sums(tasks, keep_views=True, workers=None):
    """Run every task's view; returns (per-view results in task order, or [] without keep_views; totals) with
    totals = {tag: {key: float64 sum over the views}} for each precision tag ("f32", "f64", "f32r" when asked
    for) and "excuse" = the union of the views' excused rows (tasks with a GPU image)."""
    w = workers or workers_for(len(tasks))
    idx = [list(range(len(tasks)))[i::w] for i in range(w)]
    idx = [ix for ix in idx if ix]
    with _pool(len(idx)) as pool:
        outs = pool.map(_chunk, [([tasks[i] for i in ix], keep_views) for ix in idx], chunksize=1)
    views = [None] * len(tasks) if keep_views else []
    total = {}
    for ix, (vs, part) in zip(idx, outs):
        for i, r in zip(ix, vs):
            views[i] = r
        for tag, v in part.items():
            if tag == "excuse":
                total["excuse"] = v if "excuse" not in total else (total["excuse"] | v)
                continue
            acc = total.setdefault(tag, {})
            for k, x in v.items():
                acc[k] = acc.get(k, 0.0) + x
    return views, total

"""View-batched rasterization: one set of Gaussians, V cameras, one autograd node.

Equivalent to calling GaussianRasterizer once per view (same per-view outputs and gradients), but the
views are rendered as view sets of up to 64 (include/gsr.h, gsr_set_*): every stage — preprocess,
depth sort, instance emission, tile sort, blend, backward blend, per-Gaussian backward — is ONE launch
per set instead of one per view, sorts are segmented by view, and the instance counts of all views are
read back with one host sync.  The reference renders a batch with a Python loop over views
(renderer/gaussian_batch_renderer.py:9-122); this replaces the loop's V rasterizer calls.

Per-view outputs (color, radii, depth, alpha) and per-view means2D gradients (the densification
statistic of geometry/gaussian_base.py:815-818) are kept; shared-parameter gradients are summed over
views inside the per-Gaussian kernel.
"""
from __future__ import annotations

import ctypes
import math
import os
import time

import torch

from . import _C

SET_MAX = 64
# device memory the backward may use at once for gradient rows (views are walked in groups that fit)
WORK_BUDGET = int(os.environ.get("GSR_BWD_WORK_BYTES", str(24 << 30))) & ~255  # (256-byte granularity)


def _arr(ctype, values):
    return (ctype * len(values))(*values)


def _ptrs(ts):
    return _arr(ctypes.c_void_p, [t.data_ptr() for t in ts])


class _ViewSet:
    """Forward state of one set of views."""

    def __init__(self, lo, hi, cams, tanx, tany):
        self.lo, self.hi = lo, hi
        self.cams = cams  # [(view, proj, campos, bg)] contiguous fp32 device tensors
        self.tanx, self.tany = tanx, tany
        self.K = None
        self.geom = self.binning = self.image = None
        # the host arrays the C ABI takes, built once for the forward and the backward
        self.arrays = (_ptrs([c[0] for c in cams]), _ptrs([c[1] for c in cams]), _ptrs([c[2] for c in cams]),
                       _arr(ctypes.c_float, tanx), _arr(ctypes.c_float, tany))
        self.bgs = _ptrs([c[3] for c in cams])
        self.Karr = None

    @property
    def V(self):
        return self.hi - self.lo

    def cam_arrays(self):
        return self.arrays


# A two-colour forward hands colors2 to the preprocess too (gsr_set_preprocess_ex), which writes each Gaussian's
# second colour into the record it writes anyway; the blends then read it from the record's line.  False: the
# blends gather colors2 apart (the same bits; tests/test_gpu_configs.py compares the two).
EMBED_COLORS2 = True


class _RasterizeViews(torch.autograd.Function):
    @staticmethod
    def forward(ctx, settings_list, grad_reduce, two_color_bwd, clamp, means3D, sh, colors_precomp, opacities, scales,
                rotations, cov3D_precomp, composite_bg, colors2, *means2D):
        t0 = time.perf_counter()
        lib = _C.load_library()
        V = len(settings_list)
        dev = means3D.device
        _C._require_gpu(dev)
        P = int(means3D.shape[0])
        s0 = settings_list[0]
        H, W = int(s0.image_height), int(s0.image_width)
        if any(int(s.image_height) != H or int(s.image_width) != W for s in settings_list):
            raise _C.GSRError("all views of a batch must have the same image size")
        f = lambda t, n: _C._f32(t, n, dev)  # noqa: E731
        m3, shc, col, op, sc, rot, c3 = (f(means3D, "means3D"), f(sh, "sh"), f(colors_precomp, "colors_precomp"),
                                         f(opacities, "opacities"), f(scales, "scales"), f(rotations, "rotations"),
                                         f(cov3D_precomp, "cov3D_precomp"))
        if (shc is None) == (col is None):
            raise Exception("Please provide excatly one of either SHs or precomputed colors!")
        M = _C.sh_coeff_count(shc)
        p = _C._ptr
        stream = _C._stream(dev)
        fopt = dict(dtype=torch.float32, device=dev)
        color = torch.empty((V, 3, H, W), **fopt)
        cbg = None
        # the renderer's clamp(0, 1) fused into the blends without a background image (clamp_only) or with it
        clamp_only = bool(clamp) and composite_bg is None
        if composite_bg is not None:
            cbg = _C._f32(composite_bg, "background", dev).reshape(V, H, W, 3)
        fused_out = cbg is not None or clamp_only
        if fused_out:
            render = torch.empty((V, 3, H, W), **fopt)
        depth = torch.empty((V, 1, H, W), **fopt)
        alpha = torch.empty((V, 1, H, W), **fopt)
        c2 = None
        if colors2 is not None:
            c2 = _C._f32(colors2, "colors2", dev)
            if c2.numel() != 3 * P:
                raise _C.GSRError(f"colors2 has {c2.numel()} elements, expected {3 * P}")
            color2 = torch.empty((V, 3, H, W), **fopt)
        radii = torch.empty((V, P), dtype=torch.int32, device=dev)
        sets = []
        for lo in range(0, V, SET_MAX):
            hi = min(V, lo + SET_MAX)
            cams = [(f(s.viewmatrix, "viewmatrix"), f(s.projmatrix, "projmatrix"), f(s.campos, "campos"),
                     f(s.bg, "bg")) for s in settings_list[lo:hi]]
            vs = _ViewSet(lo, hi, cams, [float(s.tanfovx) for s in settings_list[lo:hi]],
                          [float(s.tanfovy) for s in settings_list[lo:hi]])
            vs.geom = torch.empty(int(lib.gsr_set_geom_bytes(vs.V, P)), dtype=torch.uint8, device=dev)
            views, projs, campos, tx, ty = vs.cam_arrays()
            t0 = _C.host_mark("fwd_setup", t0)
            # (the second colour set, when there is one, rides in the records the preprocess writes: the two-colour
            # blends then read it with the record instead of gathering it apart)
            _C._check(lib.gsr_set_preprocess_ex(
                vs.V, P, int(s0.sh_degree), M, p(m3), p(sc), float(s0.scale_modifier), p(rot), p(op), p(shc), p(col),
                p(c3), views, projs, campos, tx, ty, W, H, int(bool(s0.prefiltered)), p(radii[lo:hi]), p(vs.geom),
                p(c2) if c2 is not None and EMBED_COLORS2 else None, stream))
            sets.append(vs)
            t0 = _C.host_mark("fwd_preprocess_launch", t0)
        for vs in sets:
            K = (ctypes.c_int * vs.V)()
            L = (ctypes.c_int * vs.V)()
            # the reference's one host sync: the instance counts size the binning buffers
            _C._check(lib.gsr_set_num_rendered_ex(vs.V, p(vs.geom), P, K, None, L, stream))
            t0 = _C.host_mark("fwd_sync_wait", t0)
            vs.K = list(K)
            _C.RECENT_LISTED.extend(L)
            _C.RECENT_FORWARDS.extend((k, H, W) for k in vs.K)
            Karr = vs.Karr = _arr(ctypes.c_int, vs.K)
            vs.binning = torch.empty(int(lib.gsr_set_binning_bytes(vs.V, P, Karr, W, H)), dtype=torch.uint8, device=dev)
            vs.image = torch.empty(int(lib.gsr_set_image_bytes_ex(vs.V, P, Karr, W, H, int(c2 is not None))),
                                   dtype=torch.uint8, device=dev)
            sl = slice(vs.lo, vs.hi)
            if c2 is not None:
                _C._check(lib.gsr_set_render_two_colors(
                    vs.V, P, Karr, W, H, vs.bgs, p(vs.geom), p(vs.binning), p(vs.image),
                    p(color[sl]), p(depth[sl]), p(alpha[sl]), p(cbg[sl]) if cbg is not None else None,
                    p(render[sl]) if fused_out else None, p(c2), p(color2[sl]), stream))
            elif not fused_out:
                _C._check(lib.gsr_set_render(vs.V, P, Karr, W, H, vs.bgs, p(vs.geom),
                                             p(vs.binning), p(vs.image), p(color[sl]), p(depth[sl]), p(alpha[sl]),
                                             stream))
            else:
                _C._check(lib.gsr_set_render_composite(
                    vs.V, P, Karr, W, H, vs.bgs, p(vs.geom), p(vs.binning), p(vs.image),
                    p(color[sl]), p(depth[sl]), p(alpha[sl]), p(cbg[sl]) if cbg is not None else None,
                    p(render[sl]), stream))
            t0 = _C.host_mark("fwd_render_launch", t0)
        ctx.settings = settings_list
        ctx.grad_reduce = grad_reduce
        ctx.two_color_bwd = two_color_bwd
        ctx.sets = sets
        ctx.bg_shape = tuple(composite_bg.shape) if composite_bg is not None else None
        ctx.save_for_backward(m3, shc, col, sc, rot, c3, radii, cbg, color if fused_out else None, c2)
        ctx.mark_non_differentiable(radii)
        if c2 is not None:
            return (render if fused_out else color), radii, depth, alpha, color2
        return (render if fused_out else color), radii, depth, alpha

    @staticmethod
    def backward(ctx, g_color, _g_radii, g_depth, g_alpha, g_color2=None):
        t0 = time.perf_counter()
        lib = _C.load_library()
        m3, shc, col, sc, rot, c3, radii, cbg, color, c2 = ctx.saved_tensors
        second = c2 is not None and g_color2 is not None
        settings = ctx.settings
        V = len(settings)
        s0 = settings[0]
        dev = m3.device
        P = int(m3.shape[0])
        M = _C.sh_coeff_count(shc)
        H, W = int(s0.image_height), int(s0.image_width)
        fopt = dict(dtype=torch.float32, device=dev)
        d_m2 = torch.empty((V, P, 3), **fopt)
        # the per-Gaussian gradients are carved from one buffer (means3D, scales, rotations, opacities,
        # SH, cov3D, colours): autograd hands these views to the leaves as their .grad, and
        # view_shard.allreduce_grads then sums them over ranks in place as one span, without copies
        widths = [("m3", (3,)), ("sc", (3,) if c3 is None else None), ("rot", (4,) if c3 is None else None),
                  ("op", (1,)), ("sh", (M, 3) if shc is not None else None), ("c3", (6,) if c3 is not None else None),
                  ("col", (3,))]
        flat = torch.empty(P * sum(math.prod(w) for _, w in widths if w is not None), **fopt)
        carved, off = {}, 0
        for name, w in widths:
            carved[name] = None
            if w is not None:
                n = P * math.prod(w)
                carved[name] = flat[off:off + n].view((P,) + w)
                off += n
        d_m3, d_sc, d_rot, d_op = carved["m3"], carved["sc"], carved["rot"], carved["op"]
        d_sh, d_c3, d_col = carved["sh"], carved["c3"], carved["col"]
        d_bg = torch.empty_like(cbg) if cbg is not None and ctx.needs_input_grad[11] else None
        # more than one view set in the scale / rotation path: the running dL/dcov3D the later sets
        # continue from (include/gsr.h gsr_set_backward, accumulate)
        d_c2 = torch.zeros((P, 3), **fopt) if second else None
        if d_c3 is None and (len(ctx.sets) > 1 or second):
            d_c3 = torch.empty((P, 6), **fopt)
            ctx.needs_c3_scratch = True
        if P == 0:
            if d_bg is not None:
                d_bg.zero_()
            for t in (d_m2, d_m3, d_op, d_col, d_sh, d_c3, d_sc, d_rot, d_c2):
                if t is not None:
                    t.zero_()
        else:
            gc = g_color.float().contiguous()
            gd = g_depth.float().contiguous() if g_depth is not None else None
            ga = g_alpha.float().contiguous() if g_alpha is not None else None
            stream = _C._stream(dev)
            p = _C._ptr
            # both calls of a two-colour forward in one backward pass (gsr_set_backward_two_colors);
            # two_color_backward="separate" runs the second call's backward after the first's instead
            fused2 = second and ctx.two_color_bwd != "separate"
            if fused2:
                g2 = g_color2.float().contiguous()
            reducer = ctx.grad_reduce if ctx.grad_reduce is not None and ctx.grad_reduce.active() else None
            # per-range events only when the last set's call is the last writer of the per-Gaussian sums: with
            # the second colour's backward run separately after it (two_color_backward="separate"), that call
            # adds into the same gradients, so the reduction waits for the whole stream instead
            events = reducer.chunk_events(dev) if reducer is not None and (fused2 or not second) else None
            for si, vs in enumerate(ctx.sets):
                if events is not None and si == len(ctx.sets) - 1:
                    # the last set's call forms the final per-Gaussian sums: in ranges, an event after each
                    _C._check(lib.gsr_set_backward_chunks(
                        len(events), _arr(ctypes.c_void_p, [e.cuda_event for e in events])))
                Karr = vs.Karr
                # (the scratch grows with K: the largest single view bounds what a view group needs)
                kmax = _arr(ctypes.c_int, [max(vs.K)])
                if fused2:
                    need = int(lib.gsr_set_backward_two_colors_bytes(vs.V, P, Karr))
                    largest = int(lib.gsr_set_backward_two_colors_bytes(1, P, kmax))
                else:
                    need = int(lib.gsr_set_backward_bytes(vs.V, P, Karr))
                    largest = int(lib.gsr_set_backward_bytes(1, P, kmax))
                work = torch.empty(max(largest, min(need, WORK_BUDGET)), dtype=torch.uint8, device=dev)
                views, projs, campos, tx, ty = vs.cam_arrays()
                sl = slice(vs.lo, vs.hi)
                gdp = p(gd[sl]) if gd is not None else None
                gap = p(ga[sl]) if ga is not None else None
                if fused2:
                    _C._check(lib.gsr_set_backward_two_colors(
                        vs.V, P, int(s0.sh_degree), M, Karr, W, H, vs.bgs, p(m3), p(sc),
                        float(s0.scale_modifier), p(rot), p(shc), p(c3), views, projs, campos, tx, ty, p(radii[sl]),
                        p(vs.geom), p(vs.binning), p(vs.image), p(cbg[sl]) if cbg is not None else None,
                        p(color[sl]) if color is not None else None, p(gc[sl]), gdp, gap,
                        p(d_bg[sl]) if d_bg is not None else None, p(c2), p(g2[sl]), p(d_m2[sl]), p(d_col), p(d_c2),
                        p(d_op), p(d_m3), p(d_c3), p(d_sh), p(d_sc), p(d_rot), 1 if si > 0 else 0, p(work),
                        work.numel(), stream))
                    continue
                if color is None:
                    _C._check(lib.gsr_set_backward(
                        vs.V, P, int(s0.sh_degree), M, Karr, W, H, vs.bgs, p(m3), p(sc),
                        float(s0.scale_modifier), p(rot), p(shc), p(c3), views, projs, campos, tx, ty, p(radii[sl]),
                        p(vs.geom), p(vs.binning), p(vs.image), p(gc[sl]), gdp, gap, p(d_m2[sl]), p(d_col), p(d_op),
                        p(d_m3), p(d_c3), p(d_sh), p(d_sc), p(d_rot), 1 if si > 0 else 0, p(work), work.numel(),
                        stream))
                else:
                    _C._check(lib.gsr_set_backward_composite(
                        vs.V, P, int(s0.sh_degree), M, Karr, W, H, vs.bgs, p(m3), p(sc),
                        float(s0.scale_modifier), p(rot), p(shc), p(c3), views, projs, campos, tx, ty, p(radii[sl]),
                        p(vs.geom), p(vs.binning), p(vs.image), p(cbg[sl]) if cbg is not None else None,
                        p(color[sl]), p(gc[sl]), gdp, gap,
                        p(d_bg[sl]) if d_bg is not None else None, p(d_m2[sl]), p(d_col), p(d_op), p(d_m3), p(d_c3),
                        p(d_sh), p(d_sc), p(d_rot), 1 if si > 0 else 0, p(work), work.numel(), stream))
                if second:
                    # the second call's backward on the shared forward state (its screen-space gradient
                    # is discarded, as the reference's fresh zero means2D of that call is)
                    g2 = g_color2.float().contiguous()
                    m2_scratch = torch.empty((vs.V, P, 3), **fopt)
                    _C._check(lib.gsr_set_backward_colors(
                        vs.V, P, Karr, W, H, vs.bgs, p(m3), p(sc), float(s0.scale_modifier),
                        p(rot), p(c3), views, projs, campos, tx, ty, p(radii[sl]), p(vs.geom), p(vs.binning),
                        p(vs.image), p(c2), p(g2[sl]), p(m2_scratch), p(d_c2), p(d_op), p(d_m3), p(d_c3), p(d_sc),
                        p(d_rot), 1, p(work), work.numel(), stream))
        if d_bg is not None:
            d_bg = d_bg.reshape(ctx.bg_shape)
        if getattr(ctx, "needs_c3_scratch", False):
            d_c3 = None
        grads = [None, None, None, None, d_m3, d_sh, d_col, d_op, d_sc, d_rot, d_c3, d_bg, d_c2] + \
            [d_m2[v] for v in range(V)]
        for k, need in enumerate(ctx.needs_input_grad):
            if not need:
                grads[k] = None
        if ctx.grad_reduce is not None and P > 0:
            # the per-Gaussian gradients' sums over ranks, range by range as the backward finishes them
            shared = [grads[k] for k in (4, 5, 6, 7, 8, 9, 10, 12)]
            ctx.grad_reduce.launch(shared, P, events if P > 0 else None)
        _C.host_mark("bwd_host", t0)
        return tuple(grads)


def rasterize_views(settings_list, means3D, means2D_list, opacities, shs=None, colors_precomp=None, scales=None,
                    rotations=None, cov3D_precomp=None, background=None, colors2=None, grad_reduce=None,
                    two_color_backward="fused", clamp=False):
    """Render V views of one set of Gaussians.  settings_list: V GaussianRasterizationSettings (same image
    size, same sh_degree, scale_modifier and prefiltered flag); means2D_list: V screen-space placeholders
    (P, 3) whose .grad receives each view's viewspace gradient.  Returns (color (V,3,H,W), radii (V,P),
    depth (V,1,H,W), alpha (V,1,H,W)).

    background: the background renderer's composite fused into the blends — the background network's
    images (V, H, W, 3) (renderer/diff_gaussian_rasterizer_background.py:116,129-132,139); the first
    output is then render = clamp(color + (1 - alpha) * background, 0, 1) (bit-identical to the torch
    expression, same gradients incl. the background's) instead of color.

    clamp=True without a background: the first output is the renderers' ``rendered_image.clamp(0, 1)``
    (e.g. renderer/diff_sugar_rasterizer_normal.py:212, renderer/diff_gaussian_rasterizer.py:141) formed in the
    blend kernels, its gradient mask in the backward's per-pixel prologue: the same bits as clamping the colour
    output in torch, without its four elementwise passes over the images.

    colors2 (P, 3): a second rasterizer call that differs only in its colours — the SuGaR normal renderer's
    ``rasterizer(..., means2D=zeros_like(means2D), shs=None, colors_precomp=pc.get_gs_normals, ...)``
    (renderer/diff_sugar_rasterizer_normal.py:182-191) — rendered from the same geometry, sorts and blend
    weights (include/gsr.h gsr_set_render_two_colors); a fifth output holds its colour image (V, 3, H, W).
    Its backward adds that call's parameter gradients (colors2 receives its colour gradient); its
    screen-space gradient is not added to means2D, as in the reference.

    grad_reduce (view_shard.ChunkedGradReduce): with torch.distributed initialised, the per-Gaussian
    parameter gradients are summed over ranks inside the backward, range by range as they are formed
    (overlapping the per-Gaussian backward); the screen-space and background gradients stay per rank.

    two_color_backward: "fused" (default) replays both calls of a colors2 forward in one backward pass;
    "separate" runs the second call's backward after the first's, as two rasterizer calls would (same
    gradients up to fp32 summation order; tests compare the two)."""
    if (shs is None) == (colors_precomp is None):
        raise Exception("Please provide excatly one of either SHs or precomputed colors!")
    if ((scales is None or rotations is None) and cov3D_precomp is None) or (
            (scales is not None or rotations is not None) and cov3D_precomp is not None):
        raise Exception("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
    if len(means2D_list) != len(settings_list):
        raise ValueError("one means2D placeholder per view")
    if not settings_list:
        raise ValueError("at least one view")
    s0 = settings_list[0]
    if any(int(s.sh_degree) != int(s0.sh_degree) or float(s.scale_modifier) != float(s0.scale_modifier)
           or bool(s.prefiltered) != bool(s0.prefiltered) for s in settings_list):
        raise ValueError("sh_degree, scale_modifier and prefiltered must be shared by the views of a batch")
    if background is not None:
        H, W = int(s0.image_height), int(s0.image_width)
        if background.numel() != len(settings_list) * H * W * 3:
            raise ValueError("background must hold (V, H, W, 3) values")
    if two_color_backward not in ("fused", "separate"):
        raise ValueError("two_color_backward is 'fused' or 'separate'")
    return _RasterizeViews.apply(list(settings_list), grad_reduce, two_color_backward, bool(clamp), means3D, shs,
                                 colors_precomp, opacities, scales, rotations, cov3D_precomp, background, colors2,
                                 *means2D_list)

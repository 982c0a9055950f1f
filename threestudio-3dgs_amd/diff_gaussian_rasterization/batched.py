"""View-batched rasterization: one set of Gaussians, V cameras, one autograd node.

Equivalent to calling GaussianRasterizer once per view (same kernels, same per-view outputs), but:
  * forward: all views' preprocess is enqueued first and the V instance counts are read back with ONE
    host sync (the per-view API syncs once per view, idling the GPU while the host catches up);
  * backward: each view's tile blend writes its gradient rows, then one fused per-Gaussian kernel walks
    up to 16 views per launch and sums the shared-parameter gradients (means3D, opacity, SH, scales,
    rotations) in registers — the parameters and SH rows are read once and the gradients written once,
    instead of once per view plus a per-view autograd accumulation of 192 MB SH gradients.
Per-view outputs (color, radii, depth, alpha) and per-view means2D gradients (the densification
statistic of geometry/gaussian_base.py:815-818) are kept.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _C

# device memory the backward may use at once for per-view gradient rows (views are processed in groups)
WORK_BUDGET = int(os.environ.get("GSR_BWD_WORK_BYTES", str(24 << 30)))
# HIP streams the views of a batch are dealt over (views are independent until the per-Gaussian
# backward): one view's latency-bound sort/scan launches and blend tails overlap another's bulk work
N_STREAMS = int(os.environ.get("GSR_STREAMS", "4"))

_side: dict = {}


class _Fork:
    """Deal per-view work over side streams that start after everything enqueued so far on the
    current stream; join() makes the current stream wait for all of them.  Buffers are allocated on
    the current stream before the fork and released on it after the join, so the caching allocator
    never hands a side stream memory that is still in use."""

    def __init__(self, dev, n_views):
        self.main = torch.cuda.current_stream(dev)
        n = max(1, min(N_STREAMS, n_views))
        pool = _side.setdefault(dev, [])
        while len(pool) < n:
            pool.append(torch.cuda.Stream(dev))
        self.streams = pool[:n] if n > 1 else [self.main]
        if n > 1:
            ev = self.main.record_event()
            for st in self.streams:
                st.wait_event(ev)

    def stream(self, v):
        return ctypes.c_void_p(self.streams[v % len(self.streams)].cuda_stream)

    def join(self):
        if self.streams[0] is not self.main:
            for st in self.streams:
                self.main.wait_event(st.record_event())


def _arr(ctype, values):
    return (ctype * len(values))(*values)


class _RasterizeViews(torch.autograd.Function):
    @staticmethod
    def forward(ctx, settings_list, means3D, sh, colors_precomp, opacities, scales, rotations, cov3D_precomp,
                *means2D):
        lib = _C.load_library()
        V = len(settings_list)
        dev = means3D.device
        _C._require_gpu(dev)
        P = int(means3D.shape[0])
        H, W = int(settings_list[0].image_height), int(settings_list[0].image_width)
        if any(int(s.image_height) != H or int(s.image_width) != W for s in settings_list):
            raise _C.GSRError("all views of a batch must have the same image size")
        f = lambda t, n: _C._f32(t, n, dev)  # noqa: E731
        m3, shc, col, op, sc, rot, c3 = (f(means3D, "means3D"), f(sh, "sh"), f(colors_precomp, "colors_precomp"),
                                         f(opacities, "opacities"), f(scales, "scales"), f(rotations, "rotations"),
                                         f(cov3D_precomp, "cov3D_precomp"))
        if (shc is None) == (col is None):
            raise Exception("Please provide excatly one of either SHs or precomputed colors!")
        M = _C.sh_coeff_count(shc)
        cams = [(f(s.viewmatrix, "viewmatrix"), f(s.projmatrix, "projmatrix"), f(s.campos, "campos"), f(s.bg, "bg"))
                for s in settings_list]
        fopt = dict(dtype=torch.float32, device=dev)
        color = torch.empty((V, 3, H, W), **fopt)
        depth = torch.empty((V, 1, H, W), **fopt)
        alpha = torch.empty((V, 1, H, W), **fopt)
        radii = torch.zeros((V, P), dtype=torch.int32, device=dev)
        stream = _C._stream(dev)
        p = _C._ptr
        geoms = []
        if P > 0:
            geoms = [torch.empty(int(lib.gsr_geom_bytes(P)), dtype=torch.uint8, device=dev) for _ in range(V)]
            fork = _Fork(dev, V)
            for v, s in enumerate(settings_list):
                view, proj, campos, _ = cams[v]
                _C._check(lib.gsr_forward_preprocess(
                    P, int(s.sh_degree), M, p(m3), p(sc), float(s.scale_modifier), p(rot), p(op), p(shc), p(col),
                    p(c3), p(view), p(proj), p(campos), W, H, float(s.tanfovx), float(s.tanfovy),
                    int(bool(s.prefiltered)), p(radii[v]), p(geoms[v]), fork.stream(v)))
            fork.join()
            Ks = (ctypes.c_int * V)()
            _C._check(lib.gsr_num_rendered_many(V, _arr(ctypes.c_void_p, [g.data_ptr() for g in geoms]), P, Ks,
                                                stream))
            Ks = [int(k) for k in Ks]
            if len(_C.RECENT_FORWARDS) < 4096:
                _C.RECENT_FORWARDS.extend((k, H, W) for k in Ks)
        else:
            color.zero_(), depth.zero_(), alpha.zero_()
            Ks = [0] * V
        binnings, images = [], []
        if P > 0:
            binnings = [torch.empty(int(lib.gsr_binning_bytes(Ks[v], W, H)), dtype=torch.uint8, device=dev)
                        for v in range(V)]
            images = [torch.empty(int(lib.gsr_image_bytes(W, H)), dtype=torch.uint8, device=dev) for _ in range(V)]
            fork = _Fork(dev, V)
            for v in range(V):
                _C._check(lib.gsr_forward_render(P, Ks[v], W, H, p(cams[v][3]), p(geoms[v]), p(binnings[v]),
                                                 p(images[v]), p(color[v]), p(depth[v]), p(alpha[v]), fork.stream(v)))
            fork.join()
        ctx.settings = settings_list
        ctx.Ks = Ks
        ctx.geoms, ctx.binnings, ctx.images = geoms, binnings, images
        ctx.cams = cams
        ctx.save_for_backward(m3, shc, col, sc, rot, c3, radii)
        ctx.mark_non_differentiable(radii)
        return color, radii, depth, alpha

    @staticmethod
    def backward(ctx, g_color, _g_radii, g_depth, g_alpha):
        lib = _C.load_library()
        m3, shc, col, sc, rot, c3, radii = ctx.saved_tensors
        settings = ctx.settings
        V = len(settings)
        dev = m3.device
        P = int(m3.shape[0])
        M = _C.sh_coeff_count(shc)
        H, W = int(settings[0].image_height), int(settings[0].image_width)
        fopt = dict(dtype=torch.float32, device=dev)
        d_m2 = torch.zeros((V, P, 3), **fopt)
        d_m3 = torch.zeros((P, 3), **fopt)
        d_op = torch.zeros((P, 1), **fopt)
        d_col = torch.zeros((P, 3), **fopt) if col is not None else None
        d_sh = torch.zeros((P, M, 3), **fopt) if shc is not None else None
        d_c3 = torch.zeros((P, 6), **fopt) if c3 is not None else None
        d_sc = torch.zeros((P, 3), **fopt) if c3 is None else None
        d_rot = torch.zeros((P, 4), **fopt) if c3 is None else None
        if P > 0:
            gc = g_color.float().contiguous()
            gd = g_depth.float().contiguous() if g_depth is not None else None
            ga = g_alpha.float().contiguous() if g_alpha is not None else None
            stream = _C._stream(dev)
            p = _C._ptr
            # group views so the gradient rows of one group fit the work budget
            sizes = [int(lib.gsr_backward_bytes(P, k)) for k in ctx.Ks]
            groups, cur, cur_b = [], [], 0
            for v in range(V):
                if cur and (cur_b + sizes[v] > WORK_BUDGET or len(cur) == 16):
                    groups.append(cur)
                    cur, cur_b = [], 0
                cur.append(v)
                cur_b += sizes[v]
            groups.append(cur)
            for gi, grp in enumerate(groups):
                works = [torch.empty(sizes[v], dtype=torch.uint8, device=dev) for v in grp]
                fork = _Fork(dev, len(grp))
                for j, v in enumerate(grp):
                    _C._check(lib.gsr_backward_render(
                        P, ctx.Ks[v], W, H, p(ctx.cams[v][3]), p(ctx.geoms[v]), p(ctx.binnings[v]), p(ctx.images[v]),
                        p(gc[v]), p(gd[v]) if gd is not None else None, p(ga[v]) if ga is not None else None,
                        p(works[j]), fork.stream(j)))
                fork.join()
                n = len(grp)
                vp = lambda xs: _arr(ctypes.c_void_p, [x.data_ptr() for x in xs])  # noqa: E731
                _C._check(lib.gsr_backward_gaussians_many(
                    n, P, int(settings[0].sh_degree), M, _arr(ctypes.c_int, [W] * n), _arr(ctypes.c_int, [H] * n),
                    _arr(ctypes.c_float, [float(settings[v].tanfovx) for v in grp]),
                    _arr(ctypes.c_float, [float(settings[v].tanfovy) for v in grp]),
                    vp([ctx.cams[v][0] for v in grp]), vp([ctx.cams[v][1] for v in grp]),
                    vp([ctx.cams[v][2] for v in grp]), vp([radii[v] for v in grp]), vp([ctx.geoms[v] for v in grp]),
                    vp([ctx.images[v] for v in grp]), vp(works), _arr(ctypes.c_int, [ctx.Ks[v] for v in grp]),
                    p(m3), p(sc), float(settings[0].scale_modifier), p(rot), p(shc), p(c3), vp([d_m2[v] for v in grp]),
                    p(d_col), p(d_op), p(d_m3), p(d_c3), p(d_sh), p(d_sc), p(d_rot), 1 if gi > 0 else 0, stream))
        grads = [None, d_m3, d_sh, d_col, d_op, d_sc, d_rot, d_c3] + [d_m2[v] for v in range(V)]
        for k, need in enumerate(ctx.needs_input_grad):
            if not need:
                grads[k] = None
        return tuple(grads)


def rasterize_views(settings_list, means3D, means2D_list, opacities, shs=None, colors_precomp=None, scales=None,
                    rotations=None, cov3D_precomp=None):
    """Render V views of one set of Gaussians.  settings_list: V GaussianRasterizationSettings (same image
    size, same sh_degree and scale_modifier); means2D_list: V screen-space placeholders (P, 3) whose .grad
    receives each view's viewspace gradient.  Returns (color (V,3,H,W), radii (V,P), depth (V,1,H,W),
    alpha (V,1,H,W))."""
    if (shs is None) == (colors_precomp is None):
        raise Exception("Please provide excatly one of either SHs or precomputed colors!")
    if ((scales is None or rotations is None) and cov3D_precomp is None) or (
            (scales is not None or rotations is not None) and cov3D_precomp is not None):
        raise Exception("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
    if len(means2D_list) != len(settings_list):
        raise ValueError("one means2D placeholder per view")
    s0 = settings_list[0]
    if any(int(s.sh_degree) != int(s0.sh_degree) or float(s.scale_modifier) != float(s0.scale_modifier)
           for s in settings_list):
        raise ValueError("sh_degree and scale_modifier must be shared by the views of a batch")
    return _RasterizeViews.apply(list(settings_list), means3D, shs, colors_precomp, opacities, scales, rotations,
                                 cov3D_precomp, *means2D_list)

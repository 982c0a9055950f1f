"""Fused shading / depth-normal epilogue (include/gsr.h gsr_shade_*, csrc/gsr_shading.hip).

The MVDream shading renderer follows each rasterizer call with the depth-to-normal, point-light material
and background composite in ~25 torch ops (renderer/diff_gaussian_rasterizer_shading.py:169-208 with
``Depth2Normal`` :22-51 and ``GaussianDiffuseWithPointLightMaterial.forward``
material/gaussian_material.py:41-104); the SuGaR normal renderer uses the depth-to-normal part
(renderer/diff_sugar_rasterizer_normal.py:170-197).  Here each is one HIP pass forward and one backward
over a set of views, with the same results and gradients (including the in-place ``detach`` of the
normal map and depth where ``alpha <= 0.99``):

    shade_views(color, depth, alpha, rays_o, rays_d, bg, light_positions, ...) -> (render, normal, depth)
        render = the shading renderer's ``render`` (clamped), normal = its ``normal`` map,
        depth = ``depth`` (gradient masked)
    depth_normal_views(depth, alpha, rays_o, rays_d) -> (normal_from_dist, normal_map_from_dist)
        SuGaR's ``raw_normal_from_dist`` and ``normal_from_dist`` outputs (both gradient masked)

Shapes: one view ``color (3, H, W)``, ``depth / alpha (1, H, W)``, ``rays_o / rays_d (H, W, 3)``,
``bg (H, W, 3)`` (the background network's output) or ``(3,)``, ``light_positions (3,)``; or the same
with a leading view dimension V.  Ambient / diffuse light colours and the shading mode are the
material's (its ``ambient_ratio`` / soft-shading choice is made by the caller, as in the reference).
"""
from __future__ import annotations

import ctypes

import torch

from . import _C

MATERIAL = 1
_MODES = {"diffuse": 0, "albedo": 1, "textureless": 2}


def _light_table(x, V):
    """Light colours as V x 3 floats: one (3,) colour for every view, or (V, 3) per view."""
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu().reshape(-1).tolist()
    else:
        x = [float(t) for row in x for t in (row if isinstance(row, (list, tuple)) else [row])]
    if len(x) == 3:
        x = x * V
    if len(x) != 3 * V:
        raise ValueError(f"light colours need 3 or 3 x {V} components, got {len(x)}")
    return tuple(float(t) for t in x)


def _mode_table(shading, V):
    modes = [shading] * V if isinstance(shading, str) else list(shading)
    if len(modes) != V:
        raise ValueError(f"{len(modes)} shading modes for {V} views")
    for m in modes:
        if m not in _MODES:
            raise ValueError(f"Unknown shading type {m}")
    return tuple(_MODES[m] for m in modes)


def _c(ctype, values):
    return (ctype * max(1, len(values)))(*values)


class _Shade(torch.autograd.Function):
    @staticmethod
    def forward(ctx, color, depth, alpha, rays_o, rays_d, bg, light, pred_normal, flags, modes, bg_layout, ka, kd):
        lib = _C.load_library()
        dev = depth.device
        _C._require_gpu(dev)
        V, _, H, W = depth.shape
        t = {}
        for name, x in (("color", color), ("depth", depth), ("alpha", alpha), ("rays_o", rays_o), ("rays_d", rays_d),
                        ("bg", bg), ("light", light), ("pred_normal", pred_normal)):
            t[name] = _C._f32(x, name, dev) if x is not None else None
        material = bool(flags & MATERIAL)
        new = lambda c: torch.empty((V, c, H, W), dtype=torch.float32, device=dev)  # noqa: E731
        render = new(3) if material else None
        nmap, depth_out = new(3), new(1)
        unit = None if material else new(3)
        _C._check(lib.gsr_shade_views_forward(
            V, H, W, flags, _c(ctypes.c_int, modes), _C._ptr(t["color"]), _C._ptr(t["depth"]), _C._ptr(t["alpha"]), _C._ptr(t["rays_o"]),
            _C._ptr(t["rays_d"]), _C._ptr(t["bg"]), bg_layout, _C._ptr(t["light"]), _C._ptr(t["pred_normal"]),
            _c(ctypes.c_float, ka), _c(ctypes.c_float, kd), _C._ptr(render), _C._ptr(nmap), _C._ptr(unit),
            _C._ptr(depth_out), _C._stream(dev)))
        ctx.meta = (flags, modes, bg_layout, ka, kd)
        ctx.save_for_backward(t["color"], t["depth"], t["alpha"], t["rays_o"], t["rays_d"], t["bg"], t["light"],
                              t["pred_normal"])
        if material:
            return render, nmap, depth_out
        return unit, nmap, depth_out

    @staticmethod
    def backward(ctx, g0, g_nmap, g_depth):
        lib = _C.load_library()
        color, depth, alpha, rays_o, rays_d, bg, light, pred_normal = ctx.saved_tensors
        flags, modes, bg_layout, ka, kd = ctx.meta
        material = bool(flags & MATERIAL)
        dev = depth.device
        V, _, H, W = depth.shape
        g = lambda x: None if x is None else x.float().contiguous()  # noqa: E731
        g_render, g_unit = (g(g0), None) if material else (None, g(g0))
        g_nmap, g_depth = g(g_nmap), g(g_depth)
        d_depth, d_alpha = torch.empty_like(depth), torch.empty_like(alpha)
        d_color = torch.empty_like(color) if material else None
        want_bg = material and ctx.needs_input_grad[5] and bg_layout == 1
        d_bg = torch.empty_like(bg) if want_bg else None
        _C._check(lib.gsr_shade_views_backward(
            V, H, W, flags, _c(ctypes.c_int, modes), _C._ptr(color), _C._ptr(depth), _C._ptr(alpha), _C._ptr(rays_o),
            _C._ptr(rays_d), _C._ptr(bg), bg_layout, _C._ptr(light), _C._ptr(pred_normal), _c(ctypes.c_float, ka),
            _c(ctypes.c_float, kd), _C._ptr(g_render), _C._ptr(g_nmap), _C._ptr(g_unit), _C._ptr(g_depth), _C._ptr(d_color),
            _C._ptr(d_depth), _C._ptr(d_alpha), _C._ptr(d_bg), _C._stream(dev)))
        if material and ctx.needs_input_grad[5] and bg_layout == 0:
            # constant background colour per view: sum over pixels of g (1 - alpha), masked by the clamp
            d_bg = _constant_bg_grad(ctx, g_render, color, depth, alpha, rays_o, rays_d, bg, light, pred_normal)
        return d_color, d_depth, d_alpha, None, None, d_bg, None, None, None, None, None, None, None


def _constant_bg_grad(ctx, g_render, color, depth, alpha, rays_o, rays_d, bg, light, pred_normal):
    """dL/dbg for a constant background colour: sum_p g (1 - alpha) [0 <= img <= 1].  The HIP backward
    forms the per-pixel image gradient for an HWC background; a broadcast one is formed as an expanded
    HWC image and summed (a rare path: the reference passes the background network's image)."""
    lib = _C.load_library()
    flags, modes, _, ka, kd = ctx.meta
    V, _, H, W = depth.shape
    dev = depth.device
    bg_img = bg.view(V, 1, 1, 3).expand(V, H, W, 3).contiguous()
    d_bg = torch.empty_like(bg_img)
    scratch = [torch.empty_like(depth), torch.empty_like(alpha), torch.empty_like(color)]
    _C._check(lib.gsr_shade_views_backward(
        V, H, W, flags, _c(ctypes.c_int, modes), _C._ptr(color), _C._ptr(depth), _C._ptr(alpha), _C._ptr(rays_o),
        _C._ptr(rays_d), _C._ptr(bg_img), 1, _C._ptr(light), _C._ptr(pred_normal), _c(ctypes.c_float, ka),
        _c(ctypes.c_float, kd), _C._ptr(g_render),
        None, None, None, _C._ptr(scratch[2]), _C._ptr(scratch[0]), _C._ptr(scratch[1]), _C._ptr(d_bg),
        _C._stream(dev)))
    return d_bg.sum(dim=(1, 2))


def _views(x, dims):
    """Add the view dimension to a single-view tensor."""
    return x.unsqueeze(0) if x is not None and x.dim() == dims else x


def shade_views(color, depth, alpha, rays_o, rays_d, bg, light_positions, ambient=(0.1, 0.1, 0.1),
                diffuse=(0.9, 0.9, 0.9), shading="diffuse", pred_normal=None):
    """The shading renderer's post-raster epilogue (renderer/diff_gaussian_rasterizer_shading.py:169-208)
    for one view or V views.  Returns ``(render, normal, depth)`` = the renderer's ``render``
    (``clamp(0, 1)`` applied), ``normal`` map and ``depth`` outputs.  ``pred_normal`` is the rasterized
    predicted-normal image when ``pc.cfg.pred_normal`` (used detached, as in the reference).
    ``ambient`` / ``diffuse`` are one (3,) light colour or (V, 3) per view, ``shading`` one mode or a
    sequence of V modes: the material draws them per view (material/gaussian_material.py:59-64,80-88)."""
    single = depth.dim() == 3
    color, depth, alpha = _views(color, 3), _views(depth, 3), _views(alpha, 3)
    rays_o, rays_d = _views(rays_o, 3), _views(rays_d, 3)
    pred_normal = _views(pred_normal.detach(), 3) if pred_normal is not None else None
    V, _, H, W = depth.shape
    if bg.dim() <= 2 and bg.shape[-1] == 3 and bg.numel() in (3, 3 * V):
        bg_layout, bg = 0, bg.reshape(-1, 3).expand(V, 3)
    else:
        bg_layout, bg = 1, bg.reshape(-1, H, W, 3).expand(V, H, W, 3)
    light = light_positions.reshape(-1, 3).expand(V, 3)
    rays_o, rays_d = rays_o.expand(V, H, W, 3), rays_d.expand(V, H, W, 3)
    out = _Shade.apply(color, depth, alpha, rays_o, rays_d, bg, light, pred_normal, MATERIAL, _mode_table(shading, V),
                       bg_layout, _light_table(ambient, V), _light_table(diffuse, V))
    return tuple(o[0] for o in out) if single else out


def depth_normal_views(depth, alpha, rays_o, rays_d):
    """SuGaR's normal-from-distance maps (renderer/diff_sugar_rasterizer_normal.py:170-177,196-197) for
    one view or V views: ``(normal_from_dist, normal_map_from_dist)`` with the gradient of both kept
    only where ``alpha > 0.99``."""
    single = depth.dim() == 3
    depth, alpha = _views(depth, 3), _views(alpha, 3)
    V, _, H, W = depth.shape
    rays_o, rays_d = _views(rays_o, 3).expand(V, H, W, 3), _views(rays_d, 3).expand(V, H, W, 3)
    unit, nmap, _ = _Shade.apply(None, depth, alpha, rays_o, rays_d, None, None, None, 0, (), 0, (), ())
    return (unit[0], nmap[0]) if single else (unit, nmap)


def depth_normal_maps(depth, alpha, rays_o, rays_d):
    """The normal renderer's depth-to-normal epilogue (renderer/diff_gaussian_rasterizer_normal.py:172-193)
    for V views: ``(normal, depth)`` = its ``normal`` output (``u * 0.5 * alpha + 0.5`` of the unit
    Depth2Normal normal) and its ``depth`` output, both with the gradient kept only where ``alpha > 0.99``."""
    single = depth.dim() == 3
    depth, alpha = _views(depth, 3), _views(alpha, 3)
    V, _, H, W = depth.shape
    rays_o, rays_d = _views(rays_o, 3).expand(V, H, W, 3), _views(rays_d, 3).expand(V, H, W, 3)
    _, nmap, depth_out = _Shade.apply(None, depth, alpha, rays_o, rays_d, None, None, None, 0, (), 0, (), ())
    return (nmap[0], depth_out[0]) if single else (nmap, depth_out)


class _NormalMap(torch.autograd.Function):
    @staticmethod
    def forward(ctx, normal, alpha):
        lib = _C.load_library()
        dev = normal.device
        _C._require_gpu(dev)
        V, _, H, W = normal.shape
        n = _C._f32(normal, "normal", dev)
        a = _C._f32(alpha, "alpha", dev)
        out = torch.empty((V, 3, H, W), dtype=torch.float32, device=dev)
        _C._check(lib.gsr_normal_map_forward(V, H, W, _C._ptr(n), _C._ptr(a), _C._ptr(out), _C._stream(dev)))
        ctx.save_for_backward(n, a)
        return out

    @staticmethod
    def backward(ctx, g_out):
        lib = _C.load_library()
        n, a = ctx.saved_tensors
        V, _, H, W = n.shape
        dev = n.device
        g = g_out.float().contiguous()
        dn = torch.empty_like(n)
        da = torch.empty_like(a)
        _C._check(lib.gsr_normal_map_backward(V, H, W, _C._ptr(g), _C._ptr(n), _C._ptr(a), _C._ptr(dn), _C._ptr(da),
                                              _C._stream(dev)))
        return dn, da


def sugar_normal_map(normal, alpha):
    """The SuGaR normal renderer's normal map from its second rasterizer call (face normals blended):
    ``F.normalize(normal)``, x / y negated (p3d -> threestudio axes), ``normal * 0.5 * alpha + 0.5``, with the
    gradient kept only where ``alpha > 0.99`` (renderer/diff_sugar_rasterizer_normal.py:192-197) — one HIP pass
    each way.  normal (3, H, W) or (V, 3, H, W), alpha (1, H, W) or (V, 1, H, W)."""
    single = normal.dim() == 3
    if single:
        normal, alpha = normal.unsqueeze(0), alpha.unsqueeze(0)
    out = _NormalMap.apply(normal, alpha)
    return out[0] if single else out


def sugar_shade_views(color, depth, alpha, normal, rays_o, rays_d, bg, light_positions, ambient, diffuse, shading):
    """The SuGaR shading renderer's epilogue over a view set (renderer/diff_sugar_rasterizer_shading.py:170-213):
    positions X = rays_o + depth rays_d; shading normal = F.normalize of the second call's blended face normals
    (differentiated: the material's gradient reaches the normals, unlike the MVDream renderer's detached
    predicted normal, so this is not the HIP shading pass); the point-light material of
    material/gaussian_material.py:41-104 with the view's drawn (ka, kd, shading); the composite
    ``fg alpha + (1 - alpha) bg``; the normal map ``n 0.5 alpha + 0.5`` and depth, detached where alpha <= 0.99.
    Batched torch ops over the views (one call per set instead of the reference's ~30 per view).
    color / normal (V, 3, H, W), depth / alpha (V, 1, H, W), rays (V, H, W, 3), bg (V, H, W, 3), light (V, 3);
    ambient / diffuse: V triples, shading: V of "diffuse" | "albedo" | "textureless".
    Returns render clamped to [0, 1] (V, 3, H, W), normal map (V, 3, H, W), depth (V, 1, H, W)."""
    import torch.nn.functional as F

    V = depth.shape[0]
    dt, dev = depth.dtype, depth.device
    xyz = rays_o + depth.permute(0, 2, 3, 1) * rays_d
    nrm = F.normalize(normal, dim=1)
    s = nrm.permute(0, 2, 3, 1)
    albedo = (color / (alpha + 1e-6)).permute(0, 2, 3, 1)
    lp = light_positions.reshape(V, 1, 1, 3)
    ka = torch.tensor(ambient, dtype=dt, device=dev).reshape(V, 1, 1, 3)
    kd = torch.tensor(diffuse, dtype=dt, device=dev).reshape(V, 1, 1, 3)
    light_dir = F.normalize(lp - xyz, dim=-1)
    diffuse_light = torch.sum(s * light_dir, -1, keepdim=True).clamp(min=0.0) * kd
    textureless = diffuse_light + ka
    shaded = albedo.clamp(0.0, 1.0) * textureless
    # per view, the material's return for its shading mode ("+ x * 0" as the material writes it)
    outs = {"albedo": albedo + textureless * 0, "textureless": albedo * 0 + textureless, "diffuse": shaded}
    for m in set(shading):
        if m not in outs:
            raise ValueError(f"Unknown shading type {m}")
    sel = [torch.tensor([m == k for m in shading], device=dev).reshape(V, 1, 1, 1) for k in ("albedo", "textureless")]
    fg = torch.where(sel[0], outs["albedo"], torch.where(sel[1], outs["textureless"], outs["diffuse"]))
    render = fg.permute(0, 3, 1, 2) * alpha + (1 - alpha) * bg.permute(0, 3, 1, 2)
    nmap = nrm * 0.5 * alpha + 0.5
    mask = alpha > 0.99
    nmap = torch.where(mask.expand_as(nmap), nmap, nmap.detach())
    depth_m = torch.where(mask, depth, depth.detach())
    return render.clamp(0, 1), nmap, depth_m

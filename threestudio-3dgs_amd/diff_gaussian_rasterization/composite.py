"""Fused background composite: the background renderer's post-raster epilogue as one HIP pass.

The reference composites the rasterizer's image with the background network's output and clamps
(renderer/diff_gaussian_rasterizer_background.py:129-132 and the ``.clamp(0, 1)`` of :139):

    rendered_image = rendered_image + (1 - rendered_alpha) * comp_rgb_bg.reshape(H, W, 3).permute(2, 0, 1)
    render = rendered_image.clamp(0, 1)

``composite_background(color, alpha, bg)`` returns the same tensor (bit-identical forward) with the
same gradients for color, alpha and bg, in one kernel each way (include/gsr.h gsr_composite_*)
instead of torch's four elementwise passes forward and five backward.
"""
from __future__ import annotations

import torch

from . import _C

_LAYOUTS = {"constant": 0, "hwc": 1, "chw": 2}


class _Composite(torch.autograd.Function):
    @staticmethod
    def forward(ctx, color, alpha, bg, layout):
        lib = _C.load_library()
        dev = color.device
        _C._require_gpu(dev)
        V, _, H, W = color.shape
        c = _C._f32(color, "color", dev)
        a = _C._f32(alpha, "alpha", dev)
        b = _C._f32(bg, "bg", dev)
        out = torch.empty((V, 3, H, W), dtype=torch.float32, device=dev)
        _C._check(lib.gsr_composite_forward(V, H, W, _C._ptr(c), _C._ptr(a), _C._ptr(b), layout, _C._ptr(out),
                                            _C._stream(dev)))
        ctx.layout = layout
        ctx.save_for_backward(c, a, b)
        return out

    @staticmethod
    def backward(ctx, g_out):
        lib = _C.load_library()
        c, a, b = ctx.saved_tensors
        V, _, H, W = c.shape
        dev = c.device
        g = g_out.float().contiguous()
        d_c = torch.empty_like(c)
        d_a = torch.empty_like(a)
        want_bg = ctx.needs_input_grad[2] and ctx.layout != 0
        d_b = torch.empty_like(b) if want_bg else None
        _C._check(lib.gsr_composite_backward(V, H, W, _C._ptr(g), _C._ptr(c), _C._ptr(a), _C._ptr(b), ctx.layout,
                                             _C._ptr(d_c), _C._ptr(d_a), _C._ptr(d_b), _C._stream(dev)))
        if ctx.needs_input_grad[2] and ctx.layout == 0:
            # constant background: dL/dbg = sum over pixels of g (1 - alpha), masked like the image layouts
            pre = c + (1 - a) * b.view(V, 3, 1, 1)
            m = ((pre >= 0) & (pre <= 1)).to(g.dtype)
            d_b = (g * m * (1 - a)).sum(dim=(2, 3))
        return d_c, d_a, d_b, None


def composite_background(color, alpha, bg, bg_layout: str | None = None):
    """clamp(color + (1 - alpha) * bg, 0, 1) with color (3, H, W) or (V, 3, H, W), alpha (1, H, W) or
    (V, 1, H, W) and bg either the background network's image, (H, W, 3) / (V, H, W, 3) ("hwc", the
    reference's layout) or (3, H, W) / (V, 3, H, W) ("chw"), or a constant colour (3,) / (V, 3)."""
    single = color.dim() == 3
    if single:
        color, alpha = color.unsqueeze(0), alpha.unsqueeze(0)
    V, _, H, W = color.shape
    if bg_layout is None:
        if bg.dim() <= 2:
            bg_layout = "constant"
        elif bg.shape[-1] == 3 and tuple(bg.shape[-3:-1]) == (H, W):
            bg_layout = "hwc"
        else:
            bg_layout = "chw"
    layout = _LAYOUTS[bg_layout]
    if layout == 0:
        bg = bg.reshape(-1, 3).expand(V, 3)
    elif layout == 1:
        bg = bg.reshape(-1, H, W, 3).expand(V, H, W, 3)
    else:
        bg = bg.reshape(-1, 3, H, W).expand(V, 3, H, W)
    out = _Composite.apply(color, alpha, bg, layout)
    return out[0] if single else out

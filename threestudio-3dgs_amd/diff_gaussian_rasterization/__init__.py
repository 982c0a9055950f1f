"""MI355X-native drop-in for the ``diff_gaussian_rasterization`` package.

The reference (lizhiqi49/threestudio-3dgs) imports, in 9 renderer files,

    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer

(e.g. renderer/diff_gaussian_rasterizer.py:8-11) and calls ``GaussianRasterizer(raster_settings=...)``
with keyword arguments ``means3D, means2D, shs, colors_precomp, opacities, scales, rotations,
cov3D_precomp`` (renderer/diff_gaussian_rasterizer.py:122-131), unpacking the ashawkey 4-output
tuple ``(color, radii, depth, alpha)`` (renderer/diff_gaussian_rasterizer_advanced.py:122).
This package keeps that API — names, argument meaning, exceptions — over hand-written gfx950
kernels reached through the C ABI in include/gsr.h (see _C.py).  The wrappers run unchanged.
"""
from __future__ import annotations

from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C

__all__ = [
    "GaussianRasterizationSettings",
    "GaussianRasterizer",
    "rasterize_gaussians",
    "cpu_deep_copy_tuple",
]


def cpu_deep_copy_tuple(input_tuple):
    """Debug helper of the reference package: copy tensors of a tuple to the CPU."""
    return tuple(item.cpu().clone() if isinstance(item, torch.Tensor) else item for item in input_tuple)


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings)


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings):
        s = raster_settings
        num_rendered, color, depth, alpha, radii, geom, binning, image = _C.rasterize_gaussians(
            s.bg, means3D, colors_precomp, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp,
            s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width, sh, s.sh_degree,
            s.campos, s.prefiltered, s.debug)
        ctx.raster_settings = s
        ctx.num_rendered = num_rendered
        # saved buffers are never written by the backward -> repeated backward (retain_graph) is safe
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geom,
                              binning, image, alpha)
        ctx.mark_non_differentiable(radii)
        return color, radii, depth, alpha

    @staticmethod
    def backward(ctx, grad_out_color, _grad_radii, grad_out_depth, grad_out_alpha):
        s = ctx.raster_settings
        (colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geom, binning, image,
         alpha) = ctx.saved_tensors
        (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_sh,
         grad_scales, grad_rotations) = _C.rasterize_gaussians_backward(
            s.bg, means3D, radii, colors_precomp, scales, rotations, s.scale_modifier, cov3Ds_precomp,
            s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, grad_out_color, grad_out_depth, grad_out_alpha,
            sh, s.sh_degree, s.campos, geom, ctx.num_rendered, binning, image, alpha, s.debug)
        grads = [grad_means3D, grad_means2D, grad_sh, grad_colors_precomp, grad_opacities, grad_scales,
                 grad_rotations, grad_cov3Ds_precomp, None]
        # inputs that arrived as empty placeholders get no gradient
        for k, need in enumerate(ctx.needs_input_grad[:8]):
            if not need:
                grads[k] = None
        return tuple(grads)


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        # frustum mask of the points (view z > 0.2); API completeness, unused by the reference
        with torch.no_grad():
            s = self.raster_settings
            visible = _C.mark_visible(positions, s.viewmatrix, s.projmatrix)
        return visible

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None):
        s = self.raster_settings
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception("Please provide excatly one of either SHs or precomputed colors!")
        if ((scales is None or rotations is None) and cov3D_precomp is None) or (
                (scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
        empty = torch.Tensor([])
        if shs is None:
            shs = empty
        if colors_precomp is None:
            colors_precomp = empty
        if scales is None:
            scales = empty
        if rotations is None:
            rotations = empty
        if cov3D_precomp is None:
            cov3D_precomp = empty
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales, rotations,
                                   cov3D_precomp, s)

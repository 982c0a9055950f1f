"""Drop-in ``GaussianBatchRenderer`` on the view-set path.

The reference renders a batch with a serial Python loop (renderer/gaussian_batch_renderer.py:9-76): per
view it builds the camera (``get_cam_info_gaussian`` + ``Camera``, :22-49), calls the renderer's
``forward`` (one rasterizer call, one host sync and ~30 launches per view), then stacks the per-view
outputs into the batch dict (:78-121).  This mixin keeps that contract — same input batch dict
(``c2w``, ``fovy``, ``height``, ``width``, ``rays_o``, ``rays_d``, ``light_positions``,
``override_color``), same output keys (``comp_rgb``, ``comp_depth``, ``comp_mask``, ``comp_normal``,
``comp_normal_from_dist``, ``comp_pred_normal``, ``comp_rgb_bg`` as (B, H, W, C), and the per-view
lists ``viewspace_points``, ``visibility_filter``, ``radii``) — but renders the whole batch with one
``rasterize_views`` call (every kernel stage is one launch per set of up to 64 views) followed by the
renderer's epilogue fused on the GPU:

    "plain"         renderer/diff_gaussian_rasterizer.py:45-145          bg (randomly inverted), clamp
    "background"    renderer/diff_gaussian_rasterizer_background.py:44-145  bg = 0, background network
                                                                         composite + clamp fused into the blends
    "advanced"      renderer/diff_gaussian_rasterizer_advanced.py:45-146 bg (randomly inverted), clamp,
                                                                         depth and alpha outputs
    "shading"       renderer/diff_gaussian_rasterizer_shading.py:79-231  Depth2Normal + point-light
                                                                         material + composite (gsr_shade_*)
    "normal"        renderer/diff_gaussian_rasterizer_normal.py:79-210   bg (randomly inverted), clamp,
                                                                         Depth2Normal map + masked depth
    "sugar_normal"  renderer/diff_sugar_rasterizer_normal.py:80-223      two passes (colours, face normals)
                                                                         + normal-from-distance (gsr_shade_*)
    "sugar_shading" renderer/diff_sugar_rasterizer_shading.py:80-224     two passes (colours, face normals) +
                                                                         point-light material on the blended
                                                                         normals + composite (batched torch)

The mode comes from the renderer's ``batch_render_mode`` attribute or, when unset, from the module the
renderer class is defined in (the reference's file names above).  Any other renderer (st, temporal) keeps the
reference's per-view loop, still on the HIP rasterizer.

With ``torch.distributed`` initialised, every rank renders its contiguous slice of the batch
(view_shard.shard_range) and the image outputs are all-gathered (RCCL over xGMI); the per-view lists
hold the rank's own views and ``view_range`` says which.  Ranks with no view (batch < world) still take
part in every gather with empty slices, so the collectives always match.

Randomness follows the reference's per-view loop draw for draw: the background inversion
(``np.random.rand()`` per view, renderer/diff_gaussian_rasterizer.py:59-64) and the material's soft-shading
ambient ratio and shading mode (``random.random()`` per view, material/gaussian_material.py:59-64,80-88,
called once per view by renderer/diff_gaussian_rasterizer_shading.py:200-205) are drawn for every view of
the batch in view order — also on a rank that renders only some of them, so the draws consumed and the
values each view gets are those of the single-process reference whatever the world size — and the fused
shading epilogue takes one (ambient, diffuse, mode) per view.
"""
from __future__ import annotations

import math
import random
from typing import NamedTuple

import numpy as np
import torch

from .cameras import get_cam_info_gaussian
from . import view_shard
from .view_shard import _world, all_gather_views, shard_range

MODES = ("plain", "background", "advanced", "shading", "normal", "sugar_normal", "sugar_shading")
_MODULE_MODES = {
    "diff_gaussian_rasterizer": "plain",
    "diff_gaussian_rasterizer_background": "background",
    "diff_gaussian_rasterizer_advanced": "advanced",
    "diff_gaussian_rasterizer_shading": "shading",
    "diff_gaussian_rasterizer_normal": "normal",
    "diff_sugar_rasterizer_normal": "sugar_normal",
    "diff_sugar_rasterizer_shading": "sugar_shading",
}
# modes whose renderer draws a background inversion per view / calls the material per view
_INVERT_BG = ("plain", "advanced", "normal", "sugar_normal")
_MATERIAL = ("shading", "sugar_shading")
# modes whose second rasterizer call blends the face normals (the second colour set of one call)
_TWO_COLOR = ("sugar_normal", "sugar_shading")
# batch dict image keys of the reference (renderer/gaussian_batch_renderer.py:78-121) -> channels
_OUT_KEYS = (("comp_rgb", 3), ("comp_normal", 3), ("comp_normal_from_dist", 3), ("comp_pred_normal", 3),
             ("comp_depth", 1), ("comp_mask", 1))


class Camera(NamedTuple):
    """geometry/gaussian_base.py:175-184 (A15), for the per-view fallback loop."""
    FoVx: torch.Tensor
    FoVy: torch.Tensor
    camera_center: torch.Tensor
    image_width: int
    image_height: int
    world_view_transform: torch.Tensor
    full_proj_transform: torch.Tensor
    timestamp: torch.Tensor = None
    frame_idx: torch.Tensor = None


def batch_mode(renderer):
    """The fused path for `renderer` (one of MODES), or None for the reference's per-view loop."""
    mode = getattr(renderer, "batch_render_mode", None)
    if mode is not None:
        if mode not in MODES and mode != "per_view":
            raise ValueError(f"unknown batch_render_mode {mode!r}")
        return None if mode == "per_view" else mode
    return _MODULE_MODES.get(type(renderer).__module__.rsplit(".", 1)[-1])


def _rasterize_views(*args, **kwargs):
    from .batched import rasterize_views

    return rasterize_views(*args, **kwargs)


def _shade_views(*args, **kwargs):
    from .shading import shade_views

    return shade_views(*args, **kwargs)


def _depth_normal_views(*args, **kwargs):
    from .shading import depth_normal_views

    return depth_normal_views(*args, **kwargs)


def _sugar_shade_views(*args, **kwargs):
    from .shading import sugar_shade_views

    return sugar_shade_views(*args, **kwargs)


def _sugar_normal_map(*args, **kwargs):
    from .shading import sugar_normal_map

    return sugar_normal_map(*args, **kwargs)


def _depth_normal_maps(*args, **kwargs):
    from .shading import depth_normal_maps

    return depth_normal_maps(*args, **kwargs)


def material_params(material, training: bool):
    """The point-light material's light colours and shading mode for one view
    (material/gaussian_material.py:52-96 with ambient_ratio = shading = None, as the shading renderer calls
    it once per view): the same random draws, in the same order."""
    cfg = material.cfg
    if training and cfg.soft_shading:
        kd = random.random()
        ka, kd = (1.0 - kd,) * 3, (kd,) * 3
    else:
        ka = tuple(float(x) for x in material.ambient_light_color.reshape(-1))
        kd = tuple(float(x) for x in material.diffuse_light_color.reshape(-1))
    if training:
        if material.ambient_only or random.random() > cfg.diffuse_prob:
            mode = "albedo"
        elif random.random() < cfg.textureless_prob:
            mode = "textureless"
        else:
            mode = "diffuse"
    else:
        mode = "albedo" if material.ambient_only else "diffuse"
    return ka, kd, mode


def _settings(pc, cams, bgs, H, W, scaling_modifier):
    from . import GaussianRasterizationSettings

    w2c, proj, campos, fovs = cams
    return [GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=math.tan(f * 0.5),
                                          tanfovy=math.tan(f * 0.5), bg=bgs[v], scale_modifier=scaling_modifier,
                                          viewmatrix=w2c[v], projmatrix=proj[v], sh_degree=pc.active_sh_degree,
                                          campos=campos[v], prefiltered=False, debug=False)
            for v, f in enumerate(fovs)]


def _inverted_bgs(renderer, n):
    """Per-view background colour of the plain / advanced / normal / SuGaR renderers: inverted unless a draw
    keeps it (renderer/diff_gaussian_rasterizer.py:59-64, renderer/diff_sugar_rasterizer_normal.py:94-99)."""
    bg = renderer.background_tensor
    out = []
    for _ in range(n):
        invert = (np.random.rand() > renderer.cfg.invert_bg_prob) if renderer.training else True
        out.append(1.0 - bg if invert else bg)
    return out


def batch_draws(renderer, mode: str, bs: int) -> dict:
    """The random draws the reference's per-view loop makes for a batch of `bs` views, in view order:
    "bgs" (per-view background colour) for the modes that invert it, "lights" (per-view (ka, kd, shading))
    for the modes that call the material.  Every rank makes all of them and keeps its slice."""
    out = {}
    if mode in _INVERT_BG:
        out["bgs"] = _inverted_bgs(renderer, bs)
    if mode in _MATERIAL:
        out["lights"] = [material_params(renderer.material, renderer.training) for _ in range(bs)]
    return out


def view_camera(batch: dict, batch_idx: int):
    """The per-view camera of the reference's loop (renderer/gaussian_batch_renderer.py:22-49), including the
    optional timestamp / frame index the temporal and spacetime renderers read."""
    fovy = batch["fovy"][batch_idx]
    w2c, proj, cam_p = get_cam_info_gaussian(c2w=batch["c2w"][batch_idx], fovx=fovy, fovy=fovy, znear=0.1, zfar=100)
    dev = batch["c2w"].device
    return Camera(FoVx=fovy, FoVy=fovy, image_width=batch["width"], image_height=batch["height"],
                  world_view_transform=w2c.to(dev), full_proj_transform=proj.to(dev), camera_center=cam_p.to(dev),
                  timestamp=batch["timestamp"][batch_idx] if "timestamp" in batch else None,
                  frame_idx=batch["frame_indices"][batch_idx] if "frame_indices" in batch else None)


def render_view_reference(renderer, batch: dict, batch_idx: int) -> dict:
    """One iteration of the reference's loop: camera, then the renderer's forward in fp32 (autocast off,
    renderer/gaussian_batch_renderer.py:51-54)."""
    batch["batch_idx"] = batch_idx
    cam = view_camera(batch, batch_idx)
    with torch.autocast(device_type=batch["c2w"].device.type, enabled=False):
        return renderer.forward(cam, renderer.background_tensor, **batch)


def _placeholders(P, n, dev, dtype):
    """One screen-space placeholder per view (renderer/diff_gaussian_rasterizer.py:67-77): leaves whose
    .grad is the view's viewspace gradient.  Their values are zeros and never read, so each is one zero
    broadcast to (P, 3) (no (n, P, 3) fill; .grad is a dense (P, 3) tensor as for the reference's zeros)."""
    zero = torch.zeros((1, 1), device=dev, dtype=dtype)
    return [zero.expand(P, 3).requires_grad_(True) for _ in range(n)]


def _has_pred_normal(pc, mode: str) -> bool:
    return mode in ("shading", "normal") and bool(getattr(pc.cfg, "pred_normal", False))


def _active_reduce(renderer):
    reduce = getattr(renderer, "grad_reduce", None)
    return reduce if reduce is not None and reduce.active() else None


def _reduce_tensors(pc, mode, override, means3D, shs, common, normals):
    """(name, tensor) pairs whose gradients the renderer's reduction sums over ranks, in the order the
    reducing call lists them: the rasterizer's inputs (means3D, shs, colors_precomp, opacities, scales,
    rotations, colors2; batched._RasterizeViews.backward) for one call, plus the normals of the
    predicted-normal call when that reduction runs once after both calls.  Only tensors requiring grad."""
    pairs = [("means3D", means3D), ("shs", shs), ("override", override), ("opacities", common["opacities"]),
             ("scales", common["scales"]), ("rotations", common["rotations"])]
    if mode in _TWO_COLOR:
        pairs.append(("colors2", pc.get_gs_normals))
    if normals is not None:
        pairs.append(("normals", normals))
    return [(k, t) for k, t in pairs if t is not None and t.requires_grad]


def _join_reduce(renderer, batch: dict, mode: str, shapes):
    """A rank without views: empty outputs of `shapes` joining the reduction the other ranks' rasterizer
    backward issues (view_shard.join_grad_reduce), with the tensors that call differentiates."""
    pc = renderer.geometry
    override = batch.get("override_color")
    common = dict(opacities=pc.get_opacity, scales=pc.get_scaling, rotations=pc.get_rotation)
    normals = pc.get_normal if _has_pred_normal(pc, mode) else None
    pairs = _reduce_tensors(pc, mode, override, pc.get_xyz, pc.get_features if override is None else None, common,
                            normals)
    return view_shard.join_grad_reduce(_active_reduce(renderer), [t for _, t in pairs], shapes)


def render_views_local(renderer, batch: dict, mode: str, lo: int, hi: int, draws: dict | None = None) -> dict:
    """Render views [lo, hi) of the batch with the fused path of `mode`.  Returns per-view stacked images
    (n, C, H, W) under the batch dict's keys, plus the per-view lists.  `draws`: batch_draws of the whole
    batch (made here for [lo, hi) only when not given)."""
    pc = renderer.geometry
    H, W = int(batch["height"]), int(batch["width"])
    means3D = pc.get_xyz
    dev, P = means3D.device, int(means3D.shape[0])
    n = hi - lo
    out = {"viewspace_points": [], "visibility_filter": [], "radii": []}
    if n <= 0:
        return out
    fovy = torch.as_tensor(batch["fovy"])[lo:hi].reshape(-1)
    w2c, proj, campos = get_cam_info_gaussian(batch["c2w"][lo:hi], fovy, fovy, znear=0.1, zfar=100)
    cams = (w2c.to(dev), proj.to(dev), campos.to(dev), [float(f) for f in fovy])
    scaling_modifier = float(batch.get("scaling_modifier", 1.0))
    override = batch.get("override_color")
    shs = pc.get_features if override is None else None
    if draws is None:
        draws = {k: [None] * lo + v for k, v in batch_draws(renderer, mode, n).items()}
    draws = {k: v[lo:hi] for k, v in draws.items()}
    m2 = _placeholders(P, n, dev, means3D.dtype)
    common = dict(opacities=pc.get_opacity, scales=pc.get_scaling, rotations=pc.get_rotation)
    normals = pc.get_normal if _has_pred_normal(pc, mode) else None
    reduce = _active_reduce(renderer)
    common_main = common
    if reduce is not None and normals is None:
        # the main call's per-Gaussian gradients summed over ranks inside its backward, range by range
        common_main = dict(common, grad_reduce=reduce)
    elif reduce is not None:
        # two rasterizer calls on the same parameters: one reduction of the gradients both accumulate, after
        # both backward passes (view-less ranks join it with the same tensors, render_batch)
        names, tensors = zip(*_reduce_tensors(pc, mode, override, means3D, shs, common, normals))
        red = dict(zip(names, view_shard.reduce_on_backward(reduce, list(tensors))))
        means3D, shs, override = red.get("means3D", means3D), red.get("shs", shs), red.get("override", override)
        normals = red.get("normals", normals)
        common = common_main = {k: red.get(k, v) for k, v in common.items()}

    def pred_normal_pass(settings):
        # the predicted-normal call (renderer/diff_gaussian_rasterizer_shading.py:177-187,
        # renderer/diff_gaussian_rasterizer_normal.py:175-185): same settings, SH = the geometry's normals
        # (degree 0 through M = 1), a fresh zero means2D per view
        zeros = [torch.zeros_like(m) for m in m2]
        pred, _, _, _ = _rasterize_views(settings, means3D, zeros, shs=normals.unsqueeze(1),
                                         colors_precomp=None, **common)
        return pred

    with torch.autocast(device_type=dev.type, enabled=False):
        if mode in ("plain", "advanced"):
            settings = _settings(pc, cams, draws["bgs"], H, W, scaling_modifier)
            # (the renderer's clamp(0, 1) formed in the blends)
            color, radii, depth, alpha = _rasterize_views(settings, means3D, m2, shs=shs, colors_precomp=override,
                                                          clamp=True, **common_main)
            out["comp_rgb"] = color
            if mode == "advanced":
                out.update(comp_depth=depth, comp_mask=alpha)
        elif mode == "normal":
            settings = _settings(pc, cams, draws["bgs"], H, W, scaling_modifier)
            color, radii, depth, alpha = _rasterize_views(settings, means3D, m2, shs=shs, colors_precomp=override,
                                                          clamp=True, **common_main)
            nmap, depth_m = _depth_normal_maps(depth, alpha, batch["rays_o"][lo:hi], batch["rays_d"][lo:hi])
            if getattr(pc.cfg, "pred_normal", False):
                out["comp_pred_normal"] = pred_normal_pass(settings)
            out.update(comp_rgb=color, comp_normal=nmap, comp_depth=depth_m, comp_mask=alpha)
        elif mode == "background":
            zero = [renderer.background_tensor * 0] * n
            settings = _settings(pc, cams, zero, H, W, scaling_modifier)
            bg_img = renderer.background(dirs=batch["rays_d"][lo:hi])
            render, radii, _, _ = _rasterize_views(settings, means3D, m2, shs=shs, colors_precomp=override,
                                                   background=bg_img.reshape(n, H, W, 3), **common_main)
            out["comp_rgb"] = render
        elif mode == "shading":
            zero = [renderer.background_tensor * 0] * n
            settings = _settings(pc, cams, zero, H, W, scaling_modifier)
            color, radii, depth, alpha = _rasterize_views(settings, means3D, m2, shs=shs, colors_precomp=override,
                                                          **common_main)
            rays_o, rays_d = batch["rays_o"][lo:hi], batch["rays_d"][lo:hi]
            if batch.get("override_bg_color") is not None:
                bg_img = batch["override_bg_color"].reshape(1, 1, 1, 3).expand(n, H, W, 3)
            else:
                bg_img = renderer.background(dirs=rays_d)
            pred = None
            if getattr(pc.cfg, "pred_normal", False):
                pred = pred_normal_pass(settings)
                out["comp_pred_normal"] = pred
            lights = draws["lights"]
            render, nmap, depth_m = _shade_views(color, depth, alpha, rays_o, rays_d, bg_img.reshape(n, H, W, 3),
                                                 batch["light_positions"][lo:hi], [x[0] for x in lights],
                                                 [x[1] for x in lights], [x[2] for x in lights], pred_normal=pred)
            out.update(comp_rgb=render, comp_normal=nmap, comp_depth=depth_m, comp_mask=alpha,
                       comp_rgb_bg=bg_img.reshape(n, H, W, 3))
        elif mode == "sugar_normal":
            settings = _settings(pc, cams, draws["bgs"], H, W, scaling_modifier)
            # both rasterizer calls of the renderer (:157-166 colours, :182-191 face normals with a zero
            # means2D) from one geometry, sort and blend: the normals are the second colour set
            color, radii, depth, alpha, normal = _rasterize_views(settings, means3D, m2, shs=shs,
                                                                  colors_precomp=override,
                                                                  colors2=pc.get_gs_normals, clamp=True,
                                                                  **common_main)
            if batch.get("compute_normal_from_dist", True):
                _, nmap_dist = _depth_normal_views(depth, alpha, batch["rays_o"][lo:hi], batch["rays_d"][lo:hi])
                out["comp_normal_from_dist"] = nmap_dist
            # normalize, p3d -> threestudio axes, alpha-weighted map, alpha > 0.99 gradient mask (:192-197)
            nmap = _sugar_normal_map(normal, alpha)
            mask = alpha > 0.99
            out.update(comp_rgb=color, comp_normal=nmap,
                       comp_depth=torch.where(mask, depth, depth.detach()), comp_mask=alpha)
        elif mode == "sugar_shading":
            zero = [renderer.background_tensor * 0] * n
            settings = _settings(pc, cams, zero, H, W, scaling_modifier)
            # the renderer's two calls (:158-167 colours or SH, :183-192 face normals with a zero means2D) from one
            # geometry, sort and blend
            color, radii, depth, alpha, normal = _rasterize_views(settings, means3D, m2, shs=shs,
                                                                  colors_precomp=override,
                                                                  colors2=pc.get_gs_normals, **common_main)
            rays_o, rays_d = batch["rays_o"][lo:hi], batch["rays_d"][lo:hi]
            if batch.get("override_bg_color") is not None:
                bg_img = batch["override_bg_color"].reshape(1, 1, 1, 3).expand(n, H, W, 3)
            else:
                bg_img = renderer.background(dirs=rays_d).reshape(n, H, W, 3)
            lights = draws["lights"]
            render, nmap, depth_m = _sugar_shade_views(color, depth, alpha, normal, rays_o, rays_d, bg_img,
                                                       batch["light_positions"][lo:hi], [x[0] for x in lights],
                                                       [x[1] for x in lights], [x[2] for x in lights])
            out.update(comp_rgb=render, comp_normal=nmap, comp_depth=depth_m, comp_mask=alpha, comp_rgb_bg=bg_img)
        else:
            raise ValueError(f"unknown mode {mode!r}")
    out["viewspace_points"] = m2
    out["radii"] = [radii[v] for v in range(n)]
    out["visibility_filter"] = [radii[v] > 0 for v in range(n)]
    return out


def _mode_keys(renderer, mode):
    keys = {"plain": ["comp_rgb"], "background": ["comp_rgb"], "advanced": ["comp_rgb", "comp_depth", "comp_mask"],
            "shading": ["comp_rgb", "comp_normal", "comp_depth", "comp_mask"],
            "normal": ["comp_rgb", "comp_normal", "comp_depth", "comp_mask"],
            "sugar_normal": ["comp_rgb", "comp_normal", "comp_depth", "comp_mask"],
            "sugar_shading": ["comp_rgb", "comp_normal", "comp_depth", "comp_mask"]}[mode]
    if mode in ("shading", "normal") and getattr(renderer.geometry.cfg, "pred_normal", False):
        keys.append("comp_pred_normal")
    return keys


def render_batch(renderer, batch: dict, mode: str, group=None, shard: bool = True) -> dict:
    """batch_forward of the fused path: this rank's slice of views, images gathered over ranks."""
    bs = int(batch["c2w"].shape[0])
    world, rank = _world() if shard else (1, 0)
    lo, hi = shard_range(bs, world, rank)
    local = render_views_local(renderer, batch, mode, lo, hi, draws=batch_draws(renderer, mode, bs))
    H, W = int(batch["height"]), int(batch["width"])
    dev, dtype = renderer.geometry.get_xyz.device, renderer.geometry.get_xyz.dtype
    keys = _mode_keys(renderer, mode)
    if mode == "sugar_normal" and batch.get("compute_normal_from_dist", True):
        keys.append("comp_normal_from_dist")
    outputs = {"viewspace_points": local["viewspace_points"], "visibility_filter": local["visibility_filter"],
               "radii": local["radii"]}
    if world > 1:
        outputs["view_range"] = (lo, hi)
    channels = dict(_OUT_KEYS)
    joined = {}
    if hi <= lo and world > 1 and _active_reduce(renderer) is not None:
        # the other ranks sum their gradients inside the rasterizer's backward: this rank's empty slices come
        # from a node whose backward joins those collectives with zeros (no deadlock, same replica gradients)
        joined = dict(zip(keys, _join_reduce(renderer, batch, mode, [(0, channels[k], H, W) for k in keys])))
    for key in keys:
        img = local.get(key, joined.get(key))
        if img is None:  # a rank without views: an empty slice of the agreed shape (a leaf, so that the
            # rank's loss still has a graph and its backward runs; its parameter gradients stay None and
            # view_shard.allreduce_grads contributes zeros for them)
            img = torch.empty((0, channels[key], H, W), device=dev, dtype=dtype, requires_grad=True)
        full = all_gather_views(img, bs, group) if world > 1 else img
        outputs[key] = full.permute(0, 2, 3, 1)
    if mode in _MATERIAL:
        bgl = local.get("comp_rgb_bg")
        if bgl is None:
            bgl = torch.empty((0, H, W, 3), device=dev, dtype=dtype)
        full = all_gather_views(bgl, bs, group) if world > 1 else bgl
        # torch.cat of the views' (1, H, W, 3) backgrounds, then the reference's permute(0, 2, 3, 1)
        # (renderer/gaussian_batch_renderer.py:116-120: a (B, W, 3, H) tensor, kept as the reference has it)
        outputs["comp_rgb_bg"] = full.permute(0, 2, 3, 1)
    return outputs


def reference_batch_forward(renderer, batch: dict) -> dict:
    """The reference's per-view loop (renderer/gaussian_batch_renderer.py:9-122), for renderers without a
    fused path; each view still runs on the HIP rasterizer through the renderer's own forward."""
    bs = batch["c2w"].shape[0]
    lists = {k: [] for k in ("render", "viewspace_points", "visibility_filter", "radii", "normal",
                             "normal_from_dist", "pred_normal", "depth", "mask", "comp_rgb_bg")}
    for batch_idx in range(bs):
        pkg = render_view_reference(renderer, batch, batch_idx)
        for k in ("render", "viewspace_points", "visibility_filter", "radii"):
            lists[k].append(pkg[k])
        for k in ("normal", "depth", "mask", "comp_rgb_bg"):
            if k in pkg:
                lists[k].append(pkg[k])
        for k in ("normal_from_dist", "pred_normal"):
            if pkg.get(k) is not None:
                lists[k].append(pkg[k])
    out = {"comp_rgb": torch.stack(lists["render"], 0).permute(0, 2, 3, 1),
           "viewspace_points": lists["viewspace_points"], "visibility_filter": lists["visibility_filter"],
           "radii": lists["radii"]}
    for k, name in (("normal", "comp_normal"), ("normal_from_dist", "comp_normal_from_dist"),
                    ("pred_normal", "comp_pred_normal"), ("depth", "comp_depth"), ("mask", "comp_mask")):
        if lists[k]:
            out[name] = torch.stack(lists[k], 0).permute(0, 2, 3, 1)
    if lists["comp_rgb_bg"]:
        out["comp_rgb_bg"] = torch.cat(lists["comp_rgb_bg"], 0).permute(0, 2, 3, 1)
    return out


class GaussianBatchRenderer:
    """Mixin replacing renderer/gaussian_batch_renderer.py:GaussianBatchRenderer (same ``batch_forward``
    contract).  Set ``batch_render_mode`` to force a mode ("per_view" = the reference loop); set
    ``shard_views = False`` to render every view on every rank."""

    batch_render_mode = None
    shard_views = True
    shard_group = None
    # view_shard.ChunkedGradReduce: the fused path's rasterizer call sums its per-Gaussian gradients over ranks
    # inside the backward (overlapped with it); with the predicted-normal pass, one reduction after both calls.
    # Ranks without views (batch < world) join the same collectives with zero gradients.  Parameter-direct
    # loss terms are not covered: reduce those with allreduce_grads.
    grad_reduce = None

    def batch_forward(self, batch):
        mode = batch_mode(self)
        if mode is None:
            return reference_batch_forward(self, batch)
        return render_batch(self, batch, mode, group=self.shard_group, shard=self.shard_views)


__all__ = ["GaussianBatchRenderer", "Camera", "MODES", "batch_mode", "batch_draws", "material_params", "render_batch",
           "render_views_local", "render_view_reference", "reference_batch_forward", "view_camera"]

"""Stand-ins for the reference's renderer objects, for the batch-renderer tests (test infrastructure).

``make_renderer(mode, scene, device)`` builds an object with what the reference's renderers use —
``geometry`` (getters of geometry/gaussian_base.py:371-411 / geometry/sugar.py:547-556 as leaves),
``background`` (a per-ray function standing in for the background network), ``material`` (the point
light material's fields, material/gaussian_material.py:17-41), ``background_tensor``, ``cfg`` and
``training`` — whose per-view ``forward`` restates the reference's DiffGaussian.forward for that mode:

    plain         renderer/diff_gaussian_rasterizer.py:45-145
    background    renderer/diff_gaussian_rasterizer_background.py:44-145
    shading       renderer/diff_gaussian_rasterizer_shading.py:79-231 (Depth2Normal + material: the
                  tests/torch_reference.shading_epilogue restatement)
    sugar_normal  renderer/diff_sugar_rasterizer_normal.py:80-223
    sugar_shading renderer/diff_sugar_rasterizer_shading.py:80-224 (the point-light material restated:
                  point_light_material below)

The per-view rasterizer call goes through ``RASTERIZE`` (GaussianRasterizer on the GPU); the CPU tests
swap it for the torch formulation (tests/torch_reference.render) together with the batch renderer's
``_rasterize_views`` so the batching / sharding logic runs without a GPU.
"""
from __future__ import annotations

import math
from types import SimpleNamespace

import numpy as np
import torch

import torch_reference as tr
from diff_gaussian_rasterization import GaussianRasterizationSettings
from diff_gaussian_rasterization.batch_renderer import GaussianBatchRenderer, material_params


def gpu_rasterize(settings, **kw):
    from diff_gaussian_rasterization import GaussianRasterizer

    return GaussianRasterizer(raster_settings=settings)(**kw)


def torch_rasterize(settings, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None,
                    rotations=None, cov3D_precomp=None):
    """GaussianRasterizer's call restated with the dense torch formulation (CPU / any device)."""
    s = settings
    dt = means3D.dtype
    deg = s.sh_degree
    if shs is not None:  # the rasterizer reads sqrt(M) - 1 degrees at most (the pred-normal pass: M = 1)
        deg = min(deg, int(round(math.sqrt(shs.shape[1]))) - 1)
    return tr.render(means3D, means2D, opacities, s.viewmatrix.reshape(-1).to(dt), s.projmatrix.reshape(-1).to(dt),
                     s.campos.to(dt), s.tanfovx, s.tanfovy, s.image_width, s.image_height, s.bg.to(dt), sh=shs,
                     deg=deg, colors=colors_precomp, scales=scales, rotations=rotations, cov3D=cov3D_precomp,
                     mod=s.scale_modifier)


RASTERIZE = gpu_rasterize


def torch_rasterize_views(settings_list, means3D, means2D_list, opacities, shs=None, colors_precomp=None,
                          scales=None, rotations=None, cov3D_precomp=None, background=None, colors2=None,
                          grad_reduce=None, clamp=False):
    """batched.rasterize_views restated as a loop over torch_rasterize (for the CPU tests).  grad_reduce: the
    call's per-Gaussian gradients are summed over ranks in its backward, as the HIP call does (here through
    view_shard.reduce_on_backward on its inputs, in the HIP call's gradient order)."""
    if grad_reduce is not None and grad_reduce.active():
        from diff_gaussian_rasterization.view_shard import reduce_on_backward

        names = ("means3D", "shs", "colors_precomp", "opacities", "scales", "rotations", "colors2")
        vals = dict(zip(names, (means3D, shs, colors_precomp, opacities, scales, rotations, colors2)))
        keep = [k for k in names if vals[k] is not None and vals[k].requires_grad]
        vals.update(zip(keep, reduce_on_backward(grad_reduce, [vals[k] for k in keep])))
        means3D, shs, colors_precomp, opacities, scales, rotations, colors2 = (vals[k] for k in names)
    outs = [torch_rasterize(s, means3D, m2, opacities, shs=shs, colors_precomp=colors_precomp, scales=scales,
                            rotations=rotations, cov3D_precomp=cov3D_precomp)
            for s, m2 in zip(settings_list, means2D_list)]
    color, radii, depth, alpha = (torch.stack([o[i] for o in outs]) for i in range(4))
    if background is not None:
        color = (color + (1 - alpha) * background.permute(0, 3, 1, 2)).clamp(0, 1)
    elif clamp:
        color = color.clamp(0, 1)
    if colors2 is None:
        return color, radii, depth, alpha
    second = [torch_rasterize(s, means3D, torch.zeros_like(m2), opacities, colors_precomp=colors2, scales=scales,
                              rotations=rotations, cov3D_precomp=cov3D_precomp)[0]
              for s, m2 in zip(settings_list, means2D_list)]
    return color, radii, depth, alpha, torch.stack(second)


def torch_shade_views(color, depth, alpha, rays_o, rays_d, bg, light_positions, ambient, diffuse, shading,
                      pred_normal=None):
    """shading.shade_views restated per view with tests/torch_reference.shading_epilogue (for the CPU tests);
    ambient / diffuse / shading per view."""
    outs = []
    for v in range(depth.shape[0]):
        dt = depth.dtype
        ka = torch.tensor(ambient[v], dtype=dt, device=depth.device)
        kd = torch.tensor(diffuse[v], dtype=dt, device=depth.device)
        outs.append(tr.shading_epilogue(color[v], depth[v], alpha[v], rays_o[v], rays_d[v], bg[v], light_positions[v],
                                        ka, kd, shading[v], pred_normal[v] if pred_normal is not None else None))
    return tuple(torch.stack([o[i] for o in outs]) for i in range(3))


def _normal_maps_one(depth, alpha, rays_o, rays_d):
    """The normal renderer's epilogue (renderer/diff_gaussian_rasterizer_normal.py:172-193) for one view."""
    xyz = rays_o + depth.permute(1, 2, 0) * rays_d
    n = torch.nn.functional.normalize(tr.depth_to_normal(xyz.permute(2, 0, 1).unsqueeze(0))[0], dim=0)
    nmap = n * 0.5 * alpha + 0.5
    mask = alpha.float() > 0.99
    return (torch.where(mask.repeat(3, 1, 1), nmap, nmap.detach()), torch.where(mask, depth, depth.detach()))


def torch_depth_normal_maps(depth, alpha, rays_o, rays_d):
    outs = [_normal_maps_one(depth[v], alpha[v], rays_o[v], rays_d[v]) for v in range(depth.shape[0])]
    return torch.stack([o[0] for o in outs]), torch.stack([o[1] for o in outs])


def torch_depth_normal_views(depth, alpha, rays_o, rays_d):
    outs = [tr.sugar_normal_from_dist(depth[v], alpha[v], rays_o[v], rays_d[v]) for v in range(depth.shape[0])]
    return torch.stack([o[0] for o in outs]), torch.stack([o[1] for o in outs])


def torch_sugar_normal_map(normal, alpha):
    """renderer/diff_sugar_rasterizer_normal.py:192-197 per view (the torch lines the fused pass replaces)."""
    outs = []
    for v in range(normal.shape[0]):
        n = torch.nn.functional.normalize(normal[v], dim=0)
        n = torch.cat([-n[:2], n[2:]], 0)
        nmap = n * 0.5 * alpha[v] + 0.5
        mask = (alpha[v] > 0.99).repeat(3, 1, 1)
        outs.append(torch.where(mask, nmap, nmap.detach()))
    return torch.stack(outs)


class FakeGeometry:
    def __init__(self, scene, device, dtype=torch.float32, pred_normal=False):
        leaf = lambda x: torch.tensor(x, device=device, dtype=dtype, requires_grad=True)  # noqa: E731
        self.params = {k: leaf(scene[k]) for k in ("means3D", "shs", "opacities", "scales", "rotations")}
        if "normals" in scene:
            self.params["normals"] = leaf(scene["normals"])
        elif pred_normal:  # the geometry's per-Gaussian normal (pc.get_normal) for the predicted-normal pass
            g = torch.Generator().manual_seed(17)
            n = torch.randn(len(scene["means3D"]), 3, generator=g, dtype=torch.float64)
            self.params["normals"] = leaf((n / n.norm(dim=-1, keepdim=True)).numpy())
        self.active_sh_degree = int(scene.get("sh_degree", 0))
        self.cfg = SimpleNamespace(pred_normal=pred_normal)

    get_xyz = property(lambda self: self.params["means3D"])
    get_features = property(lambda self: self.params["shs"])
    get_opacity = property(lambda self: self.params["opacities"])
    get_scaling = property(lambda self: self.params["scales"])
    get_rotation = property(lambda self: self.params["rotations"])
    get_gs_normals = property(lambda self: self.params["normals"])
    get_normal = property(lambda self: self.params["normals"])


def point_light_material(positions, shading_normal, light_positions, albedo, ka, kd, shading):
    """material/gaussian_material.py:41-104 (GaussianDiffuseWithPointLightMaterial.forward) with the light colours
    and shading mode the material would draw (batch_renderer.material_params, same draws in the same order)."""
    F = torch.nn.functional
    ka = torch.tensor(ka, dtype=albedo.dtype, device=albedo.device)
    kd = torch.tensor(kd, dtype=albedo.dtype, device=albedo.device)
    light_directions = F.normalize(light_positions - positions, dim=-1)
    diffuse_light = torch.sum(shading_normal * light_directions, -1, keepdim=True).clamp(min=0.0) * kd
    textureless_color = diffuse_light + ka
    color = albedo.clamp(0.0, 1.0) * textureless_color
    if shading == "albedo":
        return albedo + textureless_color * 0
    if shading == "textureless":
        return albedo * 0 + textureless_color
    return color


def _background_net(dirs):
    """Per-ray background colours (stands in for the background MLP: (n, H, W, 3) -> (n, H, W, 3))."""
    return torch.sigmoid(2.0 * dirs)


class FakeRenderer(GaussianBatchRenderer):
    def __init__(self, mode, scene, device, dtype=torch.float32, training=False, soft_shading=False,
                 pred_normal=False):
        self.batch_render_mode = mode
        self.geometry = FakeGeometry(scene, device, dtype, pred_normal=pred_normal)
        self.background_tensor = torch.tensor([1.0, 1.0, 1.0], device=device, dtype=dtype)
        self.background = lambda dirs: _background_net(dirs)
        # the MVDream config's material (configs/gaussian_splatting_mvdream.yaml:62-67: soft_shading true)
        self.material = SimpleNamespace(cfg=SimpleNamespace(soft_shading=soft_shading, diffuse_prob=0.75,
                                                            textureless_prob=0.5),
                                        ambient_light_color=torch.tensor([0.1, 0.1, 0.1]),
                                        diffuse_light_color=torch.tensor([0.9, 0.9, 0.9]), ambient_only=False)
        self.cfg = SimpleNamespace(invert_bg_prob=0.5, debug=False)
        self.training = training
        self.mode = mode

    # the reference's per-view DiffGaussian.forward of each mode
    def forward(self, cam, bg_color, scaling_modifier=1.0, override_color=None, **kwargs):
        pc = self.geometry
        if self.mode in ("background", "shading", "sugar_shading"):
            bg_color = bg_color * 0
        else:  # renderer/diff_gaussian_rasterizer.py:59-64
            invert = (np.random.rand() > self.cfg.invert_bg_prob) if self.training else True
            bg_color = 1.0 - bg_color if invert else bg_color
        sp = torch.zeros_like(pc.get_xyz, requires_grad=True) + 0
        sp.retain_grad()
        settings = GaussianRasterizationSettings(
            image_height=int(cam.image_height), image_width=int(cam.image_width),
            tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5), bg=bg_color,
            scale_modifier=scaling_modifier, viewmatrix=cam.world_view_transform,
            projmatrix=cam.full_proj_transform, sh_degree=pc.active_sh_degree, campos=cam.camera_center,
            prefiltered=False, debug=False)
        shs = pc.get_features if override_color is None else None
        kw = dict(means3D=pc.get_xyz, means2D=sp, shs=shs, colors_precomp=override_color, opacities=pc.get_opacity,
                  scales=pc.get_scaling, rotations=pc.get_rotation, cov3D_precomp=None)
        img, radii, depth, alpha = RASTERIZE(settings, **kw)
        _, H, W = img.shape
        b = kwargs["batch_idx"]
        pkg = {"viewspace_points": sp, "visibility_filter": radii > 0, "radii": radii}
        pred = None
        if self.mode in ("shading", "normal") and pc.cfg.pred_normal:
            # renderer/diff_gaussian_rasterizer_shading.py:177-187 (normal.py:175-185)
            kwp = dict(kw, means2D=torch.zeros_like(sp), shs=pc.get_normal.unsqueeze(1), colors_precomp=None)
            pred, _, _, _ = RASTERIZE(settings, **kwp)
        if self.mode == "plain":
            pkg["render"] = img.clamp(0, 1)
        elif self.mode == "advanced":
            pkg.update(render=img.clamp(0, 1), depth=depth, mask=alpha)
        elif self.mode == "normal":
            nmap, depth_m = _normal_maps_one(depth, alpha, kwargs["rays_o"][b], kwargs["rays_d"][b])
            pkg.update(render=img.clamp(0, 1), normal=nmap, pred_normal=pred, mask=alpha, depth=depth_m)
        elif self.mode == "background":
            comp_rgb_bg = self.background(dirs=kwargs["rays_d"][b].unsqueeze(0))
            img = img + (1 - alpha) * comp_rgb_bg.reshape(H, W, 3).permute(2, 0, 1)
            pkg["render"] = img.clamp(0, 1)
        elif self.mode == "shading":
            comp_rgb_bg = self.background(dirs=kwargs["rays_d"][b].unsqueeze(0))
            ka, kd, smode = material_params(self.material, self.training)
            dt = img.dtype
            render, nmap, depth_m = tr.shading_epilogue(
                img, depth, alpha, kwargs["rays_o"][b], kwargs["rays_d"][b], comp_rgb_bg, kwargs["light_positions"][b],
                torch.tensor(ka, device=img.device, dtype=dt), torch.tensor(kd, device=img.device, dtype=dt), smode,
                pred)
            pkg.update(render=render, normal=nmap, pred_normal=pred, mask=alpha, depth=depth_m, comp_rgb_bg=comp_rgb_bg)
        elif self.mode == "sugar_normal":
            nfd, nmap_dist = tr.sugar_normal_from_dist(depth, alpha, kwargs["rays_o"][b], kwargs["rays_d"][b])
            kw2 = dict(kw, means2D=torch.zeros_like(sp), shs=None, colors_precomp=pc.get_gs_normals)
            normal, _, _, _ = RASTERIZE(settings, **kw2)
            normal = torch.nn.functional.normalize(normal, dim=0)
            normal = torch.cat([-normal[:2], normal[2:]], 0)
            nmap = normal * 0.5 * alpha + 0.5
            mask = alpha > 0.99
            nmap = torch.where(mask.expand_as(nmap), nmap, nmap.detach())
            depth = torch.where(mask, depth, depth.detach())
            pkg.update(render=img.clamp(0, 1), normal=nmap, normal_from_dist=nmap_dist, mask=alpha, depth=depth)
        elif self.mode == "sugar_shading":
            # renderer/diff_sugar_rasterizer_shading.py:170-213
            rays_d, rays_o = kwargs["rays_d"][b], kwargs["rays_o"][b]
            if kwargs.get("override_bg_color") is not None:
                comp_rgb_bg = kwargs["override_bg_color"].expand(1, H, W, -1)
            else:
                comp_rgb_bg = self.background(dirs=rays_d.unsqueeze(0))
            xyz_map = rays_o + depth.permute(1, 2, 0) * rays_d
            kw2 = dict(kw, means2D=torch.zeros_like(sp), shs=None, colors_precomp=pc.get_gs_normals)
            normal_map, _, _, _ = RASTERIZE(settings, **kw2)
            normal_map = torch.nn.functional.normalize(normal_map, dim=0)
            light = kwargs["light_positions"][b, None, None, :].expand(H, W, -1)
            ka, kd, smode = material_params(self.material, self.training)
            rgb_fg = point_light_material(xyz_map, normal_map.permute(1, 2, 0), light,
                                          (img / (alpha + 1e-6)).permute(1, 2, 0), ka, kd, smode).permute(2, 0, 1)
            img = rgb_fg * alpha + (1 - alpha) * comp_rgb_bg.reshape(H, W, 3).permute(2, 0, 1)
            normal_map = normal_map * 0.5 * alpha + 0.5
            mask = alpha > 0.99
            normal_map = torch.where(mask.repeat(3, 1, 1), normal_map, normal_map.detach())
            depth = torch.where(mask, depth, depth.detach())
            pkg.update(render=img.clamp(0, 1), normal=normal_map, mask=alpha, depth=depth, comp_rgb_bg=comp_rgb_bg)
        return pkg


class PerViewRenderer(FakeRenderer):
    """The same renderer with the reference's per-view batch loop (batch_render_mode = "per_view")."""

    def __init__(self, mode, scene, device, dtype=torch.float32, **kw):
        super().__init__(mode, scene, device, dtype, **kw)
        self.batch_render_mode = "per_view"


def make_batch(B, H, W, device, dtype=torch.float32, seed=0):
    """The data module's batch dict (data/uncond.py:338-352): orbit cameras, rays, light positions."""
    from diff_gaussian_rasterization.cameras import light_positions_dreamfusion, orbit_c2w, ray_bundle

    g = torch.Generator().manual_seed(seed)
    elev = torch.rand(B, generator=g) * 30.0
    azim = torch.rand(B, generator=g) * 360.0
    c2w = orbit_c2w(torch.full((B,), 2.5), elev, azim)
    fovy = torch.full((B,), math.radians(60.0))
    rays_o, rays_d = ray_bundle(c2w, fovy, H, W)
    return {"c2w": c2w.to(device), "fovy": fovy.to(device), "height": H, "width": W,
            "rays_o": rays_o.to(device, dtype), "rays_d": rays_d.to(device, dtype),
            "light_positions": light_positions_dreamfusion(c2w, 2.0).to(device, dtype)}


def loss_of(out, seed=1):
    g = torch.Generator().manual_seed(seed)
    total = 0
    for k in ("comp_rgb", "comp_depth", "comp_mask", "comp_normal", "comp_normal_from_dist", "comp_pred_normal"):
        if k in out:
            w = torch.randn(out[k].shape, generator=g, dtype=torch.float64).to(out[k].device, out[k].dtype)
            total = total + (out[k] * w).sum()
    return total

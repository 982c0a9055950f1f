"""Restatement of the reference geometry's densify / prune state machine (test infrastructure).

GaussianBaseModel (geometry/gaussian_base.py) keeps the raw parameters (_xyz, _features_dc,
_features_rest, _opacity, _scaling, _rotation) in an Adam optimizer and, in ``update_states``
(:821-869), accumulates the densification statistics per view, then prunes (:802-808) and densifies
(:795-800: clone :771-793, split :715-769 with torch.normal samples) on a schedule, with a random
``torch.randperm`` prune above ``max_num`` (:836-841).  This class restates exactly that logic on any
device so the sharded tests can check that replicas on different ranks stay identical through it.
"""
from __future__ import annotations

from types import SimpleNamespace

import torch
import torch.nn as nn


def inverse_sigmoid(x):
    return torch.log(x / (1 - x))


def build_rotation(r):
    """geometry/gaussian_base.py:99-122."""
    norm = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    R = torch.zeros((q.size(0), 3, 3), device=r.device, dtype=r.dtype)
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - w * z)
    R[:, 0, 2] = 2 * (x * z + w * y)
    R[:, 1, 0] = 2 * (x * y + w * z)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - w * x)
    R[:, 2, 0] = 2 * (x * z - w * y)
    R[:, 2, 1] = 2 * (y * z + w * x)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


class DensifyModel:
    NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")

    def __init__(self, scene, device, **cfg):
        t = lambda x: torch.tensor(x, device=device, dtype=torch.float32)  # noqa: E731
        sh = t(scene["shs"])
        self._xyz = nn.Parameter(t(scene["means3D"]))
        self._features_dc = nn.Parameter(sh[:, :1].contiguous())
        self._features_rest = nn.Parameter(sh[:, 1:].contiguous())
        self._opacity = nn.Parameter(inverse_sigmoid(t(scene["opacities"]).clamp(1e-4, 1 - 1e-4)))
        self._scaling = nn.Parameter(torch.log(t(scene["scales"])))
        self._rotation = nn.Parameter(t(scene["rotations"]))
        self.active_sh_degree = int(scene["sh_degree"])
        self.cfg = SimpleNamespace(split_thresh=0.01, sugar_prune_at=None, sugar_prune_threshold=0.5,
                                   max_num=10_000_000, prune_from_iter=0, prune_until_iter=10_000, prune_interval=1,
                                   opacity_reset_interval=10_000, min_opac_prune=0.05, radii2d_thresh=1000,
                                   densify_from_iter=0, densify_until_iter=10_000, densification_interval=1,
                                   densify_grad_threshold=0.01, prune_big_points=False, pred_normal=False)
        for k, v in cfg.items():
            setattr(self.cfg, k, v)
        self.optimize_params = list(self.NAMES)
        groups = [{"params": [p], "lr": 1e-3, "name": n} for n, p in zip(
            self.NAMES, (self._xyz, self._features_dc, self._features_rest, self._opacity, self._scaling,
                         self._rotation))]
        self.optimizer = torch.optim.Adam(groups, lr=0.0, eps=1e-15)
        P = self._xyz.shape[0]
        self.xyz_gradient_accum = torch.zeros((P, 1), device=device)
        self.denom = torch.zeros((P, 1), device=device)
        self.max_radii2D = torch.zeros((P,), device=device)
        self.device = device

    # getters (:371-411)
    get_xyz = property(lambda self: self._xyz)
    get_scaling = property(lambda self: torch.exp(self._scaling))
    get_rotation = property(lambda self: torch.nn.functional.normalize(self._rotation))
    get_opacity = property(lambda self: torch.sigmoid(self._opacity))
    get_features = property(lambda self: torch.cat((self._features_dc, self._features_rest), dim=1))

    def scaling_inverse_activation(self, x):
        return torch.log(x)

    def parameters(self):
        return [self._xyz, self._features_dc, self._features_rest, self._opacity, self._scaling, self._rotation]

    # optimizer surgery (:606-680)
    def _prune_optimizer(self, mask):
        out = {}
        for group in self.optimizer.param_groups:
            st = self.optimizer.state.get(group["params"][0], None)
            if st is not None:
                st["exp_avg"] = st["exp_avg"][mask]
                st["exp_avg_sq"] = st["exp_avg_sq"][mask]
                del self.optimizer.state[group["params"][0]]
                group["params"][0] = nn.Parameter(group["params"][0][mask].requires_grad_(True))
                self.optimizer.state[group["params"][0]] = st
            else:
                group["params"][0] = nn.Parameter(group["params"][0][mask].requires_grad_(True))
            out[group["name"]] = group["params"][0]
        return out

    def _set(self, t):
        self._xyz, self._features_dc, self._features_rest = t["xyz"], t["f_dc"], t["f_rest"]
        self._opacity, self._scaling, self._rotation = t["opacity"], t["scaling"], t["rotation"]

    def prune_points(self, mask):
        valid = ~mask
        self._set(self._prune_optimizer(valid))
        self.xyz_gradient_accum = self.xyz_gradient_accum[valid]
        self.denom = self.denom[valid]
        self.max_radii2D = self.max_radii2D[valid]

    def cat_tensors_to_optimizer(self, d):
        out = {}
        for group in self.optimizer.param_groups:
            ext = d[group["name"]]
            st = self.optimizer.state.get(group["params"][0], None)
            if st is not None:
                st["exp_avg"] = torch.cat((st["exp_avg"], torch.zeros_like(ext)), dim=0)
                st["exp_avg_sq"] = torch.cat((st["exp_avg_sq"], torch.zeros_like(ext)), dim=0)
                del self.optimizer.state[group["params"][0]]
                group["params"][0] = nn.Parameter(torch.cat((group["params"][0], ext), dim=0).requires_grad_(True))
                self.optimizer.state[group["params"][0]] = st
            else:
                group["params"][0] = nn.Parameter(torch.cat((group["params"][0], ext), dim=0).requires_grad_(True))
            out[group["name"]] = group["params"][0]
        return out

    def densification_postfix(self, xyz, f_dc, f_rest, opacity, scaling, rotation):
        self._set(self.cat_tensors_to_optimizer(dict(xyz=xyz, f_dc=f_dc, f_rest=f_rest, opacity=opacity,
                                                     scaling=scaling, rotation=rotation)))
        P = self._xyz.shape[0]
        self.xyz_gradient_accum = torch.zeros((P, 1), device=self.device)
        self.denom = torch.zeros((P, 1), device=self.device)
        self.max_radii2D = torch.zeros((P,), device=self.device)

    def densify_and_split(self, grads, grad_threshold, N=2):
        n0 = self._xyz.shape[0]
        padded = torch.zeros((n0,), device=self.device)
        padded[: grads.shape[0]] = grads.squeeze()
        sel = torch.where(padded >= grad_threshold, True, False)
        sel = torch.logical_and(sel, torch.norm(self.get_scaling, dim=1) > self.cfg.split_thresh)
        stds = self.get_scaling[sel].repeat(N, 1) / N
        means = torch.zeros((stds.size(0), 3), device=self.device)
        samples = torch.normal(mean=means, std=stds)
        rots = build_rotation(self._rotation[sel]).repeat(N, 1, 1)
        new_xyz = torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + self._xyz[sel].repeat(N, 1)
        new_scaling = self.scaling_inverse_activation(self.get_scaling[sel].repeat(N, 1) / (0.8 * N))
        self.densification_postfix(new_xyz, self._features_dc[sel].repeat(N, 1, 1),
                                   self._features_rest[sel].repeat(N, 1, 1), self._opacity[sel].repeat(N, 1),
                                   new_scaling, self._rotation[sel].repeat(N, 1))
        prune = torch.cat((sel, torch.zeros(N * sel.sum(), device=self.device, dtype=bool)))
        self.prune_points(prune)

    def densify_and_clone(self, grads, grad_threshold):
        sel = torch.where(torch.norm(grads, dim=-1) >= grad_threshold, True, False)
        sel = torch.logical_and(sel, torch.norm(self.get_scaling, dim=1) <= self.cfg.split_thresh)
        self.densification_postfix(self._xyz[sel], self._features_dc[sel], self._features_rest[sel],
                                   self._opacity[sel], self._scaling[sel], self._rotation[sel])

    def densify(self, max_grad):
        grads = self.xyz_gradient_accum / self.denom
        grads[grads.isnan()] = 0.0
        self.densify_and_clone(grads, max_grad)
        self.densify_and_split(grads, max_grad)

    def prune(self, min_opacity, max_screen_size):
        mask = (self.get_opacity < min_opacity).squeeze()
        if self.cfg.prune_big_points:
            mask = torch.logical_or(mask, self.max_radii2D > (torch.mean(self.max_radii2D) * 3))
        self.prune_points(mask)

    def reset_opacity(self):
        pass

    def add_densification_stats(self, viewspace_point_tensor, update_filter):
        self.xyz_gradient_accum[update_filter] += torch.norm(viewspace_point_tensor.grad[update_filter, :2], dim=-1,
                                                             keepdim=True)
        self.denom[update_filter] += 1

    @torch.no_grad()
    def update_states(self, iteration, visibility_filter, radii, viewspace_point_tensor):
        """geometry/gaussian_base.py:821-869."""
        self.pruned_or_densified = False
        if self.cfg.sugar_prune_at is not None and iteration == self.cfg.sugar_prune_at:
            self.pruned_or_densified = True
            self.prune_points((self.get_opacity < self.cfg.sugar_prune_threshold).squeeze())
            return
        if self._xyz.shape[0] >= self.cfg.max_num + 100:
            self.pruned_or_densified = True
            prune_mask = torch.randperm(self._xyz.shape[0]).to(self._xyz.device)
            self.prune_points(prune_mask > self.cfg.max_num)
            return
        for i in range(len(viewspace_point_tensor)):
            self.max_radii2D = torch.max(self.max_radii2D, radii[i].float())
            self.add_densification_stats(viewspace_point_tensor[i], visibility_filter[i])
        if (self.cfg.prune_from_iter < iteration < self.cfg.prune_until_iter
                and iteration % self.cfg.prune_interval == 0):
            self.pruned_or_densified = True
            self.prune(self.cfg.min_opac_prune, self.cfg.radii2d_thresh)
            if iteration % self.cfg.opacity_reset_interval == 0:
                self.reset_opacity()
        if (self.cfg.densify_from_iter < iteration < self.cfg.densify_until_iter
                and iteration % self.cfg.densification_interval == 0):
            self.pruned_or_densified = True
            self.densify(self.cfg.densify_grad_threshold)

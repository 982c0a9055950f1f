"""Dense, differentiable PyTorch formulation of the reference rasterizer (test infrastructure).

Used to check the CPU restatement's analytic backward (oracle/gsr_oracle.c) against torch autograd,
and as a device-agnostic renderer for the multi-process (gloo) sharding tests.  Same semantics as the
kernels: 16x16 tile binning from the 3-sigma radius rect, per-tile (depth, index) order, alpha =
min(0.99, o e^power), skip alpha < 1/255, stop at T (1 - alpha) < 1e-4, +0.3 EWA dilation, SH + 0.5
clamped at 0.  The discrete decisions (culling, radius, skip/stop masks) are taken on detached values;
gradients flow through everything else, so autograd equals the reference's analytic gradient except
for its documented conventions (0.99 clamp ignored, frustum-clamp zeroing, denom2inv + 1e-7), which
the tests avoid or bound.  means2D is added to the projected NDC xy, so its gradient is the
reference's viewspace gradient (pixel gradient x W/2, H/2).
"""
from __future__ import annotations

import math

import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435]


def sh_color(deg, sh, dirs):
    x, y, z = dirs[:, 0:1], dirs[:, 1:2], dirs[:, 2:3]
    res = SH_C0 * sh[:, 0]
    if deg > 0:
        res = res - SH_C1 * y * sh[:, 1] + SH_C1 * z * sh[:, 2] - SH_C1 * x * sh[:, 3]
        if deg > 1:
            xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
            res = (res + SH_C2[0] * xy * sh[:, 4] + SH_C2[1] * yz * sh[:, 5] + SH_C2[2] * (2 * zz - xx - yy) * sh[:, 6]
                   + SH_C2[3] * xz * sh[:, 7] + SH_C2[4] * (xx - yy) * sh[:, 8])
            if deg > 2:
                res = (res + SH_C3[0] * y * (3 * xx - yy) * sh[:, 9] + SH_C3[1] * xy * z * sh[:, 10]
                       + SH_C3[2] * y * (4 * zz - xx - yy) * sh[:, 11]
                       + SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12]
                       + SH_C3[4] * x * (4 * zz - xx - yy) * sh[:, 13] + SH_C3[5] * z * (xx - yy) * sh[:, 14]
                       + SH_C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return res


def rot_matrix(q):
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    return torch.stack([
        torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], -1),
        torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], -1),
        torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1)], -2)


def render(means3D, means2D, opacities, view, proj, campos, tanx, tany, W, H, bg, sh=None, deg=0, colors=None,
           scales=None, rotations=None, cov3D=None, mod=1.0):
    """Returns (color (3,H,W), radii (P,), depth (1,H,W), alpha (1,H,W))."""
    dt = means3D.dtype
    P = means3D.shape[0]
    M4v = view.reshape(4, 4).to(dt)
    M4p = proj.reshape(4, 4).to(dt)
    ph = torch.cat([means3D, torch.ones(P, 1, dtype=dt)], 1)
    p_view = (ph @ M4v)[:, :3]
    p_hom = ph @ M4p
    pw = 1.0 / (p_hom[:, 3] + 1e-7)
    ndc = p_hom[:, :2] * pw[:, None] + means2D[:, :2]
    if cov3D is None:
        R = rot_matrix(rotations)
        S = torch.diag_embed(mod * scales)
        Lm = R @ S
        Sig = Lm @ Lm.transpose(1, 2)
    else:
        c = cov3D
        Sig = torch.stack([torch.stack([c[:, 0], c[:, 1], c[:, 2]], -1), torch.stack([c[:, 1], c[:, 3], c[:, 4]], -1),
                           torch.stack([c[:, 2], c[:, 4], c[:, 5]], -1)], -2)
    # the C ABI carries tan(fov/2) as float32 and computes the focal lengths in float32
    import numpy as np

    tanx, tany = float(np.float32(tanx)), float(np.float32(tany))
    fx = float(np.float32(W) / (np.float32(2.0) * np.float32(tanx)))
    fy = float(np.float32(H) / (np.float32(2.0) * np.float32(tany)))
    t = p_view
    limx, limy = 1.3 * tanx, 1.3 * tany
    tx = torch.clamp(t[:, 0] / t[:, 2], -limx, limx) * t[:, 2]
    ty = torch.clamp(t[:, 1] / t[:, 2], -limy, limy) * t[:, 2]
    tz = t[:, 2]
    zero = torch.zeros_like(tz)
    J = torch.stack([torch.stack([fx / tz, zero, -fx * tx / tz ** 2], -1),
                     torch.stack([zero, fy / tz, -fy * ty / tz ** 2], -1)], -2)
    Wr = M4v[:3, :3].T  # world -> camera rotation
    Tm = J @ Wr
    cov2 = Tm @ Sig @ Tm.transpose(1, 2)
    a = cov2[:, 0, 0] + 0.3
    b = cov2[:, 0, 1]
    c = cov2[:, 1, 1] + 0.3
    det = a * c - b * b
    ca, cb, cc = c / det, -b / det, a / det
    with torch.no_grad():
        mid = 0.5 * (a + c)
        l1 = mid + torch.sqrt(torch.clamp(mid * mid - det, min=0.1))
        l2 = mid - torch.sqrt(torch.clamp(mid * mid - det, min=0.1))
        rad = torch.ceil(3 * torch.sqrt(torch.maximum(l1, l2)))
    px = ((ndc[:, 0] + 1) * W - 1) * 0.5
    py = ((ndc[:, 1] + 1) * H - 1) * 0.5
    gx, gy = (W + 15) // 16, (H + 15) // 16
    with torch.no_grad():
        r = rad.to(torch.int64)
        pxd, pyd = px.detach(), py.detach()
        xmin = torch.clamp(((pxd - r) / 16).to(torch.int64), 0, gx)
        ymin = torch.clamp(((pyd - r) / 16).to(torch.int64), 0, gy)
        xmax = torch.clamp(((pxd + r + 15) / 16).to(torch.int64), 0, gx)
        ymax = torch.clamp(((pyd + r + 15) / 16).to(torch.int64), 0, gy)
        valid = (p_view[:, 2] > 0.2) & (det != 0) & ((xmax - xmin) * (ymax - ymin) > 0)
        radii = torch.where(valid, r, torch.zeros_like(r)).to(torch.int32)
    if colors is None:
        d = means3D - campos.to(dt)
        d = d / d.norm(dim=1, keepdim=True)
        rgb = torch.clamp_min(sh_color(deg, sh, d) + 0.5, 0.0)
    else:
        rgb = colors
    depth = p_view[:, 2]
    op = opacities.reshape(-1)
    out_c = torch.zeros(3, H, W, dtype=dt)
    out_d = torch.zeros(1, H, W, dtype=dt)
    out_a = torch.zeros(1, H, W, dtype=dt)
    order = sorted(range(P), key=lambda i: (float(depth[i].detach()), i))
    bgv = bg.to(dt)
    rows_c, rows_d, rows_a = [], [], []
    for ty_ in range(gy):
        for tx_ in range(gx):
            ids = [i for i in order if valid[i] and xmin[i] <= tx_ < xmax[i] and ymin[i] <= ty_ < ymax[i]]
            ys = torch.arange(ty_ * 16, min(ty_ * 16 + 16, H))
            xs = torch.arange(tx_ * 16, min(tx_ * 16 + 16, W))
            yy, xx = torch.meshgrid(ys, xs, indexing="ij")
            pxy = torch.stack([xx.reshape(-1), yy.reshape(-1)], 1).to(dt)
            npix = pxy.shape[0]
            if not ids:
                Tf = torch.ones(npix, dtype=dt)
                C = torch.zeros(npix, 3, dtype=dt)
                Dp = torch.zeros(npix, dtype=dt)
            else:
                idx = torch.tensor(ids)
                dx = px[idx][None, :] - pxy[:, 0:1]
                dy = py[idx][None, :] - pxy[:, 1:2]
                power = -0.5 * (ca[idx][None] * dx * dx + cc[idx][None] * dy * dy) - cb[idx][None] * dx * dy
                alpha = torch.clamp_max(op[idx][None] * torch.exp(power), 0.99)
                with torch.no_grad():
                    m0 = (power <= 0) & (alpha >= 1.0 / 255.0)
                    am = torch.where(m0, alpha, torch.zeros_like(alpha))
                    T0 = torch.cumprod(torch.cat([torch.ones(npix, 1, dtype=dt), 1 - am[:, :-1]], 1), 1)
                    term = m0 & (T0 * (1 - alpha) < 1e-4)
                    first = torch.where(term.any(1), term.float().argmax(1), torch.full((npix,), len(ids)))
                    m = m0 & (torch.arange(len(ids))[None, :] < first[:, None])
                am = torch.where(m, alpha, torch.zeros_like(alpha))
                one_m = 1 - am
                Texcl = torch.cumprod(torch.cat([torch.ones(npix, 1, dtype=dt), one_m[:, :-1]], 1), 1)
                w = am * Texcl
                C = w @ rgb[idx]
                Dp = w @ depth[idx]
                Tf = torch.prod(one_m, 1)
            col = C + Tf[:, None] * bgv[None, :]
            rows_c.append((ys, xs, col))
            rows_d.append(Dp)
            rows_a.append(1 - Tf)
    # assemble without in-place writes on tensors that need grad
    k = 0
    for ty_ in range(gy):
        for tx_ in range(gx):
            ys, xs, col = rows_c[k]
            h, w_ = len(ys), len(xs)
            pad = (xs[0].item(), W - xs[-1].item() - 1, ys[0].item(), H - ys[-1].item() - 1)
            out_c = out_c + torch.nn.functional.pad(col.T.reshape(3, h, w_), pad)
            out_d = out_d + torch.nn.functional.pad(rows_d[k].reshape(1, h, w_), pad)
            out_a = out_a + torch.nn.functional.pad(rows_a[k].reshape(1, h, w_), pad)
            k += 1
    return out_c, radii, out_d, out_a


def camera_tensors(cam, dtype=torch.float64):
    return (torch.tensor(cam["view"], dtype=dtype).reshape(-1), torch.tensor(cam["proj"], dtype=dtype).reshape(-1),
            torch.tensor(cam["campos"], dtype=dtype))


__all__ = ["render", "camera_tensors", "sh_color", "rot_matrix", "math"]


# ---- post-raster epilogues of the shading / SuGaR renderers (torch restatement, for tests/test_shading.py) ----

def depth_to_normal(xyz_chw):
    """``Depth2Normal.forward`` (renderer/diff_gaussian_rasterizer_shading.py:22-51): central differences
    of the (1, 3, H, W) xyz map by two 3x3 convolutions with zero padding, normal = -(d/dx x d/dy)."""
    B, C, H, W = xyz_chw.shape
    kx = torch.zeros(1, 1, 3, 3, dtype=xyz_chw.dtype, device=xyz_chw.device)
    kx[0, 0, 1, 0], kx[0, 0, 1, 2] = -1.0, 1.0
    ky = torch.zeros(1, 1, 3, 3, dtype=xyz_chw.dtype, device=xyz_chw.device)
    ky[0, 0, 0, 1], ky[0, 0, 2, 1] = -1.0, 1.0
    flat = xyz_chw.reshape(B * C, 1, H, W)
    dx = torch.nn.functional.conv2d(flat, kx, padding=1).reshape(B, C, H, W)
    dy = torch.nn.functional.conv2d(flat, ky, padding=1).reshape(B, C, H, W)
    return -torch.cross(dx, dy, dim=1)


def shading_epilogue(color, depth, alpha, rays_o, rays_d, bg_hwc, light, ambient, diffuse, shading="diffuse",
                     pred_normal=None):
    """One view of renderer/diff_gaussian_rasterizer_shading.py:169-208 with the point-light material
    (material/gaussian_material.py:86-104): returns (render, normal, depth) as the renderer does."""
    F = torch.nn.functional
    H, W = depth.shape[-2:]
    xyz = rays_o + depth.permute(1, 2, 0) * rays_d
    normal_map = F.normalize(depth_to_normal(xyz.permute(2, 0, 1).unsqueeze(0))[0], dim=0)
    if pred_normal is not None:
        sn = F.normalize(pred_normal.permute(1, 2, 0).detach() * 2 - 1, dim=2)
    else:
        sn = normal_map.permute(1, 2, 0)
    lpos = light[None, None, :].expand(H, W, -1)
    ldir = F.normalize(lpos - xyz, dim=-1)
    dl = torch.sum(sn * ldir, -1, keepdim=True).clamp(min=0.0) * diffuse
    tl = dl + ambient
    albedo = (color / (alpha + 1e-6)).permute(1, 2, 0)
    if shading == "albedo":
        fg = albedo + tl * 0
    elif shading == "textureless":
        fg = albedo * 0 + tl
    else:
        fg = albedo.clamp(0.0, 1.0) * tl
    fg = fg.permute(2, 0, 1)
    img = fg * alpha + (1 - alpha) * bg_hwc.reshape(H, W, 3).permute(2, 0, 1)
    nmap = normal_map * 0.5 * alpha + 0.5
    mask = alpha.float() > 0.99  # the reference's fp32 comparison, also when this runs in fp64
    nmask = mask.repeat(3, 1, 1)
    nmap = torch.where(nmask, nmap, nmap.detach())
    depth = torch.where(mask, depth, depth.detach())
    return img.clamp(0, 1), nmap, depth


def sugar_normal_from_dist(depth, alpha, rays_o, rays_d):
    """renderer/diff_sugar_rasterizer_normal.py:170-177,196-197: (normal_from_dist, normal_map_from_dist)."""
    F = torch.nn.functional
    xyz = rays_o + depth.permute(1, 2, 0) * rays_d
    n = F.normalize(depth_to_normal(xyz.permute(2, 0, 1).unsqueeze(0))[0], dim=0)
    nmap = n * 0.5 * alpha + 0.5
    nmask = (alpha.float() > 0.99).repeat(3, 1, 1)
    return torch.where(nmask, n, n.detach()), torch.where(nmask, nmap, nmap.detach())

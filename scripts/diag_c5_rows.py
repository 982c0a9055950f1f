"""Diagnostic (GPU box): which C5 gradient rows does the HIP rasterizer move away from the fp32 restatement,
and what do those Gaussians look like.  One SuGaR colour pass at the C5 size (1.97M Gaussians, 800^2), the
same upstream gradients into the GPU backward and the fp32 / fp64 oracle backward; writes
gpurun_out/diag_c5_rows.npz with, for the rows the row rule rejects (and a sample of passing rows): the
gradients (GPU, fp32, fp64), the GPU's per-Gaussian preprocess state and the oracle's (fp32 / fp64)."""
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "threestudio-3dgs_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import oracle  # noqa: E402
from gsr_testutil import gs, make_camera, oracle_cam  # noqa: E402


def main():
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    from diff_gaussian_rasterization.batched import rasterize_views

    sub = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 800
    two = len(sys.argv) > 3 and sys.argv[3] == "two"
    scene = gs.make_sugar_scene(sub, sh_degree=0, seed=0)
    P = scene["means3D"].shape[0]
    colors = (scene["shs"][:, 0, :] * np.float32(gs.C0) + np.float32(0.5)).astype(np.float32)
    sc = dict(scene, colors_precomp=colors)
    sc.pop("shs")
    cam = make_camera(S, S, elevation=15.0, azimuth=40.0)
    rng = np.random.default_rng(77)
    up = [rng.standard_normal((3, S, S)).astype(np.float32), rng.standard_normal((1, S, S)).astype(np.float32),
          rng.standard_normal((1, S, S)).astype(np.float32)]
    oc = oracle_cam(cam)
    bg = np.zeros(3, np.float32)
    sc2 = dict(sc, colors_precomp=scene["normals"])
    if two:
        # the C5 test's upstream gradients: the torch fp32 epilogue on the oracle's fp32 outputs of both calls
        import test_gpu_configs as tc
        import torch_reference as tr
        from diff_gaussian_rasterization.cameras import orbit_c2w, ray_bundle

        ro, rd = ray_bundle(orbit_c2w(2.5, 15.0, 40.0)[None], math.radians(60.0), S, S)
        ro, rd = ro[0].float(), rd[0].float()
        f1, f2 = oracle.forward(sc, oc, bg, "f32"), oracle.forward(sc2, oc, bg, "f32")
        ups = {k: rng.standard_normal((1 if k in ("mask", "depth") else 3, S, S)).astype(np.float32)
               for k in tc.SUGAR_OUT}
        lc, ld, la, ln = (torch.tensor(x, requires_grad=True) for x in (f1["color"], f1["depth"], f1["alpha"],
                                                                          f2["color"]))
        o = tc._sugar_epilogue(torch, lc, ld, la, ln, ro, rd, lambda dd, aa: tr.sugar_normal_from_dist(dd, aa, ro, rd))
        sum((o[k] * torch.tensor(ups[k])).sum() for k in tc.SUGAR_OUT).backward()
        up = [x.grad.numpy().astype(np.float32) for x in (lc, ld, la)]
        up2 = ln.grad.numpy().astype(np.float32)
        print("upstream |max|: color %.3g depth %.3g alpha %.3g normal %.3g" % tuple(
            float(np.abs(x).max()) for x in up + [up2]), flush=True)
    dev = "cuda"
    leaf = lambda x: torch.tensor(x, device=dev, requires_grad=True)  # noqa: E731
    t = dict(means3D=leaf(sc["means3D"]), scales=leaf(sc["scales"]), rotations=leaf(sc["rotations"]),
             opacities=leaf(sc["opacities"]), colors=leaf(colors))
    if two:
        t["normals"] = leaf(scene["normals"])
    s = GaussianRasterizationSettings(image_height=S, image_width=S, tanfovx=cam["tanx"], tanfovy=cam["tany"],
                                      bg=torch.zeros(3, device=dev), scale_modifier=1.0,
                                      viewmatrix=torch.tensor(cam["view"], device=dev),
                                      projmatrix=torch.tensor(cam["proj"], device=dev), sh_degree=0,
                                      campos=torch.tensor(cam["campos"], device=dev), prefiltered=False, debug=False)
    m2 = torch.zeros((P, 3), device=dev, requires_grad=True)
    if two:
        c, r, d, a, n2 = rasterize_views([s], t["means3D"], [m2], t["opacities"], colors_precomp=t["colors"],
                                         scales=t["scales"], rotations=t["rotations"], colors2=t["normals"])
        torch.autograd.backward((c[0], d[0], a[0], n2[0]), [torch.tensor(x, device=dev) for x in up + [up2]])
    else:
        c, r, d, a = rasterize_views([s], t["means3D"], [m2], t["opacities"], colors_precomp=t["colors"],
                                     scales=t["scales"], rotations=t["rotations"])
        torch.autograd.backward((c[0], d[0], a[0]), [torch.tensor(x, device=dev) for x in up])
    gpu = {k: v.grad.cpu().numpy().astype(np.float64) for k, v in t.items()}
    gpu["means2D"] = m2.grad.cpu().numpy().astype(np.float64)
    b32 = oracle.backward(sc, oc, bg, *up, prec="f32")
    b64 = oracle.backward(sc, oc, bg, *up, prec="f64")
    names = dict(means3D="means3D", scales="scales", rotations="rotations", opacities="opacity", colors="colors",
                 means2D="means2D")
    if two:
        c32 = oracle.backward(sc2, oc, bg, up2, None, None, prec="f32")
        c64 = oracle.backward(sc2, oc, bg, up2, None, None, prec="f64")
        for k in ("means3D", "scales", "rotations", "opacity"):
            b32["p1_" + k], b64["p1_" + k] = b32[k], b64[k]
            b32["p2_" + k], b64["p2_" + k] = c32[k], c64[k]
            b32[k] = np.asarray(b32[k], np.float64) + np.asarray(c32[k], np.float64)
            b64[k] = np.asarray(b64[k], np.float64) + np.asarray(c64[k], np.float64)
        b32["normals"], b64["normals"] = c32["colors"], c64["colors"]
        names["normals"] = "normals"
        for k in ("means3D", "scales"):
            for pfx in ("p1_", "p2_"):
                names_k = pfx + k
                out_k = names_k
                b32[names_k] = np.asarray(b32[names_k], np.float64)
    out = {}
    bad_any = np.zeros(P, bool)
    for gk, ok in names.items():
        g, r32, r64 = gpu[gk].reshape(P, -1), np.asarray(b32[ok], np.float64).reshape(P, -1), \
            np.asarray(b64[ok], np.float64).reshape(P, -1)
        bar = 1e-4 * np.maximum(1.0, np.abs(r64))
        eg, e3 = np.abs(g - r64), np.abs(r32 - r64)
        beyond = (eg > np.maximum(bar, 4 * e3)).any(1)
        print(f"{ok:10s} beyond {int(beyond.sum())}  gpu_miss {int((eg > bar).any(1).sum())}  "
              f"f32_miss {int((e3 > bar).any(1).sum())}", flush=True)
        bad_any |= beyond
        out["g_" + ok], out["r32_" + ok], out["r64_" + ok] = g, r32, r64
    rows = np.nonzero(bad_any)[0]
    sample = rng.choice(np.nonzero(~bad_any & (np.asarray(b64["opacity"]).reshape(-1) != 0))[0], 2000, replace=False)
    keep = np.concatenate([rows[:20000], sample])
    aux32 = oracle.gauss_aux(sc, oc, "f32")
    aux64 = oracle.gauss_aux(sc, oc, "f64")
    res = dict(rows=rows, sample=sample, keep=keep, P=P)
    for k, v in out.items():
        res[k] = v[keep]
    if two:
        for k in ("means3D", "scales"):
            for pfx in ("p1_", "p2_"):
                res["r32_" + pfx + k] = np.asarray(b32[pfx + k], np.float64)[keep]
                res["r64_" + pfx + k] = np.asarray(b64[pfx + k], np.float64)[keep]
    for k in ("px", "py", "conic", "opacity", "depth", "rad3", "tiles"):
        res["a32_" + k] = np.asarray(aux32[k])[keep]
        res["a64_" + k] = np.asarray(aux64[k])[keep]
    for k in ("means3D", "scales", "rotations", "opacities"):
        res["in_" + k] = np.asarray(sc[k])[keep]
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"diag_c5_rows{'_two' if two else ''}.npz"), **res)
    print("rows rejected:", len(rows), "saved", len(keep), flush=True)


if __name__ == "__main__":
    main()

"""Diagnostic (GPU box): how much of each tile's depth-ordered list a two-phase binning would need.

One C3 view (1M Gaussians, 1024^2, SH3, bench scene and orbit camera 0) through the per-view forward; the
tile lists, the depth order and the per-pixel state are read back from the forward's buffers (offsets as
csrc/gsr_common.h carves them).  For a phase-A threshold X (the nearest X of the visible Gaussians in
depth order), a tile is finished in phase A when its list ends inside phase A, or when every pixel of it
terminated at a list position inside phase A (estimated: a terminated pixel keeps T >= 1e-4 but below
1e-2, the next Gaussian's T (1 - alpha) < 1e-4 with alpha <= 0.99; pixels with T >= 1e-2 walked the whole list); the other tiles need phase B (their list's
remainder).  Prints, per X, the instances phase A and phase B would emit and sort against the full lists.

  python profiles/diag_depth_split.py [view]
"""
import json
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "threestudio-3dgs_amd"))

import bench  # noqa: E402
import gsr_synthetic as gs  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402


def align(x):
    return (x + 255) // 256 * 256


def carve(sizes):
    off, out = 0, []
    for n in sizes:
        off = align(off)
        out.append(off)
        off += n
    return out


def main():
    vi = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    dev = torch.device("cuda:0")
    P, res = 1_000_000, 1024
    scene = gs.make_scene(P, sh_degree=3, seed=0)
    rep = bench.Replica(scene, dev)
    cams = bench.build_views(64, res, dev)
    cam = cams[vi]
    bg = torch.zeros(3, device=dev)
    with torch.no_grad():
        K, color, depth, alpha, radii, geom, binning, image = _C.rasterize_gaussians(
            bg, rep.means3D, None, rep.opacities, rep.scales, rep.rotations, 1.0, None, cam["view"], cam["proj"],
            cam["tan"], cam["tan"], res, res, rep.shs, 3, cam["campos"], False, False)
    torch.cuda.synchronize()
    g = geom.cpu().numpy()
    b = binning.cpu().numpy()
    im = image.cpu().numpy()
    gx = gy = (res + 15) // 16
    T = gx * gy
    HW = res * res
    # geom: rec (64 P), tiles (8 P), dkey0, dkey1, dval0, dval1 (4 P each), sort_counts, sort_totals,
    # kept_counts, counters, goff, goff_part, vis_part, drange
    radix, sort_tile, dup_tile, goff_tile = 256, 4096, 64, 4096
    sb = -(-P // sort_tile)
    gb = -(-P // goff_tile)
    offs = carve([64 * P, 8 * P, 4 * P, 4 * P, 4 * P, 4 * P, 4 * radix * sb, 4 * radix, 4 * -(-P // dup_tile),
                  4 * (3 + 64), 4 * P, 4 * gb, 4 * gb, 4 * 132])
    drange = g[offs[13]:offs[13] + 4 * 132].view(np.uint32)
    which = 1 if drange[129] else 0
    dkey = g[offs[2 + which]:offs[2 + which] + 4 * P].view(np.uint32)
    dval = g[offs[4 + which]:offs[4 + which] + 4 * P].view(np.uint32)
    vbits = max(1, math.ceil(math.log2(max(P, 2))))
    nvis = int((dkey != 0xFFFFFFFF).sum())
    rank = np.full(P, -1, np.int64)
    rank[dval[:nvis] & ((1 << vbits) - 1)] = np.arange(nvis)
    # image: ranges (8 T), quad_maxc (16 T), tile_info (16 T), cut (8 T), final_T (4 HW), n_contrib (4 HW)
    io = carve([8 * T, 16 * T, 16 * T, 8 * T, 4 * HW, 4 * HW])
    ranges = im[io[0]:io[0] + 8 * T].view(np.uint32).reshape(T, 2)
    final_T = im[io[4]:io[4] + 4 * HW].view(np.float32).reshape(res, res)
    n_contrib = im[io[5]:io[5] + 4 * HW].view(np.uint32).reshape(res, res)
    keys = b[0:4 * int(ranges[:, 1].max())].view(np.uint32)  # packed tile << gbits | Gaussian, result in key[0]
    gbits = vbits
    L = (ranges[:, 1] - ranges[:, 0]).astype(np.int64)
    qm = im[io[1]:io[1] + 16 * T].view(np.uint32).reshape(T, 4)
    maxc = qm.max(1).astype(np.int64)
    pct = lambda x, q: int(np.percentile(x, q))  # noqa: E731
    maxc_stats = {"p50": pct(maxc, 50), "p90": pct(maxc, 90), "p99": pct(maxc, 99), "max": int(maxc.max()),
                  "sum": int(maxc.sum()), "tiles_over": {str(c): int((maxc > c).sum()) for c in (128, 256, 512, 1024)},
                  "sum_over_cap": {str(c): int(np.maximum(maxc - c, 0).sum()) for c in (128, 256, 512)}}
    # per tile: the list position where its last pixel terminated (or the list end when some pixel never did)
    need = np.zeros(T, np.int64)
    for t in range(T):
        ty, tx = divmod(t, gx)
        fT = final_T[16 * ty:16 * ty + 16, 16 * tx:16 * tx + 16]
        nc = n_contrib[16 * ty:16 * ty + 16, 16 * tx:16 * tx + 16]
        need[t] = L[t] if (fT >= 1e-2).any() else int(nc.max()) + 1
    out = {"view": vi, "visible": nvis, "listed": int(L.sum()), "tiles": T, "blended_prefix_maxc": maxc_stats,
           "tiles_never_saturated": int(sum(1 for t in range(T) if need[t] >= L[t] and L[t] > 0)),
           "needed_prefix_instances": int(np.minimum(need, L).sum()), "splits": []}
    for X in (0.05, 0.1, 0.15, 0.2, 0.3, 0.5):
        thr = X * nvis
        a_inst = b_inst = 0
        b_tiles = 0
        for t in range(T):
            if L[t] == 0:
                continue
            lst = keys[ranges[t, 0]:ranges[t, 1]] & ((1 << gbits) - 1)
            r = rank[lst]
            pa = int((r < thr).sum())  # depth order inside the list: phase A is a prefix
            a_inst += pa
            if pa < L[t] and need[t] > pa:
                b_inst += int(L[t]) - pa
                b_tiles += 1
        out["splits"].append({"X": X, "phase_a_instances": a_inst, "phase_b_instances": b_inst,
                              "phase_b_tiles": b_tiles, "fraction_of_listed": round((a_inst + b_inst) / L.sum(), 4)})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

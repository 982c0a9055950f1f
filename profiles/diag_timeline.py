"""Per-block timelines of the blend kernels (diagnostic build, `make -C threestudio-3dgs_amd/csrc diag`).

Renders views of the benchmark workload through libgsr_hip_diag.so and summarises, per kernel:
span, block-duration percentiles, the longest blocks and their work (fwd: last contributor;
bwd: kept instances), per-XCD finish time, and the occupancy profile over time (how much of the
span runs with few blocks resident = tail).  Usage (GPU box):  python profiles/diag_timeline.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GSR_HIP_LIB"] = os.path.join(ROOT, "threestudio-3dgs_amd", "csrc", "build_diag", "libgsr_hip_diag.so")
sys.path.insert(0, os.path.join(ROOT, "threestudio-3dgs_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import gsr_synthetic as gs  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402


def summarise(tl, name):
    tl = tl[tl[:, 1] != 0]
    if len(tl) == 0:
        return {"kernel": name, "blocks": 0}
    t0 = int(tl[:, 0].min())
    st = (tl[:, 0].astype(np.int64) - t0) * 10  # ns
    en = (tl[:, 1].astype(np.int64) - t0) * 10
    dur = en - st
    xcc = tl[:, 3] >> 24
    work = tl[:, 3] & 0xFFFFFF
    span = int(en.max())
    # occupancy over time in 100 bins
    bins = np.linspace(0, span, 101)
    occ = [int(((st <= b) & (en > b)).sum()) for b in bins[:-1]]
    order = np.argsort(-dur)[:8]
    busy = dur.sum()
    return {
        "kernel": name, "blocks": int(len(tl)), "span_us": span / 1e3,
        "block_us_p50_p90_p99_max": [float(np.percentile(dur, p)) / 1e3 for p in (50, 90, 99, 100)],
        "sum_block_us": busy / 1e3, "mean_resident_blocks": busy / max(1, span),
        "longest": [{"us": int(dur[i]) / 1e3, "work": int(work[i]), "start_us": int(st[i]) / 1e3} for i in order],
        "work_vs_us_corr": float(np.corrcoef(work, dur)[0, 1]) if len(tl) > 2 else None,
        "ns_per_work_unit_median": float(np.median(dur[work > 16] / work[work > 16])) if (work > 16).any() else None,
        "xcd_finish_us": [int(en[xcc == x].max()) / 1e3 if (xcc == x).any() else None for x in range(8)],
        "xcd_busy_us": [int(dur[xcc == x].sum()) / 1e3 for x in range(8)],
        "occupancy_profile_10": [int(np.mean(occ[i * 10:(i + 1) * 10])) for i in range(10)],
        "time_frac_below_512_blocks": float(np.mean(np.array(occ) < 512)),
        # bwd only: z = sum over batches of 4 x the busiest quadrant's kept count -> lockstep slots per kept pair
        "work_sum": int(work.astype(np.int64).sum()),
        "bwd_lockstep_slots_per_pair": (float(tl[:, 2].astype(np.float64).sum() / max(1, work.sum()))
                                        if name == "k_render_bwd" else None),
        # bwd: block duration = fixed + per-slot cost (least squares over the recorded blocks): the fixed part is
        # what a workgroup spends outside its candidate groups (prologue loads, staging latency, barriers)
        "bwd_fit_fixed_us_per_slot_ns": ([float(x) for x in np.polyfit(tl[:, 2].astype(np.float64), dur, 1)[::-1] /
                                          np.array([1e3, 1.0])] if name == "k_render_bwd" and len(tl) > 2 else None),
        "bwd_us_blocks_without_kept_p50": (float(np.median(dur[tl[:, 2] == 0])) / 1e3
                                           if name == "k_render_bwd" and (tl[:, 2] == 0).any() else None),
    }


def main():
    lib = _C.load_library()
    lib.gsr_diag_timeline.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    scene = gs.make_scene(1_000_000, sh_degree=3, seed=0)
    rep = bench.Replica(scene, dev)
    cams = bench.build_views(64, 1024, dev)
    bg0 = torch.zeros(3, device=dev)
    bgc = torch.full((1024, 1024, 3), 0.5, device=dev)
    gx = gy = 64
    nb = 128 * ((((gx + 1) // 2) * ((gy + 1) // 2) + 7) // 8)
    out = []
    if len(sys.argv) > 1 and sys.argv[1] == "set":  # one 64-view set (the bench's launch); the first 64k blocks
        gen = torch.Generator(device=dev).manual_seed(7)
        settings = [bench.settings_for(rep, cm, bg0) for cm in cams]
        bg_img = torch.rand((64, 1024, 1024, 3), generator=gen, device=dev)
        ups = [torch.randn((64, 3, 1024, 1024), generator=gen, device=dev),
               torch.randn((64, 1, 1024, 1024), generator=gen, device=dev),
               torch.randn((64, 1, 1024, 1024), generator=gen, device=dev)]
        for _ in range(2):
            c, d, a, _ = bench.render_views(rep, settings, bg_img)
            torch.autograd.backward((c, d, a), ups)
            rep.zero_grad()
        torch.cuda.synchronize()
        res = {}
        nbs = 65536
        for which, name in ((0, "k_render_fwd"), (1, "k_render_bwd")):
            buf = np.zeros((nbs, 4), np.uint32)
            assert lib.gsr_diag_timeline(which, buf.ctypes.data, nbs) == 0
            res[name] = summarise(buf, name)
        out.append({"view": "set of 64 (first 65536 blocks)", **res})
    for vi in (0, 40):
        for rep_i in range(2):  # second pass = warm
            c, d, a, _ = bench.render_view(rep, cams[vi], bg0, bgc)
            loss = (c * 0.1).sum() + (d * 0.01).sum() + a.sum()
            loss.backward()
            rep.zero_grad()
        torch.cuda.synchronize()
        res = {}
        # (one view: the quadrant-wave forward has 16 blocks per super-tile, the backward 4; only the
        # launched blocks are read, later slots may hold an earlier, larger launch's stamps)
        for which, name, n in ((0, "k_render_fwd", nb), (1, "k_render_bwd", nb // 4)):
            buf = np.zeros((n, 4), np.uint32)
            assert lib.gsr_diag_timeline(which, buf.ctypes.data, n) == 0
            res[name] = summarise(buf, name)
        out.append({"view": vi, **res})
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "timeline.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

"""Per-block phase stamps of the compaction / depth sort / emission / tile sort kernels
(diagnostic build: `make -C threestudio-3dgs_amd/csrc diag`).

For each kernel (the last launch of its kind in one forward of the benchmark view): span, block start
spread, and per-phase durations (local work, look-back, write-out) as percentiles, plus the
look-back time vs ticket id.  Usage (GPU box):  python profiles/diag_sort.py
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

KINDS = {0: ("compact", "gsr_diag_phases_bin"), 1: ("sort_depth_last", "gsr_diag_phases_sort"),
         2: ("sort_tile_last", "gsr_diag_phases_sort"), 3: ("duplicate", "gsr_diag_phases_bin")}


def pct(x):
    return [round(float(np.percentile(x, p)), 2) for p in (0, 50, 90, 100)] if len(x) else None


def main():
    lib = _C.load_library()
    dev = torch.device("cuda", 0)
    scene = gs.make_scene(int(os.environ.get("DIAG_N", "1000000")), sh_degree=3, seed=0)
    rep = bench.Replica(scene, dev)
    cams = bench.build_views(64, 1024, dev)
    bg0 = torch.zeros(3, device=dev)
    bgc = torch.tensor([0.5, 0.5, 0.5], device=dev)
    with torch.no_grad():
        for _ in range(3):
            bench.render_view(rep, cams[0], bg0, bgc)
    torch.cuda.synchronize()
    out = {}
    for kind, (name, fn) in KINDS.items():
        f = getattr(lib, fn)
        f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        buf = np.zeros((8192, 2, 4), np.uint32)
        assert f(kind, buf.ctypes.data, 8192) == 0
        rec = buf[buf[:, 0, 3] != 0]
        if not len(rec):
            continue
        rec = rec[np.argsort(rec[:, 1, 2])]
        t = rec[:, 0, :].astype(np.int64)
        t0 = t[:, 0].min()
        t = (t - t0) * 10 / 1000.0  # us
        xcc = rec[:, 1, 1]
        out[name] = {
            "blocks": int(len(rec)), "span_us": round(float(t[:, 3].max()), 2),
            "start_us": pct(t[:, 0]), "local_us": pct(t[:, 1] - t[:, 0]), "lookback_us": pct(t[:, 2] - t[:, 1]),
            "write_us": pct(t[:, 3] - t[:, 2]),
            "lookback_end_vs_ticket": [round(float(x), 2) for x in t[:: max(1, len(t) // 16), 2]],
            "blocks_per_xcd": [int((xcc == x).sum()) for x in range(8)],
        }
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "diag_sort.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

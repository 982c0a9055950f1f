"""Device-counted (pixel, Gaussian) pairs of the blend kernels on the benchmark workload (diagnostic build,
`make -C threestudio-3dgs_amd/csrc diag`): one 64-view set of bench.py's default workload (1M Gaussians,
1024^2, SH3, fused background composite) forward + backward through rasterize_views, then the counters
of gsr_diag_pairs.  Writes gpurun_out/pairs_<tag>.json (copy to profiles/<tag>_pairs.json); bench.py
reads it for the VALU roofline.  Usage (GPU box):  python profiles/diag_pairs.py <tag> [workload]"""
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


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    lib = _C.load_library()
    lib.gsr_diag_pairs.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    workload = sys.argv[2] if len(sys.argv) > 2 else "c3"
    V, R = 64, (800 if workload == "sugar" else 1024)
    scene = gs.make_sugar_scene(7, sh_degree=3, seed=0) if workload == "sugar" else \
        gs.make_scene(1_000_000, sh_degree=3, seed=0)
    rep = bench.Replica(scene, dev)
    cams = bench.build_views(V, R, dev)
    bg0 = torch.zeros(3, device=dev)
    settings = [bench.settings_for(rep, c, bg0) for c in cams]
    gen = torch.Generator(device=dev).manual_seed(7)
    bg_img = torch.rand((V, R, R, 3), generator=gen, device=dev)
    ups = [torch.randn((V, 3, R, R), generator=gen, device=dev), torch.randn((V, 1, R, R), generator=gen, device=dev),
           torch.randn((V, 1, R, R), generator=gen, device=dev)]
    buf = np.zeros(7, np.uint64)
    for it in range(2):  # the second pass is the counted one
        assert lib.gsr_diag_pairs(buf.ctypes.data, 1) == 0
        _C.RECENT_LISTED.clear()
        if workload == "sugar":
            shade = bench.shading_inputs(cams, dev)
            outs = bench.render_views_sugar(rep, settings, shade)
            torch.autograd.backward(outs, (ups[0], ups[1], ups[2], ups[0], ups[0]))
        else:
            c, d, a, _ = bench.render_views(rep, settings, bg_img)
            torch.autograd.backward((c, d, a), ups)
        rep.zero_grad()
        torch.cuda.synchronize()
    assert lib.gsr_diag_pairs(buf.ctypes.data, 1) == 0
    listed = float(np.mean(list(_C.RECENT_LISTED)))
    out = {
        "workload": (f"bench.py --workload sugar: {scene['means3D'].shape[0]} SuGaR Gaussians, {R}x{R}, two passes "
                     f"(colours, normals), {V}-view set" if workload == "sugar" else
                     f"bench.py default: 1M Gaussians, {R}x{R}, SH3, {V}-view set, fused background composite"),
        "views": V,
        "build_id": _C.build_id(lib),  # the sources the counted kernels were built from (bench.py checks it)
        "fwd_pairs_evaluated_per_view": float(buf[0]) / V,
        "fwd_pair_slots_per_view": float(buf[1]) / V,
        "bwd_pairs_replayed_per_view": float(buf[2]) / V,
        "bwd_lockstep_pair_slots_per_view": float(buf[3]) / V,
        "bwd_lockstep_slots_per_kept_pair": float(buf[3]) / max(1.0, float(buf[2])),
        # lower bound of any batch-level rebalancing (ring, larger batches): the tile's busiest quadrant
        "bwd_tile_bound_slots_per_kept_pair": float(buf[4]) / max(1.0, float(buf[2])),
        "mean_listed_instances": listed,
        # backward blend: candidates staged (every listed instance before the tile's deepest blended one) and
        # those at least one quadrant keeps (the rest are gathered, culled and given a zero row)
        "bwd_staged_candidates_per_view": float(buf[5]) / V,
        "bwd_kept_candidates_per_view": float(buf[6]) / V,
        "note": "fwd evaluated = (pixel, candidate) iterations of lanes not yet terminated; slots include "
                "terminated lanes; bwd pairs = kept (candidate, 8x8 quadrant) pairs x 64 pixels",
    }
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"pairs_{tag}{'_sugar' if workload == 'sugar' else ''}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

"""Diagnostic (GPU box): the two-colour hit-list backward as one wave per tile (GSR_BWD_KERNEL=tile) vs the
lockstep quadrant waves (quadrant) on the test_forward_kernels_bitwise[sugar_two_colors] scene: per gradient
tensor the number of differing elements and the largest difference, and the first differing Gaussians."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "threestudio-3dgs_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

from gsr_testutil import gs, make_camera  # noqa: E402


def main():
    from diff_gaussian_rasterization.batched import rasterize_views
    from test_gpu_configs import _settings

    two = len(sys.argv) < 2 or sys.argv[1] == "two"
    os.environ["GSR_BWD_SUMS"] = "hits" if two or (len(sys.argv) > 2 and sys.argv[2] == "hits") else "mfma"
    os.environ["GSR_BWD_SPLIT"] = "0"
    dev = "cuda"
    scene = gs.make_sugar_scene(5, sh_degree=0, seed=3)
    W_, H_ = 256, 256
    rng = np.random.default_rng(8)
    cams = [make_camera(W_, H_, elevation=12.0 * i, azimuth=55.0 * i + 5.0) for i in range(3)]
    ups = [torch.tensor(rng.standard_normal((3, 3, H_, W_)).astype(np.float32), device=dev) for _ in range(3)]

    def run(kernel):
        os.environ["GSR_BWD_KERNEL"] = kernel
        P = scene["means3D"].shape[0]
        t = {k: torch.tensor(scene[k], device=dev, requires_grad=True)
             for k in ("means3D", "scales", "rotations", "opacities", "shs")}
        m2 = [torch.zeros((P, 3), device=dev, requires_grad=True) for _ in cams]
        st = [_settings(c, [0.1, 0.2, 0.3], int(scene["sh_degree"])) for c in cams]
        common = dict(opacities=t["opacities"], scales=t["scales"], rotations=t["rotations"])
        if two:
            t["normals"] = torch.tensor(scene["normals"], device=dev, requires_grad=True)
            outs = rasterize_views(st, t["means3D"], m2, shs=t["shs"], colors2=t["normals"], **common)
        else:
            outs = rasterize_views(st, t["means3D"], m2, shs=t["shs"], **common)
        c, r, d, a = outs[:4]
        loss = (c * ups[0]).sum() + (d * ups[1][:, :1]).sum() + (a * ups[1][:, 1:2]).sum()
        if len(outs) > 4:
            loss = loss + (outs[4] * ups[2]).sum()
        loss.backward()
        res = {f"m2_{i}": m.grad.clone() for i, m in enumerate(m2)}
        res.update({k: v.grad.clone() for k, v in t.items()})
        return res

    for rep in range(2):
        a, b = run("tile"), run("quadrant")
        b2 = run("quadrant")
        for k in a:
            x, y, y2 = a[k].double(), b[k].double(), b2[k].double()
            diff = (x - y).abs()
            rows = torch.nonzero(diff.reshape(diff.shape[0], -1).amax(1) > 0).flatten()
            print(f"[{rep}] {k:10s} tile-vs-quad differing elements {int((diff > 0).sum())} max {float(diff.max()):.3e}"
                  f"  quad-vs-quad max {float((y - y2).abs().max()):.3e}  rows {rows[:8].tolist()}")


if __name__ == "__main__":
    main()

"""``simple_knn._C.distCUDA2`` over the C ABI (include/gsr.h gsr_knn_mean_dist, csrc/gsr_knn.hip).

The reference initialises Gaussian scales from the point cloud (geometry/gaussian_base.py:434-438):

    dist2 = torch.clamp_min(distCUDA2(torch.from_numpy(np.asarray(pcd.points)).float().cuda()), 0.0000001)

``distCUDA2(points)`` takes a float (P, 3) GPU tensor and returns the (P,) float tensor of mean squared
distances to each point's 3 nearest other points, like the external graphdeco-inria/simple-knn
extension.  The workspace comes from the PyTorch caching allocator; the kernels run on the current
stream.  No CPU path: a CPU tensor or a missing library raises.
"""
from __future__ import annotations

import torch

from diff_gaussian_rasterization import _C as _gsr

__all__ = ["distCUDA2"]


def distCUDA2(points: torch.Tensor) -> torch.Tensor:
    if not isinstance(points, torch.Tensor) or points.dim() != 2 or points.shape[1] != 3:
        raise ValueError("distCUDA2 expects a (P, 3) tensor")
    dev = points.device
    _gsr._require_gpu(dev)
    lib = _gsr.load_library()
    pts = _gsr._f32(points, "points", dev)
    P = points.shape[0]
    out = torch.empty((P,), dtype=torch.float32, device=dev)
    if P == 0:
        return out
    nbytes = int(lib.gsr_knn_workspace_bytes(P))
    ws = torch.empty((nbytes,), dtype=torch.uint8, device=dev)
    _gsr._check(lib.gsr_knn_mean_dist(P, _gsr._ptr(pts), _gsr._ptr(out), _gsr._ptr(ws), nbytes,
                                      _gsr._stream(dev)))
    return out

"""ctypes binding of libgsr_hip.so (include/gsr.h) exposing the reference extension's entry points.

The reference imports the pybind module ``diff_gaussian_rasterization._C`` (external, ashawkey
4-output fork; call sites e.g. renderer/diff_gaussian_rasterizer_background.py:119-128 through the
Python wrapper).  This module provides the same three functions with the same argument order and
return tuples, implemented over the C ABI:

    rasterize_gaussians(...)          -> (num_rendered, color, depth, alpha, radii, geomBuf, binningBuf, imgBuf)
    rasterize_gaussians_backward(...) -> (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D,
                                          dL_dcov3D, dL_dsh, dL_dscales, dL_drotations)
    mark_visible(means3D, viewmatrix, projmatrix) -> bool (P,)

All buffers are torch tensors from the caching allocator on ``means3D.device``; kernels run on the
current HIP stream.  There is no CPU fallback: a missing library or a non-GPU tensor raises.
"""
from __future__ import annotations

import collections
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GSR_HIP_LIB", os.path.join(_HERE, "libgsr_hip.so"))

_lib = None

_vp = ctypes.c_void_p
_i = ctypes.c_int
_f = ctypes.c_float
_sz = ctypes.c_size_t

# name -> (restype, argtypes); must match include/gsr.h exactly (checked by tests/test_abi.py)
SIGNATURES = {
    "gsr_version": (ctypes.c_char_p, []),
    "gsr_abi_version": (_i, []),
    "gsr_last_error": (ctypes.c_char_p, []),
    "gsr_geom_bytes": (_sz, [_i]),
    "gsr_binning_bytes": (_sz, [_i, _i, _i]),
    "gsr_image_bytes": (_sz, [_i, _i]),
    "gsr_backward_bytes": (_sz, [_i, _i]),
    "gsr_forward_preprocess": (
        _i,
        [_i, _i, _i, _vp, _vp, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _f, _f, _i, _vp, _vp, _vp],
    ),
    "gsr_num_rendered": (_i, [_vp, _i, ctypes.POINTER(_i), ctypes.POINTER(_i), _vp]),
    "gsr_forward_render": (_i, [_i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gsr_backward": (
        _i,
        [_i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f, _f,
         _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    ),
    "gsr_mark_visible": (_i, [_i, _vp, _vp, _vp, _vp, _vp]),
    "gsr_composite_forward": (_i, [_i, _i, _i, _vp, _vp, _vp, _i, _vp, _vp]),
    "gsr_composite_backward": (_i, [_i, _i, _i, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp]),
    "gsr_normal_map_forward": (_i, [_i, _i, _i, _vp, _vp, _vp, _vp]),
    "gsr_normal_map_backward": (_i, [_i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gsr_shade_forward": (_i, [_i, _i, _i, _i, _i] + [_vp] * 6 + [_i] + [_vp] * 8 + [_vp]),
    "gsr_shade_backward": (_i, [_i, _i, _i, _i, _i] + [_vp] * 6 + [_i] + [_vp] * 12 + [_vp]),
    "gsr_shade_views_forward": (_i, [_i, _i, _i, _i, ctypes.POINTER(_i)] + [_vp] * 6 + [_i] + [_vp] * 2
                                + [ctypes.POINTER(_f)] * 2 + [_vp] * 4 + [_vp]),
    "gsr_shade_views_backward": (_i, [_i, _i, _i, _i, ctypes.POINTER(_i)] + [_vp] * 6 + [_i] + [_vp] * 2
                                 + [ctypes.POINTER(_f)] * 2 + [_vp] * 8 + [_vp]),
    "gsr_sort_work_bytes": (_sz, [_i, ctypes.POINTER(_i)]),
    "gsr_sort_pairs": (_i, [_i, ctypes.POINTER(_i), _vp, _vp, _i, _i, _vp, _sz, _vp]),
    "gsr_sort_rank_mode": (_i, []),
    "gsr_knn_workspace_bytes": (_sz, [_i]),
    "gsr_knn_mean_dist": (_i, [_i, _vp, _vp, _vp, _sz, _vp]),
    "gsr_set_geom_bytes": (_sz, [_i, _i]),
    "gsr_set_binning_bytes": (_sz, [_i, _i, ctypes.POINTER(_i), _i, _i]),
    "gsr_set_image_bytes": (_sz, [_i, _i, _i]),
    "gsr_set_image_bytes_ex": (_sz, [_i, _i, ctypes.POINTER(_i), _i, _i, _i]),
    "gsr_profile_kernel": (ctypes.c_char_p, [_i]),
    "gsr_set_backward_bytes": (_sz, [_i, _i, ctypes.POINTER(_i)]),
    "gsr_set_preprocess": (
        _i,
        [_i, _i, _i, _i, _vp, _vp, _f, _vp, _vp, _vp, _vp, _vp] + [ctypes.POINTER(_vp)] * 3
        + [ctypes.POINTER(_f)] * 2 + [_i, _i, _i, _vp, _vp, _vp],
    ),
    "gsr_set_preprocess_ex": (
        _i,
        [_i, _i, _i, _i, _vp, _vp, _f, _vp, _vp, _vp, _vp, _vp] + [ctypes.POINTER(_vp)] * 3
        + [ctypes.POINTER(_f)] * 2 + [_i, _i, _i, _vp, _vp, _vp, _vp],
    ),
    "gsr_set_num_rendered": (_i, [_i, _vp, _i, ctypes.POINTER(_i), ctypes.POINTER(_i), _vp]),
    "gsr_set_num_rendered_ex": (_i, [_i, _vp, _i, ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.POINTER(_i), _vp]),
    "gsr_set_gauss_state": (_i, [_i, _vp, _i, _vp, _vp, _vp]),
    "gsr_set_render": (_i, [_i, _i, ctypes.POINTER(_i), _i, _i, ctypes.POINTER(_vp)] + [_vp] * 7),
    "gsr_set_backward": (
        _i,
        [_i, _i, _i, _i, ctypes.POINTER(_i), _i, _i, ctypes.POINTER(_vp), _vp, _vp, _f, _vp, _vp, _vp]
        + [ctypes.POINTER(_vp)] * 3 + [ctypes.POINTER(_f)] * 2 + [_vp] * 4 + [_vp] * 3 + [_vp] * 8
        + [_i, _vp, _sz, _vp],
    ),
    "gsr_set_render_composite": (_i, [_i, _i, ctypes.POINTER(_i), _i, _i, ctypes.POINTER(_vp)] + [_vp] * 9),
    "gsr_set_backward_composite": (
        _i,
        [_i, _i, _i, _i, ctypes.POINTER(_i), _i, _i, ctypes.POINTER(_vp), _vp, _vp, _f, _vp, _vp, _vp]
        + [ctypes.POINTER(_vp)] * 3 + [ctypes.POINTER(_f)] * 2 + [_vp] * 4 + [_vp] * 6 + [_vp] * 8
        + [_i, _vp, _sz, _vp],
    ),
    "gsr_set_render_two_colors": (_i, [_i, _i, ctypes.POINTER(_i), _i, _i, ctypes.POINTER(_vp)] + [_vp] * 11),
    "gsr_set_backward_two_colors_bytes": (_sz, [_i, _i, ctypes.POINTER(_i)]),
    "gsr_set_backward_two_colors": (
        _i,
        [_i, _i, _i, _i, ctypes.POINTER(_i), _i, _i, ctypes.POINTER(_vp), _vp, _vp, _f, _vp, _vp, _vp]
        + [ctypes.POINTER(_vp)] * 3 + [ctypes.POINTER(_f)] * 2 + [_vp] * 4 + [_vp] * 8 + [_vp] * 9
        + [_i, _vp, _sz, _vp],
    ),
    "gsr_set_backward_colors": (
        _i,
        [_i, _i, ctypes.POINTER(_i), _i, _i, ctypes.POINTER(_vp), _vp, _vp, _f, _vp, _vp]
        + [ctypes.POINTER(_vp)] * 3 + [ctypes.POINTER(_f)] * 2 + [_vp] * 4 + [_vp] * 2 + [_vp] * 7
        + [_i, _vp, _sz, _vp],
    ),
    "gsr_set_backward_chunks": (_i, [_i, ctypes.POINTER(_vp)]),
    "gsr_grad_chunk_range": (_i, [_i, _i, _i, ctypes.POINTER(_i), ctypes.POINTER(_i)]),
    "gsr_profile_enable": (_i, [_i]),
    "gsr_profile_read": (_i, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong), _i]),
}

PHASES = ("preprocess", "depth_sort", "binning", "render_fwd", "render_bwd", "gauss_bwd")
# (num_rendered, H, W) of the most recent forward calls, for instrumentation (bench.py roofline numbers)
RECENT_FORWARDS: collections.deque = collections.deque(maxlen=4096)
# tests set KEEP_GEOM to keep the last per-view forward's geometry buffer in LAST_GEOM (gauss_state)
KEEP_GEOM = False
LAST_GEOM = None
# instances the tile lists held (after the exact tile culling) for recent batched forwards
RECENT_LISTED: collections.deque = collections.deque(maxlen=4096)


class GSRError(RuntimeError):
    pass


# Host-side time of the rasterizer's Python phases (GSR_HOST_TRACE=1; bench.py reports it): seconds per
# phase name, accumulated until host_trace_read(reset=True).  Off: one attribute test per phase.
HOST_TRACE = os.environ.get("GSR_HOST_TRACE") == "1"
_HOST = collections.defaultdict(float)


def host_mark(name: str, t0: float) -> float:
    """Add the time since t0 to phase `name`; returns now (the next phase's t0)."""
    import time

    now = time.perf_counter()
    if HOST_TRACE:
        _HOST[name] += now - t0
    return now


def host_trace_read(reset: bool = True) -> dict:
    out = dict(_HOST)
    if reset:
        _HOST.clear()
    return out


ABI_VERSION = 5  # include/gsr.h GSR_ABI_VERSION this binding is written against


def load_library(path: str | None = None):
    """Load (once) and type the C-ABI library.  Raises ImportError if it is missing or of another ABI."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise ImportError(
            f"diff_gaussian_rasterization: HIP library not found at {p}; "
            "build it with `make -C threestudio-3dgs_amd/csrc` (or __graft_entry__.build())"
        )
    lib = ctypes.CDLL(p)
    abi = getattr(lib, "gsr_abi_version", None)
    got = abi() if abi is not None else 1
    if got != ABI_VERSION:
        raise ImportError(f"diff_gaussian_rasterization: {p} has C-ABI revision {got}, this binding needs "
                          f"{ABI_VERSION}; rebuild it with `make -C threestudio-3dgs_amd/csrc`")
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def _check(rc: int):
    if rc != 0:
        msg = load_library().gsr_last_error().decode(errors="replace")
        if rc == 1:
            raise GSRError(msg)
        raise GSRError(f"HIP failure: {msg}")


def _ptr(t):
    if t is None or t.numel() == 0:
        return None
    return ctypes.c_void_p(t.data_ptr())


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _f32(t, name, device):
    if t is None or t.numel() == 0:
        return None
    if not t.is_cuda:
        raise GSRError(f"{name} must be a GPU tensor (the rasterizer has no CPU path)")
    if t.device != device:
        raise GSRError(f"{name} is on {t.device}, expected {device}")
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


def _require_gpu(device):
    if device.type != "cuda":
        raise GSRError("diff_gaussian_rasterization requires tensors on a ROCm GPU (device 'cuda')")


def sh_coeff_count(sh) -> int:
    return 0 if sh is None or sh.numel() == 0 else int(sh.shape[1])


def rasterize_gaussians(bg, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                        viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree,
                        campos, prefiltered, debug):
    """Forward pass; argument order of the reference's _C.rasterize_gaussians."""
    if means3D.dim() != 2 or means3D.size(1) != 3:
        raise GSRError("means3D must have dimensions (num_points, 3)")
    device = means3D.device
    _require_gpu(device)
    lib = load_library()
    P = int(means3D.size(0))
    H, W = int(image_height), int(image_width)
    fopt = dict(dtype=torch.float32, device=device)
    u8 = dict(dtype=torch.uint8, device=device)
    if P == 0:
        return (0, torch.zeros((3, H, W), **fopt), torch.zeros((1, H, W), **fopt), torch.zeros((1, H, W), **fopt),
                torch.zeros((0,), dtype=torch.int32, device=device), torch.empty(0, **u8), torch.empty(0, **u8),
                torch.empty(0, **u8))
    # (no zero fill: the preprocess writes every radius and the blend every pixel, as on the batched path)
    out_color = torch.empty((3, H, W), **fopt)
    out_depth = torch.empty((1, H, W), **fopt)
    out_alpha = torch.empty((1, H, W), **fopt)
    radii = torch.empty((P,), dtype=torch.int32, device=device)

    means3D = _f32(means3D, "means3D", device)
    colors = _f32(colors, "colors_precomp", device)
    opacity = _f32(opacity, "opacities", device)
    scales = _f32(scales, "scales", device)
    rotations = _f32(rotations, "rotations", device)
    cov3D_precomp = _f32(cov3D_precomp, "cov3D_precomp", device)
    sh = _f32(sh, "sh", device)
    view = _f32(viewmatrix, "viewmatrix", device)
    proj = _f32(projmatrix, "projmatrix", device)
    cam = _f32(campos, "campos", device)
    bg = _f32(bg, "bg", device)
    M = sh_coeff_count(sh)
    for name, t, n in (("opacities", opacity, P), ("scales", scales, 3 * P), ("rotations", rotations, 4 * P),
                       ("colors_precomp", colors, 3 * P), ("cov3D_precomp", cov3D_precomp, 6 * P),
                       ("sh", sh, 3 * M * P)):
        if t is not None and t.numel() != n:
            raise GSRError(f"{name} has {t.numel()} elements, expected {n}")
    if view is None or view.numel() != 16 or proj is None or proj.numel() != 16:
        raise GSRError("viewmatrix and projmatrix must be 4x4")
    if cam is None or cam.numel() != 3 or bg is None or bg.numel() != 3:
        raise GSRError("campos and bg must have 3 elements")

    stream = _stream(device)
    geom = torch.empty(int(lib.gsr_geom_bytes(P)), **u8)
    _check(lib.gsr_forward_preprocess(
        P, int(degree), M, _ptr(means3D), _ptr(scales), float(scale_modifier), _ptr(rotations), _ptr(opacity),
        _ptr(sh), _ptr(colors), _ptr(cov3D_precomp), _ptr(view), _ptr(proj), _ptr(cam), W, H,
        float(tan_fovx), float(tan_fovy), int(bool(prefiltered)), _ptr(radii), _ptr(geom), stream))
    K = ctypes.c_int(0)
    nvis = ctypes.c_int(0)
    _check(lib.gsr_num_rendered(_ptr(geom), P, ctypes.byref(K), ctypes.byref(nvis), stream))
    num_rendered = int(K.value)
    RECENT_FORWARDS.append((num_rendered, H, W))
    if KEEP_GEOM:
        global LAST_GEOM
        LAST_GEOM = geom
    binning = torch.empty(int(lib.gsr_binning_bytes(num_rendered, W, H)), **u8)
    # sized for this forward's split decision (no split checkpoints unless the forward writes them)
    image = torch.empty(int(lib.gsr_set_image_bytes_ex(1, P, (ctypes.c_int * 1)(num_rendered), W, H, 0)), **u8)
    _check(lib.gsr_forward_render(P, num_rendered, W, H, _ptr(bg), _ptr(geom), _ptr(binning), _ptr(image),
                                  _ptr(out_color), _ptr(out_depth), _ptr(out_alpha), stream))
    return num_rendered, out_color, out_depth, out_alpha, radii, geom, binning, image


def rasterize_gaussians_backward(bg, means3D, radii, colors, scales, rotations, scale_modifier, cov3D_precomp,
                                 viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, dL_dout_depth,
                                 dL_dout_alpha, sh, degree, campos, geomBuffer, R, binningBuffer, imageBuffer,
                                 alpha, debug):
    """Backward pass; argument order and return tuple of the reference's _C.rasterize_gaussians_backward."""
    device = means3D.device
    _require_gpu(device)
    lib = load_library()
    P = int(means3D.size(0))
    H, W = int(dL_dout_color.size(1)), int(dL_dout_color.size(2))
    M = sh_coeff_count(sh)
    fopt = dict(dtype=torch.float32, device=device)
    dL_dmeans3D = torch.zeros((P, 3), **fopt) if P == 0 else torch.empty((P, 3), **fopt)
    dL_dmeans2D = torch.zeros((P, 3), **fopt) if P == 0 else torch.empty((P, 3), **fopt)
    dL_dcolors = torch.zeros((P, 3), **fopt) if P == 0 else torch.empty((P, 3), **fopt)
    dL_dopacity = torch.zeros((P, 1), **fopt) if P == 0 else torch.empty((P, 1), **fopt)
    dL_dcov3D = torch.zeros((P, 6), **fopt) if P == 0 else torch.empty((P, 6), **fopt)
    dL_dsh = torch.zeros((P, M, 3), **fopt) if (P == 0 or M == 0) else torch.empty((P, M, 3), **fopt)
    # (written whole by the kernels unless cov3D_precomp replaces scales / rotations)
    pre = cov3D_precomp is not None and cov3D_precomp.numel() > 0
    dL_dscales = torch.zeros((P, 3), **fopt) if (P == 0 or pre) else torch.empty((P, 3), **fopt)
    dL_drotations = torch.zeros((P, 4), **fopt) if (P == 0 or pre) else torch.empty((P, 4), **fopt)
    if P == 0:
        return dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations

    means3D = _f32(means3D, "means3D", device)
    scales = _f32(scales, "scales", device)
    rotations = _f32(rotations, "rotations", device)
    cov3D_precomp = _f32(cov3D_precomp, "cov3D_precomp", device)
    sh = _f32(sh, "sh", device)
    colors = _f32(colors, "colors_precomp", device)
    view = _f32(viewmatrix, "viewmatrix", device)
    proj = _f32(projmatrix, "projmatrix", device)
    cam = _f32(campos, "campos", device)
    bg = _f32(bg, "bg", device)
    gc = _f32(dL_dout_color, "dL_dout_color", device)
    gd = _f32(dL_dout_depth, "dL_dout_depth", device)
    ga = _f32(dL_dout_alpha, "dL_dout_alpha", device)
    if radii.dtype != torch.int32:
        radii = radii.int()
    radii = radii.contiguous()
    K = int(R)
    stream = _stream(device)
    work = torch.empty(int(lib.gsr_backward_bytes(P, K)), dtype=torch.uint8, device=device)
    _check(lib.gsr_backward(
        P, int(degree), M, K, W, H, _ptr(bg), _ptr(means3D), _ptr(scales), float(scale_modifier), _ptr(rotations),
        None, _ptr(sh), _ptr(colors), _ptr(cov3D_precomp), _ptr(view), _ptr(proj), _ptr(cam),
        float(tan_fovx), float(tan_fovy), _ptr(radii), _ptr(geomBuffer), _ptr(binningBuffer), _ptr(imageBuffer),
        _ptr(gc), _ptr(gd), _ptr(ga), _ptr(dL_dmeans2D), _ptr(dL_dcolors), _ptr(dL_dopacity), _ptr(dL_dmeans3D),
        _ptr(dL_dcov3D), _ptr(dL_dsh), _ptr(dL_dscales), _ptr(dL_drotations), _ptr(work), stream))
    return dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations


def mark_visible(means3D, viewmatrix, projmatrix):
    device = means3D.device
    _require_gpu(device)
    lib = load_library()
    P = int(means3D.size(0))
    present = torch.zeros((P,), dtype=torch.uint8, device=device)
    if P > 0:
        _check(lib.gsr_mark_visible(P, _ptr(_f32(means3D, "means3D", device)), _ptr(_f32(viewmatrix, "viewmatrix", device)),
                                    _ptr(_f32(projmatrix, "projmatrix", device)), _ptr(present), _stream(device)))
    return present.bool()


def gauss_state(geom, V: int, P: int):
    """Preprocess state of a view set's geometry buffer (include/gsr.h gsr_set_gauss_state): returns
    (rec (V, P, 16) float32 — integer words viewed as float bits —, tiles (V, P, 2) int32) on the device."""
    lib = load_library()
    dev = geom.device
    rec = torch.zeros((V, P, 16), dtype=torch.float32, device=dev)
    tiles = torch.zeros((V, P, 2), dtype=torch.int32, device=dev)
    _check(lib.gsr_set_gauss_state(V, _ptr(geom), P, _ptr(rec), _ptr(tiles), _stream(dev)))
    return rec, tiles


def profile_enable(on: bool = True):
    _check(load_library().gsr_profile_enable(1 if on else 0))


def profile_read(reset: bool = True) -> dict:
    """Accumulated per-phase kernel milliseconds and launch counts (HIP events on the launch stream)."""
    n = len(PHASES)
    ms = (ctypes.c_double * n)()
    cnt = (ctypes.c_longlong * n)()
    _check(load_library().gsr_profile_read(ms, cnt, 1 if reset else 0))
    return {PHASES[i]: (float(ms[i]), int(cnt[i])) for i in range(n)}


def build_id(lib=None) -> str:
    """The library's build id (include/gsr.h gsr_version: a hash of the sources it was built from, csrc/Makefile)."""
    v = (lib or load_library()).gsr_version().decode()
    return v.split(" build ", 1)[1] if " build " in v else "unknown"


def profile_kernels() -> dict:
    """The blend kernels the last forward / backward blend launches used (include/gsr.h gsr_profile_kernel), as
    rocprofv3 names them: {"render_fwd": ..., "render_bwd": ...}."""
    lib = load_library()
    return {PHASES[i]: lib.gsr_profile_kernel(i).decode() for i in (3, 4)}

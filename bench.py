#!/usr/bin/env python
"""Benchmark: rendered views/sec, forward+backward, 1M Gaussians, 1024^2, SH degree 3 (BASELINE.json).

A step is one pass of the hot path over one batch of views: every view of the batch is rendered
through the drop-in GaussianRasterizer API (preprocess, binning, forward blend), composited on a
per-view background image and clamped exactly like renderer/diff_gaussian_rasterizer_background.py:
129-132,139 (batched path: the fused HIP epilogue, diff_gaussian_rasterization/composite.py), the
rendered images are all-gathered across ranks (RCCL over xGMI; the north_star exchange), then the
backward runs from fixed seeded upstream gradients dL/d(image, depth, alpha) (a loss's gradient,
injected with torch.autograd.backward) through the composite and the rasterizer, and the
per-Gaussian parameter gradients are all-reduced (sum) so every replica holds the full-batch gradient.

Workload (BASELINE.json configs[2] / configs[3]): C3 per view (1M Gaussians, 1024^2,
SH3, background path: bg = 0, then composite with a (H, W, 3) background image + clamp) over the C4
64-view MVDream-style orbit batch
(4 elevations x 16 azimuths), views sharded across ranks (strong scaling: the 64-view batch is fixed).

Single GPU:  python bench.py [--steps K --warmup W]
N GPUs:      python bench.py --gpus N ...   (starts N ranks itself through torch.distributed.run), or
             python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
                 --master-port P bench.py --gpus N --steps K --warmup W
--gpus must equal the launched world size.  Rank 0 prints one JSON line; at N = 1 it carries the C5 (SuGaR
normal renderer) and 8-view-set lines as sub-objects (--extra-lines).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "threestudio-3dgs_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "rendered views/sec fwd+bwd @1M Gaussians, 1024², SH=3; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)
# VALU issue peak: 256 CUs x 4 SIMDs x 2.4 GHz, one wave64 fp32 instruction per SIMD every 4 cycles (MI355X_MICROARCH.md,
# measured issue cost of one wave's stream on one SIMD: v_fma_f32 / v_add_f32 4 cycles, v_exp_f32 / v_rcp_f32 8; the
# 157.3 TFLOP/s fp32 peak counts packed v_pk_fma_f32, two lanes' worth per instruction).  Until round 5 this was
# taken as 2 cycles, which halved every valu_frac.
VALU_PEAK_INSTS = 256 * 4 * 2.4e9 / 4
FP32_PEAK_TFLOPS = 157.3
SH_C0 = 0.28209479177387814


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--gaussians", type=int, default=1_000_000)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--views", type=int, default=64, help="global views per step (sharded over ranks)")
    ap.add_argument("--sh-degree", type=int, default=3)
    ap.add_argument("--cpu-views", type=int, default=3, help="views of the same workload timed on the CPU oracle")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-knn", action="store_true", help="skip the distCUDA2 timing line")
    ap.add_argument("--workload", choices=["c3", "sugar"], default="c3",
                    help="c3: the metric's scene (1M ball Gaussians, SH3); sugar: C5, ~2M surface-aligned SuGaR "
                         "Gaussians (icosphere, 6 per face), 800x800, the SuGaR normal renderer's two passes "
                         "(shs image + depth, then face normals as colors_precomp) with normal-from-depth")
    ap.add_argument("--epilogue", choices=["background", "shading"], default="background",
                    help="post-raster epilogue: the background renderer's composite (C3) or the MVDream shading "
                         "renderer's depth-normal + point-light material + composite")
    ap.add_argument("--path", choices=["batched", "per-view"], default="batched",
                    help="batched: rasterize_views (one autograd node per rank's views); per-view: one "
                         "GaussianRasterizer call per view, exactly as the reference renderer loop does")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "r06h_traffic.json"),
                    help="PMC summary (profiles/summarize.py) supplying roofline.traffic and the VALU counts")
    ap.add_argument("--pairs", default=os.path.join(ROOT, "profiles", "r06h_pairs.json"),
                    help="device-counted blend pairs (profiles/diag_pairs.py) for the VALU roofline")
    ap.add_argument("--traffic-sugar", default=os.path.join(ROOT, "profiles", "r06h_sugar_traffic.json"),
                    help="PMC summary of the C5 line (--workload sugar, profiles/summarize.py r06h_sugar)")
    ap.add_argument("--fused-clamp", choices=["on", "off"], default="on",
                    help="C5: the renderer's render.clamp(0, 1) formed in the blends (rasterize_views clamp=True) "
                         "or by torch on the colour output (off: the A/B baseline)")
    ap.add_argument("--overlap-reduce", choices=["on", "off"], default="on",
                    help="N > 1: sum the Gaussian gradients over ranks inside the backward, range by range as the "
                         "per-Gaussian backward forms them (view_shard.ChunkedGradReduce, overlapped on a side "
                         "stream) instead of one flat all-reduce after it")
    ap.add_argument("--grad-chunks", type=int, default=4, help="Gaussian ranges of the overlapped reduction")
    ap.add_argument("--gather", choices=["overlap", "sync"], default="sync",
                    help="N > 1: the image all-gather completes before the backward (sync, the headline: the "
                         "reference's guidance consumes the gathered comp_rgb before loss.backward(), "
                         "system/gaussian_splatting.py:65-67,129), or runs asynchronously beside it (overlap: valid "
                         "when the loss decomposes over views or rank-aligned view groups; with sync the overlapped "
                         "variant is timed after the headline and reported as gather_overlap)")
    ap.add_argument("--extra-lines", default="c5,views8",
                    help="N = 1, default workload: secondary workloads timed after the headline and reported as "
                         "sub-objects (c5: BASELINE configs[4], the SuGaR normal renderer; views8: a rank's 8-view "
                         "share of the batch at N = 8); 'none' to skip")
    ap.add_argument("--per-view-views", type=int, default=16,
                    help="views of the drop-in per-view path (one GaussianRasterizer call per view, the "
                         "reference's loop) timed after the headline, reported beside it (0 = skip)")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class Replica:
    """Gaussian parameters (activated values, as the geometry getters return them) on one GPU."""

    def __init__(self, scene, device):
        def leaf(x):
            return torch.tensor(x, device=device, requires_grad=True)

        self.means3D = leaf(scene["means3D"])
        self.scales = leaf(scene["scales"])
        self.rotations = leaf(scene["rotations"])
        self.opacities = leaf(scene["opacities"])
        self.shs = leaf(scene["shs"])
        self.sh_degree = int(scene["sh_degree"])
        self.params = [self.means3D, self.scales, self.rotations, self.opacities, self.shs]
        if "normals" in scene:  # SuGaR: per-Gaussian face normals, rasterized as colors_precomp
            self.normals = leaf(scene["normals"])
            self.params.append(self.normals)

    def zero_grad(self):
        for p in self.params:
            p.grad = None


def build_views(n_views, res, device):
    from diff_gaussian_rasterization.cameras import get_cam_info_gaussian, orbit_c2w

    n_el = 4
    per = max(1, n_views // n_el)
    elev = torch.tensor([[0.0, 10.0, 20.0, 30.0][(i // per) % n_el] for i in range(n_views)])
    azim = torch.tensor([(i % per) * 360.0 / per for i in range(n_views)])
    fovy = math.radians(60.0)
    c2w = orbit_c2w(torch.full((n_views,), 2.5), elev, azim)
    wv, fp, cc = get_cam_info_gaussian(c2w, fovy, fovy, 0.1, 100.0)
    tan = math.tan(fovy * 0.5)
    return [dict(view=wv[i].to(device), proj=fp[i].to(device), campos=cc[i].to(device), tan=tan, H=res, W=res,
                 c2w=c2w[i], fovy=fovy) for i in range(n_views)]


def shading_inputs(cams, device):
    """Rays and light positions of the views (the MVDream data module's batch, data/uncond.py:316-344)."""
    from diff_gaussian_rasterization.cameras import light_positions_dreamfusion, ray_bundle

    c2w = torch.stack([c["c2w"] for c in cams])
    rays_o, rays_d = ray_bundle(c2w, cams[0]["fovy"], cams[0]["H"], cams[0]["W"])
    light = light_positions_dreamfusion(c2w, 2.0)
    return rays_o.to(device), rays_d.contiguous().to(device), light.to(device)


def render_view(rep: Replica, cam, bg_zero, bg_img, shade=None):
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer

    P = rep.means3D.shape[0]
    screenspace = torch.zeros((P, 3), device=rep.means3D.device, requires_grad=True) + 0
    s = GaussianRasterizationSettings(image_height=cam["H"], image_width=cam["W"], tanfovx=cam["tan"],
                                      tanfovy=cam["tan"], bg=bg_zero, scale_modifier=1.0,
                                      viewmatrix=cam["view"], projmatrix=cam["proj"], sh_degree=rep.sh_degree,
                                      campos=cam["campos"], prefiltered=False, debug=False)
    color, radii, depth, alpha = GaussianRasterizer(raster_settings=s)(
        means3D=rep.means3D, means2D=screenspace, shs=rep.shs, colors_precomp=None, opacities=rep.opacities,
        scales=rep.scales, rotations=rep.rotations, cov3D_precomp=None)
    H, W = cam["H"], cam["W"]
    if shade is not None:
        # the shading renderer's epilogue (renderer/diff_gaussian_rasterizer_shading.py:169-208) for this one view,
        # through the product's fused shading kernels (shading.shade_views)
        from diff_gaussian_rasterization.shading import shade_views

        rays_o, rays_d, light = shade
        render, normal, depth_m = shade_views(color, depth, alpha, rays_o, rays_d, bg_img, light, SHADE_KA,
                                              SHADE_KD, "diffuse")
        return render, depth_m, alpha, radii, normal
    # background path composite + clamp, the reference's torch lines
    # (renderer/diff_gaussian_rasterizer_background.py:129-132, 139)
    comp = (color + (1 - alpha) * bg_img.reshape(H, W, 3).permute(2, 0, 1)).clamp(0, 1)
    return comp, depth, alpha, radii


def settings_for(rep: Replica, cam, bg_zero):
    from diff_gaussian_rasterization import GaussianRasterizationSettings

    return GaussianRasterizationSettings(image_height=cam["H"], image_width=cam["W"], tanfovx=cam["tan"],
                                         tanfovy=cam["tan"], bg=bg_zero, scale_modifier=1.0,
                                         viewmatrix=cam["view"], projmatrix=cam["proj"], sh_degree=rep.sh_degree,
                                         campos=cam["campos"], prefiltered=False, debug=False)


def placeholders(rep: Replica, V: int):
    """The views' screen-space placeholders (renderer/diff_gaussian_rasterizer.py:73-81 creates one zero
    (P, 3) tensor per view): V leaves, each one zero broadcast to (P, 3) — their values are never read, so no
    (V, P, 3) fill; .grad is a dense (P, 3) tensor as for the reference's zeros."""
    zero = torch.zeros((1, 1), device=rep.means3D.device)
    return [zero.expand(rep.means3D.shape[0], 3).requires_grad_(True) for _ in range(V)]


COMPOSITE = os.environ.get("GSR_BENCH_COMPOSITE", "fused")  # "separate": gsr_composite_* as its own pass
SUGAR_SEPARATE = os.environ.get("GSR_BENCH_SUGAR_SEPARATE") == "1"  # C5: two separate rasterizer passes
SHADE_KA, SHADE_KD = (0.1, 0.1, 0.1), (0.9, 0.9, 0.9)  # the material's default ambient / diffuse colours


GRAD_REDUCE = None  # view_shard.ChunkedGradReduce when the reduction is overlapped with the backward (N > 1)
FUSED_CLAMP = True  # C5: the renderer's clamp formed in the blends (--fused-clamp)


def render_views(rep: Replica, settings, bg_img, shade=None):
    """The rank's views through rasterize_views; one means2D placeholder per view, as the renderer loop
    creates (renderer/diff_gaussian_rasterizer.py:73-81); the background composite + clamp of
    renderer/diff_gaussian_rasterizer_background.py:129-132,139 through the fused epilogue."""
    from diff_gaussian_rasterization.batched import rasterize_views
    from diff_gaussian_rasterization.composite import composite_background

    m2 = placeholders(rep, len(settings))
    if shade is not None:
        from diff_gaussian_rasterization.shading import shade_views

        color, radii, depth, alpha = rasterize_views(settings, rep.means3D, m2, rep.opacities, shs=rep.shs,
                                                     scales=rep.scales, rotations=rep.rotations,
                                                     grad_reduce=GRAD_REDUCE)
        rays_o, rays_d, light = shade
        render, normal, depth_m = shade_views(color, depth, alpha, rays_o, rays_d, bg_img, light,
                                              SHADE_KA, SHADE_KD, "diffuse")
        return render, depth_m, alpha, radii, normal
    if COMPOSITE == "separate":
        color, radii, depth, alpha = rasterize_views(settings, rep.means3D, m2, rep.opacities, shs=rep.shs,
                                                     scales=rep.scales, rotations=rep.rotations,
                                                     grad_reduce=GRAD_REDUCE)
        return composite_background(color, alpha, bg_img), depth, alpha, radii
    # the composite + clamp fused into the forward / backward blends (bit-identical to the separate pass)
    comp, radii, depth, alpha = rasterize_views(settings, rep.means3D, m2, rep.opacities, shs=rep.shs,
                                                scales=rep.scales, rotations=rep.rotations, background=bg_img,
                                                grad_reduce=GRAD_REDUCE)
    return comp, depth, alpha, radii


def render_views_sugar(rep: Replica, settings, shade):
    """C5: the SuGaR normal renderer (renderer/diff_sugar_rasterizer_normal.py:157-213) over a view set:
    pass 1 (colors_precomp = SH2RGB(dc), the SuGaR refinement's override_color) -> render, depth, alpha; normal-from-depth maps (fused HIP epilogue); pass 2 with
    the face normals as colors_precomp and a fresh zero means2D (no viewspace gradient, :179-189); then
    normalize, flip x/y, normal map and the alpha > 0.99 gradient masks in torch (:190-197)."""
    from diff_gaussian_rasterization.batched import rasterize_views
    from diff_gaussian_rasterization.shading import depth_normal_views, sugar_normal_map

    P = rep.means3D.shape[0]
    dev = rep.means3D.device
    m2 = placeholders(rep, len(settings))
    # pass 1 colours: SuGaRModel.get_points_rgb() = SH2RGB of the DC coefficients, passed as override_color
    # (system/sugar_static.py:117-121, geometry/sugar.py:650-660)
    colors = rep.shs[:, 0, :] * SH_C0 + 0.5
    if SUGAR_SEPARATE:  # the two rasterizer calls as two view-set renders (A/B of the shared-geometry path)
        color, radii, depth, alpha = rasterize_views(settings, rep.means3D, m2, rep.opacities, colors_precomp=colors,
                                                     scales=rep.scales, rotations=rep.rotations, clamp=True)
        zeros = [torch.zeros((P, 3), device=dev) for _ in settings]
        normal, _, _, _ = rasterize_views(settings, rep.means3D, zeros, rep.opacities, colors_precomp=rep.normals,
                                          scales=rep.scales, rotations=rep.rotations)
    else:
        # pass 2 (face normals, zero means2D) shares pass 1's geometry, sorts and blend (colors2)
        # (the renderer's render.clamp(0, 1), :212, formed in the blends: clamp=True)
        color, radii, depth, alpha, normal = rasterize_views(settings, rep.means3D, m2, rep.opacities,
                                                             colors_precomp=colors, scales=rep.scales,
                                                             rotations=rep.rotations, colors2=rep.normals,
                                                             grad_reduce=GRAD_REDUCE, clamp=FUSED_CLAMP)
        if not FUSED_CLAMP:
            color = color.clamp(0, 1)
    rays_o, rays_d, _ = shade
    _, nmap_dist = depth_normal_views(depth, alpha, rays_o, rays_d)
    nmap = sugar_normal_map(normal, alpha)  # normalize, flip x / y, alpha-weighted map, alpha > 0.99 mask (fused)
    depth = torch.where(alpha > 0.99, depth, depth.detach())
    return color, depth, alpha, nmap, nmap_dist


PROFILE_VIEWS_PER_LAUNCH = 64  # profiles/run_profiles.sh: bench.py defaults, one 64-view set per launch
# the blend kernels of the default workloads (forward, backward), as rocprofv3 demangles them: C3's 64-view
# launch takes the tile-wave forward and the lockstep matrix-core backward; C5 the two-colour
# quadrant-wave forward and the one-wave-per-tile hit-list backward (gsr_render.hip).  A run uses the names the
# library reports it launched (gsr_profile_kernel); the committed counters must name these (test_bench_fields)
KERNELS = {"c3": ("k_render_fwd_tile<false>", "k_render_bwd"),
           "sugar": ("k_render_fwd<true, false>", "k_render_bwd_tw<true>")}


def read_traffic(path, kernel, field="per_launch_bytes"):
    """Per-launch value of `kernel` (its exact demangled name, KERNELS) from a committed PMC summary
    (profiles/summarize.py): HBM bytes (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, separate --pmc passes)
    or SQ_INSTS_VALU; None if the file holds no counters of that kernel."""
    try:
        with open(path) as f:
            t = json.load(f)[field]
    except (OSError, KeyError, ValueError, TypeError):
        return None
    return float(t[kernel]) if kernel in t else None


def read_json(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def file_build(path):
    """The build id a committed counter / pair file was captured on (profiles/summarize.py, diag_pairs.py)."""
    d = read_json(path)
    return d.get("build_id") if isinstance(d, dict) else None


def time_knn(points, reps=10):
    """distCUDA2 (simple_knn drop-in, the scale initialisation of geometry/gaussian_base.py:434-438) on the
    scene's points, HIP events on the launch (current) stream; not part of the step."""
    from simple_knn._C import distCUDA2

    for _ in range(2):
        distCUDA2(points)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        distCUDA2(points)
    e1.record()
    torch.cuda.synchronize()
    return {"op": "distCUDA2 (3-NN mean squared distance)", "points": int(points.shape[0]),
            "ms": round(e0.elapsed_time(e1) / reps, 4)}


def _cpu_threads():
    """Threads for the CPU baseline: the job's CPU share (OMP_NUM_THREADS on the GPU box = 16), else the
    CPUs this process may run on."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_baseline(c3_scene, c3_res, c3_views):
    """The CPU restatement of the reference algorithm (oracle/gsr_oracle.c, fp32, OpenMP over tiles with
    per-thread gradient partials) timed on this host's cores: BASELINE.md's C1 (10k Gaussians, 256^2,
    SH0, 1 view: forward, and forward + backward) as the reported value, plus a bounded sample of the
    benchmark workload itself (C3 views, forward + backward)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure; timed here only as the reported CPU baseline

    import gsr_synthetic as gs
    from diff_gaussian_rasterization.cameras import get_cam_info_gaussian, orbit_c2w

    threads = _cpu_threads()
    oracle.lib().oracle_set_threads(threads)
    fovy = math.radians(60.0)
    tan = math.tan(fovy / 2)

    def cam(res, el, az):
        wv, fp, cc = get_cam_info_gaussian(orbit_c2w(2.5, el, az), fovy, fovy, 0.1, 100.0)
        return (wv.numpy().ravel(), fp.numpy().ravel(), cc.numpy(), tan, tan, res, res)

    # C1: 10k Gaussians, 256^2, SH0, white background; repeated until ~3 s per mode
    c1 = gs.make_scene(10_000, sh_degree=0, seed=0)
    c1_cam = cam(256, 15.0, 0.0)
    g1 = gs.upstream_grads(256, 256, seed=1)
    bg1 = np.ones(3, np.float32)
    oracle.forward(c1, c1_cam, bg1, "f32")  # warm (thread pool)

    def rate(fn, budget=3.0):
        n, t0 = 0, time.perf_counter()
        while True:
            fn()
            n += 1
            dt = time.perf_counter() - t0
            if dt >= budget or n >= 2000:
                return n / dt, n, dt

    fwd, n_f, t_f = rate(lambda: oracle.forward(c1, c1_cam, bg1, "f32"))
    # oracle.backward re-runs the forward first (as the reference's backward reads the forward's state,
    # the restatement recomputes it): one call = forward + backward
    fb, n_fb, t_fb = rate(lambda: oracle.backward(c1, c1_cam, bg1, *g1, prec="f32"))
    # C3 sample: views of the benchmark workload, forward + backward
    g3 = gs.upstream_grads(c3_res, c3_res, seed=1)
    bg3 = np.zeros(3, np.float32)
    t0 = time.perf_counter()
    for i in range(c3_views):
        oracle.backward(c3_scene, cam(c3_res, 0.0, i * 360.0 / 16), bg3, *g3, prec="f32")
    t3 = time.perf_counter() - t0
    oracle.lib().oracle_set_threads(1)
    host = f"{_cpu_model()}, {os.cpu_count()} logical CPUs on the host, {threads} threads used"
    return dict(
        value=fb, unit="views/s", cores=threads, kind="port",
        sample=f"C1 (10k Gaussians, 256x256, SH0, 1 view): forward + backward, oracle/gsr_oracle.c fp32 restatement "
               f"of the reference algorithm, OpenMP over tiles, {n_fb} repetitions in {t_fb:.2f} s on {host}",
        c1={"fwd_views_per_s": fwd, "fwd_bwd_views_per_s": fb, "fwd_reps": n_f, "fwd_bwd_reps": n_fb},
        c3_sample={"views_per_s": c3_views / t3, "views": c3_views, "seconds": t3,
                   "workload": f"{c3_scene['means3D'].shape[0]} Gaussians, {c3_res}x{c3_res}, "
                               f"SH{c3_scene['sh_degree']}, forward + backward"},
        host_logical_cpus=os.cpu_count(), cpu_model=_cpu_model())


def time_per_view_path(rep, cams, bg_zero, bg_img, upstream, n_views):
    """The drop-in per-view path — one GaussianRasterizer call per view, exactly the reference's loop
    (renderer/gaussian_batch_renderer.py:21-76) with the background composite in torch — timed on
    n_views views of the same workload (views/s; 1 GPU)."""
    n = min(n_views, len(cams))
    # one background tensor per view, as the reference's background network returns a fresh (H, W, 3) image
    # per view (renderer/diff_gaussian_rasterizer_background.py:116); slices of one batch leaf would make
    # autograd zero-fill the whole batch's gradient once per view
    bgs = [bg_img[i].detach().clone().requires_grad_(True) for i in range(n)]

    def run():
        outs = [render_view(rep, cams[i], bg_zero, bgs[i]) for i in range(n)]
        ts = [t for o in outs for t in o[:3]]
        torch.autograd.backward(ts, [g for u in upstream[:n] for g in u])
        rep.zero_grad()
        for b in bgs:
            b.grad = None

    run()
    torch.cuda.synchronize()
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    return {"views_per_s": round(n / dt, 2), "views": n, "repetitions": reps,
            "path": "GaussianRasterizer per view + torch composite (the reference's unchanged renderer loop)"}


def roofline_fields(args, phases, Ks, Ls, H, W, launched=None, build=None):
    """roofline (the dominant kernel) and roofline_fwd_blend, per launch, from the live HIP-event phase
    timings of this run.

    achieved = SURVEY.md §8d algorithmic bytes per launch / the launch's average duration, with K = the
    instances the tile lists hold (after the exact tile culling):
      forward blend   44 K + 28 H W + 8 tiles
      backward blend  44 K + 32 H W   (§8d's further 2 x 40 K of atomic read-modify-write is what the
                                       reference's atomic backward moves; this design writes one row per
                                       instance with plain stores and never performs it — reported as
                                       reference_rmw_bytes, not counted)
    counter_frac = PMC HBM bytes per launch (profiles/<tag>_traffic.json) / duration / 8 TB/s;
    valu = SQ_INSTS_VALU per launch (profiles/<tag>_traffic.json) against the VALU issue peak (one wave64 fp32
    instruction per SIMD per 4 cycles, MI355X_MICROARCH.md) and the device-counted pairs
    (profiles/<tag>_pairs.json, diagnostic build): the blends are issue / latency bound, not HBM bound."""
    tiles = math.ceil(W / 16) * math.ceil(H / 16)
    # the committed counters (profiles/run_profiles.sh) are of bench.py's default workload at N = 1: one
    # 64-view launch per blend.  Other workloads get no counter fields; a rank of an N > 1 run launches
    # fewer views: the per-launch counts scale with the views (per-view work is the same)
    profiled = (args.workload == "c3" and args.epilogue == "background" and args.res == 1024
                and args.gaussians == 1_000_000 and args.sh_degree == 3 and args.path == "batched")
    # the C5 line's counters (profiles/summarize.py r03d_sugar: the same command with --workload sugar)
    sugar = (args.workload == "sugar" and args.res == 800 and args.sh_degree == 3 and args.path == "batched"
             and not SUGAR_SEPARATE)
    traffic_path = args.traffic_sugar if sugar else args.traffic
    pairs = read_json(args.pairs) if profiled else None
    out = {}
    # counters and pair counts describe the build they were captured on: with `build` (the loaded library's id,
    # include/gsr.h gsr_version) a file of another build contributes nothing
    mismatch = []
    if build is not None:
        if (profiled or sugar) and file_build(traffic_path) != build:
            mismatch.append(f"{os.path.relpath(traffic_path, ROOT)} (build {file_build(traffic_path)})")
        # (pair counts come from the diagnostic build of the same sources: its id carries a "-diag" suffix)
        if pairs is not None and pairs.get("build_id") not in (build, build + "-diag"):
            mismatch.append(f"{os.path.relpath(args.pairs, ROOT)} (build {pairs.get('build_id')})")
            pairs = None
    n_fw = max(1, len(Ks))
    rows = {}
    names = KERNELS["sugar" if sugar else "c3"]
    if launched:  # the kernels the library reports it launched (gsr_profile_kernel) win over the defaults
        names = (launched.get("render_fwd") or names[0], launched.get("render_bwd") or names[1])
    profiled_here = profiled or sugar
    stale = []
    for phase, kernel in (("render_fwd", names[0]), ("render_bwd", names[1])):
        ms, n = phases[phase]
        n = max(1, n)
        if phase == "render_fwd":
            alg = (44.0 * sum(Ls) + (28.0 * H * W + 8.0 * tiles) * n_fw) / n
        else:
            alg = (44.0 * sum(Ls) + 32.0 * H * W * n_fw) / n
        sec = ms / n * 1e-3
        gbs = alg / sec / 1e9 if sec > 0 else 0.0
        views_per_launch = n_fw / n
        scale = views_per_launch / PROFILE_VIEWS_PER_LAUNCH
        # the forward kernel depends on the views per launch (gsr_render.hip fwd_tile_kernel: the tile-wave
        # kernel from 16 views, quadrant-wave below): its counters apply to the profiled 64-view launch only
        use = profiled_here and (phase == "render_bwd" or views_per_launch == PROFILE_VIEWS_PER_LAUNCH)
        use = use and not any(m.startswith(os.path.relpath(traffic_path, ROOT)) for m in mismatch)
        traffic = read_traffic(traffic_path, kernel) if use else None
        valu = read_traffic(traffic_path, kernel, "valu_insts_per_launch") if use else None
        if use and traffic is None:
            stale.append(kernel)
        traffic = round(traffic * scale) if traffic is not None else None
        valu = round(valu * scale) if valu is not None else None
        r = {"kernel": kernel, "bound": "hbm",
             "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "avg_launch_us": round(1e6 * sec, 2),
             "algorithmic_bytes": round(alg), "views_per_launch": round(views_per_launch, 2)}
        if traffic is not None and sec > 0:
            r["counter_frac"] = round(traffic / sec / (HBM_PEAK_GBS * 1e9), 4)
        if phase == "render_bwd":
            r["reference_rmw_bytes"] = round(80.0 * sum(Ls) / n)
        if traffic is not None:
            r["counters"] = {"file": os.path.relpath(traffic_path, ROOT), "kernel": kernel}
        v = {}
        if valu is not None and sec > 0:
            v["insts_per_launch"] = valu
            v["valu_frac"] = round(valu / sec / VALU_PEAK_INSTS, 4)
        key = "fwd_pairs_evaluated_per_view" if phase == "render_fwd" else "bwd_pairs_replayed_per_view"
        if pairs and pairs.get(key, 0) > 0:
            pl = pairs[key] * views_per_launch
            v["pairs_per_launch"] = round(pl)
            v["pairs_per_s"] = round(pl / sec) if sec > 0 else None
            if valu is not None:
                v["valu_insts_per_64_pairs"] = round(valu / (pl / 64.0), 2)
            if phase == "render_bwd":
                v["lockstep_slots_per_kept_pair"] = round(pairs["bwd_lockstep_slots_per_kept_pair"], 3)
        if v:
            v["peak_insts_per_s"] = VALU_PEAK_INSTS
            v["source"] = ("SQ_INSTS_VALU: " + os.path.relpath(traffic_path, ROOT) +
                           ("; pairs: " + os.path.relpath(args.pairs, ROOT) if pairs else ""))
            r["valu"] = v
        r["limiter"] = "VALU issue / LDS latency per (pixel, Gaussian) pair, not HBM (see counter_frac, valu)"
        if sugar and phase == "render_bwd":
            r["limiter"] = ("latency of the per-candidate replay chain and its LDS round trips (the four quadrants of "
                            "a tile walked in turn by one wave, 2 waves per SIMD at 225 VGPRs), not HBM")
        rows[phase] = r
    dominant = max(phases.items(), key=lambda kv: kv[1][0])[0]
    blend = "render_bwd" if phases["render_bwd"][0] >= phases["render_fwd"][0] else "render_fwd"
    out["roofline"] = rows[blend]
    out["roofline_fwd_blend"] = rows["render_fwd"]
    out["dominant_kernel"] = dominant
    if not profiled and not sugar:
        out["counters_note"] = ("no counter fields: profiles/ holds PMC counters of the default workload "
                                "(C3 background path, 1M, 1024^2) and of the C5 line only")
    elif stale:
        out["counters_note"] = (f"no counter fields for {', '.join(stale)}: {os.path.relpath(traffic_path, ROOT)} "
                                "holds no counters of that kernel (profiled on another build)")
    if mismatch:
        out["counters_note"] = (out.get("counters_note", "") + "; " if "counters_note" in out else "") + (
            f"dropped counters captured on another build than the loaded library ({build}): " + ", ".join(mismatch))
    if build is not None:
        out["library_build"] = build
    out["roofline_note"] = ("frac = SURVEY.md §8d algorithmic bytes / HIP-event duration (backward without the "
                            "reference's 80 B/instance atomic RMW, never performed here); counter_frac = PMC HBM "
                            "bytes / duration; valu_frac = SQ_INSTS_VALU / (duration x VALU issue peak). Both "
                            "blends are issue/latency bound; DESIGN.md §6")
    return out


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_command(args_list, n):
    """The torchrun command that runs this script as n ranks (one process per GPU), as the driver does."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(args_list)


def launch_ranks(args_list, n):
    """`python bench.py --gpus N` without a launcher: start the N ranks as child processes (nothing here has
    touched the GPU yet) and return their exit status."""
    import subprocess

    log(f"[bench] --gpus {n} without WORLD_SIZE: launching {n} ranks (torch.distributed.run)")
    return subprocess.call(launch_command(args_list, n))


def check_world(gpus, world):
    """--gpus must name the world the ranks run in (a mismatch would report another configuration)."""
    if gpus != world:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}: launch one rank per GPU "
                         f"(python bench.py --gpus {gpus}, or torch.distributed.run --nproc-per-node {gpus})")


def config_fields(args, world, per, comm, K_mean, L_mean, chunked_reduce):
    """The bench line's `config`: the workload (naming only the collectives that run: none at N = 1), the
    parallelism, and the collective backend / world size as torch.distributed reports them (comm_backend None
    without a process group), so a multi-rank run shows that RCCL saw N ranks."""
    cfg = {
        "workload": ("C5: ~2M surface-aligned SuGaR Gaussians (icosphere, 6 per face), 800x800, SH3, SuGaR "
                     "normal renderer (2 passes + normal-from-depth) over a 64-view orbit batch, fwd+bwd"
                     if args.workload == "sugar" else
                     ("C3 per view (1M Gaussians, 1024x1024, SH3, background path)" if args.epilogue ==
                      "background" else "1M Gaussians, 1024x1024, SH3, MVDream shading path (depth-normal, "
                      "point-light material, composite)") + f" over the C4 {args.views}-view orbit batch, fwd+bwd "
                     "(fixed random upstream image gradients)")
                    + (" + image all-gather + gradient all-reduce" if world > 1 else ""),
        "n_gaussians": args.gaussians, "resolution": [args.res, args.res], "sh_degree": args.sh_degree,
        "global_views_per_step": args.views, "views_per_rank": per,
        "parallelism": (f"views sharded over {world} rank(s) ({comm} all-gather of the images" + (
            " overlapped with the backward, " if args.gather == "overlap" else " before the backward, ") + (
            f"all-reduce of the Gaussian gradients in {args.grad_chunks} ranges overlapped with the "
            "per-Gaussian backward)" if chunked_reduce else "in-place all-reduce of the Gaussian "
            "gradients)") if world > 1 else "1 rank, no collectives"),
        "mean_instances_K": round(K_mean),
        "mean_listed_instances": round(L_mean),
        "path": args.path,
        "epilogue": "sugar_normal (normal-from-depth, 2 passes)" if args.workload == "sugar" else args.epilogue,
    }
    cfg["comm_backend"] = dist.get_backend() if dist.is_initialized() else None
    cfg["comm_world_size"] = dist.get_world_size() if dist.is_initialized() else 1
    return cfg


def run_workload(args, world, rank, device, comm, headline=True):
    """Build the workload of `args`, run W warm-up and K timed steps (barrier + synchronize on both sides, max
    over ranks) and return (result dict on rank 0 else None, scene).  headline: also the per-view-path and
    distCUDA2 lines and, for N > 1, the overlapped-gather variant of the same step."""
    import gsr_synthetic as gs
    from diff_gaussian_rasterization import _C
    from diff_gaussian_rasterization.view_shard import (ChunkedGradReduce, all_gather_views, all_gather_views_async,
                                                        allreduce_grads, shard_range)

    global GRAD_REDUCE, FUSED_CLAMP
    FUSED_CLAMP = args.fused_clamp == "on"
    overlap = world > 1 and args.overlap_reduce == "on" and args.path == "batched" and args.views >= world \
        and not SUGAR_SEPARATE
    GRAD_REDUCE = ChunkedGradReduce(n_chunks=args.grad_chunks) if overlap else None

    t_setup = time.perf_counter()
    if args.workload == "sugar":
        if args.res == 1024:
            args.res = 800
        scene = gs.make_sugar_scene(7, sh_degree=args.sh_degree, seed=0)
        args.gaussians = scene["means3D"].shape[0]
    else:
        scene = gs.make_scene(args.gaussians, sh_degree=args.sh_degree, seed=0)  # identical replica on every rank
    rep = Replica(scene, device)
    cams = build_views(args.views, args.res, device)
    v0, v1 = shard_range(args.views, world, rank)
    per = v1 - v0
    mine = cams[v0:v1]
    H = W = args.res
    gen = torch.Generator(device=device).manual_seed(1234 + rank)
    upstream = [(torch.randn((3, H, W), generator=gen, device=device),
                 torch.randn((1, H, W), generator=gen, device=device),
                 torch.randn((1, H, W), generator=gen, device=device)) for _ in mine]
    bg_zero = torch.zeros(3, device=device)
    # the background network's output per view, (H, W, 3) as the reference's background MLP returns it
    # (renderer/diff_gaussian_rasterizer_background.py:116); a trainable leaf so its gradient is formed
    bg_img = torch.rand((len(mine), H, W, 3), generator=gen, device=device).requires_grad_(True)
    # the per-view path's backgrounds: one leaf per view (the background network's per-view output)
    bg_views = [bg_img[i].detach().clone().requires_grad_(True) for i in range(len(mine))] \
        if args.path == "per-view" else []
    log(f"[bench] rank {rank}/{world}: {args.workload} setup {time.perf_counter() - t_setup:.1f}s, "
        f"{len(mine)} views/rank")

    settings = [settings_for(rep, cam, bg_zero) for cam in mine]
    up_c = torch.stack([u[0] for u in upstream]) if upstream else None
    up_d = torch.stack([u[1] for u in upstream]) if upstream else None
    up_a = torch.stack([u[2] for u in upstream]) if upstream else None

    shade = None
    up_n = None
    if args.epilogue == "shading" or args.workload == "sugar":
        shade = shading_inputs(mine, device)
        up_n = torch.randn((len(mine), 3, H, W), generator=gen, device=device)

    pending = []
    gather_mode = [args.gather]

    def gather(img):
        # forward exchange: every rank receives the whole batch of rendered images (the composited RGB the
        # batch renderer returns; depth / alpha terms are per view).  sync: the gathered batch exists before the
        # backward starts, as in the reference's step, where the guidance consumes comp_rgb before
        # loss.backward() (system/gaussian_splatting.py:65-67,129)
        if gather_mode[0] == "overlap":
            pending.append(all_gather_views_async(img, args.views))
        else:
            full = all_gather_views(img, args.views)
            return full

    def step():
        if args.workload == "sugar":
            outs = render_views_sugar(rep, settings, shade)
            if world > 1:
                gather(outs[0])
            torch.autograd.backward(outs, (up_c, up_d, up_a, up_n, up_n))
        elif args.path == "batched":
            outs = render_views(rep, settings, bg_img, shade)
            c, d, a = outs[:3]
            if world > 1:
                gather(c)
            # the loss's gradient w.r.t. the rendered images is injected as fixed upstream gradients
            if shade is None:
                torch.autograd.backward((c, d, a), (up_c, up_d, up_a))
            else:
                torch.autograd.backward((c, d, a, outs[4]), (up_c, up_d, up_a, up_n))
        else:
            outs = [render_view(rep, cam, bg_zero, bg_views[i],
                                None if shade is None else tuple(t[i] for t in shade))
                    for i, cam in enumerate(mine)]
            if world > 1:
                gather(torch.stack([o[0] for o in outs]))
            ts = [t for o in outs for t in o[:3]]
            gs_ = [t for g in upstream for t in g]
            if shade is not None:
                ts += [o[4] for o in outs]
                gs_ += list(up_n)
            torch.autograd.backward(ts, gs_)
        while pending:  # the overlapped gather completes within the step
            pending.pop().wait()
        if GRAD_REDUCE is None:
            allreduce_grads(rep.params)  # one flat RCCL all-reduce of the Gaussian parameter gradients
        # (else the rasterizer's backward summed them over ranks range by range, overlapped with it)
        rep.zero_grad()
        bg_img.grad = None
        for b in bg_views:
            b.grad = None

    def timed(steps):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], device=device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    _C.RECENT_FORWARDS.clear()
    _C.RECENT_LISTED.clear()
    _C.host_trace_read(reset=True)
    if not args.no_profile:
        _C.profile_read(reset=True)
        _C.profile_enable(True)
    elapsed = timed(args.steps)
    phases = None
    if not args.no_profile:
        _C.profile_enable(False)
        phases = _C.profile_read(reset=True)
    Ks = [k for k, _, _ in _C.RECENT_FORWARDS]
    # instances the kernels actually walk: the tile lists after the exact ellipse-vs-tile culling
    Ls = list(_C.RECENT_LISTED) if args.path == "batched" else list(Ks)
    host_trace = _C.host_trace_read() if _C.HOST_TRACE else None
    launched = _C.profile_kernels()

    variant = None
    if headline and world > 1 and args.gather == "sync":
        # the same step with the image all-gather overlapped with the backward (valid when the loss decomposes
        # over views or rank-aligned view groups; reported beside the headline, never as it)
        gather_mode[0] = "overlap"
        step()
        el = timed(args.steps)
        gather_mode[0] = args.gather
        variant = {"value": round(args.views * args.steps / el, 3), "ms_per_step": round(1000.0 * el / args.steps, 3),
                   "gather": "asynchronous, awaited at step end (beside the backward)"}

    total_views = args.views * args.steps
    value = total_views / elapsed
    K_mean = float(np.mean(Ks)) if Ks else 0.0
    L_mean = float(np.mean(Ls)) if Ls else 0.0

    if rank != 0:
        return None, scene

    res = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "views/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (seeded scene per SURVEY.md §8d; no datasets offline)",
        "config": config_fields(args, world, per, comm, K_mean, L_mean, GRAD_REDUCE is not None),
    }
    if world > 1:
        res["config"]["gather"] = args.gather
    if variant is not None:
        res["gather_overlap"] = variant
    if args.workload == "sugar":
        # how the two rasterizer calls run: one forward blending both colour sets + one backward pass for
        # both (gsr_set_backward_two_colors), or A/B variants
        res["config"]["two_calls"] = ("separate renders" if SUGAR_SEPARATE
                                      else "shared forward, one two-colour backward pass")
    if host_trace is not None:  # GSR_HOST_TRACE=1: host (Python + ctypes) time per step of the rasterizer's phases
        res["host_ms_per_step"] = {k: round(1000.0 * v / args.steps, 3) for k, v in host_trace.items()}
    if phases is not None:
        nv = max(1, args.steps * per)
        kern = {k: {"ms_per_view": round(ms / nv, 4), "launches": n} for k, (ms, n) in phases.items()}
        res["kernels"] = kern
        # wall time per step not covered by the rasterizer's kernels (the composite / collectives / torch ops
        # and the GPU idling while the host prepares launches)
        res["gap_ms_per_step"] = round(1000.0 * elapsed / args.steps - sum(ms for ms, _ in phases.values()) /
                                       args.steps, 3)
        res.update(roofline_fields(args, phases, Ks, Ls, H, W, launched, build=_C.build_id()))
    if headline and not args.no_knn:
        res["init_knn"] = time_knn(rep.means3D.detach())
    if headline and world == 1 and args.per_view_views > 0 and args.workload == "c3" \
            and args.epilogue == "background" and args.path == "batched":
        res["per_view_path"] = time_per_view_path(rep, mine, bg_zero, bg_img, upstream, args.per_view_views)
    return res, scene


def compact(res, keep_roofline=True):
    """A secondary workload's line as a sub-object of the headline: its rate, config and kernel times (and its
    dominant blend's roofline)."""
    out = {k: res[k] for k in ("value", "unit", "ms_per_step", "steps", "warmup") if k in res}
    out["config"] = res["config"]
    for k in ("kernels", "gap_ms_per_step"):
        if k in res:
            out[k] = res[k]
    if keep_roofline:
        for k in ("roofline", "roofline_fwd_blend", "dominant_kernel"):
            if k in res:
                out[k] = res[k]
    return out


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    check_world(args.gpus, world)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    comm = "none"
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # GSR_BENCH_BACKEND=gloo / GSR_BENCH_SHARE_GPU=1: rehearse the multi-rank path on a one-GPU box
        if os.environ.get("GSR_BENCH_SHARE_GPU") == "1":
            local = 0
        torch.cuda.set_device(local)
        backend = os.environ.get("GSR_BENCH_BACKEND", "nccl")
        comm = "RCCL" if backend == "nccl" else backend
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    elif os.environ.get("GSR_BENCH_SHARE_GPU") == "1":
        local = 0
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    res, scene = run_workload(args, world, rank, device, comm, headline=True)
    default_c3 = (args.workload == "c3" and args.epilogue == "background" and args.path == "batched"
                  and args.res == 1024 and args.gaussians == 1_000_000 and args.views == 64)
    extra = [] if args.extra_lines == "none" else args.extra_lines.split(",")
    if world == 1 and default_c3 and extra:
        c3_scene = scene
        for name in extra:
            sub = argparse.Namespace(**vars(args))
            sub.steps, sub.warmup = max(3, min(args.steps, 10)), max(1, min(args.warmup, 2))
            if name == "c5":  # BASELINE configs[4]: the SuGaR normal renderer (2M Gaussians, 800^2, two calls)
                sub.workload, sub.res = "sugar", 800
            elif name == "views8":  # a rank's share of the 64-view batch at N = 8
                sub.views = 8
                # as many views timed as the 64-view line's steps (an 8-view step is ≈ 2.5 ms: 5 of them were
                # dominated by host jitter, 2.5–2.7 ms per step for the same kernel times)
                sub.steps, sub.warmup = 8 * max(3, min(args.steps, 10)), 5
            else:
                raise SystemExit(f"unknown --extra-lines entry {name!r}")
            r, _ = run_workload(sub, world, rank, device, comm, headline=False)
            torch.cuda.empty_cache()
            res[name] = compact(r)
        scene = c3_scene
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(scene, args.res, args.cpu_views)
        rnd = lambda v: round(v, 5) if isinstance(v, float) else v  # noqa: E731
        res["cpu_baseline"] = {k: ({kk: rnd(vv) for kk, vv in v.items()} if isinstance(v, dict) else rnd(v))
                               for k, v in cb.items()}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

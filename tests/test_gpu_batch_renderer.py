"""The drop-in batch renderer on the HIP path (diff_gaussian_rasterization/batch_renderer.py).

- Each fused mode (one rasterize_views call per batch + the fused epilogue) against the reference's
  per-view loop (renderer/gaussian_batch_renderer.py:9-122) over the reference's per-view
  DiffGaussian.forward (tests/renderer_fixtures.py; GaussianRasterizer per view, torch epilogues):
  same output dict, images within 1e-5, gradients elementwise within 1e-4 max(1, |g|) (1e-2 for the
  modes whose epilogue differentiates a depth -> normal stencil, see the test).
- The sharded HIP path: two ranks (gloo backend, both on the one GPU of the box) render their view
  slices through rasterize_views, all-gather the images, run the backward, all-reduce the gradients
  (view_shard.allreduce_grads) and update the densification state (view_shard.update_states_sharded,
  the reference's densify / prune restated in tests/densify_reference.py): images bit-identical to one
  process rendering the whole batch, gradients within 1e-5 relative, and bitwise-identical replicas
  after densification.  (Scaling on 1/2/4/8 GPUs is measured by the driver's multi-GPU bench.)
"""
import math
import os
import socket

import numpy as np
import pytest
import torch

import renderer_fixtures as rf
from gsr_testutil import gs

pytestmark = pytest.mark.gpu

H, W = 96, 128


def _scene(mode):
    if mode in ("sugar_normal", "sugar_shading"):
        s = gs.make_sugar_scene(4, sh_degree=0, seed=2)
        s["shs"] = s["shs"][:, :1]
        return s
    return gs.make_scene(20_000, sh_degree=3, seed=4)


def _close(a, b, tol, what):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    err = (a - b).abs() / b.abs().clamp(min=1.0)
    assert float(err.max()) <= tol, f"{what}: {float(err.max())} (at {int(err.argmax())})"


@pytest.mark.parametrize("mode,training,pred_normal", [
    ("plain", False, False), ("background", False, False), ("advanced", False, False), ("shading", False, False),
    ("normal", False, False), ("sugar_normal", False, False), ("sugar_shading", False, False),
    # training: per-view background inversion / soft-shading ambient ratio and shading mode, drawn as the loop does
    ("plain", True, False), ("advanced", True, False), ("shading", True, False), ("normal", True, False),
    ("sugar_shading", True, False),
    # the predicted-normal second pass, both paths
    ("shading", True, True), ("normal", False, True),
])
def test_fused_mode_matches_per_view_loop(mode, training, pred_normal):
    import random

    batch = rf.make_batch(4, H, W, "cuda", seed=3)
    kw = dict(training=training, soft_shading=training, pred_normal=pred_normal)
    fused = rf.FakeRenderer(mode, _scene(mode), "cuda", **kw)
    ref = rf.PerViewRenderer(mode, _scene(mode), "cuda", **kw)
    random.seed(21), np.random.seed(21)
    out_f = fused.batch_forward(dict(batch))
    after_f = (random.random(), np.random.rand())
    random.seed(21), np.random.seed(21)
    out_r = ref.batch_forward(dict(batch))
    assert after_f == (random.random(), np.random.rand()), "different random draws than the per-view loop"
    keys = sorted(k for k in out_r if k.startswith("comp_"))
    assert keys == sorted(k for k in out_f if k.startswith("comp_")), (keys, list(out_f))
    for k in keys:
        assert out_f[k].shape == out_r[k].shape, k
        _close(out_f[k], out_r[k], 1e-5, k)
    for v in range(4):
        assert torch.equal(out_f["radii"][v], out_r["radii"][v])
        assert torch.equal(out_f["visibility_filter"][v], out_r["visibility_filter"][v])
    rf.loss_of(out_f).backward()
    rf.loss_of(out_r).backward()
    # the depth -> normal stencil (shading, SuGaR) is ill-conditioned: the fused HIP epilogue and torch's
    # fp32 ops (different operation order, both faithful; tests/test_shading.py checks each against torch
    # fp64) differ by up to ~3e-3 relative in the depth gradients that reach the Gaussians
    tol = 1e-4 if mode in ("plain", "background", "advanced") else 1e-2
    for v in range(4):
        _close(out_f["viewspace_points"][v].grad, out_r["viewspace_points"][v].grad, tol, f"viewspace {v}")
    for k, p in fused.geometry.params.items():
        q = ref.geometry.params[k]
        if q.grad is None:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, k
            continue
        _close(p.grad, q.grad, tol, "grad " + k)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _step(rank_world, B, tmp, tag, overlap=False):
    """One training step of the background renderer on this process's views; saves the results.  overlap:
    the rasterizer's per-Gaussian gradients are summed over ranks inside its backward (ChunkedGradReduce)
    instead of by allreduce_grads afterwards."""
    import torch.distributed as dist

    import densify_reference as dr
    from diff_gaussian_rasterization.view_shard import (ChunkedGradReduce, allreduce_grads, replica_checksum,
                                                        update_states_sharded)

    rank, world = rank_world
    scene = _scene("background")
    r = rf.FakeRenderer("background", scene, "cuda")
    model = dr.DensifyModel(scene, "cuda", densify_grad_threshold=2e-4)
    r.geometry = model
    if overlap:
        r.grad_reduce = ChunkedGradReduce(n_chunks=3)
    batch = rf.make_batch(B, H, W, "cuda", seed=5)
    out = r.batch_forward(batch)
    rf.loss_of(out).backward()
    params = model.parameters()
    if not overlap:
        allreduce_grads(params)
    else:
        assert r.grad_reduce.launched == (1 if dist.is_initialized() else 0)
    grads = [p.grad.detach().cpu().numpy().copy() for p in params]
    update_states_sharded(model, 5, out)
    same = replica_checksum(model.parameters() + [model.max_radii2D]) if world > 1 else True
    np.savez(os.path.join(tmp, f"{tag}{rank}.npz"), comp_rgb=out["comp_rgb"].detach().cpu().numpy(),
             P=model.get_xyz.shape[0], same=same, **{f"g{i}": g for i, g in enumerate(grads)})
    if world > 1:
        dist.barrier()


def _worker(rank, world, port, tmp, B, overlap=False):
    import torch.distributed as dist

    torch.cuda.set_device(0)
    # file rendezvous (no TCP port to race for); `port` only makes the file name unique
    dist.init_process_group("gloo", init_method="file://" + os.path.join(tmp, f"rendezvous_{port}"), rank=rank,
                            world_size=world)
    try:
        torch.manual_seed(100 + rank)
        _step((rank, world), B, tmp, "shard", overlap=overlap)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("B,overlap", [(5, False), (4, False), (5, True)])
def test_sharded_hip_path_world2(B, overlap, tmp_path):
    """overlap: ChunkedGradReduce — the per-Gaussian backward in Gaussian ranges with an event after each,
    each range's rows all-reduced on a side stream while the next is formed (gsr_set_backward_chunks)."""
    import torch.multiprocessing as mp

    _step((0, 1), B, str(tmp_path), "single")
    single = np.load(tmp_path / "single0.npz")
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), B, overlap), nprocs=2, join=True)
    for rank in range(2):
        z = np.load(tmp_path / f"shard{rank}.npz")
        np.testing.assert_array_equal(z["comp_rgb"], single["comp_rgb"], err_msg=f"rank {rank} images")
        for i in range(6):
            g, ref = z[f"g{i}"].astype(np.float64), single[f"g{i}"].astype(np.float64)
            err = np.abs(g - ref) / np.maximum(np.abs(ref), 1.0)
            assert err.max() <= 1e-5, f"rank {rank} grad {i}: {err.max()}"
        assert bool(z["same"]), f"rank {rank}: replicas differ after densification"
        assert int(z["P"]) == int(single["P"]) > 20_000


class _ForceChunks:
    """A grad_reduce stand-in that makes a one-process backward run chunked (the ranges and events of
    ChunkedGradReduce) without reducing anything."""

    def __init__(self, n):
        from diff_gaussian_rasterization.view_shard import ChunkedGradReduce

        self._r = ChunkedGradReduce(n_chunks=n)
        self.n_chunks = n
        self.ranges_seen = 0

    def active(self):
        return True

    def chunk_events(self, device):
        return self._r.chunk_events(device)

    def launch(self, grads, P, events=None):
        for e in events:
            e.synchronize()  # every range's event was recorded by the library
        self.ranges_seen = len(events)


class _SnapshotReduce:
    """A grad_reduce stand-in that reads the gradients on a side stream the way ChunkedGradReduce's all-reduces
    do: after the library's per-range events when it is given them, else after the whole main stream."""

    def __init__(self, n):
        from diff_gaussian_rasterization.view_shard import ChunkedGradReduce

        self._r = ChunkedGradReduce(n_chunks=n)
        self.snap = None
        self.used_events = None

    def active(self):
        return True

    def chunk_events(self, device):
        return self._r.chunk_events(device)

    def launch(self, grads, P, events=None):
        side = torch.cuda.Stream()
        if events:
            for e in events:
                side.wait_event(e)
        else:
            side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self.snap = [g.clone() for g in grads if g is not None]
        self.grads = [g for g in grads if g is not None]
        self.used_events = bool(events)


@pytest.mark.parametrize("bwd", ["fused", "separate"])
def test_chunked_reduce_reads_finished_gradients(bwd):
    """with the SuGaR normal renderer's second rasterizer call backpropagated separately
    (two_color_backward="separate") its kernels still add into the shared gradients after the first call's
    ranges are formed, so the reduction must wait for the whole stream (no per-range events); with the fused
    two-colour backward the per-range events cover every writer.  The gradients a side-stream reader sees equal
    the final ones either way."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    from diff_gaussian_rasterization.batched import rasterize_views
    from diff_gaussian_rasterization.cameras import get_cam_info_gaussian

    scene = gs.make_sugar_scene(4, sh_degree=0, seed=5)
    P = scene["means3D"].shape[0]
    batch = rf.make_batch(3, H, W, "cuda", seed=11)
    fovy = batch["fovy"]
    w2c, proj, campos = get_cam_info_gaussian(batch["c2w"], fovy, fovy, znear=0.1, zfar=100)
    tan = math.tan(float(fovy[0]) * 0.5)
    settings = [GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=tan, tanfovy=tan,
                                              bg=torch.zeros(3, device="cuda"), scale_modifier=1.0,
                                              viewmatrix=w2c[v], projmatrix=proj[v], sh_degree=0, campos=campos[v],
                                              prefiltered=False, debug=False) for v in range(3)]
    t = {k: torch.tensor(scene[k], device="cuda", requires_grad=True)
         for k in ("means3D", "opacities", "scales", "rotations", "normals")}
    cols = torch.tensor(scene["shs"][:, 0, :] * np.float32(gs.C0) + np.float32(0.5), device="cuda",
                        requires_grad=True)
    m2 = [torch.zeros((P, 3), device="cuda", requires_grad=True) for _ in range(3)]
    snap = _SnapshotReduce(4)
    outs = rasterize_views(settings, t["means3D"], m2, t["opacities"], colors_precomp=cols, scales=t["scales"],
                           rotations=t["rotations"], colors2=t["normals"], grad_reduce=snap, two_color_backward=bwd)
    up = [torch.randn_like(o, generator=torch.Generator("cuda").manual_seed(20 + i)) if o.is_floating_point()
          else None for i, o in enumerate(outs)]
    torch.autograd.backward([o for o, u in zip(outs, up) if u is not None], [u for u in up if u is not None])
    torch.cuda.synchronize()
    assert snap.snap is not None
    # the separate second-colour backward writes after the first call's ranges: no per-range events then
    assert snap.used_events == (bwd == "fused")
    for i, (a, b) in enumerate(zip(snap.snap, snap.grads)):  # what the reader saw vs the finished buffers
        assert torch.equal(a, b), f"gradient buffer {i} read before its last writer finished"


@pytest.mark.parametrize("n_chunks,P", [(4, 20_000), (3, 4096 * 5 + 17), (16, 9000)])
def test_chunked_gauss_backward_bitwise(n_chunks, P):
    """gsr_set_backward_chunks: the per-Gaussian backward in Gaussian ranges (with events) gives bitwise the
    gradients of the one-pass backward, also with the background composite and several view sets."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    from diff_gaussian_rasterization.batched import rasterize_views

    scene = gs.make_scene(P, sh_degree=2, seed=6)
    batch = rf.make_batch(3, H, W, "cuda", seed=9)
    from diff_gaussian_rasterization.cameras import get_cam_info_gaussian

    fovy = batch["fovy"]
    w2c, proj, campos = get_cam_info_gaussian(batch["c2w"], fovy, fovy, znear=0.1, zfar=100)
    tan = math.tan(float(fovy[0]) * 0.5)
    settings = [GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=tan, tanfovy=tan,
                                              bg=torch.zeros(3, device="cuda"), scale_modifier=1.0,
                                              viewmatrix=w2c[v], projmatrix=proj[v], sh_degree=2, campos=campos[v],
                                              prefiltered=False, debug=False) for v in range(3)]
    bg_img = torch.rand((3, H, W, 3), device="cuda", generator=torch.Generator("cuda").manual_seed(2))
    up = torch.randn((3, 3, H, W), device="cuda", generator=torch.Generator("cuda").manual_seed(3))

    def run(reduce):
        t = {k: torch.tensor(scene[k], device="cuda", requires_grad=True)
             for k in ("means3D", "shs", "opacities", "scales", "rotations")}
        m2 = [torch.zeros((P, 3), device="cuda", requires_grad=True) for _ in range(3)]
        out, _, _, _ = rasterize_views(settings, t["means3D"], m2, t["opacities"], shs=t["shs"], scales=t["scales"],
                                       rotations=t["rotations"], background=bg_img, grad_reduce=reduce)
        (out * up).sum().backward()
        torch.cuda.synchronize()
        return {k: v.grad.cpu() for k, v in t.items()}, [m.grad.cpu() for m in m2]

    ref, ref_m2 = run(None)
    force = _ForceChunks(n_chunks)
    got, got_m2 = run(force)
    assert force.ranges_seen == n_chunks
    for k in ref:
        assert torch.equal(ref[k], got[k]), k
    for a, b in zip(ref_m2, got_m2):
        assert torch.equal(a, b)


# ---- C4: the 64-view MVDream-style batch at 1M Gaussians, single process vs two ranks ----------------------

C4_P = 1_000_000


def _c4_batch(B, S, dev):
    """The bench's orbit (4 elevations x 16 azimuths, bench.py) as the data module's batch dict."""
    from diff_gaussian_rasterization.cameras import light_positions_dreamfusion, orbit_c2w, ray_bundle

    per = max(1, B // 4)
    elev = torch.tensor([[0.0, 10.0, 20.0, 30.0][(i // per) % 4] for i in range(B)])
    azim = torch.tensor([(i % per) * 360.0 / per for i in range(B)])
    c2w = orbit_c2w(torch.full((B,), 2.5), elev, azim)
    fovy = torch.full((B,), math.radians(60.0))
    rays_o, rays_d = ray_bundle(c2w, fovy, S, S)
    return {"c2w": c2w.to(dev), "fovy": fovy.to(dev), "height": S, "width": S, "rays_o": rays_o.to(dev),
            "rays_d": rays_d.to(dev), "light_positions": light_positions_dreamfusion(c2w, 2.0).to(dev)}


def _c4_upstream(B, S):
    g = torch.Generator().manual_seed(123)
    return torch.randn((B, S, S, 3), generator=g)


def _c4_step(rank_world, B, S, tmp, tag, check_views=()):
    """One training step of the background renderer (renderer/diff_gaussian_rasterizer_background.py) over the
    C4 batch through GaussianBatchRenderer.batch_forward: forward (this rank's views, images all-gathered),
    fixed upstream gradient, backward, gradient all-reduce, densification (update_states_sharded).  Saves the
    gathered images, the all-reduced gradients, the replica checksum, and for `check_views` the per-view
    screen-space gradients and radii (checked against the oracle by the caller)."""
    import torch.distributed as dist

    import densify_reference as dr
    from diff_gaussian_rasterization.view_shard import allreduce_grads, replica_checksum, update_states_sharded

    rank, world = rank_world
    scene = gs.make_scene(C4_P, sh_degree=3, seed=0)
    r = rf.FakeRenderer("background", scene, "cuda")
    model = dr.DensifyModel(scene, "cuda", densify_grad_threshold=2e-4)
    r.geometry = model
    batch = _c4_batch(B, S, "cuda")
    out = r.batch_forward(batch)
    w = _c4_upstream(B, S).to("cuda")
    (out["comp_rgb"] * w).sum().backward()
    params = model.parameters()
    grads = {f"pre{i}": p.grad.detach().cpu().numpy().copy() for i, p in enumerate(params)}  # this rank's sums
    allreduce_grads(params)
    grads.update({f"g{i}": p.grad.detach().cpu().numpy().copy() for i, p in enumerate(params)})
    lo = out.get("view_range", (0, B))[0]
    extra = {}
    if check_views:  # the cameras exactly as render_views_local builds them (batched, on the device)
        from diff_gaussian_rasterization.cameras import get_cam_info_gaussian

        fovy = batch["fovy"].reshape(-1)
        w2c, proj, campos = get_cam_info_gaussian(batch["c2w"], fovy, fovy, znear=0.1, zfar=100)
        extra.update(w2c=w2c.cpu().numpy(), proj=proj.cpu().numpy(), campos=campos.cpu().numpy(),
                     bg_img=rf._background_net(batch["rays_d"]).cpu().numpy())
    for v in check_views:
        i = v - lo
        if 0 <= i < len(out["radii"]):
            extra[f"m2_{v}"] = out["viewspace_points"][i].grad.detach().cpu().numpy()
            extra[f"radii_{v}"] = out["radii"][i].cpu().numpy()
    update_states_sharded(model, 5, out)
    same = replica_checksum(model.parameters() + [model.max_radii2D]) if world > 1 else True
    np.savez(os.path.join(tmp, f"{tag}{rank}.npz"), comp_rgb=out["comp_rgb"].detach().cpu().numpy(),
             P=model.get_xyz.shape[0], same=same, **grads, **extra)
    if world > 1:
        dist.barrier()


def _c4_worker(rank, world, port, tmp, B, S):
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method="file://" + os.path.join(tmp, f"rendezvous_{port}"), rank=rank,
                            world_size=world)
    try:
        torch.manual_seed(100 + rank)
        _c4_step((rank, world), B, S, tmp, "shard")
    finally:
        dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.parametrize("B,S", [(64, 256), (8, 1024)])
def test_c4_batch_single_vs_two_ranks(B, S, tmp_path):
    """C4 (BASELINE.json configs[3]): 1M Gaussians, SH3, a 64-view batch at the MVDream config's native 256^2
    (configs/gaussian_splatting_mvdream.yaml:8-12) — and 8 views at the metric's 1024^2 — through the drop-in
    GaussianBatchRenderer.batch_forward (renderer/gaussian_batch_renderer.py:9-122), once as one process and
    once as two ranks sharing the GPU (gloo): images bitwise equal, all-reduced gradients within 1e-5
    relative, bitwise-identical replicas with equal Gaussian counts after update_states_sharded
    (geometry/gaussian_base.py:821-869); two of the views (one per rank) against the fp64 / fp32 oracle:
    composited image, radii and the per-view screen-space gradient (the densification statistic)."""
    import torch.multiprocessing as mp

    check = (1, B - 2)
    _c4_step((0, 1), B, S, str(tmp_path), "single", check_views=check)
    single = np.load(tmp_path / "single0.npz")
    torch.cuda.empty_cache()
    mp.spawn(_c4_worker, args=(2, _free_port(), str(tmp_path), B, S), nprocs=2, join=True)
    zs = [np.load(tmp_path / f"shard{rank}.npz") for rank in range(2)]
    for rank, z in enumerate(zs):
        np.testing.assert_array_equal(z["comp_rgb"], single["comp_rgb"], err_msg=f"rank {rank} images")
        for i in range(6):
            # one process sums the 64 views' terms in view order, two ranks each sum their half and the
            # all-reduce adds the halves: an fp32 reassociation whose rounding scales with the halves'
            # magnitudes (they may cancel), so the bar is relative to max(1, |g|, |half_0| + |half_1|)
            g, ref = z[f"g{i}"].astype(np.float64), single[f"g{i}"].astype(np.float64)
            halves = np.abs(zs[0][f"pre{i}"].astype(np.float64)) + np.abs(zs[1][f"pre{i}"].astype(np.float64))
            err = np.abs(g - ref) / np.maximum(np.maximum(np.abs(ref), halves), 1.0)
            assert err.max() <= 1e-5, f"rank {rank} grad {i}: {err.max()}"
        assert bool(z["same"]), f"rank {rank}: replicas differ after densification"
        assert int(z["P"]) == int(single["P"]) > C4_P
    _c4_oracle_views(single, B, S, check)
    _c4_oracle_sums(single, B, S)


def _c4_oracle_sums(single, B, S):
    """The batch's summed parameter gradients (the ones the optimizer steps on, all B views) against the fp64 /
    fp32 oracle summed over the same views: the oracle's per-view gradients w.r.t. the activated parameters
    (means3D, SH, opacity, scales, rotations) summed over views in fp64 (and in fp32 for the allowance), then
    taken through the model's activations in fp64 — sigmoid (opacity), exp (scaling), normalize (rotation) —
    against the GPU's gradients of the raw parameters (tests/densify_reference.py getters).  Gaussians blended at
    a pixel whose composited value the GPU flipped on its own in any view are excused (flip_excuse's rule, applied
    per view in the oracle workers).  The views run in a pool of processes (tests/oracle_pool.py: ~20 s of
    serial oracle per 1M-Gaussian view)."""
    import oracle_pool
    from gsr_testutil import check_grads

    spec = ("ball", C4_P, 3, 0)
    scene = oracle_pool.scene_of(spec)
    w2c, proj, campos, bg_img = single["w2c"], single["proj"], single["campos"], single["bg_img"]
    w = _c4_upstream(B, S).numpy()
    tan = math.tan(float(np.float32(math.radians(60.0))) * 0.5)
    zero = np.zeros((1, S, S), np.float32)
    tasks = []
    for v in range(B):
        cam = dict(view=w2c[v].astype(np.float32), proj=proj[v].astype(np.float32),
                   campos=campos[v].astype(np.float32), tanx=tan, tany=tan, W=S, H=S)
        g_r = w[v].transpose(2, 0, 1).astype(np.float32)
        tasks.append((spec, cam, [0.0, 0.0, 0.0], (g_r, zero, zero), bg_img[v], single["comp_rgb"][v].transpose(2, 0, 1),
                      ("f32r",)))
    _, tot = oracle_pool.views_and_sums(tasks, keep_views=False)
    sums = {tag: tot[tag] for tag in ("f32", "f64", "f32r")}

    # through the activations of DensifyModel (raw parameters as the model holds them, in fp64)
    raw_op = np.log(np.clip(scene["opacities"].astype(np.float64), 1e-4, 1 - 1e-4)) - np.log1p(
        -np.clip(scene["opacities"].astype(np.float64), 1e-4, 1 - 1e-4))
    raw_op = np.float32(raw_op).astype(np.float64)  # (inverse_sigmoid of the float32 tensor)
    sig = 1.0 / (1.0 + np.exp(-raw_op))
    scl = np.exp(np.log(scene["scales"].astype(np.float32)).astype(np.float64))
    rot = scene["rotations"].astype(np.float64)
    nrm = np.maximum(np.linalg.norm(rot, axis=1, keepdims=True), 1e-12)
    q = rot / nrm

    def raw(s):
        g_rot = (s["rotations"] - q * (q * s["rotations"]).sum(1, keepdims=True)) / nrm
        return {"g_xyz": s["means3D"], "g_f_dc": s["sh"][:, :1], "g_f_rest": s["sh"][:, 1:],
                "g_opacity": s["opacity"] * (sig * (1.0 - sig)), "g_scaling": s["scales"] * scl, "g_rotation": g_rot}

    r = {"b32": {k[2:]: v for k, v in raw(sums["f32"]).items()}, "b64": {k[2:]: v for k, v in raw(sums["f64"]).items()},
         "b32r": {k[2:]: v for k, v in raw(sums["f32r"]).items()}}
    names = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")  # DensifyModel.parameters() order
    gpu = {"g_" + n: single[f"g{i}"].reshape(r["b64"][n].shape) for i, n in enumerate(names)}
    check_grads(gpu, r, names, f"C4 {S}^2 summed over {B} views", excuse=tot.get("excuse"))


def _c4_oracle_views(single, B, S, views):
    import oracle
    from gsr_testutil import adjudicate, check_radii, flip_excuse, oracle_cam, run_oracle
    from test_gpu_configs import _composite, _composite_upstream

    scene = gs.make_scene(C4_P, sh_degree=3, seed=0)
    w2c, proj, campos, bg_img = single["w2c"], single["proj"], single["campos"], single["bg_img"]
    w = _c4_upstream(B, S).numpy()
    tan = math.tan(float(np.float32(math.radians(60.0))) * 0.5)  # as the settings: float32 fovy
    for v in views:
        cam = dict(view=w2c[v].astype(np.float32), proj=proj[v].astype(np.float32),
                   campos=campos[v].astype(np.float32), tanx=tan, tany=tan, W=S, H=S)
        ref = run_oracle(scene, cam, [0.0, 0.0, 0.0])
        g_r = w[v].transpose(2, 0, 1).astype(np.float32)
        b = {}
        for prec, dt in (("f32", np.float32), ("f64", np.float64)):
            f = ref[prec]
            render, pre = _composite(f["color"].astype(dt), f["alpha"].astype(dt), bg_img[v].astype(dt))
            b["render_" + prec] = render
            gcol, ga = _composite_upstream(g_r, np.zeros((1, S, S), np.float32), pre, bg_img[v])
            b[prec] = oracle.backward(scene, oracle_cam(cam), np.zeros(3, np.float32), gcol.astype(np.float32),
                                      np.zeros((1, S, S), np.float32), ga.astype(np.float32), prec=prec)
            if prec == "f32":
                b["f32r"] = oracle.backward(scene, oracle_cam(cam), np.zeros(3, np.float32), gcol.astype(np.float32),
                                            np.zeros((1, S, S), np.float32), ga.astype(np.float32), prec="f32c", order=1)
        px = lambda a: np.asarray(a).reshape(3, -1).T  # noqa: E731
        gpu_img = single["comp_rgb"][v].transpose(2, 0, 1)
        adjudicate(px(gpu_img), px(b["render_f32"]), px(b["render_f64"]), 1e-5, f"C4 {S}^2 view {v}", "comp_rgb",
                   cap=0.02)
        check_radii(single[f"radii_{v}"], ref, f"C4 {S}^2 view {v}")
        # pixels where the GPU's composited image missed the fp64 value and the fp32 oracle's did not: a discrete
        # decision (alpha >= 1/255, T < 1e-4) taken differently; the Gaussians blended there are excused
        e_g = np.abs(px(gpu_img) - px(b["render_f64"])).max(1)
        e_3 = np.abs(px(b["render_f32"]) - px(b["render_f64"])).max(1)
        ref["gpu_only_px"] = np.nonzero((e_g > 1e-5) & ~(e_3 > 1e-5))[0]
        m64 = b["f64"]["means2D"]
        adjudicate(single[f"m2_{v}"], b["f32"]["means2D"], m64, 1e-4 * np.maximum(1.0, np.abs(m64)),
                   f"C4 {S}^2 view {v}", "grad means2D", rowwise=True, r32b=b["f32r"]["means2D"],
                   excuse=flip_excuse([ref]))

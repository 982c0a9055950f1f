"""View sharding across ranks with the gloo backend on CPU, world_size 2 and 3:
the gathered batch images, the all-reduced Gaussian gradients and the reduced densification statistics
must equal a single-process render of the whole batch.  The per-view renderer is the differentiable
torch formulation (tests/torch_reference.py) so the sharding/collective logic runs without a GPU."""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import torch_reference as tr
from diff_gaussian_rasterization.cameras import get_cam_info_gaussian, orbit_c2w
from diff_gaussian_rasterization.view_shard import (ViewShardedBatchRenderer, allreduce_grads,
                                                    reduce_densify_stats, shard_range)
from gsr_testutil import gs

H = W = 24
B = 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _params():
    scene = gs.make_scene(40, sh_degree=1, seed=3, radius=0.5)
    return {k: torch.tensor(scene[k], dtype=torch.float64, requires_grad=True)
            for k in ("means3D", "scales", "rotations", "opacities", "shs")}


def _batch():
    c2w = orbit_c2w(torch.full((B,), 2.5), torch.linspace(0, 30, B), torch.linspace(0, 288, B))
    return {"c2w": c2w, "fovy": torch.full((B,), math.radians(60.0)), "height": H, "width": W}


def _render_view(params):
    def fn(batch_idx, batch):
        fov = float(batch["fovy"][batch_idx])
        wv, fp, cc = get_cam_info_gaussian(batch["c2w"][batch_idx], fov, fov)
        P = params["means3D"].shape[0]
        sp = torch.zeros(P, 3, dtype=torch.float64, requires_grad=True)
        sp.retain_grad()
        tan = math.tan(fov / 2)
        color, radii, depth, alpha = tr.render(params["means3D"], sp, params["opacities"], wv.reshape(-1),
                                               fp.reshape(-1), cc, tan, tan, W, H, torch.zeros(3), sh=params["shs"],
                                               deg=1, scales=params["scales"], rotations=params["rotations"])
        return {"render": color, "depth": depth, "mask": alpha, "viewspace_points": sp,
                "visibility_filter": radii > 0, "radii": radii}
    return fn


def _loss(out):
    g = torch.Generator().manual_seed(0)
    wc = torch.randn(out["comp_rgb"].shape, generator=g, dtype=torch.float64)
    wd = torch.randn(out["comp_depth"].shape, generator=g, dtype=torch.float64)
    return (out["comp_rgb"] * wc).sum() + (out["comp_depth"] * wd).sum() + out["comp_mask"].sum()


def _regularisers(params):
    """Parameter-direct loss terms as the systems add them (lambda_position / lambda_opacity / lambda_scales,
    system/gaussian_splatting.py:89-106): computed on every rank from the replicated parameters."""
    return (0.3 * (params["means3D"] ** 2).sum() + 0.2 * params["opacities"].sum()
            + 0.1 * params["scales"].norm(dim=-1).mean())


def _single_process(reg=False):
    params = _params()
    r = ViewShardedBatchRenderer(_render_view(params))
    out = r.batch_forward(_batch())
    loss = _loss(out) + (_regularisers(params) if reg else 0)
    loss.backward()
    stats = reduce_densify_stats(out["radii"], out["viewspace_points"], out["visibility_filter"], 40)
    return ({k: out[k].detach().numpy() for k in ("comp_rgb", "comp_depth", "comp_mask")},
            {k: v.grad.numpy() for k, v in params.items()}, [s.numpy() for s in stats])


def _worker(rank, world, port, tmp, reg=False):
    from diff_gaussian_rasterization.view_shard import replicated_loss

    # file rendezvous (no TCP port to race for); `port` only makes the file name unique
    dist.init_process_group("gloo", init_method="file://" + os.path.join(tmp, f"rendezvous_{port}"), rank=rank,
                            world_size=world)
    try:
        params = _params()
        r = ViewShardedBatchRenderer(_render_view(params))
        out = r.batch_forward(_batch())
        assert out["view_range"] == shard_range(B, world, rank)
        loss = _loss(out) + (replicated_loss(_regularisers(params)) if reg else 0)
        loss.backward()
        allreduce_grads(list(params.values()))
        stats = reduce_densify_stats(out["radii"], out["viewspace_points"], out["visibility_filter"], 40)
        np.savez(os.path.join(tmp, f"rank{rank}.npz"),
                 **{k: out[k].detach().numpy() for k in ("comp_rgb", "comp_depth", "comp_mask")},
                 **{"grad_" + k: v.grad.numpy() for k, v in params.items()},
                 **{f"stat{i}": s.numpy() for i, s in enumerate(stats)})
    finally:
        dist.destroy_process_group()


def test_shard_range_covers_batch():
    for bs in (1, 5, 8, 64):
        for world in (1, 2, 3, 8):
            spans = [shard_range(bs, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == bs
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("world,reg", [(2, False), (3, False), (2, True)])
def test_sharded_batch_equals_single_process(world, reg, tmp_path):
    """reg: the loss also holds parameter-direct regularisers, added through replicated_loss on every rank
    (without the 1/world scaling the summed all-reduce would count them `world` times)."""
    ref_imgs, ref_grads, ref_stats = _single_process(reg)
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), reg), nprocs=world, join=True)
    for rank in range(world):
        z = np.load(tmp_path / f"rank{rank}.npz")
        for k, v in ref_imgs.items():
            np.testing.assert_array_equal(z[k], v, err_msg=f"rank {rank} {k}")
        for k, v in ref_grads.items():
            np.testing.assert_allclose(z["grad_" + k], v, rtol=1e-10, atol=1e-12, err_msg=f"rank {rank} grad {k}")
        for i, v in enumerate(ref_stats):
            np.testing.assert_allclose(z[f"stat{i}"], v, rtol=1e-6, atol=1e-9, err_msg=f"rank {rank} stat {i}")


class _CarvedGrads(torch.autograd.Function):
    """Backward returns its inputs' gradients as views of one buffer, as batched.py's backward does."""

    @staticmethod
    def forward(ctx, scale, *xs):
        ctx.scale = scale
        ctx.shapes = [x.shape for x in xs]
        return sum(x.sum() for x in xs) * 0.0

    @staticmethod
    def backward(ctx, g):
        n = [math.prod(s) for s in ctx.shapes]
        flat = torch.empty(sum(n), dtype=torch.float64)
        out, off = [], 0
        for s, k in zip(ctx.shapes, n):
            out.append(flat[off:off + k].view(s))
            off += k
        flat.copy_(torch.arange(flat.numel(), dtype=torch.float64) * ctx.scale)
        return (None, *out)


def _span_worker(rank, world, port, tmp):
    # file rendezvous (no TCP port to race for); `port` only makes the file name unique
    dist.init_process_group("gloo", init_method="file://" + os.path.join(tmp, f"rendezvous_{port}"), rank=rank,
                            world_size=world)
    try:
        params = [torch.zeros(s, dtype=torch.float64, requires_grad=True) for s in ((7, 3), (7, 1), (7, 16, 3))]
        _CarvedGrads.apply(float(rank + 1), *params).backward()
        base = params[0].grad.untyped_storage().data_ptr()
        shared = all(p.grad.untyped_storage().data_ptr() == base for p in params)
        ptrs = [p.grad.data_ptr() for p in params]
        allreduce_grads(params)
        same = [p.grad.data_ptr() for p in params] == ptrs
        np.savez(os.path.join(tmp, f"span{rank}.npz"), shared=shared, same=same,
                 **{f"g{i}": p.grad.numpy() for i, p in enumerate(params)})
    finally:
        dist.destroy_process_group()


def test_allreduce_carved_grads_in_place(tmp_path):
    """Gradients carved from one buffer reach the leaves without a copy and are summed in place."""
    world = 2
    mp.spawn(_span_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    total = sum(r + 1 for r in range(world))
    for rank in range(world):
        z = np.load(tmp_path / f"span{rank}.npz")
        assert bool(z["shared"]) and bool(z["same"])
        flat = np.concatenate([z[f"g{i}"].reshape(-1) for i in range(3)])
        np.testing.assert_array_equal(flat, np.arange(flat.size, dtype=np.float64) * total)


def test_contiguous_span_detection():
    from diff_gaussian_rasterization.view_shard import _contiguous_span
    buf = torch.arange(20.0)
    a, b, c = buf[0:6].view(2, 3), buf[6:10], buf[10:20].view(5, 2)
    span = _contiguous_span([c, a, b])
    assert span is not None and span.data_ptr() == buf.data_ptr() and span.numel() == 20
    assert _contiguous_span([a, c]) is None            # gap
    assert _contiguous_span([buf[0:6], buf[4:10]]) is None  # overlap
    assert _contiguous_span([a, torch.zeros(4)]) is None    # another buffer
    assert _contiguous_span([buf[0:10:2]]) is None          # strided


def _densify_views(P, B, lo, hi):
    """Per-view densification inputs of views [lo, hi) (as the renderer returns them), deterministic per
    view so that the union over ranks is the single-process batch."""
    radii, vps, vis = [], [], []
    for v in range(lo, hi):
        g = torch.Generator().manual_seed(1000 + v)
        r = torch.randint(0, 6, (P,), generator=g, dtype=torch.int32)
        vp = torch.zeros(P, 3, requires_grad=True)
        vp.grad = torch.randn(P, 3, generator=g) * 0.02
        radii.append(r)
        vps.append(vp)
        vis.append(r > 0)
    return {"radii": radii, "viewspace_points": vps, "visibility_filter": vis}


def _densify_worker(rank, world, port, tmp, synced):
    import densify_reference as dr
    from diff_gaussian_rasterization.view_shard import replica_checksum, update_states_sharded

    # file rendezvous (no TCP port to race for); `port` only makes the file name unique
    dist.init_process_group("gloo", init_method="file://" + os.path.join(tmp, f"rendezvous_{port}"), rank=rank,
                            world_size=world)
    try:
        torch.manual_seed(100 + rank)  # the usual per-rank seeding
        scene = gs.make_scene(200, sh_degree=1, seed=8, radius=0.5)
        model = dr.DensifyModel(scene, "cpu", densify_grad_threshold=0.005)
        B = 6
        lo, hi = shard_range(B, world, rank)
        outs = _densify_views(200, B, lo, hi)
        if synced:
            update_states_sharded(model, 5, outs)
        else:  # the reduced statistics, but the densification draws left to each rank's RNG
            max_r, gsum, cnt = reduce_densify_stats(outs["radii"], outs["viewspace_points"], outs["visibility_filter"], 200)
            model.max_radii2D = torch.max(model.max_radii2D, max_r)
            model.xyz_gradient_accum += gsum[:, None]
            model.denom += cnt[:, None]
            model.update_states(5, [], [], [])
        tensors = model.parameters() + [model.xyz_gradient_accum, model.max_radii2D]
        same = replica_checksum(tensors)
        np.savez(os.path.join(tmp, f"dens{int(synced)}_{rank}.npz"), same=same, P=model.get_xyz.shape[0],
                 xyz=model.get_xyz.detach().numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("synced", [True, False])
def test_densify_keeps_replicas_identical(synced, tmp_path):
    """update_states_sharded: reduced statistics + replica_rng -> every rank densifies and prunes the same
    Gaussians with the same random split samples (bitwise-identical replicas); without the shared RNG the
    split samples differ between ranks (the test is sensitive to it)."""
    import densify_reference as dr

    world = 2
    mp.spawn(_densify_worker, args=(world, _free_port(), str(tmp_path), synced), nprocs=world, join=True)
    z = [np.load(tmp_path / f"dens{int(synced)}_{r}.npz") for r in range(world)]
    # single process over the whole batch: same Gaussian count (the decisions do not depend on the samples)
    model = dr.DensifyModel(gs.make_scene(200, sh_degree=1, seed=8, radius=0.5), "cpu", densify_grad_threshold=0.005)
    outs = _densify_views(200, 6, 0, 6)
    model.update_states(5, outs["visibility_filter"], outs["radii"], outs["viewspace_points"])
    assert int(z[0]["P"]) == int(z[1]["P"]) == model.get_xyz.shape[0] > 200
    if synced:
        assert bool(z[0]["same"]) and bool(z[1]["same"])
        np.testing.assert_array_equal(z[0]["xyz"], z[1]["xyz"])
    else:
        assert not bool(z[0]["same"])


def _grad_flag_worker(rank, world, port, tmp):
    dist.init_process_group("gloo", init_method="file://" + os.path.join(tmp, f"rendezvous_{port}"), rank=rank,
                            world_size=world)
    try:
        used = torch.zeros(4, dtype=torch.float64, requires_grad=True)      # every rank
        only0 = torch.zeros(3, dtype=torch.float64, requires_grad=True)     # rank 0 only (a rank without views)
        unused = torch.zeros(2, dtype=torch.float64, requires_grad=True)    # no rank
        loss = (used * (rank + 1)).sum() + ((only0 * 2.0).sum() if rank == 0 else 0)
        loss.backward()
        allreduce_grads([used, only0, unused])
        np.savez(os.path.join(tmp, f"flags{rank}.npz"), used=used.grad.numpy(), only0=only0.grad.numpy(),
                 unused_none=unused.grad is None)
    finally:
        dist.destroy_process_group()


def test_allreduce_keeps_untouched_grads_none(tmp_path):
    """A parameter no rank has a gradient for keeps .grad = None (the single-process reference's state, which
    optimizers skip); one only some ranks touched is summed with zeros from the others."""
    world = 2
    mp.spawn(_grad_flag_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for rank in range(world):
        z = np.load(tmp_path / f"flags{rank}.npz")
        np.testing.assert_array_equal(z["used"], np.full(4, 3.0))
        np.testing.assert_array_equal(z["only0"], np.full(3, 2.0))
        assert bool(z["unused_none"])


class _TemporalRenderer:
    """A per-view renderer that reads the camera's timestamp / frame index, as the temporal and spacetime
    renderers do (renderer/diff_sugar_rasterizer_temporal.py:150,181, renderer/diff_gaussian_rasterizer_st.py:135),
    and records the autocast state its forward runs under."""

    def __init__(self, params):
        self.geometry = object()
        self.background_tensor = torch.zeros(3)
        self.params = params
        self.seen = []

    def forward(self, cam, bg, **batch):
        self.seen.append((float(cam.timestamp), int(cam.frame_idx), torch.is_autocast_enabled("cpu")))
        t = self.params["means3D"].sum() * float(cam.timestamp)
        P = 3
        sp = torch.zeros(P, 3, requires_grad=True)
        img = torch.ones(3, 4, 4, dtype=torch.float64) * t
        return {"render": img, "viewspace_points": sp, "visibility_filter": torch.ones(P, dtype=torch.bool),
                "radii": torch.ones(P, dtype=torch.int32)}


def test_per_view_fallback_passes_timestamp_and_disables_autocast():
    params = _params()
    r = _TemporalRenderer(params)
    batch = _batch()
    batch.update(timestamp=torch.linspace(0.1, 0.5, B), frame_indices=torch.arange(B) + 7, height=4, width=4)
    with torch.autocast(device_type="cpu", dtype=torch.bfloat16):
        out = ViewShardedBatchRenderer(r).batch_forward(batch)
    assert [s[1] for s in r.seen] == list(range(7, 7 + B))
    np.testing.assert_allclose([s[0] for s in r.seen], np.linspace(0.1, 0.5, B), rtol=1e-6)
    assert not any(s[2] for s in r.seen)
    assert out["comp_rgb"].shape == (B, 4, 4, 3)


def test_grad_chunk_range_matches_library():
    from diff_gaussian_rasterization import _C
    from diff_gaussian_rasterization.view_shard import grad_chunk_range

    lib = _C.load_library()
    import ctypes

    for P in (0, 1, 4095, 4096, 4097, 100_000, 1_000_000, 1_966_080):
        for n in (1, 2, 3, 4, 7, 16):
            covered = 0
            for c in range(n):
                a, b = ctypes.c_int(), ctypes.c_int()
                assert lib.gsr_grad_chunk_range(P, n, c, ctypes.byref(a), ctypes.byref(b)) == 0
                assert (a.value, b.value) == grad_chunk_range(P, n, c)
                assert a.value == min(covered, P) and b.value >= a.value
                assert a.value % 4096 == 0 or a.value == P
                covered = b.value
            assert covered == P


def _chunk_worker(rank, world, port, tmp):
    from diff_gaussian_rasterization.view_shard import ChunkedGradReduce

    dist.init_process_group("gloo", init_method="file://" + os.path.join(tmp, f"rendezvous_{port}"), rank=rank,
                            world_size=world)
    try:
        P = 10_000
        g = torch.Generator().manual_seed(rank)
        shapes = [(P, 3), (P, 1), (P, 16, 3), (P, 4)]
        a = [torch.randn(s, generator=g) for s in shapes]
        b = [t.clone() for t in a]
        params = [torch.zeros(s, requires_grad=True) for s in shapes]
        for p, t in zip(params, a):
            p.grad = t
        allreduce_grads(params)
        ChunkedGradReduce(n_chunks=3).launch(b, P)
        np.savez(os.path.join(tmp, f"chunk{rank}.npz"), **{f"a{i}": p.grad.numpy() for i, p in enumerate(params)},
                 **{f"b{i}": t.numpy() for i, t in enumerate(b)})
    finally:
        dist.destroy_process_group()


def test_chunked_reduce_equals_flat(tmp_path):
    """ChunkedGradReduce (range-by-range grouped all-reduces, overlapped with the backward on the GPU) gives
    bitwise the flat all-reduce's sums."""
    world = 2
    mp.spawn(_chunk_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for rank in range(world):
        z = np.load(tmp_path / f"chunk{rank}.npz")
        for i in range(4):
            np.testing.assert_array_equal(z[f"a{i}"], z[f"b{i}"])


def _async_gather_worker(rank, world, port, tmp, batch):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        from diff_gaussian_rasterization.view_shard import all_gather_views, all_gather_views_async

        lo, hi = shard_range(batch, world, rank)
        local = (torch.arange(lo, hi, dtype=torch.float32)[:, None, None] * 10.0
                 + torch.arange(6, dtype=torch.float32).reshape(1, 2, 3)).requires_grad_(True)
        pending = all_gather_views_async(local, batch)
        sync = all_gather_views(local, batch)
        out = pending.wait()
        np.save(os.path.join(tmp, f"async{rank}.npy"), out.numpy())
        np.save(os.path.join(tmp, f"sync{rank}.npy"), sync.detach().numpy())
        assert not out.requires_grad
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,batch", [(2, 8), (3, 7)])
def test_async_gather_equals_sync(world, batch, tmp_path):
    """all_gather_views_async (the bench's gather overlapped with the backward) returns the same batch as the
    synchronous all_gather_views, for even and uneven shards."""
    mp.spawn(_async_gather_worker, args=(world, _free_port(), str(tmp_path), batch), nprocs=world, join=True)
    want = (np.arange(batch, dtype=np.float32)[:, None, None] * 10.0
            + np.arange(6, dtype=np.float32).reshape(1, 2, 3))
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"async{r}.npy"), want)
        np.testing.assert_array_equal(np.load(tmp_path / f"sync{r}.npy"), want)


def test_world_one_group_skips_collectives_unless_opted_in(tmp_path):
    """a world-size-1 process group (a single-GPU run under a launcher) issues no collectives by
    default — the gather returns the local slice itself and the chunked reduction is inactive; with
    view_shard.COLLECTIVES_AT_WORLD_ONE (the one-GPU RCCL test) the same calls run the collectives, as identities."""
    from diff_gaussian_rasterization import view_shard

    dist.init_process_group("gloo", init_method="file://" + os.path.join(str(tmp_path), "rdv_w1"), rank=0,
                            world_size=1)
    try:
        x = torch.randn(3, 2, 4, requires_grad=True)
        assert view_shard.all_gather_views(x, 3) is x
        assert not view_shard.ChunkedGradReduce(n_chunks=2).active()
        view_shard.COLLECTIVES_AT_WORLD_ONE = True
        try:
            g = view_shard.all_gather_views(x, 3)
            assert g is not x and torch.equal(g, x.detach()) and g.grad_fn is not None
            assert view_shard.ChunkedGradReduce(n_chunks=2).active()
        finally:
            view_shard.COLLECTIVES_AT_WORLD_ONE = False
    finally:
        dist.destroy_process_group()

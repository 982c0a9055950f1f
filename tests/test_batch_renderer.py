"""The drop-in batch renderer (diff_gaussian_rasterization/batch_renderer.py) on CPU: the fused
view-set path against the reference's per-view loop (renderer/gaussian_batch_renderer.py:9-122) with
the same renderer, and sharded over gloo ranks (world 2 and 3, including a batch smaller than the world,
where a rank renders no view but still joins every gather).  The rasterizer is the torch formulation
(tests/renderer_fixtures.py), so this checks the batching, camera, key and sharding logic; the HIP
path is checked by tests/test_gpu_batch_renderer.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import renderer_fixtures as rf
from diff_gaussian_rasterization import batch_renderer as br
from diff_gaussian_rasterization.view_shard import ViewShardedBatchRenderer, allreduce_grads, shard_range
from gsr_testutil import gs

H, W = 24, 20


def _scene():
    return gs.make_scene(30, sh_degree=1, seed=5, radius=0.5)


_SWAPS = (("_rasterize_views", rf.torch_rasterize_views), ("_shade_views", rf.torch_shade_views),
          ("_depth_normal_maps", rf.torch_depth_normal_maps), ("_depth_normal_views", rf.torch_depth_normal_views),
          ("_sugar_normal_map", rf.torch_sugar_normal_map))


def _cpu(monkeypatch=None):
    if monkeypatch is not None:
        monkeypatch.setattr(rf, "RASTERIZE", rf.torch_rasterize)
        for name, fn in _SWAPS:
            monkeypatch.setattr(br, name, fn)
    else:
        rf.RASTERIZE = rf.torch_rasterize
        for name, fn in _SWAPS:
            setattr(br, name, fn)


def _run(renderer, batch):
    out = renderer.batch_forward(batch)
    rf.loss_of(out).backward()
    grads = {k: v.grad.clone() for k, v in renderer.geometry.params.items() if v.grad is not None}
    return out, grads


def _mode_scene(mode):
    if mode in ("sugar_normal", "sugar_shading"):
        sc = gs.make_sugar_scene(1, sh_degree=0, seed=2)
        sc["shs"] = sc["shs"][:, :1]
        return sc
    return _scene()


@pytest.mark.parametrize("mode,training,pred_normal", [
    ("plain", False, False), ("background", False, False), ("advanced", False, False), ("shading", False, False),
    ("normal", False, False), ("sugar_normal", False, False), ("sugar_shading", False, False),
    # training: the per-view random draws (background inversion; soft-shading ambient ratio and shading mode)
    ("plain", True, False), ("advanced", True, False), ("normal", True, False), ("shading", True, False),
    ("sugar_normal", True, False), ("sugar_shading", True, False),
    # the predicted-normal second pass (renderer/diff_gaussian_rasterizer_shading.py:177-197, _normal.py:175-185)
    ("shading", True, True), ("normal", False, True),
])
def test_fused_equals_per_view_loop(mode, training, pred_normal, monkeypatch):
    """Each fused mode against the reference's per-view loop over the same renderer: same outputs, gradients
    and — with the RNGs seeded alike — the same per-view random draws (B = 7 views, so that a per-batch draw
    would differ from the per-view ones)."""
    import random

    _cpu(monkeypatch)
    batch = rf.make_batch(7, H, W, "cpu", torch.float64)
    kw = dict(training=training, soft_shading=training, pred_normal=pred_normal)
    random.seed(11), np.random.seed(11)
    fused, g_fused = _run(rf.FakeRenderer(mode, _mode_scene(mode), "cpu", torch.float64, **kw), dict(batch))
    draws_fused = (random.random(), np.random.rand())
    random.seed(11), np.random.seed(11)
    ref, g_ref = _run(rf.PerViewRenderer(mode, _mode_scene(mode), "cpu", torch.float64, **kw), dict(batch))
    assert draws_fused == (random.random(), np.random.rand()), "the fused path consumed other draws than the loop"
    assert set(k for k in ref if k.startswith("comp_")) == set(k for k in fused if k.startswith("comp_"))
    for k in ref:
        if k.startswith("comp_"):
            assert fused[k].shape == ref[k].shape, k
            torch.testing.assert_close(fused[k], ref[k], rtol=1e-12, atol=1e-12)
    if pred_normal:
        assert "comp_pred_normal" in fused and "normals" in g_ref
    for i in range(7):
        assert torch.equal(fused["radii"][i], ref["radii"][i])
        assert torch.equal(fused["visibility_filter"][i], ref["visibility_filter"][i])
        torch.testing.assert_close(fused["viewspace_points"][i].grad, ref["viewspace_points"][i].grad,
                                   rtol=1e-10, atol=1e-12)
    for k in g_ref:
        torch.testing.assert_close(g_fused[k], g_ref[k], rtol=1e-10, atol=1e-12)


def test_mode_detection():
    class Plain:
        pass

    Plain.__module__ = "threestudio_3dgs.renderer.diff_gaussian_rasterizer_background"
    assert br.batch_mode(Plain()) == "background"
    Plain.__module__ = "threestudio_3dgs.renderer.diff_gaussian_rasterizer_advanced"
    assert br.batch_mode(Plain()) == "advanced"
    Plain.__module__ = "threestudio_3dgs.renderer.diff_gaussian_rasterizer_normal"
    assert br.batch_mode(Plain()) == "normal"
    Plain.__module__ = "threestudio_3dgs.renderer.diff_sugar_rasterizer_shading"
    assert br.batch_mode(Plain()) == "sugar_shading"
    Plain.__module__ = "threestudio_3dgs.renderer.diff_sugar_rasterizer_temporal"
    assert br.batch_mode(Plain()) is None  # keeps the per-view loop
    p = Plain()
    p.batch_render_mode = "shading"
    assert br.batch_mode(p) == "shading"
    p.batch_render_mode = "nope"
    with pytest.raises(ValueError):
        br.batch_mode(p)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, tmp, B, kind):
    # file rendezvous (no TCP port to race for); `port` only makes the file name unique
    dist.init_process_group("gloo", init_method="file://" + os.path.join(tmp, f"rendezvous_{port}"), rank=rank,
                            world_size=world)
    try:
        _cpu()
        batch = rf.make_batch(B, H, W, "cpu", torch.float64)
        if kind == "fused":
            r = rf.FakeRenderer("background", _scene(), "cpu", torch.float64)
            out, _ = _run(r, batch)
        elif kind == "fused_shading_train":  # per-view random lights: the rank's views get the loop's draws
            import random

            random.seed(5)
            r = rf.FakeRenderer("shading", _scene(), "cpu", torch.float64, training=True, soft_shading=True)
            out, _ = _run(r, batch)
        else:  # the callback form of ViewShardedBatchRenderer (per-view forward)
            r = rf.PerViewRenderer("background", _scene(), "cpu", torch.float64)
            out = ViewShardedBatchRenderer(r).batch_forward(batch)
            rf.loss_of(out).backward()
        lo, hi = shard_range(B, world, rank)
        assert out["view_range"] == (lo, hi) and len(out["radii"]) == hi - lo
        allreduce_grads(list(r.geometry.params.values()))
        np.savez(os.path.join(tmp, f"{kind}{rank}.npz"), comp_rgb=out["comp_rgb"].detach().numpy(),
                 **{"g" + k: v.grad.numpy() for k, v in r.geometry.params.items()})
    finally:
        dist.destroy_process_group()


def _reduce_worker(rank, world, port, tmp, B, mode, pred_normal):
    from diff_gaussian_rasterization.view_shard import ChunkedGradReduce

    dist.init_process_group("gloo", init_method="file://" + os.path.join(tmp, f"rendezvous_{port}"), rank=rank,
                            world_size=world)
    try:
        _cpu()
        batch = rf.make_batch(B, H, W, "cpu", torch.float64)
        r = rf.FakeRenderer(mode, _mode_scene(mode), "cpu", torch.float64, pred_normal=pred_normal)
        r.grad_reduce = ChunkedGradReduce(n_chunks=3)
        out, _ = _run(r, batch)  # gradients already summed over ranks inside the backward (no allreduce_grads)
        lo, hi = shard_range(B, world, rank)
        assert len(out["radii"]) == hi - lo
        np.savez(os.path.join(tmp, f"red{rank}.npz"), comp_rgb=out["comp_rgb"].detach().numpy(),
                 **{"g" + k: v.grad.numpy() for k, v in r.geometry.params.items() if v.grad is not None})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,B,mode,pred_normal", [
    (2, 1, "background", False),   # rank 1 renders no view
    (3, 2, "background", False),   # rank 2 renders no view
    (2, 3, "shading", True),       # main + predicted-normal call: one reduction after both
    (2, 1, "normal", True),        # ... and a view-less rank joining it
    (2, 1, "sugar_normal", False),  # two colour sets (colors2 gradient in the reduction)
    (2, 3, "sugar_shading", False),  # ... with the material on the blended normals, views split 2 / 1
])
def test_grad_reduce_with_viewless_ranks(world, B, mode, pred_normal, tmp_path, monkeypatch):
    """renderer.grad_reduce (the per-Gaussian gradients summed over ranks inside the rasterizer's backward) with
    a batch smaller than the world: ranks without views join the ranged collectives with zero gradients
    (batch_renderer._join_reduce), so no rank blocks and every replica ends with the single-process gradient;
    with the predicted-normal pass one reduction covers both calls."""
    _cpu(monkeypatch)
    batch = rf.make_batch(B, H, W, "cpu", torch.float64)
    r = rf.FakeRenderer(mode, _mode_scene(mode), "cpu", torch.float64, pred_normal=pred_normal)
    out, grads = _run(r, batch)
    mp.spawn(_reduce_worker, args=(world, _free_port(), str(tmp_path), B, mode, pred_normal), nprocs=world,
             join=True)
    for rank in range(world):
        z = np.load(tmp_path / f"red{rank}.npz")
        np.testing.assert_array_equal(z["comp_rgb"], out["comp_rgb"].detach().numpy())
        assert set(k[1:] for k in z.files if k.startswith("g")) == set(grads), f"rank {rank}"
        for k, v in grads.items():
            np.testing.assert_allclose(z["g" + k], v.numpy(), rtol=1e-10, atol=1e-12, err_msg=f"rank {rank} {k}")


@pytest.mark.parametrize("world,B", [(2, 5), (3, 2)])
@pytest.mark.parametrize("kind", ["fused", "callback", "fused_shading_train"])
def test_sharded_equals_single_process(world, B, kind, tmp_path, monkeypatch):
    import random

    _cpu(monkeypatch)
    batch = rf.make_batch(B, H, W, "cpu", torch.float64)
    if kind == "fused_shading_train":
        random.seed(5)
        r = rf.FakeRenderer("shading", _scene(), "cpu", torch.float64, training=True, soft_shading=True)
    else:
        r = rf.FakeRenderer("background", _scene(), "cpu", torch.float64)
    out, grads = _run(r, batch)
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), B, kind), nprocs=world, join=True)
    for rank in range(world):
        z = np.load(tmp_path / f"{kind}{rank}.npz")
        np.testing.assert_array_equal(z["comp_rgb"], out["comp_rgb"].detach().numpy())
        for k, v in grads.items():
            np.testing.assert_allclose(z["g" + k], v.numpy(), rtol=1e-10, atol=1e-12, err_msg=f"rank {rank} {k}")

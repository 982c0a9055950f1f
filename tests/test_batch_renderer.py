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


def _cpu(monkeypatch=None):
    if monkeypatch is not None:
        monkeypatch.setattr(rf, "RASTERIZE", rf.torch_rasterize)
        monkeypatch.setattr(br, "_rasterize_views", rf.torch_rasterize_views)
    else:
        rf.RASTERIZE = rf.torch_rasterize
        br._rasterize_views = rf.torch_rasterize_views


def _run(renderer, batch):
    out = renderer.batch_forward(batch)
    rf.loss_of(out).backward()
    grads = {k: v.grad.clone() for k, v in renderer.geometry.params.items() if v.grad is not None}
    return out, grads


@pytest.mark.parametrize("mode", ["plain", "background"])
def test_fused_equals_per_view_loop(mode, monkeypatch):
    _cpu(monkeypatch)
    batch = rf.make_batch(3, H, W, "cpu", torch.float64)
    fused, g_fused = _run(rf.FakeRenderer(mode, _scene(), "cpu", torch.float64), dict(batch))
    ref, g_ref = _run(rf.PerViewRenderer(mode, _scene(), "cpu", torch.float64), dict(batch))
    assert set(k for k in ref if k.startswith("comp_")) == set(k for k in fused if k.startswith("comp_"))
    for k in ref:
        if k.startswith("comp_"):
            assert fused[k].shape == ref[k].shape, k
            torch.testing.assert_close(fused[k], ref[k], rtol=1e-12, atol=1e-12)
    for i in range(3):
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


@pytest.mark.parametrize("world,B", [(2, 5), (3, 2)])
@pytest.mark.parametrize("kind", ["fused", "callback"])
def test_sharded_equals_single_process(world, B, kind, tmp_path, monkeypatch):
    _cpu(monkeypatch)
    batch = rf.make_batch(B, H, W, "cpu", torch.float64)
    r = rf.FakeRenderer("background", _scene(), "cpu", torch.float64)
    out, grads = _run(r, batch)
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), B, kind), nprocs=world, join=True)
    for rank in range(world):
        z = np.load(tmp_path / f"{kind}{rank}.npz")
        np.testing.assert_array_equal(z["comp_rgb"], out["comp_rgb"].detach().numpy())
        for k, v in grads.items():
            np.testing.assert_allclose(z["g" + k], v.numpy(), rtol=1e-10, atol=1e-12, err_msg=f"rank {rank} {k}")

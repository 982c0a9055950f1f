"""The RCCL (torch.distributed "nccl") code path of the view-sharded batch renderer executed on one GPU
(VERDICT r04 "missing" 1 / "next" 6): a child process opens a world-size-1 "nccl" process group
(device_id = cuda:0, before any other GPU work in that process), then renders one training step of the
background renderer through the batch renderer twice — with the gradient all-reduce inside the rasterizer's
backward (view_shard.ChunkedGradReduce: per-range events, a side stream, grouped RCCL all-reduces) and with
view_shard.allreduce_grads afterwards (one in-place flat RCCL all-reduce) — plus the synchronous and the
asynchronous image all-gather (all_gather_into_tensor), with view_shard.COLLECTIVES_AT_WORLD_ONE set (by default a
world-1 group skips the collectives).  At world size 1 every collective is an identity, so
images, gradients and the gathered batches must be bitwise those of the same step without a process group.
Multi-rank RCCL (xGMI) stays for the driver's 8-GPU run; the multi-rank logic is covered by the gloo tests.

Reference: renderer/gaussian_batch_renderer.py:21-76 (the batch the ranks split), SURVEY.md §8e.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))

CHILD = r'''
import os, sys, socket
import numpy as np
import torch
import torch.distributed as dist

s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))  # before any other GPU work here
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
import test_gpu_batch_renderer as t
from diff_gaussian_rasterization import view_shard
view_shard.COLLECTIVES_AT_WORLD_ONE = True  # run the RCCL path although the world has one rank

out = sys.argv[1]
torch.manual_seed(100)
t._step((0, 1), 5, out, "rccl_overlap", overlap=True)    # ChunkedGradReduce inside the backward
torch.manual_seed(100)
t._step((0, 1), 5, out, "rccl_flat", overlap=False)      # allreduce_grads afterwards
x = torch.randn((5, 3, 32, 32), device="cuda", requires_grad=True)
g = view_shard.all_gather_views(x, 5)
g.backward(torch.ones_like(g))
a = view_shard.all_gather_views_async(x.detach() * 2, 5).wait()
torch.cuda.synchronize()
np.savez(os.path.join(out, "gather.npz"), x=x.detach().cpu().numpy(), g=g.detach().cpu().numpy(),
         xg=x.grad.cpu().numpy(), a=a.cpu().numpy())
dist.destroy_process_group()
print("rccl child ok")
'''


def test_rccl_world1_equals_no_collectives(tmp_path):
    import test_gpu_batch_renderer as t

    import torch

    torch.manual_seed(100)
    t._step((0, 1), 5, str(tmp_path), "plain")  # the same step without a process group
    env = dict(os.environ, PYTHONPATH=os.pathsep.join(p for p in sys.path if p))
    res = subprocess.run([sys.executable, "-c", CHILD, str(tmp_path)], cwd=HERE, env=env, capture_output=True,
                         text=True, timeout=280)
    assert res.returncode == 0 and "rccl child ok" in res.stdout, (res.stdout[-2000:], res.stderr[-4000:])
    plain = np.load(tmp_path / "plain0.npz")
    for tag in ("rccl_overlap", "rccl_flat"):
        z = np.load(tmp_path / f"{tag}0.npz")
        np.testing.assert_array_equal(z["comp_rgb"], plain["comp_rgb"], err_msg=tag)
        for i in range(6):
            np.testing.assert_array_equal(z[f"g{i}"], plain[f"g{i}"], err_msg=f"{tag} grad {i}")
        assert int(z["P"]) == int(plain["P"])
    gz = np.load(tmp_path / "gather.npz")
    np.testing.assert_array_equal(gz["g"], gz["x"])
    np.testing.assert_array_equal(gz["xg"], np.ones_like(gz["x"]))
    np.testing.assert_array_equal(gz["a"], 2 * gz["x"])

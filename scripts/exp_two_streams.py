"""Timing experiment (not part of the product or the bench): one 64-view set vs two 32-view sets issued on two HIP
streams, forward + backward of bench.py's default workload.  Prints one JSON line per mode.

    python scripts/exp_two_streams.py [--steps 10] [--warmup 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "threestudio-3dgs_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import gsr_synthetic as gs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--views", type=int, default=64)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    scene = gs.make_scene(1_000_000, sh_degree=3, seed=0)
    rep = bench.Replica(scene, dev)
    cams = bench.build_views(a.views, 1024, dev)
    bg_zero = torch.zeros(3, device=dev)
    st = [bench.settings_for(rep, c, bg_zero) for c in cams]
    gen = torch.Generator(device=dev).manual_seed(1234)
    V, H = a.views, 1024
    bg_img = torch.rand((V, H, H, 3), generator=gen, device=dev).requires_grad_(True)
    up = [torch.randn((V, c, H, H), generator=gen, device=dev) for c in (3, 1, 1)]
    half = V // 2
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def one_set():
        c, d, al, _ = bench.render_views(rep, st, bg_img)
        torch.autograd.backward((c, d, al), tuple(up))

    def two_sets(streams):
        outs, grads = [], []
        cur = torch.cuda.current_stream(dev)
        for i, sl in enumerate((slice(0, half), slice(half, V))):
            s = streams[i] if streams else cur
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                c, d, al, _ = bench.render_views(rep, st[sl], bg_img[sl])
            outs += [c, d, al]
            grads += [u[sl] for u in up]
        torch.autograd.backward(tuple(outs), tuple(grads))
        if streams:
            for s in streams:
                cur.wait_stream(s)

    modes = {"one_set_64": one_set, "two_sets_serial": lambda: two_sets(None),
             "two_sets_two_streams": lambda: two_sets((s1, s2))}
    for rnd in range(2):
        for name, fn in modes.items():
            for _ in range(a.warmup):
                fn()
                rep.zero_grad()
                bg_img.grad = None
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                fn()
                rep.zero_grad()
                bg_img.grad = None
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.steps * 1e3
            print(json.dumps({"mode": name, "round": rnd, "ms_per_step": round(ms, 3),
                              "views_per_s": round(V / ms * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()

"""View-sharded batch rendering across the GPUs of one node.

The reference renders a batch with a serial per-view Python loop on one device
(GaussianBatchRenderer.batch_forward, renderer/gaussian_batch_renderer.py:9-122) and has no
distributed code.  Views are independent given replicated Gaussians, so here rank r of G renders
views [r*B/G, (r+1)*B/G) of the batch with a full replica of the Gaussian parameters, and:

  forward   the rendered images are all-gathered (RCCL over xGMI; the north_star exchange) so that
            every rank holds the full batch for batch-level losses (e.g. MVDream's multi-view SDS).
            Only the local slice carries autograd history, so each view's gradient is computed on
            exactly one rank.
  backward  allreduce_grads() sums the per-Gaussian parameter gradients (one flat bucket), giving every
            replica the full-batch gradient; reduce_densify_stats() pre-reduces the densification
            statistics (max radii, sum of |means2D.grad[:, :2]|, visibility counts) that
            geometry/gaussian_base.py:815-851 would otherwise need per view from every rank.

One process per GPU; `torch.distributed` backend "nccl" is RCCL on ROCm.  Everything here is also
exercised with the gloo backend on CPU (tests/test_view_shard.py).
"""
from __future__ import annotations

import contextlib
from typing import Callable

import torch
import torch.distributed as dist

# render_pkg keys of the reference wrappers that are per-view images (C, H, W) -> stacked to BHWC
_IMAGE_KEYS = (("render", "comp_rgb"), ("normal", "comp_normal"), ("normal_from_dist", "comp_normal_from_dist"),
               ("pred_normal", "comp_pred_normal"), ("depth", "comp_depth"), ("mask", "comp_mask"))


def _world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


# Opt-in: issue the collectives also in a world-size-1 process group, where they are identities — the
# one-GPU run of the RCCL path (tests/test_gpu_rccl.py sets it).  Off by default, so a single-GPU run under a
# launcher that opens a process group pays for no per-range events, side-stream reductions or gather copies.
COLLECTIVES_AT_WORLD_ONE = False


def _collect() -> bool:
    """The view gather and the gradient reductions issue their collectives when a process group of more than one
    rank exists (or of one rank with COLLECTIVES_AT_WORLD_ONE); otherwise they are skipped."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size() > 1 or COLLECTIVES_AT_WORLD_ONE


def shard_range(batch_size: int, world: int, rank: int):
    """Contiguous view slice of `rank`; views are split as evenly as possible (first ranks take the remainder)."""
    base, extra = divmod(batch_size, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


class _GatherViews(torch.autograd.Function):
    """All-gather of per-rank view slices; the gradient of the gathered batch flows back to the local
    slice only (each view's gradient is computed on exactly one rank)."""

    @staticmethod
    def forward(ctx, local, batch_size, group):
        world, rank = _world()
        counts = [shard_range(batch_size, world, r) for r in range(world)]
        s, e = counts[rank]
        ctx.slice = (s, e)
        n_max = max(b - a for a, b in counts)
        even = all(b - a == n_max for a, b in counts)
        if dist.get_backend(group) == "nccl" and even:
            # equal slices: RCCL writes every rank's slice straight into the batch tensor (no staging copies)
            out = local.new_empty((batch_size,) + tuple(local.shape[1:]))
            dist.all_gather_into_tensor(out, local.detach().contiguous(), group=group)
            return out
        pad = local.new_zeros((n_max,) + tuple(local.shape[1:]))
        pad[: local.shape[0]] = local.detach()
        if dist.get_backend(group) == "nccl":
            buf = local.new_empty((world * n_max,) + tuple(local.shape[1:]))
            dist.all_gather_into_tensor(buf, pad.contiguous(), group=group)
            parts = list(buf.split(n_max))
        else:
            parts = [torch.empty_like(pad) for _ in range(world)]
            dist.all_gather(parts, pad.contiguous(), group=group)
        return torch.cat([parts[r][: b - a] for r, (a, b) in enumerate(counts)], 0)

    @staticmethod
    def backward(ctx, grad):
        s, e = ctx.slice
        return grad[s:e], None, None


def all_gather_views(local: torch.Tensor, batch_size: int, group=None) -> torch.Tensor:
    """Gather per-rank view slices (n_r, ...) into the full (batch_size, ...) tensor on every rank.

    Autograd: the gathered tensor's gradient reaches the local slice only; the other ranks' slices are
    constants here (their views' gradients are computed on their own ranks).
    """
    if not _collect():
        return local
    return _GatherViews.apply(local, batch_size, group)


class PendingGather:
    """An all-gather of view slices in flight (all_gather_views_async): wait() returns the (batch_size, ...)
    tensor, a constant (no autograd history), after making the current stream wait for the collective."""

    def __init__(self, work, finish):
        self._work, self._finish, self._out = work, finish, None

    def wait(self) -> torch.Tensor:
        if self._out is None:
            if self._work is not None:
                self._work.wait()
            self._out = self._finish()
        return self._out


def all_gather_views_async(local: torch.Tensor, batch_size: int, group=None) -> PendingGather:
    """all_gather_views launched asynchronously (RCCL runs it on its own stream once `local` is ready, beside
    whatever the caller enqueues next).  For a loss that decomposes over views (or over groups of views
    rendered on one rank, e.g. MVDream's 4-view guidance groups with group-aligned shards), each view's
    gradient needs only its own rank's image, so the gather of the full batch (the batch renderer's output
    contract) can overlap the backward; the gathered batch carries no gradient.  Same values as
    all_gather_views."""
    world, rank = _world()
    if not _collect():
        out = local.detach()
        return PendingGather(None, lambda: out)
    counts = [shard_range(batch_size, world, r) for r in range(world)]
    n_max = max(b - a for a, b in counts)
    even = all(b - a == n_max for a, b in counts)
    src = local.detach().contiguous()
    if dist.get_backend(group) == "nccl" and even:
        out = local.new_empty((batch_size,) + tuple(local.shape[1:]))
        work = dist.all_gather_into_tensor(out, src, group=group, async_op=True)
        return PendingGather(work, lambda: out)
    pad = local.new_zeros((n_max,) + tuple(local.shape[1:]))
    pad[: local.shape[0]] = src
    if dist.get_backend(group) == "nccl":
        buf = local.new_empty((world * n_max,) + tuple(local.shape[1:]))
        work = dist.all_gather_into_tensor(buf, pad, group=group, async_op=True)
        parts = None

        def finish():
            ps = list(buf.split(n_max))
            return torch.cat([ps[r][: b - a] for r, (a, b) in enumerate(counts)], 0)
        return PendingGather(work, finish)
    parts = [torch.empty_like(pad) for _ in range(world)]
    work = dist.all_gather(parts, pad, group=group, async_op=True)
    return PendingGather(work, lambda: torch.cat([parts[r][: b - a] for r, (a, b) in enumerate(counts)], 0))


def _contiguous_span(grads):
    """The tensors as one 1-D view when they tile a gap-free range of a single storage (in any order,
    same dtype and device, each contiguous, no overlaps), else None."""
    g0 = grads[0]
    base = g0.untyped_storage().data_ptr()
    if any(g.dtype != g0.dtype or g.device != g0.device or not g.is_contiguous()
           or g.untyped_storage().data_ptr() != base for g in grads):
        return None
    order = sorted(grads, key=lambda g: g.storage_offset())
    start = end = order[0].storage_offset()
    for g in order:
        if g.storage_offset() != end:
            return None
        end += g.numel()
    return g0.as_strided((end - start,), (1,), start)


def _span_in_order(grads):
    """The one-buffer span of `grads` when they tile it in exactly the given order, else None."""
    span = _contiguous_span(grads)
    if span is None:
        return None
    offs = [g.storage_offset() for g in grads]
    return span if all(a < b for a, b in zip(offs, offs[1:])) else None


def replicated_loss(term: torch.Tensor, group=None) -> torch.Tensor:
    """A loss term every rank computes identically from the replicated parameters (the systems'
    lambda_position / lambda_opacity / lambda_scales regularisers, system/gaussian_splatting.py:89-106),
    scaled by 1/world: allreduce_grads SUMS the ranks' gradients, so the unscaled term would count `world`
    times.  Image terms on the gathered batch need no scaling (their gradient reaches each view's own rank
    only, view_shard.all_gather_views)."""
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    return term if world == 1 else term / world


def _has_grad_flags(params, group):
    """Per parameter: does any rank hold a gradient for it (one small MAX all-reduce)?"""
    mine = torch.tensor([p.grad is not None for p in params], dtype=torch.int32, device=_coll_device(group))
    dist.all_reduce(mine, op=dist.ReduceOp.MAX, group=group)
    return [bool(x) for x in mine.cpu().tolist()]


def allreduce_grads(params, group=None, average: bool = False):
    """Sum (or average) the .grad of `params` over ranks in one flat bucket (one RCCL all-reduce).

    Every rank reduces the same elements in the same order — the order of `params` — so a rank whose
    gradients are missing (a rank that rendered no view: .grad is None) takes part with zeros.  A parameter
    no rank has a gradient for keeps .grad = None, as in the single-process reference (optimizers skip it).
    When the gradients tile one buffer in that order (the batched rasterizer's carved gradients, batched.py:
    means3D, scales, rotations, opacities, SH, ... — pass the parameters in that order) the buffer is
    reduced in place, without a copy.  Loss terms computed on every rank from the parameters directly go
    through replicated_loss first."""
    world, _ = _world()
    if not _collect() or not params:
        return
    flags = _has_grad_flags(params, group)  # collective on every rank (which ranks lack a grad is rank-local)
    params = [p for p, f in zip(params, flags) if f]
    if not params:
        return
    for p in params:
        if p.grad is None:
            p.grad = torch.zeros_like(p)
    grads = [p.grad for p in params]
    span = _span_in_order(grads)
    if span is not None:  # the batched rasterizer's gradients: one buffer, reduced in place
        dist.all_reduce(span, group=group)
        if average:
            span /= world
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, group=group)
    if average:
        flat /= world
    off = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n


GRAD_CHUNKS_MAX = 16      # include/gsr.h GSR_GRAD_CHUNKS_MAX
GRAD_CHUNK_ALIGN = 4096   # include/gsr.h GSR_GRAD_CHUNK_ALIGN


def grad_chunk_range(P: int, n_chunks: int, chunk: int):
    """Gaussian range [g0, g1) of gradient chunk `chunk` (include/gsr.h gsr_grad_chunk_range)."""
    q = -(-P // n_chunks)
    size = -(-q // GRAD_CHUNK_ALIGN) * GRAD_CHUNK_ALIGN
    return min(chunk * size, P), min((chunk + 1) * size, P)


def _coalesced_all_reduce(tensors, group):
    """One grouped collective for a list of tensors (RCCL group call), or one call each."""
    try:
        from torch.distributed.distributed_c10d import _coalescing_manager
    except ImportError:  # pragma: no cover
        _coalescing_manager = None
    if _coalescing_manager is not None and len(tensors) > 1 and dist.get_backend(group) == "nccl":
        with _coalescing_manager(group=group, device=tensors[0].device):
            for t in tensors:
                dist.all_reduce(t, group=group)
        return
    for t in tensors:
        dist.all_reduce(t, group=group)


class ChunkedGradReduce:
    """Sum over ranks of the rasterizer's per-Gaussian parameter gradients, overlapped with the backward that
    forms them.

    Passed to ``batched.rasterize_views(..., grad_reduce=...)``.  The backward then forms its final
    per-Gaussian sums in `n_chunks` Gaussian ranges (include/gsr.h gsr_set_backward_chunks) with an event after
    each; a communication stream waits on range c's event and all-reduces that range's rows of every
    parameter gradient (one grouped RCCL call per range) while the later ranges are computed; the launch stream
    then waits for the communication stream (GPU-side, no host block) before autograd hands the gradients to
    the leaves.  Bitwise the same sums as allreduce_grads over the finished gradients.  Every rank must render
    at least one view (the ranges' collectives are issued from the backward); the rasterizer's gradients are
    then already reduced — do not pass those parameters to allreduce_grads again.  Parameter-direct loss terms
    are not reduced here and need no replicated_loss scaling."""

    def __init__(self, n_chunks: int = 4, group=None, average: bool = False):
        if not 1 <= n_chunks <= GRAD_CHUNKS_MAX:
            raise ValueError(f"n_chunks must be 1..{GRAD_CHUNKS_MAX}")
        self.n_chunks, self.group, self.average = n_chunks, group, average
        self._comm = None
        self.launched = 0

    def active(self) -> bool:
        return _collect()

    def chunk_events(self, device):
        """Events the backward records after each range (created now: torch creates them on first record)."""
        if device.type != "cuda":
            return None
        evs = [torch.cuda.Event() for _ in range(self.n_chunks)]
        for e in evs:
            e.record()
        return evs

    def _stream(self, device):
        if self._comm is None:
            self._comm = torch.cuda.Stream(device=device)
        return self._comm

    def launch(self, grads, P: int, events=None):
        """Reduce `grads` ((P, ...) tensors, rows = Gaussians) range by range; with `events` each range waits
        for its event on the communication stream."""
        grads = [g for g in grads if g is not None]
        if not grads or not self.active():
            return
        world = _world()[0]
        dev = grads[0].device
        comm = self._stream(dev) if dev.type == "cuda" else None
        for c in range(self.n_chunks):
            g0, g1 = grad_chunk_range(P, self.n_chunks, c)
            if g1 <= g0:
                continue
            parts = [g[g0:g1] for g in grads]
            if comm is None:
                _coalesced_all_reduce(parts, self.group)
            else:
                if events is not None:
                    comm.wait_event(events[c])
                else:
                    comm.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(comm):
                    _coalesced_all_reduce(parts, self.group)
                    if self.average:
                        for t in parts:
                            t.div_(world)
            if comm is None and self.average:
                for t in parts:
                    t.div_(world)
        if comm is not None:
            for g in grads:
                g.record_stream(comm)
            torch.cuda.current_stream(dev).wait_stream(comm)
        self.launched += 1


class _ReduceOnBackward(torch.autograd.Function):
    """Identity on (P, ...) tensors whose backward sums their accumulated gradients over ranks
    (ChunkedGradReduce.launch, without events: the ranges wait for the whole launch stream)."""

    @staticmethod
    def forward(ctx, grad_reduce, P, *tensors):
        ctx.grad_reduce, ctx.P = grad_reduce, P
        ctx.like = [(t.shape, t.dtype, t.device) for t in tensors]
        return tuple(t.view_as(t) for t in tensors)

    @staticmethod
    def backward(ctx, *grads):
        grads = [torch.zeros(s, dtype=d, device=v) if g is None else g.contiguous()
                 for g, (s, d, v) in zip(grads, ctx.like)]
        ctx.grad_reduce.launch(grads, ctx.P, None)
        return (None, None) + tuple(grads)


def reduce_on_backward(grad_reduce, tensors):
    """The tensors (rows = Gaussians, all requiring grad) through an identity whose backward all-reduces the
    gradients every use of them accumulated — one reduction for several rasterizer calls on the same
    parameters (the shading / normal renderers' main and predicted-normal calls,
    renderer/diff_gaussian_rasterizer_shading.py:119-128,177-187), issued after both calls' backward."""
    if not tensors:
        return []
    return list(_ReduceOnBackward.apply(grad_reduce, int(tensors[0].shape[0]), *tensors))


class _JoinReduce(torch.autograd.Function):
    """A rank that renders no view (batch < world) in place of the rasterizer call whose backward issues the
    per-Gaussian gradient reduction: empty image slices in the forward; in the backward zero gradients for
    the same tensors, passed through the same ranged collectives, so the other ranks' reductions complete
    and this replica receives their sum."""

    @staticmethod
    def forward(ctx, grad_reduce, P, shapes, *tensors):
        ctx.grad_reduce, ctx.P = grad_reduce, P
        ctx.like = [(t.shape, t.dtype, t.device) for t in tensors]
        t0 = tensors[0]
        return tuple(t0.new_empty(s) for s in shapes)

    @staticmethod
    def backward(ctx, *_grads):
        grads = [torch.zeros(s, dtype=d, device=v) for s, d, v in ctx.like]
        ctx.grad_reduce.launch(grads, ctx.P, None)
        return (None, None, None) + tuple(grads)


def join_grad_reduce(grad_reduce, tensors, shapes):
    """Empty outputs of the given shapes whose backward joins `grad_reduce`'s collectives with zero gradients
    of `tensors` (the tensors the other ranks' reducing call differentiates, in that call's order)."""
    tensors = [t for t in tensors if t is not None and t.requires_grad]
    if not tensors:
        raise ValueError("join_grad_reduce: no tensor requires grad")
    return list(_JoinReduce.apply(grad_reduce, int(tensors[0].shape[0]), [tuple(s) for s in shapes], *tensors))


def reduce_densify_stats(radii, viewspace_points, visibility_filter, num_points: int, group=None, device=None):
    """Per-Gaussian densification statistics over the whole batch (all ranks).

    Returns (max_radii, grad_norm_sum, count) with the semantics of update_states /
    add_densification_stats (geometry/gaussian_base.py:815-851) applied to every view of the batch:
      max_radii     = max over views of radii
      grad_norm_sum = sum over views of |viewspace_points.grad[:, :2]| where visible
      count         = number of views in which the Gaussian is visible
    A rank without views passes empty lists (and `device`); it still joins the reductions.
    """
    dev = device if device is not None else (radii[0].device if radii else torch.device("cpu"))
    max_r = torch.zeros(num_points, device=dev, dtype=torch.float32)
    gsum = torch.zeros(num_points, device=dev, dtype=torch.float32)
    cnt = torch.zeros(num_points, device=dev, dtype=torch.float32)
    for r, vp, vis in zip(radii, viewspace_points, visibility_filter):
        max_r = torch.maximum(max_r, r.float())
        if vp.grad is not None:
            gsum[vis] += torch.norm(vp.grad[vis, :2], dim=-1)
        cnt[vis] += 1
    world, _ = _world()
    if world > 1:
        dist.all_reduce(max_r, op=dist.ReduceOp.MAX, group=group)
        both = torch.stack([gsum, cnt])
        dist.all_reduce(both, group=group)
        gsum, cnt = both[0], both[1]
    return max_r, gsum, cnt


class ViewShardedBatchRenderer:
    """batch_forward() with the output contract of GaussianBatchRenderer (renderer/gaussian_batch_renderer.py:78-121),
    rendering only this rank's views.

    Built either from a renderer object (a DiffGaussian of the reference): its fused view-set path
    (batch_renderer.render_batch: one rasterize_views call for the rank's views + the fused epilogue)
    when it has one, else its per-view ``forward``; or from a callback ``render_view(batch_idx, batch) ->
    render_pkg`` rendering one view.  Image outputs are gathered to the full batch on every rank; the
    per-view lists (viewspace_points, visibility_filter, radii) hold the local views, with "view_range"
    telling which batch indices they are.  Every rank issues the same gathers, also a rank that gets no
    view (batch smaller than the world): it contributes empty slices of the shapes the other ranks report.
    """

    def __init__(self, render_view_or_renderer, group=None):
        self.group = group
        if hasattr(render_view_or_renderer, "geometry"):
            self.renderer, self.render_view = render_view_or_renderer, None
        else:
            self.renderer, self.render_view = None, render_view_or_renderer

    def batch_forward(self, batch: dict) -> dict:
        if self.renderer is not None:
            from .batch_renderer import batch_mode, render_batch

            mode = batch_mode(self.renderer)
            if mode is not None:
                return render_batch(self.renderer, batch, mode, group=self.group, shard=True)
        return self._per_view(batch)

    def _render_one(self, batch_idx, batch):
        if self.render_view is not None:
            return self.render_view(batch_idx, batch)
        from .batch_renderer import render_view_reference

        # the reference loop's camera (with timestamp / frame index for the temporal and spacetime renderers)
        # and its fp32 forward (autocast off), renderer/gaussian_batch_renderer.py:22-54
        return render_view_reference(self.renderer, batch, batch_idx)

    def _per_view(self, batch: dict) -> dict:
        bs = int(batch["c2w"].shape[0])
        world, rank = _world()
        start, end = shard_range(bs, world, rank)
        pkgs = []
        for batch_idx in range(start, end):
            batch["batch_idx"] = batch_idx
            pkgs.append(self._render_one(batch_idx, batch))
        out = {
            "viewspace_points": [p["viewspace_points"] for p in pkgs],
            "visibility_filter": [p["visibility_filter"] for p in pkgs],
            "radii": [p["radii"] for p in pkgs],
            "view_range": (start, end),
        }
        # agree on the gathered keys and per-view shapes (a rank without views knows neither)
        local = {}
        for key, name in _IMAGE_KEYS:
            if pkgs and key in pkgs[0] and pkgs[0][key] is not None:
                local[name] = torch.stack([p[key] for p in pkgs], 0)
        if pkgs and "comp_rgb_bg" in pkgs[0]:
            local["comp_rgb_bg_raw"] = torch.cat([p["comp_rgb_bg"] for p in pkgs], 0)
        meta = {k: (tuple(v.shape[1:]), str(v.dtype).replace("torch.", "")) for k, v in local.items()} if pkgs else None
        metas = [meta]
        if world > 1:
            metas = [None] * world
            dist.all_gather_object(metas, meta, group=self.group)
        agreed = next((m for m in metas if m is not None), {})
        dev = batch["c2w"].device if not pkgs else next(iter(local.values())).device
        for name in sorted(agreed):
            shape, dtype = agreed[name]
            t = local.get(name)
            if t is None:
                t = torch.empty((0,) + tuple(shape), device=dev, dtype=getattr(torch, dtype), requires_grad=True)
            full = all_gather_views(t, bs, self.group).permute(0, 2, 3, 1)
            out["comp_rgb_bg" if name == "comp_rgb_bg_raw" else name] = full
        return out


# ---- keeping the replicas identical through densification -------------------------------------------

def _coll_device(group=None):
    """Device for small control tensors of the collective backend (RCCL needs device memory)."""
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")


@contextlib.contextmanager
def replica_rng(group=None):
    """Run the body with the torch RNG (CPU and every GPU) seeded identically on all ranks.

    The reference's densification draws random numbers — ``torch.normal`` samples for split Gaussians
    (geometry/gaussian_base.py:733) and a ``torch.randperm`` prune above max_num (:838).  With the usual
    per-rank seeding those draws differ between ranks and the replicas stop being identical, after which
    the gradient all-reduce would sum gradients of different models.  Inside this context the draws are
    the same everywhere (rank 0 picks the seed; the outer RNG state is restored afterwards)."""
    world, rank = _world()
    if world == 1:
        yield
        return
    seed = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64) if rank == 0 else torch.zeros(1, dtype=torch.int64)
    seed = seed.to(_coll_device(group))
    dist.broadcast(seed, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    devices = list(range(torch.cuda.device_count())) if torch.cuda.is_available() else []
    with torch.random.fork_rng(devices=devices):
        torch.manual_seed(int(seed.item()))
        yield


def update_states_sharded(geometry, iteration, outputs: dict, group=None):
    """``geometry.update_states`` (geometry/gaussian_base.py:821-869) for a view-sharded batch.

    The reference loops over the batch's per-view lists, taking the max of the radii and adding
    |viewspace grad[:, :2]| and a visibility count per view (:845-851).  Each rank holds only its own
    views, so the statistics are reduced over the ranks first (reduce_densify_stats: MAX / SUM), applied
    exactly where the reference applies them (not when it returns early for the SuGaR prune or the max_num
    prune, :827-841), and the rest of update_states — prune and densify — runs with no views under
    replica_rng, so every rank takes the same decisions and draws the same samples."""
    P = int(geometry.get_xyz.shape[0])
    max_r, gsum, cnt = reduce_densify_stats(outputs["radii"], outputs["viewspace_points"],
                                            outputs["visibility_filter"], P, group, device=geometry.get_xyz.device)
    cfg = geometry.cfg
    early = (getattr(cfg, "sugar_prune_at", None) is not None and iteration == cfg.sugar_prune_at) or \
        P >= cfg.max_num + 100
    with torch.no_grad():
        if not early:
            geometry.max_radii2D = torch.max(geometry.max_radii2D, max_r)
            geometry.xyz_gradient_accum += gsum[:, None]
            geometry.denom += cnt[:, None]
        with replica_rng(group):
            geometry.update_states(iteration, [], [], [])


def replica_checksum(tensors, group=None) -> bool:
    """True when every rank holds bitwise-identical `tensors` (one small all-gather of checksums)."""
    world, _ = _world()
    if world == 1:
        return True
    dev = _coll_device(group)
    sums = []
    for t in tensors:
        b = t.detach().contiguous().view(-1).view(torch.uint8) if t.numel() else torch.zeros(1, dtype=torch.uint8)
        w = torch.arange(1, b.numel() + 1, device=b.device, dtype=torch.int64) % 65521
        sums += [float(b.numel()), float((b.to(torch.int64) * w).sum().item())]
    mine = torch.tensor(sums, dtype=torch.float64, device=dev)
    allv = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine, group=group)
    return all(torch.equal(a, allv[0]) for a in allv)


def broadcast_replica(tensors, group=None, src: int = 0):
    """Overwrite `tensors` on every rank with rank `src`'s values (e.g. parameters and optimizer moments
    after a checkpoint load); shapes must already agree."""
    world, _ = _world()
    if world == 1:
        return
    for t in tensors:
        dist.broadcast(t.data, src=src, group=group)

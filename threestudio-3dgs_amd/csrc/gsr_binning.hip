// gsr_binning.hip — tile binning (replaces duplicateWithKeys,
// the 64-bit (tile | depth) radix sort and identifyTileRanges of the reference [EXT]).
//
// MI355X design: instead of radix-sorting K 64-bit (tile<<32 | depth) keys (41-45 key bits ->
// 6 passes over K), the visible Gaussians are depth-sorted once (N keys, 32 bits), the instances
// are emitted in depth order, and a stable sort on the tile id alone (12 bits at 1024^2 -> 2 passes
// over K) finishes the job.  Stability makes the result identical to the reference's order:
// per tile, ascending depth, ties by Gaussian index.  The scans between these steps are fused
// into the kernels that produce their inputs (decoupled look-back), so a view costs
// memset + preprocess + compaction + 4 depth passes, then memset + emission + 2 tile passes +
// ranges + blend.
#include "gsr_kernels.h"
#include "gsr_wave.h"

namespace gsr {

__device__ __forceinline__ uint32_t n_of(const uint32_t* n_dev, int n_max) {
  const uint32_t n = *n_dev;
  return n < (uint32_t)n_max ? n : (uint32_t)n_max;
}

// Compact the visible Gaussians (tiles_touched > 0) into (depth bits, index) pairs in index
// order, fused with everything else that needs one look at them:
//   * the block's visible count -> decoupled look-back -> its compacted output offset,
//   * the digit counts of all 4 depth-sort passes (LDS histogram, flushed with global atomics),
//   * K = sum of tiles_touched and the visible count (integer atomics: order-independent).
// Thread t owns the 16 consecutive Gaussians [base + 16 t, base + 16 t + 16) (4 x 16-B loads).
struct CompactLDS {
  uint32_t hist[4][GSR_RADIX];
  uint32_t wave[8];
  uint32_t vid, prefix;
};

__global__ __launch_bounds__(256) void k_compact_visible(int P, GeomState g) {
  __shared__ CompactLDS s;
  GSR_PH_DECL
  const int t = threadIdx.x;
  if (t == 0) s.vid = atomicAdd(g.counters + GSR_CTR_TICKET_COMPACT, 1u);
#pragma unroll
  for (int p = 0; p < 4; ++p) s.hist[p][t] = 0u;
  __syncthreads();
  const int vid = (int)s.vid;
  const int i0 = vid * GSR_COMPACT_TILE + t * GSR_COMPACT_ITEMS;
  uint32_t tt[GSR_COMPACT_ITEMS];
  if (i0 + GSR_COMPACT_ITEMS <= P) {
    const uint4* src = reinterpret_cast<const uint4*>(g.tiles_touched + i0);
#pragma unroll
    for (int q = 0; q < GSR_COMPACT_ITEMS / 4; ++q) {
      const uint4 v = src[q];
      tt[4 * q] = v.x, tt[4 * q + 1] = v.y, tt[4 * q + 2] = v.z, tt[4 * q + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < GSR_COMPACT_ITEMS; ++k) tt[k] = i0 + k < P ? g.tiles_touched[i0 + k] : 0u;
  }
  uint32_t nvis = 0u, ksum = 0u;
#pragma unroll
  for (int k = 0; k < GSR_COMPACT_ITEMS; ++k) {
    nvis += tt[k] > 0u ? 1u : 0u;
    ksum += tt[k];
  }
  uint32_t btot;
  const uint32_t local = block_exclusive_scan<256>(nvis, &btot, s.wave);
  const uint32_t kblock = block_sum_u32<256>(ksum, s.wave);
  GSR_PH_MARK(1)
  if (t < 64) {
    uint32_t* st = g.compact_state + vid;
    uint32_t prefix = 0u;
    if (vid == 0) {
      if (t == 0) lb_publish(st, GSR_LB_INC, btot);
    } else {
      if (t == 0) lb_publish(st, GSR_LB_AGG, btot);
      prefix = lb_prefix_wave(g.compact_state, vid, g.counters + GSR_CTR_ERR);
      if (t == 0) lb_publish(st, GSR_LB_INC, prefix + btot);
    }
    if (t == 0) {
      s.prefix = prefix;
      if (btot) atomicAdd(g.counters + GSR_CTR_VISIBLE, btot);
      if (kblock) atomicAdd(g.counters + GSR_CTR_K, kblock);
    }
  }
  __syncthreads();
  GSR_PH_MARK(2)
  uint32_t o = s.prefix + local;
#pragma unroll
  for (int k = 0; k < GSR_COMPACT_ITEMS; ++k) {
    if (tt[k] > 0u) {
      const int i = i0 + k;
      const uint32_t key = __float_as_uint(g.rec1[i].z);  // view depth > 0.2: float bits are monotone
      g.dkey[0][o] = key;
      g.dval[0][o] = (uint32_t)i;
      ++o;
#pragma unroll
      for (int p = 0; p < 4; ++p) atomicAdd(&s.hist[p][(key >> (8 * p)) & 0xffu], 1u);
    }
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const uint32_t c = s.hist[p][t];
    if (c) atomicAdd(g.dsort.digit_count + p * GSR_RADIX + t, c);
  }
  GSR_PH_STORE(GSR_PH_COMPACT, (uint32_t)vid, btot)
}

void launch_compact_visible(int P, const GeomState& g, hipStream_t stream) {
  if (P <= 0) return;
  hipLaunchKernelGGL(k_compact_visible, dim3(div_up(P, GSR_COMPACT_TILE)), dim3(256), 0, stream, P, g);
}

// Emit one (tile id, Gaussian) instance per tile of each visible Gaussian, in depth order, fused with
//   * the exclusive scan of tiles_touched in depth order (block scan + decoupled look-back),
//   * goff[g] = the Gaussian's first instance,
//   * the digit counts of every tile-sort pass (LDS histogram, flushed with global atomics),
//   * zeroing the per-tile ranges.
// A block owns 1024 consecutive depth-sorted Gaussians (4 per thread); its instances are one
// contiguous range, written cooperatively: instance j of the block is found by binary search
// over the block's offsets in LDS, so consecutive lanes write consecutive addresses.
struct DupLDS {
  uint32_t off[GSR_DUP_TILE + 1];
  uint32_t gi[GSR_DUP_TILE];
  uint2 rect[GSR_DUP_TILE];
  uint32_t hist[GSR_MAX_PASSES][GSR_RADIX];
  uint32_t wave[8];
  uint32_t vid, prefix;
};

__global__ __launch_bounds__(256) void k_duplicate(int P, int grid_x, int n_tiles, int passes, int dbits,
                                                   const uint32_t* __restrict__ order, GeomState g,
                                                   uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                   uint32_t* dup_state, uint32_t* ticket,
                                                   uint32_t* __restrict__ digit_count, uint2* __restrict__ ranges) {
  __shared__ DupLDS s;
  GSR_PH_DECL
  const int t = threadIdx.x;
  if (t == 0) s.vid = atomicAdd(ticket, 1u);
#pragma unroll
  for (int p = 0; p < GSR_MAX_PASSES; ++p) s.hist[p][t] = 0u;
  __syncthreads();
  const int vid = (int)s.vid;
  const uint32_t n = n_of(g.counters + GSR_CTR_VISIBLE, P);
  const uint32_t nblocks = (n + GSR_DUP_TILE - 1) / GSR_DUP_TILE;
  for (uint32_t i = (uint32_t)vid * 256u + t; i < (uint32_t)n_tiles; i += (nblocks > 0 ? nblocks : 1u) * 256u)
    ranges[i] = make_uint2(0u, 0u);
  const uint32_t base = (uint32_t)vid * GSR_DUP_TILE;
  if (base >= n) return;

  uint32_t gi[GSR_DUP_ITEMS], cnt[GSR_DUP_ITEMS];
  uint32_t sum = 0u;
#pragma unroll
  for (int k = 0; k < GSR_DUP_ITEMS; ++k) {
    const uint32_t r = base + t * GSR_DUP_ITEMS + k;
    gi[k] = r < n ? order[r] : 0u;
    cnt[k] = r < n ? g.tiles_touched[gi[k]] : 0u;
    s.gi[t * GSR_DUP_ITEMS + k] = gi[k];
    s.rect[t * GSR_DUP_ITEMS + k] = r < n ? g.rect[gi[k]] : make_uint2(0u, 0u);
    sum += cnt[k];
  }
  uint32_t btot;
  const uint32_t local = block_exclusive_scan<256>(sum, &btot, s.wave);
  GSR_PH_MARK(1)
  if (t < 64) {
    uint32_t* st = dup_state + vid;
    uint32_t prefix = 0u;
    if (vid == 0) {
      if (t == 0) lb_publish(st, GSR_LB_INC, btot);
    } else {
      if (t == 0) lb_publish(st, GSR_LB_AGG, btot);
      prefix = lb_prefix_wave(dup_state, vid, g.counters + GSR_CTR_ERR);
      if (t == 0) lb_publish(st, GSR_LB_INC, prefix + btot);
    }
    if (t == 0) s.prefix = prefix;
  }
  {
    uint32_t o = local;
#pragma unroll
    for (int k = 0; k < GSR_DUP_ITEMS; ++k) {
      s.off[t * GSR_DUP_ITEMS + k] = o;
      o += cnt[k];
    }
    if (t == 255) s.off[GSR_DUP_TILE] = btot;
  }
  __syncthreads();
  GSR_PH_MARK(2)
  const uint32_t prefix = s.prefix;
#pragma unroll
  for (int k = 0; k < GSR_DUP_ITEMS; ++k)
    if (base + t * GSR_DUP_ITEMS + k < n) g.goff[gi[k]] = prefix + s.off[t * GSR_DUP_ITEMS + k];
  const uint32_t dmask = (1u << dbits) - 1u;
  for (uint32_t j = t; j < btot; j += 256u) {
    // owner m: last m with off[m] <= j (empty owners share their successor's offset)
    int lo = 0, hi = GSR_DUP_TILE;  // off[lo] <= j < off[hi]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (s.off[mid] <= j) lo = mid;
      else hi = mid;
    }
    const uint2 rc = s.rect[lo];
    const uint32_t xmin = rc.x & 0xffffu, ymin = rc.x >> 16, xmax = rc.y & 0xffffu;
    const uint32_t w = xmax - xmin, l = j - s.off[lo];
    const uint32_t ty = l / w, tx = l - ty * w;
    const uint32_t tile = (ymin + ty) * (uint32_t)grid_x + xmin + tx;
    keys[prefix + j] = tile;
    vals[prefix + j] = s.gi[lo];
    for (int p = 0; p < passes; ++p) atomicAdd(&s.hist[p][(tile >> (p * dbits)) & dmask], 1u);
  }
  __syncthreads();
  for (int p = 0; p < passes; ++p) {
    const uint32_t c = s.hist[p][t];
    if (c) atomicAdd(digit_count + p * GSR_RADIX + t, c);
  }
  GSR_PH_STORE(GSR_PH_DUP, (uint32_t)vid, btot)
}

void launch_duplicate(int P, int W, int H, const uint32_t* order, const GeomState& g, const BinningState& b,
                      uint2* ranges, hipStream_t stream) {
  const int gx = div_up(W, GSR_TILE_X), gy = div_up(H, GSR_TILE_Y);
  if (P <= 0) return;
  const DigitPlan plan = digit_plan(tile_key_bits(W, H));
  hipLaunchKernelGGL(k_duplicate, dim3(div_up(P, GSR_DUP_TILE)), dim3(256), 0, stream, P, gx, gx * gy,
                     plan.passes, plan.bits, order, g, b.key[0], b.val[0], b.dup_state,
                     b.tsort.tickets + 32, b.tsort.digit_count, ranges);
}

// After the tile sort: per-tile [start, end) ranges of the sorted instance list.
__global__ __launch_bounds__(256) void k_tile_ranges(int K, const uint32_t* __restrict__ keys,
                                                     uint2* __restrict__ ranges) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= K) return;
  const uint32_t tile = keys[p];
  if (p == 0 || keys[p - 1] != tile) ranges[tile].x = (uint32_t)p;
  if (p == K - 1 || keys[p + 1] != tile) ranges[tile].y = (uint32_t)(p + 1);
}

void launch_tile_ranges(int K, const uint32_t* keys, uint2* ranges, hipStream_t stream) {
  if (K <= 0) return;
  hipLaunchKernelGGL(k_tile_ranges, dim3((K + 255) / 256), dim3(256), 0, stream, K, keys, ranges);
}

// markVisible / checkFrustum of the reference (API completeness).
__global__ __launch_bounds__(256) void k_mark_visible(int P, const float* __restrict__ means3D,
                                                      const float* __restrict__ view,
                                                      const float* __restrict__ proj,
                                                      uint8_t* __restrict__ present) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  const float3 p = make_float3(means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]);
  const float z = view[2] * p.x + view[6] * p.y + view[10] * p.z + view[14];
  present[i] = z > GSR_NEAR_CULL ? 1 : 0;
  (void)proj;
}

void launch_mark_visible(int P, const float* means3D, const float* view, const float* proj,
                         uint8_t* present, hipStream_t stream) {
  if (P <= 0) return;
  hipLaunchKernelGGL(k_mark_visible, dim3((P + 255) / 256), dim3(256), 0, stream, P, means3D, view,
                     proj, present);
}

}  // namespace gsr

#ifdef GSR_TIMELINE
GSR_PH_READER(gsr_diag_phases_bin)
#endif

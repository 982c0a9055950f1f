// gsr_binning.hip — tile binning of a view set (replaces the
// InclusiveSum over tiles_touched, duplicateWithKeys, the 64-bit (tile | depth) radix sort and
// identifyTileRanges of the reference [EXT]).
//
// MI355X design: instead of radix-sorting K 64-bit (tile<<32 | depth) keys (41-45 key bits ->
// 6 passes over K per view), each view's Gaussians are depth-sorted once (P keys, 32 bits;
// gsr_sort.hip), the instances are emitted in depth order, and a stable sort on the tile id alone
// (12 bits at 1024^2 -> 2 passes over K) finishes the job.  Stability makes the result identical
// to the reference's order: per tile, ascending depth, ties by Gaussian index.  Every step runs
// once for all views of a set (segments of flat arrays), so a 64-view batch costs the same
// number of launches as one view.
#include "gsr_kernels.h"
#include "gsr_wave.h"

namespace gsr {

// Kept tiles of each 64-Gaussian group of every view's depth order (GSR_INST_GROUPS consecutive groups per
// wave, 4 waves per block: a block per 4 groups made the launch a quarter-million 1-KB blocks):
// kept_counts[v][group].  The counts ride in the depth-sorted values (streamed); a count that did not fit its
// field is read from tiles.y.
#ifndef GSR_INST_GROUPS
#define GSR_INST_GROUPS 8
#endif
__global__ __launch_bounds__(256) void k_inst_count(int P, int nbe, GeomState g) {
  const uint32_t* __restrict__ order = g.sorted_dval();
  constexpr int GPB = 4 * GSR_INST_GROUPS;  // groups per block
  const int nbb = (nbe + GPB - 1) / GPB;
  const int v = blockIdx.x / nbb;
  const int lb0 = (blockIdx.x - v * nbb) * GPB + (threadIdx.x >> 6) * GSR_INST_GROUPS;
  const int lane = threadIdx.x & 63;
  const size_t vo = (size_t)v * P;
  const uint32_t ks = g.vsent();
  uint32_t val[GSR_INST_GROUPS];
#pragma unroll
  for (int k = 0; k < GSR_INST_GROUPS; ++k) {  // (all loads first)
    const int r = (lb0 + k) * GSR_DUP_TILE + lane;
    val[k] = lb0 + k < nbe && r < P ? order[vo + r] : 0u;
  }
  uint32_t mine = 0u;  // lane k keeps group lb0 + k's total
#pragma unroll
  for (int k = 0; k < GSR_INST_GROUPS; ++k) {
    uint32_t kept = 0u;
    if (lb0 + k < nbe && (lb0 + k) * GSR_DUP_TILE + lane < P) {
      kept = g.vbits <= 26 ? val[k] >> g.vbits : ks;
      if (kept == ks) kept = g.tiles[vo + (val[k] & g.vmask())].y;
    }
    const uint32_t ktot = __builtin_amdgcn_readlane((int)wave_incl_sum_dpp(kept), 63);
    if (lane == k) mine = ktot;
  }
  if (lane < GSR_INST_GROUPS && lb0 + lane < nbe) g.kept_counts[(size_t)v * nbe + lb0 + lane] = mine;
}

// One 1024-thread workgroup per view: exclusive scan of its kept counts in place, GSR_ISCAN_PER x 1024 entries
// per round, staged through LDS so that the loads and stores are coalesced and each thread scans
// GSR_ISCAN_PER consecutive entries (one pad word per 8: conflict-free runs); kept instances -> counters[2V + v].
// (One view's 15.6K entries in two rounds: this scan is a single workgroup's latency on the one-view path.)
#define GSR_ISCAN_PER 8
__global__ __launch_bounds__(1024) void k_inst_scan(int nbe, GeomState g) {
  constexpr int CH = 1024 * GSR_ISCAN_PER;
  __shared__ uint32_t s_x[CH + CH / 8];
  __shared__ uint32_t s_w[16];
  const int v = blockIdx.x, t = threadIdx.x, w = t >> 6, lane = t & 63;
  uint32_t* kept = g.kept_counts + (size_t)v * nbe;
  auto pad = [](int i) { return i + (i >> 3); };
  uint32_t carry = 0u;
  for (int c0 = 0; c0 < nbe; c0 += CH) {
#pragma unroll
    for (int k = 0; k < GSR_ISCAN_PER; ++k) {
      const int i = k * 1024 + t;
      s_x[pad(i)] = c0 + i < nbe ? kept[c0 + i] : 0u;
    }
    __syncthreads();
    uint32_t x[GSR_ISCAN_PER], run = 0u;
#pragma unroll
    for (int k = 0; k < GSR_ISCAN_PER; ++k) {
      x[k] = run;
      run += s_x[pad(t * GSR_ISCAN_PER + k)];
    }
    uint32_t inc = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)inc, o, 64);
      if (lane >= o) inc += y;
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    uint32_t before = 0u, tot = 0u;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t sw = s_w[i];
      before += i < w ? sw : 0u;
      tot += sw;
    }
    const uint32_t off = carry + before + (inc - run);
#pragma unroll
    for (int k = 0; k < GSR_ISCAN_PER; ++k) s_x[pad(t * GSR_ISCAN_PER + k)] = off + x[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < GSR_ISCAN_PER; ++k) {
      const int i = k * 1024 + t;
      if (c0 + i < nbe) kept[c0 + i] = s_x[pad(i)];
    }
    carry += tot;
    __syncthreads();  // s_x and s_w are rewritten by the next round
  }
  if (t == 0) g.counters[2 * gridDim.x + v] = carry;
}

// Gradient-row slots: goff[v][i] = sum of tiles[v][j].x over j < i (each visible Gaussian owns
// tiles.x consecutive rows, one per rectangle tile), in three coalesced passes: block sums, one
// scan per view, block scans + offsets.
__global__ __launch_bounds__(256) void k_goff_count(int P, int nbg, GeomState g) {
  __shared__ uint32_t s_wave[8];
  const int v = blockIdx.x / nbg, b = blockIdx.x - v * nbg, t = threadIdx.x;
  const uint2* tl = g.tiles + (size_t)v * P;
  uint32_t sum = 0u, vis = 0u;
#pragma unroll
  for (int k = 0; k < GSR_GOFF_TILE / 256; ++k) {
    const int i = b * GSR_GOFF_TILE + k * 256 + t;
    const uint32_t x = i < P ? tl[i].x : 0u;
    sum += x;
    vis += x > 0u ? 1u : 0u;
  }
  sum = block_sum_u32<256>(sum, s_wave);
  vis = block_sum_u32<256>(vis, s_wave);
  if (t == 0) g.goff_part[(size_t)v * nbg + b] = sum, g.vis_part[(size_t)v * nbg + b] = vis;
}

__global__ __launch_bounds__(1024) void k_goff_scan(int nbg, GeomState g) {
  __shared__ uint32_t s_w[16];
  const int v = blockIdx.x, t = threadIdx.x, w = t >> 6, lane = t & 63;
  uint32_t* row = g.goff_part + (size_t)v * nbg;
  uint32_t carry = 0u, vis = 0u;
  for (int i = t; i < nbg; i += 1024) vis += g.vis_part[(size_t)v * nbg + i];
  for (int c0 = 0; c0 < nbg; c0 += 1024 * 4) {
    const int i0 = c0 + 4 * t;
    uint32_t x[4], run = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      x[k] = run;
      run += i0 + k < nbg ? row[i0 + k] : 0u;
    }
    uint32_t inc = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)inc, o, 64);
      if (lane >= o) inc += y;
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    uint32_t before = 0u, tot = 0u;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t sw = s_w[i];
      before += i < w ? sw : 0u;
      tot += sw;
    }
    __syncthreads();
    const uint32_t off = carry + before + (inc - run);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i0 + k < nbg) row[i0 + k] = off + x[k];
    carry += tot;
  }
  // rectangle tiles K_v (the reference's num_rendered) -> counters[v], visible Gaussians -> counters[V + v]
  __syncthreads();
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) vis += (uint32_t)__shfl_xor((int)vis, o, 64);
  if (lane == 0) s_w[w] = vis;
  __syncthreads();
  if (t == 0) {
    uint32_t vt = 0u;
    for (int i = 0; i < 16; ++i) vt += s_w[i];
    g.counters[v] = carry;
    g.counters[gridDim.x + v] = vt;
  }
}

// (coalesced loads and stores; each thread scans 16 consecutive entries through LDS, one pad word
// per 16 so the per-thread runs are bank-conflict free)
__global__ __launch_bounds__(256) void k_goff_write(int P, int nbg, GeomState g) {
  __shared__ uint32_t s_x[GSR_GOFF_TILE + GSR_GOFF_TILE / 16];
  __shared__ uint32_t s_wave[8];
  const int v = blockIdx.x / nbg, b = blockIdx.x - v * nbg, t = threadIdx.x;
  const uint2* tl = g.tiles + (size_t)v * P + (size_t)b * GSR_GOFF_TILE;
  uint32_t* go = g.goff + (size_t)v * P + (size_t)b * GSR_GOFF_TILE;
  const int n = min(GSR_GOFF_TILE, P - b * GSR_GOFF_TILE);
  constexpr int PER = GSR_GOFF_TILE / 256;
  auto pad = [](int i) { return i + (i >> 4); };
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int i = k * 256 + t;
    s_x[pad(i)] = i < n ? tl[i].x : 0u;
  }
  __syncthreads();
  uint32_t x[PER], run = 0u;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t c = s_x[pad(t * PER + k)];
    x[k] = run;
    run += c;
  }
  uint32_t tot;
  const uint32_t off = g.goff_part[(size_t)v * nbg + b] + block_exclusive_scan<256>(run, &tot, s_wave);
#pragma unroll
  for (int k = 0; k < PER; ++k) s_x[pad(t * PER + k)] = off + x[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int i = k * 256 + t;
    if (i < n) go[i] = s_x[pad(i)];
  }
}

// Emit one (tile id, Gaussian) instance per kept tile (span_row) of each visible Gaussian, in
// depth order (gradient-row slots come from k_goff_*, in Gaussian order: a scattered 4-byte goff
// store per Gaussian here cost ~20 us/view, DRAM-transaction bound).  One wave per 64 consecutive depth-sorted
// Gaussians, no workgroup barriers.  Two levels of owner maps (each Gaussian / row marks its first
// position in the wave's LDS, a DPP max-scan spreads the marks):
//   rows:  the group's rectangle rows, 64 at a time; one span_row per (Gaussian, row) gives the row's
//          kept tiles [t0, t1) and, by a DPP prefix sum, their place in the group's output range;
//   kept:  the kept positions of those rows, 64 at a time; lane j's row owner gives its tile directly
//          (row tile t0 + offset), so every instance is written with a coalesced store, in order,
//          without per-position span tests, divisions or ballots.
template <bool QM>
struct EmitLDS {
  uint32_t gi[GSR_DUP_TILE];
  uint32_t roff[GSR_DUP_TILE];  // per Gaussian: its first row in the group's row list
  uint2 rect[GSR_DUP_TILE];
  SpanPrep sp[GSR_DUP_TILE];
  uint32_t own[64];             // row -> 1 + owning Gaussian (marks)
  uint32_t rk[64];              // per row of the chunk: its first kept position (chunk-relative)
  uint32_t rtile[64];           // per row of the chunk: tile id of its first kept tile
  uint32_t rgi[64];             // per row of the chunk: the Gaussian
  uint32_t rx0[QM ? 64 : 1];    // per row of the chunk (QM): its first kept tile column
  uint2 rq[QM ? 64 : 1];        // per row of the chunk (QM): span_quads of its upper and lower 8-pixel band
  // (without QM the struct is 4.6 KB: 8 single-wave workgroups per SIMD instead of 7)
  uint32_t kown[64];            // kept position -> 1 + owning row (marks)
};

#ifndef GSR_EMIT_GROUPS
#define GSR_EMIT_GROUPS 2  // consecutive 64-Gaussian groups per wave (the next group's gathers prefetched)
#endif

// QM (unpacked keys): each key also carries the instance's quadrant mask (GSR_QMASK_SHIFT): per row the
// quadrant-column ranges of its two 8-pixel bands (span_quads, the span_row bound at half the tile size), per
// instance four integer compares.
template <bool QM>
__global__ __launch_bounds__(64) void k_emit(int P, int nbe, int grid_x, GeomState g, SegInfo inst, int gbits,
                                             uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const uint32_t* __restrict__ order = g.sorted_dval();
  const uint32_t* __restrict__ dkeys = g.sorted_dkey();
  __shared__ EmitLDS<QM> s;
  const int nw = div_up(nbe, GSR_EMIT_GROUPS);
  const int v = blockIdx.x / nw;
  const int lb0 = (blockIdx.x % nw) * GSR_EMIT_GROUPS, lb1 = min(nbe, lb0 + GSR_EMIT_GROUPS);
  const int lane = threadIdx.x;
  const size_t vo = (size_t)v * P;
  uint32_t* kout = keys + inst.start[v];
  uint32_t* vout = vals ? vals + inst.start[v] : nullptr;
  // group prefetch: order, visibility and the record pieces of group lb + 1 load while lb emits
  uint32_t n_gi = 0u, n_koff = 0u;
  bool n_vis = false;
  float4 n_ra = make_float4(0.f, 0.f, 0.f, 0.f), n_rb = n_ra;
  uint2 n_d = make_uint2(0u, 0u);
  auto fetch = [&](int lb) {
    const int r = lb * GSR_DUP_TILE + lane;
    n_gi = r < P ? (order[vo + r] & g.vmask()) : 0u;
    n_vis = r < P && dkeys[vo + r] != 0xFFFFFFFFu;
    n_koff = g.kept_counts[(size_t)v * nbe + lb];
    if (n_vis) {
      const GaussRec& rc = g.rec[vo + n_gi];
      const uint4 d = rc.d;
      n_d = make_uint2(d.x, d.y);
      n_ra = rc.a;
      n_rb = rc.b;
    }
  };
  if (lb0 < lb1) fetch(lb0);
  for (int lb = lb0; lb < lb1; ++lb) {
    const uint32_t gi = n_gi;
    const bool vis = n_vis;
    const float4 ra = n_ra, rb = n_rb;
    const uint2 d = n_d;
    uint32_t kbase = n_koff;
    if (lb + 1 < lb1) fetch(lb + 1);
    uint32_t cnt = 0u, h = 0u;
    if (vis) {
      const uint32_t wd = (d.y & 0xffffu) - (d.x & 0xffffu);
      h = (d.y >> 16) - (d.x >> 16);
      cnt = wd * h;  // rectangle tiles
      if (cnt == 0u) h = 0u;
    }
    const uint32_t rincl = wave_incl_sum_dpp(h);
    const uint32_t roff = rincl - h;
    const uint32_t R = (uint32_t)__builtin_amdgcn_readlane((int)rincl, 63);
    s.gi[lane] = gi;
    s.roff[lane] = roff;
    s.rect[lane] = d;
    if (h) s.sp[lane] = span_prep(ra.x, ra.y, ra.z, ra.w, rb.x, rb.y);
    uint32_t carry = 0u;  // 1 + owner of the previous chunk's last row
    for (uint32_t r0 = 0; r0 < R; r0 += 64) {
      s.own[lane] = 0u;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (h && roff >= r0 && roff < r0 + 64) s.own[roff - r0] = (uint32_t)lane + 1u;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const uint32_t ow1 = max(carry, wave_incl_max_dpp(s.own[lane]));
      carry = (uint32_t)__builtin_amdgcn_readlane((int)ow1, 63);
      const uint32_t r = r0 + (uint32_t)lane;
      uint32_t kc = 0u, tile0 = 0u, rg = 0u;
      if (r < R) {
        const uint32_t ow = ow1 - 1u;
        const uint2 rc = s.rect[ow];
        const int xmin = (int)(rc.x & 0xffffu), xmax = (int)(rc.y & 0xffffu);
        const int row = (int)(rc.x >> 16) + (int)(r - s.roff[ow]);
        int t0, t1;
        span_row(s.sp[ow], row, xmin, xmax, t0, t1);
        kc = (uint32_t)(t1 - t0);
        tile0 = (uint32_t)row * (uint32_t)grid_x + (uint32_t)t0;
        rg = s.gi[ow];
        if (QM) {
          const float v1 = s.sp[ow].py - (float)(row * GSR_TILE_Y);
          s.rx0[lane] = (uint32_t)t0;
          s.rq[lane] = make_uint2(span_quads(s.sp[ow], v1), span_quads(s.sp[ow], v1 - 8.0f));
        }
      }
      const uint32_t kincl = wave_incl_sum_dpp(kc);
      const uint32_t kstart = kincl - kc;
      const uint32_t KC = (uint32_t)__builtin_amdgcn_readlane((int)kincl, 63);
      s.rk[lane] = kstart;
      s.rtile[lane] = tile0;
      s.rgi[lane] = rg;
      uint32_t kcarry = 0u;  // 1 + owning row of the previous chunk's last kept position
      for (uint32_t k0 = 0; k0 < KC; k0 += 64) {
        s.kown[lane] = 0u;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (kc && kstart >= k0 && kstart < k0 + 64) s.kown[kstart - k0] = (uint32_t)lane + 1u;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const uint32_t kw1 = max(kcarry, wave_incl_max_dpp(s.kown[lane]));
        kcarry = (uint32_t)__builtin_amdgcn_readlane((int)kw1, 63);
        const uint32_t j = k0 + (uint32_t)lane;
        if (j < KC) {
          const uint32_t rr = kw1 - 1u;
          const uint32_t tile = s.rtile[rr] + (j - s.rk[rr]);
          const uint32_t gv = s.rgi[rr];
          uint32_t qm = 0u;
          if (QM) {
            const uint2 rq = s.rq[rr];
            qm = quads_of_tile(rq.x, rq.y, (int)(s.rx0[rr] + (j - s.rk[rr])));
          }
          kout[kbase + j] = vout ? (QM ? tile | qm << GSR_QMASK_SHIFT : tile) : ((tile << gbits) | gv);
          if (vout) vout[kbase + j] = gv;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // kown[] is rewritten by the next chunk
      }
      kbase += KC;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the row table is rewritten by the next chunk
    }
  }
}

// After the tile sort: per-tile [start, end) ranges (view-local positions) of each view's list, by search
// (identifyTileRanges of the reference streams every sorted key instead): one thread per (view, tile boundary t in
// [0, n_tiles]) finds the first listed instance whose tile is >= t (lower bound over the view's sorted list, a
// fixed number of halving steps: the trip count is uniform) and writes it as tile t's start and tile t - 1's
// end.  ~V x tiles x log2(K) dependent loads whose upper levels every thread shares (cache hits), instead of
// streaming every listed key (C3: 4.95M keys = 20 MB per view; that scan, measured 472 vs 30 us per 64-view
// launch, profiles/r04/tile_ranges_ab.txt, was removed in round 5).
__global__ __launch_bounds__(256) void k_tile_bounds(SegInfo inst, int n_tiles, int gbits, uint32_t tmask,
                                                     const uint32_t* __restrict__ keys, uint2* __restrict__ ranges) {
  const int v = blockIdx.y;
  const int t = blockIdx.x * 256 + threadIdx.x;  // boundary t: start of tile t, end of tile t - 1
  if (t > n_tiles) return;
  const uint32_t K = seg_live(inst, v);
  const uint32_t* kv = keys + inst.start[v];
  uint32_t lo = 0u;  // invariant: every i < lo has tile < t
  uint32_t step = K == 0u ? 0u : 1u << (31 - __builtin_clz(K));
  for (; step > 0u; step >>= 1) {
    const uint32_t m = lo + step;  // probe i = m - 1
    if (m <= K && ((kv[m - 1] >> gbits) & tmask) < (uint32_t)t) lo = m;
  }
  uint2* rv = ranges + (size_t)v * n_tiles;
  if (t < n_tiles) rv[t].x = lo;
  if (t > 0) rv[t - 1].y = lo;
}

void launch_binning_counts(int V, int P, const GeomState& g, hipStream_t stream) {
  if (V <= 0) return;
  const int nbe = GeomState::dup_blocks(P);
  const int nbg = GeomState::goff_blocks(P);
  if (P > 0) hipLaunchKernelGGL(k_goff_count, dim3(V * nbg), dim3(256), 0, stream, P, nbg, g);
  hipLaunchKernelGGL(k_goff_scan, dim3(V), dim3(1024), 0, stream, P > 0 ? nbg : 0, g);  // K_v, visible
  if (P > 0) hipLaunchKernelGGL(k_goff_write, dim3(V * nbg), dim3(256), 0, stream, P, nbg, g);
  if (P > 0)
    hipLaunchKernelGGL(k_inst_count, dim3(V * ((nbe + 4 * GSR_INST_GROUPS - 1) / (4 * GSR_INST_GROUPS))), dim3(256),
                       0, stream, P, nbe, g);
  hipLaunchKernelGGL(k_inst_scan, dim3(V), dim3(1024), 0, stream, P > 0 ? nbe : 0, g);
}

void launch_emit(int V, int P, int W, const GeomState& g, const SegInfo& inst, const TilePack& tp, uint32_t* keys,
                 uint32_t* vals, hipStream_t stream) {
  if (V <= 0 || P <= 0) return;
  const int nbe = GeomState::dup_blocks(P);
  const dim3 grid(V * div_up(nbe, GSR_EMIT_GROUPS));
  if (tp.qmask)
    hipLaunchKernelGGL(k_emit<true>, grid, dim3(64), 0, stream, P, nbe, div_up(W, GSR_TILE_X), g, inst, tp.gbits,
                       keys, vals);
  else
    hipLaunchKernelGGL(k_emit<false>, grid, dim3(64), 0, stream, P, nbe, div_up(W, GSR_TILE_X), g, inst, tp.gbits,
                       keys, vals);
}

void launch_tile_ranges(SegInfo inst, int n_tiles, const TilePack& tp, const uint32_t* keys, uint2* ranges,
                        hipStream_t stream) {
  if (inst.V <= 0 || n_tiles <= 0) return;
  hipLaunchKernelGGL(k_tile_bounds, dim3(div_up(n_tiles + 1, 256), inst.V), dim3(256), 0, stream, inst, n_tiles,
                     tp.gbits, tp.tmask, keys, ranges);
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

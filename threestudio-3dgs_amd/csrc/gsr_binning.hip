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

// Rectangle tiles, visible Gaussians and kept tiles of each 64-Gaussian group of every view's depth
// order (one wave per group, 4 groups per block): counts[v][group].
__global__ __launch_bounds__(256) void k_inst_count(int P, int nbe, GeomState g) {
  const uint32_t* __restrict__ order = g.sorted_dval();
  const int nb4 = (nbe + 3) / 4;
  const int v = blockIdx.x / nb4;
  const int lb = (blockIdx.x - v * nb4) * 4 + (threadIdx.x >> 6);
  if (lb >= nbe) return;
  const int lane = threadIdx.x & 63;
  const size_t vo = (size_t)v * P;
  const int r = lb * GSR_DUP_TILE + lane;
  const uint2 tt = r < P ? g.tiles[vo + order[vo + r]] : make_uint2(0u, 0u);
  const uint32_t tot = __builtin_amdgcn_readlane((int)wave_incl_sum_dpp(tt.x), 63);
  const uint32_t vtot = __builtin_amdgcn_readlane((int)wave_incl_sum_dpp(tt.x > 0u ? 1u : 0u), 63);
  const uint32_t ktot = __builtin_amdgcn_readlane((int)wave_incl_sum_dpp(tt.y), 63);
  if (lane == 0) {
    g.inst_counts[(size_t)v * nbe + lb] = tot;
    g.vis_counts[(size_t)v * nbe + lb] = vtot;
    g.kept_counts[(size_t)v * nbe + lb] = ktot;
  }
}

// One 1024-thread workgroup per view: exclusive scans of its block counts in place, in one pass per
// 16K blocks (16 consecutive entries per thread; rectangle and kept counts packed as rect << 32 | kept
// into one 64-bit scan: a view's kept total is < 2^32).  Rectangle tiles K_v -> counters[v], visible
// Gaussians -> counters[V + v], kept instances -> counters[2V + v].
#define GSR_ISCAN_PER 16
__global__ __launch_bounds__(1024) void k_inst_scan(int nbe, GeomState g) {
  __shared__ unsigned long long s_w[16];
  __shared__ uint32_t s_v[16];
  const int v = blockIdx.x, t = threadIdx.x, w = t >> 6, lane = t & 63;
  uint32_t* rect = g.inst_counts + (size_t)v * nbe;
  uint32_t* kept = g.kept_counts + (size_t)v * nbe;
  const uint32_t* vis = g.vis_counts + (size_t)v * nbe;
  unsigned long long carry = 0ull;
  uint32_t vis_total = 0u;
  for (int c0 = 0; c0 < nbe; c0 += 1024 * GSR_ISCAN_PER) {
    const int i0 = c0 + t * GSR_ISCAN_PER;
    unsigned long long x[GSR_ISCAN_PER], run = 0ull;
    uint32_t vs = 0u;
#pragma unroll
    for (int k = 0; k < GSR_ISCAN_PER; ++k) {
      const int i = i0 + k;
      const bool in = i < nbe;
      x[k] = run;
      run += in ? ((unsigned long long)rect[i] << 32 | kept[i]) : 0ull;
      vs += in ? vis[i] : 0u;
    }
    unsigned long long inc = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned long long y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) vs += (uint32_t)__shfl_xor((int)vs, o, 64);
    if (lane == 63) s_w[w] = inc;
    if (lane == 0) s_v[w] = vs;
    __syncthreads();
    unsigned long long before = 0ull, tot = 0ull;
    uint32_t vt = 0u;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const unsigned long long sw = s_w[i];
      before += i < w ? sw : 0ull;
      tot += sw;
      vt += s_v[i];
    }
    __syncthreads();
    const unsigned long long off = carry + before + (inc - run);
#pragma unroll
    for (int k = 0; k < GSR_ISCAN_PER; ++k) {
      const int i = i0 + k;
      if (i < nbe) {
        const unsigned long long r = off + x[k];
        rect[i] = (uint32_t)(r >> 32);
        kept[i] = (uint32_t)r;
      }
    }
    carry += tot;
    vis_total += vt;
  }
  if (t == 0) {
    g.counters[v] = (uint32_t)(carry >> 32);
    g.counters[gridDim.x + v] = vis_total;
    g.counters[2 * gridDim.x + v] = (uint32_t)carry;
  }
}

// Emit one (tile id, Gaussian) instance per kept tile (span_row) of each visible Gaussian, in
// depth order, and goff[g] = the Gaussian's first rectangle slot (gradient rows are indexed by
// rectangle position, the lists hold the kept tiles only).  One wave per 64 consecutive depth-sorted
// Gaussians, no workgroup barriers: the group's rectangle positions are walked 64 at a time, the
// owner of every position comes from an owner map in the wave's LDS (each Gaussian marks its first
// position, a DPP max-scan spreads the marks), and the kept positions are compacted in order with
// ballots into the group's contiguous output range (offset from k_inst_scan).
struct EmitLDS {
  uint32_t off[GSR_DUP_TILE];
  uint32_t gi[GSR_DUP_TILE];
  uint2 rect[GSR_DUP_TILE];
  SpanPrep sp[GSR_DUP_TILE];
  uint32_t own[64];
};

#define GSR_EMIT_GROUPS 2  // consecutive 64-Gaussian groups per wave (the next group's gathers prefetched)

__global__ __launch_bounds__(64) void k_emit(int P, int nbe, int grid_x, GeomState g, SegInfo inst, int gbits,
                                             uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const uint32_t* __restrict__ order = g.sorted_dval();
  const uint32_t* __restrict__ dkeys = g.sorted_dkey();
  __shared__ EmitLDS s;
  const int nw = div_up(nbe, GSR_EMIT_GROUPS);
  const int v = blockIdx.x / nw;
  const int lb0 = (blockIdx.x % nw) * GSR_EMIT_GROUPS, lb1 = min(nbe, lb0 + GSR_EMIT_GROUPS);
  const int lane = threadIdx.x;
  const size_t vo = (size_t)v * P;
  uint32_t* kout = keys + inst.start[v];
  uint32_t* vout = vals ? vals + inst.start[v] : nullptr;
  // group prefetch: order, visibility and the record pieces of group lb + 1 load while lb emits
  uint32_t n_gi = 0u, n_ioff = 0u, n_koff = 0u;
  bool n_vis = false;
  float4 n_ra = make_float4(0.f, 0.f, 0.f, 0.f), n_rb = n_ra;
  uint2 n_d = make_uint2(0u, 0u);
  auto fetch = [&](int lb) {
    const int r = lb * GSR_DUP_TILE + lane;
    n_gi = r < P ? order[vo + r] : 0u;
    n_vis = r < P && dkeys[vo + r] != 0xFFFFFFFFu;
    n_ioff = g.inst_counts[(size_t)v * nbe + lb];
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
    const uint32_t gi = n_gi, ioff = n_ioff;
    const bool vis = n_vis;
    const float4 ra = n_ra, rb = n_rb;
    const uint2 d = n_d;
    uint32_t kbase = n_koff;
    if (lb + 1 < lb1) fetch(lb + 1);
    uint32_t cnt = 0u;
    s.gi[lane] = gi;
    s.rect[lane] = make_uint2(0u, 0u);
    if (vis) {
      cnt = ((d.y & 0xffffu) - (d.x & 0xffffu)) * ((d.y >> 16) - (d.x >> 16));  // rectangle tiles
      s.rect[lane] = d;
      s.sp[lane] = span_prep(ra.x, ra.y, ra.z, ra.w, rb.x, rb.y);
    }
    const uint32_t incl = wave_incl_sum_dpp(cnt);
    const uint32_t myoff = incl - cnt;
    const uint32_t btot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    s.off[lane] = myoff;
    // gradient-row slots: rectangle offsets (all of a visible Gaussian's rectangle, kept or not)
    if (cnt) g.rec[vo + gi].d.z = ioff + myoff;
    uint32_t carry = 0u;  // 1 + owner of the previous chunk's last position
    for (uint32_t c0 = 0; c0 < btot; c0 += 64) {
      s.own[lane] = 0u;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (cnt && myoff >= c0 && myoff < c0 + 64) s.own[myoff - c0] = (uint32_t)lane + 1u;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const uint32_t ow1 = max(carry, wave_incl_max_dpp(s.own[lane]));
      carry = (uint32_t)__builtin_amdgcn_readlane((int)ow1, 63);
      const uint32_t j = c0 + (uint32_t)lane;
      bool kp = false;
      uint32_t key = 0u, gv = 0u;
      if (j < btot) {
        const uint32_t ow = ow1 - 1u;
        const uint2 rc = s.rect[ow];
        const uint32_t xmin = rc.x & 0xffffu, ymin = rc.x >> 16, xmax = rc.y & 0xffffu;
        const uint32_t wd = xmax - xmin, l = j - s.off[ow];
        // l / wd without the ~35-instruction integer division: l < 2^24, so the float quotient is
        // within one of the true one; one correction step makes it exact
        int ty = (int)((float)l * __builtin_amdgcn_rcpf((float)wd));
        int tx = (int)l - ty * (int)wd;
        if (tx < 0) { --ty; tx += (int)wd; }
        else if (tx >= (int)wd) { ++ty; tx -= (int)wd; }
        const int row = (int)ymin + ty, col = (int)xmin + tx;
        const SpanPrep sp = s.sp[ow];
        int t0, t1;
        span_row(sp, row, (int)xmin, (int)xmax, t0, t1);
        kp = col >= t0 && col < t1;
        const uint32_t tile = (uint32_t)row * (uint32_t)grid_x + (uint32_t)col;
        gv = s.gi[ow];
        key = vout ? tile : ((tile << gbits) | gv);
      }
      const unsigned long long bal = __ballot(kp);
      if (kp) {
        const uint32_t o = kbase + mask_rank(bal);
        kout[o] = key;
        if (vout) vout[o] = gv;
      }
      kbase += (uint32_t)__popcll(bal);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own[] is rewritten by the next chunk
    }
  }
}

// After the tile sort: per-tile [start, end) ranges (view-local positions) of each view's list.
// One wave streams GSR_RANGE_ROUNDS x 64 consecutive instances, lane-interleaved (coalesced): all
// rounds' keys are loaded first, neighbours come from the adjacent lanes (shuffles) and, at round
// edges, from the neighbouring round (readlane).
#define GSR_RANGE_ROUNDS 16
__global__ __launch_bounds__(256) void k_tile_ranges(SegInfo inst, int n_tiles, int gbits,
                                                     const uint32_t* __restrict__ keys,
                                                     uint2* __restrict__ ranges) {
  uint32_t lb;
  const int v = seg_of_block(inst, blockIdx.x, lb);
  const int lane = threadIdx.x & 63;
  const uint32_t base = (lb * 4 + (threadIdx.x >> 6)) * (64u * GSR_RANGE_ROUNDS);
  const uint32_t K = seg_live(inst, v);
  if (base >= K) return;  // wave-uniform
  const uint32_t* kv = keys + inst.start[v];
  uint2* rv = ranges + (size_t)v * n_tiles;
  uint32_t t[GSR_RANGE_ROUNDS];
#pragma unroll
  for (int r = 0; r < GSR_RANGE_ROUNDS; ++r) {
    const uint32_t i = base + 64u * r + lane;
    t[r] = i < K ? kv[i] >> gbits : 0xFFFFFFFFu;
  }
  const uint32_t before = base > 0 ? kv[base - 1] >> gbits : 0xFFFFFFFFu;
  const uint32_t e = base + 64u * GSR_RANGE_ROUNDS;
  const uint32_t after = e < K ? kv[e] >> gbits : 0xFFFFFFFFu;
#pragma unroll
  for (int r = 0; r < GSR_RANGE_ROUNDS; ++r) {
    const uint32_t p = base + 64u * r + lane;
    if (base + 64u * r >= K) break;  // wave-uniform
    uint32_t prev = (uint32_t)__shfl_up((int)t[r], 1, 64);
    uint32_t next = (uint32_t)__shfl_down((int)t[r], 1, 64);
    if (lane == 0) prev = r == 0 ? before : (uint32_t)__builtin_amdgcn_readlane((int)t[r > 0 ? r - 1 : 0], 63);
    if (lane == 63)
      next = r == GSR_RANGE_ROUNDS - 1 ? after
                                       : (uint32_t)__builtin_amdgcn_readlane((int)t[r + 1 < GSR_RANGE_ROUNDS ? r + 1 : r], 0);
    if (p < K) {
      if (prev != t[r]) rv[t[r]].x = p;
      if (next != t[r]) rv[t[r]].y = p + 1;
    }
  }
}

void launch_binning_counts(int V, int P, const GeomState& g, hipStream_t stream) {
  if (V <= 0) return;
  const int nbe = GeomState::dup_blocks(P);
  if (P > 0)
    hipLaunchKernelGGL(k_inst_count, dim3(V * ((nbe + 3) / 4)), dim3(256), 0, stream, P, nbe, g);
  hipLaunchKernelGGL(k_inst_scan, dim3(V), dim3(1024), 0, stream, P > 0 ? nbe : 0, g);
}

void launch_emit(int V, int P, int W, const GeomState& g, const SegInfo& inst, int gbits, uint32_t* keys,
                 uint32_t* vals, hipStream_t stream) {
  if (V <= 0 || P <= 0) return;
  const int nbe = GeomState::dup_blocks(P);
  hipLaunchKernelGGL(k_emit, dim3(V * div_up(nbe, GSR_EMIT_GROUPS)), dim3(64), 0, stream, P, nbe,
                     div_up(W, GSR_TILE_X), g, inst, gbits, keys, vals);
}

void launch_tile_ranges(SegInfo inst, int n_tiles, int gbits, const uint32_t* keys, uint2* ranges, hipStream_t stream) {
  seg_fill_blocks(inst, GSR_RANGE_TILE);
  if (inst.blk[inst.V] == 0) return;
  hipLaunchKernelGGL(k_tile_ranges, dim3(inst.blk[inst.V]), dim3(256), 0, stream, inst, n_tiles, gbits, keys, ranges);
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

// gsr_render.hip — per-tile alpha blending of a view set, forward and backward.
//
// One 64-thread wave per (view, 16x16 tile, 8x8 quadrant); the views of a set are consecutive
// ranges of the grid, so one launch blends every view and the heavy tiles of one view overlap the
// light tiles of the others.  Gaussian records (48 B: xy, conic, opacity, depth, rgb) are gathered
// by sorted instance in chunks of 64; a conservative quadrant test (bounding box of the
// alpha >= 1/255 ellipse, padded) drops Gaussians that cannot reach the wave's pixels before they
// are compacted into LDS (ballot) and read back as broadcast ds_read_b128.  The dropped pairs are
// exactly pairs the reference rejects with alpha < 1/255, so results are unchanged.
//
// Forward replaces FORWARD::renderCUDA [EXT] (ashawkey 4-output: color, depth = sum z a T,
// alpha = 1 - T).  Backward replaces BACKWARD::renderCUDA [EXT]: instead of 9 global float atomics
// per (pixel, Gaussian) pair it reduces each pair's gradient moments over 16-lane rows with DPP,
// parks the 4 row partials per Gaussian in LDS, and every 32 Gaussians sums them and writes ONE
// 48-byte row per (instance, quadrant) into the Gaussian's own slot (gsr_backward.hip sums a
// Gaussian's rows in a fixed order -> deterministic, no atomics, no inverse permutation).
#include <cstdlib>
#include <cstring>

#include "gsr_kernels.h"
#include "gsr_wave.h"

#ifndef GSR_FWD_PREFETCH
// the quadrant-wave forward reads the next candidate's staged record before blending the current one (left to
// itself the compiler sinks those reads to their use; the two-colour variant then runs at 7 waves per SIMD
// instead of 8)
#define GSR_FWD_PREFETCH 1
#endif
#ifndef GSR_FWD_WPE
#define GSR_FWD_WPE 1  // k_render_fwd minimum waves per SIMD (7 / 8 spill the two-colour variant)
#endif
#ifndef GSR_BWD_OVERLAP
#define GSR_BWD_OVERLAP 1  // replay steps of a full group scheduled together (k_render_bwd; 2 spills 4 VGPRs)
#endif

namespace gsr {

// blockIdx -> (tile, quadrant).  Blocks b and b+8 share an XCD under round-robin dispatch (speed
// only, never correctness).  Units are grouped in 2x2-tile super-tiles (16 quadrant waves that share
// most of their Gaussians -> one L2), and super-tiles are dealt round-robin over the 8 XCD groups so
// the spatially clustered heavy tiles spread evenly over the chip (contiguous bands per XCD left the
// scene centre on 2-3 XCDs).  Grid = 128 * ceil(super-tiles / 8); surplus blocks return false.
#ifdef GSR_TIMELINE
// Diagnostic build only (make diag): per-block (start, end) in s_memrealtime ticks (100 MHz), HW_ID,
// XCC_ID << 24 | work count.  [0] = k_render_fwd, [1] = k_render_bwd.
#define GSR_TL_MAX 65536
__device__ uint4 g_timeline[2][GSR_TL_MAX];
// pair counters (vector global atomics, diagnostic build only): [0] forward (pixel, Gaussian) pairs
// evaluated (lanes not yet terminated), [1] forward pair slots issued (64 lanes x candidates walked),
// [2] backward kept (candidate, quadrant) pairs replayed x 64 pixels, [3] backward pair slots of the
// lockstep batches (4 x the busiest quadrant's kept count x 64)
__device__ unsigned long long g_pairs[8];
#define GSR_TL_BEGIN const uint32_t tl_t0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
#define GSR_TL_END(which, work)                                                                  \
  if (threadIdx.x == 0 && blockIdx.x < GSR_TL_MAX)                                                \
    g_timeline[which][blockIdx.x] =                                                               \
        make_uint4(tl_t0, (uint32_t)__builtin_amdgcn_s_memrealtime(),                             \
                   (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4),                           \
                   ((uint32_t)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 24) | ((work) & 0xffffffu));
#else
#define GSR_TL_BEGIN
#define GSR_TL_END(which, work)
#endif

// blockIdx -> (view of the launch, tile, quadrant) for PER blocks per 2x2-tile super-tile (4: a workgroup
// per tile; 16: a wave per 8x8 quadrant).  Groups of 8 consecutive super-tiles are dealt one to each XCD
// (x = b & 7) with all blocks of a super-tile on the same XCD (its tiles share Gaussians in L2).  With an
// order (rs.order): chunks of GSR_ORDER_CHUNK views in turn, inside a chunk all its views' super-tiles
// heaviest first — a launch lasts at least its slowest workgroup, so the long tiles start first and the
// short ones fill the tail; chunks bound how many views' records compete in L2 at once (chunk 1 / 4 / 8 /
// 16 / all 64: C3 backward 0.0976 / 0.0955 / 0.0955 / 0.098 / 0.100 ms/view, 8-view launches best fully
// interleaved; profiles/r02_tile_order_ab.txt).  Without: the views in turn, super-tiles in raster order.
// The chunk is rs.ochunk (order_chunk): 8 views, and for sets of GSR_ORDER_BIG_SET views or more of views with
// GSR_ORDER_BIG_VIEW super-tiles or more 2 in the forwards and 4 in the backwards — re-measured on the round-6
// kernels (profiles/r06/ab_r06z3.txt, ab_r06z5.txt): 64-view C3 forward 0.0436 -> 0.0388 ms/view at chunk 2 (fewer
// views' records compete in the caches), C5 backward 0.227 -> 0.221 at 4; 8-view sets stay fully interleaved (their
// forward 0.045 -> 0.048 at chunk 2), and so do small views (64 views at 256^2: 64 super-tiles a view, forward
// 0.019 -> 0.023 at chunk 2 — two views' heaviest tiles cannot fill the chip, the later chunks' start late).
#ifndef GSR_ORDER_CHUNK
#define GSR_ORDER_CHUNK 8
#endif
#ifndef GSR_ORDER_BIG_SET
#define GSR_ORDER_BIG_SET 32
#endif
#ifndef GSR_ORDER_BIG_VIEW
#define GSR_ORDER_BIG_VIEW 512  // super-tiles per view (1024^2: 1024, C5's 800^2: 625, 256^2: 64)
#endif
#ifndef GSR_ORDER_CHUNK_FWD_BIG
#define GSR_ORDER_CHUNK_FWD_BIG 2
#endif
#ifndef GSR_ORDER_CHUNK_BWD_BIG
#define GSR_ORDER_CHUNK_BWD_BIG 4
#endif
int order_chunk(int V, int gx, int gy, bool forward) {
  const int S = ((gx + 1) >> 1) * ((gy + 1) >> 1);  // super-tiles per view (block_map)
  if (V >= GSR_ORDER_BIG_SET && S >= GSR_ORDER_BIG_VIEW) return forward ? GSR_ORDER_CHUNK_FWD_BIG : GSR_ORDER_CHUNK_BWD_BIG;
  return GSR_ORDER_CHUNK;
}
template <int PER>
__device__ __forceinline__ bool block_map(int b, const RenderSet& rs, int& v, int& tile, int& q) {
  const int sgx = (rs.gx + 1) >> 1, sgy = (rs.gy + 1) >> 1, S = sgx * sgy;
  int s, w;
  if (rs.order != nullptr) {
    const int x = b & 7, k = b >> 3;
    w = k & (PER - 1);
    const int m = ((k / PER) << 3) + x;
    if (m >= rs.V * S) return false;
    // chunks of GSR_ORDER_CHUNK views, interleaved inside a chunk (all its views' heaviest super-tiles
    // first), the chunks in turn
    const int ch = rs.ochunk;
    const int c = m / (ch * S), local = m - c * ch * S;
    const int vc = min(ch, rs.V - c * ch);
    v = c * ch + local % vc;
    s = (int)rs.order[(size_t)(rs.v0 + v) * S + local / vc];
  } else {
    const int G = PER * 8 * ((S + 7) >> 3);
    v = b / G;
    const int bl = b - v * G, x = bl & 7, k = bl >> 3;
    w = k & (PER - 1);
    s = ((k / PER) << 3) + x;
    if (s >= S) return false;
  }
  const int tx = (s % sgx) * 2 + (PER == 16 ? (w >> 2) & 1 : w & 1);
  const int ty = (s / sgx) * 2 + (PER == 16 ? w >> 3 : w >> 1);
  if (tx >= rs.gx || ty >= rs.gy) return false;
  tile = ty * rs.gx + tx;
  q = w & 3;
  return true;
}
// launch sizes for block_map
static int block_grid(const RenderSet& rs, int per) {
  const int S = ((rs.gx + 1) >> 1) * ((rs.gy + 1) >> 1);
  return rs.order != nullptr ? per * 8 * div_up((long long)rs.V * S, 8) : rs.V * per * 8 * ((S + 7) >> 3);
}


__device__ __forceinline__ void tile_pixel(int t, int& lx, int& ly) {
  const int w = t >> 6, l = t & 63;
  lx = ((w & 1) << 3) | (l & 7);
  ly = ((w >> 1) << 3) | (l >> 3);
}

// per-lane select by a wave mask: one v_cndmask_b32 (keeps the replay's state updates branch-free;
// left to itself the compiler turns a run of selects on one condition into an exec-masked branch)
__device__ __forceinline__ float vsel(unsigned long long m, float if_set, float if_clear) {
  float r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if_clear), "v"(if_set), "s"(m));
  return r;
}

typedef float f2 __attribute__((ext_vector_type(2)));  // packed fp32 pairs (v_pk_*_f32)

// one screen-mean gradient component, k dd (2 a m_a + b m_b), in an explicit operation order: the backward
// kernels stage the conic in different slots, and left to itself the compiler contracts the sum differently
// per kernel, which breaks the variants' bitwise agreement
__device__ __forceinline__ float mean_grad(float k, float dd, float a, float b, float m_a, float m_b) {
  return k * dd * fmaf(2.0f * a, m_a, b * m_b);
}

// a wave-uniform float kept in a scalar register
__device__ __forceinline__ float sgpr_f(float x) {
  float r;
  // (the builtin is folded away for a uniform x; the nops cover the VALU-write -> readlane hazard inline asm hides
  // from the compiler; once per kernel)
  asm volatile("s_nop 4\n\tv_readfirstlane_b32 %0, %1" : "=s"(r) : "v"(x));
  return r;
}

// a copy the compiler cannot fold away: it ends the source register's live range at this point
__device__ __forceinline__ float vcopy(float x) {
  float r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// The set's preprocess embedded exactly this col2 array in the records (GaussRec b.w, c.w, d.z): the two-colour
// blends then read the second colours with the record (one 4-byte load beside it) instead of gathering col2 apart
__device__ __forceinline__ bool col2_embedded(const RenderSet& rs) {
#ifdef GSR_EXP_NOEMBED
  return false;  // (timing only: the second colours gathered from col2 as before the records carried them)
#endif
  if (rs.col2 == nullptr || rs.col2_rec == nullptr) return false;
  const unsigned long long e = (unsigned long long)rs.col2_rec[0] | ((unsigned long long)rs.col2_rec[1] << 32);
  return e == (unsigned long long)(uintptr_t)rs.col2;
}

// bg . dL/dpixel with an explicit operation order (the backward kernels' background terms: every kernel
// variant forms the same bits, independent of how the compiler would contract the expression)
__device__ __forceinline__ float bg_dot3(const float* bg, float d0, float d1, float d2) {
  return fmaf(bg[2], d2, fmaf(bg[1], d1, bg[0] * d0));
}

// Forward: one wave (64 threads) per 8x8 quadrant of a 16x16 tile.  The wave streams the tile's
// depth-sorted instance list 64 at a time, keeps (ballot compaction, order preserved) only the
// Gaussians whose alpha >= 1/255 ellipse can reach its quadrant, and blends them with a
// branch-free predicated body.  No workgroup barriers couple quadrants that terminate at
// different depths, and 4x more independent waves balance the load across the 256 CUs.
// CK: also the split backward's per-chunk states (rs.ckpt, gsr_common.h ckpt_offset).
template <bool C2, bool CK>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GSR_FWD_WPE, 8))) void k_render_fwd(RenderSet rs,
                                                   const uint2* __restrict__ ranges,
                                                   const uint32_t* __restrict__ sorted_gauss,
                                                   const GaussRec* __restrict__ rec,
                                                   float* __restrict__ out_color,
                                                   float* __restrict__ out_depth,
                                                   float* __restrict__ out_alpha,
                                                   float* __restrict__ final_T,
                                                   uint32_t* __restrict__ n_contrib,
                                                   uint32_t* __restrict__ quad_maxc) {
  // 65 slots: the loop reads candidate k+1 while blending k (slot 64 is never used)
  __shared__ float4 s0[65], s1[65], s2[65];
  __shared__ float4 s3[C2 ? 65 : 1];  // the second colour (C2)
  int v, tile, q;
  if (!block_map<16>(blockIdx.x, rs, v, tile, q)) return;
  GSR_TL_BEGIN
  const int W = rs.W, H = rs.H, grid_x = rs.gx;
  {
    const size_t vg = (size_t)(rs.v0 + v), tiles = (size_t)rs.gx * rs.gy, HWs = (size_t)W * H;
    ranges += vg * tiles;
    quad_maxc += vg * 4 * tiles;
    sorted_gauss += rs.inst_start[v];
    rec += vg * rs.P;
    out_color += vg * 3 * HWs;
    out_depth += vg * HWs;
    out_alpha += vg * HWs;
    final_T += vg * HWs;
    n_contrib += vg * HWs;
  }
  const float* bg = rs.bg[v];
  const int unit = 4 * tile + q;
  const int lane = threadIdx.x;
  const int qx0 = (tile % grid_x) * GSR_TILE_X + (q & 1) * 8;
  const int qy0 = (tile / grid_x) * GSR_TILE_Y + (q >> 1) * 8;
  const int px = qx0 + (lane & 7), py = qy0 + (lane >> 3);
  const bool inside = px < W && py < H;
  const float pxf = (float)px, pyf = (float)py;
  const f2 pxy = {pxf, pyf};
  const uint2 range = ranges[tile];
  const int n = (int)(range.y - range.x);

  unsigned long long dmk = __ballot(!inside);  // lanes whose pixel is done (outside, or terminated)
  // running totals, packed in pairs (v_pk_fma_f32: two exact fmas per instruction): (r, g), (b, depth), second
  // colour (r, g) and b
  float T = 1.0f;
  f2 CrCg = {0.f, 0.f}, CbD = {0.f, 0.f};
  f2 ErEg = {0.f, 0.f};  // second colour (C2)
  float Eb = 0.f;
  uint32_t last_contributor = 0;
#ifdef GSR_TIMELINE
  unsigned long long pc_eval = 0, pc_slot = 0;
#endif
  // two-stage prefetch (as in the backward): indices two batches ahead, records one batch ahead
  const uint32_t gmask = rs.gmask;
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 n0 = zero4, n1 = zero4, n2 = zero4, n3 = zero4;
  uint32_t gi_next = 0u;
  const float* col2 = rs.col2;
  const bool emb = C2 && col2_embedded(rs);  // (n3 then read from the record's b.w, c.w, d.z: the same line)
  // quadrant masks in the keys (TilePack::qmask): the keep decision comes with the index, and only this
  // quadrant's candidates are gathered.  k_emit forms the masks with span_quads (a band / column bound on the
  // alpha >= 1/255 ellipse), not with quadrant_hit: the two tests differ, but each keeps every quadrant that holds
  // a blending pixel, so the blended candidates per pixel, and the outputs, are the same
  // (tests/test_quadrant_bounds.py)
  const uint32_t* qkeys = rs.qkeys ? rs.qkeys + rs.inst_start[v] + range.x : nullptr;
  const int qsh = GSR_QMASK_SHIFT + q;
  // (gi_next and its key word stay raw until the next batch: masked or tested right after their load, the wave
  // would wait there for every load in flight, the records just issued included)
  bool kn = false;           // the keep bit of the batch in n0..n3
  uint32_t kw_next = ~0u;    // gi_next's key word (qkeys; all ones without)
  if (lane < n) kn = qkeys == nullptr || ((qkeys[lane] >> qsh) & 1u);
  if (kn) {
    const uint32_t g0 = sorted_gauss[range.x + lane] & gmask;
    n0 = rec[g0].a;
    n1 = rec[g0].b;
#ifndef GSR_EXP_FWD_NOC
    n2 = rec[g0].c;
#endif
#ifdef GSR_EXP_NOCOL2
    if (C2) n3 = make_float4(__uint_as_float(g0), 0.f, 0.f, 0.f);  // timing only: no col2 gather
#else
    if (C2 && emb) n3 = make_float4(rec[g0].b.w, rec[g0].c.w, __uint_as_float(rec[g0].d.z), 0.f);
    else if (C2) n3 = make_float4(col2[3 * g0], col2[3 * g0 + 1], col2[3 * g0 + 2], 0.f);
#endif
  }
  if (64 + lane < n) {
    gi_next = sorted_gauss[range.x + 64 + lane];
    if (qkeys != nullptr) kw_next = qkeys[64 + lane];
  }
  // split backward: T at each chunk boundary the walk reaches, and each chunk's own colour / depth sums
  float* const ckpt = CK ? rs.ckpt + ckpt_offset((size_t)(rs.v0 + v), (size_t)rs.gx * rs.gy, tile, 0) : nullptr;
  const int cpix = 64 * q + lane;
  if (CK && blockIdx.x == 0 && lane == 0) rs.split_items[0] = 0u;  // k_ckpt_suffix lists the split items
  f2 PrPg = {0.f, 0.f}, PbPd = {0.f, 0.f};
  int chunk = 0;
  // the previous batch's cull byte, stored once the next batch's loads are issued (a store at the batch end would
  // hold up the next batch's wait for its records)
  uint8_t* qbp = nullptr;
  uint8_t qbv = 0u;
  for (int base = 0; base < n; base += 64) {
    if (dmk == ~0ull) break;
    if (CK && base > 0 && base % GSR_SPLIT_CH == 0 && base <= GSR_SPLIT_NCK * GSR_SPLIT_CH) {
      // chunk `chunk` ends: its sums into its slot, T into the next one's slot
      reinterpret_cast<float4*>(ckpt + (size_t)chunk * GSR_CKPT_FIELDS * 256 + 256)[cpix] =
          make_float4(PrPg.x, PrPg.y, PbPd.x, PbPd.y);
      ++chunk;
      ckpt[(size_t)chunk * GSR_CKPT_FIELDS * 256 + cpix] = T;
      PrPg = f2{0.f, 0.f};
      PbPd = f2{0.f, 0.f};
    }
    const int i = base + lane;
    const float4 r0 = n0, r1 = n1, r2 = n2, r3 = n3;
    const bool kc = kn;
    kn = base + 64 + lane < n && ((kw_next >> qsh) & 1u);
    const uint32_t gn = gi_next & gmask;
    if (kn) {
      n0 = rec[gn].a;
      n1 = rec[gn].b;
#ifndef GSR_EXP_FWD_NOC
      n2 = rec[gn].c;
#endif
#ifdef GSR_EXP_NOCOL2
      if (C2) n3 = make_float4(__uint_as_float(gn), 0.f, 0.f, 0.f);  // timing only: no col2 gather
#else
      if (C2 && emb) n3 = make_float4(rec[gn].b.w, rec[gn].c.w, __uint_as_float(rec[gn].d.z), 0.f);
      else if (C2) n3 = make_float4(col2[3 * gn], col2[3 * gn + 1], col2[3 * gn + 2], 0.f);
#endif
    }
    if (base + 128 + lane < n) {
      gi_next = sorted_gauss[range.x + base + 128 + lane];
      if (qkeys != nullptr) kw_next = qkeys[base + 128 + lane];
    }
    if (qbp != nullptr) *qbp = qbv;
    bool keep = false;
    if (i < n) keep = qkeys ? kc : quadrant_hit(r0, r1, (float)qx0, (float)qy0);
    const unsigned long long bal = __ballot(keep);
    const int cnt = __popcll(bal);
    if (keep) {
      // the conic pre-multiplied for gauss_power2, staged as s0 = (x, y, B, C), s1 = (A, opacity, depth, 1 + list
      // position), s2 = (r, g, b, depth): the pairs the step packs are adjacent
      const uint32_t pos = mask_rank(bal);
      s0[pos] = make_float4(r0.x, r0.y, GSR_CONIC_K_B * r0.w, GSR_CONIC_K_AC * r1.x);
      s1[pos] = make_float4(GSR_CONIC_K_AC * r0.z, r1.y, r1.z, __uint_as_float((uint32_t)(i + 1)));
      s2[pos] = make_float4(r2.x, r2.y, r2.z, r1.z);
      if (C2) s3[pos] = r3;
    }
    __syncthreads();
    // one blend step: candidate k from the register set `cur`, the next staged record into `nxt` (the loop runs
    // the step twice with the sets swapped: no register copies); done / ok / term / blend as uniform lane masks
    int k = 0;
    unsigned long long hbm = 0ull;  // staged candidates (by position) that blended at least one pixel (uniform)
    // (true while candidates remain; the wave's termination is tested every second step, in the loop below)
    auto step = [&](const float4& a, const float4& b, const float4& c, const float4& e, float4& an, float4& bn,
                    float4& cn, float4& en) -> bool {
      an = s0[k + 1], bn = s1[k + 1], cn = s2[k + 1];
      en = C2 ? s3[k + 1] : zero4;
#if GSR_FWD_PREFETCH
      asm volatile("" ::: "memory");  // (the next candidate's reads stay ahead of this step: a prefetch)
#endif
      // gauss_power2(A, B, C, dx, dy) = fma(dx, fma(A, dx, B dy), (C dy) dy), with (B dy, C dy) as one product
      const f2 dd = f2{a.x, a.y} - pxy;
      const f2 bc = f2{a.z, a.w} * f2{dd.y, dd.y};
      const float power2 = fmaf(dd.x, fmaf(b.x, dd.x, bc.x), bc.y * dd.y);  // log2(e) * power
      const float alpha = fminf(GSR_ALPHA_MAX, b.y * __builtin_amdgcn_exp2f(power2));
#ifdef GSR_TIMELINE
      pc_eval += (dmk >> lane) & 1ull ? 0ull : 1ull;
      pc_slot += 1ull;
#endif
      const unsigned long long okm = (__ballot(power2 <= 0.0f) & __ballot(alpha >= GSR_ALPHA_MIN)) & ~dmk;
      const float test_T = T * (1.0f - alpha);
      const unsigned long long termm = okm & __ballot(test_T < GSR_T_EPS);
      const unsigned long long blendm = okm & ~termm;
      // non-blending lanes run the same arithmetic with alpha = 0 (no change), no selects of state
      const float a_eff = vsel(blendm, alpha, 0.0f);
      const float aT = a_eff * T;
      // the running totals in list order whatever the launch (the outputs' bits do not depend on whether the
      // launch writes checkpoints), and beside them the chunk's own sums for the split backward
      const f2 aT2 = {aT, aT};
      CrCg = __builtin_elementwise_fma(f2{c.x, c.y}, aT2, CrCg);
      CbD = __builtin_elementwise_fma(f2{c.z, c.w}, aT2, CbD);
      if (CK) {
        PrPg = __builtin_elementwise_fma(f2{c.x, c.y}, aT2, PrPg);
        PbPd = __builtin_elementwise_fma(f2{c.z, c.w}, aT2, PbPd);
      }
      if (C2) {
        ErEg = __builtin_elementwise_fma(f2{e.x, e.y}, aT2, ErEg);
        Eb = fmaf(e.z, aT, Eb);
      }
      T = vsel(blendm, test_T, T);  // = T (1 - a_eff)
      last_contributor = __float_as_uint(vsel(blendm, b.w, __uint_as_float(last_contributor)));
      dmk |= termm;
      hbm |= blendm != 0ull ? 1ull << k : 0ull;
      ++k;
      return k < cnt;
    };
    if (cnt > 0) {
      float4 pa = s0[0], pb = s1[0], pc = s2[0], pd = C2 ? s3[0] : zero4;
      float4 ya, yb, yc, yd;
      while (dmk != ~0ull && step(pa, pb, pc, pd, ya, yb, yc, yd) && step(ya, yb, yc, yd, pa, pb, pc, pd)) {
      }
    }
    // the backward's exact cull (RenderSet::qbytes, layout 2: byte 4 i + q of the set's listed instance i): whether
    // candidate i blended any pixel of this quadrant (a pair the forward blended nowhere has no backward hit: same
    // alpha, power and position tests).  Batches past the quadrant's termination are never walked, and the backward
    // reads only below its deepest blend.
    if (rs.qbytes != nullptr && i < n) {
      qbp = rs.qbytes + 4 * ((size_t)rs.inst_start[v] + range.x + i) + q;
      qbv = keep && ((hbm >> mask_rank(bal)) & 1ull) ? 1u : 0u;
    } else {
      qbp = nullptr;
    }
    __syncthreads();
  }
  if (qbp != nullptr) *qbp = qbv;
  if (inside) {
    const size_t pid = (size_t)py * W + px;
    const size_t HW = (size_t)H * W;
    final_T[pid] = T;
    n_contrib[pid] = last_contributor;
    const float Cr = CrCg.x, Cg = CrCg.y, Cb = CbD.x, D = CbD.y;
    {
      // C + T bg as a rounded product then a rounded sum (the oracle's order, and the same value the fused
      // composite below starts from), never contracted: every instantiation stores the same bits
#pragma clang fp contract(off)
      out_color[pid] = Cr + T * bg[0];
      out_color[HW + pid] = Cg + T * bg[1];
      out_color[2 * HW + pid] = Cb + T * bg[2];
    }
    out_depth[pid] = D;
    out_alpha[pid] = 1.0f - T;
    if (C2) {
#pragma clang fp contract(off)
      float* o2 = rs.out_col2 + (size_t)(rs.v0 + v) * 3 * HW + pid;
      o2[0] = ErEg.x + T * bg[0];
      o2[HW] = ErEg.y + T * bg[1];
      o2[2 * HW] = Eb + T * bg[2];
    }
    if (rs.comp != nullptr) {
      // fused composite (without background images: the renderer's clamp alone), the same operations as the torch
      // epilogue on the stored outputs (bit-identical)
#pragma clang fp contract(off)
      float p0 = Cr + T * bg[0], p1 = Cg + T * bg[1], p2 = Cb + T * bg[2];
      if (rs.cbg != nullptr) {
        const float am = 1.0f - (1.0f - T);
        const float* bgi = rs.cbg + ((size_t)v * HW + pid) * 3;
        p0 = p0 + am * bgi[0];
        p1 = p1 + am * bgi[1];
        p2 = p2 + am * bgi[2];
      }
      float* cp = rs.comp + (size_t)v * 3 * HW + pid;
      cp[0] = fminf(fmaxf(p0, 0.0f), 1.0f);
      cp[HW] = fminf(fmaxf(p1, 0.0f), 1.0f);
      cp[2 * HW] = fminf(fmaxf(p2, 0.0f), 1.0f);
    }
  }
  if (CK && chunk > 0) {
    // the chunk the walk ended in (the backward reads chunks up to the quadrant's deepest blend only)
    reinterpret_cast<float4*>(ckpt + (size_t)chunk * GSR_CKPT_FIELDS * 256 + 256)[cpix] =
        make_float4(PrPg.x, PrPg.y, PbPd.x, PbPd.y);
  }
  uint32_t mc = last_contributor;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mc = max(mc, (uint32_t)__shfl_xor((int)mc, o, 64));
  if (lane == 0) quad_maxc[unit] = mc;
#ifdef GSR_TIMELINE
  atomicAdd(&g_pairs[0], pc_eval);  // per-lane values; the backend's atomic optimizer combines the wave
  atomicAdd(&g_pairs[1], pc_slot);
#endif
  GSR_TL_END(0, mc)
}

// Per tile: instances [0, maxc) were blended by some pixel (max over the 4 quadrants); record the
// (depth key, Gaussian) of the first instance nobody blended.  The backward writes gradient rows
// for exactly the instances [0, maxc) of each tile (all 4 quadrants), so the per-Gaussian
// gather-sum can test validity per instance against this cutoff.
__global__ __launch_bounds__(256) void k_tile_info(RenderSet rs, const uint2* __restrict__ ranges,
                                                   const uint32_t* __restrict__ quad_maxc,
                                                   const uint32_t* __restrict__ sorted_gauss,
                                                   const GaussRec* __restrict__ rec,
                                                   uint4* __restrict__ tile_info, uint2* __restrict__ cut) {
  const int n_tiles = rs.gx * rs.gy;
  const int nb = div_up(n_tiles, 256);
  const int v = blockIdx.x / nb;
  const int tile = (blockIdx.x - v * nb) * blockDim.x + threadIdx.x;
  if (tile >= n_tiles) return;
  {
    const size_t vg = (size_t)(rs.v0 + v);
    ranges += vg * n_tiles;
    quad_maxc += vg * 4 * n_tiles;
    tile_info += vg * n_tiles;
    cut += vg * n_tiles;
    sorted_gauss += rs.inst_start[v];
    rec += vg * rs.P;
  }
  const uint4 m = reinterpret_cast<const uint4*>(quad_maxc)[tile];
  const uint32_t maxc = max(max(m.x, m.y), max(m.z, m.w));
  const uint2 range = ranges[tile];
  uint4 info = make_uint4(maxc, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u);
  if (maxc < range.y - range.x) {
    const uint32_t gi = sorted_gauss[range.x + maxc] & rs.gmask;
    info.y = __float_as_uint(rec[gi].b.z);
    info.z = gi;
  }
  tile_info[tile] = info;
  cut[tile] = make_uint2(info.y, info.z);
}

// ---------------------------------------------------------------------------------------
// Backward.  Per pixel the reference's back-to-front replay: T recovered by division, the colour
// accumulated behind each contributor, background term.  Per candidate the 10 gradient sums are
//   0 sum u  1,2 sum u dx, u dy  3,4,5 sum u dx^2, u dx dy, u dy^2  6,7,8,9 sum w dL/d(r,g,b,depth)
// with u = G dL/dalpha, w = alpha T (the reference's dmean2D / dconic / dopacity / dcolor / ddepth
// are these sums times per-candidate factors).
#define NGV 10

// Backward: one 256-thread workgroup per (view, tile); wave q owns quadrant q.  The four waves walk
// the tile's list back to front in lockstep batches of 64 candidates: the batch's records are
// staged in LDS once for all four (one global gather per candidate instead of four), each wave culls
// the batch for its quadrant, replays its kept candidates per pixel and sums them over its 64 pixels
// on the matrix cores, 8 candidates per 16x16 product, into per-(candidate, quadrant) sums in LDS;
// one thread per candidate then adds the four quadrants and writes ONE 48-byte gradient row per
// instance.

// (The SuGaR renderer's two-colour backward, whose Gaussians blend at ~13 pixels, forms its sums from hit
// lists instead: k_render_bwd_tw below.)
#define NGV2 16
#define GSR_QSUM_STRIDE 41   // floats per candidate: 4 quadrants x 10 raw sums, +1 pad
// uw: offset of the A operand's 16-pixel group g (256 floats each): groups 0, 2 at 0, 256 and groups 1, 3 at 528, 784,
// so the groups a 4-B write's lane half holds (0-1 for lanes 0-31, 2-3 for 32-63) lie 16 banks apart (the writes
// of pixels p and p + 16 do not conflict) and every 16-B read stays conflict-free (offsets of 16 dwords only
// rotate a read group's banks); 16 floats of padding in all (a pad per group would cost the 5th workgroup per CU:
// LDS is allocated in 1280-byte granules, 5 x 25 of 128 per CU)
// One wave's LDS accesses are performed in program order (the DS unit takes a wave's instructions in issue order),
// so a wave reading what its own lanes just wrote needs no s_waitcnt — only that the compiler keep the accesses in
// program order (a memory clobber): the wave keeps issuing while the writes drain.
#define GSR_WAVE_LDS_ORDER() asm volatile("" ::: "memory")
__device__ __forceinline__ int gsr_uw_pg(int g) { return 256 * (g >> 1) + ((g & 1) ? 528 : 0); }
#define GSR_HCAP2 160
// (LDS is allocated in 1280-byte granules: 5 workgroups of the backward per CU need <= 25 of the 128)
#define GSR_BWD_LDS_5WG (25 * 1280)
struct BwdLDS {
  float4 s0[65], s1[65], s2[65];
  uint32_t slot[64];
  uint32_t gidx[64];     // the staged candidates' Gaussians (their reach bits are set after the cull)
  uint32_t list[4][64];  // per wave: the batch indices of its kept candidates
  float qsum[64 * GSR_QSUM_STRIDE];
  // per wave: the group's A operand, u = G dL/dalpha (slots 0-7) and w = alpha T (slots 8-15) of
  // its 8 candidates, stored so that MFMA lane l's 16 values are 4 chunks of 16 B (swizzled:
  // conflict-free 16-B reads); 16-pixel group g at gsr_uw_pg(g), so a row's 4-B writes from pixels p and
  // p + 16 land in different banks (conflict-free)
  float uw[4][3 * 256 + 16 + 256];
  unsigned long long kmask[4];  // per quadrant: kept candidates of the batch
#ifdef GSR_TIMELINE
  int tl_cnt[4];
#endif
#ifdef GSR_EXP_LDSPAD
  char pad[GSR_EXP_LDSPAD];  // timing only: occupancy sensitivity (fewer workgroups per CU)
#endif
};


// Forward, one 64-thread wave per 16x16 tile (4 pixels per lane: the same pixel of each 8x8 quadrant).
// The wave gathers each tile candidate once (the quadrant-wave kernel above gathers it in each of the
// four waves), tests it against the four quadrants (quadrant_hit, the same conservative test) and keeps
// the 4-bit mask with the staged record; the blend walks the staged candidates and evaluates a quadrant's
// pixel only for candidates whose mask has that quadrant — per pixel exactly the candidates, in the same
// order, with the same operations as the quadrant-wave kernel, so the outputs are bitwise identical.
// Finished quadrants leave the mask (uniform), and the wave stops when all four are done.
template <bool C2>
// 6 waves per SIMD for the one-colour variant (89 -> 80 VGPRs, 3 spilled outside the candidate loop:
// render_fwd 0.049 -> 0.047 ms/view at C3, profiles/r02_fwd_occupancy_ab.txt); the two-colour one would
// spill 32 VGPRs and keeps the compiler's choice
__attribute__((amdgpu_waves_per_eu(C2 ? 1 : 6, 8)))
__global__ __launch_bounds__(64) void k_render_fwd_tile(RenderSet rs, const uint2* __restrict__ ranges,
                                                        const uint32_t* __restrict__ sorted_gauss,
                                                        const GaussRec* __restrict__ rec, float* __restrict__ out_color,
                                                        float* __restrict__ out_depth, float* __restrict__ out_alpha,
                                                        float* __restrict__ final_T, uint32_t* __restrict__ n_contrib,
                                                        uint32_t* __restrict__ quad_maxc) {
  __shared__ float4 s0[64], s1[64], s2[64];
  __shared__ float4 s3[C2 ? 64 : 1];
  int v, tile, q_unused;
  if (!block_map<4>(blockIdx.x, rs, v, tile, q_unused)) return;
  const int W = rs.W, H = rs.H, grid_x = rs.gx;
  const size_t HWs = (size_t)W * H;
  {
    const size_t vg = (size_t)(rs.v0 + v), tiles = (size_t)rs.gx * rs.gy;
    ranges += vg * tiles;
    quad_maxc += vg * 4 * tiles;
    sorted_gauss += rs.inst_start[v];
    rec += vg * rs.P;
    out_color += vg * 3 * HWs;
    out_depth += vg * HWs;
    out_alpha += vg * HWs;
    final_T += vg * HWs;
    n_contrib += vg * HWs;
  }
  const float* bg = rs.bg[v];
  const int lane = threadIdx.x;
  const int tx0 = (tile % grid_x) * GSR_TILE_X, ty0 = (tile / grid_x) * GSR_TILE_Y;
  // per quadrant: the pixel, T, and the running totals packed in pairs (v_pk_fma_f32): (r, g), (b, depth),
  // second colour (r, g) and b
  float T[4], Eb[4];
  f2 pxy[4], CrCg[4], CbD[4], ErEg[4];
  uint32_t last[4];
  bool inside[4];
  // per quadrant the lanes whose pixel is done (outside the image, or terminated): uniform 64-bit masks, so the
  // step's conditions combine in scalar registers and the selects read them directly
  unsigned long long dm[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int px = tx0 + (q & 1) * 8 + (lane & 7), py = ty0 + (q >> 1) * 8 + (lane >> 3);
    inside[q] = px < W && py < H;
    dm[q] = __ballot(!inside[q]);
    pxy[q] = f2{(float)px, (float)py};
    T[q] = 1.0f;
    CrCg[q] = CbD[q] = ErEg[q] = f2{0.f, 0.f};
    Eb[q] = 0.f;
    last[q] = 0u;
  }
  // the quadrant origins of the cull (wave-uniform: held in scalar registers, not reloaded from spill slots)
  const float qox[2] = {sgpr_f((float)tx0), sgpr_f((float)(tx0 + 8))};
  const float qoy[2] = {sgpr_f((float)ty0), sgpr_f((float)(ty0 + 8))};
  const uint2 range = ranges[tile];
  uint8_t* const qbytes = rs.qbytes ? rs.qbytes + rs.inst_start[v] + range.x : nullptr;
  const int n = (int)(range.y - range.x);
  const uint32_t gmask = rs.gmask;
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  const float* col2 = rs.col2;
  const bool emb = C2 && col2_embedded(rs);  // (n3 then read from the record's b.w, c.w, d.z: the same line)
  float4 n0 = zero4, n1 = zero4, n2 = zero4, n3 = zero4;
  uint32_t gi_next = 0u;
  if (lane < n) {
    const uint32_t g0 = sorted_gauss[range.x + lane] & gmask;
    n0 = rec[g0].a;
    n1 = rec[g0].b;
    n2 = rec[g0].c;
    if (C2 && emb) n3 = make_float4(rec[g0].b.w, rec[g0].c.w, __uint_as_float(rec[g0].d.z), 0.f);
    else if (C2) n3 = make_float4(col2[3 * g0], col2[3 * g0 + 1], col2[3 * g0 + 2], 0.f);
  }
  // (gi_next stays raw until the next batch: masked right after its load, the wave would wait there for every
  // load in flight, the records just issued included)
  if (64 + lane < n) gi_next = sorted_gauss[range.x + 64 + lane];
  // quadrants with a pixel still blending (uniform)
  auto active_mask = [&]() -> uint32_t {
    uint32_t m = 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q) m |= dm[q] == ~0ull ? 0u : (1u << q);
    return m;
  };
  uint32_t qactive = active_mask();
#ifdef GSR_TIMELINE
  unsigned long long pc_eval = 0, pc_slot = 0;
#endif
  // the previous batch's cull byte, stored once the next batch's loads are issued (a store at the batch end would
  // hold up the next batch's wait for its records)
  uint8_t qbv = 0u;
  int qbi = -1;
  for (int base = 0; base < n && qactive != 0u; base += 64) {
    const int i = base + lane;
    const float4 r0 = n0, r1 = n1, r2 = n2, r3 = n3;
    if (base + 64 + lane < n) {
      const uint32_t gn = gi_next & gmask;
      n0 = rec[gn].a;
      n1 = rec[gn].b;
      n2 = rec[gn].c;
      if (C2 && emb) n3 = make_float4(rec[gn].b.w, rec[gn].c.w, __uint_as_float(rec[gn].d.z), 0.f);
      else if (C2) n3 = make_float4(col2[3 * gn], col2[3 * gn + 1], col2[3 * gn + 2], 0.f);
    }
    if (base + 128 + lane < n) gi_next = sorted_gauss[range.x + base + 128 + lane];
    if (qbi >= 0) qbytes[qbi] = qbv;
    uint32_t m = 0u;
    if (i < n) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        m |= quadrant_hit(r0, r1, qox[q & 1], qoy[q >> 1]) ? (1u << q) : 0u;
    }
    // the conic pre-multiplied for gauss_power2, staged as s0 = (x, y, B, C), s1 = (A, opacity, depth, 1 + list
    // position), s2 = (r, g, b, depth): the pairs the step packs are adjacent (as k_render_fwd)
    s0[lane] = make_float4(r0.x, r0.y, GSR_CONIC_K_B * r0.w, GSR_CONIC_K_AC * r1.x);
    s1[lane] = make_float4(GSR_CONIC_K_AC * r0.z, r1.y, r1.z, __uint_as_float((uint32_t)(i + 1)));
    s2[lane] = make_float4(r2.x, r2.y, r2.z, r1.z);
    if (C2) s3[lane] = r3;
    // per quadrant the batch's candidates whose mask has it (uniform, in scalar registers)
    unsigned long long qb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) qb[q] = (qactive >> q) & 1u ? __ballot((m >> q) & 1u) : 0ull;
    __syncthreads();
    // The quadrants in turn, each walking its own candidates in list order: a pixel lies in one quadrant, so it
    // sees exactly the candidates, order and operations of the quadrant-wave kernel (bitwise), and a step is one
    // (candidate, quadrant) pair with no per-candidate quadrant tests (the union walk branched on four mask bits
    // per candidate: as many scalar as vector instructions, r05 SQ counters).  The next candidate's staged record
    // is read while the current one blends; a finished quadrant stops its walk (its lanes would blend nothing).
    // per quadrant the batch's candidates that blended at least one of its pixels (uniform): the backward's exact
    // cull (a (candidate, quadrant) pair the forward blended nowhere has no backward hit either: same alpha, power
    // and list-position tests, and a pixel's hits are exactly its blends before its last contributor)
    unsigned long long hb[4] = {0ull, 0ull, 0ull, 0ull};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      unsigned long long rest = qb[q];
      if (rest == 0ull) continue;
      int k = (int)__builtin_ctzll(rest);
      // one step: candidate k from the register set `cur`, the next candidate's staged record into `nxt` (the step
      // runs twice per loop iteration with the sets swapped: no register copies); false when the walk ends.  The
      // bookkeeping is scalar and as short as it goes: k's bit cleared by one xor with the bit the exact mask also
      // records, the next index by one find-first over rest with bit 63 forced (63 when rest is empty: a valid
      // staged slot, read but never blended)
      auto step = [&](float4& a, float4& b, float4& c, float4& e, float4& an, float4& bn, float4& cn,
                      float4& en) -> bool {
        const unsigned long long kbit = 1ull << k;
        rest ^= kbit;
        const int kn = (int)__builtin_ctzll(rest | (1ull << 63));
        an = s0[kn], bn = s1[kn], cn = s2[kn];
        en = C2 ? s3[kn] : zero4;
        // (the next record's reads issued before any of this step's arithmetic: a whole step to arrive)
        __builtin_amdgcn_sched_barrier(0);
#ifdef GSR_TIMELINE
        pc_eval += (dm[q] >> lane) & 1ull ? 0ull : 1ull;
        pc_slot += 1ull;
#endif
        const float dx = a.x - pxy[q].x, dy = a.y - pxy[q].y;
        const float power2 = fmaf(dx, fmaf(b.x, dx, a.z * dy), (a.w * dy) * dy);  // log2(e) * power
        const float alpha = fminf(GSR_ALPHA_MAX, b.y * __builtin_amdgcn_exp2f(power2));
        const unsigned long long okm = (__ballot(power2 <= 0.0f) & __ballot(alpha >= GSR_ALPHA_MIN)) & ~dm[q];
        const float test_T = T[q] * (1.0f - alpha);
        const unsigned long long termm = okm & __ballot(test_T < GSR_T_EPS);
        const unsigned long long blendm = okm & ~termm;
        const float a_eff = vsel(blendm, alpha, 0.0f);
        const float aT = a_eff * T[q];
        const f2 aT2 = {aT, aT};
        CrCg[q] = __builtin_elementwise_fma(f2{c.x, c.y}, aT2, CrCg[q]);
        CbD[q] = __builtin_elementwise_fma(f2{c.z, c.w}, aT2, CbD[q]);
        if (C2) {
          ErEg[q] = __builtin_elementwise_fma(f2{e.x, e.y}, aT2, ErEg[q]);
          Eb[q] = fmaf(e.z, aT, Eb[q]);
        }
        T[q] = vsel(blendm, test_T, T[q]);
        last[q] = __float_as_uint(vsel(blendm, b.w, __uint_as_float(last[q])));
        dm[q] |= termm;
        hb[q] |= blendm != 0ull ? kbit : 0ull;
        k = kn;
        return rest != 0ull;
      };
      float4 pa = s0[k], pb = s1[k], pc = s2[k];
      float4 pd = C2 ? s3[k] : zero4;
      float4 ya, yb, yc, yd;
      // (a finished quadrant stops its walk, tested every second step: its lanes would blend nothing)
      while (dm[q] != ~0ull && step(pa, pb, pc, pd, ya, yb, yc, yd) && step(ya, yb, yc, yd, pa, pb, pc, pd)) {
      }
    }
    // the backward's cull of this batch: candidate i's 4-bit mask of quadrants it blended in (batches past the last
    // blend are never read by it)
    qbi = qbytes != nullptr && i < n ? i : -1;
    qbv = (uint8_t)(((hb[0] >> lane) & 1ull) | (((hb[1] >> lane) & 1ull) << 1) | (((hb[2] >> lane) & 1ull) << 2) |
                    (((hb[3] >> lane) & 1ull) << 3));
    __syncthreads();
    qactive = active_mask();
  }
  if (qbi >= 0) qbytes[qbi] = qbv;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int px = tx0 + (q & 1) * 8 + (lane & 7), py = ty0 + (q >> 1) * 8 + (lane >> 3);
    if (inside[q]) {
      const size_t pid = (size_t)py * W + px;
      const float Tq = T[q];
      final_T[pid] = Tq;
      n_contrib[pid] = last[q];
      {
#pragma clang fp contract(off)
        out_color[pid] = CrCg[q].x + Tq * bg[0];
        out_color[HWs + pid] = CrCg[q].y + Tq * bg[1];
        out_color[2 * HWs + pid] = CbD[q].x + Tq * bg[2];
      }
      out_depth[pid] = CbD[q].y;
      out_alpha[pid] = 1.0f - Tq;
      if (C2) {
#pragma clang fp contract(off)
        float* o2 = rs.out_col2 + (size_t)(rs.v0 + v) * 3 * HWs + pid;
        o2[0] = ErEg[q].x + Tq * bg[0];
        o2[HWs] = ErEg[q].y + Tq * bg[1];
        o2[2 * HWs] = Eb[q] + Tq * bg[2];
      }
      if (rs.comp != nullptr) {
#pragma clang fp contract(off)
        float p0 = CrCg[q].x + Tq * bg[0], p1 = CrCg[q].y + Tq * bg[1], p2 = CbD[q].x + Tq * bg[2];
        if (rs.cbg != nullptr) {
          const float am = 1.0f - (1.0f - Tq);
          const float* bgi = rs.cbg + ((size_t)v * HWs + pid) * 3;
          p0 = p0 + am * bgi[0];
          p1 = p1 + am * bgi[1];
          p2 = p2 + am * bgi[2];
        }
        float* cp = rs.comp + (size_t)v * 3 * HWs + pid;
        cp[0] = fminf(fmaxf(p0, 0.0f), 1.0f);
        cp[HWs] = fminf(fmaxf(p1, 0.0f), 1.0f);
        cp[2 * HWs] = fminf(fmaxf(p2, 0.0f), 1.0f);
      }
    }
    uint32_t mc = last[q];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mc = max(mc, (uint32_t)__shfl_xor((int)mc, o, 64));
    if (lane == 0) quad_maxc[4 * tile + q] = mc;
  }
#ifdef GSR_TIMELINE
  atomicAdd(&g_pairs[0], pc_eval);  // per-lane values (vector atomics)
  atomicAdd(&g_pairs[1], pc_slot);
#endif
}

// One block per view: bucket its super-tiles by the bit length of their listed instances (sum over the
// 2x2 tiles), heaviest bucket first (LDS counts, exclusive scan, LDS-atomic placement: the order inside a
// bucket may vary between runs — it only changes which workgroup starts first, never a result).
__global__ __launch_bounds__(256) void k_tile_order(int gx, int gy, const uint2* __restrict__ ranges,
                                                    uint32_t* __restrict__ order) {
  __shared__ uint32_t cnt[33], cur[33];
  const int t = threadIdx.x, v = blockIdx.x;
  const int sgx = (gx + 1) >> 1, sgy = (gy + 1) >> 1, S = sgx * sgy;
  ranges += (size_t)v * gx * gy;
  order += (size_t)v * S;
  if (t < 33) cnt[t] = 0u;
  __syncthreads();
  auto bucket = [&](int s) -> int {
    const int x0 = (s % sgx) * 2, y0 = (s / sgx) * 2;
    uint32_t w = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int x = x0 + (k & 1), y = y0 + (k >> 1);
      if (x < gx && y < gy) {
        const uint2 r = ranges[y * gx + x];
        w += r.y - r.x;
      }
    }
    return 32 - (w ? 32 - __clz((int)w) : 0);  // 0 = the most instances (bit length 32) ... 32 = none
  };
  for (int s = t; s < S; s += 256) atomicAdd(&cnt[bucket(s)], 1u);
  __syncthreads();
  if (t == 0) {
    uint32_t run = 0u;
    for (int b = 0; b < 33; ++b) {
      cur[b] = run;
      run += cnt[b];
    }
  }
  __syncthreads();
  for (int s = t; s < S; s += 256) order[atomicAdd(&cur[bucket(s)], 1u)] = (uint32_t)s;
}

void launch_tile_order(int V, int gx, int gy, const uint2* ranges, uint32_t* order, hipStream_t stream) {
  if (V > 0 && gx > 0 && gy > 0) hipLaunchKernelGGL(k_tile_order, dim3(V), dim3(256), 0, stream, gx, gy, ranges, order);
}


// The split backward's chunk sums -> suffix sums (slot k: the colour / depth blended from candidate k CH to
// the quadrant's last blend), in place; one workgroup per tile, a wave per quadrant, slots 1 .. the one
// holding the quadrant's deepest blend (only those were written).  All loads are issued before the sums.
__global__ __launch_bounds__(256) void k_ckpt_suffix(RenderSet rs, const uint32_t* __restrict__ quad_maxc) {
  const int tiles = rs.gx * rs.gy;
  const int v = blockIdx.x / tiles, tile = blockIdx.x % tiles;
  const int t = threadIdx.x, q = t >> 6;
  const size_t vg = (size_t)(rs.v0 + v);
  const int qmaxc = (int)quad_maxc[(vg * tiles + tile) * 4 + q];
  const int cl = qmaxc > 0 ? min(GSR_SPLIT_NCK, (qmaxc - 1) / GSR_SPLIT_CH) : 0;
  if (t == 0) {
    // the tile's chunks after the first (its block_map workgroup replays chunk 0) as backward items
    const uint4 qm = reinterpret_cast<const uint4*>(quad_maxc)[vg * tiles + tile];
    const int maxc = (int)max(max(qm.x, qm.y), max(qm.z, qm.w));
    const int nc = maxc > 0 ? min(GSR_SPLIT_NCK, (maxc - 1) / GSR_SPLIT_CH) : 0;
    // the deepest chunks first: when the list is full, the tile's own workgroup walks the remaining
    // (shallowest) ones, [0, cap), in one contiguous stretch
    uint32_t cap = 0xffffffffu;
    if (nc > 0) {
      const uint32_t at = atomicAdd(rs.split_items, (uint32_t)nc);
      const uint32_t E = (uint32_t)rs.split_extra;
      const int m = (int)min((uint32_t)nc, at < E ? E - at : 0u);
      for (int j = 0; j < m; ++j)
        rs.split_items[1 + at + j] = ((uint32_t)vg << 26) | ((uint32_t)(nc - j) << 22) | (uint32_t)tile;
      if (m > 0) cap = (uint32_t)(nc - m + 1) * GSR_SPLIT_CH;
    }
    rs.split_cap[vg * tiles + tile] = cap;
  }
  if (cl < 2) return;  // (wave-uniform) one chunk behind the first boundary at most: already its sum
  float4* const part = reinterpret_cast<float4*>(rs.ckpt + ckpt_offset(vg, (size_t)tiles, tile, 0) + 256) + t;
  constexpr size_t SL = GSR_CKPT_FIELDS * 256 / 4;  // float4 per slot
  float4 p[GSR_SPLIT_NCK + 1];
#pragma unroll
  for (int j = 1; j <= GSR_SPLIT_NCK; ++j) p[j] = part[(size_t)min(j, cl) * SL];
  float4 acc = p[GSR_SPLIT_NCK];
#pragma unroll
  for (int j = GSR_SPLIT_NCK - 1; j >= 1; --j) {
    if (j < cl) {
      acc = make_float4(p[j].x + acc.x, p[j].y + acc.y, p[j].z + acc.z, p[j].w + acc.w);
      part[(size_t)j * SL] = acc;
    } else if (j == cl) {
      acc = p[j];
    }
  }
}

// Which forward: the tile-wave kernel gathers each candidate once but walks a quadrant's candidates one
// branch at a time and the whole tile list to the tile's deepest termination; it wins when Gaussians span
// several tiles (C3: 6.7 rectangle tiles per Gaussian, render_fwd -3 %), the quadrant-wave kernel when
// they are small (C5 SuGaR, 1.7 tiles per Gaussian: the tile kernel is 1.6x slower).  A launch's duration
// is also bounded by its slowest wave — a heavy tile's whole list for the tile kernel, only a quadrant's
// for the other — which many views hide.  Round 2 (profiles/r02_fwd_kernel_ab.txt) put the C3 crossover at
// 48 views; with round 4's tile kernel (scalar-mask walk, packed pairs) and the backward's cull from its
// masks it is 16 views (C3 views/s, tile vs quadrant: 8 views 2697 vs 2699, 16 views 2991 vs 2968, 32 views
// 3154 vs 3111; profiles/r04/fwd_small_sets_ab.txt).  Both give identical outputs.  GSR_FWD_KERNEL=
// tile|quadrant forces one (A/B and tests).
static bool fwd_tile_kernel(long long instances, long long gaussians, int views) {
  const char* e = getenv("GSR_FWD_KERNEL");
  if (e != nullptr && strcmp(e, "quadrant") == 0) return false;
  if (e != nullptr && strcmp(e, "tile") == 0) return true;
  return views >= 16 && gaussians > 0 && instances >= 3 * gaussians;
}
bool fwd_tile_chosen(long long instances, long long gaussians, int views) {
  return fwd_tile_kernel(instances, gaussians, views);
}
// (Measured and removed, round 4 — the forward's free-running quadrant waves beat every variant that gathers a
// record once per tile, their 5.6x redundant C5 record traffic included, profiles/r04/fwd_shared_ab.txt,
// profiles/r04/tile_wave_ab.txt: the quadrant waves of a tile sharing one staged copy of each batch in LDS with a
// barrier per batch, C5 render_fwd 0.146 -> 0.277 ms/view, 8-view C3 sets 0.052 -> 0.070; one wave per tile
// walking the quadrants in turn, C5 0.142 -> 0.237, C3 0.045 -> 0.066.)

// the blend kernels a launch used (gsr_profile_kernel; rocprofv3's names of them)
static const char* g_blend_kernel[2] = {"", ""};
const char* blend_kernel_name(int which) { return which >= 0 && which < 2 ? g_blend_kernel[which] : ""; }

void launch_render_forward(const RenderSet& rs, const GeomState& g, const uint32_t* sorted_gauss,
                           const ImageState& img, float* out_color, float* out_depth, float* out_alpha,
                           long long instances, hipStream_t stream) {
  const int nt = rs.gx * rs.gy;
  if (nt <= 0 || rs.V <= 0) return;
  if (fwd_tile_kernel(instances, (long long)rs.V * rs.P, rs.V)) {
    const dim3 grid(block_grid(rs, 4));
    g_blend_kernel[0] = rs.col2 != nullptr ? "k_render_fwd_tile<true>" : "k_render_fwd_tile<false>";
    if (rs.col2 != nullptr)
      hipLaunchKernelGGL(k_render_fwd_tile<true>, grid, dim3(64), 0, stream, rs, (const uint2*)img.ranges,
                         sorted_gauss, (const GaussRec*)g.rec, out_color, out_depth, out_alpha, img.final_T,
                         img.n_contrib, img.quad_maxc);
    else
      hipLaunchKernelGGL(k_render_fwd_tile<false>, grid, dim3(64), 0, stream, rs, (const uint2*)img.ranges,
                         sorted_gauss, (const GaussRec*)g.rec, out_color, out_depth, out_alpha, img.final_T,
                         img.n_contrib, img.quad_maxc);
  } else {
    auto kern = rs.col2 != nullptr ? (rs.ckpt != nullptr ? k_render_fwd<true, true> : k_render_fwd<true, false>)
                                   : (rs.ckpt != nullptr ? k_render_fwd<false, true> : k_render_fwd<false, false>);
    g_blend_kernel[0] = rs.col2 != nullptr ? (rs.ckpt != nullptr ? "k_render_fwd<true, true>" : "k_render_fwd<true, false>")
                                           : (rs.ckpt != nullptr ? "k_render_fwd<false, true>" : "k_render_fwd<false, false>");
    hipLaunchKernelGGL(kern, dim3(block_grid(rs, 16)), dim3(64), 0, stream, rs, (const uint2*)img.ranges,
                       sorted_gauss, (const GaussRec*)g.rec, out_color, out_depth, out_alpha, img.final_T,
                       img.n_contrib, img.quad_maxc);
    if (rs.ckpt != nullptr)
      hipLaunchKernelGGL(k_ckpt_suffix, dim3(rs.V * nt), dim3(256), 0, stream, rs, (const uint32_t*)img.quad_maxc);
  }
  hipLaunchKernelGGL(k_tile_info, dim3(rs.V * div_up(nt, 256)), dim3(256), 0, stream, rs,
                     (const uint2*)img.ranges, (const uint32_t*)img.quad_maxc, sorted_gauss,
                     (const GaussRec*)g.rec, img.tile_info, img.cut);
}

// One workgroup's backward of one tile: the whole blended prefix, or with `split` (split_on) chunk `chunk`,
// candidates [chunk CH, (chunk + 1) CH) (chunk GSR_SPLIT_NCK: to the end of the prefix).
__device__ __forceinline__ void bwd_tile(BwdLDS& s, const RenderSet& rs, int v, int tile, int chunk, bool split,
                                         const uint2* __restrict__ ranges, const uint32_t* __restrict__ quad_maxc,
                                         const uint32_t* __restrict__ sorted_gauss, const GaussRec* __restrict__ rec,
                                         const uint32_t* __restrict__ goff, const float* __restrict__ final_Ts,
                                         const uint32_t* __restrict__ n_contrib, const float* __restrict__ dL_dcolor,
                                         const float* __restrict__ dL_ddepth, const float* __restrict__ dL_dalpha,
                                         float4* __restrict__ grow, unsigned long long* __restrict__ reach) {
  constexpr int NG = NGV;               // raw sums per (candidate, quadrant)
  constexpr int QS = GSR_QSUM_STRIDE;    // per candidate
  constexpr int GS = 8;                  // candidates per 16x16 product
  constexpr int NPL = 4;                 // dL/dpixel planes in the B operand
  constexpr int RW = 3;                  // float4 per gradient row
  GSR_TL_BEGIN
  const int W = rs.W, H = rs.H, grid_x = rs.gx;
  const size_t vgs = (size_t)(rs.v0 + v);
  {
    const size_t vg = vgs, tiles = (size_t)rs.gx * rs.gy, HWs = (size_t)W * H;
    ranges += vg * tiles;
    quad_maxc += vg * 4 * tiles;
    sorted_gauss += rs.inst_start[v];
    rec += vg * rs.P;
    goff += vg * rs.P;
    final_Ts += vg * HWs;
    n_contrib += vg * HWs;
    dL_dcolor += (size_t)v * 3 * HWs;
    if (dL_ddepth) dL_ddepth += (size_t)v * HWs;
    if (dL_dalpha) dL_dalpha += (size_t)v * HWs;
    grow += (size_t)RW * rs.row_start[v];
  }
  const float* bg = rs.bg[v];
  int tl_work = 0, tl_max = 0;
  int tl_q[4] = {0, 0, 0, 0};  // per-quadrant kept totals of the tile (the per-tile imbalance bound)
  int tl_staged = 0, tl_any = 0;  // staged candidates / candidates kept by at least one quadrant
  // (the wave's quadrant is wave-uniform: readfirstlane keeps it and what derives from it in scalars)
  const int t = threadIdx.x, q = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
  const int txi = tile % grid_x, tyi = tile / grid_x;
  const int qx0 = txi * GSR_TILE_X + (q & 1) * 8;
  const int qy0 = tyi * GSR_TILE_Y + (q >> 1) * 8;
  const int px = qx0 + (lane & 7), py = qy0 + (lane >> 3);
  const bool inside = px < W && py < H;
  const float pxf = (float)px, pyf = (float)py;
  const uint2 range = ranges[tile];
  const uint4 qm = reinterpret_cast<const uint4*>(quad_maxc)[tile];
  const int qmaxc = (int)(q == 0 ? qm.x : q == 1 ? qm.y : q == 2 ? qm.z : qm.w);
  const int maxc = (int)max(max(qm.x, qm.y), max(qm.z, qm.w));
  // the candidates [lo, hi) of the tile list this workgroup replays
  int lo = 0, hi = maxc;
  if (split) {
    lo = chunk * GSR_SPLIT_CH;
    if (chunk == 0)
      hi = (int)min((uint32_t)maxc, rs.split_cap[vgs * rs.gx * rs.gy + tile]);
    else
      hi = chunk == GSR_SPLIT_NCK ? maxc : min(maxc, lo + GSR_SPLIT_CH);
  }
  lo = __builtin_amdgcn_readfirstlane(lo);  // (workgroup-uniform: scalars)
  hi = __builtin_amdgcn_readfirstlane(hi);
  const size_t pid = (size_t)py * W + px;
  const size_t HW = (size_t)H * W;

  const float T_final = inside ? final_Ts[pid] : 0.0f;
  float T = T_final;
  const uint32_t last_contributor = inside ? n_contrib[pid] : 0u;
  float dpix[3] = {0.f, 0.f, 0.f};
  float dpix_d = 0.f, dpix_a = 0.f;
  if (inside) {
    dpix[0] = dL_dcolor[pid];
    dpix[1] = dL_dcolor[HW + pid];
    dpix[2] = dL_dcolor[2 * HW + pid];
    if (dL_ddepth) dpix_d = dL_ddepth[pid];
    if (dL_dalpha) dpix_a = dL_dalpha[pid];
    if (rs.cbg != nullptr) {
      // fused composite backward: dL/dcomp masked by the clamp -> dL/dcolor, dL/dalpha, dL/dbg
#pragma clang fp contract(off)
      const float am = 1.0f - (1.0f - T_final);
      const float* bgi = rs.cbg + ((size_t)v * HW + pid) * 3;
      const float* col = rs.ccolor + (size_t)v * 3 * HW + pid;
      float da = 0.0f;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        const float b = bgi[ch];
        const float pre = col[(size_t)ch * HW] + am * b;
        const float gch = (pre >= 0.0f && pre <= 1.0f) ? dpix[ch] : 0.0f;
        dpix[ch] = gch;
        da -= gch * b;
        if (rs.dcbg != nullptr && chunk == 0) rs.dcbg[((size_t)v * HW + pid) * 3 + ch] = gch * am;
      }
      dpix_a = da + dpix_a;
    } else if (rs.ccolor != nullptr) {
      // the clamp alone: dL/dclamped masked by the forward's colour
      const float* col = rs.ccolor + (size_t)v * 3 * HW + pid;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        const float pre = col[(size_t)ch * HW];
        dpix[ch] = (pre >= 0.0f && pre <= 1.0f) ? dpix[ch] : 0.0f;
      }
    }
  }
  const float bg_dot = bg_dot3(bg, dpix[0], dpix[1], dpix[2]);

  // The reference keeps per channel the colour accumulated behind the current Gaussian
  // (accum_rec = last_alpha last_c + (1 - last_alpha) accum_rec, deferred by one contributor) and
  // forms dL/dalpha = T sum_ch (c_ch - accum_ch) dL/dpix_ch - T_final / (1 - alpha) bg . dL/dpix.
  // Only the dot product with dL/dpix enters, and the update is linear, so one scalar carries the
  // colour and alpha channels (r, g, b, alpha with c_alpha = 1):
  //   S = sum_ch accum_ch dL/dpix_ch,  cd = sum_ch c_ch dL/dpix_ch,  S <- alpha cd + (1 - alpha) S
  // applied eagerly after each contributor's own dL/dalpha (non-contributors: alpha = 0, identity).
  // The depth channel keeps its own accumulated depth Sd and enters as (depth - Sd) dL/ddepth, the
  // reference's order: the depths of a surface's Gaussians nearly coincide, so folded into S the
  // difference would be taken after the multiplication by dL/ddepth (which reaches ~1e3 through a
  // normal-from-depth loss) and lose its significant bits.
  float S = 0.f, Sd = 0.f;
  const float nbg = -T_final * bg_dot;
  const f2 pxy = {pxf, pyf};
  if (split && hi < maxc && qmaxc > hi) {
    // A chunk that ends before the quadrant's deepest blend starts from the forward's state at candidate
    // hi: T there, and the colour / alpha / depth blended behind it over T (the reference's accum_rec
    // there): the later chunks' own sums (slots up to the one holding the quadrant's last blend)
    const size_t tiles = (size_t)rs.gx * rs.gy;
    const float* ck = rs.ckpt + ckpt_offset(vgs, tiles, tile, hi / GSR_SPLIT_CH);
    const float Th = ck[t];
    const float4 b4 = reinterpret_cast<const float4*>(ck + 256)[t];  // k_ckpt_suffix: all later blends
    const float br = b4.x, bgc = b4.y, bb = b4.z, bd = b4.w;
    const float inv = 1.0f / Th;
    T = Th;
    S = (br * dpix[0] + bgc * dpix[1] + bb * dpix[2]) * inv + (1.0f - T_final * inv) * dpix_a;
    Sd = bd * inv;
  }
  // (uniform: kept in scalar registers, not in vector registers the loop would spill)
  const float ddelx_dx = sgpr_f(0.5f * W), ddely_dy = sgpr_f(0.5f * H);
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);

  // All 256 threads stage the batches: thread t moves 16-byte piece (t & 3) of candidate t >> 2's
  // 64-byte record (4 lanes read one line: coalesced).  Two-stage prefetch: indices two batches
  // ahead, record pieces one ahead.
  const uint32_t gmask = rs.gmask;
  const int cs = t >> 2, piece = t & 3;
  // the list entry (packed keys: the Gaussian index in the low bits) — masked where it is used, not where it is
  // loaded: a use right after the load made the wave wait for every memory operation in flight (the batch's
  // record gathers included) before the staging barrier
  auto fetch_raw = [&](int h) -> uint32_t {
    const int r = h - 1 - cs;
    return r >= 0 ? sorted_gauss[range.x + r] : 0u;
  };
  auto fetch_index = [&](int h) -> uint32_t { return fetch_raw(h) & gmask; };
  float4 npc = zero4;  // the next batch's piece
  uint32_t ngo = 0u;   // piece 3: the Gaussian's first row slot; piece 2: the Gaussian (staged for the reach bit)
  uint32_t gi_next = 0u;
  // this view's reach bit: word v >> 5 of the Gaussian's 64 bits, set for every candidate some quadrant of the tile
  // keeps (k_view_grad walks the rows of exactly the reached (view, Gaussian) pairs; the rows of a staged candidate
  // no quadrant kept are zeros, and a Gaussian no tile kept has only such rows)
  unsigned int* const reach32 = reinterpret_cast<unsigned int*>(reach) + (v >> 5);
  const unsigned int vbit = 1u << (v & 31);
  // the forward's per-instance quadrant cull (ImageState::split_mode[1]): the cull is read, one
  // batch ahead, instead of recomputed (both bounds are conservative: a pair either keeps has no blend beyond
  // the other's, so the sums agree)
  // (layout 1, the tile-wave forward: byte i = the 4-bit mask of instance i; layout 2, the quadrant-wave forward:
  // byte 4 i + q = quadrant q keeps instance i)
  // (split_mode[1] is set by a byte memset: its low byte is the layout)
  const uint32_t qlayout = rs.qbytes != nullptr && rs.split_mode != nullptr ? (rs.split_mode[1] & 0xffu) : 0u;
  const size_t qpos0 = (size_t)rs.inst_start[v] + range.x;
  const uint8_t* const qbm = qlayout == 0u ? nullptr : qlayout == 1u ? rs.qbytes + qpos0 : rs.qbytes + 4 * qpos0 + q;
  const uint32_t qstride = qlayout == 2u ? 4u : 1u, qsh = qlayout == 2u ? 0u : (uint32_t)q;
  uint32_t nqb = 0u;
  if (qbm != nullptr && hi - 1 - lane >= lo) nqb = qbm[qstride * (uint32_t)(hi - 1 - lane)];
  if (hi > lo) {
    const uint32_t g0 = fetch_index(hi);
    if (hi - 1 - cs >= lo) {
#ifdef GSR_EXP_HOTREC  // timing only: the staging gathers from 4096 cache-resident records (wrong results)
      npc = reinterpret_cast<const float4*>(rec + (g0 & 4095u))[piece];
#else
      npc = reinterpret_cast<const float4*>(rec + g0)[piece];
#endif
      if (piece == 2 && rs.col2 != nullptr)  // the second rasterizer call's colours replace the first's
        npc = make_float4(rs.col2[3 * g0], rs.col2[3 * g0 + 1], rs.col2[3 * g0 + 2], 0.f);
      if (piece == 2) ngo = g0;
      if (piece == 3) ngo = goff[g0];
    }
    if (hi - 64 > lo) gi_next = fetch_raw(hi - 64);
  }

  // branch-free replay step; non-contributing lanes run it with alpha = 0 (state unchanged) and
  // contribute zeros.  Returns per pixel u = G dL/dalpha (the mean2D / conic / opacity
  // gradients are linear in u's moments over the pixel offsets) and w = alpha T (the colour / depth
  // weights); the sums over the quadrant's 64 pixels are formed by the matrix cores (below).
  // The replay's running state as packed fp32 pairs (v_pk_mul_f32 / v_pk_fma_f32 issue two lanes' worth at the
  // cost of one): SS = (S, Sd) and TT = (dL/dalpha of the step, T).  Staged record ga = (x, y, B, C), gb = (A,
  // opacity, depth, list position), gc = (r, g, b, ·): the pairs (x, y) and (B, C) are adjacent (the forwards'
  // layout), so the offsets and the exponent's two products are one instruction each.  Every lane's operations
  // are the scalar ones, in the same order: the same bits.
  f2 SS = {S, Sd};
  f2 TT = {0.f, T};
  auto replay = [&](const float4& ga, const float4& gb, const float4& gc, float& u, float& w) {
    const uint32_t rel = __float_as_uint(gb.w);
    const f2 dd = f2{ga.x, ga.y} - pxy;
    const f2 bcp = f2{ga.z, ga.w} * f2{dd.y, dd.y};
    const float power2 = fmaf(dd.x, fmaf(gb.x, dd.x, bcp.x), bcp.y * dd.y);  // gauss_power2: log2(e) * power
    const float G = __builtin_amdgcn_exp2f(power2);
    const float alpha = fminf(GSR_ALPHA_MAX, gb.y * G);
    const bool hit = rel < last_contributor && power2 <= 0.0f && alpha >= GSR_ALPHA_MIN;
    const f2 ga2 = {hit ? G : 0.0f, hit ? alpha : 0.0f};  // (G, alpha) of a contributor, zeros otherwise
    const float a_eff = ga2.y;
    const float oma = 1.f - a_eff;
    const float inv_1ma = fast_rcp(oma);  // 1 for non-contributors
    TT.y = TT.y * inv_1ma;                // T
    const float cd = fmaf(gc.x, dpix[0], fmaf(gc.y, dpix[1], fmaf(gc.z, dpix[2], dpix_a)));
    TT.x = fmaf(TT.y, fmaf(gb.z - SS.y, dpix_d, cd - SS.x), inv_1ma * nbg);  // dL/dalpha
    const f2 uw2 = ga2 * TT;  // u = G dL/dalpha, w = alpha T
    u = uw2.x;
    w = uw2.y;
    const f2 om = f2{oma, oma} * SS;
    SS.x = fmaf(a_eff, cd, om.x);
    SS.y = fmaf(a_eff, gb.z, om.y);
  };


  // Matrix-core reduction.  For a group of 8 candidates c, one 16x16 product over the quadrant's
  // 64 pixels p: A rows 0-7 = u of the candidates, rows 8-15 = their w; B columns 0-5 =
  // F(p) = (1, x, y, x^2, x y, y^2) of the pixel's coordinates relative to the quadrant's centre
  // (x, y in -3.5 .. 3.5, exact in fp32: the flush's conversion to moments about the mean cancels
  // 4x less than with the quadrant's corner as origin — the sums' rounding is what the cancellation
  // amplifies for small Gaussians), columns 6-9 = the
  // pixel's dL/d(r, g, b, depth).  Rows 0-7 x columns 0-5 are the u moments, rows 8-15 x columns
  // 6-9 the colour / depth sums; the other quarters are not used.  16 v_mfma_f32_16x16x4_f32
  // (exact fp32 fma chains, 2 interleaved accumulators for the 40-cycle dependency).
  // Operand maps (16x16x4): lane l holds A[l & 15][k = l >> 4], B[k = l >> 4][l & 15];
  // result lane l: column l & 15, rows 4 (l >> 4) + r.
  // k-step i, k = l >> 4 covers pixel p = 16 k + i: x = (p & 7) - 3.5 = (i & 7) - 3.5 (uniform),
  // y = (p >> 3) - 3.5 = 2 k + (i >> 3) - 3.5, so F = fa[i >> 3] + x (fbb[i >> 3] + x fc).
  const int ncol = lane & 15;
  const bool dcol = ncol >= 6 && ncol < 6 + NPL;
  float fa[2], fbb[2], fc;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float y = (float)(2 * (lane >> 4) + h) - 3.5f;
    fa[h] = ncol == 0 ? 1.f : ncol == 2 ? y : ncol == 5 ? y * y : 0.f;
    fbb[h] = ncol == 1 ? 1.f : ncol == 4 ? y : 0.f;
  }
  fc = ncol == 3 ? 1.f : 0.f;
  // The B operand is the same for every group: bv[i] = D + F for k-step i, kept in registers.  D
  // (other lanes' pixels) goes through LDS once, in the qsum area (first written after the first
  // staging barrier, by which time every wave has read its bv).
  float bv[16];
  {
    float* sdp = s.qsum + q * (NPL * 68 + 16);
    sdp[0 * 68 + lane] = dpix[0];
    sdp[1 * 68 + lane] = dpix[1];
    sdp[2 * 68 + lane] = dpix[2];
    sdp[3 * 68 + lane] = dpix_d;
    if (lane < 16) sdp[NPL * 68 + lane] = 0.f;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const float4* dsrc =
        reinterpret_cast<const float4*>(sdp + (dcol ? (ncol - 6) * 68 + 16 * (lane >> 4) : NPL * 68));
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 d4 = dsrc[k];
      const float dk[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * k + e;
        const float x = (float)(i & 7) - 3.5f;
        // one of the two terms is zero: D for columns 6-9 (zeros row otherwise), F for 0-5
        bv[i] = dk[e] + (fa[i >> 3] + x * (fbb[i >> 3] + x * fc));
      }
    }
  }
  float* uw = s.uw[q];
  // writer side: (slot r, pixel p = lane) -> 16 r + PG(p >> 4) + 4 (((p >> 2) & 3) ^ ((r >> 2) & 3)) + (p & 3),
  // PG = gsr_uw_pg
  int wa[4];
#pragma unroll
  for (int sgrp = 0; sgrp < 4; ++sgrp)
    wa[sgrp] = gsr_uw_pg(lane >> 4) + 4 * (((lane >> 2) & 3) ^ sgrp) + (lane & 3);
  // reader side: chunk k of lane l at 16 (l & 15) + PG(l >> 4) + 4 (k ^ ((l >> 2) & 3))
  const float4* asrc = reinterpret_cast<const float4*>(uw + 16 * (lane & 15) + gsr_uw_pg(lane >> 4));
  const int aswz = (lane >> 2) & 3;
  // result side: lane l holds rows 4 (l >> 4) + r -> candidate mb + r of the group, u (rows 0-7,
  // columns 0-5 used) or w (rows 8-15, columns 6-9 used)
  const int mb = 4 * ((lane >> 4) & 1);
  const bool useful = (lane < 32) ? (ncol < 6) : dcol;
  const int field = ncol;

  uint32_t* mylist = s.list[q];  // per kept candidate: its offset (batch index x QS) in qsum
  float* myq = s.qsum + q * NG;

  // The flush of a batch hb (its candidates [hb - 64, hb)): four threads per candidate (t = 4 c + quadrant): per
  // quadrant, turn the sums over pixel coordinates relative to the quadrant centre into the moments of u over
  // dx = mean - pixel (dx = mx' - x with mx' = mean - quadrant centre); add the 4 quadrants (quad DPP); form the
  // reference's terms
  //   dmean2D = -o (W/2, H/2) (a m1 + b m2, c m2 + b m1), dconic = -o/2 (m3, m4, m5), dopacity = m0
  // as one 16-byte piece of the 48-byte row per thread (piece 3: none).  It runs at the start of the NEXT batch's
  // iteration, before that batch's staging (the same four threads of one wave read candidate cs's entries here and
  // rewrite them there: in order), and its stores are issued right after the staging has waited for the gathers
  // (one in-order vmcnt counts loads and stores: stores issued just after that wait are a whole batch old at the
  // next one, so no wave ever waits for a store it has just issued).
  float4 rowv = zero4;
  float4* rowp = nullptr;
  auto flush = [&](int hb) {
    rowp = nullptr;
#ifdef GSR_EXP_NOFLUSH
    if (hi < 0)
#else
    if (hb - 1 - cs >= lo)
#endif
    {
      int qq = piece;
      asm volatile("" : "+v"(qq));  // (the quadrant centres formed here, not held in vector registers across the loop)
      const float4 ga = s.s0[cs];
      const float4 gb = s.s1[cs];
      constexpr int NM = NGV;
      float m[NM];
#pragma unroll
      for (int i = 0; i < NM; ++i) m[i] = 0.f;
      if ((s.kmask[qq] >> cs) & 1ull) {
        const float* C = s.qsum + cs * QS + NG * qq;
        const float mx = ga.x - ((float)(txi * GSR_TILE_X + (qq & 1) * 8) + 3.5f);
        const float my = ga.y - ((float)(tyi * GSR_TILE_Y + (qq >> 1) * 8) + 3.5f);
        m[0] = C[0];
        m[1] = mx * C[0] - C[1];
        m[2] = my * C[0] - C[2];
        m[3] = mx * (mx * C[0] - 2.f * C[1]) + C[3];
        m[4] = mx * (my * C[0] - C[2]) - my * C[1] + C[4];
        m[5] = my * (my * C[0] - 2.f * C[2]) + C[5];
        m[6] = C[6];
        m[7] = C[7];
        m[8] = C[8];
        m[9] = C[9];
      }
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        m[i] += dpp_f32<0xB1>(m[i]);  // quad_perm [1,0,3,2]
        m[i] += dpp_f32<0x4E>(m[i]);  // quad_perm [2,3,0,1]
      }
      const float o = gb.y;
#ifdef GSR_EXP_COALROWS
      float4* row = grow + RW * ((size_t)blockIdx.x * 64 + cs);  // timing only: coalesced, wrong slots
#else
      float4* row = grow + RW * (size_t)s.slot[cs];
#endif
      // -o (W/2) (a m1 + b m2) etc. with the staged A = -log2e a / 2, B = -log2e b, C = -log2e c / 2
      const float k = o * (1.0f / 1.4426950408889634f);
      if (qq == 0) {
        const float dmx = mean_grad(k, ddelx_dx, gb.x, ga.z, m[1], m[2]);  // (A, B): staged s1.x, s0.z
        const float dmy = mean_grad(k, ddely_dy, ga.w, ga.z, m[2], m[1]);  // (C, B): staged s0.w, s0.z
        rowv = make_float4(dmx, dmy, -0.5f * o * m[3], -0.5f * o * m[4]);
        rowp = row;
      } else if (qq == 1) {
        rowv = make_float4(-0.5f * o * m[5], m[0], m[6], m[7]);
        rowp = row + 1;
      } else if (qq == 2) {
        rowv = make_float4(m[8], m[9], 0.f, 0.f);
        rowp = row + 2;
      }
    }
  };

  // One wait point per batch.  The vector memory counter is one in-order count of loads and stores, and a wait for
  // an operation also waits for every older one; the compiler counts conservatively across the branches of this
  // loop, so a use of a loaded value after new loads or stores were issued waited for those too (the next batch's
  // gathers, the rows just stored).  Here each batch starts with one explicit wait for everything in flight —
  // issued during the previous batch, so done by now — then consumes every loaded value (staging, the cull bits,
  // the list entries) before it issues anything new: the previous batch's row stores, the next batch's gathers,
  // the list entries after them and (after the cull) the next cull bits.
  for (int h = hi; h > lo; h -= 64) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (h != hi) flush(h + 64);  // the previous batch's rows (LDS reads before this batch's staging rewrites them)
    uint32_t qcur;
    asm volatile("v_mov_b32 %0, %1" : "=v"(qcur) : "v"(nqb));  // (a real copy: consumed before new loads)
    const uint32_t gnx = gi_next & gmask;
    // (the quad's conic a from piece 0 and c from piece 1, for the other's staged half)
    const float conic_a = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, npc.z), 0x00, 0xf, 0xf, false));
    const float conic_c = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, npc.x), 0x55, 0xf, 0xf, false));
    {
      const int rel_c = h - 1 - cs;
      // (the candidate's LDS addresses formed here each batch, not held in vector registers across the loop)
      int cst = cs;
      asm volatile("" : "+v"(cst));
      if (rel_c >= lo) {
        // the conic pre-multiplied for gauss_power2, s0 = (x, y, B, C), s1 = (A, opacity, depth, list position):
        // conic a and c come from the quad's other pieces (piece 0 holds (x, y, a, b), piece 1 (c, o, depth, ·))
        if (piece == 0) {
          s.s0[cst] = make_float4(npc.x, npc.y, GSR_CONIC_K_B * npc.w, GSR_CONIC_K_AC * conic_c);
        } else if (piece == 1) {
          s.s1[cst] = make_float4(GSR_CONIC_K_AC * conic_a, npc.y, npc.z, __uint_as_float((uint32_t)rel_c));
        } else if (piece == 2) {
          s.s2[cst] = npc;
          s.gidx[cst] = ngo;  // (the Gaussian, for its reach bit)
        } else {
          const uint32_t dx_ = __float_as_uint(npc.x), dy_ = __float_as_uint(npc.y);
          const int xmin = dx_ & 0xffff, ymin = dx_ >> 16, xmax = dy_ & 0xffff;
          s.slot[cst] = ngo + (uint32_t)((tyi - ymin) * (xmax - xmin) + (txi - xmin));
        }
      }
      if (rowp != nullptr) *rowp = rowv;  // (the previous batch's row piece)
      if (h - 64 > lo) {
        // the next batch's Gaussians (their list entries were loaded a batch ago), then the entries of the batch
        // after it (into the same register)
        if (h - 65 - cs >= lo) {
          // (32-bit byte offsets from the view's scalar base: one VGPR per address, nothing hoisted out of the loop)
#ifdef GSR_EXP_HOTREC
          npc = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(rec) + (((gnx & 4095u) * 4u + piece) << 4));
#else
          npc = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(rec) + ((gnx * 4u + (uint32_t)piece) << 4));
#endif
          if (piece == 2 && rs.col2 != nullptr)
            npc = make_float4(rs.col2[3 * gnx], rs.col2[3 * gnx + 1], rs.col2[3 * gnx + 2], 0.f);
          if (piece == 2) ngo = gnx;  // (before the load below: a select after it would wait for the load)
          if (piece == 3) ngo = goff[gnx];
        }
        if (h - 128 > lo) gi_next = fetch_raw(h - 128);
      }
    }
    __syncthreads();
    // this wave's quadrant: cull the staged batch, list the kept candidates, zero the others' sums
    const int rel_l = h - 1 - lane;
    bool keep = false;
#ifdef GSR_EXP_NOCULL
    if (rel_l >= lo && rel_l < qmaxc) keep = s.s0[lane].x > -1e30f;
#else
    // (every forward records its masks — layout 1 or 2 — whenever a list is non-empty; without them, which no
    // forward of this library leaves, every candidate before the quadrant's deepest blend is replayed: the replay's
    // own alpha tests keep that exact)
    keep = rel_l >= lo && rel_l < qmaxc && (qbm == nullptr || ((qcur >> qsh) & 1u));
#endif
    // the next batch's cull, read after this one's into the same register (a copy at the loop latch waited for
    // every memory operation in flight, the flush's row stores included)
    if (qbm != nullptr && h - 65 - lane >= lo) nqb = qbm[qstride * (uint32_t)(h - 65 - lane)];
    const unsigned long long bal = __ballot(keep);
    const int cnt = __popcll(bal);
    if (lane == 0) s.kmask[q] = bal;  // the flush reads this quadrant's sums of kept candidates only
#ifndef GSR_EXP_NOREACH
    // the reach bits of the kept candidates: with the tile-wave forward's 4-bit masks (layout 1) wave 0 sets one
    // per candidate any quadrant kept (a set mask bit is a blend, which lies below that quadrant's deepest blend);
    // otherwise each wave for its own kept candidates (the same bit, set up to four times)
    if (qlayout == 1u ? (q == 0 && rel_l >= lo && (qcur & 0xfu) != 0u) : keep) {
      uint32_t vb;
      asm volatile("v_mov_b32 %0, %1" : "=v"(vb) : "s"(vbit));  // (moved into a vector register here, not held)
      atomicOr(reach32 + 2 * s.gidx[lane], vb);
    }
#endif
#ifdef GSR_TIMELINE
    if (lane == 0) s.tl_cnt[q] = cnt;
#endif
    if (keep) mylist[mask_rank(bal)] = (uint32_t)lane * (uint32_t)QS;  // (the candidate's row in qsum)
    GSR_WAVE_LDS_ORDER();  // this wave's list is read back by its own lanes
    // kept candidates in groups of 8: replay -> (u, w) rows in LDS -> matrix-core sums.
    // The kept set is the uniform ballot mask: walk it with scalar bit scans, prefetching the next
    // candidate's staged record while the current one is replayed.
    unsigned long long rest = bal;
#ifdef GSR_EXP_NOGROUP
    if (cnt < 0)
#endif
    for (int g0 = 0; g0 < cnt; g0 += GS) {
      const int gn = min(GS, cnt - g0);
      if (gn == GS) {
        // a full group: the 8 replay steps without per-step branches, one basic block, so the independent
        // per-candidate terms (staged-record reads, alpha, exp2, 1 / (1 - alpha)) of later candidates can be
        // scheduled under earlier candidates' dependent updates (same operations, same order per pixel)
        int jj[GS];
#pragma unroll
        for (int c = 0; c < GS; ++c) {
          jj[c] = (int)__builtin_ctzll(rest);
          rest &= rest - 1ull;
        }
        float4 ca = s.s0[jj[0]], cb = s.s1[jj[0]], cc = s.s2[jj[0]];
#pragma unroll
        for (int c = 0; c < GS; ++c) {
          // the next candidate's staged record read ahead of this step (kept ahead by the compiler barrier; none
          // after the last: a read nobody uses still holds registers the matrix-core operands then wait for)
          float4 na, nb, nc;
          if (c + 1 < GS) {
            na = s.s0[jj[c + 1]], nb = s.s1[jj[c + 1]], nc = s.s2[jj[c + 1]];
            asm volatile("" ::: "memory");
          }
          float u, w;
          replay(ca, cb, cc, u, w);
          uw[16 * c + wa[c >> 2]] = u;
          uw[16 * (c + 8) + wa[2 + (c >> 2)]] = w;
          if ((c & (GSR_BWD_OVERLAP - 1)) == GSR_BWD_OVERLAP - 1) __builtin_amdgcn_sched_barrier(0);  // (VGPR budget)
          if (c + 1 < GS) {
            ca = na;
            cb = nb;
            cc = nc;
          }
        }
      } else {
      // the group's last, partial batch of gn < 8 candidates: the same steps, guarded (uniform branches), and no
      // read ahead after the last one (a dead read's registers made the matrix-core operand reads wait for it)
      int jj[GS];
#pragma unroll
      for (int c = 0; c < GS; ++c) {
        jj[c] = (int)__builtin_ctzll(rest | (1ull << 63));
        rest &= rest - 1ull;
      }
      float4 ca = s.s0[jj[0]], cb = s.s1[jj[0]], cc = s.s2[jj[0]];
#pragma unroll
      for (int c = 0; c < GS; ++c) {
        if (c < gn) {
          const bool more = c + 1 < gn;
          float4 na, nb, nc;
          if (more) {
            na = s.s0[jj[c + 1]], nb = s.s1[jj[c + 1]], nc = s.s2[jj[c + 1]];
            asm volatile("" ::: "memory");
          }
          float u, w;
#ifdef GSR_EXP_NOREPLAY
          u = ca.x * pxf;
          w = cb.x * pyf;
#else
          replay(ca, cb, cc, u, w);
#endif
          uw[16 * c + wa[c >> 2]] = u;
          uw[16 * (c + 8) + wa[2 + (c >> 2)]] = w;
          if (more) {
            ca = na;
            cb = nb;
            cc = nc;
          }
        }
      }
      }
      GSR_WAVE_LDS_ORDER();  // the wave reads its own lanes' rows
#ifdef GSR_EXP_NOMFMA
      continue;
#endif
      float av[16];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float4 a4 = asrc[k ^ aswz];
        av[4 * k] = a4.x, av[4 * k + 1] = a4.y, av[4 * k + 2] = a4.z, av[4 * k + 3] = a4.w;
      }
      // the candidates of this lane's 4 result rows (m = mb + r)
      const uint4 jl = *reinterpret_cast<const uint4*>(mylist + g0 + mb);
      typedef float f4 __attribute__((ext_vector_type(4)));
      f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (i & 1)
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[i], acc1, 0, 0, 0);
        else
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[i], acc0, 0, 0, 0);
      }
      // lane l: column ncol, rows 4 (l >> 4) + r; u rows 0-7 (columns 0-5), w rows 8-15 (6-9)
      if (useful) {
        const uint32_t jr[4] = {jl.x, jl.y, jl.z, jl.w};
        if (gn == GS) {
#pragma unroll
          for (int r = 0; r < 4; ++r) myq[jr[r] + (uint32_t)field] = acc0[r] + acc1[r];
        } else {
          // rows past the group's end go to candidate 0's padding word (qsum[QS - 1], never read): no branches
#pragma unroll
          for (int r = 0; r < 4; ++r)
            myq[mb + r < gn ? jr[r] + (uint32_t)field : (uint32_t)(QS - 1 - NG * q)] = acc0[r] + acc1[r];
        }
      }
      GSR_WAVE_LDS_ORDER();  // rows are rewritten by the next group
    }
    __syncthreads();
#ifdef GSR_TIMELINE
    if (t == 0) {
      const int c0 = s.tl_cnt[0], c1 = s.tl_cnt[1], c2 = s.tl_cnt[2], c3 = s.tl_cnt[3];
      tl_work += c0 + c1 + c2 + c3;                                  // kept (candidate, quadrant) pairs
      tl_max += 4 * max(max(c0, c1), max(c2, c3));                  // lockstep cost in pair slots
      tl_q[0] += c0, tl_q[1] += c1, tl_q[2] += c2, tl_q[3] += c3;
      tl_staged += min(h - lo, 64);
      tl_any += __popcll(s.kmask[0] | s.kmask[1] | s.kmask[2] | s.kmask[3]);
    }
#endif
  }
  if (hi > lo) {
    // the last batch's rows
    flush(lo + ((hi - lo - 1) & 63) + 1);
    if (rowp != nullptr) *rowp = rowv;
  }
#ifdef GSR_TIMELINE
  // bwd record: z = sum over batches of 4 x the busiest quadrant's kept count (not HW_ID)
  if (threadIdx.x == 0) {
    atomicAdd(&g_pairs[2], 64ull * (unsigned long long)tl_work);
    atomicAdd(&g_pairs[3], 64ull * (unsigned long long)tl_max);
    // any batch-level scheme still waits for the tile's busiest quadrant: 4 x its total
    atomicAdd(&g_pairs[4], 256ull * (unsigned long long)max(max(tl_q[0], tl_q[1]), max(tl_q[2], tl_q[3])));
    atomicAdd(&g_pairs[5], (unsigned long long)tl_staged);
    atomicAdd(&g_pairs[6], (unsigned long long)tl_any);
  }
  if (threadIdx.x == 0 && blockIdx.x < GSR_TL_MAX)
    g_timeline[1][blockIdx.x] = make_uint4(tl_t0, (uint32_t)__builtin_amdgcn_s_memrealtime(), (uint32_t)tl_max,
                                           ((uint32_t)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 24) |
                                               ((uint32_t)tl_work & 0xffffffu));
#endif
  (void)tl_work;
  (void)tl_max;
  (void)tl_q;
  (void)tl_staged;
  (void)tl_any;
}

// The backward blend: a workgroup per tile (block_map: heaviest first, XCD-aware), after `extra` workgroups
// that replay the split tiles' later chunks (split_on: the items k_ckpt_suffix listed, view << 26 | chunk << 22
// | tile, count in items[0], at most rs.split_extra; a heavy tile's chunks run side by side instead of one
// after the other, its own workgroup walks the chunks not listed, from ImageState::split_cap down).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5, 8))) void k_render_bwd(
    RenderSet rs, const uint2* __restrict__ ranges, const uint32_t* __restrict__ quad_maxc,
    const uint32_t* __restrict__ sorted_gauss, const GaussRec* __restrict__ rec, const uint32_t* __restrict__ goff,
    const float* __restrict__ final_Ts, const uint32_t* __restrict__ n_contrib, const float* __restrict__ dL_dcolor,
    const float* __restrict__ dL_ddepth, const float* __restrict__ dL_dalpha, float4* __restrict__ grow,
    unsigned long long* __restrict__ reach, int extra, const uint32_t* __restrict__ items) {
  __shared__ BwdLDS s;
  static_assert(sizeof(BwdLDS) <= GSR_BWD_LDS_5WG, "backward blend: 5 workgroups per CU");
  int v, tile, chunk = 0;
  // the forward's split decision (ImageState::split_mode): checkpoints and items exist only then
  const bool split = rs.ckpt != nullptr && *rs.split_mode != 0u;
  if ((int)blockIdx.x < extra) {
    if (!split || blockIdx.x >= items[0]) return;
    const uint32_t it = items[1 + blockIdx.x];
    v = (int)(it >> 26) - rs.v0;
    if (v < 0 || v >= rs.V) return;  // another view group's tile
    tile = (int)(it & 0x3fffffu);
    chunk = (int)((it >> 22) & 15u);
  } else {
    int q_unused;
    if (!block_map<4>((int)blockIdx.x - extra, rs, v, tile, q_unused)) return;
  }
  // (workgroup-uniform, loaded from memory: readfirstlane keeps them and the per-tile pointers derived from them in
  // scalar registers)
  v = __builtin_amdgcn_readfirstlane(v);
  tile = __builtin_amdgcn_readfirstlane(tile);
  chunk = __builtin_amdgcn_readfirstlane(chunk);
  bwd_tile(s, rs, v, tile, chunk, split, ranges, quad_maxc, sorted_gauss, rec, goff, final_Ts,
                n_contrib, dL_dcolor, dL_ddepth, dL_dalpha, grow, reach);
}

// Backward with hit-list sums, one wave per 16x16 tile walking the four quadrants in turn (each lane holds the
// same pixel of each quadrant) — the small-Gaussian regime (C5: SuGaR's surface Gaussians blend at ~13 pixels, a
// candidate usually in one quadrant).  A 64-pixel matrix-core product would carry mostly zeros there, and
// lockstep quadrant waves would wait for the busiest quadrant of each batch (2.25 slots per kept pair at C5);
// here a batch costs the sum of its quadrants' kept (candidate, quadrant) pairs and nothing waits on another wave.
// Per batch: lane c stages candidate c's record and its cull against the four quadrants; per quadrant the kept
// candidates are replayed back to front (the replay of k_render_bwd: per pixel the same candidates, order and
// operations); the lanes that blended append (u, u_1, w, pixel) to the wave's hit list; lane c then forms
// candidate c's sums from its hits (moments about the candidate's mean, d = mean - pixel per hit as the reference
// forms it), adds the quadrants as ((q0 + q1) + (q2 + q3)) and writes
// one row per staged candidate.  A full hit list is summed early (each pair's sums are formed once, whenever).
// Two colours (TWO, the SuGaR normal renderer's two rasterizer calls on shared geometry): the replay forms both
// calls' dL/dalpha (the second with its own dL/dpixel and accumulated colour, no depth / alpha terms),
// u_1 = G dL/dalpha_1 and u = u_1 + u_2; 16 sums per candidate: 0-5 the u moments, 6-9 sum w dL/d(r,g,b,depth),
// 10-12 sum u_1 (1, x, y), 13-15 sum w dL/d(r2,g2,b2); 64-byte rows.
#define GSR_HCAP_TW 256
template <bool TWO>
__global__ __launch_bounds__(64) void k_render_bwd_tw(
    RenderSet rs, const uint2* __restrict__ ranges, const uint32_t* __restrict__ quad_maxc,
    const uint32_t* __restrict__ sorted_gauss, const GaussRec* __restrict__ rec, const uint32_t* __restrict__ goff,
    const float* __restrict__ final_Ts, const uint32_t* __restrict__ n_contrib, const float* __restrict__ dL_dcolor,
    const float* __restrict__ dL_ddepth, const float* __restrict__ dL_dalpha, float4* __restrict__ grow,
    unsigned long long* __restrict__ reach) {
  constexpr int NG = TWO ? NGV2 : NGV;  // raw sums per (candidate, quadrant)
  constexpr int NM = TWO ? 15 : NGV;    // moments per candidate
  constexpr int RW = TWO ? 4 : 3;       // float4 per gradient row
  constexpr int NQ = 4;                 // quadrants per wave
  __shared__ float4 s0[65], s1[65], s2[65];
  __shared__ float4 s3[65];  // (b, b2) of the interleaved colours
  __shared__ uint32_t slot[64];
  __shared__ uint32_t list[64];                  // the current quadrant: first hit | hits << 16
  __shared__ float4 hits[GSR_HCAP_TW];            // (u, u_1, w, pixel) of the current quadrant's blends
  __shared__ float4 planes[TWO ? 128 : 64];       // the current quadrant's dL/dpixel per pixel
  int v, tile, q_unused;
  if (!block_map<4>(blockIdx.x, rs, v, tile, q_unused)) return;
  GSR_TL_BEGIN
  const int W = rs.W, H = rs.H, grid_x = rs.gx;
  const size_t vgs = (size_t)(rs.v0 + v);
  const size_t HW = (size_t)H * W;
  {
    const size_t tiles = (size_t)rs.gx * rs.gy;
    ranges += vgs * tiles;
    quad_maxc += vgs * 4 * tiles;
    sorted_gauss += rs.inst_start[v];
    rec += vgs * rs.P;
    goff += vgs * rs.P;
    final_Ts += vgs * HW;
    n_contrib += vgs * HW;
    dL_dcolor += (size_t)v * 3 * HW;
    if (dL_ddepth) dL_ddepth += (size_t)v * HW;
    if (dL_dalpha) dL_dalpha += (size_t)v * HW;
    grow += (size_t)RW * rs.row_start[v];
  }
  const float* bg = rs.bg[v];
  const int lane = threadIdx.x & 63;
  constexpr int qb = 0;  // (the wave's first quadrant)
  const int txi = tile % grid_x, tyi = tile / grid_x;
  const uint2 range = ranges[tile];
  const uint4 qm = reinterpret_cast<const uint4*>(quad_maxc)[tile];
  const int qmaxc[4] = {(int)qm.x, (int)qm.y, (int)qm.z, (int)qm.w};
  const int hi = __builtin_amdgcn_readfirstlane((int)max(max(qm.x, qm.y), max(qm.z, qm.w)));
  const int lo = 0;

  // per pixel (one per quadrant of this wave) the replay state and the pixel's upstream gradients, the two colours'
  // terms packed in pairs for v_pk_*_f32 (two exact operations per instruction): de_k = (dL/dpix_k, dL/dpix2_k),
  // dpa0 = (dL/dalpha term, -0: the second colour's chain starts with a product, fma(x, y, -0) = x y exactly),
  // nbgs = the two background terms, SS2 = (S, S2)
  float T[NQ], Sd[NQ], dpd[NQ];
  f2 de0[NQ], de1[NQ], de2[NQ], dpa0[NQ], nbgs[NQ], SS2[NQ];
  uint32_t last[NQ];
  const float lxf = (float)(txi * GSR_TILE_X + (lane & 7)), lyf = (float)(tyi * GSR_TILE_Y + (lane >> 3));
#pragma unroll
  for (int j = 0; j < NQ; ++j) {
    const int q = qb + j;
    const int px = txi * GSR_TILE_X + (q & 1) * 8 + (lane & 7), py = tyi * GSR_TILE_Y + (q >> 1) * 8 + (lane >> 3);
    const bool inside = px < W && py < H;
    const size_t pid = (size_t)py * W + px;
    const float T_final = inside ? final_Ts[pid] : 0.0f;
    T[j] = T_final;
    last[j] = inside ? n_contrib[pid] : 0u;
    float d[3] = {0.f, 0.f, 0.f};
    float dd = 0.f, da = 0.f;
    if (inside) {
      d[0] = dL_dcolor[pid];
      d[1] = dL_dcolor[HW + pid];
      d[2] = dL_dcolor[2 * HW + pid];
      if (dL_ddepth) dd = dL_ddepth[pid];
      if (dL_dalpha) da = dL_dalpha[pid];
      if (rs.cbg != nullptr) {
#pragma clang fp contract(off)
        const float am = 1.0f - (1.0f - T_final);
        const float* bgi = rs.cbg + ((size_t)v * HW + pid) * 3;
        const float* col = rs.ccolor + (size_t)v * 3 * HW + pid;
        float dsum = 0.0f;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
          const float b = bgi[ch];
          const float pre = col[(size_t)ch * HW] + am * b;
          const float gch = (pre >= 0.0f && pre <= 1.0f) ? d[ch] : 0.0f;
          d[ch] = gch;
          dsum -= gch * b;
          if (rs.dcbg != nullptr) rs.dcbg[((size_t)v * HW + pid) * 3 + ch] = gch * am;
        }
        da = dsum + da;
      } else if (rs.ccolor != nullptr) {
        // the clamp alone: dL/dclamped masked by the forward's colour
        const float* col = rs.ccolor + (size_t)v * 3 * HW + pid;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
          const float pre = col[(size_t)ch * HW];
          d[ch] = (pre >= 0.0f && pre <= 1.0f) ? d[ch] : 0.0f;
        }
      }
    }
    float e[3] = {0.f, 0.f, 0.f};
    if (TWO && inside) {
      const float* d2 = rs.dpix2 + (size_t)v * 3 * HW;
      e[0] = d2[pid];
      e[1] = d2[HW + pid];
      e[2] = d2[2 * HW + pid];
    }
    de0[j] = f2{d[0], e[0]};
    de1[j] = f2{d[1], e[1]};
    de2[j] = f2{d[2], e[2]};
    dpd[j] = dd;
    dpa0[j] = f2{da, -0.0f};
    nbgs[j] = f2{-T_final * bg_dot3(bg, d[0], d[1], d[2]), TWO ? -T_final * bg_dot3(bg, e[0], e[1], e[2]) : 0.f};
    SS2[j] = f2{0.f, 0.f};
    Sd[j] = 0.f;
  }
  const float ddelx_dx = 0.5f * W, ddely_dy = 0.5f * H;
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);

  // lane c stages candidate c (list position h - 1 - c) of each batch, one batch ahead; indices two batches
  // ahead: rec.a, rec.b (the cull), rec.d + the row slot, rec.c and the second colour.
  const uint32_t gmask = rs.gmask;
  unsigned int* const reach32 = reinterpret_cast<unsigned int*>(reach) + (v >> 5);
  const unsigned int vbit = 1u << (v & 31);
  float4 na = zero4, nb = zero4, nc = zero4, nd = zero4, n2 = zero4;
  uint32_t ngo = 0u, gi_next = 0u, ng = 0u;
  const bool emb = col2_embedded(rs);  // the second colours in the records (b.w, c.w, d.z): no gather of col2
  auto load = [&](uint32_t g) {
    const float4* r = reinterpret_cast<const float4*>(rec + g);
    {
      na = r[0];
      nb = r[1];
      nd = r[3];
      ngo = goff[g];
      ng = g;  // (its reach bit is set at the staging, once the cull is known)
    }
    {
      nc = r[2];
      if (rs.col2 != nullptr && !(TWO && emb)) {  // (embedded: the record's b.w, c.w, d.z, read at the staging)
        const float4 c2 = make_float4(rs.col2[3 * g], rs.col2[3 * g + 1], rs.col2[3 * g + 2], 0.f);
        if (TWO)
          n2 = c2;
        else  // the second rasterizer call's colours replace the first's
          nc = c2;
      }
    }
  };
  // The cull is read, not recomputed: the forward's exact masks when it recorded them (ImageState::split_mode[1];
  // layout 1, the tile-wave forward: byte i = the 4-bit mask of the quadrants instance i blended in; layout 2, the
  // quadrant-wave forward: byte 4 i + q = quadrant q blended instance i — a pair the forward blended nowhere has no
  // backward hit), else the quadrant masks the keys carry (TilePack::qmask, conservative).
  const uint32_t qlayout = rs.qbytes != nullptr && rs.split_mode != nullptr ? (rs.split_mode[1] & 0xffu) : 0u;
  const uint8_t* const qbm = qlayout != 0u ? rs.qbytes + (qlayout == 2u ? 4 : 1) * ((size_t)rs.inst_start[v] + range.x)
                                           : nullptr;
  const uint32_t* qkeys = qbm == nullptr && rs.qkeys ? rs.qkeys + rs.inst_start[v] + range.x : nullptr;
  // (loaded raw, decoded where used: a use right after the load would wait for every memory operation in flight)
  auto cull_raw = [&](int pos) -> uint32_t {
    if (qlayout == 2u) return reinterpret_cast<const uint32_t*>(qbm)[pos];  // bytes q0..q3, each 0 or 1
    if (qlayout == 1u) return qbm[pos];
    return qkeys[pos];
  };
  auto cull_decode = [&](uint32_t b) -> uint32_t {
    if (qlayout == 2u) return (b & 1u) | ((b >> 7) & 2u) | ((b >> 14) & 4u) | ((b >> 21) & 8u);
    if (qlayout == 1u) return b;
    return b >> GSR_QMASK_SHIFT;
  };
  const bool masks = qbm != nullptr || qkeys != nullptr;
  uint32_t nqm = 0u, qm_next = 0u;  // the mask of the staged-next candidate / the raw mask word of gi_next
  if (hi > lo) {
    if (hi - 1 - lane >= lo) {
      load(sorted_gauss[range.x + hi - 1 - lane] & gmask);
      if (masks) nqm = cull_decode(cull_raw(hi - 1 - lane));
    }
    if (hi - 64 > lo) {
      gi_next = sorted_gauss[range.x + max(hi - 65 - lane, lo)];  // (raw: masked where used)
      if (masks) qm_next = cull_raw(max(hi - 65 - lane, lo));
    }
  }

  // hit-list sums of one (candidate, quadrant) pair -> moments about the candidate's mean (the flush of
  // k_render_bwd); acc = q0 + q1, accb = q2 + q3
  float acc[NM], accb[NM];
  // The u moments are taken directly about the mean, per hit d = mean - pixel as the reference forms it: SuGaR's
  // Gaussians blend a few pixels, often away from the quadrant's centre, where moments about the centre turned into
  // moments about the mean cancel to a few bits (the scale gradients of flat Gaussians amplify that).
  auto pair_moments = [&](const int qq, const uint32_t e, float (&m)[NM]) {
    const int st = (int)(e & 0xffffu), n = (int)(e >> 16);
    const float4 ga = s0[lane];
    const float qx0 = (float)(txi * GSR_TILE_X + (qq & 1) * 8), qy0 = (float)(tyi * GSR_TILE_Y + (qq >> 1) * 8);
    float C[NG];
#pragma unroll
    for (int f = 0; f < NG; ++f) C[f] = 0.f;
    for (int k = st; k < st + n; ++k) {
      const float4 hv = hits[k];
      const uint32_t p = __float_as_uint(hv.w);
      const float dx = ga.x - (qx0 + (float)(p & 7u)), dy = ga.y - (qy0 + (float)(p >> 3));
      const float u = hv.x, w = hv.z;
      C[0] += u;
      C[1] = fmaf(u, dx, C[1]);
      C[2] = fmaf(u, dy, C[2]);
      C[3] = fmaf(u, dx * dx, C[3]);
      C[4] = fmaf(u, dx * dy, C[4]);
      C[5] = fmaf(u, dy * dy, C[5]);
      const float4 d = planes[TWO ? 2 * p : p];
      C[6] = fmaf(w, d.x, C[6]);
      C[7] = fmaf(w, d.y, C[7]);
      C[8] = fmaf(w, d.z, C[8]);
      C[9] = fmaf(w, d.w, C[9]);
      if constexpr (TWO) {
        const float u1 = hv.y;
        const float4 d2 = planes[2 * p + 1];
        C[10 % NG] += u1;
        C[11 % NG] = fmaf(u1, dx, C[11 % NG]);
        C[12 % NG] = fmaf(u1, dy, C[12 % NG]);
        C[13 % NG] = fmaf(w, d2.x, C[13 % NG]);
        C[14 % NG] = fmaf(w, d2.y, C[14 % NG]);
        C[15 % NG] = fmaf(w, d2.z, C[15 % NG]);
      }
    }
#pragma unroll
    for (int f = 0; f < 10; ++f) m[f] = C[f];
    if (TWO) {
      m[10 % NM] = C[11 % NG];
      m[11 % NM] = C[12 % NG];
      m[12 % NM] = C[13 % NG];
      m[13 % NM] = C[14 % NG];
      m[14 % NM] = C[15 % NG];
    }
  };
  // the pending pairs of this wave's quadrant j (lanes whose bit is set) into the running total
  auto flush = [&](const int j, const unsigned long long pend) {
    if (!((pend >> lane) & 1ull)) return;
    float m[NM];
    pair_moments(qb + j, list[lane], m);
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      if (j == 0) acc[i] = m[i];
      else if (j == 1) acc[i] = acc[i] + m[i];
      else if (j == 2) accb[i] = m[i];
      else accb[i] = accb[i] + m[i];
    }
  };

  // The previous batch's row: ((q0 + q1) + (q2 + q3)) per moment, then the reference's terms (k_render_bwd's flush),
  // written at the start of the next batch (before its staging rewrites the staged record and slot).
  // (computed from the staged record and slot before the next staging rewrites them; stored after that staging)
  float4 rv[RW];
  uint32_t rslot = 0u;
  auto make_row = [&]() {
    float m[NM];
#pragma unroll
    for (int i = 0; i < NM; ++i) m[i] = acc[i] + accb[i];
    const float4 ga = s0[lane];
    const float4 gb = s1[lane];
    const float o = gb.y;
    rslot = slot[lane];
    const float k = o * (1.0f / 1.4426950408889634f);
    {
      // (A = gb.x, B = ga.z, C = ga.w in this kernel's staging)
      const float dmx = mean_grad(k, ddelx_dx, gb.x, ga.z, m[1], m[2]);
      const float dmy = mean_grad(k, ddely_dy, ga.w, ga.z, m[2], m[1]);
      rv[0] = make_float4(dmx, dmy, -0.5f * o * m[3], -0.5f * o * m[4]);
    }
    rv[1] = make_float4(-0.5f * o * m[5], m[0], m[6], m[7]);
    rv[2] = TWO ? make_float4(m[8], m[9], m[12 % NM], m[13 % NM]) : make_float4(m[8], m[9], 0.f, 0.f);
    if (TWO) {
      const float dmx1 = mean_grad(k, ddelx_dx, gb.x, ga.z, m[10 % NM], m[11 % NM]);
      const float dmy1 = mean_grad(k, ddely_dy, ga.w, ga.z, m[11 % NM], m[10 % NM]);
      rv[RW - 1] = make_float4(m[14 % NM], dmx1, dmy1, 0.f);
    }
  };
  auto store_row = [&]() {
    float4* row = grow + RW * (size_t)rslot;
#pragma unroll
    for (int i = 0; i < RW; ++i) row[i] = rv[i];
  };
  // One wait point per batch (as k_render_bwd): everything in flight was issued during the previous batch; every
  // loaded value is consumed before anything new is issued (a memory operation issued ahead of a use of an earlier
  // load, in a branch some lanes skip, turns the compiler's wait for that load into a wait for everything).
  for (int h = hi; h > lo; h -= 64) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const bool row_pending = h != hi && h + 63 - lane >= lo;  // (the previous batch staged this lane)
    if (row_pending) make_row();
    // the loaded record, copied out of the load registers here (the staging packs it into LDS tuples; packing the
    // load registers themselves had the compiler copy them at the loop end, right after the loads, waiting on them)
    const float4 ca = make_float4(vcopy(na.x), vcopy(na.y), vcopy(na.z), vcopy(na.w));
    const float4 cb = make_float4(vcopy(nb.x), vcopy(nb.y), vcopy(nb.z), 0.f);
    const float4 cc = make_float4(vcopy(nc.x), vcopy(nc.y), vcopy(nc.z), 0.f);
    const float4 c2 = !TWO ? zero4
                      : emb ? make_float4(vcopy(nb.w), vcopy(nc.w), vcopy(nd.z), 0.f)
                            : make_float4(vcopy(n2.x), vcopy(n2.y), vcopy(n2.z), 0.f);
    const uint32_t cdx = __float_as_uint(vcopy(nd.x)), cdy = __float_as_uint(vcopy(nd.y));
    const uint32_t cgo = __float_as_uint(vcopy(__uint_as_float(ngo)));
    const int rel_c = h - 1 - lane;
    const bool staged = rel_c >= lo;
    uint32_t keep4 = 0u;
    if (staged) {
      // the pre-multiplied conic as s0 = (x, y, B, C), s1 = (A, opacity, depth, list position): the products the
      // step packs are adjacent; row slot
      s0[lane] = make_float4(ca.x, ca.y, GSR_CONIC_K_B * ca.w, GSR_CONIC_K_AC * cb.x);
      s1[lane] = make_float4(GSR_CONIC_K_AC * ca.z, cb.y, cb.z, __uint_as_float((uint32_t)rel_c));
      const int xmin = cdx & 0xffff, ymin = cdx >> 16, xmax = cdy & 0xffff;
      slot[lane] = cgo + (uint32_t)((tyi - ymin) * (xmax - xmin) + (txi - xmin));
      if (masks) {
#pragma unroll
        for (int q = 0; q < 4; ++q) keep4 |= rel_c < qmaxc[q] ? nqm & (1u << q) : 0u;
      } else {
        // the (padded, conservative) cull on the record's conic
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (rel_c < qmaxc[q] &&
              quadrant_hit(ca, cb, (float)(txi * GSR_TILE_X + (q & 1) * 8), (float)(tyi * GSR_TILE_Y + (q >> 1) * 8)))
            keep4 |= 1u << q;
      }
    }
    if (staged) {
      // colours interleaved with the second colours (zeros for one colour): (r, r2, g, g2), (b, b2)
      s2[lane] = make_float4(cc.x, c2.x, cc.y, c2.y);
      s3[lane] = make_float4(cc.z, c2.z, 0.f, 0.f);
    }
    // (the next batch's record index and cull, from values loaded a batch ago: formed here, not where used)
    uint32_t g_next = gi_next & gmask;
    nqm = cull_decode(qm_next);
    asm volatile("" : "+v"(g_next), "+v"(nqm)::"memory");
#ifndef GSR_EXP_NOREACH
    // the reach bit of a candidate some quadrant keeps (k_view_grad / k_gauss_fused walk exactly the reached pairs;
    // a staged candidate no quadrant keeps gets a zero row)
    if (staged && keep4 != 0u) atomicOr(reach32 + 2 * ng, vbit);
#endif
    if (row_pending) store_row();
    // the next batch's records and the one after's indices: every lane loads (positions clamped into the list, an
    // unstaged lane's record is never read) so the loaded values replace the registers without merges
    if (h - 64 > lo) {
      load(g_next);
      const int pn = max(h - 129 - lane, lo);
      gi_next = sorted_gauss[range.x + pn];
      if (masks) qm_next = cull_raw(pn);
    }
#pragma unroll
    for (int i = 0; i < NM; ++i) acc[i] = 0.f;
#pragma unroll
    for (int i = 0; i < NM; ++i) accb[i] = 0.f;
    __syncthreads();  // (the staging of every wave before any wave's reads)
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int q = qb + j;
      const unsigned long long kq = __ballot((keep4 >> q) & 1u);
      if (kq == 0ull) continue;
      // this quadrant's dL/dpixel planes for the sums
      planes[TWO ? 2 * lane : lane] = make_float4(de0[j].x, de1[j].x, de2[j].x, dpd[j]);
      if (TWO) planes[2 * lane + 1] = make_float4(de0[j].y, de1[j].y, de2[j].y, 0.f);
      const f2 pxy = {lxf + (float)((q & 1) * 8), lyf + (float)((q >> 1) * 8)};
      int fill = 0;
      unsigned long long pend = 0ull, rest = kq;
      // candidate records in two register sets used in turn (the loop body twice, roles swapped: no register
      // copies between steps); each step reads the next candidate's into the other set
      int jc = (int)__builtin_ctzll(rest);
      float4 pa = s0[jc], pb = s1[jc], pc = s2[jc];
      float4 pd = s3[jc];
      float4 ya, yb, yc, yd;
      auto step = [&](const float4& ga, const float4& gb, const float4& gc, const float4& gd, float4& xa, float4& xb,
                      float4& xc, float4& xd) -> bool {
        rest &= rest - 1ull;
        const int jn = rest != 0ull ? (int)__builtin_ctzll(rest) : jc;
        xa = s0[jn], xb = s1[jn], xc = s2[jn];
        xd = s3[jn];
        // the replay step of k_render_bwd (replay / replay2) on this quadrant's pixel, in packed pairs
        const uint32_t rel = __float_as_uint(gb.w);
        const f2 dd = f2{ga.x, ga.y} - pxy;
        const f2 bc = f2{ga.z, ga.w} * f2{dd.y, dd.y};
        const float power2 = fmaf(dd.x, fmaf(gb.x, dd.x, bc.x), bc.y * dd.y);  // gauss_power2(A, B, C, dx, dy)
        const float G = __builtin_amdgcn_exp2f(power2);
        const float alpha = fminf(GSR_ALPHA_MAX, gb.y * G);
        // (the step's blend condition as a uniform lane mask: the selects read it directly)
        const unsigned long long hm = (__ballot(rel < last[j]) & __ballot(power2 <= 0.0f)) & __ballot(alpha >= GSR_ALPHA_MIN);
        const bool hit = (hm >> lane) & 1ull;
        const float a_eff = vsel(hm, alpha, 0.0f);
        const float g_eff = vsel(hm, G, 0.0f);
        const float oma = 1.f - a_eff;
        const float inv_1ma = fast_rcp(oma);
        T[j] = T[j] * inv_1ma;
        // (cd, cd2): cd = fma(r, d0, fma(g, d1, fma(b, d2, dpa))), cd2 = fma(r2, e0, fma(g2, e1, b2 e2))
        f2 cdp = __builtin_elementwise_fma(f2{gd.x, gd.y}, de2[j], dpa0[j]);
        cdp = __builtin_elementwise_fma(f2{gc.z, gc.w}, de1[j], cdp);
        cdp = __builtin_elementwise_fma(f2{gc.x, gc.y}, de0[j], cdp);
        const f2 dif = cdp - SS2[j];                            // (cd - S, cd2 - S2)
        const f2 ibg = f2{inv_1ma, inv_1ma} * nbgs[j];          // (inv nbg, inv nbg2)
        float u, u1 = 0.f;
        if (TWO) {
          u1 = g_eff * fmaf(T[j], fmaf(gb.z - Sd[j], dpd[j], dif.x), ibg.x);
          u = fmaf(g_eff, fmaf(T[j], dif.y, ibg.y), u1);
        } else {
          u = g_eff * fmaf(T[j], fmaf(gb.z - Sd[j], dpd[j], dif.x), ibg.x);
        }
        const float w = a_eff * T[j];
        SS2[j] = __builtin_elementwise_fma(f2{a_eff, a_eff}, cdp, f2{oma, oma} * SS2[j]);  // (S, S2)
        Sd[j] = fmaf(a_eff, gb.z, oma * Sd[j]);
        const int n = __popcll(hm);
        if (fill + n > GSR_HCAP_TW) {
          // list full: the finished pairs' sums now, then start over (this wave's own LDS: in-order)
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          flush(j, pend);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          fill = 0;
          pend = 0ull;
        }
        if (hit) hits[fill + (int)mask_rank(hm)] = make_float4(u, u1, w, __uint_as_float((uint32_t)lane));
        if (lane == 0) list[jc] = (uint32_t)fill | ((uint32_t)n << 16);
        fill += n;
        pend |= 1ull << jc;
        if (rest == 0ull) return false;
        jc = jn;
        return true;
      };
      while (step(pa, pb, pc, pd, ya, yb, yc, yd) && step(ya, yb, yc, yd, pa, pb, pc, pd)) {
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      flush(j, pend);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (hits, list and planes are rewritten next)
    }
    __syncthreads();  // (the staged batch is rewritten next)
  }
  // (the last batch's rows)
  if (hi > lo && lo + ((hi - lo - 1) & 63) - lane >= lo) {
    make_row();
    store_row();
  }
  GSR_TL_END(1, hi)
}

// The backward blend kernel of a launch: the two-colour backward (the SuGaR normal renderer's two calls in one
// replay, C5) walks each tile's quadrants in turn on one wave with hit-list sums (k_render_bwd_tw); every other
// backward runs the workgroup of four lockstep quadrant waves with the matrix-core sums (k_render_bwd).
// (Measured and removed, round 4-5 — profiles/r04/tile_wave_ab.txt, tw_waves_ab.txt: the matrix-core tile wave at
// C3, 0.098 -> 0.102 ms/view, 8-view sets 0.104 -> 0.119; the hit-list tile kernel with two waves per tile, C5
// 0.3275 -> 0.3489; the lockstep workgroup with hit-list sums, C5 0.397 vs 0.329.)
void launch_render_backward(const RenderSet& rs, const GeomState& g, const uint32_t* sorted_gauss,
                            const ImageState& img, const float* dL_dcolor, const float* dL_ddepth,
                            const float* dL_dalpha, const BackwardState& bw, hipStream_t stream) {
  const int nt = rs.gx * rs.gy;
  if (nt <= 0 || rs.V <= 0) return;
  // split tiles' later chunks: a workgroup per listed item (C3 per view: ~800 items)
  const bool split = rs.ckpt != nullptr && rs.dpix2 == nullptr && rs.col2 == nullptr;  // (one colour only)
  const int extra = split ? rs.split_extra : 0;  // (the count k_ckpt_suffix lists at most)
  const dim3 grid(block_grid(rs, 4) + extra);
  const uint32_t* items = split ? img.split_items : nullptr;
  if (rs.dpix2 != nullptr) {
    g_blend_kernel[1] = "k_render_bwd_tw<true>";
    hipLaunchKernelGGL(k_render_bwd_tw<true>, dim3(block_grid(rs, 4)), dim3(64), 0, stream, rs,
                       (const uint2*)img.ranges, (const uint32_t*)img.quad_maxc, sorted_gauss, (const GaussRec*)g.rec,
                       (const uint32_t*)g.goff, (const float*)img.final_T, (const uint32_t*)img.n_contrib, dL_dcolor,
                       dL_ddepth, dL_dalpha, bw.grow, bw.reach);
    return;
  }
  g_blend_kernel[1] = "k_render_bwd";
  hipLaunchKernelGGL(k_render_bwd, grid, dim3(256), 0, stream, rs, (const uint2*)img.ranges,
                     (const uint32_t*)img.quad_maxc, sorted_gauss, (const GaussRec*)g.rec, (const uint32_t*)g.goff,
                     (const float*)img.final_T, (const uint32_t*)img.n_contrib, dL_dcolor, dL_ddepth, dL_dalpha,
                     bw.grow, bw.reach, extra, items);
}

// Split backward for launches of few tiles (split_fits): such a launch lasts as long as its deepest tile's
// backward (one workgroup walks the whole blended prefix), so the forward keeps each pixel's state every
// GSR_SPLIT_CH candidates and the backward replays the chunks in parallel.  Only the quadrant-wave forward
// writes the states.  GSR_BWD_SPLIT=0 turns it off (A/B).
bool split_on(int V, int P, int width, int height, long long instances) {
  const size_t tiles = (size_t)div_up(width, GSR_TILE_X) * div_up(height, GSR_TILE_Y);
  if (!split_fits(V, tiles)) return false;
  const char* e = getenv("GSR_BWD_SPLIT");
  if (e != nullptr && strcmp(e, "0") == 0) return false;
  return !fwd_tile_kernel(instances, (long long)V * P, V);
}

}  // namespace gsr

#ifdef GSR_TIMELINE
// diagnostic build only: read (and optionally reset) the pair counters (7 x u64, see g_pairs)
extern "C" int gsr_diag_pairs(void* host, int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(gsr::g_pairs), 7 * sizeof(unsigned long long), 0,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  if (reset) {
    const unsigned long long z[7] = {0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(gsr::g_pairs), z, sizeof(z), 0, hipMemcpyHostToDevice) != hipSuccess) return -1;
  }
  return 0;
}
extern "C" int gsr_diag_timeline(int which, void* host, int n) {
  if (which < 0 || which > 1 || n > GSR_TL_MAX) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(gsr::g_timeline), sizeof(uint4) * n,
                          sizeof(uint4) * GSR_TL_MAX * which, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return 0;
}
#endif

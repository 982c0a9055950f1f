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
#include "gsr_kernels.h"
#include "gsr_wave.h"

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

__host__ __device__ __forceinline__ int unit_grid(int gx, int gy) {
  const int S = ((gx + 1) >> 1) * ((gy + 1) >> 1);
  return 128 * ((S + 7) >> 3);
}
__device__ __forceinline__ bool unit_of_block(int b, int gx, int gy, int& tile, int& q) {
  const int sgx = (gx + 1) >> 1, sgy = (gy + 1) >> 1;
  const int x = b & 7, k = b >> 3;
  const int s = ((k >> 4) << 3) + x;
  const int w = k & 15;
  if (s >= sgx * sgy) return false;
  const int tx = (s % sgx) * 2 + ((w >> 2) & 1), ty = (s / sgx) * 2 + (w >> 3);
  if (tx >= gx || ty >= gy) return false;
  tile = ty * gx + tx;
  q = w & 3;
  return true;
}

__device__ __forceinline__ void tile_pixel(int t, int& lx, int& ly) {
  const int w = t >> 6, l = t & 63;
  lx = ((w & 1) << 3) | (l & 7);
  ly = ((w >> 1) << 3) | (l >> 3);
}

// Can some pixel centre of the 8x8 quadrant with origin (qx, qy) reach alpha >= 1/255 for this
// Gaussian?  alpha = o exp(-q/2), q = a dx^2 + 2 b dx dy + c dy^2 (dx = mean - pixel), so the pair
// can blend only if q <= 2 ln(255 o).  The test takes the exact minimum of q over the continuous
// rectangle spanned by the quadrant's pixel centres (<= the minimum over the pixels themselves) and
// compares it with a padded threshold, so it never drops a pair the reference would blend; for
// rotated, elongated footprints it is much tighter than the ellipse's bounding box.
__device__ __forceinline__ float quad_form(float a, float b, float c, float u, float v) {
  return fmaf(a * u, u, fmaf(2.0f * b * u, v, c * v * v));
}
__device__ __forceinline__ bool quadrant_hit(const float4 r0, const float4 r1, float qx, float qy) {
  const float o = r1.y;
  if (!(o >= GSR_ALPHA_MIN * 0.9999f)) return false;
  const float a = r0.z, b = r0.w, c = r1.x;
  if (!(a > 0.0f && c > 0.0f && a * c - b * b > 0.0f)) return true;
  const float tau = fmaxf(0.0f, __logf(255.0f * o));
  const float thr = 2.0f * (tau * 1.002f + 2e-3f);
  // dx ranges over [u0, u1], dy over [v0, v1]
  const float u1 = r0.x - qx, u0 = u1 - 7.0f;
  const float v1 = r0.y - qy, v0 = v1 - 7.0f;
  if (u0 <= 0.0f && u1 >= 0.0f && v0 <= 0.0f && v1 >= 0.0f) return true;
  const float ia = 1.0f / a, ic = 1.0f / c;
  // edges u = u0, u1: best v = clamp(-b u / c); edges v = v0, v1: best u = clamp(-b v / a)
  const float q0 = quad_form(a, b, c, u0, fminf(fmaxf(-b * u0 * ic, v0), v1));
  const float q1 = quad_form(a, b, c, u1, fminf(fmaxf(-b * u1 * ic, v0), v1));
  const float q2 = quad_form(a, b, c, fminf(fmaxf(-b * v0 * ia, u0), u1), v0);
  const float q3 = quad_form(a, b, c, fminf(fmaxf(-b * v1 * ia, u0), u1), v1);
  const float qmin = fminf(fminf(q0, q1), fminf(q2, q3));
  return qmin * 0.998f <= thr;
}

// Forward: one wave (64 threads) per 8x8 quadrant of a 16x16 tile.  The wave streams the tile's
// depth-sorted instance list 64 at a time, keeps (ballot compaction, order preserved) only the
// Gaussians whose alpha >= 1/255 ellipse can reach its quadrant, and blends them with a
// branch-free predicated body.  No workgroup barriers couple quadrants that terminate at
// different depths, and 4x more independent waves balance the load across the 256 CUs.
__global__ __launch_bounds__(64) void k_render_fwd(RenderSet rs,
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
  const int U = unit_grid(rs.gx, rs.gy);
  const int v = blockIdx.x / U;
  int tile, q;
  if (!unit_of_block(blockIdx.x - v * U, rs.gx, rs.gy, tile, q)) return;
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
  const uint2 range = ranges[tile];
  const int n = (int)(range.y - range.x);

  bool done = !inside;
  float T = 1.0f, Cr = 0.f, Cg = 0.f, Cb = 0.f, D = 0.f;
  uint32_t last_contributor = 0;
  // two-stage prefetch (as in the backward): indices two batches ahead, records one batch ahead
  const uint32_t gmask = rs.gmask;
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 n0 = zero4, n1 = zero4, n2 = zero4;
  uint32_t gi_next = 0u;
  if (lane < n) {
    const uint32_t g0 = sorted_gauss[range.x + lane] & gmask;
    n0 = rec[g0].a;
    n1 = rec[g0].b;
    n2 = rec[g0].c;
  }
  if (64 + lane < n) gi_next = sorted_gauss[range.x + 64 + lane] & gmask;
  for (int base = 0; base < n; base += 64) {
    if (__all(done)) break;
    const int i = base + lane;
    const float4 r0 = n0, r1 = n1, r2 = n2;
    if (base + 64 + lane < n) {
      n0 = rec[gi_next].a;
      n1 = rec[gi_next].b;
      n2 = rec[gi_next].c;
    }
    if (base + 128 + lane < n) gi_next = sorted_gauss[range.x + base + 128 + lane] & gmask;
    bool keep = false;
    if (i < n) keep = quadrant_hit(r0, r1, (float)qx0, (float)qy0);
    const unsigned long long bal = __ballot(keep);
    const int cnt = __popcll(bal);
    if (keep) {
      const uint32_t pos = mask_rank(bal);
      s0[pos] = r0;
      s1[pos] = make_float4(r1.x, r1.y, r1.z, __uint_as_float((uint32_t)(i + 1)));  // .w: 1 + list position
      s2[pos] = r2;
    }
    __syncthreads();
    float4 a = s0[0], b = s1[0], c = s2[0];
    for (int k = 0; k < cnt; ++k) {
      if ((k & 7) == 0 && __all(done)) break;
      const float4 an = s0[k + 1], bn = s1[k + 1], cn = s2[k + 1];
      const float dx = a.x - pxf, dy = a.y - pyf;
      const float power = gauss_power(a.z, a.w, b.x, dx, dy);
      const float alpha = fminf(GSR_ALPHA_MAX, b.y * __expf(power));
      const bool ok = !done && power <= 0.0f && alpha >= GSR_ALPHA_MIN;
      const float test_T = T * (1.0f - alpha);
      const bool term = ok && test_T < GSR_T_EPS;
      const bool blend = ok && !term;
      Cr = blend ? Cr + c.x * alpha * T : Cr;
      Cg = blend ? Cg + c.y * alpha * T : Cg;
      Cb = blend ? Cb + c.z * alpha * T : Cb;
      D = blend ? D + b.z * alpha * T : D;
      T = blend ? test_T : T;
      last_contributor = blend ? __float_as_uint(b.w) : last_contributor;
      done = done || term;
      a = an;
      b = bn;
      c = cn;
    }
    __syncthreads();
  }
  if (inside) {
    const size_t pid = (size_t)py * W + px;
    const size_t HW = (size_t)H * W;
    final_T[pid] = T;
    n_contrib[pid] = last_contributor;
    out_color[pid] = Cr + T * bg[0];
    out_color[HW + pid] = Cg + T * bg[1];
    out_color[2 * HW + pid] = Cb + T * bg[2];
    out_depth[pid] = D;
    out_alpha[pid] = 1.0f - T;
  }
  uint32_t mc = last_contributor;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mc = max(mc, (uint32_t)__shfl_xor((int)mc, o, 64));
  if (lane == 0) quad_maxc[unit] = mc;
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

void launch_render_forward(const RenderSet& rs, const GeomState& g, const uint32_t* sorted_gauss,
                           const ImageState& img, float* out_color, float* out_depth, float* out_alpha,
                           hipStream_t stream) {
  const int nt = rs.gx * rs.gy;
  if (nt <= 0 || rs.V <= 0) return;
  hipLaunchKernelGGL(k_render_fwd, dim3(rs.V * unit_grid(rs.gx, rs.gy)), dim3(64), 0, stream, rs,
                     (const uint2*)img.ranges, sorted_gauss, (const GaussRec*)g.rec, out_color, out_depth, out_alpha,
                     img.final_T, img.n_contrib, img.quad_maxc);
  hipLaunchKernelGGL(k_tile_info, dim3(rs.V * div_up(nt, 256)), dim3(256), 0, stream, rs,
                     (const uint2*)img.ranges, (const uint32_t*)img.quad_maxc, sorted_gauss,
                     (const GaussRec*)g.rec, img.tile_info, img.cut);
}

// ---------------------------------------------------------------------------------------
// Backward.  Per pixel the reference's back-to-front replay: T recovered by division, suffix
// colour/depth/alpha accumulators, background term.  Per pair the 10 gradient terms are
//   0,1 dmean2D (x W/2, H/2)  2,3,4 dconic (a, b[half], c)  5 dopacity  6,7,8 dcolor  9 ddepth
#define NGV 10

__device__ __forceinline__ float swap_add32(float& x, float& y) {
  // v_permlane32_swap: lanes 32-63 of x <-> lanes 0-31 of y, then add:
  // result = [x_lo + x_hi | y_lo + y_hi]
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap_add16(float x, float y) {
  // v_permlane16_swap: in each 32-lane half, lanes 16-31 of x <-> lanes 0-15 of y, then add:
  // rows (16 lanes) of the result = [x_r0 + x_r1, y_r0 + y_r1, x_r2 + x_r3, y_r2 + y_r3]
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// Sum two candidates' 10 per-lane values over the 64 lanes.  Transposed reduction: the 32-lane and
// 16-lane exchanges each halve the register count (one swap + one add per pair), after which register
// j holds, per 16-lane row, (va[j], va[j+5], vb[j], vb[j+5]) summed over 4 lanes; a 4-step DPP row
// reduction finishes.  Lane 15 ends with va[0..4], lane 31 va[5..9], lane 47 vb[0..4], lane 63 vb[5..9].
__device__ __forceinline__ void pair_reduce(float (&va)[NGV], float (&vb)[NGV], float (&out)[5]) {
  float y[NGV];
#pragma unroll
  for (int i = 0; i < NGV; ++i) y[i] = swap_add32(va[i], vb[i]);  // [va_i | vb_i], 2 lanes each
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    float z = swap_add16(y[j], y[j + 5]);  // rows: va_j, va_{j+5}, vb_j, vb_{j+5}
    z += dpp_f32<0x111>(z);
    z += dpp_f32<0x112>(z);
    z += dpp_f32<0x114>(z);
    z += dpp_f32<0x118>(z);
    out[j] = z;
  }
}

// One wave per 8x8 quadrant (as the forward).  The wave walks its tile's list back to front from
// the tile's deepest blended instance, 64 at a time, keeps (ballot compaction, order kept) the
// Gaussians that are above the quadrant's own deepest blended instance and whose alpha >= 1/255
// ellipse reaches the quadrant, replays them per pixel, reduces each Gaussian's 10 terms over
// 16-lane rows with DPP, parks the 4 row partials in LDS and every 32 Gaussians writes one 48-byte
// row per (instance, quadrant) at 4 * slot + quadrant, where slot is the instance's place in its
// Gaussian's contiguous row range.  Instances the quadrant skips get zero rows, so every instance
// above the tile cutoff has all 4 rows written.
// Backward: one 256-thread workgroup per (view, tile); wave q owns quadrant q.  The four waves walk
// the tile's list back to front in lockstep batches of 64 candidates: the batch's records are
// staged in LDS once for all four (one global gather per candidate instead of four), each wave culls
// the batch for its quadrant and reduces its kept candidates in pairs (pair_reduce) into per-
// (candidate, quadrant) moment sums in LDS, and one thread per candidate adds the four quadrants
// and writes ONE 48-byte gradient row per instance (4x fewer row bytes than a row per quadrant,
// for this kernel's writes and the per-Gaussian gather's reads).
#define GSR_QSUM_STRIDE 52  // floats per candidate: 4 quadrants x 13 (10 used); 208 B, conflict-free
struct BwdLDS {
  float4 s0[65], s1[65], s2[65];
  uint32_t slot[64];
  uint32_t list[4][64];
  float qsum[64 * GSR_QSUM_STRIDE];
};

__host__ __device__ __forceinline__ int tile_grid(int gx, int gy) {
  const int S = ((gx + 1) >> 1) * ((gy + 1) >> 1);
  return 32 * ((S + 7) >> 3);
}
// blockIdx -> tile: 2x2-tile super-tiles dealt round-robin over the 8 XCD groups (as unit_of_block)
__device__ __forceinline__ bool tile_of_block(int b, int gx, int gy, int& tile) {
  const int sgx = (gx + 1) >> 1, sgy = (gy + 1) >> 1;
  const int x = b & 7, k = b >> 3;
  const int s = ((k >> 2) << 3) + x;
  const int w = k & 3;
  if (s >= sgx * sgy) return false;
  const int tx = (s % sgx) * 2 + (w & 1), ty = (s / sgx) * 2 + (w >> 1);
  if (tx >= gx || ty >= gy) return false;
  tile = ty * gx + tx;
  return true;
}

__global__ __launch_bounds__(256) void k_render_bwd(RenderSet rs,
                                                    const uint2* __restrict__ ranges,
                                                    const uint32_t* __restrict__ quad_maxc,
                                                    const uint32_t* __restrict__ sorted_gauss,
                                                    const GaussRec* __restrict__ rec,
                                                    const float* __restrict__ final_Ts,
                                                    const uint32_t* __restrict__ n_contrib,
                                                    const float* __restrict__ dL_dcolor,
                                                    const float* __restrict__ dL_ddepth,
                                                    const float* __restrict__ dL_dalpha,
                                                    float4* __restrict__ grow) {
  __shared__ BwdLDS s;
  const int TG = tile_grid(rs.gx, rs.gy);
  const int v = blockIdx.x / TG;
  int tile;
  if (!tile_of_block(blockIdx.x - v * TG, rs.gx, rs.gy, tile)) return;
  GSR_TL_BEGIN
  const int W = rs.W, H = rs.H, grid_x = rs.gx;
  {
    const size_t vg = (size_t)(rs.v0 + v), tiles = (size_t)rs.gx * rs.gy, HWs = (size_t)W * H;
    ranges += vg * tiles;
    quad_maxc += vg * 4 * tiles;
    sorted_gauss += rs.inst_start[v];
    rec += vg * rs.P;
    final_Ts += vg * HWs;
    n_contrib += vg * HWs;
    dL_dcolor += (size_t)v * 3 * HWs;
    if (dL_ddepth) dL_ddepth += (size_t)v * HWs;
    if (dL_dalpha) dL_dalpha += (size_t)v * HWs;
    grow += (size_t)3 * rs.row_start[v];
  }
  const float* bg = rs.bg[v];
  int tl_work = 0;
  const int t = threadIdx.x, q = t >> 6, lane = t & 63;
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
  }
  const float bg_dot = bg[0] * dpix[0] + bg[1] * dpix[1] + bg[2] * dpix[2];

  float acc_r = 0.f, acc_g = 0.f, acc_b = 0.f, acc_d = 0.f, acc_a = 0.f;
  float last_alpha = 0.f, last_r = 0.f, last_g = 0.f, last_b = 0.f, last_depth = 0.f;
  const float ddelx_dx = 0.5f * W, ddely_dy = 0.5f * H;
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);

  // wave 0 stages the batches; two-stage prefetch (indices two batches ahead, records one ahead)
  const uint32_t gmask = rs.gmask;
  auto fetch_index = [&](int h) -> uint32_t {
    const int r = h - 1 - lane;
    return r >= 0 ? (sorted_gauss[range.x + r] & gmask) : 0u;
  };
  float4 n0 = zero4, n1 = zero4, n2 = zero4;
  uint4 nd = make_uint4(0u, 0u, 0u, 0u);
  uint32_t gi_next = 0u;
  if (q == 0 && maxc > 0) {
    const uint32_t g0 = fetch_index(maxc);
    if (maxc - 1 - lane >= 0) {
      n0 = rec[g0].a;
      n1 = rec[g0].b;
      n2 = rec[g0].c;
      nd = rec[g0].d;
    }
    if (maxc > 64) gi_next = fetch_index(maxc - 64);
  }

  // branch-free replay step (reference order of operations); non-contributing lanes keep their
  // state and contribute zeros.  Per pair: moments of u = G dL/dalpha over the pixel offsets
  // (mean2D / conic / opacity gradients are linear in them) and the colour / depth weights.
  auto replay = [&](const float4& ga, const float4& gb, const float4& gc, float (&vv)[NGV]) -> bool {
    const uint32_t rel = __float_as_uint(gb.w);
    const float dx = ga.x - pxf, dy = ga.y - pyf;
    const float power = gauss_power(ga.z, ga.w, gb.x, dx, dy);
    const float G = __expf(power);
    const float alpha = fminf(GSR_ALPHA_MAX, gb.y * G);
    const bool hit = rel < last_contributor && power <= 0.0f && alpha >= GSR_ALPHA_MIN;
    const float inv_1ma = fast_rcp(1.f - alpha);
    T = hit ? T * inv_1ma : T;
    const float oml = 1.f - last_alpha;
    const float nr = last_alpha * last_r + oml * acc_r;
    const float ng = last_alpha * last_g + oml * acc_g;
    const float nb = last_alpha * last_b + oml * acc_b;
    const float nd = last_alpha * last_depth + oml * acc_d;
    const float na = last_alpha * 1.0f + oml * acc_a;
    float dL_dalpha = 0.0f;
    dL_dalpha += (gc.x - nr) * dpix[0];
    dL_dalpha += (gc.y - ng) * dpix[1];
    dL_dalpha += (gc.z - nb) * dpix[2];
    dL_dalpha += (gb.z - nd) * dpix_d;
    dL_dalpha += (1.f - na) * dpix_a;
    dL_dalpha *= T;
    dL_dalpha += (-T_final * inv_1ma) * bg_dot;
    const float u = hit ? G * dL_dalpha : 0.0f;  // dL/dG / opacity
    const float w = hit ? alpha * T : 0.0f;      // dL/dcolor per unit dL/dpixel
    acc_r = hit ? nr : acc_r;
    acc_g = hit ? ng : acc_g;
    acc_b = hit ? nb : acc_b;
    acc_d = hit ? nd : acc_d;
    acc_a = hit ? na : acc_a;
    last_r = hit ? gc.x : last_r;
    last_g = hit ? gc.y : last_g;
    last_b = hit ? gc.z : last_b;
    last_depth = hit ? gb.z : last_depth;
    last_alpha = hit ? alpha : last_alpha;
    const float udx = u * dx, udy = u * dy;
    vv[0] = u;
    vv[1] = udx;
    vv[2] = udy;
    vv[3] = udx * dx;
    vv[4] = udx * dy;
    vv[5] = udy * dy;
    vv[6] = w * dpix[0];
    vv[7] = w * dpix[1];
    vv[8] = w * dpix[2];
    vv[9] = w * dpix_d;
    return hit;
  };

  uint32_t* mylist = s.list[q];
  float* myq = s.qsum + q * 13;
  for (int hi = maxc; hi > 0; hi -= 64) {
    if (q == 0) {
      const int rel_l = hi - 1 - lane;
      if (rel_l >= 0) {
        const int xmin = nd.x & 0xffff, ymin = nd.x >> 16, xmax = nd.y & 0xffff;
        s.s0[lane] = n0;
        s.s1[lane] = make_float4(n1.x, n1.y, n1.z, __uint_as_float((uint32_t)rel_l));  // .w: list position
        s.s2[lane] = n2;
        s.slot[lane] = nd.z + (uint32_t)((tyi - ymin) * (xmax - xmin) + (txi - xmin));
      }
      if (hi > 64) {
        if (hi - 65 - lane >= 0) {
          n0 = rec[gi_next].a;
          n1 = rec[gi_next].b;
          n2 = rec[gi_next].c;
          nd = rec[gi_next].d;
        }
        if (hi > 128) gi_next = fetch_index(hi - 128);
      }
    }
    __syncthreads();
    // this wave's quadrant: cull the staged batch, list the kept candidates, zero the others' sums
    const int rel_l = hi - 1 - lane;
    bool keep = false;
    if (rel_l >= 0 && rel_l < qmaxc) keep = quadrant_hit(s.s0[lane], s.s1[lane], (float)qx0, (float)qy0);
    if (rel_l >= 0 && !keep) {
      float* z = myq + lane * GSR_QSUM_STRIDE;
#pragma unroll
      for (int i = 0; i < NGV; ++i) z[i] = 0.f;
    }
    const unsigned long long bal = __ballot(keep);
    const int cnt = __popcll(bal);
    tl_work += cnt;
    if (keep) mylist[mask_rank(bal)] = (uint32_t)lane;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's list is read back by its own lanes
    // kept candidates in pairs: transposed reduction of the 2 x 10 per-lane values (pair_reduce)
    for (int k = 0; k < cnt; k += 2) {
      const int j0 = __builtin_amdgcn_readfirstlane(mylist[k]);
      const int j1 = k + 1 < cnt ? __builtin_amdgcn_readfirstlane(mylist[k + 1]) : -1;
      float va[NGV], vb[NGV];
      bool hit = replay(s.s0[j0], s.s1[j0], s.s2[j0], va);
      if (j1 >= 0) {
        hit = replay(s.s0[j1], s.s1[j1], s.s2[j1], vb) || hit;
      } else {
#pragma unroll
        for (int i = 0; i < NGV; ++i) vb[i] = 0.f;
      }
      // lane 15: candidate j0 values 0-4, lane 31: j0 values 5-9, lanes 47 / 63: candidate j1
      const int jj = (lane >> 5) ? j1 : j0;
      float r[5];
      if (__any(hit)) {
        pair_reduce(va, vb, r);
      } else {
#pragma unroll
        for (int i = 0; i < 5; ++i) r[i] = 0.f;
      }
      if ((lane & 15) == 15 && jj >= 0) {
        float* dst = myq + jj * GSR_QSUM_STRIDE + ((lane >> 4) & 1) * 5;
#pragma unroll
        for (int i = 0; i < 5; ++i) dst[i] = r[i];
      }
    }
    __syncthreads();
    if (t < 64 && hi - 1 - t >= 0) {
      // one thread per candidate: add the 4 quadrants' moments, turn them into the reference's terms
      //   dmean2D = -o (W/2, H/2) (a m1 + b m2, c m2 + b m1), dconic = -o/2 (m3, m4, m5), dopacity = m0
      const float* qs = s.qsum + t * GSR_QSUM_STRIDE;
      float m[NGV];
#pragma unroll
      for (int i = 0; i < NGV; ++i) m[i] = qs[i] + qs[13 + i] + qs[26 + i] + qs[39 + i];
      const float4 ga = s.s0[t];
      const float4 gb = s.s1[t];
      const float o = gb.y;
      const float dmx = -o * ddelx_dx * (ga.z * m[1] + ga.w * m[2]);
      const float dmy = -o * ddely_dy * (gb.x * m[2] + ga.w * m[1]);
      float4* row = grow + 3 * (size_t)s.slot[t];
      row[0] = make_float4(dmx, dmy, -0.5f * o * m[3], -0.5f * o * m[4]);
      row[1] = make_float4(-0.5f * o * m[5], m[0], m[6], m[7]);
      row[2] = make_float4(m[8], m[9], 0.f, 0.f);
    }
    __syncthreads();
  }
  GSR_TL_END(1, tl_work)
  (void)tl_work;
}

void launch_render_backward(const RenderSet& rs, const GeomState& g, const uint32_t* sorted_gauss,
                            const ImageState& img, const float* dL_dcolor, const float* dL_ddepth,
                            const float* dL_dalpha, const BackwardState& bw, hipStream_t stream) {
  const int nt = rs.gx * rs.gy;
  if (nt <= 0 || rs.V <= 0) return;
  hipLaunchKernelGGL(k_render_bwd, dim3(rs.V * tile_grid(rs.gx, rs.gy)), dim3(256), 0, stream, rs,
                     (const uint2*)img.ranges, (const uint32_t*)img.quad_maxc, sorted_gauss,
                     (const GaussRec*)g.rec, (const float*)img.final_T,
                     (const uint32_t*)img.n_contrib, dL_dcolor, dL_ddepth, dL_dalpha, bw.grow);
}

}  // namespace gsr

#ifdef GSR_TIMELINE
extern "C" int gsr_diag_timeline(int which, void* host, int n) {
  if (which < 0 || which > 1 || n > GSR_TL_MAX) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(gsr::g_timeline), sizeof(uint4) * n,
                          sizeof(uint4) * GSR_TL_MAX * which, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return 0;
}
#endif

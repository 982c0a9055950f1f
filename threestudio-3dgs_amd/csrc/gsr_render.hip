// gsr_render.hip — per-tile alpha blending, forward and backward.
//
// One 256-thread workgroup per 16x16 tile; the four waves each own an 8x8 pixel quadrant
// (compact wave footprints: a Gaussian that misses a quadrant costs that wave nothing in the
// backward pass, and whole waves finish early together in the forward pass).
// Gaussian records (48 B: xy, conic, opacity, depth, rgb) are gathered by sorted instance into
// LDS in chunks of 256 and read back as broadcast ds_read_b128.
//
// Forward replaces FORWARD::renderCUDA [EXT] (ashawkey 4-output: color, depth = sum z a T,
// alpha = 1 - T).  Backward replaces BACKWARD::renderCUDA [EXT] but, instead of 9 global float
// atomics per (pixel, Gaussian) pair, reduces each pair's 10 gradient terms over the wave with
// DPP, sums the 4 waves in LDS, and writes ONE 48-byte row per sorted instance with coalesced
// stores; gsr_backward.hip then sums each Gaussian's rows in a fixed order (deterministic).
#include "gsr_kernels.h"
#include "gsr_wave.h"

namespace gsr {

// blockIdx -> tile index: blocks b and b+8 share an XCD (round-robin dispatch), so give each
// group of blocks with equal b % 8 one contiguous band of tile rows -> neighbouring tiles, which
// share most of their Gaussians, hit the same L2.  Bijective for any tile count.
__device__ __forceinline__ int xcd_tile(int b, int nt) {
  const int xcd = b & 7, k = b >> 3;
  const int q = nt >> 3, r = nt & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

__device__ __forceinline__ void tile_pixel(int t, int& lx, int& ly) {
  const int w = t >> 6, l = t & 63;
  lx = ((w & 1) << 3) | (l & 7);
  ly = ((w >> 1) << 3) | (l >> 3);
}

__global__ __launch_bounds__(256) void k_render_fwd(int W, int H, int grid_x, int n_tiles,
                                                    const uint2* __restrict__ ranges,
                                                    const uint32_t* __restrict__ sorted_gauss,
                                                    const float4* __restrict__ rec0,
                                                    const float4* __restrict__ rec1,
                                                    const float4* __restrict__ rec2,
                                                    const float* __restrict__ bg,
                                                    float* __restrict__ out_color,
                                                    float* __restrict__ out_depth,
                                                    float* __restrict__ out_alpha,
                                                    float* __restrict__ final_T,
                                                    uint32_t* __restrict__ n_contrib) {
  __shared__ float4 s0[256], s1[256], s2[256];
  const int tile = xcd_tile(blockIdx.x, n_tiles);
  const int t = threadIdx.x;
  int lx, ly;
  tile_pixel(t, lx, ly);
  const int px = (tile % grid_x) * GSR_TILE_X + lx;
  const int py = (tile / grid_x) * GSR_TILE_Y + ly;
  const bool inside = px < W && py < H;
  const float pxf = (float)px, pyf = (float)py;
  const uint2 range = ranges[tile];

  bool done = !inside;
  float T = 1.0f, Cr = 0.f, Cg = 0.f, Cb = 0.f, D = 0.f;
  uint32_t contributor = 0, last_contributor = 0;
  int todo = (int)(range.y - range.x);
  for (uint32_t start = range.x; start < range.y; start += 256, todo -= 256) {
    if (__syncthreads_count(done) == 256) break;
    const uint32_t p = start + t;
    if (p < range.y) {
      const uint32_t gi = sorted_gauss[p];
      s0[t] = rec0[gi];
      s1[t] = rec1[gi];
      s2[t] = rec2[gi];
    }
    __syncthreads();
    const int cnt = todo < 256 ? todo : 256;
    for (int j = 0; !done && j < cnt; ++j) {
      ++contributor;
      const float4 a = s0[j];
      const float4 b = s1[j];
      const float dx = a.x - pxf, dy = a.y - pyf;
      const float power = gauss_power(a.z, a.w, b.x, dx, dy);
      if (power > 0.0f) continue;
      const float alpha = fminf(GSR_ALPHA_MAX, b.y * __expf(power));
      if (alpha < GSR_ALPHA_MIN) continue;
      const float test_T = T * (1.0f - alpha);
      if (test_T < GSR_T_EPS) {
        done = true;
        continue;
      }
      const float4 c = s2[j];
      Cr += c.x * alpha * T;
      Cg += c.y * alpha * T;
      Cb += c.z * alpha * T;
      D += b.z * alpha * T;
      T = test_T;
      last_contributor = contributor;
    }
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
}

void launch_render_forward(int W, int H, const GeomState& g, const BinningState& b,
                           const ImageState& img, const float* bg, float* out_color,
                           float* out_depth, float* out_alpha, hipStream_t stream) {
  const int gx = div_up(W, GSR_TILE_X), gy = div_up(H, GSR_TILE_Y);
  const int nt = gx * gy;
  if (nt <= 0) return;
  hipLaunchKernelGGL(k_render_fwd, dim3(nt), dim3(256), 0, stream, W, H, gx, nt,
                     (const uint2*)img.ranges, (const uint32_t*)b.sorted_gauss,
                     (const float4*)g.rec0, (const float4*)g.rec1, (const float4*)g.rec2, bg,
                     out_color, out_depth, out_alpha, img.final_T, img.n_contrib);
}

// ---------------------------------------------------------------------------------------
// Backward.  Per pixel the reference's back-to-front replay: T recovered by division, suffix
// colour/depth/alpha accumulators, background term.  Per pair the 10 gradient terms are
//   0,1 dmean2D (x W/2, H/2)  2,3,4 dconic (a, b[half], c)  5 dopacity  6,7,8 dcolor  9 ddepth
#define NGV 10

__global__ __launch_bounds__(256) void k_render_bwd(int W, int H, int grid_x, int n_tiles,
                                                    const uint2* __restrict__ ranges,
                                                    const uint32_t* __restrict__ sorted_gauss,
                                                    const float4* __restrict__ rec0,
                                                    const float4* __restrict__ rec1,
                                                    const float4* __restrict__ rec2,
                                                    const float* __restrict__ bg,
                                                    const float* __restrict__ final_Ts,
                                                    const uint32_t* __restrict__ n_contrib,
                                                    const float* __restrict__ dL_dcolor,
                                                    const float* __restrict__ dL_ddepth,
                                                    const float* __restrict__ dL_dalpha,
                                                    float4* __restrict__ grow) {
  __shared__ float4 s0[256], s1[256], s2[256];
  __shared__ float s_part[4][NGV][256];
  __shared__ uint32_t s_red[8];
  const int tile = xcd_tile(blockIdx.x, n_tiles);
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  int lx, ly;
  tile_pixel(t, lx, ly);
  const int px = (tile % grid_x) * GSR_TILE_X + lx;
  const int py = (tile / grid_x) * GSR_TILE_Y + ly;
  const bool inside = px < W && py < H;
  const float pxf = (float)px, pyf = (float)py;
  const uint2 range = ranges[tile];
  const int n = (int)(range.y - range.x);
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

  // the deepest instance any pixel of the tile blended
  uint32_t mc = last_contributor;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mc = max(mc, (uint32_t)__shfl_xor((int)mc, o, 64));
  if (lane == 0) s_red[w] = mc;
  __syncthreads();
  const int maxc = (int)max(max(s_red[0], s_red[1]), max(s_red[2], s_red[3]));

  // instances nobody blended contribute nothing: zero their rows
  for (int rel = maxc + t; rel < n; rel += 256) {
    const size_t p = (size_t)range.x + rel;
    grow[3 * p] = make_float4(0.f, 0.f, 0.f, 0.f);
    grow[3 * p + 1] = make_float4(0.f, 0.f, 0.f, 0.f);
    grow[3 * p + 2] = make_float4(0.f, 0.f, 0.f, 0.f);
  }

  float acc_r = 0.f, acc_g = 0.f, acc_b = 0.f, acc_d = 0.f, acc_a = 0.f;
  float last_alpha = 0.f, last_r = 0.f, last_g = 0.f, last_b = 0.f, last_depth = 0.f;
  const float ddelx_dx = 0.5f * W, ddely_dy = 0.5f * H;
  uint32_t contributor = (uint32_t)maxc;

  for (int hi = maxc; hi > 0; hi -= 256) {
    const int cnt = hi < 256 ? hi : 256;
    if (t < cnt) {
      const uint32_t gi = sorted_gauss[range.x + hi - 1 - t];
      s0[t] = rec0[gi];
      s1[t] = rec1[gi];
      s2[t] = rec2[gi];
    }
    __syncthreads();
    for (int j = 0; j < cnt; ++j) {
      --contributor;
      float v[NGV];
#pragma unroll
      for (int k = 0; k < NGV; ++k) v[k] = 0.f;
      bool hit = false;
      if (contributor < last_contributor) {
        const float4 a = s0[j];
        const float4 b = s1[j];
        const float dx = a.x - pxf, dy = a.y - pyf;
        const float power = gauss_power(a.z, a.w, b.x, dx, dy);
        if (power <= 0.0f) {
          const float G = __expf(power);
          const float alpha = fminf(GSR_ALPHA_MAX, b.y * G);
          if (alpha >= GSR_ALPHA_MIN) {
            hit = true;
            const float4 c = s2[j];
            T = T / (1.f - alpha);
            const float dchannel_dcolor = alpha * T;
            float dL_dalpha = 0.0f;
            acc_r = last_alpha * last_r + (1.f - last_alpha) * acc_r;
            acc_g = last_alpha * last_g + (1.f - last_alpha) * acc_g;
            acc_b = last_alpha * last_b + (1.f - last_alpha) * acc_b;
            last_r = c.x;
            last_g = c.y;
            last_b = c.z;
            dL_dalpha += (c.x - acc_r) * dpix[0];
            dL_dalpha += (c.y - acc_g) * dpix[1];
            dL_dalpha += (c.z - acc_b) * dpix[2];
            v[6] = dchannel_dcolor * dpix[0];
            v[7] = dchannel_dcolor * dpix[1];
            v[8] = dchannel_dcolor * dpix[2];
            acc_d = last_alpha * last_depth + (1.f - last_alpha) * acc_d;
            last_depth = b.z;
            dL_dalpha += (b.z - acc_d) * dpix_d;
            v[9] = dchannel_dcolor * dpix_d;
            acc_a = last_alpha * 1.0f + (1.f - last_alpha) * acc_a;
            dL_dalpha += (1.f - acc_a) * dpix_a;
            dL_dalpha *= T;
            last_alpha = alpha;
            dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
            const float dL_dG = b.y * dL_dalpha;
            const float gdx = G * dx, gdy = G * dy;
            const float dG_ddelx = -gdx * a.z - gdy * a.w;
            const float dG_ddely = -gdy * b.x - gdx * a.w;
            v[0] = dL_dG * dG_ddelx * ddelx_dx;
            v[1] = dL_dG * dG_ddely * ddely_dy;
            v[2] = -0.5f * gdx * dx * dL_dG;
            v[3] = -0.5f * gdx * dy * dL_dG;
            v[4] = -0.5f * gdy * dy * dL_dG;
            v[5] = G * dL_dalpha;
          }
        }
      }
      // wave-uniform: reduce only when some pixel of this quadrant used the Gaussian
      if (__any(hit)) {
#pragma unroll
        for (int k = 0; k < NGV; ++k) {
          const float s = wave_sum(v[k]);
          if (lane == 0) s_part[w][k][j] = s;
        }
      } else if (lane == 0) {
#pragma unroll
        for (int k = 0; k < NGV; ++k) s_part[w][k][j] = 0.f;
      }
    }
    __syncthreads();
    if (t < cnt) {
      float r[NGV];
#pragma unroll
      for (int k = 0; k < NGV; ++k) r[k] = (s_part[0][k][t] + s_part[1][k][t]) + (s_part[2][k][t] + s_part[3][k][t]);
      const size_t p = (size_t)range.x + hi - 1 - t;
      grow[3 * p] = make_float4(r[0], r[1], r[2], r[3]);
      grow[3 * p + 1] = make_float4(r[4], r[5], r[6], r[7]);
      grow[3 * p + 2] = make_float4(r[8], r[9], 0.f, 0.f);
    }
    __syncthreads();
  }
}

void launch_render_backward(int W, int H, int K, const GeomState& g, const BinningState& b,
                            const ImageState& img, const float* bg, const float* dL_dcolor,
                            const float* dL_ddepth, const float* dL_dalpha,
                            const BackwardState& bw, hipStream_t stream) {
  const int gx = div_up(W, GSR_TILE_X), gy = div_up(H, GSR_TILE_Y);
  const int nt = gx * gy;
  if (nt <= 0 || K <= 0) return;
  hipLaunchKernelGGL(k_render_bwd, dim3(nt), dim3(256), 0, stream, W, H, gx, nt,
                     (const uint2*)img.ranges, (const uint32_t*)b.sorted_gauss,
                     (const float4*)g.rec0, (const float4*)g.rec1, (const float4*)g.rec2, bg,
                     (const float*)img.final_T, (const uint32_t*)img.n_contrib, dL_dcolor,
                     dL_ddepth, dL_dalpha, bw.grow);
}

}  // namespace gsr

// gsr_epilogue.hip — fused post-raster background composite (SURVEY.md §8f "fused epilogue").
//
// The reference's background renderer composites the rasterizer's image with a background image and
// clamps (renderer/diff_gaussian_rasterizer_background.py:129-132, 139):
//     render = clamp(color + (1 - alpha) * bg, 0, 1)
// with color (3, H, W), alpha (1, H, W) and bg the background network's (H, W, 3) output.  In torch
// that is 4 elementwise passes forward and 5 backward over 3HW floats; here one pass each way.
// Operation order (no contraction) matches torch's, so the forward is bit-identical; the backward
// masks by the pre-clamp value exactly like clamp's gradient (inclusive bounds).
//   backward: g = dL/drender * [0 <= pre <= 1];  dL/dcolor = g;  dL/dalpha = -sum_c g_c bg_c;
//             dL/dbg = g * (1 - alpha)  (optional)
// One thread per 4 pixels of one view (16-byte loads of each plane when H*W % 4 == 0).  HBM bound:
// forward reads 16 B (+12 B HWC background) and writes 12 B per pixel, backward reads 28 B (+12) and
// writes 16 B (+12 B background gradient).
#include "gsr_kernels.h"

namespace gsr {

// bg layouts: 0 = per view constant [V][3], 1 = image [V][H][W][3] (HWC), 2 = image [V][3][H][W]
__device__ __forceinline__ float bg_at(const float* bg, int layout, int v, size_t HW, size_t p, int c) {
  if (layout == 0) return bg[3 * v + c];
  if (layout == 1) return bg[((size_t)v * HW + p) * 3 + c];
  return bg[((size_t)v * 3 + c) * HW + p];
}

__global__ __launch_bounds__(256) void k_composite_fwd(int V, size_t HW, const float* __restrict__ color,
                                                       const float* __restrict__ alpha, const float* __restrict__ bg,
                                                       int layout, float* __restrict__ out) {
#pragma clang fp contract(off)
  const size_t nq = (HW + 3) / 4;
  const size_t gid = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (size_t)V * nq) return;
  const int v = (int)(gid / nq);
  const size_t p0 = (gid - (size_t)v * nq) * 4;
  const float* a = alpha + (size_t)v * HW;
  float am[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) am[k] = p0 + k < HW ? 1.0f - a[p0 + k] : 0.f;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float* col = color + ((size_t)v * 3 + c) * HW;
    float* o = out + ((size_t)v * 3 + c) * HW;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const size_t p = p0 + k;
      if (p < HW) {
        const float pre = col[p] + am[k] * bg_at(bg, layout, v, HW, p, c);
        o[p] = fminf(fmaxf(pre, 0.0f), 1.0f);
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_composite_bwd(int V, size_t HW, const float* __restrict__ dout,
                                                       const float* __restrict__ color, const float* __restrict__ alpha,
                                                       const float* __restrict__ bg, int layout,
                                                       float* __restrict__ dcolor, float* __restrict__ dalpha,
                                                       float* __restrict__ dbg) {
#pragma clang fp contract(off)
  const size_t nq = (HW + 3) / 4;
  const size_t gid = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (size_t)V * nq) return;
  const int v = (int)(gid / nq);
  const size_t p0 = (gid - (size_t)v * nq) * 4;
  const float* a = alpha + (size_t)v * HW;
  float am[4], da[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 4; ++k) am[k] = p0 + k < HW ? 1.0f - a[p0 + k] : 0.f;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const size_t plane = ((size_t)v * 3 + c) * HW;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const size_t p = p0 + k;
      if (p < HW) {
        const float b = bg_at(bg, layout, v, HW, p, c);
        const float pre = color[plane + p] + am[k] * b;
        const float g = (pre >= 0.0f && pre <= 1.0f) ? dout[plane + p] : 0.0f;
        dcolor[plane + p] = g;
        da[k] -= g * b;
        if (dbg != nullptr && layout != 0) {
          const size_t bi = layout == 1 ? ((size_t)v * HW + p) * 3 + c : plane + p;
          dbg[bi] = g * am[k];
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (p0 + k < HW) dalpha[(size_t)v * HW + p0 + k] = da[k];
}

// Fast path (HW % 4 == 0, bg constant or HWC): every access a 16-byte load / store.
__device__ __forceinline__ void bg4(const float* bg, int layout, int v, size_t HW, size_t p0, float4 (&b)[3]) {
  if (layout == 0) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float x = bg[3 * v + c];
      b[c] = make_float4(x, x, x, x);
    }
  } else {  // HWC: 12 floats = pixels p0..p0+3 x (r, g, b)
    const float4* s = reinterpret_cast<const float4*>(bg + ((size_t)v * HW + p0) * 3);
    const float4 q0 = s[0], q1 = s[1], q2 = s[2];
    b[0] = make_float4(q0.x, q0.w, q1.z, q2.y);
    b[1] = make_float4(q0.y, q1.x, q1.w, q2.z);
    b[2] = make_float4(q0.z, q1.y, q2.x, q2.w);
  }
}

__global__ __launch_bounds__(256) void k_composite_fwd4(int V, size_t HW, const float* __restrict__ color,
                                                        const float* __restrict__ alpha, const float* __restrict__ bg,
                                                        int layout, float* __restrict__ out) {
#pragma clang fp contract(off)
  const size_t nq = HW / 4;
  const size_t gid = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (size_t)V * nq) return;
  const int v = (int)(gid / nq);
  const size_t q = gid - (size_t)v * nq;
  const float4 a = reinterpret_cast<const float4*>(alpha + (size_t)v * HW)[q];
  const float4 am = make_float4(1.0f - a.x, 1.0f - a.y, 1.0f - a.z, 1.0f - a.w);
  float4 b[3];
  bg4(bg, layout, v, HW, 4 * q, b);
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const size_t plane = ((size_t)v * 3 + c) * HW;
    const float4 col = reinterpret_cast<const float4*>(color + plane)[q];
    float4 r;
    r.x = fminf(fmaxf(col.x + am.x * b[c].x, 0.0f), 1.0f);
    r.y = fminf(fmaxf(col.y + am.y * b[c].y, 0.0f), 1.0f);
    r.z = fminf(fmaxf(col.z + am.z * b[c].z, 0.0f), 1.0f);
    r.w = fminf(fmaxf(col.w + am.w * b[c].w, 0.0f), 1.0f);
    reinterpret_cast<float4*>(out + plane)[q] = r;
  }
}

__global__ __launch_bounds__(256) void k_composite_bwd4(int V, size_t HW, const float* __restrict__ dout,
                                                        const float* __restrict__ color, const float* __restrict__ alpha,
                                                        const float* __restrict__ bg, int layout,
                                                        float* __restrict__ dcolor, float* __restrict__ dalpha,
                                                        float* __restrict__ dbg) {
#pragma clang fp contract(off)
  const size_t nq = HW / 4;
  const size_t gid = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (size_t)V * nq) return;
  const int v = (int)(gid / nq);
  const size_t q = gid - (size_t)v * nq;
  const float4 a = reinterpret_cast<const float4*>(alpha + (size_t)v * HW)[q];
  const float am[4] = {1.0f - a.x, 1.0f - a.y, 1.0f - a.z, 1.0f - a.w};
  float4 b[3];
  bg4(bg, layout, v, HW, 4 * q, b);
  float da[4] = {0.f, 0.f, 0.f, 0.f};
  float gb[3][4];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const size_t plane = ((size_t)v * 3 + c) * HW;
    const float4 col4 = reinterpret_cast<const float4*>(color + plane)[q];
    const float4 d4 = reinterpret_cast<const float4*>(dout + plane)[q];
    const float col[4] = {col4.x, col4.y, col4.z, col4.w}, d[4] = {d4.x, d4.y, d4.z, d4.w};
    const float bb[4] = {b[c].x, b[c].y, b[c].z, b[c].w};
    float g[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float pre = col[k] + am[k] * bb[k];
      g[k] = (pre >= 0.0f && pre <= 1.0f) ? d[k] : 0.0f;
      da[k] -= g[k] * bb[k];
      gb[c][k] = g[k] * am[k];
    }
    reinterpret_cast<float4*>(dcolor + plane)[q] = make_float4(g[0], g[1], g[2], g[3]);
  }
  reinterpret_cast<float4*>(dalpha + (size_t)v * HW)[q] = make_float4(da[0], da[1], da[2], da[3]);
  if (dbg != nullptr && layout == 1) {
    float4* s = reinterpret_cast<float4*>(dbg + ((size_t)v * HW + 4 * q) * 3);
    s[0] = make_float4(gb[0][0], gb[1][0], gb[2][0], gb[0][1]);
    s[1] = make_float4(gb[1][1], gb[2][1], gb[0][2], gb[1][2]);
    s[2] = make_float4(gb[2][2], gb[0][3], gb[1][3], gb[2][3]);
  }
}

// ---- SuGaR normal map (renderer/diff_sugar_rasterizer_normal.py:192-197) -------------------------------
// The second rasterizer call's blended face normals n (V, 3, H, W) become
//     u = n / max(|n|, 1e-12)  (F.normalize over the channels),  f = (-u_x, -u_y, u_z)  (p3d -> threestudio),
//     nmap = f * 0.5 * alpha + 0.5,  gradient only where alpha > 0.99 (the rest detached)
// in one pass each way instead of torch's ~10 elementwise kernels forward and ~15 backward.  Operation order
// of the torch lines (no contraction): (f * 0.5) * alpha + 0.5.
//   backward (alpha > 0.99):  df = g * alpha * 0.5,  dalpha = sum_c g_c f_c 0.5,  du = (-df_x, -df_y, df_z),
//                             dn = (du - u (u . du)) / |n|  (|n| > 1e-12; else du / 1e-12)
__global__ __launch_bounds__(256) void k_normal_map_fwd(int V, size_t HW, const float* __restrict__ normal,
                                                        const float* __restrict__ alpha, float* __restrict__ out) {
#pragma clang fp contract(off)
  const size_t gid = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (size_t)V * HW) return;
  const size_t v = gid / HW, p = gid - v * HW;
  const float* n = normal + v * 3 * HW + p;
  const float x = n[0], y = n[HW], z = n[2 * HW];
  const float len = sqrtf(x * x + y * y + z * z);
  const float d = fmaxf(len, 1e-12f);
  const float f[3] = {-(x / d), -(y / d), z / d};
  const float a = alpha[v * HW + p];
  float* o = out + v * 3 * HW + p;
#pragma unroll
  for (int c = 0; c < 3; ++c) o[(size_t)c * HW] = f[c] * 0.5f * a + 0.5f;
}

__global__ __launch_bounds__(256) void k_normal_map_bwd(int V, size_t HW, const float* __restrict__ dout,
                                                        const float* __restrict__ normal,
                                                        const float* __restrict__ alpha, float* __restrict__ dnormal,
                                                        float* __restrict__ dalpha) {
#pragma clang fp contract(off)
  const size_t gid = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (size_t)V * HW) return;
  const size_t v = gid / HW, p = gid - v * HW;
  const float a = alpha[v * HW + p];
  float* dn = dnormal + v * 3 * HW + p;
  if (!(a > 0.99f)) {
    dn[0] = 0.f;
    dn[HW] = 0.f;
    dn[2 * HW] = 0.f;
    dalpha[v * HW + p] = 0.f;
    return;
  }
  const float* n = normal + v * 3 * HW + p;
  const float x = n[0], y = n[HW], z = n[2 * HW];
  const float len = sqrtf(x * x + y * y + z * z);
  const float d = fmaxf(len, 1e-12f);
  const float u[3] = {x / d, y / d, z / d};
  const float f[3] = {-u[0], -u[1], u[2]};
  const float* g = dout + v * 3 * HW + p;
  const float gc[3] = {g[0], g[HW], g[2 * HW]};
  dalpha[v * HW + p] = gc[0] * (f[0] * 0.5f) + gc[1] * (f[1] * 0.5f) + gc[2] * (f[2] * 0.5f);
  const float du[3] = {-(gc[0] * a * 0.5f), -(gc[1] * a * 0.5f), gc[2] * a * 0.5f};
  if (len > 1e-12f) {
    const float ud = u[0] * du[0] + u[1] * du[1] + u[2] * du[2];
#pragma unroll
    for (int c = 0; c < 3; ++c) dn[(size_t)c * HW] = (du[c] - u[c] * ud) / d;
  } else {
#pragma unroll
    for (int c = 0; c < 3; ++c) dn[(size_t)c * HW] = du[c] / d;
  }
}

void launch_normal_map_fwd(int V, size_t HW, const float* normal, const float* alpha, float* out, hipStream_t stream) {
  const size_t n = (size_t)V * HW;
  if (n == 0) return;
  hipLaunchKernelGGL(k_normal_map_fwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, V, HW, normal, alpha,
                     out);
}

void launch_normal_map_bwd(int V, size_t HW, const float* dout, const float* normal, const float* alpha,
                           float* dnormal, float* dalpha, hipStream_t stream) {
  const size_t n = (size_t)V * HW;
  if (n == 0) return;
  hipLaunchKernelGGL(k_normal_map_bwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, V, HW, dout, normal,
                     alpha, dnormal, dalpha);
}

void launch_composite_fwd(int V, size_t HW, const float* color, const float* alpha, const float* bg, int layout,
                          float* out, hipStream_t stream) {
  const size_t n = (size_t)V * ((HW + 3) / 4);
  if (n == 0) return;
  if (HW % 4 == 0 && layout != 2) {
    hipLaunchKernelGGL(k_composite_fwd4, dim3((unsigned)div_up((long long)n, 256)), dim3(256), 0, stream, V, HW,
                       color, alpha, bg, layout, out);
    return;
  }
  hipLaunchKernelGGL(k_composite_fwd, dim3((unsigned)div_up((long long)n, 256)), dim3(256), 0, stream, V, HW, color,
                     alpha, bg, layout, out);
}

void launch_composite_bwd(int V, size_t HW, const float* dout, const float* color, const float* alpha,
                          const float* bg, int layout, float* dcolor, float* dalpha, float* dbg,
                          hipStream_t stream) {
  const size_t n = (size_t)V * ((HW + 3) / 4);
  if (n == 0) return;
  if (HW % 4 == 0 && layout != 2) {
    hipLaunchKernelGGL(k_composite_bwd4, dim3((unsigned)div_up((long long)n, 256)), dim3(256), 0, stream, V, HW,
                       dout, color, alpha, bg, layout, dcolor, dalpha, dbg);
    return;
  }
  hipLaunchKernelGGL(k_composite_bwd, dim3((unsigned)div_up((long long)n, 256)), dim3(256), 0, stream, V, HW, dout,
                     color, alpha, bg, layout, dcolor, dalpha, dbg);
}

}  // namespace gsr

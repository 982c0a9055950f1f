// gsr_shading.hip — fused post-raster epilogue of the shading / SuGaR renderers.
//
// The reference follows every rasterizer call of the MVDream shading renderer with ~25 torch ops per
// view (renderer/diff_gaussian_rasterizer_shading.py:169-208, Depth2Normal :22-51, material
// material/gaussian_material.py:41-104), and the SuGaR normal renderer with the depth-normal part of
// them (renderer/diff_sugar_rasterizer_normal.py:170-197):
//     X      = rays_o + depth * rays_d                                  (xyz_map, HWC)
//     a, b   = X[x+1] - X[x-1],  X[y+1] - X[y-1]                        (3x3 conv, zero padding of X)
//     u      = normalize(-(a x b))                                      (F.normalize, eps 1e-12)
//     nmap   = u * 0.5 * alpha + 0.5                                    (gradient only where alpha > 0.99)
//   material + composite (flag GSR_SHADE_MATERIAL):
//     s      = u, or normalize(2 * pred_normal - 1) (detached) when a predicted normal map is given
//     l      = normalize(light - X);  t = max(s . l, 0) * kd + ka
//     albedo = color / (alpha + 1e-6)
//     fg     = clamp(albedo, 0, 1) * t | albedo | t                     (diffuse | albedo | textureless)
//     render = clamp(fg * alpha + (1 - alpha) * bg, 0, 1)
//   depth_out = depth with its gradient kept only where alpha > 0.99 (the in-place detach of :206-208).
//
// Layout: per-view planes (V, 3, H, W) for color / render / normal maps, (V, 1, H, W) depth / alpha,
// (V, H, W, 3) rays and background image (the reference's HWC tensors), (V, 3) light positions.
//
// One 256-thread workgroup per 32x8 pixel tile.  The forward stages X for the tile plus a 1-pixel halo
// in LDS (the central differences), then each thread finishes its pixel.  The backward is one fused
// pass too: X for a 2-pixel halo in LDS; every pixel of the tile plus a 1-pixel halo runs the
// pointwise backward and leaves its two cross-product gradients Ga = gu' x b, Gb = a x gu' in LDS
// (gu' = dL/d(-n)); then dL/dX[p] = Ga[p-x] - Ga[p+x] + Gb[p-y] - Gb[p+y] + light term, and
// dL/ddepth = dL/dX . rays_d (+ masked dL/ddepth_out).  The halo's recomputation (1.33x the tile) is
// cheaper than a round trip of 24 B/pixel of G through HBM.  Bytes per pixel: forward 56 read /
// 40 written, backward 96 read / 32 written (full material path).
#include "../../include/gsr.h"
#include "gsr_kernels.h"

namespace gsr {

namespace {

constexpr int STX = 32, STY = 8;  // tile
constexpr float kEps = 1e-12f;

struct P3 {
  float x, y, z;
};
__device__ __forceinline__ P3 p3(float x, float y, float z) { return P3{x, y, z}; }
__device__ __forceinline__ P3 sub3(P3 a, P3 b) { return p3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ P3 cross3(P3 a, P3 b) {
  return p3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ float dot3(P3 a, P3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float comp(P3 a, int c) { return c == 0 ? a.x : (c == 1 ? a.y : a.z); }

// F.normalize backward: y = x / max(|x|, eps);  dx = g / den - x (g . x) / (den^2 |x|) [|x| >= eps]
__device__ __forceinline__ P3 normalize_bwd(P3 x, float len, P3 g) {
  const float den = fmaxf(len, kEps);
  const float inv = 1.0f / den;
  P3 dx = p3(g.x * inv, g.y * inv, g.z * inv);
  if (len >= kEps && len > 0.0f) {
    // here den == len: dden / len = dden * inv (one reciprocal per normalisation)
    const float dden = -dot3(g, x) * inv * inv;
    const float k = dden * inv;
    dx.x += k * x.x;
    dx.y += k * x.y;
    dx.z += k * x.z;
  }
  return dx;
}

__device__ __forceinline__ float bg_at(const ShadeArgs& A, int v, size_t HW, size_t p, int c) {
  return A.bg_layout == 0 ? A.bg[3 * v + c] : A.bg[((size_t)v * HW + p) * 3 + c];
}

// X = rays_o + depth * rays_d at image position (x, y) of view v, 0 outside the image (zero padding)
__device__ __forceinline__ P3 load_X(const ShadeArgs& A, int v, int x, int y) {
  if (x < 0 || y < 0 || x >= A.W || y >= A.H) return p3(0.f, 0.f, 0.f);
  const size_t HW = (size_t)A.H * A.W, p = (size_t)y * A.W + x;
  const float z = A.depth[(size_t)v * HW + p];
  const float* o = A.rays_o + ((size_t)v * HW + p) * 3;
  const float* d = A.rays_d + ((size_t)v * HW + p) * 3;
  return p3(o[0] + z * d[0], o[1] + z * d[1], o[2] + z * d[2]);
}

// shading normal from a predicted normal map: normalize(2 p - 1), detached
__device__ __forceinline__ P3 pred_normal(const ShadeArgs& A, int v, size_t HW, size_t p) {
  const float* q = A.pred_normal + (size_t)v * 3 * HW + p;
  const P3 s = p3(q[0] * 2.0f - 1.0f, q[HW] * 2.0f - 1.0f, q[2 * HW] * 2.0f - 1.0f);
  const float den = fmaxf(sqrtf(dot3(s, s)), kEps);
  return p3(s.x / den, s.y / den, s.z / den);
}

}  // namespace

__global__ __launch_bounds__(256) void k_shade_fwd(ShadeArgs A) {
#pragma clang fp contract(off)
  __shared__ float sX[3][STY + 2][STX + 2];
  const int lv = blockIdx.z, v = A.v0 + lv;
  const int x0 = blockIdx.x * STX, y0 = blockIdx.y * STY;
  const int t = threadIdx.x;
  for (int i = t; i < (STX + 2) * (STY + 2); i += 256) {
    const int ly = i / (STX + 2), lx = i - ly * (STX + 2);
    const P3 X = load_X(A, v, x0 + lx - 1, y0 + ly - 1);
    sX[0][ly][lx] = X.x;
    sX[1][ly][lx] = X.y;
    sX[2][ly][lx] = X.z;
  }
  __syncthreads();
  const int lx = t % STX, ly = t / STX;
  const int x = x0 + lx, y = y0 + ly;
  if (x >= A.W || y >= A.H) return;
  const size_t HW = (size_t)A.H * A.W, p = (size_t)y * A.W + x;
  const int cx = lx + 1, cy = ly + 1;
  const P3 a = p3(sX[0][cy][cx + 1] - sX[0][cy][cx - 1], sX[1][cy][cx + 1] - sX[1][cy][cx - 1],
                  sX[2][cy][cx + 1] - sX[2][cy][cx - 1]);
  const P3 b = p3(sX[0][cy + 1][cx] - sX[0][cy - 1][cx], sX[1][cy + 1][cx] - sX[1][cy - 1][cx],
                  sX[2][cy + 1][cx] - sX[2][cy - 1][cx]);
  const P3 c = cross3(a, b);
  const P3 n = p3(-c.x, -c.y, -c.z);
  const float len = sqrtf(dot3(n, n));
  const float den = fmaxf(len, kEps);
  const P3 u = p3(n.x / den, n.y / den, n.z / den);
  const float al = A.alpha[(size_t)v * HW + p];
  const size_t plane = (size_t)v * 3 * HW + p;
  if (A.unit != nullptr) {
    A.unit[plane] = u.x;
    A.unit[plane + HW] = u.y;
    A.unit[plane + 2 * HW] = u.z;
  }
  if (A.nmap != nullptr) {
#pragma unroll
    for (int k = 0; k < 3; ++k) A.nmap[plane + k * HW] = comp(u, k) * 0.5f * al + 0.5f;
  }
  if (A.depth_out != nullptr) A.depth_out[(size_t)v * HW + p] = A.depth[(size_t)v * HW + p];
  if (!(A.flags & GSR_SHADE_MATERIAL)) return;

  const P3 X = p3(sX[0][cy][cx], sX[1][cy][cx], sX[2][cy][cx]);
  const P3 s = A.pred_normal != nullptr ? pred_normal(A, v, HW, p) : u;
  const P3 L = sub3(p3(A.light[3 * v], A.light[3 * v + 1], A.light[3 * v + 2]), X);
  const float lden = fmaxf(sqrtf(dot3(L, L)), kEps);
  const P3 l = p3(L.x / lden, L.y / lden, L.z / lden);
  const float dl = fmaxf(dot3(s, l), 0.0f);
  const float ad = al + 1e-6f;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float tl = dl * A.kd[lv][k] + A.ka[lv][k];
    const float alb = A.color[plane + k * HW] / ad;
    const float fg = A.mode[lv] == GSR_SHADING_DIFFUSE ? fminf(fmaxf(alb, 0.0f), 1.0f) * tl
                                                       : (A.mode[lv] == GSR_SHADING_ALBEDO ? alb : tl);
    const float img = fg * al + (1.0f - al) * bg_at(A, v, HW, p, k);
    A.render[plane + k * HW] = fminf(fmaxf(img, 0.0f), 1.0f);
  }
}

// Pointwise backward at one pixel.  Returns the two cross-product gradients (Ga, Gb) of its normal;
// for an interior pixel (`own`) also writes the colour / alpha / background gradients and returns the
// light-direction part of dL/dX in *dX.
__device__ __forceinline__ void shade_bwd_pixel(const ShadeArgs& A, const ShadeGrads& G, int v, int x, int y,
                                                const float (*sX)[STY + 4][STX + 4], int cx, int cy, bool own,
                                                P3* Ga, P3* Gb, P3* dX) {
#pragma clang fp contract(off)
  const size_t HW = (size_t)A.H * A.W, p = (size_t)y * A.W + x;
  const size_t plane = (size_t)v * 3 * HW + p;
  const int lv = v - A.v0;
  const int mode = A.mode[lv];
  const P3 a = p3(sX[0][cy][cx + 1] - sX[0][cy][cx - 1], sX[1][cy][cx + 1] - sX[1][cy][cx - 1],
                  sX[2][cy][cx + 1] - sX[2][cy][cx - 1]);
  const P3 b = p3(sX[0][cy + 1][cx] - sX[0][cy - 1][cx], sX[1][cy + 1][cx] - sX[1][cy - 1][cx],
                  sX[2][cy + 1][cx] - sX[2][cy - 1][cx]);
  const P3 c = cross3(a, b);
  const P3 n = p3(-c.x, -c.y, -c.z);
  const float len = sqrtf(dot3(n, n));
  // the recomputed forward values that decide a clamp mask (the unit normal and light direction feed
  // dot >= 0 and the image clamp, the albedo its own clamp) use the forward kernel's IEEE divides, so
  // every mask matches the forward's — and torch autograd's — decision bit for bit; the gradient
  // arithmetic below uses one reciprocal per normalisation
  const float den = fmaxf(len, kEps);
  const P3 u = p3(n.x / den, n.y / den, n.z / den);
  const float al = A.alpha[(size_t)v * HW + p];
  const bool m = al > 0.99f;
  P3 gu = p3(0.f, 0.f, 0.f);
  float dal = 0.0f;
  if (m) {
    if (G.d_unit != nullptr) gu = p3(G.d_unit[plane], G.d_unit[plane + HW], G.d_unit[plane + 2 * HW]);
    if (G.d_nmap != nullptr) {
      const P3 gn = p3(G.d_nmap[plane], G.d_nmap[plane + HW], G.d_nmap[plane + 2 * HW]);
      const float h = 0.5f * al;
      gu = p3(gu.x + gn.x * h, gu.y + gn.y * h, gu.z + gn.z * h);
      dal += (gn.x * u.x + gn.y * u.y + gn.z * u.z) * 0.5f;
    }
  }
  P3 dXl = p3(0.f, 0.f, 0.f);
  if ((A.flags & GSR_SHADE_MATERIAL) && G.d_render != nullptr) {
    const P3 X = p3(sX[0][cy][cx], sX[1][cy][cx], sX[2][cy][cx]);
    const bool own_normal = A.pred_normal == nullptr;
    const P3 s = own_normal ? u : pred_normal(A, v, HW, p);
    const P3 L = sub3(p3(A.light[3 * v], A.light[3 * v + 1], A.light[3 * v + 2]), X);
    const float llen = sqrtf(dot3(L, L));
    const float lden = fmaxf(llen, kEps);
    const P3 l = p3(L.x / lden, L.y / lden, L.z / lden);
    const float dt = dot3(s, l);
    const float dl = fmaxf(dt, 0.0f);
    const float rad = 1.0f / (al + 1e-6f);
    float ddl = 0.0f;
    float dad = 0.0f;
    float gcol[3], gbg[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float tl = dl * A.kd[lv][k] + A.ka[lv][k];
      const float col = A.color[plane + k * HW];
      const float alb = col / (al + 1e-6f);
      const float albc = fminf(fmaxf(alb, 0.0f), 1.0f);
      const float fg = mode == GSR_SHADING_DIFFUSE ? albc * tl : (mode == GSR_SHADING_ALBEDO ? alb : tl);
      const float bgk = bg_at(A, v, HW, p, k);
      const float img = fg * al + (1.0f - al) * bgk;
      const float gi = (img >= 0.0f && img <= 1.0f) ? G.d_render[plane + k * HW] : 0.0f;
      const float dfg = gi * al;
      dal += gi * (fg - bgk);
      gbg[k] = gi * (1.0f - al);
      float dalb = 0.0f, dtl = 0.0f;
      if (mode == GSR_SHADING_DIFFUSE) {
        dalb = (alb >= 0.0f && alb <= 1.0f) ? dfg * tl : 0.0f;
        dtl = dfg * albc;
      } else if (mode == GSR_SHADING_ALBEDO) {
        dalb = dfg;
      } else {
        dtl = dfg;
      }
      ddl += dtl * A.kd[lv][k];
      gcol[k] = dalb * rad;
      dad -= dalb * alb * rad;  // col / ad^2 = alb / ad
    }
    dal += dad;
    if (own) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        if (G.d_color != nullptr) G.d_color[plane + k * HW] = gcol[k];
      }
      if (G.d_bg != nullptr && A.bg_layout != 0) {
        float* o = G.d_bg + ((size_t)v * HW + p) * 3;
        o[0] = gbg[0];
        o[1] = gbg[1];
        o[2] = gbg[2];
      }
    }
    const float ddt = dt >= 0.0f ? ddl : 0.0f;
    if (own_normal) gu = p3(gu.x + ddt * l.x, gu.y + ddt * l.y, gu.z + ddt * l.z);
    const P3 dlv = normalize_bwd(L, llen, p3(ddt * s.x, ddt * s.y, ddt * s.z));
    dXl = p3(-dlv.x, -dlv.y, -dlv.z);
  } else if (own && G.d_color != nullptr) {
#pragma unroll
    for (int k = 0; k < 3; ++k) G.d_color[plane + k * HW] = 0.0f;
  }
  // u = n / den, n = -(a x b): dL/da = gn' x b... with gc = -gn: Ga = b x gc = gn x b, Gb = gc x a = a x gn
  const P3 gn = normalize_bwd(n, len, gu);
  *Ga = cross3(gn, b);
  *Gb = cross3(a, gn);
  if (own) {
    if (G.d_alpha != nullptr) G.d_alpha[(size_t)v * HW + p] = dal;
    *dX = dXl;
  }
}

__global__ __launch_bounds__(256) void k_shade_bwd(ShadeArgs A, ShadeGrads G) {
#pragma clang fp contract(off)
  __shared__ float sX[3][STY + 4][STX + 4];
  __shared__ float sG[6][STY + 2][STX + 2];
  const int v = A.v0 + (int)blockIdx.z;
  const int x0 = blockIdx.x * STX, y0 = blockIdx.y * STY;
  const int t = threadIdx.x;
  for (int i = t; i < (STX + 4) * (STY + 4); i += 256) {
    const int ly = i / (STX + 4), lx = i - ly * (STX + 4);
    const P3 X = load_X(A, v, x0 + lx - 2, y0 + ly - 2);
    sX[0][ly][lx] = X.x;
    sX[1][ly][lx] = X.y;
    sX[2][ly][lx] = X.z;
  }
  __syncthreads();
  // pass 1: the thread's own pixel (interior); pass 2: halo ring of the G region
  const int lx = t % STX, ly = t / STX;
  const int x = x0 + lx, y = y0 + ly;
  P3 dX = p3(0.f, 0.f, 0.f);
  {
    P3 Ga = p3(0.f, 0.f, 0.f), Gb = Ga;
    if (x < A.W && y < A.H) shade_bwd_pixel(A, G, v, x, y, sX, lx + 2, ly + 2, true, &Ga, &Gb, &dX);
    sG[0][ly + 1][lx + 1] = Ga.x;
    sG[1][ly + 1][lx + 1] = Ga.y;
    sG[2][ly + 1][lx + 1] = Ga.z;
    sG[3][ly + 1][lx + 1] = Gb.x;
    sG[4][ly + 1][lx + 1] = Gb.y;
    sG[5][ly + 1][lx + 1] = Gb.z;
  }
  constexpr int RING = 2 * (STX + 2) + 2 * STY;  // 84 halo entries
  if (t < RING) {
    int gx, gy;  // G-region coordinates (0..STX+1, 0..STY+1)
    if (t < STX + 2) {
      gx = t, gy = 0;
    } else if (t < 2 * (STX + 2)) {
      gx = t - (STX + 2), gy = STY + 1;
    } else if (t < 2 * (STX + 2) + STY) {
      gx = 0, gy = t - 2 * (STX + 2) + 1;
    } else {
      gx = STX + 1, gy = t - 2 * (STX + 2) - STY + 1;
    }
    const int hx = x0 + gx - 1, hy = y0 + gy - 1;
    P3 Ga = p3(0.f, 0.f, 0.f), Gb = Ga, unused;
    if (hx >= 0 && hy >= 0 && hx < A.W && hy < A.H)
      shade_bwd_pixel(A, G, v, hx, hy, sX, gx + 1, gy + 1, false, &Ga, &Gb, &unused);
    sG[0][gy][gx] = Ga.x;
    sG[1][gy][gx] = Ga.y;
    sG[2][gy][gx] = Ga.z;
    sG[3][gy][gx] = Gb.x;
    sG[4][gy][gx] = Gb.y;
    sG[5][gy][gx] = Gb.z;
  }
  __syncthreads();
  if (x >= A.W || y >= A.H) return;
  const size_t HW = (size_t)A.H * A.W, p = (size_t)y * A.W + x;
  const int cx = lx + 1, cy = ly + 1;
  // a(y, x-1) = X(y, x) - X(y, x-2): +Ga(x-1); a(y, x+1) = X(y, x+2) - X(y, x): -Ga(x+1); same in y with Gb
  float g[3];
#pragma unroll
  for (int k = 0; k < 3; ++k)
    g[k] = comp(dX, k) + ((sG[k][cy][cx - 1] - sG[k][cy][cx + 1]) + (sG[3 + k][cy - 1][cx] - sG[3 + k][cy + 1][cx]));
  const float* d = A.rays_d + ((size_t)v * HW + p) * 3;
  float dz = g[0] * d[0] + g[1] * d[1] + g[2] * d[2];
  if (G.d_depth_out != nullptr && A.alpha[(size_t)v * HW + p] > 0.99f) dz += G.d_depth_out[(size_t)v * HW + p];
  G.d_depth[(size_t)v * HW + p] = dz;
}

void launch_shade_fwd(const ShadeArgs& A, hipStream_t stream) {
  const dim3 grid((unsigned)div_up(A.W, STX), (unsigned)div_up(A.H, STY), (unsigned)A.V);
  hipLaunchKernelGGL(k_shade_fwd, grid, dim3(256), 0, stream, A);
}

void launch_shade_bwd(const ShadeArgs& A, const ShadeGrads& G, hipStream_t stream) {
  const dim3 grid((unsigned)div_up(A.W, STX), (unsigned)div_up(A.H, STY), (unsigned)A.V);
  hipLaunchKernelGGL(k_shade_bwd, grid, dim3(256), 0, stream, A, G);
}

}  // namespace gsr

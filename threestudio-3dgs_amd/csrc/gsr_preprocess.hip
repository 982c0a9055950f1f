// gsr_preprocess.hip — per-Gaussian forward preprocess.
//
// Replaces FORWARD::preprocessCUDA of the reference rasterizer [EXT]: frustum cull
// (view z <= 0.2), projection, 3D covariance, EWA 2D covariance (+0.3 low-pass), conic,
// 3-sigma radius, 16x16 tile rect, SH -> RGB (clamped at 0, flags kept for backward).
// A block owns 128 Gaussians (two threads each) for up to GSR_PRE_VIEWS views of the set: the
// Gaussians' parameters are read once per block (SH staged through LDS with coalesced 16-byte loads
// instead of 3M strided dword loads per thread), the 3D covariance is built once, and the views
// are walked in turn.  Writes per (view, Gaussian) the 64-byte render record (incl. tile rect and
// clamp flags), radius, rectangle / kept tile counts and the depth-sort key (culled: ~0, which
// sorts after every visible depth).
#include "gsr_kernels.h"
#include "gsr_math.h"

namespace gsr {

void launch_preprocess_kernel(const PreprocessArgs& a, const SetCams& cams, const GeomState& g, hipStream_t stream);

// Views handled by one block (the Gaussians' view-independent work and SH staging are shared): the
// block's 256 threads are 128 Gaussians x 2 halves of the views, so the SH staging (128 x (3M + 1)
// floats, 24.6 KB at SH3) allows 6 blocks = 6 waves per SIMD instead of 3 with 256 Gaussians.
// 64 views per block (8 / 16 / 32 / 64: 0.032 / 0.030 / 0.0285 / 0.0276 ms per view at C3,
// profiles/r04/pre_views_ab.txt): the SH staging and the 3D covariance amortise over more views; a 64-view set
// gives 7813 blocks (30 per CU).
#ifndef GSR_PRE_VIEWS
#define GSR_PRE_VIEWS 64
#endif
#define GSR_PRE_GAUSS 128
#define GSR_PRE_LDS_FLOATS (8 * 1024)  // SH staging up to 32 KB (M <= 21); larger M reads SH from HBM

// (6 waves per SIMD: 86 -> 79 VGPRs without spills; the LDS allows 6 blocks — 1 % faster)
// SH_LDS: the SH coefficients are staged (known at compile time, so the SH evaluation reads them with ds_read,
// not flat loads through a pointer that may point either way)
template <bool SH_LDS>
__attribute__((amdgpu_waves_per_eu(6, 8)))
__global__ __launch_bounds__(256) void k_preprocess(PreprocessArgs a, SetCams cams, GeomState g) {
  extern __shared__ float s_sh[];  // [128][3M + 1] this block's SH coefficients (odd stride)
  const int nvc = (a.V + GSR_PRE_VIEWS - 1) / GSR_PRE_VIEWS;
  const int vc = blockIdx.x % nvc;
  const int idx0 = (blockIdx.x / nvc) * GSR_PRE_GAUSS;
  const int t = threadIdx.x;
  const int gl = t % GSR_PRE_GAUSS;
  const int half = __builtin_amdgcn_readfirstlane(t / GSR_PRE_GAUSS);  // wave-uniform: scalar camera loads
  const int idx = idx0 + gl;
  const int vb = vc * GSR_PRE_VIEWS, ve = min(a.V, vb + GSR_PRE_VIEWS);
  const int vh = (ve - vb + 1) / 2;
  const int v0 = vb + half * vh, v1 = half == 0 ? min(ve, vb + vh) : ve;
  const int nsh = a.colors_precomp == nullptr ? 3 * a.M : 0;
  const int sstride = nsh + 1;
  const bool staged = SH_LDS;  // (host: nsh > 0 && GSR_PRE_GAUSS * sstride <= GSR_PRE_LDS_FLOATS)
  if (staged) {
    // coalesced 16-byte loads of the block's contiguous SH slice (256 * 3M floats, 16-B aligned)
    const int n = min(GSR_PRE_GAUSS, a.P - idx0) * nsh;
    const float4* src = reinterpret_cast<const float4*>(a.shs + (size_t)idx0 * nsh);
    // (row = e / nsh through a float reciprocal: exact for e < 2^14, and a few instructions instead of an
    // integer division per element — it matters for one-view launches, where the staging is not amortised)
    const float inv_nsh = 1.0f / (float)nsh;
    for (int e4 = t; e4 * 4 < n; e4 += 256) {
      const float4 q = src[e4];
      const float qv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = 4 * e4 + k;
        const int r = (int)(((float)e + 0.5f) * inv_nsh);
        if (e < n) s_sh[r * sstride + (e - r * nsh)] = qv[k];
      }
    }
    __syncthreads();
  }
  // threads past P run on the block's first Gaussian without writing (every wave stays whole for the
  // depth-range reduction at the end)
  const bool valid = idx < a.P;
  const int ix = valid ? idx : idx0;
  uint32_t kmn = 0xFFFFFFFFu, kmx = 0u;  // this thread's visible depth keys

  // view-independent: position, 3D covariance, opacity, precomputed colour
  const float3 p_orig = make_float3(a.means3D[3 * ix], a.means3D[3 * ix + 1], a.means3D[3 * ix + 2]);
  float cov3D[6];
  if (a.cov3D_precomp != nullptr) {
#pragma unroll
    for (int i = 0; i < 6; ++i) cov3D[i] = a.cov3D_precomp[6 * ix + i];
  } else {
    const float3 s = make_float3(a.scales[3 * ix], a.scales[3 * ix + 1], a.scales[3 * ix + 2]);
    const float4 q = make_float4(a.rotations[4 * ix], a.rotations[4 * ix + 1],
                                 a.rotations[4 * ix + 2], a.rotations[4 * ix + 3]);
    cov3d_from_scale_rot(s, a.scale_modifier, q, cov3D);
  }
  const float opacity = a.opacities[ix];
  float3 rgb_pre = make_float3(0.f, 0.f, 0.f);
  if (a.colors_precomp != nullptr)
    rgb_pre = make_float3(a.colors_precomp[3 * ix], a.colors_precomp[3 * ix + 1], a.colors_precomp[3 * ix + 2]);
  const float* my_sh = staged ? s_sh + gl * sstride : a.shs + (size_t)ix * nsh;
  // the two-colour render's second colour, carried in the record's free slots (b.w, c.w, d.z; GaussRec)
  float3 c2 = make_float3(0.f, 0.f, 0.f);
  if (a.col2 != nullptr) c2 = make_float3(a.col2[3 * ix], a.col2[3 * ix + 1], a.col2[3 * ix + 2]);
  const int gx = (a.W + GSR_TILE_X - 1) / GSR_TILE_X;
  const int gy = (a.H + GSR_TILE_Y - 1) / GSR_TILE_Y;

#pragma unroll 1
  for (int v = v0; v < v1; ++v) {
    const ViewCam cam = cams.c[v];
    const size_t vi = (size_t)v * a.P + idx;
    // the view's matrices through the constant address space: wave-uniform addresses -> s_load
    typedef __attribute__((address_space(4))) const float* cfptr;
    float viewmatrix[16], projmatrix[16], cpos[3];
#pragma unroll
    for (int i = 0; i < 16; ++i) viewmatrix[i] = ((cfptr)cam.view)[i], projmatrix[i] = ((cfptr)cam.proj)[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) cpos[i] = ((cfptr)cam.campos)[i];
    const float tanfovx = cam.tanx, tanfovy = cam.tany;
    const float focal_x = cam.fx, focal_y = cam.fy;
    int radius = 0;
    uint2 tiles = make_uint2(0u, 0u);
    uint32_t dkey = 0xFFFFFFFFu;  // culled: sorts after every visible depth
    // near-plane cull on the view-space depth (in_frustum of the reference)
    const float3 p_view = xform_point4x3(p_orig, viewmatrix);
    if (p_view.z > GSR_NEAR_CULL) {
      const float4 p_hom = xform_point4x4(p_orig, projmatrix);
      const float p_w = 1.0f / (p_hom.w + 0.0000001f);
      const float3 p_proj = make_float3(p_hom.x * p_w, p_hom.y * p_w, p_hom.z * p_w);
      Cov2DState st;
      const float3 cov = cov2d_ewa(p_orig, focal_x, focal_y, tanfovx, tanfovy, cov3D, viewmatrix, st);
      const float det = cov.x * cov.z - cov.y * cov.y;
      if (det != 0.0f) {
        const float det_inv = 1.f / det;
        const float3 conic = make_float3(cov.z * det_inv, -cov.y * det_inv, cov.x * det_inv);
        const float mid = 0.5f * (cov.x + cov.z);
        const float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
        const float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
        const float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
        const float2 pimg = make_float2(ndc2pix(p_proj.x, a.W), ndc2pix(p_proj.y, a.H));
        // tile rect [min, max) clamped to the grid (getRect of the reference)
        const int r = (int)my_radius;
        const int xmin = min(gx, max(0, (int)((pimg.x - r) / GSR_TILE_X)));
        const int ymin = min(gy, max(0, (int)((pimg.y - r) / GSR_TILE_Y)));
        const int xmax = min(gx, max(0, (int)((pimg.x + r + GSR_TILE_X - 1) / GSR_TILE_X)));
        const int ymax = min(gy, max(0, (int)((pimg.y + r + GSR_TILE_Y - 1) / GSR_TILE_Y)));
        const int area = (xmax - xmin) * (ymax - ymin);
        if (area != 0) {
          float3 rgb = rgb_pre;
          uint32_t clamp_bits = 0;
          if (a.colors_precomp == nullptr)
            rgb = sh_to_rgb(a.deg, my_sh, p_orig, make_float3(cpos[0], cpos[1], cpos[2]),
                            &clamp_bits);
          GaussRec rec;
          rec.a = make_float4(pimg.x, pimg.y, conic.x, conic.y);
          rec.b = make_float4(conic.z, opacity, p_view.z, c2.x);
          rec.c = make_float4(rgb.x, rgb.y, rgb.z, c2.y);
          rec.d = make_uint4((uint32_t)xmin | ((uint32_t)ymin << 16), (uint32_t)xmax | ((uint32_t)ymax << 16),
                             __float_as_uint(c2.z), clamp_bits);
          if (valid) g.rec[vi] = rec;
          radius = r;
          uint32_t kept = 0;
          const SpanPrep sp = span_prep(rec.a.x, rec.a.y, rec.a.z, rec.a.w, rec.b.x, rec.b.y);
          for (int ty = ymin; ty < ymax; ++ty) {
            int t0, t1;
            span_row(sp, ty, xmin, xmax, t0, t1);
            kept += (uint32_t)(t1 - t0);
          }
          tiles = make_uint2((uint32_t)area, kept);
          dkey = __float_as_uint(p_view.z);  // > 0.2: float bits are monotone in depth
        }
      }
    }
    if (valid) {
      a.radii[vi] = radius;
      g.tiles[vi] = tiles;
      g.dkey[0][vi] = dkey;
      // the depth sort's value: index | kept tiles (k_inst_count reads them in depth order, streaming)
      const uint32_t ks = g.vsent();
      g.dval[0][vi] = (uint32_t)idx | (g.vbits <= 26 ? min(tiles.y, ks) << g.vbits : 0u);
      if (dkey != 0xFFFFFFFFu) kmn = min(kmn, dkey), kmx = max(kmx, dkey);
    }
  }
  // the set's visible depth-key range (rebases the depth sort: 3 passes when it spans < 24 bits):
  // wave -> block reduction, then one atomic pair per block into one of 64 slots
  __shared__ uint32_t s_rng[2][4];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    kmn = min(kmn, (uint32_t)__shfl_xor((int)kmn, o, 64));
    kmx = max(kmx, (uint32_t)__shfl_xor((int)kmx, o, 64));
  }
  if ((t & 63) == 0) s_rng[0][t >> 6] = kmn, s_rng[1][t >> 6] = kmx;
  __syncthreads();
  if (t == 0) {
    kmn = min(min(s_rng[0][0], s_rng[0][1]), min(s_rng[0][2], s_rng[0][3]));
    kmx = max(max(s_rng[1][0], s_rng[1][1]), max(s_rng[1][2], s_rng[1][3]));
    if (kmn != 0xFFFFFFFFu) {
      atomicMin(&g.drange[blockIdx.x & 63], kmn);
      atomicMax(&g.drange[64 + (blockIdx.x & 63)], kmx);
    }
  }
}

__global__ void k_depth_range_init(uint32_t* drange, unsigned long long col2) {
  drange[threadIdx.x] = 0xFFFFFFFFu;
  drange[64 + threadIdx.x] = 0u;
  if (threadIdx.x < 2) drange[130 + threadIdx.x] = (uint32_t)(col2 >> (32 * threadIdx.x));  // (see GaussRec)
}

// Fold the 64 slots: [128] = smallest visible key, [129] = 1 when every rebased visible key is below
// 2^24 - 1 (the culled marker ~0 then still ranks last after 3 passes).
__global__ void k_depth_range(uint32_t* drange) {
  const int t = threadIdx.x;  // 64 threads
  uint32_t mn = drange[t], mx = drange[64 + t];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
  }
  if (t == 0) {
    const bool any = mn != 0xFFFFFFFFu;
    drange[128] = any ? mn : 0u;
    drange[129] = (!any || mx - mn < 0x00FFFFFFu) ? 1u : 0u;
  }
}

void launch_preprocess(const PreprocessArgs& a, const SetCams& cams, const GeomState& g, hipStream_t stream) {
  hipLaunchKernelGGL(k_depth_range_init, dim3(1), dim3(64), 0, stream, g.drange,
                     (unsigned long long)(uintptr_t)(a.P > 0 ? a.col2 : nullptr));
  if (a.P > 0 && a.V > 0) launch_preprocess_kernel(a, cams, g, stream);
  hipLaunchKernelGGL(k_depth_range, dim3(1), dim3(64), 0, stream, g.drange);
}

void launch_preprocess_kernel(const PreprocessArgs& a, const SetCams& cams, const GeomState& g, hipStream_t stream) {
  const int nvc = (a.V + GSR_PRE_VIEWS - 1) / GSR_PRE_VIEWS;
  const size_t want = a.colors_precomp == nullptr ? (size_t)GSR_PRE_GAUSS * (3 * a.M + 1) : 0;
  const bool sh_lds = a.colors_precomp == nullptr && a.M > 0 && want <= GSR_PRE_LDS_FLOATS;
  const size_t lds = sh_lds ? sizeof(float) * want : 0;
  hipLaunchKernelGGL(sh_lds ? k_preprocess<true> : k_preprocess<false>,
                     dim3(nvc * ((a.P + GSR_PRE_GAUSS - 1) / GSR_PRE_GAUSS)), dim3(256), lds, stream, a, cams, g);
}

}  // namespace gsr

// gsr_backward.hip — per-Gaussian backward of a view set.
//
// Two launches per group of views:
//   A. k_view_grad, per (view, Gaussian) of the Gaussians the view's blend reached (reach bits set by
//      k_render_bwd; the others only get their zero means2D gradient): gather-sum of the Gaussian's
//      per-instance gradient rows written by k_render_bwd (fixed order -> bitwise reproducible), with the
//      tile cut-offs of the view staged in LDS so the instances no pixel reached cost one LDS read each;
//      then BACKWARD::computeCov2DCUDA (conic -> 2D cov -> 3D cov and camera-space mean) and the
//      projection / view-depth part of BACKWARD::preprocessCUDA [EXT].  Writes the view's means2D
//      gradient and a 64-byte record slot (dmean3D, dcov3D, raw dcolor, dopacity, SH clamp bits).
//   B. k_gauss_accum, one thread per Gaussian: streams its reached views' records, runs the
//      SH -> RGB backward (incl. the view-direction term) per view with dL/dSH accumulated in
//      registers, then 3D cov -> scale and (unnormalised) quaternion once (linear in dL/dcov3D).
// Splitting at the view boundary keeps A light (≈70 VGPRs, thousands of waves in flight to hide the
// gather latency) and leaves only B to carry the 48 SH accumulators.
// Gradient conventions of the reference are kept: the 0.99 alpha clamp is ignored in
// dL/dG, the frustum clamp zeroes dL/dt_x,y only, denom2inv carries +1e-7, the scale gradient is
// w.r.t. scale_modifier * scale.
#include <cstdlib>
#include <cstring>

#include "gsr_kernels.h"
#include "gsr_math.h"
#include "gsr_wave.h"

namespace gsr {

struct RowSums {
  float dmx, dmy, dca, dcb, dcc, dop, dcr, dcg, dcbl, ddep;
  float dmx1, dmy1, dr2, dg2, db2;  // two-colour rows (gsr_common.h BackwardState)
};

// Sum the rows of the Gaussian's instances that its tile's blend reached: the kept tiles of its
// rectangle (span_row, as emitted) whose (depth key, index) < the tile's first unblended
// instance (cut = (key, index) per tile).  Rows sit at rectangle positions.  Tiles are walked 4 at
// a time: the 4 cut tests first, then the valid rows' loads together, so a thread has up to 12
// loads in flight instead of waiting on each row in turn.
template <bool TWO>
__device__ __forceinline__ RowSums gather_rows(uint32_t idx, const GaussRec& gr, uint32_t i0, int grid_x,
                                               const uint2* cut, const float4* grow) {
  RowSums r = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  constexpr int RW = TWO ? 4 : 3;
  const uint4 gd = gr.d;
  const float4 ga = gr.a, gb = gr.b;
  const uint32_t dkey = __float_as_uint(gb.z);
  const int xmin = gd.x & 0xffff, ymin = gd.x >> 16, xmax = gd.y & 0xffff, ymax = gd.y >> 16;
  const int w = xmax - xmin;
  const SpanPrep sp = span_prep(ga.x, ga.y, ga.z, ga.w, gb.x, gb.y);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int ty = ymin; ty < ymax; ++ty) {
    int t0, t1;
    span_row(sp, ty, xmin, xmax, t0, t1);  // the kept tiles of this row, as emitted
    for (int tx = t0; tx < t1; tx += 4) {
      bool val[4];
      int sl[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        val[k] = false;
        sl[k] = 0;
        if (tx + k < t1) {
          const uint2 c = cut[ty * grid_x + tx + k];
          val[k] = dkey < c.x || (dkey == c.x && idx < c.y);
          sl[k] = (ty - ymin) * w + (tx + k - xmin);
        }
      }
      float4 a[4][RW];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float4* row = grow + RW * ((size_t)i0 + sl[k]);
#pragma unroll
        for (int e = 0; e < RW; ++e) a[k][e] = val[k] ? row[e] : z4;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        r.dmx += a[k][0].x; r.dmy += a[k][0].y; r.dca += a[k][0].z; r.dcb += a[k][0].w;
        r.dcc += a[k][1].x; r.dop += a[k][1].y; r.dcr += a[k][1].z; r.dcg += a[k][1].w;
        r.dcbl += a[k][2].x; r.ddep += a[k][2].y;
        if (TWO) {
          r.dr2 += a[k][2].z; r.dg2 += a[k][2].w;
          r.db2 += a[k][RW - 1].x; r.dmx1 += a[k][RW - 1].y; r.dmy1 += a[k][RW - 1].z;
        }
      }
    }
  }
  return r;
}

// Camera of one view as the chain rule needs it.
struct ViewGeom {
  const float *view, *proj;
  float tanx, tany, fx, fy;
};

// computeCov2DCUDA: conic gradient -> dL/dcov3D (6, symmetric off-diagonals as scalars) and the
// camera-space-mean part of dL/dmean.
__device__ __forceinline__ void cov2d_backward(const float3 mean, const float cov3D[6], const ViewGeom& d,
                                               float dca, float dcb, float dcc, float dcov[6], float3& dmean) {
  Cov2DState st;
  const float3 cov2 = cov2d_ewa(mean, d.fx, d.fy, d.tanx, d.tany, cov3D, d.view, st);
  const float x_grad_mul = (st.txtz < -st.limx || st.txtz > st.limx) ? 0.f : 1.f;
  const float y_grad_mul = (st.tytz < -st.limy || st.tytz > st.limy) ? 0.f : 1.f;
  const float ca = cov2.x, cb = cov2.y, cc = cov2.z;
  const float denom = ca * cc - cb * cb;
  float dL_da = 0.f, dL_db = 0.f, dL_dc = 0.f;
  const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
  const float(&T)[2][3] = st.T;
#pragma unroll
  for (int k = 0; k < 6; ++k) dcov[k] = 0.f;
  if (denom2inv != 0.f) {
    dL_da = denom2inv * (-cc * cc * dca + 2 * cb * cc * dcb + (denom - ca * cc) * dcc);
    dL_dc = denom2inv * (-ca * ca * dcc + 2 * ca * cb * dcb + (denom - ca * cc) * dca);
    dL_db = denom2inv * 2 * (cb * cc * dca - (denom + 2 * cb * cb) * dcb + ca * cb * dcc);
    dcov[0] = (T[0][0] * T[0][0] * dL_da + T[0][0] * T[1][0] * dL_db + T[1][0] * T[1][0] * dL_dc);
    dcov[3] = (T[0][1] * T[0][1] * dL_da + T[0][1] * T[1][1] * dL_db + T[1][1] * T[1][1] * dL_dc);
    dcov[5] = (T[0][2] * T[0][2] * dL_da + T[0][2] * T[1][2] * dL_db + T[1][2] * T[1][2] * dL_dc);
    dcov[1] = 2 * T[0][0] * T[0][1] * dL_da + (T[0][0] * T[1][1] + T[0][1] * T[1][0]) * dL_db +
              2 * T[1][0] * T[1][1] * dL_dc;
    dcov[2] = 2 * T[0][0] * T[0][2] * dL_da + (T[0][0] * T[1][2] + T[0][2] * T[1][0]) * dL_db +
              2 * T[1][0] * T[1][2] * dL_dc;
    dcov[4] = 2 * T[0][2] * T[0][1] * dL_da + (T[0][1] * T[1][2] + T[0][2] * T[1][1]) * dL_db +
              2 * T[1][1] * T[1][2] * dL_dc;
  }
  const float V[3][3] = {{cov3D[0], cov3D[1], cov3D[2]},
                         {cov3D[1], cov3D[3], cov3D[4]},
                         {cov3D[2], cov3D[4], cov3D[5]}};
  float dT0[3], dT1[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float tv0 = T[0][0] * V[k][0] + T[0][1] * V[k][1] + T[0][2] * V[k][2];
    const float tv1 = T[1][0] * V[k][0] + T[1][1] * V[k][1] + T[1][2] * V[k][2];
    dT0[k] = 2 * tv0 * dL_da + tv1 * dL_db;
    dT1[k] = 2 * tv1 * dL_dc + tv0 * dL_db;
  }
  const float(&Wm)[3][3] = st.W;
  const float dJ00 = Wm[0][0] * dT0[0] + Wm[0][1] * dT0[1] + Wm[0][2] * dT0[2];
  const float dJ02 = Wm[2][0] * dT0[0] + Wm[2][1] * dT0[1] + Wm[2][2] * dT0[2];
  const float dJ11 = Wm[1][0] * dT1[0] + Wm[1][1] * dT1[1] + Wm[1][2] * dT1[2];
  const float dJ12 = Wm[2][0] * dT1[0] + Wm[2][1] * dT1[1] + Wm[2][2] * dT1[2];
  const float tz = 1.f / st.t.z, tz2 = tz * tz, tz3 = tz2 * tz;
  const float hx = d.fx, hy = d.fy;
  const float dtx = x_grad_mul * -hx * tz2 * dJ02;
  const float dty = y_grad_mul * -hy * tz2 * dJ12;
  const float dtz = -hx * tz2 * dJ00 - hy * tz2 * dJ11 + (2 * hx * st.t.x) * tz3 * dJ02 +
                    (2 * hy * st.t.y) * tz3 * dJ12;
  dmean = xform_vec4x3_T(make_float3(dtx, dty, dtz), d.view);
}

// preprocessCUDA: NDC-space mean gradient -> world-space mean through the projection.
__device__ __forceinline__ void proj_backward(const float3 mean, const float* proj, float dmx, float dmy,
                                              float3& dmean) {
  const float4 m_hom = xform_point4x4(mean, proj);
  const float m_w = 1.0f / (m_hom.w + 0.0000001f);
  const float mul1 = (proj[0] * mean.x + proj[4] * mean.y + proj[8] * mean.z + proj[12]) * m_w * m_w;
  const float mul2 = (proj[1] * mean.x + proj[5] * mean.y + proj[9] * mean.z + proj[13]) * m_w * m_w;
  dmean.x += (proj[0] * m_w - proj[3] * mul1) * dmx + (proj[1] * m_w - proj[3] * mul2) * dmy;
  dmean.y += (proj[4] * m_w - proj[7] * mul1) * dmx + (proj[5] * m_w - proj[7] * mul2) * dmy;
  dmean.z += (proj[8] * m_w - proj[11] * mul1) * dmx + (proj[9] * m_w - proj[11] * mul2) * dmy;
}

// computeColorFromSH backward for one view: accumulates basis x dL/dRGB into dsh (registers, 3 x 16,
// summed over views) and adds the view-direction term to dmean.  sh = the Gaussian's (M, 3) row (LDS).
__device__ __forceinline__ void sh_backward(int deg, int M, const float* sh, float (&dsh)[48], float3 dRGB,
                                            const float3 mean, const float* campos, float3& dmean) {
  const float3 dir_orig = make_float3(mean.x - campos[0], mean.y - campos[1], mean.z - campos[2]);
  const float len = sqrtf(dir_orig.x * dir_orig.x + dir_orig.y * dir_orig.y + dir_orig.z * dir_orig.z);
  const float x = dir_orig.x / len, y = dir_orig.y / len, z = dir_orig.z / len;
  float basis[16];
  float bdx[16], bdy[16], bdz[16];  // d basis_k / d (x, y, z)
#pragma unroll
  for (int k = 0; k < 16; ++k) basis[k] = bdx[k] = bdy[k] = bdz[k] = 0.f;
  basis[0] = SH_C0;
  if (deg > 0) {
    basis[1] = -SH_C1 * y; basis[2] = SH_C1 * z; basis[3] = -SH_C1 * x;
    bdy[1] = -SH_C1; bdz[2] = SH_C1; bdx[3] = -SH_C1;
    if (deg > 1) {
      const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
      basis[4] = SH_C2[0] * xy; basis[5] = SH_C2[1] * yz;
      basis[6] = SH_C2[2] * (2.f * zz - xx - yy); basis[7] = SH_C2[3] * xz;
      basis[8] = SH_C2[4] * (xx - yy);
      bdx[4] = SH_C2[0] * y; bdy[4] = SH_C2[0] * x;
      bdy[5] = SH_C2[1] * z; bdz[5] = SH_C2[1] * y;
      bdx[6] = SH_C2[2] * 2.f * -x; bdy[6] = SH_C2[2] * 2.f * -y; bdz[6] = SH_C2[2] * 2.f * 2.f * z;
      bdx[7] = SH_C2[3] * z; bdz[7] = SH_C2[3] * x;
      bdx[8] = SH_C2[4] * 2.f * x; bdy[8] = SH_C2[4] * 2.f * -y;
      if (deg > 2) {
        basis[9] = SH_C3[0] * y * (3.f * xx - yy);
        basis[10] = SH_C3[1] * xy * z;
        basis[11] = SH_C3[2] * y * (4.f * zz - xx - yy);
        basis[12] = SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy);
        basis[13] = SH_C3[4] * x * (4.f * zz - xx - yy);
        basis[14] = SH_C3[5] * z * (xx - yy);
        basis[15] = SH_C3[6] * x * (xx - 3.f * yy);
        bdx[9] = SH_C3[0] * 3.f * 2.f * xy;          bdy[9] = SH_C3[0] * 3.f * (xx - yy);
        bdx[10] = SH_C3[1] * yz;                     bdy[10] = SH_C3[1] * xz;          bdz[10] = SH_C3[1] * xy;
        bdx[11] = SH_C3[2] * -2.f * xy;              bdy[11] = SH_C3[2] * (-3.f * yy + 4.f * zz - xx);
        bdz[11] = SH_C3[2] * 4.f * 2.f * yz;
        bdx[12] = SH_C3[3] * -3.f * 2.f * xz;        bdy[12] = SH_C3[3] * -3.f * 2.f * yz;
        bdz[12] = SH_C3[3] * 3.f * (2.f * zz - xx - yy);
        bdx[13] = SH_C3[4] * (-3.f * xx + 4.f * zz - yy); bdy[13] = SH_C3[4] * -2.f * xy;
        bdz[13] = SH_C3[4] * 4.f * 2.f * xz;
        bdx[14] = SH_C3[5] * 2.f * xz;               bdy[14] = SH_C3[5] * -2.f * yz;   bdz[14] = SH_C3[5] * (xx - yy);
        bdx[15] = SH_C3[6] * 3.f * (xx - yy);        bdy[15] = SH_C3[6] * -3.f * 2.f * xy;
      }
    }
  }
  const int ncoef = (deg + 1) * (deg + 1);
  float3 dRGBdx = make_float3(0.f, 0.f, 0.f), dRGBdy = dRGBdx, dRGBdz = dRGBdx;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (k < ncoef && k < M) {
      dsh[3 * k] += basis[k] * dRGB.x;
      dsh[3 * k + 1] += basis[k] * dRGB.y;
      dsh[3 * k + 2] += basis[k] * dRGB.z;
      if (k > 0) {
        const float3 s = make_float3(sh[3 * k], sh[3 * k + 1], sh[3 * k + 2]);
        dRGBdx.x += bdx[k] * s.x; dRGBdx.y += bdx[k] * s.y; dRGBdx.z += bdx[k] * s.z;
        dRGBdy.x += bdy[k] * s.x; dRGBdy.y += bdy[k] * s.y; dRGBdy.z += bdy[k] * s.z;
        dRGBdz.x += bdz[k] * s.x; dRGBdz.y += bdz[k] * s.y; dRGBdz.z += bdz[k] * s.z;
      }
    }
  }
  const float3 ddir = make_float3(dRGBdx.x * dRGB.x + dRGBdx.y * dRGB.y + dRGBdx.z * dRGB.z,
                                  dRGBdy.x * dRGB.x + dRGBdy.y * dRGB.y + dRGBdy.z * dRGB.z,
                                  dRGBdz.x * dRGB.x + dRGBdz.y * dRGB.y + dRGBdz.z * dRGB.z);
  // d normalize(v) / dv applied to ddir
  const float3 v = dir_orig;
  const float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
  const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
  dmean.x += ((sum2 - v.x * v.x) * ddir.x - v.y * v.x * ddir.y - v.z * v.x * ddir.z) * invsum32;
  dmean.y += (-v.x * v.y * ddir.x + (sum2 - v.y * v.y) * ddir.y - v.z * v.y * ddir.z) * invsum32;
  dmean.z += (-v.x * v.z * ddir.x - v.y * v.z * ddir.y + (sum2 - v.z * v.z) * ddir.z) * invsum32;
}

// computeCov3D backward: dL/dcov3D -> dL/d(scale_modifier * scale) and dL/d(quaternion as given).
__device__ __forceinline__ void scale_rot_backward(const float3 scale, const float4 rot, float mod,
                                                   const float dcov[6], float ds[3], float dq[4]) {
  Mat3 R;
  rot_from_quat(rot, R);
  const float s[3] = {mod * scale.x, mod * scale.y, mod * scale.z};
  // E[c][k] = s_k R[c][k];  Sigma[c][r] = sum_k E[r][k] E[c][k]; dSigma symmetric, off-diagonals split
  const float G[3][3] = {{dcov[0], 0.5f * dcov[1], 0.5f * dcov[2]},
                         {0.5f * dcov[1], dcov[3], 0.5f * dcov[4]},
                         {0.5f * dcov[2], 0.5f * dcov[4], dcov[5]}};
  float dE[3][3];
#pragma unroll
  for (int aa = 0; aa < 3; ++aa)
#pragma unroll
    for (int k = 0; k < 3; ++k)
      dE[aa][k] = 2.f * (G[aa][0] * s[k] * R.m[0][k] + G[aa][1] * s[k] * R.m[1][k] + G[aa][2] * s[k] * R.m[2][k]);
  float dR[3][3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    ds[k] = dE[0][k] * R.m[0][k] + dE[1][k] * R.m[1][k] + dE[2][k] * R.m[2][k];
#pragma unroll
    for (int aa = 0; aa < 3; ++aa) dR[aa][k] = dE[aa][k] * s[k];
  }
  const float r = rot.x, x = rot.y, y = rot.z, z = rot.w;
  // d R[c][r'] / dq for R.m as built by rot_from_quat
  dq[0] = -2.f * z * dR[0][1] + 2.f * y * dR[0][2] + 2.f * z * dR[1][0] - 2.f * x * dR[1][2] -
          2.f * y * dR[2][0] + 2.f * x * dR[2][1];
  dq[1] = 2.f * y * dR[0][1] + 2.f * z * dR[0][2] + 2.f * y * dR[1][0] - 4.f * x * dR[1][1] -
          2.f * r * dR[1][2] + 2.f * z * dR[2][0] + 2.f * r * dR[2][1] - 4.f * x * dR[2][2];
  dq[2] = -4.f * y * dR[0][0] + 2.f * x * dR[0][1] + 2.f * r * dR[0][2] + 2.f * x * dR[1][0] +
          2.f * z * dR[1][2] - 2.f * r * dR[2][0] + 2.f * z * dR[2][1] - 4.f * y * dR[2][2];
  dq[3] = -4.f * z * dR[0][0] - 2.f * r * dR[0][1] + 2.f * x * dR[0][2] + 2.f * r * dR[1][0] -
          4.f * z * dR[1][1] + 2.f * y * dR[1][2] + 2.f * x * dR[2][0] + 2.f * y * dR[2][1];
}


// LDS row stride (floats) of one Gaussian's 3M SH values: 16-byte multiple plus 16 bytes of padding so
// per-thread 16-byte LDS accesses at this stride are bank-conflict free.
static inline __host__ __device__ int sh_lds_stride(int M) { return ((3 * M + 3) & ~3) + 4; }

// ---- A: per (view, Gaussian) ----------------------------------------------------------------
// Block b -> view b % V, Gaussians [4096 (b / V), +4096) (GSR_VG_ITEMS = 16 per thread, 256 apart; 4, 8,
// 16, 32 measured: 76, 73, 72, 72 us/view with the second stage): the views of one
// Gaussian slice run together, so its parameters come from HBM once per group.  LDS: the view's
// tile cut-offs (8 B per tile, loaded once per 4096 Gaussians).
#ifndef GSR_VG_ITEMS
#define GSR_VG_ITEMS 16
#endif
// (4 waves per SIMD for both variants: the two-colour one would otherwise take 136 VGPRs and 3 waves;
// capped it spills 4 VGPRs outside the row loop and its per-Gaussian backward is 4 % faster on C5)
// CUT_LDS (= va.cut_in_lds) at compile time: the cut-off reads are ds_read from the staged copy, not flat loads
// through a pointer that may be either (a flat load of LDS waits on both counters at the memory path's latency).
template <bool TWO, bool CUT_LDS>
__attribute__((amdgpu_waves_per_eu(4, 8)))
__global__ __launch_bounds__(256) void k_view_grad(GaussBackwardArgs a, ViewGradArgs va) {
  extern __shared__ uint2 s_cut[];
  const int t = threadIdx.x;
  const int vl = blockIdx.x % va.V;
  const int vg = va.v0 + vl;
  const uint2* cut = CUT_LDS ? reinterpret_cast<const uint2*>(s_cut) : va.img.cut + (size_t)vg * va.tiles;
  if (CUT_LDS) {
    const uint4* src = reinterpret_cast<const uint4*>(va.img.cut + (size_t)vg * va.tiles);
    uint4* dst = reinterpret_cast<uint4*>(s_cut);
    for (int k = t; k < va.tiles / 2; k += 256) dst[k] = src[k];
    if ((va.tiles & 1) && t == 0) s_cut[va.tiles - 1] = va.img.cut[(size_t)vg * va.tiles + va.tiles - 1];
    __syncthreads();
  }
  const ViewCam& cam = va.cam[vl];
  // the view's matrices through the constant address space (block-uniform view: s_load, no VGPRs);
  // focal lengths once per thread instead of once per item
  typedef __attribute__((address_space(4))) const float* cfptr;
  float viewm[16], projm[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) viewm[i] = ((cfptr)cam.view)[i], projm[i] = ((cfptr)cam.proj)[i];
  ViewGeom vgm;
  vgm.view = viewm;
  vgm.proj = projm;
  vgm.tanx = cam.tanx;
  vgm.tany = cam.tany;
  vgm.fy = va.H / (2.0f * cam.tany);
  vgm.fx = va.W / (2.0f * cam.tanx);
  const float4* grow = va.grow + (size_t)(TWO ? 4 : 3) * va.row_start[vl];
  constexpr int RS = TWO ? GSR_REC_STRIDE2 : GSR_REC_STRIDE;
  float4* recv = reinterpret_cast<float4*>(va.vrec + (size_t)vl * RS * a.P);
  const unsigned long long vbit = 1ull << vl;
  // Only the Gaussians this view's blend gave a gradient row (reach bit, set by k_render_bwd; ~20 % of a
  // view at 1M) are loaded and get a record; the others write their zero means2D gradient only
  // (k_gauss_accum reads the reached records only).  Pass 1: each wave reads the reach bits of its 1024
  // items (16 per lane, 256 apart), zeroes the unreached ones' means2D gradient and lists the reached ones
  // in LDS; pass 2: the wave's lanes take the listed items in turn, so a wave walks ~4 dense rounds of
  // gathers and chain rules instead of 16 sparse ones.  The next listed item's record is loaded while the
  // current one is processed.
  __shared__ uint16_t s_list[4][64 * GSR_VG_ITEMS];
  const int wave = t >> 6, lane = t & 63;
  uint16_t* list = s_list[wave];
  const int items = va.items;  // per thread (<= GSR_VG_ITEMS; fewer for launches of few views)
  const int slice = a.g0 + (blockIdx.x / va.V) * (256 * items);
  int cnt = 0;  // wave-uniform
#pragma unroll
  for (int it = 0; it < GSR_VG_ITEMS; ++it) {
    const int local = it * 256 + t;
    const int idx = slice + local;
    const bool valid = it < items && idx < a.g1;  // (it < items: uniform)
    const bool rch = valid && (va.reach[idx] & vbit) != 0ull;
    if (valid && !rch) {
      float* m2 = va.dmeans2D + 3 * ((size_t)vg * a.P + idx);
      m2[0] = 0.f;
      m2[1] = 0.f;
      m2[2] = 0.f;
    }
    const unsigned long long bal = __ballot(rch);
    if (rch) list[cnt + mask_rank(bal)] = (uint16_t)local;
    cnt += __popcll(bal);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own list, read back by its lanes
  GaussRec nrec;
  uint32_t ngo = 0u;
  int nidx = 0;
  if (lane < cnt) {
    nidx = slice + list[lane];
    const size_t o0 = (size_t)vg * a.P + nidx;
    nrec = va.g.rec[o0], ngo = va.g.goff[o0];
  }
#pragma unroll 1
  for (int i = lane; i - lane < cnt; i += 64) {
    if (i >= cnt) break;
    const int idx = nidx;
    const size_t o = (size_t)vg * a.P + idx;
    const GaussRec gr = nrec;
    const uint32_t go = ngo;
    if (i + 64 < cnt) {
      nidx = slice + list[i + 64];
      const size_t on = (size_t)vg * a.P + nidx;
      nrec = va.g.rec[on], ngo = va.g.goff[on];
    }
    float* m2 = va.dmeans2D + 3 * o;
    float4* rec = recv + (size_t)idx * (RS / 4);
    const uint32_t clamp_bits = gr.d.w;
    const RowSums r = gather_rows<TWO>((uint32_t)idx, gr, go, va.gx, cut, grow);
    // rows that sum to zero (no pixel of the staged tiles kept the Gaussian): a zero record without the
    // chain rule
    bool reached = (r.dmx != 0.f) | (r.dmy != 0.f) | (r.dca != 0.f) | (r.dcb != 0.f) | (r.dcc != 0.f) |
                   (r.dop != 0.f) | (r.dcr != 0.f) | (r.dcg != 0.f) | (r.dcbl != 0.f) | (r.ddep != 0.f);
    if (TWO) reached = reached | (r.dr2 != 0.f) | (r.dg2 != 0.f) | (r.db2 != 0.f);
    if (!reached) {
      m2[0] = 0.f;
      m2[1] = 0.f;
      m2[2] = 0.f;
#pragma unroll
      for (int q = 0; q < RS / 4; ++q)
        rec[q] = q == 3 ? make_float4(0.f, __uint_as_float(clamp_bits), 0.f, 0.f) : make_float4(0.f, 0.f, 0.f, 0.f);
      continue;
    }
    // (two colours: the first call's own screen-space gradient; the chain below takes both calls')
    m2[0] = TWO ? r.dmx1 : r.dmx;
    m2[1] = TWO ? r.dmy1 : r.dmy;
    m2[2] = 0.f;
    const float3 mean = make_float3(a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]);
    float cov3D[6];
    if (a.cov3D_precomp) {
#pragma unroll
      for (int k = 0; k < 6; ++k) cov3D[k] = a.cov3D_precomp[6 * idx + k];
    } else {
      const float3 scale = make_float3(a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]);
      const float4 rot = make_float4(a.rotations[4 * idx], a.rotations[4 * idx + 1], a.rotations[4 * idx + 2],
                                     a.rotations[4 * idx + 3]);
      cov3d_from_scale_rot(scale, a.scale_modifier, rot, cov3D);
    }
    float dcv[6];
    float3 dm;
    cov2d_backward(mean, cov3D, vgm, r.dca, r.dcb, r.dcc, dcv, dm);
    proj_backward(mean, projm, r.dmx, r.dmy, dm);
    // view depth = view[2] x + view[6] y + view[10] z + view[14]
    dm.x += viewm[2] * r.ddep;
    dm.y += viewm[6] * r.ddep;
    dm.z += viewm[10] * r.ddep;
    // record fields: dmean3D (3), dcov3D (6), raw dcolor (3), dopacity, SH clamp bits, [second colour (3)]
    const float f[GSR_REC_STRIDE2] = {dm.x,   dm.y,  dm.z,  dcv[0], dcv[1], dcv[2], dcv[3],
                                      dcv[4], dcv[5], r.dcr, r.dcg,  r.dcbl, r.dop,  __uint_as_float(clamp_bits),
                                      r.dr2,  r.dg2, r.db2, 0.f,   0.f,    0.f};
#pragma unroll
    for (int q = 0; q < RS / 4; ++q) rec[q] = make_float4(f[4 * q], f[4 * q + 1], f[4 * q + 2], f[4 * q + 3]);
  }
}

// ---- B: per Gaussian, over the group's views ---------------------------------------------------
// 256 Gaussians per block.  The block's SH rows (contiguous in HBM) are loaded into LDS with fully
// coalesced loads; each thread reads its row from LDS for every view, accumulates dL/dSH in registers,
// writes it back into its LDS row, and the block stores the rows coalesced.
// 3 waves per SIMD (the LDS staging allows 3 blocks per CU): 233 -> 168 VGPRs with two record buffers instead of
// three and the SH row read from LDS where used; 7 VGPRs spill outside the view loop.  C3 per-Gaussian backward
// 0.0323 -> 0.0305 ms/view, 8-view sets 0.0514 -> 0.0477 (profiles/r04/gauss_accum_ab.txt)
__attribute__((amdgpu_waves_per_eu(3, 8)))
__global__ __launch_bounds__(256) void k_gauss_accum(GaussBackwardArgs a, AccumArgs b) {
  extern __shared__ __attribute__((aligned(16))) float s_sh[];
  const int t = threadIdx.x;
  const int block0 = a.g0 + blockIdx.x * 256;
  const int idx = block0 + t;
  const int nblk = min(256, a.g1 - block0);
  const int F = 3 * a.M;
  const int S = sh_lds_stride(a.M);
  const bool has_sh = a.shs != nullptr && F > 0;
  const bool acc = b.accumulate != 0;
  const float invF = has_sh ? 1.0f / (float)F : 0.0f;
  // Only the Gaussians some view of the group reached (reach bits) have records; the others keep their sums
  // (accumulate: nothing read or written) or get zero outputs.  The block's reached SH rows are staged in
  // LDS (a list of the reached rows, each row read by consecutive threads), its dL/dSH rows stored from LDS
  // with coalesced writes (all rows, zeros included; with accumulate only the reached rows).
  __shared__ uint8_t s_rl[256];
  __shared__ int s_wcnt[4];
  const unsigned long long reach_word = idx < a.g1 ? b.reach[idx] : 0ull;
  const bool reached = reach_word != 0ull;
  int nr = 0;  // reached rows of the block
  if (has_sh) {
    const unsigned long long bal = __ballot(reached);
    const int w = t >> 6;
    if ((t & 63) == 0) s_wcnt[w] = (int)__popcll(bal);
    __syncthreads();
    int base = 0;
    for (int k = 0; k < 4; ++k) {
      base += k < w ? s_wcnt[k] : 0;
      nr += s_wcnt[k];
    }
    if (reached) s_rl[base + mask_rank(bal)] = (uint8_t)t;
    __syncthreads();
    const int cnt = nr * F;
    for (int e = t; e < cnt; e += 256) {
      const int r = (int)(((float)e + 0.5f) * invF);
      const int tl = s_rl[r];
      const int k = e - r * F;
      s_sh[tl * S + k] = a.shs[(size_t)(block0 + tl) * F + k];
    }
    __syncthreads();
  }
  if (idx < a.g1 && !reached) {
    if (!acc) {
      for (int k = 0; k < 3; ++k) a.dL_dmeans3D[3 * idx + k] = 0.f;
      a.dL_dopacity[idx] = 0.f;
      if (a.dL_dcolors)
        for (int k = 0; k < 3; ++k) a.dL_dcolors[3 * idx + k] = 0.f;
      if (b.dcolors2)
        for (int k = 0; k < 3; ++k) b.dcolors2[3 * idx + k] = 0.f;
      if (b.dcov_carry)
        for (int k = 0; k < 6; ++k) b.dcov_carry[6 * idx + k] = 0.f;
      if (a.dL_dcov3D && a.dL_dcov3D != b.dcov_carry)
        for (int k = 0; k < 6; ++k) a.dL_dcov3D[6 * idx + k] = 0.f;
      if (!a.cov3D_precomp && a.dL_dscales) {
        for (int k = 0; k < 3; ++k) a.dL_dscales[3 * idx + k] = 0.f;
        for (int k = 0; k < 4; ++k) a.dL_drotations[4 * idx + k] = 0.f;
      }
      if (has_sh) {
        float* row = s_sh + t * S;
        for (int k = 0; k < F; ++k) row[k] = 0.f;
      }
    }
  } else if (idx < a.g1) {
    const float3 mean = make_float3(a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]);
    float3 dmean = make_float3(0.f, 0.f, 0.f);
    float dcov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float dop = 0.f, dcr = 0.f, dcg = 0.f, dcb = 0.f;
    float dsh[48];
#pragma unroll
    for (int k = 0; k < 48; ++k) dsh[k] = 0.f;
    if (acc) {
      // continue the earlier groups' sums in place (same summation order as one group)
      dmean = make_float3(a.dL_dmeans3D[3 * idx], a.dL_dmeans3D[3 * idx + 1], a.dL_dmeans3D[3 * idx + 2]);
      dop = a.dL_dopacity[idx];
      if (a.dL_dcolors) dcr = a.dL_dcolors[3 * idx], dcg = a.dL_dcolors[3 * idx + 1], dcb = a.dL_dcolors[3 * idx + 2];
      if (b.dcov_carry)
#pragma unroll
        for (int k = 0; k < 6; ++k) dcov[k] = b.dcov_carry[6 * idx + k];
      if (has_sh) {
        const float* prev = a.dL_dsh + (size_t)idx * F;
#pragma unroll
        for (int k = 0; k < 48; ++k)
          if (k < F) dsh[k] = prev[k];
      }
    }
    const float* sh_row = has_sh ? s_sh + t * S : nullptr;
    // The group's reached views of this Gaussian (reach bits, k_render_bwd): only their records exist.
    // They stream through two register buffers in view order: while one view's SH backward runs, the next
    // view's record (16-byte loads of the whole slot) is in flight.
    const int RS = b.dcolors2 ? GSR_REC_STRIDE2 : GSR_REC_STRIDE;
    float d2[3] = {0.f, 0.f, 0.f};  // two colours: the second colour's sums
    if (b.dcolors2 && acc)
      for (int k = 0; k < 3; ++k) d2[k] = b.dcolors2[3 * idx + k];
    unsigned long long pending = reach_word;
    auto next_view = [&]() -> int {
      if (pending == 0ull) return -1;
      const int v = __builtin_ctzll(pending);
      pending &= pending - 1ull;
      return v;
    };
    auto load = [&](float4 (&f)[4], int vl) {
      const float4* src = reinterpret_cast<const float4*>(b.vrec + ((size_t)vl * a.P + idx) * RS);
#pragma unroll
      for (int q = 0; q < 4; ++q) f[q] = src[q];
    };
    auto process = [&](const float4 (&f4)[4], int vl) {
      const float f[16] = {f4[0].x, f4[0].y, f4[0].z, f4[0].w, f4[1].x, f4[1].y, f4[1].z, f4[1].w,
                           f4[2].x, f4[2].y, f4[2].z, f4[2].w, f4[3].x, f4[3].y, f4[3].z, f4[3].w};
      dmean.x += f[0];
      dmean.y += f[1];
      dmean.z += f[2];
#pragma unroll
      for (int k = 0; k < 6; ++k) dcov[k] += f[3 + k];
      dcr += f[9];
      dcg += f[10];
      dcb += f[11];
      dop += f[12];
      if (b.dcolors2) {
        d2[0] += f[14];
        d2[1] += f[15];
        d2[2] += b.vrec[((size_t)vl * a.P + idx) * RS + 16];
      }
      // (a view whose colour gradient is zero adds nothing to dL/dSH nor, through the view direction,
      // to dL/dmean: skipped)
      if (has_sh && ((f[9] != 0.f) | (f[10] != 0.f) | (f[11] != 0.f))) {
        const uint32_t cl = __float_as_uint(f[13]);
        const float3 dRGB = make_float3((cl & 1u) ? 0.f : f[9], (cl & 2u) ? 0.f : f[10], (cl & 4u) ? 0.f : f[11]);
        // the SH row read from LDS where sh_backward uses it (not copied to 48 registers first)
        const float* shv = sh_row;
        // the camera position through scalar loads (uniform view): a vector load here would be the
        // newest in flight and its wait would drain the record prefetch
        typedef __attribute__((address_space(4))) const float* cfptr;
        const float cpos[3] = {((cfptr)b.campos[vl])[0], ((cfptr)b.campos[vl])[1], ((cfptr)b.campos[vl])[2]};
        sh_backward(a.deg, a.M, shv, dsh, dRGB, mean, cpos, dmean);
      }
    };
    float4 fa[4], fb[4];
    int va_ = next_view(), vb_ = next_view();
    if (va_ >= 0) load(fa, va_);
    if (vb_ >= 0) load(fb, vb_);
    // (buffers refill in turn, so the views are summed in ascending order, as one pass over the group)
    for (;;) {
      if (va_ < 0) break;
      process(fa, va_);
      va_ = next_view();
      if (va_ >= 0) load(fa, va_);
      if (vb_ < 0) break;
      process(fb, vb_);
      vb_ = next_view();
      if (vb_ >= 0) load(fb, vb_);
    }
    // (the sums already include the earlier groups: plain stores)
    a.dL_dmeans3D[3 * idx] = dmean.x;
    a.dL_dmeans3D[3 * idx + 1] = dmean.y;
    a.dL_dmeans3D[3 * idx + 2] = dmean.z;
    a.dL_dopacity[idx] = dop;
    if (a.dL_dcolors) {
      a.dL_dcolors[3 * idx] = dcr;
      a.dL_dcolors[3 * idx + 1] = dcg;
      a.dL_dcolors[3 * idx + 2] = dcb;
    }
    if (b.dcolors2)
      for (int k = 0; k < 3; ++k) b.dcolors2[3 * idx + k] = d2[k];
    if (b.dcov_carry)
      for (int k = 0; k < 6; ++k) b.dcov_carry[6 * idx + k] = dcov[k];
    if (a.dL_dcov3D && a.dL_dcov3D != b.dcov_carry)
      for (int k = 0; k < 6; ++k) a.dL_dcov3D[6 * idx + k] = dcov[k];
    if (!a.cov3D_precomp && a.dL_dscales) {
      // from the running dL/dcov3D total (linear, but recomputed rather than summed per group so the
      // result does not depend on the grouping)
      const float3 scale = make_float3(a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]);
      const float4 rot = make_float4(a.rotations[4 * idx], a.rotations[4 * idx + 1], a.rotations[4 * idx + 2],
                                     a.rotations[4 * idx + 3]);
      float ds[3], dq[4];
      scale_rot_backward(scale, rot, a.scale_modifier, dcov, ds, dq);
      for (int k = 0; k < 3; ++k) a.dL_dscales[3 * idx + k] = ds[k];
      for (int k = 0; k < 4; ++k) a.dL_drotations[4 * idx + k] = dq[k];
    }
    if (has_sh) {
      // this thread's SH row is no longer read: reuse it for dL/dSH
      float* row = s_sh + t * S;
      float4* row4w = reinterpret_cast<float4*>(row);
#pragma unroll
      for (int c = 0; c < 12; ++c)  // 16-byte writes; the padding past 3M is never copied out
        if (4 * c < F) row4w[c] = make_float4(dsh[4 * c], dsh[4 * c + 1], dsh[4 * c + 2], dsh[4 * c + 3]);
      for (int k = 48; k < F; ++k) row[k] = 0.f;
    }
  }
  if (has_sh) {
    __syncthreads();
    if (!acc) {
      float* dst = a.dL_dsh + (size_t)block0 * F;
      const int cnt = nblk * F;
      for (int e = t; e < cnt; e += 256) {
        const int te = (int)(((float)e + 0.5f) * invF);
        dst[e] = s_sh[te * S + (e - te * F)];
      }
    } else {
      const int cnt = nr * F;
      for (int e = t; e < cnt; e += 256) {
        const int r = (int)(((float)e + 0.5f) * invF);
        const int tl = s_rl[r];
        const int k = e - r * F;
        a.dL_dsh[(size_t)(block0 + tl) * F + k] = s_sh[tl * S + k];
      }
    }
  }
}

// ---- A+B fused, without SH (colours precomputed: the SuGaR normal renderer, C5) -------------------------
// One thread per Gaussian walks the group's views in order: for each view its blend reached (reach bit) the
// k_view_grad work (rows gathered up to the tile cut-offs, conic -> 2D cov -> 3D cov / mean, projection and
// depth terms, the view's means2D gradient) and, instead of writing a 64/80-byte record for k_gauss_accum
// to read back, the sums in registers in the same view order; the unreached views get their zero means2D
// gradient.  With no SH there is no per-view SH backward to keep apart from the gather (the reason for the
// split), and the records were ~200 MB/view of HBM writes + reads at C5.  The same operations in the same
// order as k_view_grad + k_gauss_accum: bitwise the same gradients (up to the sign of zero sums).  Lanes of a
// wave walk the same view at a time: the camera comes through scalar loads; a view's record / row slot of
// consecutive Gaussians are consecutive (coalesced); the next reached view's are loaded one view ahead.
// With SH coefficients the two-kernel path runs: a fused SH variant (one thread per Gaussian reading and writing
// its 48 coefficients) measured 0.2 ms/view slower on the per-view path (profiles/r04/fused_ab.txt).
template <bool TWO>
__global__ __launch_bounds__(256) void k_gauss_fused(GaussBackwardArgs a, ViewGradArgs va, AccumArgs b) {
  const int idx = a.g0 + blockIdx.x * 256 + threadIdx.x;
  const bool valid = idx < a.g1;
  const int ix = valid ? idx : a.g0;  // (threads past the range follow the loop uniformly, write nothing)
  const bool acc = b.accumulate != 0;
  const unsigned long long reach_word = valid ? va.reach[ix] : 0ull;
  float3 dmean = make_float3(0.f, 0.f, 0.f);
  float dcov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float dop = 0.f, dcr = 0.f, dcg = 0.f, dcb = 0.f;
  float d2[3] = {0.f, 0.f, 0.f};
  if (valid && acc) {
    // continue the earlier groups' sums in place (same summation order as one group)
    dmean = make_float3(a.dL_dmeans3D[3 * idx], a.dL_dmeans3D[3 * idx + 1], a.dL_dmeans3D[3 * idx + 2]);
    dop = a.dL_dopacity[idx];
    if (a.dL_dcolors) dcr = a.dL_dcolors[3 * idx], dcg = a.dL_dcolors[3 * idx + 1], dcb = a.dL_dcolors[3 * idx + 2];
    if (b.dcov_carry)
#pragma unroll
      for (int k = 0; k < 6; ++k) dcov[k] = b.dcov_carry[6 * idx + k];
    if (TWO)
      for (int k = 0; k < 3; ++k) d2[k] = b.dcolors2[3 * idx + k];
  }
  const float3 mean = make_float3(a.means3D[3 * ix], a.means3D[3 * ix + 1], a.means3D[3 * ix + 2]);
  float cov3D[6];
  if (reach_word != 0ull) {
    if (a.cov3D_precomp) {
#pragma unroll
      for (int k = 0; k < 6; ++k) cov3D[k] = a.cov3D_precomp[6 * ix + k];
    } else {
      const float3 scale = make_float3(a.scales[3 * ix], a.scales[3 * ix + 1], a.scales[3 * ix + 2]);
      const float4 rot = make_float4(a.rotations[4 * ix], a.rotations[4 * ix + 1], a.rotations[4 * ix + 2],
                                     a.rotations[4 * ix + 3]);
      cov3d_from_scale_rot(scale, a.scale_modifier, rot, cov3D);
    }
  }
  // the next reached view's record and row slot (one view ahead)
  GaussRec nrec;
  uint32_t ngo = 0u;
  auto fetch = [&](int vl) {
    const size_t o = (size_t)(va.v0 + vl) * a.P + ix;
    nrec = va.g.rec[o];
    ngo = va.g.goff[o];
  };
  const int vfirst = reach_word != 0ull ? (int)__builtin_ctzll(reach_word) : va.V;
  if (vfirst < va.V) fetch(vfirst);
#pragma unroll 1
  for (int vl = 0; vl < va.V; ++vl) {
    const int vg = va.v0 + vl;
    float* m2 = va.dmeans2D + 3 * ((size_t)vg * a.P + ix);
    if (!((reach_word >> vl) & 1ull)) {
      if (valid) m2[0] = 0.f, m2[1] = 0.f, m2[2] = 0.f;
      continue;
    }
    const GaussRec gr = nrec;
    const uint32_t go = ngo;
    const unsigned long long later = reach_word & ~((2ull << vl) - 1ull);
    if (later != 0ull) fetch((int)__builtin_ctzll(later));
    const ViewCam& cam = va.cam[vl];
    typedef __attribute__((address_space(4))) const float* cfptr;
    float viewm[16], projm[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) viewm[i] = ((cfptr)cam.view)[i], projm[i] = ((cfptr)cam.proj)[i];
    ViewGeom vgm;
    vgm.view = viewm;
    vgm.proj = projm;
    vgm.tanx = cam.tanx;
    vgm.tany = cam.tany;
    vgm.fy = va.H / (2.0f * cam.tany);
    vgm.fx = va.W / (2.0f * cam.tanx);
    const float4* grow = va.grow + (size_t)(TWO ? 4 : 3) * va.row_start[vl];
    const uint2* cut = va.img.cut + (size_t)vg * va.tiles;
    const RowSums r = gather_rows<TWO>((uint32_t)ix, gr, go, va.gx, cut, grow);
    bool reached = (r.dmx != 0.f) | (r.dmy != 0.f) | (r.dca != 0.f) | (r.dcb != 0.f) | (r.dcc != 0.f) |
                   (r.dop != 0.f) | (r.dcr != 0.f) | (r.dcg != 0.f) | (r.dcbl != 0.f) | (r.ddep != 0.f);
    if (TWO) reached = reached | (r.dr2 != 0.f) | (r.dg2 != 0.f) | (r.db2 != 0.f);
    if (!reached) {
      if (valid) m2[0] = 0.f, m2[1] = 0.f, m2[2] = 0.f;
      continue;
    }
    if (valid) {
      m2[0] = TWO ? r.dmx1 : r.dmx;
      m2[1] = TWO ? r.dmy1 : r.dmy;
      m2[2] = 0.f;
    }
    float dcv[6];
    float3 dm;
    cov2d_backward(mean, cov3D, vgm, r.dca, r.dcb, r.dcc, dcv, dm);
    proj_backward(mean, projm, r.dmx, r.dmy, dm);
    dm.x += viewm[2] * r.ddep;
    dm.y += viewm[6] * r.ddep;
    dm.z += viewm[10] * r.ddep;
    // the record's fields summed as k_gauss_accum sums them (view order)
    dmean.x += dm.x;
    dmean.y += dm.y;
    dmean.z += dm.z;
#pragma unroll
    for (int k = 0; k < 6; ++k) dcov[k] += dcv[k];
    dcr += r.dcr;
    dcg += r.dcg;
    dcb += r.dcbl;
    dop += r.dop;
    if (TWO) {
      d2[0] += r.dr2;
      d2[1] += r.dg2;
      d2[2] += r.db2;
    }
  }
  if (!valid) return;
  a.dL_dmeans3D[3 * idx] = dmean.x;
  a.dL_dmeans3D[3 * idx + 1] = dmean.y;
  a.dL_dmeans3D[3 * idx + 2] = dmean.z;
  a.dL_dopacity[idx] = dop;
  if (a.dL_dcolors) {
    a.dL_dcolors[3 * idx] = dcr;
    a.dL_dcolors[3 * idx + 1] = dcg;
    a.dL_dcolors[3 * idx + 2] = dcb;
  }
  if (TWO)
    for (int k = 0; k < 3; ++k) b.dcolors2[3 * idx + k] = d2[k];
  if (b.dcov_carry)
    for (int k = 0; k < 6; ++k) b.dcov_carry[6 * idx + k] = dcov[k];
  if (a.dL_dcov3D && a.dL_dcov3D != b.dcov_carry)
    for (int k = 0; k < 6; ++k) a.dL_dcov3D[6 * idx + k] = dcov[k];
  if (!a.cov3D_precomp && a.dL_dscales) {
    const float3 scale = make_float3(a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]);
    const float4 rot = make_float4(a.rotations[4 * idx], a.rotations[4 * idx + 1], a.rotations[4 * idx + 2],
                                   a.rotations[4 * idx + 3]);
    float ds[3], dq[4];
    scale_rot_backward(scale, rot, a.scale_modifier, dcov, ds, dq);
    for (int k = 0; k < 3; ++k) a.dL_dscales[3 * idx + k] = ds[k];
    for (int k = 0; k < 4; ++k) a.dL_drotations[4 * idx + k] = dq[k];
  }
}

// the fused per-Gaussian backward for launches without SH (GSR_GAUSS_FUSED=0: the split kernels, A/B)
static bool gauss_fused_on(const GaussBackwardArgs& a) {
  if (a.shs != nullptr && a.M > 0) return false;
  const char* e = getenv("GSR_GAUSS_FUSED");
  return !(e != nullptr && strcmp(e, "0") == 0);
}

// LDS budget for the staged tile cut-offs of k_view_grad (larger images read them from L2).
#define GSR_CUT_LDS_MAX (48 * 1024)

void launch_gauss_backward(const GaussBackwardArgs& a, ViewGradArgs va, const AccumArgs& b, hipStream_t stream) {
  const int n = a.g1 - a.g0;
  if (n <= 0 || va.V <= 0) return;
  if (gauss_fused_on(a)) {
    auto kern = b.dcolors2 ? k_gauss_fused<true> : k_gauss_fused<false>;
    hipLaunchKernelGGL(kern, dim3(div_up(n, 256)), dim3(256), 0, stream, a, va, b);
    return;
  }
  const size_t cut_bytes = sizeof(uint2) * (size_t)va.tiles;
  va.cut_in_lds = cut_bytes <= GSR_CUT_LDS_MAX ? 1 : 0;
  // items per thread: GSR_VG_ITEMS, halved (down to 2) while the launch would have fewer than 1024 blocks
  va.items = GSR_VG_ITEMS;
  while (va.items > 2 && (long long)va.V * div_up(n, 256 * va.items) < 1024) va.items >>= 1;
  const dim3 vg_grid(va.V * div_up(n, 256 * va.items));
  auto vg_kern = b.dcolors2 ? (va.cut_in_lds ? k_view_grad<true, true> : k_view_grad<true, false>)
                            : (va.cut_in_lds ? k_view_grad<false, true> : k_view_grad<false, false>);
  hipLaunchKernelGGL(vg_kern, vg_grid, dim3(256), va.cut_in_lds ? cut_bytes : 0, stream, a, va);
  const size_t lds = (a.shs && a.M > 0) ? (size_t)256 * sh_lds_stride(a.M) * sizeof(float) : 0;
  hipLaunchKernelGGL(k_gauss_accum, dim3(div_up(n, 256)), dim3(256), lds, stream, a, b);
}

}  // namespace gsr

// gsr_backward.hip — fused per-Gaussian backward.
//
// One thread per Gaussian:
//   1. gather-sum of the Gaussian's per-instance gradient rows written by k_render_bwd into the
//      Gaussian's own contiguous slots (fixed summation order -> bitwise reproducible);
//   2. BACKWARD::computeCov2DCUDA [EXT]: conic -> 2D cov -> 3D cov and camera-space mean;
//   3. BACKWARD::preprocessCUDA [EXT]: 2D mean -> 3D mean through the projection, view-depth
//      term (ashawkey depth output), SH -> RGB backward incl. the view-direction term,
//      3D cov -> scale and (unnormalised) quaternion.
// Replaces two N-sized kernels plus 9 per-pair atomics of the reference with one pass.
// Gradient conventions of the reference are kept: the 0.99 alpha clamp is
// ignored in dL/dG, the frustum clamp zeroes dL/dt_x,y only, denom2inv carries +1e-7, the scale
// gradient is w.r.t. scale_modifier * scale.
#include "gsr_kernels.h"
#include "gsr_math.h"

namespace gsr {

// One Gaussian.  sh_l / dsh_l point at this Gaussian's SH block and dL/dSH block in LDS (the kernel
// stages them with coalesced global accesses); both may be null without SHs.
__device__ __forceinline__ void gauss_bwd_one(const GaussBackwardArgs& a, int idx, int grid_x, const GeomState& g,
                                              const uint4* __restrict__ tile_info, const BackwardState& bw,
                                              const float* sh_l, float* dsh_l) {
  const int Mc = a.M;
  const bool visible = a.radii[idx] > 0;

  float dmx = 0.f, dmy = 0.f, dca = 0.f, dcb = 0.f, dcc = 0.f, dop = 0.f;
  float dcr = 0.f, dcg = 0.f, dcbl = 0.f, ddep = 0.f;
  if (visible) {
    // rows of this Gaussian's instances are contiguous (tile rect, row-major, 4 quadrant rows each);
    // an instance's rows are valid iff its tile's blend reached it:
    // (depth key, index) < the tile's first unblended instance
    const size_t i0 = g.goff[idx];
    const uint2 rc = g.rect[idx];
    const int xmin = rc.x & 0xffff, ymin = rc.x >> 16, xmax = rc.y & 0xffff, ymax = rc.y >> 16;
    const uint32_t dkey = __float_as_uint(g.rec1[idx].z);
    size_t i = i0;
    for (int ty = ymin; ty < ymax; ++ty)
      for (int tx = xmin; tx < xmax; ++tx, ++i) {
        const uint4 info = tile_info[ty * grid_x + tx];
        const bool valid = dkey < info.y || (dkey == info.y && (uint32_t)idx < info.z);
        if (!valid) continue;
        const float4* row = bw.grow + 12 * i;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 r0 = row[3 * q], r1 = row[3 * q + 1], r2 = row[3 * q + 2];
          dmx += r0.x; dmy += r0.y; dca += r0.z; dcb += r0.w;
          dcc += r1.x; dop += r1.y; dcr += r1.z; dcg += r1.w;
          dcbl += r2.x; ddep += r2.y;
        }
      }
  }
  a.dL_dmeans2D[3 * idx] = dmx;
  a.dL_dmeans2D[3 * idx + 1] = dmy;
  a.dL_dmeans2D[3 * idx + 2] = 0.f;
  a.dL_dopacity[idx] = dop;
  a.dL_dcolors[3 * idx] = dcr;
  a.dL_dcolors[3 * idx + 1] = dcg;
  a.dL_dcolors[3 * idx + 2] = dcbl;

  if (!visible) {
    a.dL_dmeans3D[3 * idx] = 0.f;
    a.dL_dmeans3D[3 * idx + 1] = 0.f;
    a.dL_dmeans3D[3 * idx + 2] = 0.f;
    if (a.dL_dcov3D)
      for (int k = 0; k < 6; ++k) a.dL_dcov3D[6 * idx + k] = 0.f;
    if (a.dL_dsh)
      for (int k = 0; k < 3 * Mc; ++k) dsh_l[k] = 0.f;
    if (a.dL_dscales)
      for (int k = 0; k < 3; ++k) a.dL_dscales[3 * idx + k] = 0.f;
    if (a.dL_drotations)
      for (int k = 0; k < 4; ++k) a.dL_drotations[4 * idx + k] = 0.f;
    return;
  }

  const float3 mean = make_float3(a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]);
  const float* view = a.viewmatrix;
  const float* proj = a.projmatrix;

  // ---- computeCov2DCUDA --------------------------------------------------------------
  float cov3D[6];
  float3 scale = make_float3(0.f, 0.f, 0.f);
  float4 rot = make_float4(0.f, 0.f, 0.f, 0.f);
  if (a.cov3D_precomp) {
    for (int k = 0; k < 6; ++k) cov3D[k] = a.cov3D_precomp[6 * idx + k];
  } else {
    scale = make_float3(a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]);
    rot = make_float4(a.rotations[4 * idx], a.rotations[4 * idx + 1], a.rotations[4 * idx + 2],
                      a.rotations[4 * idx + 3]);
    cov3d_from_scale_rot(scale, a.scale_modifier, rot, cov3D);
  }
  Cov2DState st;
  const float3 cov2 = cov2d_ewa(mean, a.focal_x, a.focal_y, a.tanfovx, a.tanfovy, cov3D, view, st);
  const float x_grad_mul = (st.txtz < -st.limx || st.txtz > st.limx) ? 0.f : 1.f;
  const float y_grad_mul = (st.tytz < -st.limy || st.tytz > st.limy) ? 0.f : 1.f;
  const float ca = cov2.x, cb = cov2.y, cc = cov2.z;
  const float denom = ca * cc - cb * cb;
  float dL_da = 0.f, dL_db = 0.f, dL_dc = 0.f;
  const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
  const float(&T)[2][3] = st.T;
  float dcov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
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
  const float hx = a.focal_x, hy = a.focal_y;
  const float dtx = x_grad_mul * -hx * tz2 * dJ02;
  const float dty = y_grad_mul * -hy * tz2 * dJ12;
  const float dtz = -hx * tz2 * dJ00 - hy * tz2 * dJ11 + (2 * hx * st.t.x) * tz3 * dJ02 +
                    (2 * hy * st.t.y) * tz3 * dJ12;
  float3 dmean = xform_vec4x3_T(make_float3(dtx, dty, dtz), view);

  // ---- preprocessCUDA: 2D mean -> 3D mean ----------------------------------------------
  {
    const float4 m_hom = xform_point4x4(mean, proj);
    const float m_w = 1.0f / (m_hom.w + 0.0000001f);
    const float mul1 = (proj[0] * mean.x + proj[4] * mean.y + proj[8] * mean.z + proj[12]) * m_w * m_w;
    const float mul2 = (proj[1] * mean.x + proj[5] * mean.y + proj[9] * mean.z + proj[13]) * m_w * m_w;
    dmean.x += (proj[0] * m_w - proj[3] * mul1) * dmx + (proj[1] * m_w - proj[3] * mul2) * dmy;
    dmean.y += (proj[4] * m_w - proj[7] * mul1) * dmx + (proj[5] * m_w - proj[7] * mul2) * dmy;
    dmean.z += (proj[8] * m_w - proj[11] * mul1) * dmx + (proj[9] * m_w - proj[11] * mul2) * dmy;
  }
  // view depth = view[2] x + view[6] y + view[10] z + view[14]
  dmean.x += view[2] * ddep;
  dmean.y += view[6] * ddep;
  dmean.z += view[10] * ddep;

  // ---- SH backward -------------------------------------------------------------------
  if (a.shs) {
    const float* sh = sh_l;
    float* dsh = dsh_l;
    const uint32_t cl = g.clamped[idx];
    const float3 dRGB = make_float3((cl & 1u) ? 0.f : dcr, (cl & 2u) ? 0.f : dcg, (cl & 4u) ? 0.f : dcbl);
    const float3 dir_orig = make_float3(mean.x - a.campos[0], mean.y - a.campos[1], mean.z - a.campos[2]);
    const float len = sqrtf(dir_orig.x * dir_orig.x + dir_orig.y * dir_orig.y + dir_orig.z * dir_orig.z);
    const float x = dir_orig.x / len, y = dir_orig.y / len, z = dir_orig.z / len;
    const int deg = a.deg;
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
    float3 dRGBdx = make_float3(0.f, 0.f, 0.f), dRGBdy = dRGBdx, dRGBdz = dRGBdx;
    const int ncoef = (deg + 1) * (deg + 1);
#pragma unroll
    for (int k = 1; k < 16; ++k) {
      if (k < ncoef) {
        const float3 s = make_float3(sh[3 * k], sh[3 * k + 1], sh[3 * k + 2]);
        dRGBdx.x += bdx[k] * s.x; dRGBdx.y += bdx[k] * s.y; dRGBdx.z += bdx[k] * s.z;
        dRGBdy.x += bdy[k] * s.x; dRGBdy.y += bdy[k] * s.y; dRGBdy.z += bdy[k] * s.z;
        dRGBdz.x += bdz[k] * s.x; dRGBdz.y += bdz[k] * s.y; dRGBdz.z += bdz[k] * s.z;
      }
    }
    // dL/dSH last: it overwrites the SH row in LDS (same row) that the loop above reads
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (k < Mc) {
        const float bk = k < ncoef ? basis[k] : 0.f;
        dsh[3 * k] = bk * dRGB.x;
        dsh[3 * k + 1] = bk * dRGB.y;
        dsh[3 * k + 2] = bk * dRGB.z;
      }
    }
    for (int k = 16; k < Mc; ++k) dsh[3 * k] = dsh[3 * k + 1] = dsh[3 * k + 2] = 0.f;
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
  a.dL_dmeans3D[3 * idx] = dmean.x;
  a.dL_dmeans3D[3 * idx + 1] = dmean.y;
  a.dL_dmeans3D[3 * idx + 2] = dmean.z;
  if (a.dL_dcov3D)
    for (int k = 0; k < 6; ++k) a.dL_dcov3D[6 * idx + k] = dcov[k];

  // ---- 3D covariance -> scale, quaternion ----------------------------------------------
  if (!a.cov3D_precomp && a.dL_dscales) {
    Mat3 R;
    rot_from_quat(rot, R);
    const float s[3] = {a.scale_modifier * scale.x, a.scale_modifier * scale.y, a.scale_modifier * scale.z};
    // E[c][k] = s_k R[c][k];  Sigma[c][r] = sum_k E[r][k] E[c][k]
    // dSigma (symmetric, off-diagonals split evenly)
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
    float ds[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      ds[k] = dE[0][k] * R.m[0][k] + dE[1][k] * R.m[1][k] + dE[2][k] * R.m[2][k];
#pragma unroll
      for (int aa = 0; aa < 3; ++aa) dR[aa][k] = dE[aa][k] * s[k];
    }
    a.dL_dscales[3 * idx] = ds[0];
    a.dL_dscales[3 * idx + 1] = ds[1];
    a.dL_dscales[3 * idx + 2] = ds[2];
    const float r = rot.x, x = rot.y, y = rot.z, z = rot.w;
    // dR[c][r'] / dq for R.m as built by rot_from_quat
    const float dq_r = -2.f * z * dR[0][1] + 2.f * y * dR[0][2] + 2.f * z * dR[1][0] - 2.f * x * dR[1][2] -
                       2.f * y * dR[2][0] + 2.f * x * dR[2][1];
    const float dq_x = 2.f * y * dR[0][1] + 2.f * z * dR[0][2] + 2.f * y * dR[1][0] - 4.f * x * dR[1][1] -
                       2.f * r * dR[1][2] + 2.f * z * dR[2][0] + 2.f * r * dR[2][1] - 4.f * x * dR[2][2];
    const float dq_y = -4.f * y * dR[0][0] + 2.f * x * dR[0][1] + 2.f * r * dR[0][2] + 2.f * x * dR[1][0] +
                       2.f * z * dR[1][2] - 2.f * r * dR[2][0] + 2.f * z * dR[2][1] - 4.f * y * dR[2][2];
    const float dq_z = -4.f * z * dR[0][0] - 2.f * r * dR[0][1] + 2.f * x * dR[0][2] + 2.f * r * dR[1][0] -
                       4.f * z * dR[1][1] + 2.f * y * dR[1][2] + 2.f * x * dR[2][0] + 2.f * y * dR[2][1];
    a.dL_drotations[4 * idx] = dq_r;
    a.dL_drotations[4 * idx + 1] = dq_x;
    a.dL_drotations[4 * idx + 2] = dq_y;
    a.dL_drotations[4 * idx + 3] = dq_z;
  }
}

// LDS row stride (floats) of one Gaussian's 3M SH values: 16-byte multiple plus 16 bytes of padding so
// per-thread ds_read_b128 / ds_write_b128 at this stride are bank-conflict free.
static inline __host__ __device__ int sh_lds_stride(int M) { return ((3 * M + 3) & ~3) + 4; }

// 256 Gaussians per block.  The block's SH rows (P x M x 3 floats, contiguous) are loaded into LDS with
// fully coalesced 4-byte loads, each thread computes its Gaussian reading its row from LDS and writes its
// dL/dSH row back into the same LDS row, and the block stores the rows with coalesced stores.  Direct
// per-thread 192-byte row accesses (stride 192 B across lanes) left 2/3 of the wave time waiting on memory.
__global__ __launch_bounds__(256) void k_gauss_bwd(GaussBackwardArgs a, int grid_x, GeomState g,
                                                   const uint4* __restrict__ tile_info, BackwardState bw) {
  extern __shared__ __attribute__((aligned(16))) float s_sh[];
  const int t = threadIdx.x;
  const int block0 = blockIdx.x * 256;
  const int idx = block0 + t;
  const int nblk = min(256, a.P - block0);
  const int F = 3 * a.M;
  const int S = sh_lds_stride(a.M);
  const bool has_sh = a.shs != nullptr && F > 0;
  const float invF = has_sh ? 1.0f / (float)F : 0.0f;
  if (has_sh) {
    const float* src = a.shs + (size_t)block0 * F;
    const int cnt = nblk * F;
    for (int e = t; e < cnt; e += 256) {
      const int te = (int)(((float)e + 0.5f) * invF);
      s_sh[te * S + (e - te * F)] = src[e];
    }
    __syncthreads();
  }
  if (idx < a.P) gauss_bwd_one(a, idx, grid_x, g, tile_info, bw, has_sh ? s_sh + t * S : nullptr,
                               has_sh ? s_sh + t * S : nullptr);
  if (has_sh) {
    __syncthreads();
    float* dst = a.dL_dsh + (size_t)block0 * F;
    const int cnt = nblk * F;
    for (int e = t; e < cnt; e += 256) {
      const int te = (int)(((float)e + 0.5f) * invF);
      dst[e] = s_sh[te * S + (e - te * F)];
    }
  }
}

void launch_gauss_backward(const GaussBackwardArgs& a, int W, int H, const GeomState& g,
                           const ImageState& img, const BackwardState& bw, hipStream_t stream) {
  (void)H;
  if (a.P <= 0) return;
  const size_t lds = (a.shs && a.M > 0) ? (size_t)256 * sh_lds_stride(a.M) * sizeof(float) : 0;
  hipLaunchKernelGGL(k_gauss_bwd, dim3((a.P + 255) / 256), dim3(256), lds, stream, a,
                     div_up(W, GSR_TILE_X), g, (const uint4*)img.tile_info, bw);
}

}  // namespace gsr

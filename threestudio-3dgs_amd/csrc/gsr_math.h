// gsr_math.h — per-Gaussian geometry shared by the preprocess (forward) and the fused
// per-Gaussian backward kernel.  Each function restates one step of the reference algorithm
//  with the same operation order, in plain registers.
#pragma once

#include "gsr_common.h"

namespace gsr {

// SH basis constants — identical to the reference's pure-torch twin (geometry/sugar.py:743-772).
#define SH_C0 0.28209479177387814f
#define SH_C1 0.4886025119029199f
__constant__ static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f,
                                            0.31539156525252005f, -1.0925484305920792f,
                                            0.5462742152960396f};
__constant__ static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f,
                                            -0.4570457994644658f, 0.3731763325901154f,
                                            -0.4570457994644658f, 1.445305721320277f,
                                            -0.5900435899266435f};

struct Mat3 {  // column-major, m[col][row] (glm convention of the reference kernels)
  float m[3][3];
};

// 3D covariance from scale and (w,x,y,z) quaternion: Sigma = R S S R^T, upper triangle.
// Twin: build_rotation / build_scaling_rotation / strip_symmetric (geometry/gaussian_base.py:47-134, 233-238).
__device__ __forceinline__ void rot_from_quat(const float4 q, Mat3& R) {
  const float r = q.x, x = q.y, y = q.z, z = q.w;
  R.m[0][0] = 1.f - 2.f * (y * y + z * z);
  R.m[0][1] = 2.f * (x * y - r * z);
  R.m[0][2] = 2.f * (x * z + r * y);
  R.m[1][0] = 2.f * (x * y + r * z);
  R.m[1][1] = 1.f - 2.f * (x * x + z * z);
  R.m[1][2] = 2.f * (y * z - r * x);
  R.m[2][0] = 2.f * (x * z - r * y);
  R.m[2][1] = 2.f * (y * z + r * x);
  R.m[2][2] = 1.f - 2.f * (x * x + y * y);
}

__device__ __forceinline__ void cov3d_from_scale_rot(const float3 scale, float mod, const float4 q,
                                                     float cov[6]) {
  Mat3 R;
  rot_from_quat(q, R);
  const float s[3] = {mod * scale.x, mod * scale.y, mod * scale.z};
  // M = S * R  ->  M[c][r] = s_r * R[c][r];  Sigma[c][r] = sum_k M[r][k] * M[c][k]
  float M[3][3];
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int r = 0; r < 3; ++r) M[c][r] = s[r] * R.m[c][r];
  auto sig = [&](int c, int r) {
    return M[r][0] * M[c][0] + M[r][1] * M[c][1] + M[r][2] * M[c][2];
  };
  cov[0] = sig(0, 0);
  cov[1] = sig(0, 1);
  cov[2] = sig(0, 2);
  cov[3] = sig(1, 1);
  cov[4] = sig(1, 2);
  cov[5] = sig(2, 2);
}

// EWA projection state: the clamped camera-space mean and the Jacobian-transform T = W * J.
struct Cov2DState {
  float3 t;        // camera-space mean with x/z, y/z clamped to 1.3 tan(fov)
  float txtz, tytz, limx, limy;
  float T[2][3];   // the two non-zero columns of T (glm T[c][r], c = 0,1)
  float W[3][3];   // W[c][r]
};

// cov2D = T^T Vrk T + 0.3 I  (ashawkey/graphdeco computeCov2D [EXT]).
__device__ __forceinline__ float3 cov2d_ewa(const float3 mean, float focal_x, float focal_y,
                                           float tan_fovx, float tan_fovy, const float* cov3D,
                                           const float* view, Cov2DState& st) {
  float3 t = xform_point4x3(mean, view);
  st.limx = 1.3f * tan_fovx;
  st.limy = 1.3f * tan_fovy;
  st.txtz = t.x / t.z;
  st.tytz = t.y / t.z;
  t.x = fminf(st.limx, fmaxf(-st.limx, st.txtz)) * t.z;
  t.y = fminf(st.limy, fmaxf(-st.limy, st.tytz)) * t.z;
  st.t = t;
  const float J00 = focal_x / t.z;
  const float J02 = -(focal_x * t.x) / (t.z * t.z);
  const float J11 = focal_y / t.z;
  const float J12 = -(focal_y * t.y) / (t.z * t.z);
  // W (glm columns): W[0] = (v0, v4, v8), W[1] = (v1, v5, v9), W[2] = (v2, v6, v10)
  st.W[0][0] = view[0]; st.W[0][1] = view[4]; st.W[0][2] = view[8];
  st.W[1][0] = view[1]; st.W[1][1] = view[5]; st.W[1][2] = view[9];
  st.W[2][0] = view[2]; st.W[2][1] = view[6]; st.W[2][2] = view[10];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    st.T[0][r] = st.W[0][r] * J00 + st.W[2][r] * J02;
    st.T[1][r] = st.W[1][r] * J11 + st.W[2][r] * J12;
  }
  const float V[3][3] = {{cov3D[0], cov3D[1], cov3D[2]},
                         {cov3D[1], cov3D[3], cov3D[4]},
                         {cov3D[2], cov3D[4], cov3D[5]}};
  // A = T^T * Vrk ; A[k][r] = sum_m T[r][m] * V[k][m]   (r in {0,1})
  float A[3][2];
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int r = 0; r < 2; ++r)
      A[k][r] = st.T[r][0] * V[k][0] + st.T[r][1] * V[k][1] + st.T[r][2] * V[k][2];
  // cov[c][r] = sum_k A[k][r] * T[c][k]
  float c00 = A[0][0] * st.T[0][0] + A[1][0] * st.T[0][1] + A[2][0] * st.T[0][2];
  float c01 = A[0][1] * st.T[0][0] + A[1][1] * st.T[0][1] + A[2][1] * st.T[0][2];
  float c11 = A[0][1] * st.T[1][0] + A[1][1] * st.T[1][1] + A[2][1] * st.T[1][2];
  c00 += 0.3f;
  c11 += 0.3f;
  return make_float3(c00, c01, c11);
}

// SH -> RGB at direction normalize(pos - campos), +0.5, clamp at 0 (computeColorFromSH [EXT];
// polynomial identical to eval_sh, geometry/sugar.py:775-830).  sh points at the Gaussian's
// (M,3) block.  Returns unclamped+0.5 result in *raw (for clamp flags).
__device__ __forceinline__ float3 sh_to_rgb(int deg, const float* sh, const float3 pos,
                                            const float3 campos, uint32_t* clamp_bits) {
  float3 dir = make_float3(pos.x - campos.x, pos.y - campos.y, pos.z - campos.z);
  const float len = sqrtf(dir.x * dir.x + dir.y * dir.y + dir.z * dir.z);
  dir.x = dir.x / len; dir.y = dir.y / len; dir.z = dir.z / len;
#define SHV(k) make_float3(sh[3 * (k)], sh[3 * (k) + 1], sh[3 * (k) + 2])
  float3 res;
  {
    const float3 s0 = SHV(0);
    res = make_float3(SH_C0 * s0.x, SH_C0 * s0.y, SH_C0 * s0.z);
  }
  if (deg > 0) {
    const float x = dir.x, y = dir.y, z = dir.z;
    const float3 s1 = SHV(1), s2 = SHV(2), s3 = SHV(3);
    const float k1 = SH_C1 * y, k2 = SH_C1 * z, k3 = SH_C1 * x;
    res.x = res.x - k1 * s1.x + k2 * s2.x - k3 * s3.x;
    res.y = res.y - k1 * s1.y + k2 * s2.y - k3 * s3.y;
    res.z = res.z - k1 * s1.z + k2 * s2.z - k3 * s3.z;
    if (deg > 1) {
      const float xx = x * x, yy = y * y, zz = z * z;
      const float xy = x * y, yz = y * z, xz = x * z;
      const float b4 = SH_C2[0] * xy, b5 = SH_C2[1] * yz, b6 = SH_C2[2] * (2.0f * zz - xx - yy),
                  b7 = SH_C2[3] * xz, b8 = SH_C2[4] * (xx - yy);
      const float3 s4 = SHV(4), s5 = SHV(5), s6 = SHV(6), s7 = SHV(7), s8 = SHV(8);
      res.x = res.x + b4 * s4.x + b5 * s5.x + b6 * s6.x + b7 * s7.x + b8 * s8.x;
      res.y = res.y + b4 * s4.y + b5 * s5.y + b6 * s6.y + b7 * s7.y + b8 * s8.y;
      res.z = res.z + b4 * s4.z + b5 * s5.z + b6 * s6.z + b7 * s7.z + b8 * s8.z;
      if (deg > 2) {
        const float b9 = SH_C3[0] * y * (3.0f * xx - yy), b10 = SH_C3[1] * xy * z,
                    b11 = SH_C3[2] * y * (4.0f * zz - xx - yy),
                    b12 = SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy),
                    b13 = SH_C3[4] * x * (4.0f * zz - xx - yy), b14 = SH_C3[5] * z * (xx - yy),
                    b15 = SH_C3[6] * x * (xx - 3.0f * yy);
        const float3 s9 = SHV(9), s10 = SHV(10), s11 = SHV(11), s12 = SHV(12), s13 = SHV(13),
                     s14 = SHV(14), s15 = SHV(15);
        res.x = res.x + b9 * s9.x + b10 * s10.x + b11 * s11.x + b12 * s12.x + b13 * s13.x +
                b14 * s14.x + b15 * s15.x;
        res.y = res.y + b9 * s9.y + b10 * s10.y + b11 * s11.y + b12 * s12.y + b13 * s13.y +
                b14 * s14.y + b15 * s15.y;
        res.z = res.z + b9 * s9.z + b10 * s10.z + b11 * s11.z + b12 * s12.z + b13 * s13.z +
                b14 * s14.z + b15 * s15.z;
      }
    }
  }
#undef SHV
  res.x += 0.5f;
  res.y += 0.5f;
  res.z += 0.5f;
  *clamp_bits = (res.x < 0 ? 1u : 0u) | (res.y < 0 ? 2u : 0u) | (res.z < 0 ? 4u : 0u);
  return make_float3(fmaxf(res.x, 0.0f), fmaxf(res.y, 0.0f), fmaxf(res.z, 0.0f));
}

}  // namespace gsr

// gsr_wave.h — wave64 / workgroup primitives for CDNA4 (gfx950): DPP reductions, ballot-based
// digit matching, block scans.  Wave width is hard-coded to 64.
#pragma once

#include "gsr_common.h"

namespace gsr {

__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0)); }

// popcount of the bits of `mask` below this lane (v_mbcnt).
__device__ __forceinline__ uint32_t mask_rank(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float dpp_f32(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, ROW_MASK, 0xf, true));
}

// Sum over the 64 lanes of a wave (all lanes must be active).  Row prefix via DPP row_shr
// 1/2/4/8, then row_bcast:15 / row_bcast:31 fold the four rows into lane 63, read back as a
// wave-uniform value.  6 DPP adds + 1 readlane.
__device__ __forceinline__ float wave_sum(float x) {
  x += dpp_f32<0x111>(x);
  x += dpp_f32<0x112>(x);
  x += dpp_f32<0x114>(x);
  x += dpp_f32<0x118>(x);
  x += dpp_f32<0x142, 0xa>(x);
  x += dpp_f32<0x143, 0xc>(x);
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}

// Lanes of this wave whose `bits`-bit digit equals ours (restricted to lanes with valid=true).
__device__ __forceinline__ unsigned long long match_digit(uint32_t d, int bits, bool valid) {
  // per bit b: s = 0 / all ones from the lane's bit, x |= ballot ^ s on each 32-bit half (one v_bitop3 each:
  // table 0xF6 = S0 | (S1 ^ S2)); the peers are the valid lanes with no differing bit
  uint32_t xlo = 0u, xhi = 0u;
  for (int b = 0; b < bits; ++b) {
    const uint32_t s = (uint32_t)__builtin_amdgcn_sbfe((int)d, b, 1);
    const unsigned long long bal = __ballot(s != 0u);
    xlo = __builtin_amdgcn_bitop3_b32(xlo, (uint32_t)bal, s, 0xF6);
    xhi = __builtin_amdgcn_bitop3_b32(xhi, (uint32_t)(bal >> 32), s, 0xF6);
  }
  const unsigned long long v = __ballot(valid);
  return (((unsigned long long)~xhi << 32) | ~xlo) & v;
}

template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROW_MASK, 0xf, true);
}
// Inclusive sum / max scans over the 64 lanes with DPP (row_shr 1/2/4/8, then row_bcast 15 / 31);
// lanes outside a shift read 0 (bound_ctrl), the identity of both.
__device__ __forceinline__ uint32_t wave_incl_sum_dpp(uint32_t x) {
  x += dpp_u32<0x111>(x);
  x += dpp_u32<0x112>(x);
  x += dpp_u32<0x114>(x);
  x += dpp_u32<0x118>(x);
  x += dpp_u32<0x142, 0xa>(x);
  x += dpp_u32<0x143, 0xc>(x);
  return x;
}
__device__ __forceinline__ uint32_t wave_incl_max_dpp(uint32_t x) {
  x = max(x, dpp_u32<0x111>(x));
  x = max(x, dpp_u32<0x112>(x));
  x = max(x, dpp_u32<0x114>(x));
  x = max(x, dpp_u32<0x118>(x));
  x = max(x, dpp_u32<0x142, 0xa>(x));
  x = max(x, dpp_u32<0x143, 0xc>(x));
  return x;
}

// Inclusive scan over a wave (u32), Hillis-Steele via shuffles.
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  return x;
}

// Exclusive scan of one value per thread over a workgroup of NT threads (NT/64 <= 16 waves).
// s_wave: NT/64 + 1 words of LDS.  Returns the exclusive prefix; *total gets the block sum.
template <int NT>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* total, uint32_t* s_wave) {
  constexpr int NW = NT / 64;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const uint32_t inc = wave_inclusive_scan(v);
  if (lane == 63) s_wave[w] = inc;
  __syncthreads();
  if (t == 0) {
    uint32_t run = 0;
    for (int i = 0; i < NW; ++i) {
      const uint32_t c = s_wave[i];
      s_wave[i] = run;
      run += c;
    }
    s_wave[NW] = run;
  }
  __syncthreads();
  const uint32_t res = s_wave[w] + inc - v;
  *total = s_wave[NW];
  __syncthreads();
  return res;
}

// Exclusive max-scan of one value per thread over a workgroup of NT threads (identity 0).
template <int NT>
__device__ __forceinline__ uint32_t block_exclusive_max(uint32_t v, uint32_t* s_wave) {
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)inc, o, 64);
    if (lane >= o) inc = max(inc, y);
  }
  uint32_t ex = (uint32_t)__shfl_up((int)inc, 1, 64);
  if (lane == 0) ex = 0u;
  if (lane == 63) s_wave[w] = inc;
  __syncthreads();
  uint32_t before = 0u;
  for (int i = 0; i < w; ++i) before = max(before, s_wave[i]);
  __syncthreads();
  return max(before, ex);
}

template <int NT>
__device__ __forceinline__ uint32_t block_sum_u32(uint32_t v, uint32_t* s_wave) {
  uint32_t tot;
  block_exclusive_scan<NT>(v, &tot, s_wave);
  return tot;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
  return v;
}

}  // namespace gsr

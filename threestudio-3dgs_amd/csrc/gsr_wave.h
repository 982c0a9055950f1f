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
  unsigned long long peers = __ballot(valid);
  for (int b = 0; b < bits; ++b) {
    const bool bit = (d >> b) & 1u;
    const unsigned long long bal = __ballot(bit);
    peers &= bit ? bal : ~bal;
  }
  return peers;
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

// ---- decoupled look-back over single-word states -------------------------------------------
// A state word is flag (bits 31:30; 0 = not yet published, AGG = this block's own count,
// INC = inclusive prefix through this block) | count (bits 29:0).  Flag and payload share one
// word, so relaxed agent-scope atomics (global_store/load ... sc1: write-through, L1-bypassing,
// coherent across the XCDs' L2s) are the whole protocol (MI355X_MICROARCH.md, inter-workgroup
// visibility).  Block ids come from a ticket (atomicAdd) so every predecessor a block waits on
// is already resident.  Spins are bounded: on timeout the error word is set and the result is
// garbage instead of a hung GPU.  States and tickets are zeroed by a memset before each launch.
#define GSR_LB_AGG 1u
#define GSR_LB_INC 2u
#define GSR_LB_MASK 0x3FFFFFFFu
#define GSR_LB_SPIN_LIMIT (1 << 22)

__device__ __forceinline__ void lb_publish(uint32_t* p, uint32_t flag, uint32_t v) {
  __hip_atomic_store(p, (flag << 30) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t lb_poll(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One lane: exclusive prefix of block `blk` on one channel (state of block p at st[p * stride]).
__device__ inline uint32_t lb_prefix_serial(const uint32_t* st, size_t stride, int blk, uint32_t* err) {
  uint32_t sum = 0;
  int spins = 0;
  for (int p = blk - 1; p >= 0;) {
    const uint32_t w = lb_poll(st + (size_t)p * stride);
    const uint32_t f = w >> 30;
    if (f == 0) {
      if (++spins > GSR_LB_SPIN_LIMIT) {
        atomicOr(err, 1u);
        break;
      }
      continue;
    }
    sum += w & GSR_LB_MASK;
    if (f == GSR_LB_INC) break;
    --p;
  }
  return sum;
}

// One whole wave: exclusive prefix of block `blk` (states st[p]); lane l inspects block
// end-1-l of each 64-block window, so one round trip covers 64 predecessors.
__device__ inline uint32_t lb_prefix_wave(const uint32_t* st, int blk, uint32_t* err) {
  const int lane = threadIdx.x & 63;
  uint32_t sum = 0;
  int spins = 0;
  for (int end = blk; end > 0; end -= 64) {
    const int p = end - 1 - lane;
    uint32_t w = p >= 0 ? lb_poll(st + p) : (GSR_LB_INC << 30);
    for (;;) {
      const unsigned long long inc = __ballot((w >> 30) == GSR_LB_INC);
      const unsigned long long pending = __ballot((w >> 30) == 0u);
      const int first = inc ? (int)__builtin_ctzll(inc) : 63;
      const unsigned long long need = first == 63 ? ~0ull : ((2ull << first) - 1ull);
      if ((pending & need) == 0ull) {
        sum += wave_sum_u32(lane <= first ? (w & GSR_LB_MASK) : 0u);
        if (inc) return sum;
        break;
      }
      if (++spins > GSR_LB_SPIN_LIMIT) {
        if (lane == 0) atomicOr(err, 1u);
        return sum;
      }
      if ((w >> 30) == 0u) w = lb_poll(st + p);
    }
  }
  return sum;
}

}  // namespace gsr

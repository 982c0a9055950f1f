// gsr_sort.hip — device-wide exclusive scan and stable LSD radix sort for gfx950.
//
// These replace cub::DeviceScan::InclusiveSum and cub::DeviceRadixSort::SortPairs of the
// reference rasterizer [EXT].  Both are HBM-bound integer passes:
//   scan : reduce (read n) -> top scan of block sums (1 workgroup) -> downsweep (read n, write n)
//   sort : per pass histogram (read keys) -> scan of the [digit][block] matrix -> stable scatter
// Items are loaded striped (item k of thread t at base + k*256 + t) so every global access is a
// coalesced 256-lane sweep; stable ranking inside a workgroup uses ballot digit matching.
#include "gsr_kernels.h"
#include "gsr_wave.h"

namespace gsr {

__device__ __forceinline__ uint32_t count_of(const uint32_t* n_dev, int n_max) {
  if (n_dev == nullptr) return (uint32_t)n_max;
  const uint32_t n = *n_dev;
  return n < (uint32_t)n_max ? n : (uint32_t)n_max;
}

template <int MODE>
__device__ __forceinline__ uint32_t scan_load(const uint32_t* in, const uint32_t* idx, uint32_t i) {
  if (MODE == SCAN_PLAIN) return in[i];
  if (MODE == SCAN_FLAG) return in[i] > 0u ? 1u : 0u;
  return in[idx[i]];
}

template <int MODE>
__global__ __launch_bounds__(GSR_SCAN_THREADS) void k_scan_reduce(const uint32_t* __restrict__ in,
                                                                  const uint32_t* __restrict__ idx,
                                                                  const uint32_t* n_dev, int n_max,
                                                                  uint32_t* __restrict__ blk) {
  __shared__ uint32_t s_wave[GSR_SCAN_THREADS / 64 + 1];
  const uint32_t n = count_of(n_dev, n_max);
  const uint32_t base = blockIdx.x * GSR_SCAN_TILE;
  uint32_t sum = 0;
#pragma unroll
  for (int k = 0; k < GSR_SCAN_ITEMS; ++k) {
    const uint32_t i = base + k * GSR_SCAN_THREADS + threadIdx.x;
    if (i < n) sum += scan_load<MODE>(in, idx, i);
  }
  const uint32_t tot = block_sum_u32<GSR_SCAN_THREADS>(sum, s_wave);
  if (threadIdx.x == 0) blk[blockIdx.x] = tot;
}

// One workgroup scans the block sums in place (exclusive) and publishes the grand total.
__global__ __launch_bounds__(1024) void k_scan_top(uint32_t* __restrict__ blk, int nb, uint32_t* total) {
  __shared__ uint32_t s_wave[1024 / 64 + 1];
  uint32_t carry = 0;
  for (int start = 0; start < nb; start += 1024) {
    const int i = start + threadIdx.x;
    const uint32_t v = i < nb ? blk[i] : 0u;
    uint32_t tot;
    const uint32_t ex = block_exclusive_scan<1024>(v, &tot, s_wave);
    if (i < nb) blk[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0 && total != nullptr) *total = carry;
}

template <int MODE>
__global__ __launch_bounds__(GSR_SCAN_THREADS) void k_scan_down(const uint32_t* in,
                                                                const uint32_t* __restrict__ idx,
                                                                const uint32_t* n_dev, int n_max,
                                                                const uint32_t* __restrict__ blk,
                                                                uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint32_t s_v[GSR_SCAN_TILE];
  __shared__ uint32_t s_wave[GSR_SCAN_THREADS / 64 + 1];
  const uint32_t n = count_of(n_dev, n_max);
  const uint32_t base = blockIdx.x * GSR_SCAN_TILE;
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < GSR_SCAN_ITEMS; ++k) {
    const uint32_t i = base + k * GSR_SCAN_THREADS + t;
    s_v[k * GSR_SCAN_THREADS + t] = i < n ? scan_load<MODE>(in, idx, i) : 0u;
  }
  __syncthreads();
  // thread t owns the 8 consecutive items [8t, 8t+8) of the tile
  const uint4 a = *(const uint4*)&s_v[t * 8];
  const uint4 b = *(const uint4*)&s_v[t * 8 + 4];
  uint32_t x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint32_t run = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t v = x[k];
    x[k] = run;
    run += v;
  }
  uint32_t tot;
  const uint32_t off = block_exclusive_scan<GSR_SCAN_THREADS>(run, &tot, s_wave) + blk[blockIdx.x];
  *(uint4*)&s_v[t * 8] = make_uint4(x[0] + off, x[1] + off, x[2] + off, x[3] + off);
  *(uint4*)&s_v[t * 8 + 4] = make_uint4(x[4] + off, x[5] + off, x[6] + off, x[7] + off);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < GSR_SCAN_ITEMS; ++k) {
    const uint32_t i = base + k * GSR_SCAN_THREADS + t;
    if (i < n) out[i] = s_v[k * GSR_SCAN_THREADS + t];
  }
}

template <int MODE>
static void scan_impl(const uint32_t* in, const uint32_t* idx, uint32_t* out, const uint32_t* n_dev,
                      int n_max, uint32_t* blk, uint32_t* total, hipStream_t stream) {
  const int nb = scan_blocks(n_max);
  if (n_max <= 0) {
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, stream, blk, 0, total);
    return;
  }
  hipLaunchKernelGGL(k_scan_reduce<MODE>, dim3(nb), dim3(GSR_SCAN_THREADS), 0, stream, in, idx,
                     n_dev, n_max, blk);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, stream, blk, nb, total);
  hipLaunchKernelGGL(k_scan_down<MODE>, dim3(nb), dim3(GSR_SCAN_THREADS), 0, stream, in, idx,
                     n_dev, n_max, (const uint32_t*)blk, out);
}

void scan_exclusive(ScanMode mode, const uint32_t* in, const uint32_t* idx, uint32_t* out,
                    const uint32_t* n_dev, int n_max, uint32_t* blk, uint32_t* total,
                    hipStream_t stream) {
  switch (mode) {
    case SCAN_PLAIN: scan_impl<SCAN_PLAIN>(in, idx, out, n_dev, n_max, blk, total, stream); break;
    case SCAN_FLAG: scan_impl<SCAN_FLAG>(in, idx, out, n_dev, n_max, blk, total, stream); break;
    default: scan_impl<SCAN_GATHER>(in, idx, out, n_dev, n_max, blk, total, stream); break;
  }
}

// ---- radix sort --------------------------------------------------------------------------

__global__ __launch_bounds__(GSR_SCAN_THREADS) void k_radix_hist(const uint32_t* __restrict__ keys,
                                                                 const uint32_t* n_dev, int n_max,
                                                                 int shift, int bits,
                                                                 uint32_t* __restrict__ hist, int nb) {
  __shared__ uint32_t s_h[GSR_RADIX];
  const int t = threadIdx.x;
  const uint32_t n = count_of(n_dev, n_max);
  const uint32_t mask = (1u << bits) - 1u;
  s_h[t] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * GSR_SCAN_TILE;
#pragma unroll
  for (int k = 0; k < GSR_SCAN_ITEMS; ++k) {
    const uint32_t i = base + k * GSR_SCAN_THREADS + t;
    const bool valid = i < n;
    const uint32_t d = valid ? (keys[i] >> shift) & mask : 0u;
    const unsigned long long peers = match_digit(d, bits, valid);
    if (valid && mask_rank(peers) == 0) atomicAdd(&s_h[d], (uint32_t)__popcll(peers));
  }
  __syncthreads();
  if (t <= (int)mask) hist[(size_t)t * nb + blockIdx.x] = s_h[t];
}

__global__ __launch_bounds__(GSR_SCAN_THREADS) void k_radix_scatter(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out, const uint32_t* n_dev,
    int n_max, int shift, int bits, const uint32_t* __restrict__ hist, int nb) {
  __shared__ uint32_t s_base[GSR_RADIX];
  __shared__ uint32_t s_cnt[GSR_SCAN_THREADS / 64][GSR_RADIX];
  const int t = threadIdx.x, w = t >> 6;
  const uint32_t n = count_of(n_dev, n_max);
  const uint32_t mask = (1u << bits) - 1u;
  if (t <= (int)mask) s_base[t] = hist[(size_t)t * nb + blockIdx.x];
  const uint32_t base = blockIdx.x * GSR_SCAN_TILE;
  for (int k = 0; k < GSR_SCAN_ITEMS; ++k) {
    const uint32_t i = base + k * GSR_SCAN_THREADS + t;
    const bool valid = i < n;
    const uint32_t key = valid ? keys_in[i] : 0u;
    const uint32_t val = valid ? (vals_in ? vals_in[i] : i) : 0u;
    const uint32_t d = (key >> shift) & mask;
#pragma unroll
    for (int ww = 0; ww < GSR_SCAN_THREADS / 64; ++ww) s_cnt[ww][t] = 0;
    const unsigned long long peers = match_digit(d, bits, valid);
    const uint32_t rank = mask_rank(peers);
    __syncthreads();
    if (valid && rank == 0) s_cnt[w][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (t <= (int)mask) {
      uint32_t run = s_base[t];
#pragma unroll
      for (int ww = 0; ww < GSR_SCAN_THREADS / 64; ++ww) {
        const uint32_t c = s_cnt[ww][t];
        s_cnt[ww][t] = run;
        run += c;
      }
      s_base[t] = run;
    }
    __syncthreads();
    if (valid) {
      const uint32_t dst = s_cnt[w][d] + rank;
      keys_out[dst] = key;
      vals_out[dst] = val;
    }
    __syncthreads();
  }
}

int radix_sort_pairs(uint32_t* keys[2], uint32_t* vals[2], bool vals_identity, const uint32_t* n_dev,
                     int n_max, int key_bits, uint32_t* hist, uint32_t* hist_blk, hipStream_t stream) {
  if (key_bits < 1) key_bits = 1;
  const int passes = (key_bits + GSR_RADIX_BITS - 1) / GSR_RADIX_BITS;
  const int bits_per = (key_bits + passes - 1) / passes;
  const int nb = scan_blocks(n_max);
  int src = 0;
  for (int p = 0; p < passes; ++p) {
    const int shift = p * bits_per;
    const int bits = (key_bits - shift) < bits_per ? (key_bits - shift) : bits_per;
    const int dst = src ^ 1;
    if (n_max > 0) {
      hipLaunchKernelGGL(k_radix_hist, dim3(nb), dim3(GSR_SCAN_THREADS), 0, stream,
                         (const uint32_t*)keys[src], n_dev, n_max, shift, bits, hist, nb);
      scan_exclusive(SCAN_PLAIN, hist, nullptr, hist, nullptr, (1 << bits) * nb, hist_blk, nullptr,
                     stream);
      hipLaunchKernelGGL(k_radix_scatter, dim3(nb), dim3(GSR_SCAN_THREADS), 0, stream,
                         (const uint32_t*)keys[src], (const uint32_t*)((p == 0 && vals_identity) ? nullptr : vals[src]),
                         keys[dst], vals[dst], n_dev, n_max, shift, bits, (const uint32_t*)hist, nb);
    }
    src = dst;
  }
  return src;
}

}  // namespace gsr

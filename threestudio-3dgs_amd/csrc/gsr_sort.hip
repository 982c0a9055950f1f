// gsr_sort.hip — stable LSD radix sort of (key, value) pairs, one launch per digit pass.
//
// Replaces cub::DeviceRadixSort::SortPairs of the reference rasterizer [EXT].
// Each pass is a single "onesweep" launch: the digit counts of the whole input come from the
// producer kernel that wrote the keys (compaction / instance emission build them while the keys
// are in registers), so a pass only has to
//   1. load a 2048-item tile (striped: item k of thread t at base + k*256 + t, coalesced),
//   2. rank it stably inside the block (ballot digit matching per wave + per-wave counts),
//   3. publish the block's per-digit counts and resolve its per-digit global offsets by
//      decoupled look-back over the preceding blocks (gsr_wave.h),
//   4. reorder the tile in LDS by digit and write it out in digit runs.
// HBM traffic per pass: 8 B read + 8 B written per pair, plus R words of look-back state per
// 2048 pairs.  The previous design needed a histogram launch and a 3-launch scan per pass.
#include "gsr_kernels.h"
#include "gsr_wave.h"

namespace gsr {

__device__ __forceinline__ uint32_t count_of(const uint32_t* n_dev, int n_max) {
  if (n_dev == nullptr) return (uint32_t)n_max;
  const uint32_t n = *n_dev;
  return n < (uint32_t)n_max ? n : (uint32_t)n_max;
}

struct OnesweepLDS {
  uint32_t keys[GSR_SCAN_TILE];
  uint32_t vals[GSR_SCAN_TILE];
  uint32_t cnt[GSR_SCAN_THREADS / 64][GSR_RADIX];
  uint32_t run[GSR_RADIX];    // block-local running count per digit
  uint32_t glob[GSR_RADIX];   // global position of this block's first item of each digit
  uint32_t local[GSR_RADIX];  // block-local start of each digit
  uint32_t wave[8];
  uint32_t vid;
};

__global__ __launch_bounds__(GSR_SCAN_THREADS) void k_onesweep(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out, const uint32_t* n_dev, int n_max,
    int shift, int bits, const uint32_t* __restrict__ digit_count, uint32_t* state, uint32_t* ticket,
    uint32_t* err) {
  __shared__ OnesweepLDS s;
  GSR_PH_DECL
  const int t = threadIdx.x, w = t >> 6;
  if (t == 0) s.vid = atomicAdd(ticket, 1u);
  __syncthreads();
  const int vid = (int)s.vid;
  const uint32_t n = count_of(n_dev, n_max);
  const uint32_t base = (uint32_t)vid * GSR_SCAN_TILE;
  if (base >= n) return;
  const uint32_t mask = (1u << bits) - 1u;
  const int R = 1 << bits;

  uint32_t key[GSR_SCAN_ITEMS], val[GSR_SCAN_ITEMS];
#pragma unroll
  for (int k = 0; k < GSR_SCAN_ITEMS; ++k) {
    const uint32_t i = base + k * GSR_SCAN_THREADS + t;
    const bool valid = i < n;
    key[k] = valid ? keys_in[i] : 0u;
    val[k] = valid ? (vals_in ? vals_in[i] : i) : 0u;
  }
  // global start of each digit = exclusive scan of the pass's digit counts
  uint32_t tot;
  const uint32_t gstart = block_exclusive_scan<GSR_SCAN_THREADS>(t < R ? digit_count[t] : 0u, &tot, s.wave);
  s.run[t] = 0u;

  uint32_t pos[GSR_SCAN_ITEMS];
#pragma unroll
  for (int k = 0; k < GSR_SCAN_ITEMS; ++k) {
    const bool valid = base + k * GSR_SCAN_THREADS + t < n;
    const uint32_t d = (key[k] >> shift) & mask;
#pragma unroll
    for (int ww = 0; ww < GSR_SCAN_THREADS / 64; ++ww) s.cnt[ww][t] = 0u;
    const unsigned long long peers = match_digit(d, bits, valid);
    const uint32_t rank = mask_rank(peers);
    __syncthreads();
    if (valid && rank == 0) s.cnt[w][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (t < R) {
      uint32_t run = s.run[t];
#pragma unroll
      for (int ww = 0; ww < GSR_SCAN_THREADS / 64; ++ww) {
        const uint32_t c = s.cnt[ww][t];
        s.cnt[ww][t] = run;
        run += c;
      }
      s.run[t] = run;
    }
    __syncthreads();
    pos[k] = s.cnt[w][d] + rank;
    __syncthreads();
  }

  // this block's count per digit -> look-back -> global offsets
  GSR_PH_MARK(1)
  const uint32_t own = t < R ? s.run[t] : 0u;
  if (t < R) {
    uint32_t* st = state + (size_t)vid * R + t;
    uint32_t prefix = 0u;
    if (vid == 0) {
      lb_publish(st, GSR_LB_INC, own);
    } else {
      lb_publish(st, GSR_LB_AGG, own);
      prefix = lb_prefix_serial(state + t, (size_t)R, vid, err);
      lb_publish(st, GSR_LB_INC, prefix + own);
    }
    s.glob[t] = gstart + prefix;
  }
  uint32_t btot;
  const uint32_t lstart = block_exclusive_scan<GSR_SCAN_THREADS>(own, &btot, s.wave);
  if (t < R) s.local[t] = lstart;
  __syncthreads();
  GSR_PH_MARK(2)
  // reorder by digit in LDS, then write digit runs (consecutive lanes -> consecutive addresses)
#pragma unroll
  for (int k = 0; k < GSR_SCAN_ITEMS; ++k) {
    if (base + k * GSR_SCAN_THREADS + t < n) {
      const uint32_t d = (key[k] >> shift) & mask;
      const uint32_t lp = s.local[d] + pos[k];
      s.keys[lp] = key[k];
      s.vals[lp] = val[k];
    }
  }
  __syncthreads();
  const uint32_t nv = min((uint32_t)GSR_SCAN_TILE, n - base);
#pragma unroll
  for (int k = 0; k < GSR_SCAN_ITEMS; ++k) {
    const uint32_t j = k * GSR_SCAN_THREADS + t;
    if (j < nv) {
      const uint32_t kk = s.keys[j];
      const uint32_t d = (kk >> shift) & mask;
      const uint32_t dst = s.glob[d] + (j - s.local[d]);
      keys_out[dst] = kk;
      vals_out[dst] = s.vals[j];
    }
  }
  GSR_PH_STORE(n_dev ? GSR_PH_SORT_DEPTH : GSR_PH_SORT_TILE, (uint32_t)vid, (uint32_t)shift)
}



int onesweep_sort(uint32_t* keys[2], uint32_t* vals[2], bool vals_identity, const uint32_t* n_dev, int n_max,
                  int key_bits, const SortSync& sync, uint32_t* err, hipStream_t stream) {
  const DigitPlan plan = digit_plan(key_bits);
  const int nb = scan_blocks(n_max);
  int src = 0;
  for (int p = 0; p < plan.passes; ++p) {
    const int bits = plan.width(p, key_bits);
    const int dst = src ^ 1;
    if (n_max > 0)
      hipLaunchKernelGGL(k_onesweep, dim3(nb), dim3(GSR_SCAN_THREADS), 0, stream, (const uint32_t*)keys[src],
                         (const uint32_t*)((p == 0 && vals_identity) ? nullptr : vals[src]), keys[dst], vals[dst],
                         n_dev, n_max, p * plan.bits, bits, (const uint32_t*)(sync.digit_count + p * GSR_RADIX),
                         sync.states + (size_t)p * nb * ((size_t)1 << plan.bits), sync.tickets + p, err);
    src = dst;
  }
  return src;
}

}  // namespace gsr

#ifdef GSR_TIMELINE
GSR_PH_READER(gsr_diag_phases_sort)
#endif

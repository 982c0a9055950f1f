// gsr_sort.hip — view-segmented stable LSD radix sort of (key, value) pairs.
//
// Replaces cub::DeviceRadixSort::SortPairs of the reference rasterizer [EXT],
// which sorts one view at a time.  Here every view of a set is sorted by the same launches: the
// flat array holds one segment per view and each pass is reduce-then-scan over all segments:
//   count   : per 4096-item block, the digit histogram        -> counts[seg][digit][block]
//   scan    : per (segment, digit) row, exclusive scan over the segment's blocks; row total
//   scatter : per block, stable in-block ranking, global offset = scan(totals)[digit] +
//             counts[seg][digit][block] + rank; reorder in LDS; write digit runs.
// No block ever waits on another (no look-back, no spinning, no memsets): on MI355X a
// cross-workgroup hand-off is a cross-XCD round trip (≈1-3 µs), which made single-pass
// look-back chains the critical path (measured).  HBM traffic per pass:
// 4 B (count) + 8 B read + 8 B written per pair, plus 4 B x 256 per 4096 pairs of counts.
//
// In-block ranking is wave-blocked: wave w owns items [1024 w, 1024 w + 1024) of its block and
// walks them in 16 rounds of 64; a lane's rank among equal digits comes from ballot matching,
// the wave's running count per digit lives in LDS and is touched only by that wave, so the 16
// rounds need no workgroup barrier.  Order (wave, round, lane) = index order -> stable.
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "gsr_kernels.h"
#include "gsr_wave.h"

namespace gsr {

// Histogram copies the count kernel's lanes spread their LDS atomics over (lane mod GSR_COUNT_SUB), rows padded by
// one word so the copies of a digit sit in different banks: keys whose digits come in runs (a later pass over keys
// an earlier pass grouped — e.g. SuGaR's tile rows in depth order) had up to 64 lanes of one instruction adding to
// one counter, serialised (C5's second tile-sort count pass: 537 against 137 us per launch for the first).
#ifndef GSR_COUNT_SUB
#define GSR_COUNT_SUB 4
#endif
// BITS: the digit width at compile time (6 and 8: the ballot-matching loop unrolls), 0 = runtime `bits`.
template <int BITS>
__global__ __launch_bounds__(GSR_SORT_THREADS) void k_seg_count(const uint32_t* __restrict__ keys, SegInfo seg,
                                                                int shift, int bits_rt, int last,
                                                                uint32_t* __restrict__ counts) {
  const int bits = BITS ? BITS : bits_rt;
  if (seg_skip_last(seg, last)) return;
  const uint32_t kb = seg_key_base(seg);
  __shared__ uint32_t s_hist[GSR_COUNT_SUB * (GSR_RADIX + 1)];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t lb;
  const int v = seg_of_block(seg, xcd_block(blockIdx.x, gridDim.x), lb);  // (logical block: XCD-contiguous)
  const uint32_t n = seg_live(seg, v);
  const uint32_t* src = keys + seg.start[v];
  const uint32_t mask = (1u << bits) - 1u;
  const int R = 1 << bits;
  for (int i = t; i < GSR_COUNT_SUB * (GSR_RADIX + 1); i += GSR_SORT_THREADS) s_hist[i] = 0u;
  __syncthreads();
  uint32_t* const hist = s_hist + (lane & (GSR_COUNT_SUB - 1)) * (GSR_RADIX + 1);
  const uint32_t b0 = lb * GSR_SORT_TILE + w * (GSR_SORT_TILE / 4);
  // (full blocks: no per-item bounds, as k_seg_scatter)
  auto body = [&](auto full_c) {
    constexpr bool FULL = decltype(full_c)::value;
    uint32_t key[GSR_SORT_ITEMS];
#pragma unroll
    for (int k = 0; k < GSR_SORT_ITEMS; ++k) {
      const uint32_t i = b0 + k * 64 + lane;
      key[k] = FULL || i < n ? src[i] : 0u;
    }
#pragma unroll
    for (int k = 0; k < GSR_SORT_ITEMS; ++k) {
      const bool valid = FULL || b0 + k * 64 + lane < n;
      const uint32_t d = (seg_key(kb, key[k]) >> shift) & mask;
      // one LDS atomic per key: half the time of ballot-matching the digit first (24.4 -> 12.4 us/view
      // over the 5 passes; the histogram needs no ranks)
      if (valid) atomicAdd(&hist[d], 1u);
    }
  };
  if ((lb + 1) * GSR_SORT_TILE <= n)
    body(std::true_type{});
  else
    body(std::false_type{});
  __syncthreads();
  if (t < R) {
    const uint32_t nb = seg.blk[v + 1] - seg.blk[v];
    uint32_t c = 0u;
#pragma unroll
    for (int sb = 0; sb < GSR_COUNT_SUB; ++sb) c += s_hist[sb * (GSR_RADIX + 1) + t];
    counts[(size_t)R * seg.blk[v] + (size_t)t * nb + lb] = c;
  }
}

// One workgroup per (segment, digit) row: exclusive scan of the row in place, total -> totals.
__global__ __launch_bounds__(256) void k_seg_scan(SegInfo seg, int R, int last, uint32_t* __restrict__ counts,
                                                  uint32_t* __restrict__ totals) {
  if (seg_skip_last(seg, last)) return;
  __shared__ uint32_t s_wave[8];
  const int v = blockIdx.x / R, d = blockIdx.x % R;
  const int t = threadIdx.x;
  const uint32_t nb = seg.blk[v + 1] - seg.blk[v];
  uint32_t* row = counts + (size_t)R * seg.blk[v] + (size_t)d * nb;
  uint32_t carry = 0u;
  for (uint32_t c0 = 0; c0 < nb; c0 += 256 * 4) {
    // thread t owns 4 consecutive entries of this 1024-entry chunk
    uint32_t x[4], run = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t i = c0 + 4 * t + k;
      const uint32_t c = i < nb ? row[i] : 0u;
      x[k] = run;
      run += c;
    }
    uint32_t tot;
    const uint32_t off = carry + block_exclusive_scan<256>(run, &tot, s_wave);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t i = c0 + 4 * t + k;
      if (i < nb) row[i] = off + x[k];
    }
    carry += tot;
  }
  if (t == 0) totals[(size_t)v * GSR_RADIX + d] = carry;
}

template <bool KV>
struct ScatterLDS {
  uint32_t keys[GSR_SORT_TILE];
  uint32_t vals[KV ? GSR_SORT_TILE : 1];
  uint32_t wcnt[4][GSR_RADIX];  // per-wave running count per digit -> the wave's block-local start of the digit
  uint32_t glob[GSR_RADIX];     // segment position of this block's first item of each digit, less its local start
  uint32_t wave[8];
};

// KV = false: keys only (packed tile keys); vals_in / vals_out unused.
// (keys only: 5 waves per SIMD, 88 VGPRs without spills — the LDS allows 7 workgroups per CU, but at 6 waves the
// 80-VGPR budget spills in the full-block path; with values the LDS allows 4; profiles/r05/ab_r05s5.txt)
template <bool KV, int BITS, bool ATOMIC>
__attribute__((amdgpu_waves_per_eu(KV ? 4 : 5, 8)))
__global__ __launch_bounds__(GSR_SORT_THREADS) void k_seg_scatter(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in, uint32_t* __restrict__ keys_out,
    uint32_t* __restrict__ vals_out, SegInfo seg, int shift, int bits_rt, int last, const uint32_t* __restrict__ counts,
    const uint32_t* __restrict__ totals) {
  const int bits = BITS ? BITS : bits_rt;
  if (seg_skip_last(seg, last)) return;
  const uint32_t kb = seg_key_base(seg);
  __shared__ ScatterLDS<KV> s;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t lb;
  const int v = seg_of_block(seg, xcd_block(blockIdx.x, gridDim.x), lb);  // (logical block: XCD-contiguous)
  const uint32_t n = seg_live(seg, v);
  const uint32_t start = seg.start[v];
  const uint32_t mask = (1u << bits) - 1u;
  const int R = 1 << bits;
#pragma unroll
  for (int ww = 0; ww < 4; ++ww) s.wcnt[ww][t] = 0u;
  // the digit's segment total and this block's scanned count do not depend on the keys: loaded with them, so the
  // block pays one memory latency before its writes instead of two
  const uint32_t nb = seg.blk[v + 1] - seg.blk[v];
  const uint32_t dtot = t < R ? totals[(size_t)v * GSR_RADIX + t] : 0u;
  const uint32_t dcnt = t < R ? counts[(size_t)R * seg.blk[v] + (size_t)t * nb + lb] : 0u;
  const uint32_t b0 = lb * GSR_SORT_TILE + w * (GSR_SORT_TILE / 4);
  // FULL (every block but a segment's last): no per-item bounds, so each phase's loads, LDS accesses and stores
  // issue back to back instead of one guarded item at a time
  auto body = [&](auto full_c) {
    constexpr bool FULL = decltype(full_c)::value;
    uint32_t key[GSR_SORT_ITEMS], val[GSR_SORT_ITEMS];
    uint32_t pos2[GSR_SORT_ITEMS / 2];  // in-wave positions (< 1024), two 16-bit fields per register
#pragma unroll
    for (int k = 0; k < GSR_SORT_ITEMS; ++k) {
      const uint32_t i = b0 + k * 64 + lane;
      key[k] = FULL || i < n ? keys_in[start + i] : 0u;
      if (KV) val[k] = FULL || i < n ? (vals_in ? vals_in[start + i] : i) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < GSR_SORT_ITEMS; ++k) {
      const bool valid = FULL || b0 + k * 64 + lane < n;
      const uint32_t d = (seg_key(kb, key[k]) >> shift) & mask;
    if (ATOMIC) {
      const uint32_t pk = valid ? atomicAdd(&s.wcnt[w][d], 1u) : 0u;
      pos2[k >> 1] = (k & 1) ? (pos2[k >> 1] | (pk << 16)) : pk;
    } else {
      const unsigned long long peers = match_digit(d, bits, valid);
      const uint32_t rank = mask_rank(peers);
      // every lane reads its digit's running count, then the digit's first lane advances it.  The order across lanes
      // is explicit: the compiler barrier keeps the wave's ds_read before its ds_write in the program,
      // and the write's data is the read's result, so the wave issues the write only after the read has returned —
      // every lane's read sees the count before this round's add (no broadcast of the leader's value needed)
      const uint32_t base = s.wcnt[w][d];
      asm volatile("" ::: "memory");
      if (valid && rank == 0) s.wcnt[w][d] = base + (uint32_t)__popcll(peers);
      const uint32_t pk = base + rank;
      pos2[k >> 1] = (k & 1) ? (pos2[k >> 1] | (pk << 16)) : pk;
    }
    }
    __syncthreads();
    // per digit: each wave's block-local start (the digit's block-local start + the earlier waves' counts) and the
    // segment position of the block's run less its block-local start (one LDS read per item in each phase below)
    uint32_t wc[4], bc = 0u;
    if (t < R) {
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) {
        wc[ww] = s.wcnt[ww][t];
        bc += wc[ww];
      }
    }
    uint32_t tot;
    const uint32_t lstart = block_exclusive_scan<GSR_SORT_THREADS>(bc, &tot, s.wave);
    const uint32_t dstart = block_exclusive_scan<GSR_SORT_THREADS>(dtot, &tot, s.wave);
    if (t < R) {
      uint32_t run = lstart;
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) {
        s.wcnt[ww][t] = run;
        run += wc[ww];
      }
      s.glob[t] = dstart + dcnt - lstart;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < GSR_SORT_ITEMS; ++k) {
      if (FULL || b0 + k * 64 + lane < n) {
        uint32_t d = (seg_key(kb, key[k]) >> shift) & mask;
        asm volatile("" : "+v"(d));  // (recomputed, not kept from the ranking: 16 registers fewer)
        const uint32_t lp = s.wcnt[w][d] + ((pos2[k >> 1] >> (16 * (k & 1))) & 0xFFFFu);
        s.keys[lp] = key[k];
        if (KV) s.vals[lp] = val[k];
      }
    }
    __syncthreads();
    const uint32_t nv = FULL ? (uint32_t)GSR_SORT_TILE
                             : (lb * GSR_SORT_TILE < n ? min((uint32_t)GSR_SORT_TILE, n - lb * GSR_SORT_TILE) : 0u);
#pragma unroll
    for (int k = 0; k < GSR_SORT_ITEMS; ++k) {
      const uint32_t j = k * GSR_SORT_THREADS + t;
      if (FULL || j < nv) {
        const uint32_t kk = s.keys[j];
        const uint32_t d = (seg_key(kb, kk) >> shift) & mask;
        const uint32_t dst = start + s.glob[d] + j;
        keys_out[dst] = kk;
        if (KV) vals_out[dst] = s.vals[j];
      }
    }
  };
  if ((lb + 1) * GSR_SORT_TILE <= n)
    body(std::true_type{});
  else
    body(std::false_type{});
}

// In-wave ranks from LDS atomics (k_seg_scatter<.., ATOMIC = true>) are stable only if the LDS services one
// instruction's lanes that hit the same counter in lane order — what gfx950 does (the GPU sort and parity tests
// compare against stable sorts), but nothing the ISA promises.  So it is checked once per process on the device
// (k_lds_rank_probe: 32 rounds of digit patterns — one counter for all lanes, runs, pairs, hashed — every lane's
// returned count against its ballot-matched rank); if any lane disagrees, or GSR_SORT_RANK=ballot is set, every
// pass ranks by ballot matching.
#ifndef GSR_SORT_ATOMIC_MASK
#define GSR_SORT_ATOMIC_MASK 3  // bits 0 / 1: keys-only first / later passes, bits 2 / 3: key-value first / later
#endif

__global__ __launch_bounds__(256) void k_lds_rank_probe(uint32_t* __restrict__ bad) {
  __shared__ uint32_t cnt[4][64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  cnt[w][lane] = 0u;
  __syncthreads();
  uint32_t err = 0u;
  for (int r = 0; r < 32; ++r) {
    const uint32_t h = ((uint32_t)lane * 0x9E3779B1u) ^ ((uint32_t)r * 0x85EBCA6Bu);
    uint32_t d;
    switch (r & 3) {
      case 0: d = (uint32_t)r & 63u; break;                       // every lane one counter
      case 1: d = ((uint32_t)lane >> (r & 7)) & 63u; break;       // runs of 2^k lanes
      case 2: d = ((uint32_t)lane & ((r >> 2) & 7u)) & 63u; break;  // interleaved peers
      default: d = (h >> 26) & 63u; break;                        // hashed
    }
    const uint32_t got = atomicAdd(&cnt[w][d], 1u);
    const unsigned long long peers = match_digit(d, 6, true);
    const uint32_t first = (uint32_t)__shfl((int)got, (int)__builtin_ctzll(peers), 64);
    err |= (got - first) != mask_rank(peers) ? 1u : 0u;
  }
  if (err) atomicOr(bad, 1u);
}

// 1: LDS-atomic ranks in use, 0: ballot matching (probe failed, or GSR_SORT_RANK=ballot); decided once per process
int sort_rank_mode() {
  static const int mode = [] {
    const char* e = getenv("GSR_SORT_RANK");
    if (e != nullptr && strcmp(e, "ballot") == 0) return 0;
    uint32_t* d = nullptr;
    uint32_t h = 1u;
    if (hipMalloc(&d, sizeof(uint32_t)) != hipSuccess) return 0;
    bool ok = hipMemset(d, 0, sizeof(uint32_t)) == hipSuccess;
    if (ok) {
      hipLaunchKernelGGL(k_lds_rank_probe, dim3(1), dim3(256), 0, 0, d);
      ok = hipGetLastError() == hipSuccess && hipMemcpy(&h, d, sizeof(uint32_t), hipMemcpyDeviceToHost) == hipSuccess;
    }
    (void)hipFree(d);
    return ok && h == 0u ? 1 : 0;
  }();
  return mode;
}
template <int BITS>
static void launch_pass(bool kv, int pass, const uint32_t* kin, const uint32_t* vin, uint32_t* kout, uint32_t* vout,
                        const SegInfo& seg, uint32_t nb, int shift, int bits, int last, uint32_t* counts,
                        uint32_t* totals, hipStream_t stream) {
  hipLaunchKernelGGL(k_seg_count<0>, dim3(nb), dim3(GSR_SORT_THREADS), 0, stream, kin, seg, shift, bits, last,
                     counts);
  hipLaunchKernelGGL(k_seg_scan, dim3(seg.V << bits), dim3(256), 0, stream, seg, 1 << bits, last, counts, totals);
  const int sel = (pass == 0 ? 1 : 2) << (kv ? 2 : 0);
  const bool atomic = (GSR_SORT_ATOMIC_MASK & sel) != 0 && sort_rank_mode() == 1;
  const uint32_t* cc = counts;
  const uint32_t* tt = totals;
  if (kv) {
    if (atomic)
      hipLaunchKernelGGL((k_seg_scatter<true, BITS, true>), dim3(nb), dim3(GSR_SORT_THREADS), 0, stream, kin, vin, kout,
                         vout, seg, shift, bits, last, cc, tt);
    else
      hipLaunchKernelGGL((k_seg_scatter<true, BITS, false>), dim3(nb), dim3(GSR_SORT_THREADS), 0, stream, kin, vin,
                         kout, vout, seg, shift, bits, last, cc, tt);
  } else {
    if (atomic)
      hipLaunchKernelGGL((k_seg_scatter<false, BITS, true>), dim3(nb), dim3(GSR_SORT_THREADS), 0, stream, kin,
                         (const uint32_t*)nullptr, kout, (uint32_t*)nullptr, seg, shift, bits, last, cc, tt);
    else
      hipLaunchKernelGGL((k_seg_scatter<false, BITS, false>), dim3(nb), dim3(GSR_SORT_THREADS), 0, stream, kin,
                         (const uint32_t*)nullptr, kout, (uint32_t*)nullptr, seg, shift, bits, last, cc, tt);
  }
}

int seg_sort(uint32_t* keys[2], uint32_t* vals[2], bool vals_identity, SegInfo seg, int bit_lo, int key_bits,
             uint32_t* counts, uint32_t* totals, hipStream_t stream, int max_bits) {
  const bool kv = vals != nullptr && (vals[0] != nullptr || vals_identity);
  const DigitPlan plan = digit_plan(key_bits, max_bits);
  seg_fill_blocks(seg, GSR_SORT_TILE);
  const uint32_t nb = seg.blk[seg.V];
  int src = 0;
  for (int p = 0; p < plan.passes; ++p) {
    const int bits = plan.width(p, key_bits);
    const int dst = src ^ 1;
    if (nb > 0) {
      const int shift = bit_lo + p * plan.bits;
      const int last = p == plan.passes - 1 ? 1 : 0;
      const uint32_t* vin = (p == 0 && vals_identity) ? nullptr : (kv ? vals[src] : nullptr);
      uint32_t* vout = kv ? vals[dst] : nullptr;
      if (bits == 8)
        launch_pass<8>(kv, p, keys[src], vin, keys[dst], vout, seg, nb, shift, bits, last, counts, totals, stream);
      else if (bits == 6)
        launch_pass<6>(kv, p, keys[src], vin, keys[dst], vout, seg, nb, shift, bits, last, counts, totals, stream);
      else if (bits == 4)
        launch_pass<4>(kv, p, keys[src], vin, keys[dst], vout, seg, nb, shift, bits, last, counts, totals, stream);
      else
        launch_pass<0>(kv, p, keys[src], vin, keys[dst], vout, seg, nb, shift, bits, last, counts, totals, stream);
    }
    src = dst;
  }
  return src;
}

}  // namespace gsr

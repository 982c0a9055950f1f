// gsr_binning.hip — tile binning (replaces duplicateWithKeys,
// the 64-bit (tile | depth) radix sort and identifyTileRanges of the reference [EXT]).
//
// MI355X design: instead of radix-sorting K 64-bit (tile<<32 | depth) keys (41-45 key bits ->
// 6 passes over K), the visible Gaussians are depth-sorted once (N keys, 32 bits), the instances
// are emitted in depth order, and a stable sort on the tile id alone (12 bits at 1024^2 -> 2 passes
// over K) finishes the job.  Stability makes the result identical to the reference's order:
// per tile, ascending depth, ties by Gaussian index.
#include "gsr_kernels.h"

namespace gsr {

// Compact the visible Gaussians (tiles_touched > 0) into (depth bits, index) pairs.
__global__ __launch_bounds__(256) void k_compact_visible(int P, GeomState g) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  if (g.tiles_touched[i] == 0) return;
  const uint32_t o = g.vis_off[i];
  g.dkey[0][o] = __float_as_uint(g.rec1[i].z);  // view depth > 0.2: float bits are monotone
  g.dval[0][o] = (uint32_t)i;
}

void launch_compact_visible(int P, const GeomState& g, hipStream_t stream) {
  if (P <= 0) return;
  hipLaunchKernelGGL(k_compact_visible, dim3((P + 255) / 256), dim3(256), 0, stream, P, g);
}

// Emit one (tile id, Gaussian) instance per tile of each visible Gaussian, in depth order.
// `order` is the depth-sorted Gaussian list, `point_offsets` its exclusive instance scan.
__global__ __launch_bounds__(256) void k_duplicate(const uint32_t* __restrict__ n_dev, int P,
                                                   const uint32_t* __restrict__ order,
                                                   const uint32_t* __restrict__ point_offsets,
                                                   const uint2* __restrict__ rect, int grid_x,
                                                   uint32_t* __restrict__ keys,
                                                   uint32_t* __restrict__ vals,
                                                   uint32_t* __restrict__ goff) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nv = min(*n_dev, (uint32_t)P);
  if (r >= nv) return;
  const uint32_t gi = order[r];
  uint32_t off = point_offsets[r];
  goff[gi] = off;
  const uint2 rc = rect[gi];
  const int xmin = rc.x & 0xffff, ymin = rc.x >> 16, xmax = rc.y & 0xffff, ymax = rc.y >> 16;
  for (int y = ymin; y < ymax; ++y)
    for (int x = xmin; x < xmax; ++x) {
      keys[off] = (uint32_t)(y * grid_x + x);
      vals[off] = gi;
      ++off;
    }
}

void launch_duplicate(int P, int grid_x, const uint32_t* order, const GeomState& g,
                      const BinningState& b, hipStream_t stream) {
  if (P <= 0) return;
  hipLaunchKernelGGL(k_duplicate, dim3((P + 255) / 256), dim3(256), 0, stream,
                     (const uint32_t*)(g.counters + 0), P, order,
                     (const uint32_t*)g.point_offsets, (const uint2*)g.rect, grid_x, b.key[0],
                     b.val[0], g.goff);
}

// After the tile sort: per-tile [start, end) ranges of the sorted instance list.
__global__ __launch_bounds__(256) void k_tile_ranges(int K, const uint32_t* __restrict__ keys,
                                                     uint2* __restrict__ ranges) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= K) return;
  const uint32_t tile = keys[p];
  if (p == 0 || keys[p - 1] != tile) ranges[tile].x = (uint32_t)p;
  if (p == K - 1 || keys[p + 1] != tile) ranges[tile].y = (uint32_t)(p + 1);
}

void launch_tile_ranges(int K, const uint32_t* keys, uint2* ranges, hipStream_t stream) {
  if (K <= 0) return;
  hipLaunchKernelGGL(k_tile_ranges, dim3((K + 255) / 256), dim3(256), 0, stream, K, keys, ranges);
}

// markVisible / checkFrustum of the reference (API completeness).
__global__ __launch_bounds__(256) void k_mark_visible(int P, const float* __restrict__ means3D,
                                                      const float* __restrict__ view,
                                                      const float* __restrict__ proj,
                                                      uint8_t* __restrict__ present) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  const float3 p = make_float3(means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]);
  const float z = view[2] * p.x + view[6] * p.y + view[10] * p.z + view[14];
  present[i] = z > GSR_NEAR_CULL ? 1 : 0;
  (void)proj;
}

void launch_mark_visible(int P, const float* means3D, const float* view, const float* proj,
                         uint8_t* present, hipStream_t stream) {
  if (P <= 0) return;
  hipLaunchKernelGGL(k_mark_visible, dim3((P + 255) / 256), dim3(256), 0, stream, P, means3D, view,
                     proj, present);
}

}  // namespace gsr

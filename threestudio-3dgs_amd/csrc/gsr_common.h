// gsr_common.h — shared constants, workspace layouts and device math for the MI355X 3DGS
// rasterizer.  Host + device.  See DESIGN.md for the data layout in HBM.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#define GSR_TILE_X 16
#define GSR_TILE_Y 16
#define GSR_TILE_PIX (GSR_TILE_X * GSR_TILE_Y)  // 256 pixels = 4 waves of 64

// Scans and radix passes: 256 threads x 8 items per block.
#define GSR_SCAN_THREADS 256
#define GSR_SCAN_ITEMS 8
#define GSR_SCAN_TILE (GSR_SCAN_THREADS * GSR_SCAN_ITEMS)  // 2048
#define GSR_RADIX_BITS 8
#define GSR_RADIX (1 << GSR_RADIX_BITS)

// Rasterizer constants of the reference algorithm ([EXT] graphdeco
// cuda_rasterizer/forward.cu + auxiliary.h).
#define GSR_NEAR_CULL 0.2f
#define GSR_ALPHA_MAX 0.99f
#define GSR_ALPHA_MIN (1.0f / 255.0f)
#define GSR_T_EPS 0.0001f

namespace gsr {

static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Bump allocator used identically by the size queries and the pointer carving.
struct Carver {
  char* base;
  size_t off;
  __host__ __device__ Carver(void* b) : base((char*)b), off(0) {}
  template <typename T>
  T* take(size_t count) {
    off = align_up(off, 256);
    T* p = (T*)(base ? base + off : nullptr);
    off += count * sizeof(T);
    return p;
  }
};

static inline int div_up(long long a, long long b) { return (int)((a + b - 1) / b); }
static inline int scan_blocks(long long n) { return n <= 0 ? 1 : div_up(n, GSR_SCAN_TILE); }

// Per-Gaussian forward state ("geom").  rec0/rec1/rec2 are the 48-byte render record that the
// blend kernels gather per instance: rec0 = (px, py, conic_a, conic_b),
// rec1 = (conic_c, opacity, view depth, 0), rec2 = (r, g, b, 0).
struct GeomState {
  float4* rec0;
  float4* rec1;
  float4* rec2;
  uint2* rect;               // tile rect: x = xmin | ymin << 16, y = xmax | ymax << 16
  uint32_t* clamped;         // SH clamp flags, bit c = channel c clamped to 0
  uint32_t* tiles_touched;   // instances per Gaussian (0 = culled)
  uint32_t* vis_off;         // exclusive scan of (tiles_touched > 0)
  uint32_t* dkey[2];         // depth-sort ping-pong keys (float bits of view depth)
  uint32_t* dval[2];         // depth-sort ping-pong values (Gaussian index)
  uint32_t* point_offsets;   // exclusive scan of tiles_touched in depth order
  uint32_t* goff;            // first instance (pre-tile-sort position) of each Gaussian
  uint32_t* scan_blk;        // block sums for P-sized scans
  uint32_t* hist;            // radix histogram matrix [RADIX][blocks]
  uint32_t* hist_blk;        // block sums for scanning hist
  uint32_t* counters;        // [0] visible count, [1] K
  static GeomState carve(void* base, int P, size_t* bytes) {
    Carver c(base);
    GeomState g;
    size_t n = (size_t)(P > 0 ? P : 1);
    int nb = scan_blocks(P);
    g.rec0 = c.take<float4>(n);
    g.rec1 = c.take<float4>(n);
    g.rec2 = c.take<float4>(n);
    g.rect = c.take<uint2>(n);
    g.clamped = c.take<uint32_t>(n);
    g.tiles_touched = c.take<uint32_t>(n);
    g.vis_off = c.take<uint32_t>(n);
    g.dkey[0] = c.take<uint32_t>(n);
    g.dkey[1] = c.take<uint32_t>(n);
    g.dval[0] = c.take<uint32_t>(n);
    g.dval[1] = c.take<uint32_t>(n);
    g.point_offsets = c.take<uint32_t>(n);
    g.goff = c.take<uint32_t>(n);
    g.scan_blk = c.take<uint32_t>(nb + 64);
    g.hist = c.take<uint32_t>((size_t)GSR_RADIX * nb);
    g.hist_blk = c.take<uint32_t>(scan_blocks((long long)GSR_RADIX * nb) + 64);
    g.counters = c.take<uint32_t>(16);
    if (bytes) *bytes = align_up(c.off, 256);
    return g;
  }
};

// Per-instance state for the K (Gaussian, tile) pairs ("binning").
struct BinningState {
  uint32_t* key[2];        // tile id ping-pong
  uint32_t* val[2];        // Gaussian index ping-pong; after the sort: sorted position -> Gaussian
  uint32_t* hist;
  uint32_t* hist_blk;
  static BinningState carve(void* base, int K, size_t* bytes) {
    Carver c(base);
    BinningState b;
    size_t n = (size_t)(K > 0 ? K : 1);
    int nb = scan_blocks(K);
    b.key[0] = c.take<uint32_t>(n);
    b.key[1] = c.take<uint32_t>(n);
    b.val[0] = c.take<uint32_t>(n);
    b.val[1] = c.take<uint32_t>(n);
    b.hist = c.take<uint32_t>((size_t)GSR_RADIX * nb);
    b.hist_blk = c.take<uint32_t>(scan_blocks((long long)GSR_RADIX * nb) + 64);
    if (bytes) *bytes = align_up(c.off, 256);
    return b;
  }
};

// Per-pixel / per-tile state ("image").
struct ImageState {
  uint2* ranges;       // [tiles] sorted-instance range of each tile
  uint32_t* quad_maxc; // [4*tiles] per 8x8 quadrant: instances [0, maxc) of the tile list were blended
  uint4* tile_info;    // [tiles] (tile maxc, depth key and Gaussian of the first unblended instance, 0)
  float* final_T;      // [H*W]
  uint32_t* n_contrib; // [H*W]
  static ImageState carve(void* base, int W, int H, size_t* bytes) {
    Carver c(base);
    ImageState s;
    int tiles = div_up(W, GSR_TILE_X) * div_up(H, GSR_TILE_Y);
    size_t pix = (size_t)W * H;
    s.ranges = c.take<uint2>(tiles > 0 ? tiles : 1);
    s.quad_maxc = c.take<uint32_t>(4 * (size_t)(tiles > 0 ? tiles : 1));
    s.tile_info = c.take<uint4>(tiles > 0 ? tiles : 1);
    s.final_T = c.take<float>(pix > 0 ? pix : 1);
    s.n_contrib = c.take<uint32_t>(pix > 0 ? pix : 1);
    if (bytes) *bytes = align_up(c.off, 256);
    return s;
  }
};

// Backward scratch: one 48-byte gradient row per (instance, 8x8 quadrant), stored at
// 4 * slot + quadrant, slot = goff[g] + (row-major index of the tile inside the Gaussian's tile
// rect), so each Gaussian's rows are contiguous for the per-Gaussian gather-sum:
//   g0 = (dmean2D.x, dmean2D.y, dconic.a, dconic.b)   [pixel units; b in the reference's half convention]
//   g1 = (dconic.c, dopacity, dcolor.r, dcolor.g)
//   g2 = (dcolor.b, ddepth, 0, 0)
struct BackwardState {
  float4* grow;  // [12*K], row r = grow[3r .. 3r+2], r = 4 * slot + quadrant
  static BackwardState carve(void* base, int K, size_t* bytes) {
    Carver c(base);
    BackwardState s;
    s.grow = c.take<float4>((size_t)12 * (K > 0 ? K : 1));
    if (bytes) *bytes = align_up(c.off, 256);
    return s;
  }
};

// ---------------------------------------------------------------------------------------
// Device math shared by the forward and backward kernels.  The operation order mirrors the
// published reference algorithm so fp32 results agree with the CPU restatement in oracle/.

__device__ __forceinline__ float3 xform_point4x3(const float3 p, const float* m) {
  return make_float3(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
                     m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                     m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]);
}
__device__ __forceinline__ float4 xform_point4x4(const float3 p, const float* m) {
  return make_float4(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
                     m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                     m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14],
                     m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]);
}
__device__ __forceinline__ float3 xform_vec4x3_T(const float3 p, const float* m) {
  return make_float3(m[0] * p.x + m[1] * p.y + m[2] * p.z,
                     m[4] * p.x + m[5] * p.y + m[6] * p.z,
                     m[8] * p.x + m[9] * p.y + m[10] * p.z);
}
// ndc -> pixel.  The reference evaluates this in double (double literals) and rounds once.
__device__ __forceinline__ float ndc2pix(float v, int S) {
  return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5);
}

__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// Screen-space Gaussian exponent for pixel offset (dx, dy) = mean - pixel.  Written with
// explicit fmaf so the forward and backward kernels (and oracle/) evaluate it bit-identically:
// -0.5 (a dx^2 + c dy^2) - b dx dy.
__device__ __forceinline__ float gauss_power(float a, float b, float c, float dx, float dy) {
  float q = fmaf(c * dy, dy, (a * dx) * dx);
  return fmaf(-0.5f, q, -((b * dx) * dy));
}

}  // namespace gsr

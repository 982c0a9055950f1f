// gsr_common.h — shared constants, workspace layouts and device math for the MI355X 3DGS
// rasterizer.  Host + device.  See DESIGN.md for the data layout in HBM.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#define GSR_TILE_X 16
#define GSR_TILE_Y 16
#define GSR_TILE_PIX (GSR_TILE_X * GSR_TILE_Y)  // 256 pixels = 4 waves of 64

// Radix passes: 256 threads x 8 items per block, <= 8-bit digits.
#define GSR_SCAN_THREADS 256
#define GSR_SCAN_ITEMS 8
#define GSR_SCAN_TILE (GSR_SCAN_THREADS * GSR_SCAN_ITEMS)  // 2048
#define GSR_RADIX_BITS 8
#define GSR_RADIX (1 << GSR_RADIX_BITS)
#define GSR_MAX_PASSES 4
// Visible compaction: 256 threads x 16 Gaussians per block.  Instance emission: 256 x 4.
#define GSR_COMPACT_ITEMS 16
#define GSR_COMPACT_TILE (256 * GSR_COMPACT_ITEMS)  // 4096
#define GSR_DUP_ITEMS 4
#define GSR_DUP_TILE (256 * GSR_DUP_ITEMS)  // 1024

// Rasterizer constants of the reference algorithm ([EXT] graphdeco
// cuda_rasterizer/forward.cu + auxiliary.h).
#define GSR_NEAR_CULL 0.2f
#define GSR_ALPHA_MAX 0.99f
#define GSR_ALPHA_MIN (1.0f / 255.0f)
#define GSR_T_EPS 0.0001f

namespace gsr {

#ifdef GSR_TIMELINE
// Diagnostic build only (make diag): per-block phase stamps of the sort/binning kernels.
// Record = (t0, t1, t2, t3) s_memrealtime ticks (100 MHz), (HW_ID, XCC_ID, ticket id, extra).
#define GSR_PH_MAX 8192
enum { GSR_PH_COMPACT = 0, GSR_PH_SORT_DEPTH = 1, GSR_PH_SORT_TILE = 2, GSR_PH_DUP = 3, GSR_PH_KINDS = 4 };
static __device__ uint4 g_phase_tl[GSR_PH_KINDS][GSR_PH_MAX][2];  // one copy per translation unit
#define GSR_PH_READER(fname)                                                                           \
  extern "C" int fname(int kind, void* host, int n) {                                                 \
    if (kind < 0 || kind >= gsr::GSR_PH_KINDS || n > GSR_PH_MAX) return -1;                           \
    if (hipDeviceSynchronize() != hipSuccess) return -1;                                              \
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(gsr::g_phase_tl), sizeof(uint4) * 2 * n,              \
                               sizeof(uint4) * 2 * GSR_PH_MAX * kind, hipMemcpyDeviceToHost) == hipSuccess \
               ? 0 : -1;                                                                              \
  }
#define GSR_PH_DECL uint32_t ph_t[4] = {(uint32_t)__builtin_amdgcn_s_memrealtime(), 0u, 0u, 0u};
#define GSR_PH_MARK(i) ph_t[i] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#define GSR_PH_STORE(kind, vid, extra)                                                                   \
  if (threadIdx.x == 0 && (vid) < GSR_PH_MAX) {                                                         \
    ph_t[3] = (uint32_t)__builtin_amdgcn_s_memrealtime();                                               \
    g_phase_tl[kind][vid][0] = make_uint4(ph_t[0], ph_t[1], ph_t[2], ph_t[3]);                          \
    g_phase_tl[kind][vid][1] = make_uint4((uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4),          \
                                          (uint32_t)__builtin_amdgcn_s_getreg((15 << 11) | 20), (vid), (extra)); \
  }
#else
#define GSR_PH_DECL
#define GSR_PH_MARK(i)
#define GSR_PH_STORE(kind, vid, extra)
#endif

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

// Bits of a tile id (row-major over the 16x16 tile grid).
static inline int tile_key_bits(int W, int H) {
  const int tiles = div_up(W, GSR_TILE_X) * div_up(H, GSR_TILE_Y);
  int bits = 0;
  while ((1 << bits) < tiles) ++bits;
  return bits < 1 ? 1 : bits;
}

// LSD digit split of a key_bits-wide key: passes of equal width <= 8 bits.
struct DigitPlan {
  int passes, bits;
  __host__ __device__ int width(int p, int key_bits) const {
    const int lo = p * bits;
    return key_bits - lo < bits ? key_bits - lo : bits;
  }
};
static inline DigitPlan digit_plan(int key_bits) {
  if (key_bits < 1) key_bits = 1;
  DigitPlan d;
  d.passes = (key_bits + GSR_RADIX_BITS - 1) / GSR_RADIX_BITS;
  d.bits = (key_bits + d.passes - 1) / d.passes;
  return d;
}

// Zero-before-use words of one onesweep sort: digit counts [pass][256], block tickets [pass],
// look-back states [pass][block][R] (dense, R = 2^digit bits), the last region of its sync block
// so only the used prefix is zeroed.
struct SortSync {
  uint32_t* digit_count;
  uint32_t* tickets;
  uint32_t* states;
  int blocks;  // look-back blocks per pass (capacity)
  static size_t words(int blocks) { return GSR_MAX_PASSES * GSR_RADIX + 64 + (size_t)GSR_MAX_PASSES * blocks * GSR_RADIX; }
  static SortSync carve(uint32_t* w, int blocks) {
    SortSync s;
    s.digit_count = w;
    s.tickets = w + GSR_MAX_PASSES * GSR_RADIX;
    s.states = s.tickets + 64;
    s.blocks = blocks;
    return s;
  }
  // bytes from `sync_base` through the states a sort of n items with this plan touches
  size_t used_bytes(const uint32_t* sync_base, int passes, int bits, long long n) const {
    const size_t nb = (size_t)(n <= 0 ? 1 : (n + GSR_SCAN_TILE - 1) / GSR_SCAN_TILE);
    return (size_t)(states - sync_base) * sizeof(uint32_t) + (size_t)passes * nb * ((size_t)1 << bits) * sizeof(uint32_t);
  }
};

// The counters word block of a GeomState: [0] visible Gaussians, [1] K instances, [2] error flags
// (bit 0 look-back timeout), [3] compaction ticket, [4] emission ticket.
#define GSR_CTR_VISIBLE 0
#define GSR_CTR_K 1
#define GSR_CTR_ERR 2
#define GSR_CTR_TICKET_COMPACT 3
#define GSR_CTR_TICKET_DUP 4
#define GSR_NUM_COUNTERS 16

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
  uint32_t* dkey[2];         // depth-sort ping-pong keys (float bits of view depth)
  uint32_t* dval[2];         // depth-sort ping-pong values (Gaussian index)
  uint32_t* goff;            // first instance (pre-tile-sort position) of each Gaussian
  // zero-before-use region (one memset per preprocess): counters, compaction look-back, depth sort
  uint32_t* sync;
  size_t sync_bytes;
  uint32_t* counters;        // GSR_CTR_*
  uint32_t* compact_state;   // [blocks] compaction look-back
  SortSync dsort;            // depth sort, 4 x 8-bit passes over the visible Gaussians
  static GeomState carve(void* base, int P, size_t* bytes) {
    Carver c(base);
    GeomState g;
    size_t n = (size_t)(P > 0 ? P : 1);
    g.rec0 = c.take<float4>(n);
    g.rec1 = c.take<float4>(n);
    g.rec2 = c.take<float4>(n);
    g.rect = c.take<uint2>(n);
    g.clamped = c.take<uint32_t>(n);
    g.tiles_touched = c.take<uint32_t>(n);
    g.dkey[0] = c.take<uint32_t>(n);
    g.dkey[1] = c.take<uint32_t>(n);
    g.dval[0] = c.take<uint32_t>(n);
    g.dval[1] = c.take<uint32_t>(n);
    g.goff = c.take<uint32_t>(n);
    const int ncb = div_up((long long)n, GSR_COMPACT_TILE);
    const int nsb = scan_blocks((long long)n);
    const size_t words = GSR_NUM_COUNTERS + align_up(ncb, 64) + SortSync::words(nsb);
    g.sync = c.take<uint32_t>(words);
    g.sync_bytes = words * sizeof(uint32_t);
    g.counters = g.sync;
    g.compact_state = g.sync + GSR_NUM_COUNTERS;
    g.dsort = SortSync::carve(g.compact_state + align_up(ncb, 64), nsb);
    if (bytes) *bytes = align_up(c.off, 256);
    return g;
  }
};

// Per-instance state for the K (Gaussian, tile) pairs ("binning").
struct BinningState {
  uint32_t* key[2];        // tile id ping-pong
  uint32_t* val[2];        // Gaussian index ping-pong; after the sort: sorted position -> Gaussian
  // zero-before-use region (one memset per forward render): emission look-back, tile sort
  uint32_t* sync;
  size_t sync_bytes;
  uint32_t* dup_state;     // [blocks] emission look-back (visible Gaussians <= K)
  SortSync tsort;          // stable tile sort, <= 8-bit passes over K instances
  static BinningState carve(void* base, int K, size_t* bytes) {
    Carver c(base);
    BinningState b;
    size_t n = (size_t)(K > 0 ? K : 1);
    b.key[0] = c.take<uint32_t>(n);
    b.key[1] = c.take<uint32_t>(n);
    b.val[0] = c.take<uint32_t>(n);
    b.val[1] = c.take<uint32_t>(n);
    const int ndb = div_up((long long)n, GSR_DUP_TILE);
    const int nsb = scan_blocks((long long)n);
    const size_t words = align_up(ndb, 64) + SortSync::words(nsb);
    b.sync = c.take<uint32_t>(words);
    b.sync_bytes = words * sizeof(uint32_t);
    b.dup_state = b.sync;
    b.tsort = SortSync::carve(b.sync + align_up(ndb, 64), nsb);
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

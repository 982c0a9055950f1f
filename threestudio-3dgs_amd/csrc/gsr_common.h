// gsr_common.h — shared constants, workspace layouts and device math for the MI355X 3DGS
// rasterizer.  Host + device.  See DESIGN.md for the data layout in HBM.
#pragma once

#include <hip/hip_runtime.h>

// Timing experiments (GSR_EXP_*: parts of the blends compiled out) compute wrong results by design.  They build
// only as a diagnostic library (`make exp EXP=<name>` -> build_exp_<name>/libgsr_hip_exp.so, which defines
// GSR_DIAG_BUILD), never as the product libgsr_hip.so.
#if !defined(GSR_DIAG_BUILD) &&                                                                          \
    (defined(GSR_EXP_COALROWS) || defined(GSR_EXP_FWD_NOC) || defined(GSR_EXP_LDSPAD) ||                  \
     defined(GSR_EXP_NOCULL) || defined(GSR_EXP_NOFLUSH) || defined(GSR_EXP_NOGROUP) ||                   \
     defined(GSR_EXP_NOMFMA) || defined(GSR_EXP_NOREACH) || defined(GSR_EXP_NOREPLAY) ||                \
     defined(GSR_EXP_NOCOL2) || defined(GSR_EXP_HOTREC) || defined(GSR_EXP_NOEMBED))
#error "GSR_EXP_* experiment switches build only through `make exp` (a diagnostic library, not libgsr_hip.so)"
#endif
#include <stddef.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>

#define GSR_TILE_X 16
#define GSR_TILE_Y 16
#define GSR_TILE_PIX (GSR_TILE_X * GSR_TILE_Y)  // 256 pixels = 4 waves of 64

// View sets: up to GSR_SET_MAX views of one Gaussian set rendered by the same launches.
#define GSR_SET_MAX 64
// Sort passes: 256 threads x 16 items per block, <= 8-bit digits.
#define GSR_SORT_THREADS 256
#ifndef GSR_SORT_ITEMS
#define GSR_SORT_ITEMS 16
#endif
#define GSR_SORT_TILE (GSR_SORT_THREADS * GSR_SORT_ITEMS)  // 4096
#define GSR_RADIX_BITS 8
#define GSR_RADIX (1 << GSR_RADIX_BITS)
// Instance emission: 256 threads x 4 depth-sorted Gaussians per block.
#define GSR_GOFF_TILE 4096  // Gaussians per block of the gradient-row offset scan (256 threads x 16)
#define GSR_DUP_TILE 64  // depth-sorted Gaussians per emission group (one wave)

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

__host__ __device__ static inline int div_up(long long a, long long b) { return (int)((a + b - 1) / b); }

// Bits of a tile id (row-major over the 16x16 tile grid).
static inline int tile_key_bits(int W, int H) {
  const int tiles = div_up(W, GSR_TILE_X) * div_up(H, GSR_TILE_Y);
  int bits = 0;
  while ((1 << bits) < tiles) ++bits;
  return bits < 1 ? 1 : bits;
}

// Instance key layout.  When the Gaussian index and the tile id fit one 32-bit word together
// (1M Gaussians at 1024^2: 20 + 12 bits) the tile sort moves packed keys (tile << gbits | Gaussian)
// and no values: half the bytes of every binning pass.  Otherwise keys = tile, values = Gaussian.
// Unpacked keys carry beside the tile id, in bits [GSR_QMASK_SHIFT, +4), the instance's 8x8 quadrant mask
// (quadrant_hit of each quadrant, k_emit): the tile sort and k_tile_ranges look at the tile bits only, and the
// quadrant-wave forward gathers the records of its own quadrant's candidates only.
#define GSR_QMASK_SHIFT 28
struct TilePack {
  bool packed;
  bool qmask;  // keys hold the quadrant masks (unpacked)
  int gbits, tile_bits;
  uint32_t gmask;  // sorted entry -> Gaussian
  uint32_t tmask;  // key >> gbits -> tile id
};
// force: 0 = packed whenever both fit one word, 1 = keys + values at any size (keys with quadrant masks),
// 2 = the same without masks (gsr_api.hip tile_keys_mode(): GSR_TILE_KEYS, parity tests, read once per process)
static inline TilePack tile_pack(int P, int W, int H, int force_mode) {
  const bool force = force_mode != 0;
  TilePack t;
  t.tile_bits = tile_key_bits(W, H);
  int gb = 1;
  while (gb < 32 && (1ll << gb) < (long long)P) ++gb;
  t.packed = gb + t.tile_bits <= 32 && !force;
  t.gbits = t.packed ? gb : 0;
  t.gmask = t.packed ? (uint32_t)((1ull << gb) - 1ull) : 0xFFFFFFFFu;
  t.qmask = !t.packed && t.tile_bits <= GSR_QMASK_SHIFT && force_mode != 2;
  t.tmask = t.tile_bits >= 32 ? 0xFFFFFFFFu : (uint32_t)((1ull << t.tile_bits) - 1ull);
  return t;
}

// LSD digit split of a key_bits-wide key: passes of equal width <= 8 bits.
struct DigitPlan {
  int passes, bits;
  __host__ __device__ int width(int p, int key_bits) const {
    const int lo = p * bits;
    return key_bits - lo < bits ? key_bits - lo : bits;
  }
};
static inline DigitPlan digit_plan(int key_bits, int max_bits = GSR_RADIX_BITS) {
  if (key_bits < 1) key_bits = 1;
  if (max_bits < 1 || max_bits > GSR_RADIX_BITS) max_bits = GSR_RADIX_BITS;
  DigitPlan d;
  d.passes = (key_bits + max_bits - 1) / max_bits;
  d.bits = (key_bits + d.passes - 1) / d.passes;
  return d;
}
// Segments of a view set (kernel argument): segment v = items [start[v], start[v] + n[v]) of a
// flat array, cut into blocks of `tile` items; blocks of segment v are [blk[v], blk[v+1]).
// Item counts of a set stay below 2^32 (checked on the host).
// n[] is each segment's capacity (it sizes the grid); when ndev is set, the live item count of
// segment v is ndev[v] (<= n[v], produced on the device: no host round trip).
struct SegInfo {
  int V, tile;
  uint32_t n[GSR_SET_MAX];
  uint32_t start[GSR_SET_MAX];
  uint32_t blk[GSR_SET_MAX + 1];
  const uint32_t* ndev = nullptr;
  // depth sort only: [0] = smallest visible key of the set (keys are ranked as key - [0], culled ~0
  // stays ~0), [1] != 0 when every rebased visible key is < 2^24 - 1: the last (4th) pass is then a
  // no-op and its kernels return at once (the result stays in the 3rd pass's buffer)
  const uint32_t* rebase = nullptr;
};
__device__ __forceinline__ uint32_t seg_live(const SegInfo& s, int v) {
  return s.ndev ? min(s.ndev[v], s.n[v]) : s.n[v];
}
// the sort key of a raw key given the segment info's base (load it once per kernel: seg_key_base)
__device__ __forceinline__ uint32_t seg_key_base(const SegInfo& s) { return s.rebase ? s.rebase[0] : 0u; }
__device__ __forceinline__ uint32_t seg_key(uint32_t kb, uint32_t key) {
  return key == 0xFFFFFFFFu ? key : key - kb;
}
__device__ __forceinline__ bool seg_skip_last(const SegInfo& s, int last) {
  return last && s.rebase != nullptr && s.rebase[1] != 0u;
}
static inline void seg_fill_blocks(SegInfo& s, int tile) {
  // (ndev is left as set by the caller; SegInfo is otherwise plain data)
  s.tile = tile;
  s.blk[0] = 0;
  for (int v = 0; v < s.V; ++v) s.blk[v + 1] = s.blk[v] + (uint32_t)div_up((long long)s.n[v], tile);
}
// Logical block of workgroup b of an n-workgroup launch.  Speed only, never correctness (placement is no part of
// HIP's contract): workgroups are dealt round-robin over the 8 XCDs, so b and b + 8 share one; renumbered, each XCD
// works through one contiguous range of logical blocks, and the partial lines neighbouring blocks write (a sort
// pass's digit runs, a count row) meet in one L2 instead of eight.  A bijection of [0, n) for any n.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t n) {
  const uint32_t x = b & 7u, q = n >> 3, r = n & 7u;
  return x * q + (x < r ? x : r) + (b >> 3);
}
// block -> (segment, block within segment)
__device__ __forceinline__ int seg_of_block(const SegInfo& s, uint32_t b, uint32_t& lb) {
  int lo = 0, hi = s.V;  // blk[lo] <= b < blk[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (s.blk[mid] <= b) lo = mid;
    else hi = mid;
  }
  lb = b - s.blk[lo];
  return lo;
}

// One view of a set (kernel argument): camera pointers (device, 16/16/3 floats) and tan(fov/2).
struct ViewCam {
  const float *view, *proj, *campos;
  float tanx, tany;
  float fx, fy;  // focal lengths W / (2 tanx), H / (2 tany) (set by the host for the preprocess)
};
struct SetCams {
  ViewCam c[GSR_SET_MAX];
};

// The per-(view, Gaussian) record every per-instance gather reads: one 64-byte line.
//   a = (px, py, conic_a, conic_b), b = (conic_c, opacity, view depth, c2.x), c = (r, g, b, c2.y),
//   d = (tile rect xmin | ymin << 16, xmax | ymax << 16, c2.z, SH clamp flags)
// c2 = the two-colour render's second colour of the Gaussian when the preprocess was given one (PreprocessArgs::col2,
// recorded in drange[130..131]), else 0.
struct __attribute__((aligned(64))) GaussRec {
  float4 a, b, c;
  uint4 d;
};

// Per-(view, Gaussian) forward state of a view set ("geom"); element (v, i) at v * P + i.
struct GeomState {
  GaussRec* rec;
  uint2* tiles;              // x: tiles of the Gaussian's 3-sigma rectangle (0 = culled): its gradient
                             // rows; y: of those, tiles its alpha >= 1/255 ellipse reaches (span_row):
                             // its list instances
  uint32_t* dkey[2];         // depth sort ping-pong keys (float bits of view depth; culled = ~0)
  uint32_t* dval[2];         // depth sort ping-pong values: Gaussian index | min(kept tiles, vsent) << vbits
                             // (the kept count rides along so the instance counts stream; vsent = the
                             // count did not fit: read tiles.y)
  uint32_t* sort_counts;     // [V][RADIX][sort blocks] per-block digit counts -> scanned offsets
  uint32_t* sort_totals;     // [V][RADIX] digit totals
  uint32_t* kept_counts;     // [V][emission blocks] kept instances per block -> scanned offsets
  uint32_t* goff;            // [V][P] first gradient-row slot of each visible Gaussian: exclusive scan
                             // of tiles.x in Gaussian order (any disjoint assignment works; this one is
                             // written with coalesced stores)
  uint32_t* goff_part;       // [V][goff blocks] per-4096-Gaussian sums of tiles.x -> scanned offsets
  uint32_t* vis_part;        // [V][goff blocks] visible Gaussians per 4096-Gaussian block
  int vbits;                 // bits of the Gaussian index in the depth-sort values (from P)
  __host__ __device__ uint32_t vmask() const { return vbits >= 32 ? 0xFFFFFFFFu : (1u << vbits) - 1u; }
  // kept-count field of a depth-sort value: all ones = did not fit (or no room: P > 2^26)
  __host__ __device__ uint32_t vsent() const { return vbits > 26 ? 0u : (1u << (32 - vbits)) - 1u; }
  uint32_t* drange;          // depth key range of the set: [0, 64) min slots, [64, 128) max slots,
                             // [128] = min visible key, [129] = 1 if 3 depth-sort passes suffice,
                             // [130..131] = the colors2 pointer embedded in the records (0 = none)
  // the depth-sorted (keys, Gaussians) of every view: the 4th pass's output, or the 3rd's when it was skipped
  __device__ const uint32_t* sorted_dval() const { return drange[129] ? dval[1] : dval[0]; }
  __device__ const uint32_t* sorted_dkey() const { return drange[129] ? dkey[1] : dkey[0]; }
  uint32_t* counters;        // [0, V) rectangle tiles K of each view (the reference's num_rendered),
                             // [V, 2V) visible Gaussians, [2V, 3V) kept list instances
  static int sort_blocks(int P) { return div_up(P > 0 ? P : 1, GSR_SORT_TILE); }
  static int dup_blocks(int P) { return div_up(P > 0 ? P : 1, GSR_DUP_TILE); }
  static int goff_blocks(int P) { return div_up(P > 0 ? P : 1, GSR_GOFF_TILE); }
  static GeomState carve(void* base, int V, int P, size_t* bytes) {
    Carver c(base);
    GeomState g;
    const size_t n = (size_t)(V > 0 ? V : 1) * (size_t)(P > 0 ? P : 1);
    const size_t nv = (size_t)(V > 0 ? V : 1);
    g.rec = c.take<GaussRec>(n);
    g.tiles = c.take<uint2>(n);
    g.dkey[0] = c.take<uint32_t>(n);
    g.dkey[1] = c.take<uint32_t>(n);
    g.dval[0] = c.take<uint32_t>(n);
    g.dval[1] = c.take<uint32_t>(n);
    g.sort_counts = c.take<uint32_t>(nv * GSR_RADIX * sort_blocks(P));
    g.sort_totals = c.take<uint32_t>(nv * GSR_RADIX);
    g.kept_counts = c.take<uint32_t>(nv * dup_blocks(P));
    g.counters = c.take<uint32_t>(3 * nv + 64);
    g.goff = c.take<uint32_t>(n);
    g.goff_part = c.take<uint32_t>(nv * goff_blocks(P));
    g.vis_part = c.take<uint32_t>(nv * goff_blocks(P));
    g.vbits = 1;
    while (g.vbits < 32 && (1ull << g.vbits) < (unsigned long long)(P > 1 ? P : 2)) ++g.vbits;
    g.drange = c.take<uint32_t>(132);
    if (bytes) *bytes = align_up(c.off, 256);
    return g;
  }
};

// Per-instance state of a view set ("binning"): the (tile, Gaussian) pairs of view v are
// [start_v, start_v + K_v) with start_v = K_0 + ... + K_{v-1}.
// Aliasing contract: after the tile sort, key[r] (r = the sort's result index) holds the sorted list and key[r ^ 1]
// is free.  The tile-wave forward stores there, one byte per listed instance, the instance's 4-bit quadrant mask
// (RenderSet::qbytes) and records in ImageState::split_mode[1] that it did; the set's backward reads those bytes
// for its cull.  Nothing may write key[r ^ 1] between a set's forward and its backward(s) (the binning buffer
// belongs to that one forward: gsr_set_render ... gsr_set_backward in include/gsr.h).
struct BinningState {
  uint32_t* key[2];        // tile id ping-pong
  uint32_t* val[2];        // Gaussian index ping-pong; after the sort: sorted position -> Gaussian
  uint32_t* sort_counts;   // [RADIX x sort blocks of all views]
  uint32_t* sort_totals;   // [V][RADIX]
  // with_vals = false: packed keys (tile << gbits | Gaussian), no value arrays (TilePack)
  static BinningState carve(void* base, int V, long long Ktot, long long sort_blocks, bool with_vals, size_t* bytes) {
    Carver c(base);
    BinningState b;
    const size_t n = (size_t)(Ktot > 0 ? Ktot : 1);
    b.key[0] = c.take<uint32_t>(n);
    b.key[1] = c.take<uint32_t>(n);
    b.val[0] = with_vals ? c.take<uint32_t>(n) : nullptr;
    b.val[1] = with_vals ? c.take<uint32_t>(n) : nullptr;
    b.sort_counts = c.take<uint32_t>((size_t)GSR_RADIX * (size_t)(sort_blocks > 0 ? sort_blocks : 1));
    b.sort_totals = c.take<uint32_t>((size_t)GSR_RADIX * (size_t)(V > 0 ? V : 1));
    if (bytes) *bytes = align_up(c.off, 256);
    return b;
  }
};

// Backward tile splitting for launches of few tiles (V x tiles <= GSR_SPLIT_MAX_TILES: the per-view drop-in
// path, small images, small sets), whose duration is their longest tile's: a tile's blended prefix is walked
// in chunks of GSR_SPLIT_CH candidates by separate workgroups, each starting from the forward's per-pixel
// state at its chunk's end; at most GSR_SPLIT_NCK boundaries per tile (the last chunk takes the rest).
#define GSR_SPLIT_MAX_TILES 4096  // one 1024^2 view (measured: 4-view and 64-view x 256^2 sets gain nothing)
#define GSR_SPLIT_CH 256
#define GSR_SPLIT_NCK 15
__host__ __device__ inline bool split_fits(int V, size_t tiles) {
  return V >= 1 && tiles > 0 && (size_t)V * tiles <= GSR_SPLIT_MAX_TILES;
}
// backward workgroups for the listed later chunks (the list's capacity): a quarter of the set's tiles,
// 1024 .. 4096 (C3 per view lists ~800)
__host__ __device__ inline int split_extra(int V, size_t tiles) {
  const size_t e = (size_t)V * tiles / 4;
  return e < 1024 ? 1024 : e > 4096 ? 4096 : (int)e;
}
#define GSR_CKPT_FIELDS 5  // a plane of T, a plane of float4 (r, g, b, depth)
// Slot k of a tile (quadrant q's lane l = pixel 64 q + l): T at boundary k GSR_SPLIT_CH (slot 0: unused),
// then per pixel the colour / depth blended from candidate k CH on: the forward writes each chunk's own sums
// (chunk k = candidates [k CH, (k + 1) CH), the last slot to the list's end), k_ckpt_suffix turns them
// into suffix sums over the later chunks.  The colour behind a boundary is thus a sum of the later blends,
// never a difference of running totals (which would lose its bits where T is small).
__host__ __device__ inline size_t ckpt_offset(size_t vg, size_t tiles, size_t tile, int k) {
  return ((vg * tiles + tile) * (GSR_SPLIT_NCK + 1) + (size_t)k) * GSR_CKPT_FIELDS * 256;
}

// Per-pixel / per-tile state of a view set ("image"); view v's part at v * (tiles or H*W).
struct ImageState {
  uint2* ranges;       // [V][tiles] sorted-instance range of each tile (view-local positions)
  uint32_t* quad_maxc; // [V][4*tiles] per 8x8 quadrant: instances [0, maxc) of the tile list were blended
  uint4* tile_info;    // [V][tiles] (tile maxc, depth key and Gaussian of the first unblended instance, 0)
  uint2* cut;          // [V][tiles] (depth key, Gaussian) of tile_info: the backward gather's cut-off table
  float* final_T;      // [V][H*W]
  uint32_t* n_contrib; // [V][H*W]
  uint32_t* order;     // [V][super-tiles] each view's 2x2-tile super-tiles, most listed instances first
                       // (written after binning; the blends' dispatch order, gsr_render.hip block_map)
  uint32_t* split_mode;  // [0] != 0: the forward wrote the split backward's checkpoints (set_render writes it; the
                         // backward blend reads it on the device: the forward's decision, whatever the environment
                         // says by the time the backward runs); [1] != 0: the tile-wave forward wrote each
                         // listed instance's quadrant mask (RenderSet::qbytes)
  uint32_t* split_items; // split sets: [0] count, then the tiles' later chunks (gsr_render.hip k_ckpt_suffix)
  uint32_t* split_cap;   // split sets: [V][tiles] the end of the stretch the tile's own workgroup walks
  float* ckpt;           // carved last, only for a forward that splits (with_ckpt):
                         // [V][tiles][GSR_SPLIT_NCK + 1][5][256] chunk states for the split backward (ckpt_offset):
                         // 335 MB for one 1024^2 view, held until its backward
  static ImageState carve(void* base, int V, int W, int H, size_t* bytes, bool with_ckpt = true) {
    Carver c(base);
    ImageState s;
    const size_t nv = (size_t)(V > 0 ? V : 1);
    const size_t tiles = (size_t)div_up(W, GSR_TILE_X) * div_up(H, GSR_TILE_Y);
    const size_t pix = (size_t)W * H;
    s.split_mode = c.take<uint32_t>(2);
    s.ranges = c.take<uint2>(nv * (tiles > 0 ? tiles : 1));
    s.quad_maxc = c.take<uint32_t>(nv * 4 * (tiles > 0 ? tiles : 1));
    s.tile_info = c.take<uint4>(nv * (tiles > 0 ? tiles : 1));
    s.cut = c.take<uint2>(nv * (tiles > 0 ? tiles : 1));
    s.final_T = c.take<float>(nv * (pix > 0 ? pix : 1));
    s.n_contrib = c.take<uint32_t>(nv * (pix > 0 ? pix : 1));
    const size_t st = (size_t)((div_up(W, GSR_TILE_X) + 1) >> 1) * ((div_up(H, GSR_TILE_Y) + 1) >> 1);
    s.order = c.take<uint32_t>(nv * (st > 0 ? st : 1));
    const bool split = split_fits(V, tiles);
    s.split_items = c.take<uint32_t>(split ? 1 + (size_t)split_extra(V, tiles) : 1);
    s.split_cap = c.take<uint32_t>(split ? nv * tiles : 1);
    s.ckpt = c.take<float>(split && with_ckpt ? ckpt_offset(nv, tiles, 0, 0) : 1);
    if (bytes) *bytes = align_up(c.off, 256);
    return s;
  }
};

// Backward scratch for a group of views: one 48-byte gradient row per instance (summed over the
// tile's 4 quadrants), stored at slot = (view's first instance within the group) + goff[g] +
// (row-major index of the tile inside the Gaussian's tile rect), so each Gaussian's rows are
// contiguous for the per-Gaussian gather-sum:
//   g0 = (dmean2D.x, dmean2D.y, dconic.a, dconic.b)   [pixel units; b in the reference's half convention]
//   g1 = (dconic.c, dopacity, dcolor.r, dcolor.g)
//   g2 = (dcolor.b, ddepth, 0, 0)
// The two-colour backward (one pass for both of the SuGaR normal renderer's rasterizer calls) writes
// 64-byte rows: g0, g1 as above with the conic / opacity / mean2D terms of both calls' summed
// dL/dalpha,
//   g2 = (dcolor.b, ddepth, dcolor2.r, dcolor2.g)
//   g3 = (dcolor2.b, dmean2D_1.x, dmean2D_1.y, 0)   [the first call's own screen-space gradient]
// After the rows: the per-(view, Gaussian) records of gsr_backward.hip's first kernel,
// Per-(view, Gaussian) record of the backward's second stage: dmean3D (3), dcov3D (6), raw dcolor (3),
// dopacity (1), SH clamp flags (uint bits, 1); two-colour: + raw dcolor2 (3).
#define GSR_GRAD_FIELDS 14
#define GSR_GRAD_FIELDS2 17
// [views of the group][fields][P] floats.
// One (view, Gaussian) record of k_view_grad: GSR_GRAD_FIELDS floats (two colours: GSR_GRAD_FIELDS2) in a
// 16-byte aligned slot, written and read whole (four / five 16-byte accesses).
#define GSR_REC_STRIDE 16
#define GSR_REC_STRIDE2 20
struct BackwardState {
  unsigned long long* reach;  // [P]: bit v set = view v of the group gave the Gaussian a gradient row
  float4* grow;               // [3 (two colours: 4) * instances of the group]
  float* vrec;  // [views][P][GSR_REC_STRIDE (two colours: GSR_REC_STRIDE2)]; only the reached pairs' are written
  static size_t reach_bytes(int P) { return align_up(sizeof(unsigned long long) * (size_t)(P > 0 ? P : 1), 256); }
  static size_t rows_bytes(long long K, bool two = false) {
    return align_up(sizeof(float4) * (two ? 4 : 3) * (size_t)(K > 0 ? K : 1), 256);
  }
  static size_t bytes_for(long long K, int views, int P, bool two = false) {
    return reach_bytes(P) + rows_bytes(K, two) +
           align_up(sizeof(float) * (two ? GSR_REC_STRIDE2 : GSR_REC_STRIDE) * (size_t)views * (size_t)(P > 0 ? P : 1),
                    256);
  }
  static BackwardState carve(void* base, long long K, int P, bool two = false) {
    BackwardState s;
    s.reach = (unsigned long long*)base;
    s.grow = (float4*)((char*)base + reach_bytes(P));
    s.vrec = (float*)((char*)s.grow + rows_bytes(K, two));
    return s;
  }
};

// ---------------------------------------------------------------------------------------
// Device math shared by the forward and backward kernels.  The operation order mirrors the
// published reference algorithm so fp32 results agree with the CPU restatement in oracle/.

// Point transforms with an explicit operation order (left-to-right fma chains, as a contracting
// compiler evaluates the reference's m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12]); the oracle
// (oracle/gsr_oracle.c xform4x3 / xform4x4) uses the same chain, so view depths — and with them the
// depth order of nearly coincident Gaussians — agree bit for bit.
__device__ __forceinline__ float xform_row(float m0, float m1, float m2, float m3, const float3 p) {
  return fmaf(m2, p.z, fmaf(m1, p.y, m0 * p.x)) + m3;
}
__device__ __forceinline__ float3 xform_point4x3(const float3 p, const float* m) {
  return make_float3(xform_row(m[0], m[4], m[8], m[12], p), xform_row(m[1], m[5], m[9], m[13], p),
                     xform_row(m[2], m[6], m[10], m[14], p));
}
__device__ __forceinline__ float4 xform_point4x4(const float3 p, const float* m) {
  return make_float4(xform_row(m[0], m[4], m[8], m[12], p), xform_row(m[1], m[5], m[9], m[13], p),
                     xform_row(m[2], m[6], m[10], m[14], p), xform_row(m[3], m[7], m[11], m[15], p));
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

// The blends' form of the same exponent: the conic staged pre-multiplied (A = -0.5 log2e a,
// B = -log2e b, C = -0.5 log2e c) so that log2e * power = dx (A dx + B dy) + C dy^2 takes 5 fp32
// operations and alpha = o exp2(.) needs no log2e multiply (8 VALU per (pixel, Gaussian) instead of
// 11 with the subtractions).  Equal to gauss_power * log2e up to a few ulp (the reference's own
// rounding of this expression is no closer to exact).
#define GSR_CONIC_K_AC (-0.72134752044448170f)  // -0.5 log2(e)
#define GSR_CONIC_K_B (-1.4426950408889634f)    // -log2(e)
__device__ __forceinline__ float gauss_power2(float A, float B, float C, float dx, float dy) {
  return fmaf(dx, fmaf(A, dx, B * dy), (C * dy) * dy);
}

// Tile-level culling of a Gaussian's 3-sigma rectangle (the reference bins every rectangle tile).
// Tiles of row ty (pixel rows 16 ty .. 16 ty + 15) that contain a pixel with alpha >= 1/255:
// [tx0, tx1) within [xmin, xmax).  A pixel contributes only if o exp(-Q/2) >= 1/255 with
// Q = d^T conic d, d = mean - pixel, i.e. Q <= thr = 2 ln(255 o): the u = mean_x - x extent of
// that ellipse within the row band v = mean_y - y in [v1 - 15, v1] is [umin, umax] (the ellipse's
// own x-extreme (+-ue, -+ve) when it lies in the band, else where it crosses a band edge v_e:
// u = (-b v_e +- sqrt(thr a - D v_e^2)) / a, D = ac - b^2).  The bound is widened (threshold and
// extent margins) so rounding never drops a contributing tile; dropped tiles hold only pixels
// every blend step skips, so images and gradients are unchanged.  Every kernel that enumerates
// instances runs this same code (contraction off): the preprocess count, the emission and the
// gradient gather agree exactly.
struct SpanPrep {
  float px, py, b, D, ia, thra, ue, ve;
  int mode;  // 0: no tile, 1: every rectangle tile (degenerate conic), 2: ellipse
};
__device__ __forceinline__ SpanPrep span_prep(float px, float py, float a, float b, float c, float o) {
#pragma clang fp contract(off)
  SpanPrep p;
  p.px = px;
  p.py = py;
  p.b = b;
  p.D = a * c - b * b;
  p.mode = !(o >= GSR_ALPHA_MIN * 0.9999f) ? 0 : !(a > 0.0f && c > 0.0f && p.D > 0.0f) ? 1 : 2;
  const float tau = fmaxf(0.0f, __logf(255.0f * o));
  const float thr = 2.0f * (tau * 1.002f + 2e-3f);
  p.ia = __builtin_amdgcn_rcpf(a);
  p.thra = thr * a;
  p.ue = __builtin_amdgcn_sqrtf(thr * c * __builtin_amdgcn_rcpf(p.D));
  p.ve = b * p.ue * __builtin_amdgcn_rcpf(c);
  return p;
}
__device__ __forceinline__ void span_row(const SpanPrep& p, int ty, int xmin, int xmax, int& tx0, int& tx1) {
#pragma clang fp contract(off)
  tx0 = xmin;
  tx1 = p.mode == 1 ? xmax : xmin;
  if (p.mode != 2) return;
  const float v1 = p.py - (float)(ty * GSR_TILE_Y), v0 = v1 - (float)(GSR_TILE_Y - 1);
  float umax = -3.0e38f, umin = 3.0e38f;
  if (-p.ve >= v0 && -p.ve <= v1) umax = p.ue;
  if (p.ve >= v0 && p.ve <= v1) umin = -p.ue;
  const float e0 = p.thra - p.D * (v0 * v0), e1 = p.thra - p.D * (v1 * v1);
  if (e0 >= 0.0f) {
    const float r = __builtin_amdgcn_sqrtf(e0), m = -p.b * v0;
    umax = fmaxf(umax, (m + r) * p.ia);
    umin = fminf(umin, (m - r) * p.ia);
  }
  if (e1 >= 0.0f) {
    const float r = __builtin_amdgcn_sqrtf(e1), m = -p.b * v1;
    umax = fmaxf(umax, (m + r) * p.ia);
    umin = fminf(umin, (m - r) * p.ia);
  }
  if (!(umax >= umin)) return;  // the ellipse misses the band
  // pixel x in [16 tx, 16 tx + 15] has u in [px - 16 tx - 15, px - 16 tx]
  const float lo = fminf(fmaxf((p.px - (float)(GSR_TILE_X - 1) - umax - 0.05f) * (1.0f / GSR_TILE_X), -1.0e6f), 1.0e6f);
  const float hi = fminf(fmaxf((p.px - umin + 0.05f) * (1.0f / GSR_TILE_X), -1.0e6f), 1.0e6f);
  const int a0 = (int)ceilf(lo), a1 = (int)floorf(hi) + 1;
  tx0 = max(xmin, min(a0, xmax));
  tx1 = max(tx0, min(a1, xmax));
}
// The same bound on an 8-pixel band (pixel rows y with mean_y - y in [v1 - 7, v1]) at 8-pixel column
// granularity: the 8x8 quadrant columns c (pixels 8c .. 8c + 7) of the band that can hold a pixel with
// alpha >= 1/255, as c0 | c1 << 16 for [c0, c1) clamped to [0, 0x7fff] (k_emit's quadrant masks: two bands per
// tile row).  Same derivation and margins as span_row, so never tighter than a quadrant some pixel blends.
__device__ __forceinline__ uint32_t span_quads(const SpanPrep& p, float v1) {
#pragma clang fp contract(off)
  if (p.mode != 2) return p.mode == 1 ? 0x7fffu << 16 : 0u;
  const float v0 = v1 - 7.0f;
  float umax = -3.0e38f, umin = 3.0e38f;
  if (-p.ve >= v0 && -p.ve <= v1) umax = p.ue;
  if (p.ve >= v0 && p.ve <= v1) umin = -p.ue;
  const float e0 = p.thra - p.D * (v0 * v0), e1 = p.thra - p.D * (v1 * v1);
  if (e0 >= 0.0f) {
    const float r = __builtin_amdgcn_sqrtf(e0), m = -p.b * v0;
    umax = fmaxf(umax, (m + r) * p.ia);
    umin = fminf(umin, (m - r) * p.ia);
  }
  if (e1 >= 0.0f) {
    const float r = __builtin_amdgcn_sqrtf(e1), m = -p.b * v1;
    umax = fmaxf(umax, (m + r) * p.ia);
    umin = fminf(umin, (m - r) * p.ia);
  }
  if (!(umax >= umin)) return 0u;
  const float lo = fminf(fmaxf((p.px - 7.0f - umax - 0.05f) * 0.125f, -1.0f), 32767.0f);
  const float hi = fminf(fmaxf((p.px - umin + 0.05f) * 0.125f, -1.0f), 32767.0f);
  const int c0 = max(0, (int)ceilf(lo)), c1 = max(c0, min((int)floorf(hi) + 1, 0x7fff));
  return (uint32_t)c0 | (uint32_t)c1 << 16;
}
// quadrant mask of tile column tx from its row's two band ranges (span_quads of the upper / lower band)
__device__ __forceinline__ uint32_t quads_of_tile(uint32_t up, uint32_t dn, int tx) {
  const uint32_t c = 2u * (uint32_t)tx;
  auto in = [](uint32_t r, uint32_t x) { return x >= (r & 0xffffu) && x < (r >> 16); };
  return (in(up, c) ? 1u : 0u) | (in(up, c + 1u) ? 2u : 0u) | (in(dn, c) ? 4u : 0u) | (in(dn, c + 1u) ? 8u : 0u);
}

}  // namespace gsr

// gsr_kernels.h — host-side launchers for the device kernels (internal; the public ABI is
// include/gsr.h).  All launchers enqueue on `stream` and never synchronise.
#pragma once

#include "gsr_common.h"

namespace gsr {

// Stable LSD radix sort of every segment of a view set (segment v = n[v] pairs at start[v]) on
// key bits [bit_lo, bit_lo + key_bits), digit_plan(key_bits) passes of count / scan / scatter
// (gsr_sort.hip).  Ping-pongs between keys[0]/vals[0] and keys[1]/vals[1]; returns the index (0/1)
// holding the result.  vals_identity: the input values are the positions within the segment;
// vals == nullptr or vals[0] == nullptr (and not identity): keys only.  counts needs
// RADIX x (total 4096-item blocks) words, totals RADIX x V.
int seg_sort(uint32_t* keys[2], uint32_t* vals[2], bool vals_identity, SegInfo seg, int bit_lo, int key_bits,
             uint32_t* counts, uint32_t* totals, hipStream_t stream, int max_bits = GSR_RADIX_BITS);
// The scatter's in-wave ranking: 1 = LDS-atomic ranks (the device was probed to service same-counter lanes in lane
// order), 0 = ballot matching.  Decided once per process (gsr_sort.hip).
int sort_rank_mode();

// Forward preprocess (cull, project, EWA, SH) of every (view, Gaussian) — gsr_preprocess.hip
struct PreprocessArgs {
  int V, P, deg, M;
  const float *means3D, *scales, *rotations, *opacities, *shs, *colors_precomp, *cov3D_precomp;
  float scale_modifier;
  int W, H;
  int* radii;  // (V, P)
  // the second colour set of a two-colour render (colors2, (P, 3)) or null: written into the records' free slots
  // (GaussRec: b.w, c.w, d.z) so the two-colour blends read it with the record instead of gathering it apart
  const float* col2;
};
void launch_preprocess(const PreprocessArgs& a, const SetCams& cams, const GeomState& g, hipStream_t stream);

// Binning — gsr_binning.hip.  order = the depth sort's value buffer (per view: sorted position -> Gaussian).
void launch_binning_counts(int V, int P, const GeomState& g, hipStream_t stream);
// vals == nullptr: packed keys (tile << gbits | Gaussian)
// dkeys = the depth sort's key buffer (sorted depth keys; culled = ~0)
void launch_emit(int V, int P, int W, const GeomState& g, const SegInfo& inst, const TilePack& tp, uint32_t* keys,
                 uint32_t* vals, hipStream_t stream);
// per-tile [start, end) of each view's sorted list, by search (k_tile_bounds)
void launch_tile_ranges(SegInfo inst, int n_tiles, const TilePack& tp, const uint32_t* keys, uint2* ranges,
                        hipStream_t stream);
void launch_mark_visible(int P, const float* means3D, const float* view, const float* proj,
                         uint8_t* present, hipStream_t stream);

// Tile blend — gsr_render.hip.  A launch covers views v0 .. v0+V-1 of a set (geom / image arrays
// indexed by v0 + v); sorted_gauss = the tile sort's value buffer; inst_start[v] = the view's
// first instance in it; row_start[v] = the view's first gradient row slot in the backward scratch.
// Can some pixel centre of the 8x8 quadrant with origin (qx, qy) reach alpha >= 1/255 for this
// Gaussian?  alpha = o exp(-q/2), q = a dx^2 + 2 b dx dy + c dy^2 (dx = mean - pixel), so the pair
// can blend only if q <= 2 ln(255 o).  The test takes the exact minimum of q over the continuous
// rectangle spanned by the quadrant's pixel centres (<= the minimum over the pixels themselves) and
// compares it with a padded threshold, so it never drops a pair the reference would blend; for
// rotated, elongated footprints it is much tighter than the ellipse's bounding box.
__device__ __forceinline__ float quad_form(float a, float b, float c, float u, float v) {
  return fmaf(a * u, u, fmaf(2.0f * b * u, v, c * v * v));
}
__device__ __forceinline__ bool quadrant_hit(const float4 r0, const float4 r1, float qx, float qy) {
  const float o = r1.y;
  if (!(o >= GSR_ALPHA_MIN * 0.9999f)) return false;
  const float a = r0.z, b = r0.w, c = r1.x;
  if (!(a > 0.0f && c > 0.0f && a * c - b * b > 0.0f)) return true;
  const float tau = fmaxf(0.0f, __logf(255.0f * o));
  const float thr = 2.0f * (tau * 1.002f + 2e-3f);
  // dx ranges over [u0, u1], dy over [v0, v1]
  const float u1 = r0.x - qx, u0 = u1 - 7.0f;
  const float v1 = r0.y - qy, v0 = v1 - 7.0f;
  if (u0 <= 0.0f && u1 >= 0.0f && v0 <= 0.0f && v1 >= 0.0f) return true;
  const float ia = 1.0f / a, ic = 1.0f / c;
  // edges u = u0, u1: best v = clamp(-b u / c); edges v = v0, v1: best u = clamp(-b v / a)
  const float q0 = quad_form(a, b, c, u0, fminf(fmaxf(-b * u0 * ic, v0), v1));
  const float q1 = quad_form(a, b, c, u1, fminf(fmaxf(-b * u1 * ic, v0), v1));
  const float q2 = quad_form(a, b, c, fminf(fmaxf(-b * v0 * ia, u0), u1), v0);
  const float q3 = quad_form(a, b, c, fminf(fmaxf(-b * v1 * ia, u0), u1), v1);
  const float qmin = fminf(fminf(q0, q1), fminf(q2, q3));
  return qmin * 0.998f <= thr;
}

struct RenderSet {
  int V, v0, P, W, H, gx, gy;
  uint32_t gmask;  // sorted entry -> Gaussian (TilePack)
  uint32_t inst_start[GSR_SET_MAX];
  uint32_t row_start[GSR_SET_MAX];
  const float* bg[GSR_SET_MAX];
  // fused background composite (renderer/diff_gaussian_rasterizer_background.py:129-132,139), null = off.
  // Pointers at the launch's first view; per view (H, W, 3) background images / (3, H, W) planes.
  const float* cbg;  // background network images (V, H, W, 3)
  float* comp;       // forward: clamp(color + (1 - alpha) bg, 0, 1) (V, 3, H, W)
  const float* ccolor;  // backward: the forward's colour (V, 3, H, W); dL_dcolor then holds dL/dcomp
  float* dcbg;       // backward: dL/dbg (V, H, W, 3) or null
  // a second colour per Gaussian blended with the same weights (the SuGaR normal renderer's second
  // rasterizer call, renderer/diff_sugar_rasterizer_normal.py:182-191: same geometry, colors_precomp =
  // the face normals), (P, 3); null = off.  Forward: blended into out_col2 (V, 3, H, W) beside the
  // first colour.  Backward: replaces the records' colour (the second call's backward).
  const float* col2;
  float* out_col2;
  // backward of both calls in one pass: dL/d(second colour image) (V, 3, H, W) at the launch's first
  // view; col2 then holds the second colours and the records keep the first (null = off)
  const float* dpix2;
  // dispatch order (ImageState::order of the set, indexed by v0 + v): null = views in turn, raster order
  const uint32_t* order;
  // with an order: views whose super-tiles are dealt heaviest-first together (block_map; order_chunk)
  int ochunk;
  // split backward (gsr_render.hip split_on): the forward writes its checkpoints here, the backward walks the
  // tiles in chunks from them; null = off
  float* ckpt;
  const uint32_t* split_mode;  // backward: ImageState::split_mode (did the forward write the checkpoints?)
  // GeomState::drange + 130: the colors2 pointer the set's preprocess embedded in the records (two words; 0 = none).
  // A two-colour kernel reads the second colours from the records when it equals col2, else from col2 itself
  const uint32_t* col2_rec;
  uint32_t* split_items;  // with ckpt: the later chunks' backward items (ImageState::split_items)
  uint32_t* split_cap;    // with ckpt: ImageState::split_cap
  int split_extra;        // with ckpt: split_extra(the set's V, tiles)
  // the sorted keys when they carry the quadrant masks (TilePack::qmask; indexed like the sorted Gaussians),
  // else null
  const uint32_t* qkeys;
  // per listed instance (indexed like the sorted Gaussians) its 4-bit quadrant mask, in the binning buffer's free
  // ping-pong key array: the tile-wave forward writes it, the lockstep backward reads it instead of recomputing
  // its cull when split_mode[1] says the forward wrote it
  uint8_t* qbytes;
};
// backward tile splitting on for a set of V views (split_fits) whose forward takes the quadrant-wave kernel
// (GSR_BWD_SPLIT=0 turns it off); instances = the set's K total
bool split_on(int V, int P, int width, int height, long long instances);
// the forward of a set takes the one-wave-per-tile kernel (k_render_fwd_tile)
bool fwd_tile_chosen(long long instances, long long gaussians, int views);
// the dispatch-order chunk of a blend launch over V views of gx x gy tiles (forward or backward) — gsr_render.hip
int order_chunk(int V, int gx, int gy, bool forward);
// the blend kernel the last forward (0) / backward (1) blend launch used, as rocprofv3 names it
const char* blend_kernel_name(int which);
// the forward of this set writes split checkpoints: split_on for one colour set (the two-colour backward never
// splits); the image buffer holds checkpoints only then (gsr_set_image_bytes_ex)
inline bool split_forward(int V, int P, int width, int height, long long instances, bool two_colors) {
  return !two_colors && split_on(V, P, width, height, instances);
}
// Each view's super-tiles by listed instances, heaviest first (after binning) — gsr_render.hip
void launch_tile_order(int V, int gx, int gy, const uint2* ranges, uint32_t* order, hipStream_t stream);
// instances: the set's rectangle tiles (sum of K) — picks the forward kernel (gsr_render.hip)
void launch_render_forward(const RenderSet& rs, const GeomState& g, const uint32_t* sorted_gauss,
                           const ImageState& img, float* out_color, float* out_depth, float* out_alpha,
                           long long instances, hipStream_t stream);
// dL_d* point at view v0's planes.
void launch_render_backward(const RenderSet& rs, const GeomState& g, const uint32_t* sorted_gauss,
                            const ImageState& img, const float* dL_dcolor, const float* dL_ddepth,
                            const float* dL_dalpha, const BackwardState& bw, hipStream_t stream);

// Fused per-Gaussian backward over a batch of views — gsr_backward.hip
struct GaussBackwardArgs {  // shared Gaussian parameters and the gradients of them (summed over views)
  int P, deg, M;
  int g0, g1;  // the Gaussians [g0, g1) this launch covers (all: 0, P)
  const float *means3D, *scales, *rotations, *shs, *cov3D_precomp;
  float scale_modifier;
  float *dL_dcolors, *dL_dopacity, *dL_dmeans3D, *dL_dcov3D, *dL_dsh, *dL_dscales, *dL_drotations;
};
// A: per (view, Gaussian) gather + screen-space chain rule for views v0 .. v0+V-1 of a set.
struct ViewGradArgs {
  int V, v0, W, H, gx, tiles, cut_in_lds, items;  // items: Gaussians per thread (launch_gauss_backward)
  GeomState g;
  ImageState img;
  const unsigned long long* reach;  // [P] reach bits of this group's views (k_render_bwd)
  const float4* grow;      // gradient rows of this group of views
  float* dmeans2D;         // the set's (V, P, 3)
  float* vrec;             // [V][P][GSR_REC_STRIDE(2)] records of this group (reached pairs only)
  uint32_t row_start[GSR_SET_MAX];
  ViewCam cam[GSR_SET_MAX];
};
// B: per Gaussian, sums the group's records, SH backward per view, scale / rotation once.
struct AccumArgs {
  int V, v0, accumulate, pad_;
  const unsigned long long* reach;  // [P] reach bits of this group's views: the records to read
  const float* vrec;
  // running dL/dcov3D over the groups / sets already summed (P x 6; the dL_dcov3D output itself when the
  // caller wants it): with accumulate, every sum continues from the stored value in view order, so a
  // backward split into view groups is bitwise equal to one group, and the scale / rotation gradients
  // are recomputed from the running total instead of being added per group
  float* dcov_carry;
  // two-colour backward: dL/dcolors2 (P x 3; with accumulate continued from the stored value); its
  // records have GSR_GRAD_FIELDS2 fields and rows 4 float4 (null = the one-colour layout)
  float* dcolors2;
  const float* campos[GSR_SET_MAX];
};
// Background composite epilogue — gsr_epilogue.hip.
void launch_composite_fwd(int V, size_t HW, const float* color, const float* alpha, const float* bg, int layout,
                          float* out, hipStream_t stream);
void launch_composite_bwd(int V, size_t HW, const float* dout, const float* color, const float* alpha,
                          const float* bg, int layout, float* dcolor, float* dalpha, float* dbg,
                          hipStream_t stream);
// SuGaR normal map (normalize, flip, alpha-weighted map, alpha > 0.99 gradient mask) — gsr_epilogue.hip.
void launch_normal_map_fwd(int V, size_t HW, const float* normal, const float* alpha, float* out, hipStream_t stream);
void launch_normal_map_bwd(int V, size_t HW, const float* dout, const float* normal, const float* alpha,
                           float* dnormal, float* dalpha, hipStream_t stream);
// Shading / depth-normal epilogue — gsr_shading.hip (include/gsr.h gsr_shade_*).
struct ShadeArgs {
  // a launch covers views v0 .. v0+V-1 (V <= GSR_SET_MAX); the view planes below are the whole call's
  int V, v0, H, W, flags, bg_layout;  // bg_layout: GSR_BG_CONSTANT (V, 3) or GSR_BG_HWC (V, H, W, 3)
  const float* color;        // (V, 3, H, W)   material only
  const float* depth;        // (V, 1, H, W)
  const float* alpha;        // (V, 1, H, W)
  const float* rays_o;       // (V, H, W, 3)
  const float* rays_d;       // (V, H, W, 3)
  const float* bg;           // material only
  const float* light;        // (V, 3)         material only
  const float* pred_normal;  // (V, 3, H, W) or null
  // per view of the launch (index v - v0): ambient / diffuse light colours and shading mode — the material
  // draws them per view (material/gaussian_material.py:59-64,80-88, called once per view)
  float ka[GSR_SET_MAX][3], kd[GSR_SET_MAX][3];
  int mode[GSR_SET_MAX];
  float* render;             // (V, 3, H, W)   material only
  float* nmap;               // (V, 3, H, W) or null
  float* unit;               // (V, 3, H, W) or null
  float* depth_out;          // (V, 1, H, W) or null
};
struct ShadeGrads {
  const float* d_render;     // upstream gradients, any may be null
  const float* d_nmap;
  const float* d_unit;
  const float* d_depth_out;
  float* d_color;            // outputs (d_color, d_bg: material only; d_bg null = not formed)
  float* d_depth;
  float* d_alpha;
  float* d_bg;
};
void launch_shade_fwd(const ShadeArgs& A, hipStream_t stream);
void launch_shade_bwd(const ShadeArgs& A, const ShadeGrads& G, hipStream_t stream);
// 3-NN mean squared distance (simple_knn.distCUDA2) — gsr_knn.hip.
size_t knn_workspace_bytes(int P);
int launch_knn_mean_dist(int P, const float* points, float* out, void* workspace, hipStream_t stream);
void launch_gauss_backward(const GaussBackwardArgs& a, ViewGradArgs va, const AccumArgs& b, hipStream_t stream);

}  // namespace gsr

// gsr_kernels.h — host-side launchers for the device kernels (internal; the public ABI is
// include/gsr.h).  All launchers enqueue on `stream` and never synchronise.
#pragma once

#include "gsr_common.h"

namespace gsr {

// Stable LSD radix sort of every segment of a view set (segment v = n[v] pairs at start[v]) on
// key bits [0, key_bits), digit_plan(key_bits) passes of count / scan / scatter (gsr_sort.hip).
// Ping-pongs between keys[0]/vals[0] and keys[1]/vals[1]; returns the index (0/1) holding the
// result.  vals_identity: the input values are the positions within the segment.  counts needs
// RADIX x (total 4096-item blocks) words, totals RADIX x V.
int seg_sort(uint32_t* keys[2], uint32_t* vals[2], bool vals_identity, SegInfo seg, int key_bits,
             uint32_t* counts, uint32_t* totals, hipStream_t stream);

// Forward preprocess (cull, project, EWA, SH) of every (view, Gaussian) — gsr_preprocess.hip
struct PreprocessArgs {
  int V, P, deg, M;
  const float *means3D, *scales, *rotations, *opacities, *shs, *colors_precomp, *cov3D_precomp;
  float scale_modifier;
  int W, H;
  int* radii;  // (V, P)
};
void launch_preprocess(const PreprocessArgs& a, const SetCams& cams, const GeomState& g, hipStream_t stream);

// Binning — gsr_binning.hip.  order = the depth sort's value buffer (per view: sorted position -> Gaussian).
void launch_binning_counts(int V, int P, const GeomState& g, const uint32_t* order, hipStream_t stream);
void launch_emit(int V, int P, int W, const GeomState& g, const uint32_t* order, const SegInfo& inst,
                 uint32_t* keys, uint32_t* vals, hipStream_t stream);
void launch_tile_ranges(SegInfo inst, int n_tiles, const uint32_t* keys, uint2* ranges, hipStream_t stream);
void launch_mark_visible(int P, const float* means3D, const float* view, const float* proj,
                         uint8_t* present, hipStream_t stream);

// Tile blend — gsr_render.hip.  A launch covers views v0 .. v0+V-1 of a set (geom / image arrays
// indexed by v0 + v); sorted_gauss = the tile sort's value buffer; inst_start[v] = the view's
// first instance in it; row_start[v] = the view's first gradient row slot in the backward scratch.
struct RenderSet {
  int V, v0, P, W, H, gx, gy;
  uint32_t inst_start[GSR_SET_MAX];
  uint32_t row_start[GSR_SET_MAX];
  const float* bg[GSR_SET_MAX];
};
void launch_render_forward(const RenderSet& rs, const GeomState& g, const uint32_t* sorted_gauss,
                           const ImageState& img, float* out_color, float* out_depth, float* out_alpha,
                           hipStream_t stream);
// dL_d* point at view v0's planes.
void launch_render_backward(const RenderSet& rs, const GeomState& g, const uint32_t* sorted_gauss,
                            const ImageState& img, const float* dL_dcolor, const float* dL_ddepth,
                            const float* dL_dalpha, const BackwardState& bw, hipStream_t stream);

// Fused per-Gaussian backward over a batch of views — gsr_backward.hip
struct GaussBackwardArgs {  // shared Gaussian parameters and the gradients of them (summed over views)
  int P, deg, M;
  const float *means3D, *scales, *rotations, *shs, *cov3D_precomp;
  float scale_modifier;
  float *dL_dcolors, *dL_dopacity, *dL_dmeans3D, *dL_dcov3D, *dL_dsh, *dL_dscales, *dL_drotations;
};
struct ViewDesc {  // one view's camera, forward state, gradient rows and its means2D gradient output
  const float *view, *proj, *campos;
  const int* radii;
  const float4* rec1;
  const uint2* rect;
  const uint32_t *goff, *clamped;
  const uint4* tile_info;
  const float4* grow;
  float* dmeans2D;
  float tanx, tany, fx, fy;
  int grid_x, pad_;
};
#define GSR_VIEWS_PER_LAUNCH 16
struct ViewBatch {  // passed by value as kernel arguments (16 x 112 B)
  int n, accumulate;
  ViewDesc v[GSR_VIEWS_PER_LAUNCH];
};
// View vg of a set; radii = the set's (V, P) radii; grow = the view's first gradient row.
ViewDesc make_view_desc(const ViewCam& cam, int vg, int P, const int* radii, const GeomState& g,
                        const ImageState& img, const float4* grow, float* dmeans2D, int W, int H);
void launch_gauss_backward_views(const GaussBackwardArgs& a, const ViewBatch& vb, hipStream_t stream);

}  // namespace gsr

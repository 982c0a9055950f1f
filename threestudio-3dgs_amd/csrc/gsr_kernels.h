// gsr_kernels.h — host-side launchers for the device kernels (internal; the public ABI is
// include/gsr.h).  All launchers enqueue on `stream` and never synchronise.
#pragma once

#include "gsr_common.h"

namespace gsr {

// Stable LSD radix sort of n = min(*n_dev, n_max) (key, value) pairs on key bits [0, key_bits),
// digit_plan(key_bits) passes, one onesweep launch each (gsr_sort.hip).  Ping-pongs between
// keys[0]/vals[0] and keys[1]/vals[1]; returns the index (0/1) holding the result.  The digit
// counts of every pass must already be in sync.digit_count (the key producer builds them) and the
// rest of `sync` zeroed.  vals_identity: the input values are the input positions.
int onesweep_sort(uint32_t* keys[2], uint32_t* vals[2], bool vals_identity, const uint32_t* n_dev, int n_max,
                  int key_bits, const SortSync& sync, uint32_t* err, hipStream_t stream);

// Forward preprocess (cull, project, EWA, SH) — gsr_preprocess.hip
struct PreprocessArgs {
  int P, deg, M;
  const float *means3D, *scales, *rotations, *opacities, *shs, *colors_precomp, *cov3D_precomp;
  float scale_modifier;
  const float *viewmatrix, *projmatrix, *campos;
  int W, H;
  float tanfovx, tanfovy, focal_x, focal_y;
  int* radii;
};
void launch_preprocess(const PreprocessArgs& a, const GeomState& g, hipStream_t stream);

// Binning — gsr_binning.hip
void launch_compact_visible(int P, const GeomState& g, hipStream_t stream);
void launch_duplicate(int P, int W, int H, const uint32_t* order, const GeomState& g, const BinningState& b,
                      uint2* ranges, hipStream_t stream);
void launch_tile_ranges(int K, const uint32_t* keys, uint2* ranges, hipStream_t stream);
void launch_mark_visible(int P, const float* means3D, const float* view, const float* proj,
                         uint8_t* present, hipStream_t stream);

// Tile blend — gsr_render.hip
// `sorted_gauss` = the tile sort's value buffer holding the result (sorted position -> Gaussian).
void launch_render_forward(int W, int H, const GeomState& g, const uint32_t* sorted_gauss,
                           const ImageState& img, const float* bg, float* out_color,
                           float* out_depth, float* out_alpha, hipStream_t stream);
void launch_render_backward(int W, int H, int K, const GeomState& g, const uint32_t* sorted_gauss,
                            const ImageState& img, const float* bg, const float* dL_dcolor,
                            const float* dL_ddepth, const float* dL_dalpha,
                            const BackwardState& bw, hipStream_t stream);

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
ViewDesc make_view_desc(const float* view, const float* proj, const float* campos, const int* radii,
                        const GeomState& g, const ImageState& img, const BackwardState& bw,
                        float* dmeans2D, int W, int H, float tanx, float tany);
void launch_gauss_backward_views(const GaussBackwardArgs& a, const ViewBatch& vb, hipStream_t stream);

}  // namespace gsr

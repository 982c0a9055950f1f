/*
 * gsr.h — C ABI of the MI355X-native differentiable 3D Gaussian Splatting rasterizer.
 *
 * This is the drop-in boundary for the hot path of lizhiqi49/threestudio-3dgs.  The
 * reference never ships a rasterizer: every renderer (e.g. renderer/diff_gaussian_rasterizer.py:8-11,
 * renderer/diff_gaussian_rasterizer_background.py:119-128, renderer/diff_gaussian_rasterizer_advanced.py:122)
 * imports the external pybind module `diff_gaussian_rasterization._C` (ashawkey 4-output fork,
 * README.md:17,28).  Its three entry points are
 *     _C.rasterize_gaussians(...)          -> (num_rendered, color, depth, alpha, radii, geomBuf, binningBuf, imgBuf)
 *     _C.rasterize_gaussians_backward(...) -> 8 gradients
 *     _C.mark_visible(...)                 -> bool mask
 * (SURVEY.md §8b).  This header restates them as plain C: device pointers, sizes and a HIP stream
 * handle; no torch types.  The host binding (threestudio-3dgs_amd/diff_gaussian_rasterization/_C.py)
 * calls these through ctypes with buffers allocated by the PyTorch caching allocator.
 *
 * Conventions (unchanged from the reference call sites):
 *   - all float arrays are fp32, row-major, device-resident;
 *   - viewmatrix / projmatrix are 4x4 *transposed* (row-vector) matrices read column-major
 *     (world_view_transform / full_proj_transform, geometry/sugar.py:891-896);
 *   - shs is (P, M, 3); rotations are (w, x, y, z), used as given (not renormalised);
 *   - color output is planar (3, H, W); depth and alpha are (1, H, W);
 *   - radii is int32 (P,); means2D gradient is (P, 3) in pixel units (x W/2, H/2), z = 0.
 *
 * Work is split into the phases the reference performs inside one call so that the host can
 * size the K-dependent buffers between them (the reference does the same D2H read of K,
 * SURVEY.md §2a "cub::DeviceScan ... host sync"):
 *   1. gsr_forward_preprocess   — cull/project/EWA/SH, depth sort, instance offsets, K
 *   2. gsr_num_rendered         — read K (and the visible count) back to the host
 *   3. gsr_forward_render       — duplicate, tile sort, tile ranges, front-to-back blend
 *   4. gsr_backward             — back-to-front replay + fused per-Gaussian chain rule
 *
 * Every function returns GSR_OK (0) or an error code; gsr_last_error() gives the message for
 * the calling thread.  Kernels are enqueued on `stream` (a hipStream_t; NULL = legacy stream);
 * only gsr_num_rendered synchronises.
 */
#ifndef GSR_H
#define GSR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSR_OK 0
#define GSR_EINVAL 1 /* bad argument (shape / size / null pointer)          */
#define GSR_EHIP 2   /* a HIP runtime call failed                            */

#define GSR_TILE_X 16 /* BLOCK_X of the reference algorithm (16x16 tiles)      */
#define GSR_TILE_Y 16

/* Library identification ("gsr <version> gfx950"). */
const char* gsr_version(void);
/*
 * ABI revision of this header (GSR_ABI_VERSION), for callers binding the library at run time.
 *   2  gsr_set_backward* `accumulate` CONTINUES every per-Gaussian sum from the stored value in view order
 *      (round 1's revision 1 added the new sums to the stored values); with accumulate in the scale / rotation
 *      path dL_dcov3D is required (the running dL/dcov3D carry), otherwise GSR_EINVAL.
 *   3  gsr_shade_views_forward / gsr_shade_views_backward (per-view light colours and shading modes);
 *      gsr_set_backward_chunks / gsr_grad_chunk_range (per-Gaussian sums in ranges, events for overlap).
 *   4  gsr_set_image_bytes_ex (image buffers sized for the forward's split decision, which the buffer records);
 *      gsr_profile_kernel (the blend kernels the phases ran).
 *   5  gsr_sort_work_bytes / gsr_sort_pairs / gsr_sort_rank_mode (the library's sort, for tests);
 *      gsr_set_preprocess_ex (the two-colour render's second colours written into the records).
 */
#define GSR_ABI_VERSION 5
int gsr_abi_version(void);
/* Message of the last failing call on this thread ("" if none). */
const char* gsr_last_error(void);

/* ---- workspace sizing (bytes).  Buffers are opaque, 256-byte aligned uint8 regions. ---- */
/* Per-Gaussian state: replaces the reference's geomBuffer (rasterize_points.cu, [EXT]). */
size_t gsr_geom_bytes(int P);
/* Per-instance state for K (Gaussian, tile) pairs: replaces binningBuffer. */
size_t gsr_binning_bytes(int K, int width, int height);
/* Per-pixel state (final transmittance, last contributor, tile ranges): replaces imgBuffer. */
size_t gsr_image_bytes(int width, int height);
/* Scratch for gsr_backward (per-instance gradient rows). */
size_t gsr_backward_bytes(int P, int K);

/*
 * Phase 1 — replaces FORWARD::preprocessCUDA + InclusiveSum of rasterize_points.cu [EXT]
 * (SURVEY.md §2a rows 1-2, §8a A4-A8).  Exactly one of (shs, colors_precomp) and one of
 * ((scales, rotations), cov3D_precomp) must be non-NULL (checked; GSR_EINVAL otherwise).
 * Writes radii (P,) and the geom workspace; the visible count and K stay on the device.
 *   means3D (P,3)  scales (P,3)  rotations (P,4)  opacities (P,1)  shs (P,M,3)
 *   colors_precomp (P,3)  cov3D_precomp (P,6)  viewmatrix/projmatrix (16)  campos (3)
 * `degree` is the active SH degree; the kernel uses min(degree, sqrt(M)-1).
 */
int gsr_forward_preprocess(int P, int degree, int M,
                           const float* means3D, const float* scales, float scale_modifier,
                           const float* rotations, const float* opacities, const float* shs,
                           const float* colors_precomp, const float* cov3D_precomp,
                           const float* viewmatrix, const float* projmatrix, const float* campos,
                           int width, int height, float tanfovx, float tanfovy, int prefiltered,
                           int* radii, void* geom, void* stream);

/* Phase 2 — D2H read of K (num_rendered) and of the visible-Gaussian count; synchronises `stream`. */
int gsr_num_rendered(const void* geom, int P, int* num_rendered, int* num_visible, void* stream);

/*
 * Phase 3 — replaces duplicateWithKeys + DeviceRadixSort::SortPairs + identifyTileRanges +
 * FORWARD::renderCUDA [EXT].  K must be the value from gsr_num_rendered.
 * bg is (3,) on the device.  Writes color (3,H,W), depth (1,H,W), alpha (1,H,W) and the
 * binning / image workspaces that gsr_backward reads.
 */
int gsr_forward_render(int P, int K, int width, int height, const float* bg,
                       void* geom, void* binning, void* image,
                       float* out_color, float* out_depth, float* out_alpha, void* stream);

/*
 * Phase 4 — replaces BACKWARD::renderCUDA + computeCov2DCUDA + preprocessCUDA [EXT]
 * (SURVEY.md §8a A11-A12).  Reads (never writes) geom/binning/image, so it may be called
 * repeatedly on the same forward state (retain_graph=True, system/gaussian_splatting.py:129,138).
 * Gradient outputs are fully overwritten (no pre-zeroing needed):
 *   dL_dmeans2D (P,3)  dL_dcolors (P,3)  dL_dopacity (P,1)  dL_dmeans3D (P,3)
 *   dL_dcov3D (P,6) [may be NULL if cov3D_precomp is NULL]  dL_dsh (P,M,3) [NULL if shs NULL]
 *   dL_dscales (P,3), dL_drotations (P,4) [NULL if scales/rotations NULL]
 * dL_ddepth / dL_dalpha may be NULL (treated as zero).
 */
int gsr_backward(int P, int degree, int M, int K, int width, int height, const float* bg,
                 const float* means3D, const float* scales, float scale_modifier,
                 const float* rotations, const float* opacities, const float* shs,
                 const float* colors_precomp, const float* cov3D_precomp,
                 const float* viewmatrix, const float* projmatrix, const float* campos,
                 float tanfovx, float tanfovy, const int* radii,
                 const void* geom, const void* binning, const void* image,
                 const float* dL_dcolor, const float* dL_ddepth, const float* dL_dalpha,
                 float* dL_dmeans2D, float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D,
                 float* dL_dcov3D, float* dL_dsh, float* dL_dscales, float* dL_drotations,
                 void* work, void* stream);

/*
 * View sets: one set of P Gaussians rendered from V <= GSR_SET_MAX cameras
 * of the same image size by the SAME launches (every stage runs once per set, not once per view;
 * sorts are segmented by view).  The per-view functions above are sets of one.  The reference
 * renders a batch with a Python loop over views (renderer/gaussian_batch_renderer.py:9-122), one
 * rasterizer call each; these replace that loop's V forward and V backward calls.
 * Per-view arguments are HOST arrays of V values or of V device pointers; images are stacked:
 * color (V,3,H,W), depth / alpha (V,1,H,W), radii (V,P) int32, dL_dmeans2D (V,P,3).
 * Shared-parameter gradients (means3D, opacity, SH, scales, rotations, cov3D, colors) are summed
 * over the V views inside the per-Gaussian kernel.
 */
#define GSR_SET_MAX 64
size_t gsr_set_geom_bytes(int V, int P);
size_t gsr_set_binning_bytes(int V, int P, const int* num_rendered, int width, int height);
size_t gsr_set_image_bytes(int V, int width, int height);
/* The image bytes of exactly this forward (gsr_set_image_bytes is the upper bound): the split backward's
 * checkpoints only when the forward writes them (a launch of <= 4096 tiles on the quadrant waves, one colour
 * set: 335 MB for one 1024^2 view, held until the backward).  two_colors != 0: gsr_set_render_two_colors.
 * The forward records its decision in the buffer; the backward follows it whatever the environment says then. */
size_t gsr_set_image_bytes_ex(int V, int P, const int* num_rendered, int width, int height, int two_colors);
/* Scratch holding the gradient rows and per-(view, Gaussian) records of all V views; gsr_set_backward
 * also accepts less (>= what the largest single view needs) and then walks the views in groups that fit. */
size_t gsr_set_backward_bytes(int V, int P, const int* num_rendered);
int gsr_set_preprocess(int V, int P, int degree, int M, const float* means3D, const float* scales,
                       float scale_modifier, const float* rotations, const float* opacities, const float* shs,
                       const float* colors_precomp, const float* cov3D_precomp,
                       const float* const* viewmatrices, const float* const* projmatrices,
                       const float* const* campos, const float* tanfovx, const float* tanfovy,
                       int width, int height, int prefiltered, int* radii, void* geom, void* stream);
/* As gsr_set_preprocess, for a set that gsr_set_render_two_colors will blend with colors2 (P, 3) as the second
 * colour set (the SuGaR renderers' second rasterizer call): the preprocess writes each Gaussian's second colour
 * into the per-(view, Gaussian) record it writes anyway (no extra traffic), so the two-colour blends read it with
 * the record instead of gathering it from colors2 apart.  A two-colour call given another colors2 array reads
 * that array (the set remembers which pointer it embedded).  colors2 NULL = gsr_set_preprocess. */
int gsr_set_preprocess_ex(int V, int P, int degree, int M, const float* means3D, const float* scales,
                          float scale_modifier, const float* rotations, const float* opacities, const float* shs,
                          const float* colors_precomp, const float* cov3D_precomp,
                          const float* const* viewmatrices, const float* const* projmatrices,
                          const float* const* campos, const float* tanfovx, const float* tanfovy,
                          int width, int height, int prefiltered, int* radii, void* geom, const float* colors2,
                          void* stream);
/* One D2H read of every view's K (and visible count, may be NULL); synchronises `stream`.
 * K = the reference's num_rendered (tiles of every visible Gaussian's 3-sigma rectangle): the
 * capacity the binning and backward scratch are sized by. */
int gsr_set_num_rendered(int V, const void* geom, int P, int* num_rendered, int* num_visible, void* stream);
/* As gsr_set_num_rendered, plus num_listed[v] (may be NULL): the instances the tile lists actually
 * hold after the exact ellipse-vs-tile culling (<= K).  Diagnostic / roofline use. */
int gsr_set_num_rendered_ex(int V, const void* geom, int P, int* num_rendered, int* num_visible, int* num_listed,
                            void* stream);
/* Diagnostic copy (device to device, on `stream`) of the preprocess state of every (view, Gaussian):
 * out_rec (V, P, 16) 32-bit words = (pixel x, pixel y, conic a, conic b | conic c, opacity, view depth, 0 |
 * r, g, b, 0 | tile rect xmin | ymin << 16, xmax | ymax << 16, 0, SH clamp flags), written only for
 * visible Gaussians; out_tiles (V, P, 2) u32 = (3-sigma rectangle tiles, 0 = culled; tiles the
 * alpha >= 1/255 ellipse reaches).  Either may be NULL.  Parity tests compare these with the oracle's
 * per-Gaussian preprocess values (the reference's geomBuffer has no public layout). */
int gsr_set_gauss_state(int V, const void* geom, int P, void* out_rec, void* out_tiles, void* stream);
/* The binning buffer belongs to this one forward until its last backward: besides the sorted tile lists the
 * forward may keep per listed instance a quadrant-mask byte in the buffer's second (free) key array, which the
 * backward's cull reads (csrc/gsr_common.h BinningState); the caller must not reuse the buffer in between. */
int gsr_set_render(int V, int P, const int* num_rendered, int width, int height, const float* const* bgs,
                   void* geom, void* binning, void* image, float* out_color, float* out_depth,
                   float* out_alpha, void* stream);
/* Gradient outputs are overwritten (accumulate = 0) or continued (accumulate != 0: every per-Gaussian
 * sum resumes from the stored value in view order), summed over the set's views; dL_dmeans2D is per view
 * and always overwritten.  The views are processed in groups that fit work_bytes
 * (gsr_set_backward_bytes = all in one group); any grouping gives bitwise the same gradients.  With
 * accumulate in the scale / rotation path, dL_dcov3D is required: it carries the running dL/dcov3D
 * that the scale and rotation gradients are recomputed from.  Reads forward state only. */
int gsr_set_backward(int V, int P, int degree, int M, const int* num_rendered, int width, int height,
                     const float* const* bgs, const float* means3D, const float* scales, float scale_modifier,
                     const float* rotations, const float* shs, const float* cov3D_precomp,
                     const float* const* viewmatrices, const float* const* projmatrices,
                     const float* const* campos, const float* tanfovx, const float* tanfovy, const int* radii,
                     const void* geom, const void* binning, const void* image, const float* dL_dcolor,
                     const float* dL_ddepth, const float* dL_dalpha, float* dL_dmeans2D, float* dL_dcolors,
                     float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh,
                     float* dL_dscales, float* dL_drotations, int accumulate, void* work, size_t work_bytes,
                     void* stream);
/*
 * Overlap of the per-Gaussian sums with their reduction across ranks.  A backward's final
 * per-Gaussian gradients are formed in one pass after the backward blend; gsr_set_backward_chunks asks the
 * NEXT gsr_set_backward* call made on this thread to form them in n_chunks Gaussian ranges instead, recording
 * events[c] (hipEvent_t, may be NULL) on the stream after range c, so that the caller can start reducing range
 * c (e.g. an RCCL all-reduce on another stream waiting on the event) while the later ranges are computed.
 * Range c = [c S, min(P, (c + 1) S)) with S = GSR_GRAD_CHUNK_ALIGN x ceil(ceil(P / n_chunks) / ALIGN)
 * (gsr_grad_chunk_range); ranges may be empty.  Results are bitwise those of the unchunked call.  The request
 * applies to one call only (n_chunks = 0 cancels it).
 */
#define GSR_GRAD_CHUNKS_MAX 16
#define GSR_GRAD_CHUNK_ALIGN 4096
int gsr_set_backward_chunks(int n_chunks, void* const* events);
int gsr_grad_chunk_range(int P, int n_chunks, int chunk, int* g0, int* g1);

/*
 * Two rasterizer calls that differ only in their colours, sharing one geometry (the SuGaR normal renderer,
 * renderer/diff_sugar_rasterizer_normal.py:157-191: the same Gaussians, camera and settings rendered with
 * the SH / override colours, then with colors_precomp = the face normals and a zero means2D).  The second
 * call's preprocess, sorts and binning are the first's; its blend weights too, so the forward blends both
 * colour sets in one pass:
 *   gsr_set_render_two_colors  as gsr_set_render (bg_images / out_render: the fused composite, both NULL
 *                              for none; out_render alone: the clamp alone, as gsr_set_render_composite)
 *                              plus out_color2 (V, 3, H, W) = the blend of colors2 (P, 3) with
 *                              the same weights and background: the second call's colour output (its
 *                              radii / depth / alpha equal the first call's).
 *   gsr_set_backward_colors    the second call's backward on the shared forward state: colours = colors2,
 *                              dL_dcolor = dL/d(out_color2), no depth / alpha gradient, no SH; dL_dmeans2D
 *                              receives the second call's screen-space gradient (the reference discards it:
 *                              pass scratch), dL_dcolors the gradient of colors2.  With accumulate the
 *                              parameter gradients continue the first call's (gsr_set_backward with
 *                              dL_dcov3D as the running dL/dcov3D carry).
 *   gsr_set_backward_two_colors  both calls' backward in one pass (replaces gsr_set_backward[_composite]
 *                              followed by gsr_set_backward_colors): the blend is replayed once, forming
 *                              both calls' dL/dalpha; arguments as gsr_set_backward_composite (bg_images
 *                              and color both NULL: no composite; color alone: the clamp alone) plus colors2,
 *                              dL_dcolor2 = dL/d(out_color2)
 *                              and dL_dcolors2 (P, 3) = the gradient of colors2.  dL_dmeans2D receives the
 *                              first call's screen-space gradient only (the second call's means2D is the
 *                              reference's fresh zero tensor); the parameter gradients hold both calls'
 *                              (equal to the two-call sequence up to fp32 summation order).  Scratch:
 *                              gsr_set_backward_two_colors_bytes (64-byte gradient rows).
 */
int gsr_set_render_two_colors(int V, int P, const int* num_rendered, int width, int height, const float* const* bgs,
                              void* geom, void* binning, void* image, float* out_color, float* out_depth,
                              float* out_alpha, const float* bg_images, float* out_render, const float* colors2,
                              float* out_color2, void* stream);
int gsr_set_backward_colors(int V, int P, const int* num_rendered, int width, int height, const float* const* bgs,
                            const float* means3D, const float* scales, float scale_modifier, const float* rotations,
                            const float* cov3D_precomp, const float* const* viewmatrices,
                            const float* const* projmatrices, const float* const* campos, const float* tanfovx,
                            const float* tanfovy, const int* radii, const void* geom, const void* binning,
                            const void* image, const float* colors, const float* dL_dcolor, float* dL_dmeans2D,
                            float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D,
                            float* dL_dscales, float* dL_drotations, int accumulate, void* work, size_t work_bytes,
                            void* stream);
size_t gsr_set_backward_two_colors_bytes(int V, int P, const int* num_rendered);
int gsr_set_backward_two_colors(int V, int P, int degree, int M, const int* num_rendered, int width, int height,
                                const float* const* bgs, const float* means3D, const float* scales,
                                float scale_modifier, const float* rotations, const float* shs,
                                const float* cov3D_precomp, const float* const* viewmatrices,
                                const float* const* projmatrices, const float* const* campos, const float* tanfovx,
                                const float* tanfovy, const int* radii, const void* geom, const void* binning,
                                const void* image, const float* bg_images, const float* color,
                                const float* dL_dcolor, const float* dL_ddepth, const float* dL_dalpha,
                                float* dL_dbg, const float* colors2, const float* dL_dcolor2, float* dL_dmeans2D,
                                float* dL_dcolors, float* dL_dcolors2, float* dL_dopacity, float* dL_dmeans3D,
                                float* dL_dcov3D, float* dL_dsh, float* dL_dscales, float* dL_drotations,
                                int accumulate, void* work, size_t work_bytes, void* stream);
/*
 * The background renderer's composite fused into the blends (replaces gsr_set_render + gsr_composite_forward
 * and gsr_composite_backward + gsr_set_backward for renderer/diff_gaussian_rasterizer_background.py:129-132,139):
 * bg_images (V, H, W, 3) are the background network's outputs; out_render (V, 3, H, W) =
 * clamp(color + (1 - alpha) bg, 0, 1), bit-identical to the torch expression on the stored outputs; the
 * colour / depth / alpha outputs are written as by gsr_set_render.  The backward takes dL/drender in
 * place of dL/dcolor, the forward's colour output, and forms dL/dbg (NULL: not formed) in the blend's
 * per-pixel prologue (clamp mask, dL/dalpha += -sum_c g_c bg_c, dL/dbg = g (1 - alpha)).
 * bg_images NULL: the clamp alone — out_render = clamp(color, 0, 1), the renderers' `rendered_image.clamp(0, 1)`
 * (renderer/diff_gaussian_rasterizer.py:141, renderer/diff_sugar_rasterizer_normal.py:212) bit-identical to the
 * torch expression; the backward masks dL/drender by the forward's colour (dL_dbg must be NULL).
 */
int gsr_set_render_composite(int V, int P, const int* num_rendered, int width, int height, const float* const* bgs,
                             void* geom, void* binning, void* image, float* out_color, float* out_depth,
                             float* out_alpha, const float* bg_images, float* out_render, void* stream);
int gsr_set_backward_composite(int V, int P, int degree, int M, const int* num_rendered, int width, int height,
                               const float* const* bgs, const float* means3D, const float* scales,
                               float scale_modifier, const float* rotations, const float* shs,
                               const float* cov3D_precomp, const float* const* viewmatrices,
                               const float* const* projmatrices, const float* const* campos, const float* tanfovx,
                               const float* tanfovy, const int* radii, const void* geom, const void* binning,
                               const void* image, const float* bg_images, const float* color,
                               const float* dL_drender, const float* dL_ddepth, const float* dL_dalpha,
                               float* dL_dbg, float* dL_dmeans2D, float* dL_dcolors, float* dL_dopacity,
                               float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscales,
                               float* dL_drotations, int accumulate, void* work, size_t work_bytes, void* stream);

/*
 * Optional phase timing with HIP events recorded on the launch stream around each phase's kernels.
 * Off by default; while on, every call above records one event pair per phase it runs.
 * gsr_profile_read synchronises the recorded events and returns, per phase, the accumulated
 * milliseconds and the number of timed launches since the last reset (arrays of GSR_NUM_PHASES).
 */
#define GSR_PHASE_PREPROCESS 0 /* k_preprocess                                              */
#define GSR_PHASE_DEPTH_SORT 1 /* per-view depth radix sort, instance counts and offsets     */
#define GSR_PHASE_BINNING 2    /* instance emission, tile radix sort, tile ranges           */
#define GSR_PHASE_RENDER_FWD 3 /* k_render_fwd: forward tile blend                          */
#define GSR_PHASE_RENDER_BWD 4 /* k_render_bwd: backward tile blend                         */
#define GSR_PHASE_GAUSS_BWD 5  /* k_gauss_bwd: fused per-Gaussian backward                   */
#define GSR_NUM_PHASES 6
int gsr_profile_enable(int enable);
int gsr_profile_read(double* ms, long long* launches, int reset);
/* The blend kernel the last GSR_PHASE_RENDER_FWD / GSR_PHASE_RENDER_BWD launch of this process used, as
 * rocprofv3 names it (e.g. "k_render_bwd<false, false>"); "" for other phases or before any launch.  Lets a
 * caller attribute committed PMC counters to the kernel actually timed. */
const char* gsr_profile_kernel(int phase);

/*
 * Fused background composite of the background renderer (replaces the torch epilogue of
 * renderer/diff_gaussian_rasterizer_background.py:129-132,139):
 *     out = clamp(color + (1 - alpha) * bg, 0, 1)       color, out (V, 3, H, W); alpha (V, 1, H, W)
 * bg_layout: GSR_BG_CONSTANT (V, 3), GSR_BG_HWC (V, H, W, 3) -- the background network's output --,
 * GSR_BG_CHW (V, 3, H, W).  Backward (pre-clamp value recomputed; clamp's inclusive-bounds gradient):
 * dL_dcolor = g, dL_dalpha = -sum_c g_c bg_c, dL_dbg = g (1 - alpha) (NULL: not computed; image
 * layouts only), with g = dL_dout where 0 <= pre <= 1, else 0.  Bit-identical to the torch expression
 * in the forward.
 */
#define GSR_BG_CONSTANT 0
#define GSR_BG_HWC 1
#define GSR_BG_CHW 2
int gsr_composite_forward(int V, int height, int width, const float* color, const float* alpha, const float* bg,
                          int bg_layout, float* out, void* stream);
int gsr_composite_backward(int V, int height, int width, const float* dL_dout, const float* color,
                           const float* alpha, const float* bg, int bg_layout, float* dL_dcolor, float* dL_dalpha,
                           float* dL_dbg, void* stream);

/*
 * SuGaR normal map (replaces the torch lines of renderer/diff_sugar_rasterizer_normal.py:192-197 after the
 * second rasterizer call): normal (V, 3, H, W) = the blended face normals, alpha (V, 1, H, W);
 *   out = (-u_x, -u_y, u_z) * 0.5 * alpha + 0.5 with u = normal / max(|normal|, 1e-12) (torch's order).
 * Backward: the gradient flows only where alpha > 0.99 (the rest is detached in the reference);
 * dL_dnormal (V, 3, H, W) and dL_dalpha (V, 1, H, W) are written whole (zeros where masked).
 */
int gsr_normal_map_forward(int V, int height, int width, const float* normal, const float* alpha, float* out,
                           void* stream);
int gsr_normal_map_backward(int V, int height, int width, const float* dL_dout, const float* normal,
                            const float* alpha, float* dL_dnormal, float* dL_dalpha, void* stream);

/*
 * Fused shading / depth-normal epilogue of the MVDream shading renderer and the SuGaR normal renderer
 * (replaces the torch ops of renderer/diff_gaussian_rasterizer_shading.py:169-208 with Depth2Normal
 * :22-51 and material/gaussian_material.py:41-104; renderer/diff_sugar_rasterizer_normal.py:170-197).
 * Per pixel of V views (planes (V, 3|1, H, W); rays (V, H, W, 3); light (V, 3)):
 *     X = rays_o + depth rays_d;  u = normalize(-(dX/dx x dX/dy)), central differences, X zero-padded;
 *     unit_normal = u;  normal_map = u 0.5 alpha + 0.5;  depth_out = depth
 * and with GSR_SHADE_MATERIAL the point-light material and background composite:
 *     s = u (or normalize(2 pred_normal - 1) when pred_normal != NULL, detached);
 *     t = max(s . normalize(light - X), 0) kd + ka;  albedo = color / (alpha + 1e-6);
 *     fg = clamp(albedo, 0, 1) t | albedo | t   (mode GSR_SHADING_DIFFUSE | _ALBEDO | _TEXTURELESS);
 *     render = clamp(fg alpha + (1 - alpha) bg, 0, 1),  bg GSR_BG_CONSTANT (V, 3) or GSR_BG_HWC.
 * ambient / diffuse: host arrays of 3 floats (ka, kd; ignored without the material flag).
 * Outputs may be NULL (not written) except render with the material flag.  Backward: gradients of
 * render / normal_map / unit_normal / depth_out (any may be NULL = zero); the normal-map, unit-normal
 * and depth_out gradients are kept only where alpha > 0.99 (the reference's in-place detach of the
 * other pixels).  Outputs dL_ddepth, dL_dalpha (required), dL_dcolor (material), dL_dbg (NULL = not
 * formed; GSR_BG_HWC only).
 */
#define GSR_SHADE_MATERIAL 1
#define GSR_SHADING_DIFFUSE 0
#define GSR_SHADING_ALBEDO 1
#define GSR_SHADING_TEXTURELESS 2
int gsr_shade_forward(int V, int height, int width, int flags, int mode, const float* color, const float* depth,
                      const float* alpha, const float* rays_o, const float* rays_d, const float* bg, int bg_layout,
                      const float* light, const float* pred_normal, const float* ambient, const float* diffuse,
                      float* render, float* normal_map, float* unit_normal, float* depth_out, void* stream);
int gsr_shade_backward(int V, int height, int width, int flags, int mode, const float* color, const float* depth,
                       const float* alpha, const float* rays_o, const float* rays_d, const float* bg, int bg_layout,
                       const float* light, const float* pred_normal, const float* ambient, const float* diffuse,
                       const float* dL_drender, const float* dL_dnormal_map, const float* dL_dunit_normal,
                       const float* dL_ddepth_out, float* dL_dcolor, float* dL_ddepth, float* dL_dalpha,
                       float* dL_dbg, void* stream);
/*
 * As gsr_shade_forward / gsr_shade_backward with the light colours and shading mode given PER VIEW:
 * modes (V,) host ints, ambient / diffuse (V, 3) host floats.  The reference's material draws its soft-shading
 * ambient ratio and its shading mode once per view (material/gaussian_material.py:59-64,80-88, called once per
 * view by renderer/diff_gaussian_rasterizer_shading.py:200-205 inside the per-view loop of
 * renderer/gaussian_batch_renderer.py:21-54), so a fused batch needs one (ka, kd, mode) per view.
 * modes / ambient / diffuse may be NULL without GSR_SHADE_MATERIAL.
 */
int gsr_shade_views_forward(int V, int height, int width, int flags, const int* modes, const float* color,
                            const float* depth, const float* alpha, const float* rays_o, const float* rays_d,
                            const float* bg, int bg_layout, const float* light, const float* pred_normal,
                            const float* ambient, const float* diffuse, float* render, float* normal_map,
                            float* unit_normal, float* depth_out, void* stream);
int gsr_shade_views_backward(int V, int height, int width, int flags, const int* modes, const float* color,
                             const float* depth, const float* alpha, const float* rays_o, const float* rays_d,
                             const float* bg, int bg_layout, const float* light, const float* pred_normal,
                             const float* ambient, const float* diffuse, const float* dL_drender,
                             const float* dL_dnormal_map, const float* dL_dunit_normal, const float* dL_ddepth_out,
                             float* dL_dcolor, float* dL_ddepth, float* dL_dalpha, float* dL_dbg, void* stream);

/*
 * Mean squared distance to the 3 nearest other points, for each of P points (P, 3) -> (P,): replaces
 * simple_knn._C.distCUDA2 (called at geometry/gaussian_base.py:434-437 to initialise scales; also imported by
 * geometry/sugar.py:18, geometry/gaussian_io.py:25, geometry/spacetime_gaussian.py:15,430,
 * geometry/dynamic_sugar.py:17, geometry/gaussian_dynamic.py:25).  Exact search; per-pair fp32 distance
 * fma(dz, dz, fma(dy, dy, dx * dx)); result (b0 + b1 + b2) / 3 over the sorted 3 best (FLT_MAX entries
 * kept when P < 4).  workspace: gsr_knn_workspace_bytes(P) bytes of device memory (256-B aligned).
 */
size_t gsr_knn_workspace_bytes(int P);
int gsr_knn_mean_dist(int P, const float* points, float* mean_dist, void* workspace, size_t workspace_bytes,
                      void* stream);

/*
 * The view-segmented stable LSD radix sort that every sort of this library runs (the depth sort, the tile sort and
 * distCUDA2's Morton sort: csrc/gsr_sort.hip; it replaces the reference extension's cub::DeviceRadixSort::SortPairs
 * calls of one view at a time).  Exposed for tests: V (1..64) segments of n[v] (key, value) pairs laid
 * out back to back in keys / vals (device), each sorted in place by the key's low key_bits (1..32) bits, stably
 * (equal keys keep their order), in passes of at most max_bits (1..8) bits.  vals may be NULL (keys only).
 * work: gsr_sort_work_bytes(V, n) bytes of device memory.
 */
size_t gsr_sort_work_bytes(int V, const int* n);
int gsr_sort_pairs(int V, const int* n, uint32_t* keys, uint32_t* vals, int key_bits, int max_bits, void* work,
                   size_t work_bytes, void* stream);
/* How the sort's scatter ranks equal digits within a wave, decided once per process: 1 = LDS atomic adds (the device
 * was found, by a probe kernel at the first call, to service one instruction's lanes that hit the same counter in lane
 * order, which keeps the sort stable), 0 = ballot matching (the probe failed, or GSR_SORT_RANK=ballot).  Both give
 * the same bits.  Runs the probe if it has not run yet (a device synchronisation). */
int gsr_sort_rank_mode(void);

/* Replaces markVisible/checkFrustum (API completeness; unused by the reference).  present (P,) u8. */
int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     uint8_t* present, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GSR_H */

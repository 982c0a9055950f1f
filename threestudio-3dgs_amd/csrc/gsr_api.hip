// gsr_api.hip — extern "C" entry points declared in include/gsr.h.
//
// Phase structure mirrors what the reference's _C.rasterize_gaussians does internally
// (CudaRasterizer::Rasterizer::forward / backward [EXT]); argument checking mirrors its
// TORCH_CHECKs and Python-side exceptions (SURVEY.md §8b "Errors").
#include <stdio.h>
#include <string.h>

#include <cmath>
#include <mutex>
#include <vector>

#include "../../include/gsr.h"
#include "gsr_kernels.h"

using namespace gsr;

static thread_local char g_err[512] = "";

static int fail(int code, const char* fmt, const char* what) {
  snprintf(g_err, sizeof(g_err), fmt, what);
  return code;
}

#define GSR_HIP_CHECK(expr)                                                        \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) return fail(GSR_EHIP, "HIP error: %s", hipGetErrorString(e_)); \
  } while (0)

static int last_launch() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(GSR_EHIP, "HIP launch error: %s", hipGetErrorString(e));
  g_err[0] = 0;
  return GSR_OK;
}

// ---- phase profiler: event pairs on the launch stream, resolved lazily in gsr_profile_read ----
namespace {
struct PhaseEvents {
  int phase;
  hipEvent_t a, b;
};
struct Profiler {
  std::mutex mu;
  bool on = false;
  std::vector<hipEvent_t> pool;
  std::vector<PhaseEvents> pending;
  double ms[GSR_NUM_PHASES] = {0};
  long long n[GSR_NUM_PHASES] = {0};
  hipEvent_t get() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
  }
};
Profiler& prof() {
  static Profiler p;
  return p;
}
// RAII scope: records a start event at construction and an end event at destruction.
struct PhaseScope {
  hipEvent_t a = nullptr, b = nullptr;
  hipStream_t s;
  int phase;
  PhaseScope(int ph, hipStream_t st) : s(st), phase(ph) {
    Profiler& p = prof();
    if (!p.on) return;
    std::lock_guard<std::mutex> g(p.mu);
    a = p.get();
    b = p.get();
    if (a) (void)hipEventRecord(a, s);
  }
  ~PhaseScope() {
    if (a == nullptr || b == nullptr) return;
    (void)hipEventRecord(b, s);
    Profiler& p = prof();
    std::lock_guard<std::mutex> g(p.mu);
    p.pending.push_back({phase, a, b});
  }
};
}  // namespace

static int effective_degree(int degree, int M) {
  // the reference reads sqrt(M)-1 coefficients at most (pred-normal pass quirk)
  int dm = (int)std::lround(std::sqrt((double)(M > 0 ? M : 1))) - 1;
  int d = degree < dm ? degree : dm;
  if (d < 0) d = 0;
  if (d > 3) d = 3;
  return d;
}

// ping-pong buffer holding the tile sort's result (one radix pass per <= 8 key bits)
static int tile_sort_result(int W, int H) { return digit_plan(tile_key_bits(W, H)).passes & 1; }

static GaussBackwardArgs shared_args(int P, int degree, int M, const float* means3D, const float* scales,
                                     float scale_modifier, const float* rotations, const float* shs,
                                     const float* cov3D_precomp, float* dL_dcolors, float* dL_dopacity,
                                     float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscales,
                                     float* dL_drotations) {
  GaussBackwardArgs a;
  a.P = P;
  a.deg = effective_degree(degree, M);
  a.M = shs ? M : 0;
  a.means3D = means3D;
  a.scales = scales;
  a.rotations = rotations;
  a.shs = shs;
  a.cov3D_precomp = cov3D_precomp;
  a.scale_modifier = scale_modifier;
  a.dL_dcolors = dL_dcolors;
  a.dL_dopacity = dL_dopacity;
  a.dL_dmeans3D = dL_dmeans3D;
  a.dL_dcov3D = dL_dcov3D;
  a.dL_dsh = shs ? dL_dsh : nullptr;
  a.dL_dscales = cov3D_precomp ? nullptr : dL_dscales;
  a.dL_drotations = cov3D_precomp ? nullptr : dL_drotations;
  return a;
}

extern "C" {

const char* gsr_version(void) { return "gsr 0.1.0 gfx950"; }
const char* gsr_last_error(void) { return g_err; }

size_t gsr_geom_bytes(int P) {
  size_t b = 0;
  GeomState::carve(nullptr, P, &b);
  return b;
}
size_t gsr_binning_bytes(int K, int width, int height) {
  (void)width;
  (void)height;
  size_t b = 0;
  BinningState::carve(nullptr, K, &b);
  return b;
}
size_t gsr_image_bytes(int width, int height) {
  size_t b = 0;
  ImageState::carve(nullptr, width, height, &b);
  return b;
}
size_t gsr_backward_bytes(int P, int K) {
  (void)P;
  size_t b = 0;
  BackwardState::carve(nullptr, K, &b);
  return b;
}

int gsr_forward_preprocess(int P, int degree, int M, const float* means3D, const float* scales,
                           float scale_modifier, const float* rotations, const float* opacities,
                           const float* shs, const float* colors_precomp, const float* cov3D_precomp,
                           const float* viewmatrix, const float* projmatrix, const float* campos,
                           int width, int height, float tanfovx, float tanfovy, int prefiltered,
                           int* radii, void* geom, void* stream) {
  (void)prefiltered;
  if (P < 0) return fail(GSR_EINVAL, "%s", "P must be >= 0");
  if (width <= 0 || height <= 0) return fail(GSR_EINVAL, "%s", "image size must be positive");
  if ((shs == nullptr) == (colors_precomp == nullptr))
    return fail(GSR_EINVAL, "%s", "Please provide exactly one of either SHs or precomputed colors!");
  if (((scales == nullptr || rotations == nullptr) && cov3D_precomp == nullptr) ||
      ((scales != nullptr || rotations != nullptr) && cov3D_precomp != nullptr))
    return fail(GSR_EINVAL, "%s",
                "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
  if (geom == nullptr || viewmatrix == nullptr || projmatrix == nullptr || campos == nullptr ||
      (P > 0 && (means3D == nullptr || opacities == nullptr || radii == nullptr)))
    return fail(GSR_EINVAL, "%s", "null pointer argument");
  if (shs != nullptr && M <= 0) return fail(GSR_EINVAL, "%s", "M must be >= 1 with SHs");
  hipStream_t s = (hipStream_t)stream;
  GeomState g = GeomState::carve(geom, P, nullptr);
  const DigitPlan dplan = digit_plan(32);
  GSR_HIP_CHECK(hipMemsetAsync(g.sync, 0, g.dsort.used_bytes(g.sync, dplan.passes, dplan.bits, P), s));
  if (P == 0) return last_launch();

  PreprocessArgs a;
  a.P = P;
  a.deg = effective_degree(degree, M);
  a.M = M;
  a.means3D = means3D;
  a.scales = scales;
  a.rotations = rotations;
  a.opacities = opacities;
  a.shs = shs;
  a.colors_precomp = colors_precomp;
  a.cov3D_precomp = cov3D_precomp;
  a.scale_modifier = scale_modifier;
  a.viewmatrix = viewmatrix;
  a.projmatrix = projmatrix;
  a.campos = campos;
  a.W = width;
  a.H = height;
  a.tanfovx = tanfovx;
  a.tanfovy = tanfovy;
  a.focal_y = height / (2.0f * tanfovy);
  a.focal_x = width / (2.0f * tanfovx);
  a.radii = radii;
  {
    PhaseScope ps(GSR_PHASE_PREPROCESS, s);
    launch_preprocess(a, g, s);
  }
  {
    // visible compaction (+ depth digit counts, K) -> depth sort of the visible Gaussians
    PhaseScope ps(GSR_PHASE_DEPTH_SORT, s);
    launch_compact_visible(P, g, s);
    const int res = onesweep_sort(g.dkey, g.dval, false, g.counters + GSR_CTR_VISIBLE, P, 32, g.dsort,
                                  g.counters + GSR_CTR_ERR, s);
    if (res != 0) return fail(GSR_EHIP, "%s", "internal: depth sort result buffer");
  }
  return last_launch();
}

int gsr_num_rendered(const void* geom, int P, int* num_rendered, int* num_visible, void* stream) {
  if (geom == nullptr || num_rendered == nullptr) return fail(GSR_EINVAL, "%s", "null pointer argument");
  GeomState g = GeomState::carve((void*)geom, P, nullptr);
  uint32_t h[4] = {0, 0, 0, 0};
  hipStream_t s = (hipStream_t)stream;
  if (P > 0) {
    GSR_HIP_CHECK(hipMemcpyAsync(h, g.counters, sizeof(h), hipMemcpyDeviceToHost, s));
    GSR_HIP_CHECK(hipStreamSynchronize(s));
  }
  if (h[GSR_CTR_ERR]) return fail(GSR_EHIP, "%s", "internal: look-back timeout in compaction / depth sort");
  *num_rendered = (int)h[GSR_CTR_K];
  if (num_visible) *num_visible = (int)h[0];
  g_err[0] = 0;
  return GSR_OK;
}

int gsr_forward_render(int P, int K, int width, int height, const float* bg, void* geom,
                       void* binning, void* image, float* out_color, float* out_depth,
                       float* out_alpha, void* stream) {
  if (P < 0 || K < 0 || width <= 0 || height <= 0) return fail(GSR_EINVAL, "%s", "bad sizes");
  if (geom == nullptr || binning == nullptr || image == nullptr || bg == nullptr ||
      out_color == nullptr || out_depth == nullptr || out_alpha == nullptr)
    return fail(GSR_EINVAL, "%s", "null pointer argument");
  hipStream_t s = (hipStream_t)stream;
  GeomState g = GeomState::carve(geom, P, nullptr);
  BinningState b = BinningState::carve(binning, K, nullptr);
  ImageState img = ImageState::carve(image, width, height, nullptr);
  const int gx = div_up(width, GSR_TILE_X), gy = div_up(height, GSR_TILE_Y);
  if (K > 0) {
    PhaseScope ps(GSR_PHASE_BINNING, s);
    const int kbits = tile_key_bits(width, height);
    const DigitPlan tplan = digit_plan(kbits);
    GSR_HIP_CHECK(hipMemsetAsync(b.sync, 0, b.tsort.used_bytes(b.sync, tplan.passes, tplan.bits, K), s));
    launch_duplicate(P, width, height, g.dval[0], g, b, img.ranges, s);
    const int res = onesweep_sort(b.key, b.val, false, nullptr, K, kbits, b.tsort, g.counters + GSR_CTR_ERR, s);
    if (res != tile_sort_result(width, height)) return fail(GSR_EHIP, "%s", "internal: tile sort buffer");
    launch_tile_ranges(K, b.key[res], img.ranges, s);
  } else {
    GSR_HIP_CHECK(hipMemsetAsync(img.ranges, 0, sizeof(uint2) * (size_t)gx * gy, s));
  }
  {
    PhaseScope ps(GSR_PHASE_RENDER_FWD, s);
    launch_render_forward(width, height, g, b.val[tile_sort_result(width, height)], img, bg, out_color,
                          out_depth, out_alpha, s);
  }
  return last_launch();
}

int gsr_backward(int P, int degree, int M, int K, int width, int height, const float* bg,
                 const float* means3D, const float* scales, float scale_modifier,
                 const float* rotations, const float* opacities, const float* shs,
                 const float* colors_precomp, const float* cov3D_precomp, const float* viewmatrix,
                 const float* projmatrix, const float* campos, float tanfovx, float tanfovy,
                 const int* radii, const void* geom, const void* binning, const void* image,
                 const float* dL_dcolor, const float* dL_ddepth, const float* dL_dalpha,
                 float* dL_dmeans2D, float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D,
                 float* dL_dcov3D, float* dL_dsh, float* dL_dscales, float* dL_drotations,
                 void* work, void* stream) {
  (void)opacities;
  (void)colors_precomp;
  if (P < 0 || K < 0 || width <= 0 || height <= 0) return fail(GSR_EINVAL, "%s", "bad sizes");
  if (P == 0) return last_launch();
  if (geom == nullptr || binning == nullptr || image == nullptr || work == nullptr || bg == nullptr ||
      dL_dcolor == nullptr || dL_dmeans2D == nullptr || dL_dcolors == nullptr ||
      dL_dopacity == nullptr || dL_dmeans3D == nullptr || radii == nullptr || means3D == nullptr)
    return fail(GSR_EINVAL, "%s", "null pointer argument");
  if (shs != nullptr && dL_dsh == nullptr) return fail(GSR_EINVAL, "%s", "dL_dsh required with SHs");
  if (cov3D_precomp == nullptr && (scales == nullptr || rotations == nullptr || dL_dscales == nullptr ||
                                   dL_drotations == nullptr))
    return fail(GSR_EINVAL, "%s", "scales/rotations and their gradients required");
  hipStream_t s = (hipStream_t)stream;
  GeomState g = GeomState::carve((void*)geom, P, nullptr);
  BinningState b = BinningState::carve((void*)binning, K, nullptr);
  ImageState img = ImageState::carve((void*)image, width, height, nullptr);
  BackwardState bw = BackwardState::carve(work, K, nullptr);
  {
    PhaseScope ps(GSR_PHASE_RENDER_BWD, s);
    launch_render_backward(width, height, K, g, b.val[tile_sort_result(width, height)], img, bg, dL_dcolor,
                           dL_ddepth, dL_dalpha, bw, s);
  }

  GaussBackwardArgs a = shared_args(P, degree, M, means3D, scales, scale_modifier, rotations, shs, cov3D_precomp,
                                     dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales,
                                     dL_drotations);
  ViewBatch vb;
  vb.n = 1;
  vb.accumulate = 0;
  vb.v[0] = make_view_desc(viewmatrix, projmatrix, campos, radii, g, img, bw, dL_dmeans2D, width, height,
                           tanfovx, tanfovy);
  {
    PhaseScope ps(GSR_PHASE_GAUSS_BWD, s);
    launch_gauss_backward_views(a, vb, s);
  }
  return last_launch();
}

// ---- view-batched path ---------------------------------------------------------------------

int gsr_num_rendered_many(int n_views, const void* const* geoms, int P, int* num_rendered, void* stream) {
  if (n_views < 0 || (n_views > 0 && (geoms == nullptr || num_rendered == nullptr)))
    return fail(GSR_EINVAL, "%s", "null pointer argument");
  hipStream_t s = (hipStream_t)stream;
  static thread_local uint32_t* pinned = nullptr;
  static thread_local int pinned_n = 0;
  if (pinned_n < n_views) {
    if (pinned) (void)hipHostFree(pinned);
    pinned = nullptr;
    GSR_HIP_CHECK(hipHostMalloc((void**)&pinned, 4 * sizeof(uint32_t) * (size_t)n_views, hipHostMallocDefault));
    pinned_n = n_views;
  }
  for (int v = 0; v < n_views; ++v) {
    if (geoms[v] == nullptr) return fail(GSR_EINVAL, "%s", "null geom buffer");
    GeomState g = GeomState::carve((void*)geoms[v], P, nullptr);
    if (P > 0) GSR_HIP_CHECK(hipMemcpyAsync(pinned + 4 * v, g.counters, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    else pinned[4 * v + GSR_CTR_K] = pinned[4 * v + GSR_CTR_ERR] = 0u;
  }
  GSR_HIP_CHECK(hipStreamSynchronize(s));
  for (int v = 0; v < n_views; ++v) {
    if (pinned[4 * v + GSR_CTR_ERR]) return fail(GSR_EHIP, "%s", "internal: look-back timeout in compaction / depth sort");
    num_rendered[v] = (int)pinned[4 * v + GSR_CTR_K];
  }
  g_err[0] = 0;
  return GSR_OK;
}

int gsr_backward_render(int P, int K, int width, int height, const float* bg, const void* geom,
                        const void* binning, const void* image, const float* dL_dcolor,
                        const float* dL_ddepth, const float* dL_dalpha, void* work, void* stream) {
  if (P < 0 || K < 0 || width <= 0 || height <= 0) return fail(GSR_EINVAL, "%s", "bad sizes");
  if (geom == nullptr || binning == nullptr || image == nullptr || work == nullptr || bg == nullptr ||
      dL_dcolor == nullptr)
    return fail(GSR_EINVAL, "%s", "null pointer argument");
  hipStream_t s = (hipStream_t)stream;
  GeomState g = GeomState::carve((void*)geom, P, nullptr);
  BinningState b = BinningState::carve((void*)binning, K, nullptr);
  ImageState img = ImageState::carve((void*)image, width, height, nullptr);
  BackwardState bw = BackwardState::carve(work, K, nullptr);
  {
    PhaseScope ps(GSR_PHASE_RENDER_BWD, s);
    launch_render_backward(width, height, K, g, b.val[tile_sort_result(width, height)], img, bg, dL_dcolor,
                           dL_ddepth, dL_dalpha, bw, s);
  }
  return last_launch();
}

int gsr_backward_gaussians_many(int n_views, int P, int degree, int M, const int* widths, const int* heights,
                                const float* tanfovx, const float* tanfovy, const float* const* viewmatrices,
                                const float* const* projmatrices, const float* const* campos,
                                const int* const* radii, const void* const* geoms, const void* const* images,
                                const void* const* works, const int* Ks, const float* means3D,
                                const float* scales, float scale_modifier, const float* rotations,
                                const float* shs, const float* cov3D_precomp, float* const* dL_dmeans2D,
                                float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D,
                                float* dL_dsh, float* dL_dscales, float* dL_drotations, int accumulate,
                                void* stream) {
  if (n_views < 0 || P < 0) return fail(GSR_EINVAL, "%s", "bad sizes");
  if (P == 0 || n_views == 0) return last_launch();
  if (widths == nullptr || heights == nullptr || tanfovx == nullptr || tanfovy == nullptr ||
      viewmatrices == nullptr || projmatrices == nullptr || campos == nullptr || radii == nullptr ||
      geoms == nullptr || images == nullptr || works == nullptr || Ks == nullptr || dL_dmeans2D == nullptr ||
      means3D == nullptr || dL_dopacity == nullptr || dL_dmeans3D == nullptr)
    return fail(GSR_EINVAL, "%s", "null pointer argument");
  if (shs != nullptr && dL_dsh == nullptr) return fail(GSR_EINVAL, "%s", "dL_dsh required with SHs");
  if (cov3D_precomp == nullptr && (scales == nullptr || rotations == nullptr || dL_dscales == nullptr ||
                                   dL_drotations == nullptr))
    return fail(GSR_EINVAL, "%s", "scales/rotations and their gradients required");
  hipStream_t s = (hipStream_t)stream;
  GaussBackwardArgs a = shared_args(P, degree, M, means3D, scales, scale_modifier, rotations, shs, cov3D_precomp,
                                     dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales,
                                     dL_drotations);
  for (int v0 = 0; v0 < n_views; v0 += GSR_VIEWS_PER_LAUNCH) {
    ViewBatch vb;
    vb.n = n_views - v0 < GSR_VIEWS_PER_LAUNCH ? n_views - v0 : GSR_VIEWS_PER_LAUNCH;
    vb.accumulate = (accumulate || v0 > 0) ? 1 : 0;
    for (int j = 0; j < vb.n; ++j) {
      const int v = v0 + j;
      if (widths[v] <= 0 || heights[v] <= 0 || Ks[v] < 0) return fail(GSR_EINVAL, "%s", "bad view sizes");
      if (geoms[v] == nullptr || images[v] == nullptr || works[v] == nullptr || dL_dmeans2D[v] == nullptr)
        return fail(GSR_EINVAL, "%s", "null per-view buffer");
      GeomState g = GeomState::carve((void*)geoms[v], P, nullptr);
      ImageState img = ImageState::carve((void*)images[v], widths[v], heights[v], nullptr);
      BackwardState bw = BackwardState::carve((void*)works[v], Ks[v], nullptr);
      vb.v[j] = make_view_desc(viewmatrices[v], projmatrices[v], campos[v], radii[v], g, img, bw, dL_dmeans2D[v],
                               widths[v], heights[v], tanfovx[v], tanfovy[v]);
    }
    PhaseScope ps(GSR_PHASE_GAUSS_BWD, s);
    launch_gauss_backward_views(a, vb, s);
  }
  return last_launch();
}

int gsr_profile_enable(int enable) {
  Profiler& p = prof();
  std::lock_guard<std::mutex> g(p.mu);
  p.on = enable != 0;
  return GSR_OK;
}

int gsr_profile_read(double* ms, long long* launches, int reset) {
  Profiler& p = prof();
  std::lock_guard<std::mutex> g(p.mu);
  for (const PhaseEvents& e : p.pending) {
    float t = 0.f;
    GSR_HIP_CHECK(hipEventSynchronize(e.b));
    GSR_HIP_CHECK(hipEventElapsedTime(&t, e.a, e.b));
    p.ms[e.phase] += t;
    p.n[e.phase] += 1;
    p.pool.push_back(e.a);
    p.pool.push_back(e.b);
  }
  p.pending.clear();
  for (int i = 0; i < GSR_NUM_PHASES; ++i) {
    if (ms) ms[i] = p.ms[i];
    if (launches) launches[i] = p.n[i];
    if (reset) {
      p.ms[i] = 0;
      p.n[i] = 0;
    }
  }
  return GSR_OK;
}

int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     uint8_t* present, void* stream) {
  if (P < 0) return fail(GSR_EINVAL, "%s", "P must be >= 0");
  if (P > 0 && (means3D == nullptr || viewmatrix == nullptr || present == nullptr))
    return fail(GSR_EINVAL, "%s", "null pointer argument");
  launch_mark_visible(P, means3D, viewmatrix, projmatrix, present, (hipStream_t)stream);
  return last_launch();
}

}  // extern "C"

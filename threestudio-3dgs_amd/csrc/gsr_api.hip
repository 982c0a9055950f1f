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

// The instance key layout's test override (GSR_TILE_KEYS = unpacked | plain), read ONCE per process: the forward
// and the backward of a set derive the binning buffer's layout (packed keys, quadrant masks, which ping-pong array
// holds the sorted list) from it on the host, so it must not change between them.
static int tile_keys_mode() {
  static const int mode = [] {
    const char* e = getenv("GSR_TILE_KEYS");
    if (e != nullptr && strcmp(e, "unpacked") == 0) return 1;
    if (e != nullptr && strcmp(e, "plain") == 0) return 2;
    return 0;
  }();
  return mode;
}
static TilePack set_tile_pack(int P, int W, int H) { return tile_pack(P, W, H, tile_keys_mode()); }

static int effective_degree(int degree, int M) {
  // the reference reads sqrt(M)-1 coefficients at most (pred-normal pass quirk)
  int dm = (int)std::lround(std::sqrt((double)(M > 0 ? M : 1))) - 1;
  int d = degree < dm ? degree : dm;
  if (d < 0) d = 0;
  if (d > 3) d = 3;
  return d;
}

// ping-pong buffers holding the sorts' results (one pass per <= 8 key bits)
static int tile_sort_result(int W, int H) { return digit_plan(tile_key_bits(W, H)).passes & 1; }
static int depth_sort_result() { return digit_plan(32).passes & 1; }

static GaussBackwardArgs shared_args(int P, int degree, int M, const float* means3D, const float* scales,
                                     float scale_modifier, const float* rotations, const float* shs,
                                     const float* cov3D_precomp, float* dL_dcolors, float* dL_dopacity,
                                     float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscales,
                                     float* dL_drotations) {
  GaussBackwardArgs a;
  a.P = P;
  a.g0 = 0;
  a.g1 = P;
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

// Instance segments of a set from the host copy of K (checked: the set's total < 2^32).
static int inst_segments(int V, const int* K, SegInfo& seg, long long* total) {
  seg.V = V;
  long long run = 0;
  for (int v = 0; v < V; ++v) {
    if (K[v] < 0) return fail(GSR_EINVAL, "%s", "negative instance count");
    seg.n[v] = (uint32_t)K[v];
    seg.start[v] = (uint32_t)run;
    run += K[v];
    if (run >= (1ll << 32)) return fail(GSR_EINVAL, "%s", "instances of a view set exceed 2^32: use smaller sets");
  }
  seg_fill_blocks(seg, GSR_SORT_TILE);
  if (total) *total = run;
  return GSR_OK;
}

static int set_cams(int V, const float* const* viewmatrices, const float* const* projmatrices,
                    const float* const* campos, const float* tanfovx, const float* tanfovy, SetCams& cams) {
  if (viewmatrices == nullptr || projmatrices == nullptr || campos == nullptr || tanfovx == nullptr ||
      tanfovy == nullptr)
    return fail(GSR_EINVAL, "%s", "null camera array");
  for (int v = 0; v < V; ++v) {
    if (viewmatrices[v] == nullptr || projmatrices[v] == nullptr || campos[v] == nullptr)
      return fail(GSR_EINVAL, "%s", "null camera pointer");
    cams.c[v].view = viewmatrices[v];
    cams.c[v].proj = projmatrices[v];
    cams.c[v].campos = campos[v];
    cams.c[v].tanx = tanfovx[v];
    cams.c[v].tany = tanfovy[v];
  }
  return GSR_OK;
}

static int check_set(int V, int P) {
  if (V < 1 || V > GSR_SET_MAX) return fail(GSR_EINVAL, "%s", "a view set holds 1..64 views");
  if (P < 0) return fail(GSR_EINVAL, "%s", "P must be >= 0");
  if ((long long)V * (long long)(P > 0 ? P : 1) >= (1ll << 32))
    return fail(GSR_EINVAL, "%s", "views x Gaussians of a set exceed 2^32: use smaller sets");
  return GSR_OK;
}

extern "C" {

#ifndef GSR_BUILD_ID
#define GSR_BUILD_ID "unknown"
#endif
// "gsr <version> gfx950 build <id>": the id hashes the sources the library was built from (csrc/Makefile)
const char* gsr_version(void) { return "gsr 0.4.0 gfx950 build " GSR_BUILD_ID; }
int gsr_abi_version(void) { return GSR_ABI_VERSION; }
const char* gsr_last_error(void) { return g_err; }

// ---- view sets ---------------------------------------------------------------------------

size_t gsr_set_geom_bytes(int V, int P) {
  size_t b = 0;
  GeomState::carve(nullptr, V, P, &b);
  return b;
}
size_t gsr_set_binning_bytes(int V, int P, const int* K, int width, int height) {
  SegInfo seg;
  long long total = 0;
  if (V < 1 || V > GSR_SET_MAX || K == nullptr || inst_segments(V, K, seg, &total) != GSR_OK) return 0;
  size_t b = 0;
  BinningState::carve(nullptr, V, total, seg.blk[V], !set_tile_pack(P, width, height).packed, &b);
  return b;
}
size_t gsr_set_image_bytes(int V, int width, int height) {
  size_t b = 0;
  ImageState::carve(nullptr, V, width, height, &b);
  return b;
}
size_t gsr_set_image_bytes_ex(int V, int P, const int* K, int width, int height, int two_colors) {
  SegInfo seg;
  long long total = 0;
  if (V < 1 || V > GSR_SET_MAX || K == nullptr || inst_segments(V, K, seg, &total) != GSR_OK) return 0;
  size_t b = 0;
  ImageState::carve(nullptr, V, width, height, &b, split_forward(V, P, width, height, total, two_colors != 0));
  return b;
}
// the running dL/dcov3D (P x 6) kept at the end of the work buffer across view groups
static size_t carry_bytes(int P) { return align_up(sizeof(float) * 6 * (size_t)(P > 0 ? P : 1), 256); }

size_t gsr_set_backward_bytes(int V, int P, const int* K) {
  long long total = 0;
  for (int v = 0; v < V; ++v) total += K[v];
  return BackwardState::bytes_for(total, V, P) + carry_bytes(P);
}

int gsr_set_preprocess(int V, int P, int degree, int M, const float* means3D, const float* scales,
                       float scale_modifier, const float* rotations, const float* opacities, const float* shs,
                       const float* colors_precomp, const float* cov3D_precomp, const float* const* viewmatrices,
                       const float* const* projmatrices, const float* const* campos, const float* tanfovx,
                       const float* tanfovy, int width, int height, int prefiltered, int* radii, void* geom,
                       void* stream) {
  return gsr_set_preprocess_ex(V, P, degree, M, means3D, scales, scale_modifier, rotations, opacities, shs,
                               colors_precomp, cov3D_precomp, viewmatrices, projmatrices, campos, tanfovx, tanfovy,
                               width, height, prefiltered, radii, geom, nullptr, stream);
}

int gsr_set_preprocess_ex(int V, int P, int degree, int M, const float* means3D, const float* scales,
                          float scale_modifier, const float* rotations, const float* opacities, const float* shs,
                          const float* colors_precomp, const float* cov3D_precomp, const float* const* viewmatrices,
                          const float* const* projmatrices, const float* const* campos, const float* tanfovx,
                          const float* tanfovy, int width, int height, int prefiltered, int* radii, void* geom,
                          const float* colors2, void* stream) {
  (void)prefiltered;
  if (check_set(V, P) != GSR_OK) return GSR_EINVAL;
  if (width <= 0 || height <= 0) return fail(GSR_EINVAL, "%s", "image size must be positive");
  if ((shs == nullptr) == (colors_precomp == nullptr))
    return fail(GSR_EINVAL, "%s", "Please provide exactly one of either SHs or precomputed colors!");
  if (((scales == nullptr || rotations == nullptr) && cov3D_precomp == nullptr) ||
      ((scales != nullptr || rotations != nullptr) && cov3D_precomp != nullptr))
    return fail(GSR_EINVAL, "%s",
                "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
  if (geom == nullptr || (P > 0 && (means3D == nullptr || opacities == nullptr || radii == nullptr)))
    return fail(GSR_EINVAL, "%s", "null pointer argument");
  if (shs != nullptr && M <= 0) return fail(GSR_EINVAL, "%s", "M must be >= 1 with SHs");
  SetCams cams;
  if (set_cams(V, viewmatrices, projmatrices, campos, tanfovx, tanfovy, cams) != GSR_OK) return GSR_EINVAL;
  for (int v = 0; v < V; ++v) {  // IEEE float division on the host = the device's correctly rounded one
    cams.c[v].fx = (float)width / (2.0f * cams.c[v].tanx);
    cams.c[v].fy = (float)height / (2.0f * cams.c[v].tany);
  }
  hipStream_t s = (hipStream_t)stream;
  GeomState g = GeomState::carve(geom, V, P, nullptr);

  PreprocessArgs a;
  a.V = V;
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
  a.W = width;
  a.H = height;
  a.radii = radii;
  a.col2 = colors2;
  {
    PhaseScope ps(GSR_PHASE_PREPROCESS, s);
    launch_preprocess(a, cams, g, s);
  }
  {
    // depth sort of every view's Gaussians (culled last) -> instance counts in depth order, K_v
    PhaseScope ps(GSR_PHASE_DEPTH_SORT, s);
    SegInfo seg;
    seg.V = V;
    for (int v = 0; v < V; ++v) {
      seg.n[v] = (uint32_t)P;
      seg.start[v] = (uint32_t)((size_t)v * P);
    }
    seg.rebase = g.drange + 128;  // keys ranked relative to the set's smallest visible key (preprocess)
    const int res = seg_sort(g.dkey, g.dval, false, seg, 0, 32, g.sort_counts, g.sort_totals, s);
    if (res != depth_sort_result()) return fail(GSR_EHIP, "%s", "internal: depth sort result buffer");
    launch_binning_counts(V, P, g, s);  // reads the sorted buffer the device flag names (3 or 4 passes)
  }
  return last_launch();
}

int gsr_composite_forward(int V, int height, int width, const float* color, const float* alpha, const float* bg,
                          int bg_layout, float* out, void* stream) {
  if (V < 0 || height < 0 || width < 0 || bg_layout < 0 || bg_layout > 2) return fail(GSR_EINVAL, "%s", "bad sizes");
  if (V == 0 || height == 0 || width == 0) return last_launch();
  if (color == nullptr || alpha == nullptr || bg == nullptr || out == nullptr)
    return fail(GSR_EINVAL, "%s", "null pointer argument");
  launch_composite_fwd(V, (size_t)height * width, color, alpha, bg, bg_layout, out, (hipStream_t)stream);
  return last_launch();
}

int gsr_composite_backward(int V, int height, int width, const float* dL_dout, const float* color,
                           const float* alpha, const float* bg, int bg_layout, float* dL_dcolor, float* dL_dalpha,
                           float* dL_dbg, void* stream) {
  if (V < 0 || height < 0 || width < 0 || bg_layout < 0 || bg_layout > 2) return fail(GSR_EINVAL, "%s", "bad sizes");
  if (V == 0 || height == 0 || width == 0) return last_launch();
  if (dL_dout == nullptr || color == nullptr || alpha == nullptr || bg == nullptr || dL_dcolor == nullptr ||
      dL_dalpha == nullptr)
    return fail(GSR_EINVAL, "%s", "null pointer argument");
  if (dL_dbg != nullptr && bg_layout == GSR_BG_CONSTANT)
    return fail(GSR_EINVAL, "%s", "dL_dbg is computed for image backgrounds only");
  launch_composite_bwd(V, (size_t)height * width, dL_dout, color, alpha, bg, bg_layout, dL_dcolor, dL_dalpha,
                       dL_dbg, (hipStream_t)stream);
  return last_launch();
}

int gsr_normal_map_forward(int V, int height, int width, const float* normal, const float* alpha, float* out,
                           void* stream) {
  if (V < 0 || height < 0 || width < 0) return fail(GSR_EINVAL, "%s", "bad sizes");
  if (V == 0 || height == 0 || width == 0) return last_launch();
  if (normal == nullptr || alpha == nullptr || out == nullptr) return fail(GSR_EINVAL, "%s", "null pointer argument");
  launch_normal_map_fwd(V, (size_t)height * width, normal, alpha, out, (hipStream_t)stream);
  return last_launch();
}

int gsr_normal_map_backward(int V, int height, int width, const float* dL_dout, const float* normal,
                            const float* alpha, float* dL_dnormal, float* dL_dalpha, void* stream) {
  if (V < 0 || height < 0 || width < 0) return fail(GSR_EINVAL, "%s", "bad sizes");
  if (V == 0 || height == 0 || width == 0) return last_launch();
  if (dL_dout == nullptr || normal == nullptr || alpha == nullptr || dL_dnormal == nullptr || dL_dalpha == nullptr)
    return fail(GSR_EINVAL, "%s", "null pointer argument");
  launch_normal_map_bwd(V, (size_t)height * width, dL_dout, normal, alpha, dL_dnormal, dL_dalpha, (hipStream_t)stream);
  return last_launch();
}

static int shade_args(int V, int H, int W, int flags, const int* modes, const float* color, const float* depth,
                      const float* alpha, const float* rays_o, const float* rays_d, const float* bg, int bg_layout,
                      const float* light, const float* pred_normal, const float* ambient, const float* diffuse,
                      ShadeArgs& A) {
  if (V < 0 || H < 0 || W < 0 || (flags & ~GSR_SHADE_MATERIAL) != 0)
    return fail(GSR_EINVAL, "%s", "bad sizes / flags");
  if (depth == nullptr || alpha == nullptr || rays_o == nullptr || rays_d == nullptr)
    return fail(GSR_EINVAL, "%s", "null pointer argument (depth / alpha / rays)");
  A = ShadeArgs{};
  A.V = V, A.H = H, A.W = W, A.flags = flags, A.bg_layout = bg_layout;
  A.color = color, A.depth = depth, A.alpha = alpha, A.rays_o = rays_o, A.rays_d = rays_d;
  A.bg = bg, A.light = light, A.pred_normal = pred_normal;
  if (flags & GSR_SHADE_MATERIAL) {
    if (color == nullptr || bg == nullptr || light == nullptr || ambient == nullptr || diffuse == nullptr ||
        modes == nullptr)
      return fail(GSR_EINVAL, "%s", "material: color, bg, light, ambient, diffuse and modes are required");
    if (bg_layout != GSR_BG_CONSTANT && bg_layout != GSR_BG_HWC)
      return fail(GSR_EINVAL, "%s", "material: bg_layout must be GSR_BG_CONSTANT or GSR_BG_HWC");
    for (int v = 0; v < V; ++v)
      if (modes[v] < GSR_SHADING_DIFFUSE || modes[v] > GSR_SHADING_TEXTURELESS)
        return fail(GSR_EINVAL, "%s", "bad shading mode");
  }
  return GSR_OK;
}

// Launches in chunks of GSR_SET_MAX views, each with its views' light colours and modes in the arguments.
static void shade_launch(ShadeArgs A, const ShadeGrads* G, const int* modes, const float* ambient,
                         const float* diffuse, hipStream_t s) {
  const int V = A.V;
  for (int v0 = 0; v0 < V; v0 += GSR_SET_MAX) {
    const int n = V - v0 < GSR_SET_MAX ? V - v0 : GSR_SET_MAX;
    A.v0 = v0, A.V = n;
    for (int i = 0; i < n; ++i) {
      A.mode[i] = (A.flags & GSR_SHADE_MATERIAL) ? modes[v0 + i] : 0;
      for (int k = 0; k < 3; ++k) {
        A.ka[i][k] = (A.flags & GSR_SHADE_MATERIAL) ? ambient[3 * (v0 + i) + k] : 0.0f;
        A.kd[i][k] = (A.flags & GSR_SHADE_MATERIAL) ? diffuse[3 * (v0 + i) + k] : 0.0f;
      }
    }
    if (G == nullptr)
      launch_shade_fwd(A, s);
    else
      launch_shade_bwd(A, *G, s);
  }
}

int gsr_shade_views_forward(int V, int height, int width, int flags, const int* modes, const float* color,
                            const float* depth, const float* alpha, const float* rays_o, const float* rays_d,
                            const float* bg, int bg_layout, const float* light, const float* pred_normal,
                            const float* ambient, const float* diffuse, float* render, float* normal_map,
                            float* unit_normal, float* depth_out, void* stream) {
  ShadeArgs A;
  if (shade_args(V, height, width, flags, modes, color, depth, alpha, rays_o, rays_d, bg, bg_layout, light,
                 pred_normal, ambient, diffuse, A) != GSR_OK)
    return GSR_EINVAL;
  if ((flags & GSR_SHADE_MATERIAL) && render == nullptr)
    return fail(GSR_EINVAL, "%s", "material: render output is required");
  if (V == 0 || height == 0 || width == 0) return last_launch();
  A.render = render, A.nmap = normal_map, A.unit = unit_normal, A.depth_out = depth_out;
  shade_launch(A, nullptr, modes, ambient, diffuse, (hipStream_t)stream);
  return last_launch();
}

int gsr_shade_views_backward(int V, int height, int width, int flags, const int* modes, const float* color,
                             const float* depth, const float* alpha, const float* rays_o, const float* rays_d,
                             const float* bg, int bg_layout, const float* light, const float* pred_normal,
                             const float* ambient, const float* diffuse, const float* dL_drender,
                             const float* dL_dnormal_map, const float* dL_dunit_normal, const float* dL_ddepth_out,
                             float* dL_dcolor, float* dL_ddepth, float* dL_dalpha, float* dL_dbg, void* stream) {
  ShadeArgs A;
  if (shade_args(V, height, width, flags, modes, color, depth, alpha, rays_o, rays_d, bg, bg_layout, light,
                 pred_normal, ambient, diffuse, A) != GSR_OK)
    return GSR_EINVAL;
  if (dL_ddepth == nullptr || dL_dalpha == nullptr) return fail(GSR_EINVAL, "%s", "dL_ddepth / dL_dalpha required");
  if ((flags & GSR_SHADE_MATERIAL) && dL_dcolor == nullptr)
    return fail(GSR_EINVAL, "%s", "material: dL_dcolor is required");
  if (dL_dbg != nullptr && !((flags & GSR_SHADE_MATERIAL) && bg_layout == GSR_BG_HWC))
    return fail(GSR_EINVAL, "%s", "dL_dbg is formed for GSR_BG_HWC material shading only");
  if (V == 0 || height == 0 || width == 0) return last_launch();
  ShadeGrads G{dL_drender, dL_dnormal_map, dL_dunit_normal, dL_ddepth_out, dL_dcolor, dL_ddepth, dL_dalpha, dL_dbg};
  shade_launch(A, &G, modes, ambient, diffuse, (hipStream_t)stream);
  return last_launch();
}

// one (ambient, diffuse, mode) for every view: the per-view tables filled with copies
struct SharedLight {
  std::vector<int> modes;
  std::vector<float> ka, kd;
  SharedLight(int V, int mode, const float* ambient, const float* diffuse)
      : modes(V > 0 ? V : 0, mode), ka(3 * (size_t)(V > 0 ? V : 0)), kd(3 * (size_t)(V > 0 ? V : 0)) {
    for (int v = 0; v < V; ++v)
      for (int k = 0; k < 3; ++k) {
        ka[3 * v + k] = ambient ? ambient[k] : 0.0f;
        kd[3 * v + k] = diffuse ? diffuse[k] : 0.0f;
      }
  }
};

int gsr_shade_forward(int V, int height, int width, int flags, int mode, const float* color, const float* depth,
                      const float* alpha, const float* rays_o, const float* rays_d, const float* bg, int bg_layout,
                      const float* light, const float* pred_normal, const float* ambient, const float* diffuse,
                      float* render, float* normal_map, float* unit_normal, float* depth_out, void* stream) {
  if (V < 0 || V > 65535 || mode < 0 || mode > 2) return fail(GSR_EINVAL, "%s", "bad sizes / mode / flags");
  if ((flags & GSR_SHADE_MATERIAL) && (ambient == nullptr || diffuse == nullptr))
    return fail(GSR_EINVAL, "%s", "material: color, bg, light, ambient, diffuse and modes are required");
  SharedLight L(V, mode, ambient, diffuse);
  return gsr_shade_views_forward(V, height, width, flags, L.modes.data(), color, depth, alpha, rays_o, rays_d, bg,
                                 bg_layout, light, pred_normal, L.ka.data(), L.kd.data(), render, normal_map,
                                 unit_normal, depth_out, stream);
}

int gsr_shade_backward(int V, int height, int width, int flags, int mode, const float* color, const float* depth,
                       const float* alpha, const float* rays_o, const float* rays_d, const float* bg, int bg_layout,
                       const float* light, const float* pred_normal, const float* ambient, const float* diffuse,
                       const float* dL_drender, const float* dL_dnormal_map, const float* dL_dunit_normal,
                       const float* dL_ddepth_out, float* dL_dcolor, float* dL_ddepth, float* dL_dalpha,
                       float* dL_dbg, void* stream) {
  if (V < 0 || V > 65535 || mode < 0 || mode > 2) return fail(GSR_EINVAL, "%s", "bad sizes / mode / flags");
  if ((flags & GSR_SHADE_MATERIAL) && (ambient == nullptr || diffuse == nullptr))
    return fail(GSR_EINVAL, "%s", "material: color, bg, light, ambient, diffuse and modes are required");
  SharedLight L(V, mode, ambient, diffuse);
  return gsr_shade_views_backward(V, height, width, flags, L.modes.data(), color, depth, alpha, rays_o, rays_d, bg,
                                  bg_layout, light, pred_normal, L.ka.data(), L.kd.data(), dL_drender,
                                  dL_dnormal_map, dL_dunit_normal, dL_ddepth_out, dL_dcolor, dL_ddepth, dL_dalpha,
                                  dL_dbg, stream);
}

size_t gsr_knn_workspace_bytes(int P) { return knn_workspace_bytes(P < 0 ? 0 : P); }

int gsr_knn_mean_dist(int P, const float* points, float* mean_dist, void* workspace, size_t workspace_bytes,
                      void* stream) {
  if (P < 0) return fail(GSR_EINVAL, "%s", "negative point count");
  if (P == 0) return last_launch();
  if (points == nullptr || mean_dist == nullptr || workspace == nullptr)
    return fail(GSR_EINVAL, "%s", "null pointer argument");
  if (workspace_bytes < knn_workspace_bytes(P)) return fail(GSR_EINVAL, "%s", "workspace too small");
  launch_knn_mean_dist(P, points, mean_dist, workspace, (hipStream_t)stream);
  return last_launch();
}

// ---- the view-segmented radix sort (tests: every sort of the library runs seg_sort) -----------------
struct SortWork {
  uint32_t *keys2, *vals2, *counts, *totals;
  static SortWork carve(void* base, int V, long long total, uint32_t blocks, size_t* bytes) {
    Carver c(base);
    SortWork w;
    w.keys2 = c.take<uint32_t>((size_t)(total > 0 ? total : 1));
    w.vals2 = c.take<uint32_t>((size_t)(total > 0 ? total : 1));
    w.counts = c.take<uint32_t>((size_t)GSR_RADIX * (blocks > 0 ? blocks : 1));
    w.totals = c.take<uint32_t>((size_t)GSR_RADIX * (size_t)V);
    if (bytes) *bytes = align_up(c.off, 256);
    return w;
  }
};

size_t gsr_sort_work_bytes(int V, const int* n) {
  SegInfo seg;
  long long total = 0;
  if (V < 1 || V > GSR_SET_MAX || n == nullptr || inst_segments(V, n, seg, &total) != GSR_OK) return 0;
  size_t b = 0;
  SortWork::carve(nullptr, V, total, seg.blk[V], &b);
  return b;
}

int gsr_sort_pairs(int V, const int* n, uint32_t* keys, uint32_t* vals, int key_bits, int max_bits, void* work,
                   size_t work_bytes, void* stream) {
  if (V < 1 || V > GSR_SET_MAX) return fail(GSR_EINVAL, "%s", "1..64 segments");
  if (n == nullptr || keys == nullptr || work == nullptr) return fail(GSR_EINVAL, "%s", "null pointer argument");
  if (key_bits < 1 || key_bits > 32 || max_bits < 1 || max_bits > GSR_RADIX_BITS)
    return fail(GSR_EINVAL, "%s", "key_bits must be 1..32 and max_bits 1..8");
  SegInfo seg;
  long long total = 0;
  if (inst_segments(V, n, seg, &total) != GSR_OK) return GSR_EINVAL;
  size_t need = 0;
  SortWork w = SortWork::carve(work, V, total, seg.blk[V], &need);
  if (work_bytes < need) return fail(GSR_EINVAL, "%s", "sort work buffer too small");
  if (total == 0) return last_launch();
  hipStream_t s = (hipStream_t)stream;
  uint32_t* kk[2] = {keys, w.keys2};
  uint32_t* vv[2] = {vals, vals != nullptr ? w.vals2 : nullptr};
  const int r = seg_sort(kk, vals != nullptr ? vv : nullptr, false, seg, 0, key_bits, w.counts, w.totals, s,
                         max_bits);
  if (r == 1) {  // (an odd number of passes: the result is in the work buffer)
    GSR_HIP_CHECK(hipMemcpyAsync(keys, w.keys2, sizeof(uint32_t) * (size_t)total, hipMemcpyDeviceToDevice, s));
    if (vals != nullptr)
      GSR_HIP_CHECK(hipMemcpyAsync(vals, w.vals2, sizeof(uint32_t) * (size_t)total, hipMemcpyDeviceToDevice, s));
  }
  return last_launch();
}

int gsr_sort_rank_mode(void) { return sort_rank_mode(); }

int gsr_set_num_rendered_ex(int V, const void* geom, int P, int* num_rendered, int* num_visible, int* num_listed,
                            void* stream) {
  if (check_set(V, P) != GSR_OK) return GSR_EINVAL;
  if (geom == nullptr || num_rendered == nullptr) return fail(GSR_EINVAL, "%s", "null pointer argument");
  GeomState g = GeomState::carve((void*)geom, V, P, nullptr);
  hipStream_t s = (hipStream_t)stream;
  static thread_local uint32_t* pinned = nullptr;
  if (pinned == nullptr) GSR_HIP_CHECK(hipHostMalloc((void**)&pinned, 3 * GSR_SET_MAX * sizeof(uint32_t), hipHostMallocDefault));
  GSR_HIP_CHECK(hipMemcpyAsync(pinned, g.counters, 3 * (size_t)V * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  GSR_HIP_CHECK(hipStreamSynchronize(s));
  for (int v = 0; v < V; ++v) {
    num_rendered[v] = (int)pinned[v];
    if (num_visible) num_visible[v] = (int)pinned[V + v];
    if (num_listed) num_listed[v] = (int)pinned[2 * V + v];
    if (pinned[v] > 0x7fffffffu) return fail(GSR_EINVAL, "%s", "instance count of a view exceeds 2^31");
  }
  g_err[0] = 0;
  return GSR_OK;
}

int gsr_set_gauss_state(int V, const void* geom, int P, void* out_rec, void* out_tiles, void* stream) {
  if (check_set(V, P) != GSR_OK) return GSR_EINVAL;
  if (geom == nullptr) return fail(GSR_EINVAL, "%s", "null pointer argument");
  if (P == 0) return GSR_OK;
  GeomState g = GeomState::carve((void*)geom, V, P, nullptr);
  hipStream_t s = (hipStream_t)stream;
  const size_t n = (size_t)V * (size_t)P;
  if (out_rec) GSR_HIP_CHECK(hipMemcpyAsync(out_rec, g.rec, n * sizeof(GaussRec), hipMemcpyDeviceToDevice, s));
  if (out_tiles) GSR_HIP_CHECK(hipMemcpyAsync(out_tiles, g.tiles, n * sizeof(uint2), hipMemcpyDeviceToDevice, s));
  return last_launch();
}

int gsr_set_num_rendered(int V, const void* geom, int P, int* num_rendered, int* num_visible, void* stream) {
  return gsr_set_num_rendered_ex(V, geom, P, num_rendered, num_visible, nullptr, stream);
}

static int set_render(int V, int P, const int* K, int width, int height, const float* const* bgs, void* geom,
                      void* binning, void* image, float* out_color, float* out_depth, float* out_alpha,
                      const float* comp_bg, float* out_render, void* stream, const float* colors2 = nullptr,
                      float* out_color2 = nullptr) {
  if (check_set(V, P) != GSR_OK) return GSR_EINVAL;
  if (width <= 0 || height <= 0) return fail(GSR_EINVAL, "%s", "bad sizes");
  if (K == nullptr || bgs == nullptr || geom == nullptr || binning == nullptr || image == nullptr ||
      out_color == nullptr || out_depth == nullptr || out_alpha == nullptr)
    return fail(GSR_EINVAL, "%s", "null pointer argument");
  SegInfo inst;
  long long total = 0;
  if (inst_segments(V, K, inst, &total) != GSR_OK) return GSR_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  GeomState g = GeomState::carve(geom, V, P, nullptr);
  const TilePack tp = set_tile_pack(P, width, height);
  BinningState b = BinningState::carve(binning, V, total, inst.blk[V], !tp.packed, nullptr);
  // the split decision of this forward, recorded in the image state for its backward
  const bool split = split_forward(V, P, width, height, total, colors2 != nullptr);
  ImageState img = ImageState::carve(image, V, width, height, nullptr, split);
  const int gx = div_up(width, GSR_TILE_X), gy = div_up(height, GSR_TILE_Y);
  const int tres = tile_sort_result(width, height);
  inst.ndev = g.counters + 2 * V;  // kept instances per view (<= K, the list capacity)
  GSR_HIP_CHECK(hipMemsetAsync(img.split_mode, split ? 1 : 0, sizeof(uint32_t), s));
  // the forward records its cull of each listed instance for the backward (in the free ping-pong key array of the
  // binning buffer, 4 bytes per instance); [1] says in which layout: 1 = the tile-wave forward's 4-bit mask per
  // byte, 2 = one byte per (instance, quadrant) from the quadrant-wave forward's waves
  const bool tile_masks = fwd_tile_chosen(total, (long long)V * P, V);
  GSR_HIP_CHECK(hipMemsetAsync(img.split_mode + 1, total > 0 ? (tile_masks ? 1 : 2) : 0, sizeof(uint32_t), s));
  {
    PhaseScope ps(GSR_PHASE_BINNING, s);
    GSR_HIP_CHECK(hipMemsetAsync(img.ranges, 0, sizeof(uint2) * (size_t)V * gx * gy, s));
    if (total > 0) {
      launch_emit(V, P, width, g, inst, tp, b.key[0], b.val[0], s);
      const int res = seg_sort(b.key, b.val, false, inst, tp.gbits, tp.tile_bits, b.sort_counts, b.sort_totals, s);
      if (res != tres) return fail(GSR_EHIP, "%s", "internal: tile sort buffer");
      launch_tile_ranges(inst, gx * gy, tp, b.key[res], img.ranges, s);
    }
    launch_tile_order(V, gx, gy, img.ranges, img.order, s);  // always written: the backward may use it
  }
  {
    PhaseScope ps(GSR_PHASE_RENDER_FWD, s);
    RenderSet rs;
    rs.cbg = comp_bg;
    rs.comp = out_render;
    rs.ccolor = nullptr;
    rs.dcbg = nullptr;
    rs.col2 = colors2;
    rs.col2_rec = g.drange + 130;
    rs.out_col2 = out_color2;
    rs.dpix2 = nullptr;
    rs.order = img.order;
    rs.ochunk = order_chunk(V, gx, gy, true);
    rs.ckpt = split ? img.ckpt : nullptr;
    rs.split_mode = img.split_mode;
    rs.split_items = img.split_items;
    rs.split_cap = img.split_cap;
    rs.split_extra = split_extra(V, (size_t)gx * gy);
    rs.qkeys = tp.qmask ? b.key[tres] : nullptr;
    rs.qbytes = total > 0 ? reinterpret_cast<uint8_t*>(b.key[tres ^ 1]) : nullptr;
    rs.V = V;
    rs.v0 = 0;
    rs.P = P;
    rs.W = width;
    rs.H = height;
    rs.gx = gx;
    rs.gy = gy;
    rs.gmask = tp.gmask;
    for (int v = 0; v < V; ++v) {
      if (bgs[v] == nullptr) return fail(GSR_EINVAL, "%s", "null background");
      rs.inst_start[v] = inst.start[v];
      rs.row_start[v] = 0;
      rs.bg[v] = bgs[v];
    }
    launch_render_forward(rs, g, tp.packed ? b.key[tres] : b.val[tres], img, out_color, out_depth, out_alpha, total,
                          s);
  }
  return last_launch();
}

int gsr_set_render(int V, int P, const int* K, int width, int height, const float* const* bgs, void* geom,
                   void* binning, void* image, float* out_color, float* out_depth, float* out_alpha, void* stream) {
  return set_render(V, P, K, width, height, bgs, geom, binning, image, out_color, out_depth, out_alpha, nullptr,
                    nullptr, stream);
}

int gsr_set_render_composite(int V, int P, const int* K, int width, int height, const float* const* bgs, void* geom,
                             void* binning, void* image, float* out_color, float* out_depth, float* out_alpha,
                             const float* bg_images, float* out_render, void* stream) {
  // (bg_images NULL: the clamp alone, out_render = clamp(color, 0, 1))
  if (out_render == nullptr) return fail(GSR_EINVAL, "%s", "null composite argument");
  return set_render(V, P, K, width, height, bgs, geom, binning, image, out_color, out_depth, out_alpha, bg_images,
                    out_render, stream);
}

int gsr_set_render_two_colors(int V, int P, const int* K, int width, int height, const float* const* bgs,
                              void* geom, void* binning, void* image, float* out_color, float* out_depth,
                              float* out_alpha, const float* bg_images, float* out_render, const float* colors2,
                              float* out_color2, void* stream) {
  if (colors2 == nullptr || out_color2 == nullptr) return fail(GSR_EINVAL, "%s", "null second colour argument");
  // (out_render without bg_images: the clamp alone)
  if (bg_images != nullptr && out_render == nullptr) return fail(GSR_EINVAL, "%s", "composite needs out_render");
  return set_render(V, P, K, width, height, bgs, geom, binning, image, out_color, out_depth, out_alpha, bg_images,
                    out_render, stream, colors2, out_color2);
}

// One-shot per-thread request (gsr_set_backward_chunks) for the next backward call on this thread.
struct GradChunks {
  int n = 0;
  void* events[GSR_GRAD_CHUNKS_MAX] = {};
};
static thread_local GradChunks g_next_chunks;

static int grad_chunk_size(int P, int n) {
  const int q = (P + n - 1) / n;
  return (q + GSR_GRAD_CHUNK_ALIGN - 1) / GSR_GRAD_CHUNK_ALIGN * GSR_GRAD_CHUNK_ALIGN;
}

static int set_backward(int V, int P, int degree, int M, const int* K, int width, int height, const float* const* bgs,
                        const float* means3D, const float* scales, float scale_modifier, const float* rotations,
                        const float* shs, const float* cov3D_precomp, const float* const* viewmatrices,
                        const float* const* projmatrices, const float* const* campos, const float* tanfovx,
                        const float* tanfovy, const int* radii, const void* geom, const void* binning,
                        const void* image, const float* dL_dcolor, const float* dL_ddepth, const float* dL_dalpha,
                        float* dL_dmeans2D, float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D,
                        float* dL_dcov3D, float* dL_dsh, float* dL_dscales, float* dL_drotations, int accumulate,
                        void* work, size_t work_bytes, const float* comp_bg, const float* color, float* dL_dbg,
                        void* stream, const float* colors_override = nullptr, const float* colors2 = nullptr,
                        const float* dL_dcolor2 = nullptr, float* dL_dcolors2 = nullptr) {
  const GradChunks chunks = g_next_chunks;  // consumed by this call, whatever its outcome
  g_next_chunks = GradChunks{};
  if (check_set(V, P) != GSR_OK) return GSR_EINVAL;
  // both rasterizer calls of the SuGaR normal renderer in one pass (64-byte rows, 17-field records)
  const bool two = dL_dcolor2 != nullptr;
  if (two && (colors2 == nullptr || dL_dcolors2 == nullptr || colors_override != nullptr))
    return fail(GSR_EINVAL, "%s", "two-colour backward needs colors2, dL_dcolor2 and dL_dcolors2");
  if (width <= 0 || height <= 0) return fail(GSR_EINVAL, "%s", "bad sizes");
  if (P == 0) return last_launch();
  if (K == nullptr || bgs == nullptr || geom == nullptr || binning == nullptr || image == nullptr ||
      work == nullptr || dL_dcolor == nullptr || dL_dmeans2D == nullptr || dL_dcolors == nullptr ||
      dL_dopacity == nullptr || dL_dmeans3D == nullptr || radii == nullptr || means3D == nullptr)
    return fail(GSR_EINVAL, "%s", "null pointer argument");
  if (shs != nullptr && dL_dsh == nullptr) return fail(GSR_EINVAL, "%s", "dL_dsh required with SHs");
  if (cov3D_precomp == nullptr && (scales == nullptr || rotations == nullptr || dL_dscales == nullptr ||
                                   dL_drotations == nullptr))
    return fail(GSR_EINVAL, "%s", "scales/rotations and their gradients required");
  SetCams cams;
  if (set_cams(V, viewmatrices, projmatrices, campos, tanfovx, tanfovy, cams) != GSR_OK) return GSR_EINVAL;
  SegInfo inst;
  long long total = 0;
  if (inst_segments(V, K, inst, &total) != GSR_OK) return GSR_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  GeomState g = GeomState::carve((void*)geom, V, P, nullptr);
  const TilePack tp = set_tile_pack(P, width, height);
  BinningState b = BinningState::carve((void*)binning, V, total, inst.blk[V], !tp.packed, nullptr);
  // (the checkpoints, carved last, exist when the forward split: split_mode says so on the device)
  ImageState img = ImageState::carve((void*)image, V, width, height, nullptr, true);
  const int gx = div_up(width, GSR_TILE_X), gy = div_up(height, GSR_TILE_Y);
  const size_t HW = (size_t)width * height;
  const int tres = tile_sort_result(width, height);
  const uint32_t* sorted = tp.packed ? b.key[tres] : b.val[tres];
  GaussBackwardArgs a = shared_args(P, degree, M, means3D, scales, scale_modifier, rotations, shs, cov3D_precomp,
                                     dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales,
                                     dL_drotations);
  if (accumulate != 0 && cov3D_precomp == nullptr && dL_dcov3D == nullptr)
    return fail(GSR_EINVAL, "%s", "accumulate needs dL_dcov3D: it carries the running dL/dcov3D between calls");
  if (work_bytes < carry_bytes(P)) return fail(GSR_EINVAL, "%s", "backward work buffer too small");
  // the running dL/dcov3D: the caller's output when given, else the end of the work buffer (at a 256-byte
  // boundary whatever work_bytes is)
  const size_t avail = (work_bytes - carry_bytes(P)) & ~(size_t)255;
  float* carry = dL_dcov3D ? dL_dcov3D : (float*)((char*)work + avail);
  bool first = accumulate == 0;
  // groups of consecutive views whose gradient rows and records fit the work buffer
  for (int g0 = 0; g0 < V;) {
    int g1 = g0;
    long long rows = 0;
    while (g1 < V && (g1 == g0 || BackwardState::bytes_for(rows + K[g1], g1 + 1 - g0, P, two) <= avail))
      rows += K[g1++];
    if (BackwardState::bytes_for(rows, g1 - g0, P, two) > avail)
      return fail(GSR_EINVAL, "%s", "backward work buffer smaller than one view's gradient rows");
    BackwardState bw = BackwardState::carve(work, rows, P, two);
    RenderSet rs;
    rs.cbg = comp_bg ? comp_bg + (size_t)g0 * HW * 3 : nullptr;
    rs.comp = nullptr;
    rs.ccolor = color ? color + (size_t)g0 * 3 * HW : nullptr;
    rs.dcbg = dL_dbg ? dL_dbg + (size_t)g0 * HW * 3 : nullptr;
    rs.col2 = two ? colors2 : colors_override;
    rs.col2_rec = g.drange + 130;
    rs.out_col2 = nullptr;
    rs.dpix2 = two ? dL_dcolor2 + (size_t)g0 * 3 * HW : nullptr;
    rs.order = img.order;
    // a one-colour backward of the first colour replays split chunks when the forward wrote them.  The host passes
    // the checkpoints whenever the set's size allows a split (split_fits, no environment read here: ADVICE r05) and
    // the kernels follow the decision the forward recorded on the device (split_mode): the extra workgroups of a
    // forward that did not split return at once, and the checkpoints are read only after one that did
    rs.ckpt = !two && colors_override == nullptr && split_fits(V, (size_t)gx * gy) ? img.ckpt : nullptr;
    rs.split_mode = img.split_mode;
    rs.split_items = img.split_items;
    rs.split_cap = img.split_cap;
    rs.split_extra = split_extra(V, (size_t)gx * gy);
    rs.qkeys = tp.qmask ? b.key[tres] : nullptr;
    rs.qbytes = reinterpret_cast<uint8_t*>(b.key[tres ^ 1]);  // (valid when img.split_mode[1] says so)
    rs.V = g1 - g0;
    rs.ochunk = order_chunk(rs.V, gx, gy, false);
    rs.v0 = g0;
    rs.P = P;
    rs.W = width;
    rs.H = height;
    rs.gx = gx;
    rs.gy = gy;
    rs.gmask = tp.gmask;
    ViewGradArgs va;
    va.V = g1 - g0;
    va.v0 = g0;
    va.W = width;
    va.H = height;
    va.gx = gx;
    va.tiles = gx * gy;
    va.cut_in_lds = 0;
    va.items = 0;
    va.g = g;
    va.img = img;
    va.reach = bw.reach;
    va.grow = bw.grow;
    va.dmeans2D = dL_dmeans2D;
    va.vrec = bw.vrec;
    AccumArgs ab;
    ab.V = g1 - g0;
    ab.v0 = g0;
    ab.accumulate = first ? 0 : 1;
    ab.pad_ = 0;
    ab.reach = bw.reach;
    ab.vrec = bw.vrec;
    ab.dcov_carry = carry;
    ab.dcolors2 = two ? dL_dcolors2 : nullptr;
    for (int v = g0; v < g1; ++v) {
      if (bgs[v] == nullptr) return fail(GSR_EINVAL, "%s", "null background");
      rs.inst_start[v - g0] = inst.start[v];
      rs.row_start[v - g0] = inst.start[v] - inst.start[g0];
      rs.bg[v - g0] = bgs[v];
      va.row_start[v - g0] = rs.row_start[v - g0];
      va.cam[v - g0] = cams.c[v];
      ab.campos[v - g0] = cams.c[v].campos;
    }
    {
      PhaseScope ps(GSR_PHASE_RENDER_BWD, s);
      // the group's reach bits (set by k_render_bwd, read by the per-Gaussian backward)
      GSR_HIP_CHECK(hipMemsetAsync(bw.reach, 0, sizeof(unsigned long long) * (size_t)P, s));
      launch_render_backward(rs, g, sorted, img, dL_dcolor + (size_t)g0 * 3 * HW,
                             dL_ddepth ? dL_ddepth + (size_t)g0 * HW : nullptr,
                             dL_dalpha ? dL_dalpha + (size_t)g0 * HW : nullptr, bw, s);
    }
    {
      PhaseScope ps(GSR_PHASE_GAUSS_BWD, s);
      const bool last = g1 == V;
      if (last && chunks.n > 0) {
        // the final sums in Gaussian ranges, an event after each (the caller's reduction of a range starts
        // while the next range is computed)
        const int cs = grad_chunk_size(P, chunks.n);
        for (int c = 0; c < chunks.n; ++c) {
          GaussBackwardArgs ac = a;
          ac.g0 = c * cs < P ? c * cs : P;
          ac.g1 = (c + 1) * cs < P ? (c + 1) * cs : P;
          launch_gauss_backward(ac, va, ab, s);
          if (chunks.events[c] != nullptr) GSR_HIP_CHECK(hipEventRecord((hipEvent_t)chunks.events[c], s));
        }
      } else {
        launch_gauss_backward(a, va, ab, s);
      }
    }
    first = false;
    g0 = g1;
  }
  return last_launch();
}

int gsr_set_backward_chunks(int n_chunks, void* const* events) {
  if (n_chunks < 0 || n_chunks > GSR_GRAD_CHUNKS_MAX || (n_chunks > 0 && events == nullptr))
    return fail(GSR_EINVAL, "%s", "bad gradient chunk request");
  g_next_chunks = GradChunks{};
  g_next_chunks.n = n_chunks;
  for (int c = 0; c < n_chunks; ++c) g_next_chunks.events[c] = events[c];
  return GSR_OK;
}

int gsr_grad_chunk_range(int P, int n_chunks, int chunk, int* g0, int* g1) {
  if (P < 0 || n_chunks < 1 || n_chunks > GSR_GRAD_CHUNKS_MAX || chunk < 0 || chunk >= n_chunks || g0 == nullptr ||
      g1 == nullptr)
    return fail(GSR_EINVAL, "%s", "bad gradient chunk query");
  const int cs = grad_chunk_size(P, n_chunks);
  *g0 = chunk * cs < P ? chunk * cs : P;
  *g1 = (chunk + 1) * cs < P ? (chunk + 1) * cs : P;
  return GSR_OK;
}

int gsr_set_backward(int V, int P, int degree, int M, const int* K, int width, int height, const float* const* bgs,
                     const float* means3D, const float* scales, float scale_modifier, const float* rotations,
                     const float* shs, const float* cov3D_precomp, const float* const* viewmatrices,
                     const float* const* projmatrices, const float* const* campos, const float* tanfovx,
                     const float* tanfovy, const int* radii, const void* geom, const void* binning,
                     const void* image, const float* dL_dcolor, const float* dL_ddepth, const float* dL_dalpha,
                     float* dL_dmeans2D, float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D,
                     float* dL_dcov3D, float* dL_dsh, float* dL_dscales, float* dL_drotations, int accumulate,
                     void* work, size_t work_bytes, void* stream) {
  return set_backward(V, P, degree, M, K, width, height, bgs, means3D, scales, scale_modifier, rotations, shs,
                      cov3D_precomp, viewmatrices, projmatrices, campos, tanfovx, tanfovy, radii, geom, binning, image,
                      dL_dcolor, dL_ddepth, dL_dalpha, dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D,
                      dL_dsh, dL_dscales, dL_drotations, accumulate, work, work_bytes, nullptr, nullptr, nullptr,
                      stream);
}

int gsr_set_backward_composite(int V, int P, int degree, int M, const int* K, int width, int height,
                               const float* const* bgs, const float* means3D, const float* scales,
                               float scale_modifier, const float* rotations, const float* shs,
                               const float* cov3D_precomp, const float* const* viewmatrices,
                               const float* const* projmatrices, const float* const* campos, const float* tanfovx,
                               const float* tanfovy, const int* radii, const void* geom, const void* binning,
                               const void* image, const float* bg_images, const float* color,
                               const float* dL_drender, const float* dL_ddepth, const float* dL_dalpha,
                               float* dL_dbg, float* dL_dmeans2D, float* dL_dcolors, float* dL_dopacity,
                               float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscales,
                               float* dL_drotations, int accumulate, void* work, size_t work_bytes, void* stream) {
  // (bg_images NULL: the clamp alone; no dL_dbg then)
  if (color == nullptr) return fail(GSR_EINVAL, "%s", "null composite argument");
  if (bg_images == nullptr && dL_dbg != nullptr) return fail(GSR_EINVAL, "%s", "dL_dbg needs bg_images");
  return set_backward(V, P, degree, M, K, width, height, bgs, means3D, scales, scale_modifier, rotations, shs,
                      cov3D_precomp, viewmatrices, projmatrices, campos, tanfovx, tanfovy, radii, geom, binning, image,
                      dL_drender, dL_ddepth, dL_dalpha, dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D,
                      dL_dsh, dL_dscales, dL_drotations, accumulate, work, work_bytes, bg_images, color, dL_dbg,
                      stream);
}

// ---- one view (the reference's per-call interface): a set of one --------------------------

size_t gsr_geom_bytes(int P) { return gsr_set_geom_bytes(1, P); }
// P is not known here: size for the unpacked layout, which is never smaller than the packed one.
size_t gsr_binning_bytes(int K, int width, int height) {
  SegInfo seg;
  long long total = 0;
  if (K < 0 || inst_segments(1, &K, seg, &total) != GSR_OK) return 0;
  size_t b = 0;
  BinningState::carve(nullptr, 1, total, seg.blk[1], true, &b);
  return b;
}
size_t gsr_image_bytes(int width, int height) { return gsr_set_image_bytes(1, width, height); }
int gsr_set_backward_colors(int V, int P, const int* K, int width, int height, const float* const* bgs,
                            const float* means3D, const float* scales, float scale_modifier, const float* rotations,
                            const float* cov3D_precomp, const float* const* viewmatrices,
                            const float* const* projmatrices, const float* const* campos, const float* tanfovx,
                            const float* tanfovy, const int* radii, const void* geom, const void* binning,
                            const void* image, const float* colors, const float* dL_dcolor, float* dL_dmeans2D,
                            float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D,
                            float* dL_dscales, float* dL_drotations, int accumulate, void* work, size_t work_bytes,
                            void* stream) {
  if (colors == nullptr) return fail(GSR_EINVAL, "%s", "null colours");
  return set_backward(V, P, 0, 0, K, width, height, bgs, means3D, scales, scale_modifier, rotations, nullptr,
                      cov3D_precomp, viewmatrices, projmatrices, campos, tanfovx, tanfovy, radii, geom, binning, image,
                      dL_dcolor, nullptr, nullptr, dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, nullptr,
                      dL_dscales, dL_drotations, accumulate, work, work_bytes, nullptr, nullptr, nullptr, stream, colors);
}

size_t gsr_backward_bytes(int P, int K) { return gsr_set_backward_bytes(1, P, &K); }

size_t gsr_set_backward_two_colors_bytes(int V, int P, const int* K) {
  long long total = 0;
  for (int v = 0; v < V; ++v) total += K[v];
  return BackwardState::bytes_for(total, V, P, true) + carry_bytes(P);
}

int gsr_set_backward_two_colors(int V, int P, int degree, int M, const int* K, int width, int height,
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
                                int accumulate, void* work, size_t work_bytes, void* stream) {
  if (colors2 == nullptr || dL_dcolor2 == nullptr || dL_dcolors2 == nullptr)
    return fail(GSR_EINVAL, "%s", "null second colour argument");
  // (color without bg_images: the clamp alone; neither: no composite)
  if (bg_images != nullptr && color == nullptr) return fail(GSR_EINVAL, "%s", "composite needs the forward's color");
  if (bg_images == nullptr && dL_dbg != nullptr) return fail(GSR_EINVAL, "%s", "dL_dbg needs bg_images");
  return set_backward(V, P, degree, M, K, width, height, bgs, means3D, scales, scale_modifier, rotations, shs,
                      cov3D_precomp, viewmatrices, projmatrices, campos, tanfovx, tanfovy, radii, geom, binning, image,
                      dL_dcolor, dL_ddepth, dL_dalpha, dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D,
                      dL_dsh, dL_dscales, dL_drotations, accumulate, work, work_bytes, bg_images, color, dL_dbg,
                      stream, nullptr, colors2, dL_dcolor2, dL_dcolors2);
}

int gsr_forward_preprocess(int P, int degree, int M, const float* means3D, const float* scales,
                           float scale_modifier, const float* rotations, const float* opacities,
                           const float* shs, const float* colors_precomp, const float* cov3D_precomp,
                           const float* viewmatrix, const float* projmatrix, const float* campos,
                           int width, int height, float tanfovx, float tanfovy, int prefiltered,
                           int* radii, void* geom, void* stream) {
  return gsr_set_preprocess(1, P, degree, M, means3D, scales, scale_modifier, rotations, opacities, shs,
                            colors_precomp, cov3D_precomp, &viewmatrix, &projmatrix, &campos, &tanfovx, &tanfovy,
                            width, height, prefiltered, radii, geom, stream);
}

int gsr_num_rendered(const void* geom, int P, int* num_rendered, int* num_visible, void* stream) {
  return gsr_set_num_rendered(1, geom, P, num_rendered, num_visible, stream);
}

int gsr_forward_render(int P, int K, int width, int height, const float* bg, void* geom,
                       void* binning, void* image, float* out_color, float* out_depth,
                       float* out_alpha, void* stream) {
  if (K < 0) return fail(GSR_EINVAL, "%s", "bad sizes");
  return gsr_set_render(1, P, &K, width, height, &bg, geom, binning, image, out_color, out_depth, out_alpha, stream);
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
  if (K < 0) return fail(GSR_EINVAL, "%s", "bad sizes");
  return gsr_set_backward(1, P, degree, M, &K, width, height, &bg, means3D, scales, scale_modifier, rotations, shs,
                          cov3D_precomp, &viewmatrix, &projmatrix, &campos, &tanfovx, &tanfovy, radii, geom, binning,
                          image, dL_dcolor, dL_ddepth, dL_dalpha, dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D,
                          dL_dcov3D, dL_dsh, dL_dscales, dL_drotations, 0, work, gsr_backward_bytes(P, K), stream);
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

const char* gsr_profile_kernel(int phase) {
  return phase == GSR_PHASE_RENDER_FWD ? blend_kernel_name(0) : phase == GSR_PHASE_RENDER_BWD ? blend_kernel_name(1) : "";
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

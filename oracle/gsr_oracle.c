/*
 * gsr_oracle.c — CPU restatement of the reference rasterizer algorithm.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this library, and only as the checker / CPU baseline — never as the product path.
 *
 * What it restates:
 *   the external CUDA package `diff_gaussian_rasterization` (ashawkey 4-output fork, unpinned;
 *   README.md:17,28 of the reference), which lizhiqi49/threestudio-3dgs calls from
 *   renderer/diff_gaussian_rasterizer*.py (e.g. renderer/diff_gaussian_rasterizer_background.py:119-128).
 *   Its source is not in /root/reference and cannot be fetched; the algorithm below is the
 *   published upstream one (cuda_rasterizer/{forward,backward,auxiliary}) restated as plain C:
 *     preprocess   — in_frustum (view z <= 0.2 culls), computeCov3D, computeCov2D (1.3 tan-fov clamp,
 *                    +0.3 dilation), conic, radius = ceil(3 sqrt(max eigen)) with the 0.1 floor,
 *                    ndc2Pix in double, getRect on 16x16 tiles, computeColorFromSH (+0.5, clamp 0)
 *     binning      — instances ordered by (tile, depth, Gaussian index) == the reference's stable
 *                    radix sort of (tile << 32 | depth bits) keys over index-ordered instances
 *     render fwd   — front-to-back blend, alpha = min(0.99, o e^power), skip alpha < 1/255, stop when
 *                    T (1 - alpha) < 1e-4; color + T bg, depth = sum z alpha T, alpha = 1 - T
 *     render bwd   — back-to-front replay with T recovery, suffix accumulators, background term
 *     per-Gaussian — computeCov2DCUDA, preprocessCUDA (projection, depth, SH, cov3D) backward
 *   Reference pure-torch twins pinned by golden vectors (tests/golden/make_golden.py):
 *     eval_sh + C0..C3            geometry/sugar.py:743-830
 *     build_rotation/scaling      geometry/gaussian_base.py:99-134 (cov3D = L L^T, :234-238)
 *     getProjectionMatrix         utils/sugar_utils.py:809-829 (camera construction, :880-896)
 *   Parity of the full rasterizer is UNPINNED by the reference itself: it holds no rasterizer code,
 *   tests or fixtures.  The chain of evidence is documented in DESIGN.md.
 *
 * Built twice from this file: REAL=float (symbols *_f32, fp32 mirror of the kernels' op order,
 * fmaf where the kernels use fmaf) and REAL=double (symbols *_f64).  Compiled with
 * -ffp-contract=off so the written order is the evaluated order.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef ORACLE_F64
typedef double real;
#define FN(name) name##_f64
#define EXPR exp
#define SQRTR sqrt
#define FMAR fma
#define CEILR ceil
#elif defined(ORACLE_F32C)
/* fp32 with the compiler's multiply-add contraction (built -ffp-contract=fast -mfma): another faithful fp32
 * evaluation, as nvcc's default --fmad=true compiles the reference's CUDA; tests/gsr_testutil.py uses it to
 * measure how far faithful fp32 evaluations of the reference algorithm are from each other, row by row */
typedef float real;
#define FN(name) name##_f32c
#define EXPR expf
#define SQRTR sqrtf
#define FMAR fmaf
#define CEILR ceilf
#else
typedef float real;
#define FN(name) name##_f32
#define EXPR expf
#define SQRTR sqrtf
#define FMAR fmaf
#define CEILR ceilf
#endif

#define RL(x) ((real)(x))
#define TILE 16

static const real SH_C0 = RL(0.28209479177387814);
static const real SH_C1 = RL(0.4886025119029199);
static const real SH_C2[5] = {RL(1.0925484305920792), RL(-1.0925484305920792), RL(0.31539156525252005),
                              RL(-1.0925484305920792), RL(0.5462742152960396)};
static const real SH_C3[7] = {RL(-0.5900435899266435), RL(2.890611442640554), RL(-0.4570457994644658),
                              RL(0.3731763325901154), RL(-0.4570457994644658), RL(1.445305721320277),
                              RL(-0.5900435899266435)};

static real rmin(real a, real b) { return a < b ? a : b; }
static real rmax(real a, real b) { return a > b ? a : b; }
static int imin(int a, int b) { return a < b ? a : b; }
static int imax(int a, int b) { return a > b ? a : b; }

/* ------------------------------------------------------------------------------------------ */
/* pieces (exported for golden-vector checks)                                                  */

/* transformPoint4x3 / 4x4: m[0] p.x + m[4] p.y + m[8] p.z + m[12] evaluated as the left-to-right fma
 * chain a contracting compiler emits (the kernels use the same chain, csrc/gsr_common.h xform_row), so
 * the fp32 view depths — which decide the order of nearly coincident Gaussians — agree bit for bit. */
static real xrow(real m0, real m1, real m2, real m3, const real* p) {
  return FMAR(m2, p[2], FMAR(m1, p[1], m0 * p[0])) + m3;
}
static void xform4x3(const real* p, const real* m, real* o) {
  o[0] = xrow(m[0], m[4], m[8], m[12], p);
  o[1] = xrow(m[1], m[5], m[9], m[13], p);
  o[2] = xrow(m[2], m[6], m[10], m[14], p);
}
static void xform4x4(const real* p, const real* m, real* o) {
  xform4x3(p, m, o);
  o[3] = xrow(m[3], m[7], m[11], m[15], p);
}

/* R[c][r] exactly as the kernels build it (glm column-major of the reference) */
static void rot_from_quat(const real* q, real R[3][3]) {
  const real r = q[0], x = q[1], y = q[2], z = q[3];
  R[0][0] = RL(1) - RL(2) * (y * y + z * z);
  R[0][1] = RL(2) * (x * y - r * z);
  R[0][2] = RL(2) * (x * z + r * y);
  R[1][0] = RL(2) * (x * y + r * z);
  R[1][1] = RL(1) - RL(2) * (x * x + z * z);
  R[1][2] = RL(2) * (y * z - r * x);
  R[2][0] = RL(2) * (x * z - r * y);
  R[2][1] = RL(2) * (y * z + r * x);
  R[2][2] = RL(1) - RL(2) * (x * x + y * y);
}

static void cov3d(const real* scale, real mod, const real* q, real* cov) {
  real R[3][3], M[3][3];
  const real s[3] = {mod * scale[0], mod * scale[1], mod * scale[2]};
  rot_from_quat(q, R);
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) M[c][r] = s[r] * R[c][r];
#define SIG(c, r) (M[r][0] * M[c][0] + M[r][1] * M[c][1] + M[r][2] * M[c][2])
  cov[0] = SIG(0, 0);
  cov[1] = SIG(0, 1);
  cov[2] = SIG(0, 2);
  cov[3] = SIG(1, 1);
  cov[4] = SIG(1, 2);
  cov[5] = SIG(2, 2);
#undef SIG
}

typedef struct {
  real t[3];
  real txtz, tytz, limx, limy;
  real T[2][3];
  real W[3][3];
} cov2d_state;

static void cov2d(const real* mean, real fx, real fy, real tanx, real tany, const real* c3, const real* view,
                  cov2d_state* st, real* out) {
  real t[3];
  xform4x3(mean, view, t);
  st->limx = RL(1.3) * tanx;
  st->limy = RL(1.3) * tany;
  st->txtz = t[0] / t[2];
  st->tytz = t[1] / t[2];
  t[0] = rmin(st->limx, rmax(-st->limx, st->txtz)) * t[2];
  t[1] = rmin(st->limy, rmax(-st->limy, st->tytz)) * t[2];
  memcpy(st->t, t, sizeof(t));
  const real J00 = fx / t[2], J02 = -(fx * t[0]) / (t[2] * t[2]);
  const real J11 = fy / t[2], J12 = -(fy * t[1]) / (t[2] * t[2]);
  st->W[0][0] = view[0]; st->W[0][1] = view[4]; st->W[0][2] = view[8];
  st->W[1][0] = view[1]; st->W[1][1] = view[5]; st->W[1][2] = view[9];
  st->W[2][0] = view[2]; st->W[2][1] = view[6]; st->W[2][2] = view[10];
  for (int r = 0; r < 3; ++r) {
    st->T[0][r] = st->W[0][r] * J00 + st->W[2][r] * J02;
    st->T[1][r] = st->W[1][r] * J11 + st->W[2][r] * J12;
  }
  const real V[3][3] = {{c3[0], c3[1], c3[2]}, {c3[1], c3[3], c3[4]}, {c3[2], c3[4], c3[5]}};
  real A[3][2];
  for (int k = 0; k < 3; ++k)
    for (int r = 0; r < 2; ++r) A[k][r] = st->T[r][0] * V[k][0] + st->T[r][1] * V[k][1] + st->T[r][2] * V[k][2];
  real c00 = A[0][0] * st->T[0][0] + A[1][0] * st->T[0][1] + A[2][0] * st->T[0][2];
  real c01 = A[0][1] * st->T[0][0] + A[1][1] * st->T[0][1] + A[2][1] * st->T[0][2];
  real c11 = A[0][1] * st->T[1][0] + A[1][1] * st->T[1][1] + A[2][1] * st->T[1][2];
  out[0] = c00 + RL(0.3);
  out[1] = c01;
  out[2] = c11 + RL(0.3);
}

/* basis values (16) and their partials w.r.t. the normalised direction */
static void sh_basis(int deg, real x, real y, real z, real* b, real* bx, real* by, real* bz) {
  for (int k = 0; k < 16; ++k) b[k] = bx[k] = by[k] = bz[k] = 0;
  b[0] = SH_C0;
  if (deg > 0) {
    b[1] = -SH_C1 * y; b[2] = SH_C1 * z; b[3] = -SH_C1 * x;
    by[1] = -SH_C1; bz[2] = SH_C1; bx[3] = -SH_C1;
    if (deg > 1) {
      const real xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
      b[4] = SH_C2[0] * xy; b[5] = SH_C2[1] * yz; b[6] = SH_C2[2] * (RL(2) * zz - xx - yy);
      b[7] = SH_C2[3] * xz; b[8] = SH_C2[4] * (xx - yy);
      bx[4] = SH_C2[0] * y; by[4] = SH_C2[0] * x;
      by[5] = SH_C2[1] * z; bz[5] = SH_C2[1] * y;
      bx[6] = SH_C2[2] * RL(2) * -x; by[6] = SH_C2[2] * RL(2) * -y; bz[6] = SH_C2[2] * RL(2) * RL(2) * z;
      bx[7] = SH_C2[3] * z; bz[7] = SH_C2[3] * x;
      bx[8] = SH_C2[4] * RL(2) * x; by[8] = SH_C2[4] * RL(2) * -y;
      if (deg > 2) {
        b[9] = SH_C3[0] * y * (RL(3) * xx - yy);
        b[10] = SH_C3[1] * xy * z;
        b[11] = SH_C3[2] * y * (RL(4) * zz - xx - yy);
        b[12] = SH_C3[3] * z * (RL(2) * zz - RL(3) * xx - RL(3) * yy);
        b[13] = SH_C3[4] * x * (RL(4) * zz - xx - yy);
        b[14] = SH_C3[5] * z * (xx - yy);
        b[15] = SH_C3[6] * x * (xx - RL(3) * yy);
        bx[9] = SH_C3[0] * RL(3) * RL(2) * xy; by[9] = SH_C3[0] * RL(3) * (xx - yy);
        bx[10] = SH_C3[1] * yz; by[10] = SH_C3[1] * xz; bz[10] = SH_C3[1] * xy;
        bx[11] = SH_C3[2] * RL(-2) * xy; by[11] = SH_C3[2] * (RL(-3) * yy + RL(4) * zz - xx);
        bz[11] = SH_C3[2] * RL(4) * RL(2) * yz;
        bx[12] = SH_C3[3] * RL(-3) * RL(2) * xz; by[12] = SH_C3[3] * RL(-3) * RL(2) * yz;
        bz[12] = SH_C3[3] * RL(3) * (RL(2) * zz - xx - yy);
        bx[13] = SH_C3[4] * (RL(-3) * xx + RL(4) * zz - yy); by[13] = SH_C3[4] * RL(-2) * xy;
        bz[13] = SH_C3[4] * RL(4) * RL(2) * xz;
        bx[14] = SH_C3[5] * RL(2) * xz; by[14] = SH_C3[5] * RL(-2) * yz; bz[14] = SH_C3[5] * (xx - yy);
        bx[15] = SH_C3[6] * RL(3) * (xx - yy); by[15] = SH_C3[6] * RL(-3) * RL(2) * xy;
      }
    }
  }
}

/* SH -> RGB (+0.5, clamp >= 0).  sh: (M,3).  *clamp gets bit c set when channel c < 0. */
static void sh_rgb(int deg, int M, const real* sh, const real* pos, const real* campos, real* rgb, uint32_t* clamp) {
  real d[3] = {pos[0] - campos[0], pos[1] - campos[1], pos[2] - campos[2]};
  const real len = SQRTR(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  d[0] = d[0] / len; d[1] = d[1] / len; d[2] = d[2] / len;
  real b[16], bx[16], by[16], bz[16];
  sh_basis(deg, d[0], d[1], d[2], b, bx, by, bz);
  const int nc = (deg + 1) * (deg + 1);
  uint32_t cl = 0;
  for (int c = 0; c < 3; ++c) {
    real acc = b[0] * sh[c];
    for (int k = 1; k < nc && k < M; ++k) acc = acc + b[k] * sh[3 * k + c];
    acc = acc + RL(0.5);
    if (acc < 0) cl |= 1u << c;
    rgb[c] = rmax(acc, 0);
  }
  *clamp = cl;
}

static real ndc2pix(real v, int S) { return (real)((((double)v + 1.0) * (double)S - 1.0) * 0.5); }

static real gauss_power(real a, real b, real c, real dx, real dy) {
  const real q = FMAR(c * dy, dy, (a * dx) * dx);
  return FMAR(RL(-0.5), q, -((b * dx) * dy));
}

/* exported piece wrappers (inputs/outputs as double for the golden tests) */
void FN(oracle_eval_sh)(int n, int deg, int M, const double* sh, const double* pos, const double* campos, double* out) {
  for (int i = 0; i < n; ++i) {
    real s[48], p[3], cp[3], rgb[3];
    uint32_t cl;
    for (int k = 0; k < 3 * M && k < 48; ++k) s[k] = (real)sh[(size_t)i * 3 * M + k];
    for (int k = 0; k < 3; ++k) { p[k] = (real)pos[3 * i + k]; cp[k] = (real)campos[k]; }
    sh_rgb(deg, M, s, p, cp, rgb, &cl);
    /* report the unclamped value (minus the 0.5 offset) so it matches eval_sh exactly */
    real d[3] = {p[0] - cp[0], p[1] - cp[1], p[2] - cp[2]};
    const real len = SQRTR(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    real b[16], bx[16], by[16], bz[16];
    sh_basis(deg, d[0] / len, d[1] / len, d[2] / len, b, bx, by, bz);
    for (int c = 0; c < 3; ++c) {
      real acc = b[0] * s[c];
      for (int k = 1; k < (deg + 1) * (deg + 1) && k < M; ++k) acc = acc + b[k] * s[3 * k + c];
      out[3 * i + c] = (double)acc;
    }
    (void)rgb;
  }
}

void FN(oracle_cov3d)(int n, const double* scales, double mod, const double* rots, double* out) {
  for (int i = 0; i < n; ++i) {
    real s[3], q[4], c[6];
    for (int k = 0; k < 3; ++k) s[k] = (real)scales[3 * i + k];
    for (int k = 0; k < 4; ++k) q[k] = (real)rots[4 * i + k];
    cov3d(s, (real)mod, q, c);
    for (int k = 0; k < 6; ++k) out[6 * i + k] = (double)c[k];
  }
}

/* ------------------------------------------------------------------------------------------ */
/* full rasterizer                                                                             */

typedef struct {
  int P, deg, M, W, H, gx, gy;
  const float *means, *scales, *rots, *opac, *shs, *colors, *cov3p, *viewf, *projf, *camposf, *bgf;
  real mod, tanx, tany, fx, fy;
  real view[16], proj[16], campos[3], bg[3];
} ctx_t;

typedef struct {
  int radius, tiles, xmin, ymin, xmax, ymax;
  real px, py, ca, cb, cc, op, depth, rgb[3];
  real rad3; /* 3 sqrt(max eigenvalue) before the ceil (radius adjudication), -1 if culled earlier */
  uint32_t clamp;
} gstate;

typedef struct {
  uint32_t tile;
  real depth;
  uint32_t g;
} inst_t;

static int inst_cmp(const void* a, const void* b) {
  const inst_t* x = (const inst_t*)a;
  const inst_t* y = (const inst_t*)b;
  if (x->tile != y->tile) return x->tile < y->tile ? -1 : 1;
  if (x->depth != y->depth) return x->depth < y->depth ? -1 : 1;
  return x->g < y->g ? -1 : (x->g > y->g ? 1 : 0);
}

static void load_vec(const float* src, real* dst, int n) { for (int i = 0; i < n; ++i) dst[i] = (real)src[i]; }

static void get_cov3(const ctx_t* c, int i, real* cov) {
  if (c->cov3p) {
    for (int k = 0; k < 6; ++k) cov[k] = (real)c->cov3p[6 * i + k];
  } else {
    real s[3], q[4];
    load_vec(c->scales + 3 * i, s, 3);
    load_vec(c->rots + 4 * i, q, 4);
    cov3d(s, c->mod, q, cov);
  }
}

static void preprocess(const ctx_t* c, int i, gstate* g, int* radii) {
  memset(g, 0, sizeof(*g));
  g->rad3 = -1;
  radii[i] = 0;
  real p[3];
  load_vec(c->means + 3 * i, p, 3);
  real pv[3], ph[4];
  xform4x3(p, c->view, pv);
  if (pv[2] <= RL(0.2)) return;
  xform4x4(p, c->proj, ph);
  const real pw = RL(1) / (ph[3] + RL(0.0000001));
  const real pp[2] = {ph[0] * pw, ph[1] * pw};
  real cov3[6], cv[3];
  get_cov3(c, i, cov3);
  cov2d_state st;
  cov2d(p, c->fx, c->fy, c->tanx, c->tany, cov3, c->view, &st, cv);
  const real det = cv[0] * cv[2] - cv[1] * cv[1];
  if (det == 0) return;
  const real det_inv = RL(1) / det;
  const real mid = RL(0.5) * (cv[0] + cv[2]);
  const real l1 = mid + SQRTR(rmax(RL(0.1), mid * mid - det));
  const real l2 = mid - SQRTR(rmax(RL(0.1), mid * mid - det));
  const real rad = CEILR(RL(3) * SQRTR(rmax(l1, l2)));
  const real px = ndc2pix(pp[0], c->W), py = ndc2pix(pp[1], c->H);
  g->rad3 = RL(3) * SQRTR(rmax(l1, l2));
  g->px = px; g->py = py;
  const int r = (int)rad;
  const int xmin = imin(c->gx, imax(0, (int)((px - r) / TILE)));
  const int ymin = imin(c->gy, imax(0, (int)((py - r) / TILE)));
  const int xmax = imin(c->gx, imax(0, (int)((px + r + TILE - 1) / TILE)));
  const int ymax = imin(c->gy, imax(0, (int)((py + r + TILE - 1) / TILE)));
  if ((xmax - xmin) * (ymax - ymin) == 0) return;
  if (c->colors) {
    load_vec(c->colors + 3 * i, g->rgb, 3);
  } else {
    real sh[48];
    const int n = c->M < 16 ? c->M : 16;
    load_vec(c->shs + (size_t)3 * c->M * i, sh, 3 * n);
    sh_rgb(c->deg, n, sh, p, c->campos, g->rgb, &g->clamp);
  }
  g->radius = r;
  g->tiles = (xmax - xmin) * (ymax - ymin);
  g->xmin = xmin; g->ymin = ymin; g->xmax = xmax; g->ymax = ymax;
  g->px = px; g->py = py;
  g->ca = cv[2] * det_inv; g->cb = -cv[1] * det_inv; g->cc = cv[0] * det_inv;
  g->op = (real)c->opac[i];
  g->depth = pv[2];
  radii[i] = r;
}

typedef struct {
  gstate* gs;
  inst_t* inst;
  uint32_t* range;  /* [tiles][2] */
  real* final_T;
  uint32_t* n_contrib;
  long K;
} fwd_t;

static int setup(ctx_t* c, int P, int deg, int M, const float* means, const float* scales, float mod,
                 const float* rots, const float* opac, const float* shs, const float* colors,
                 const float* cov3p, const float* view, const float* proj, const float* campos, int W,
                 int H, float tanx, float tany, const float* bg) {
  memset(c, 0, sizeof(*c));
  c->P = P; c->M = M; c->W = W; c->H = H;
  int dm = (int)lround(sqrt((double)(M > 0 ? M : 1))) - 1;
  c->deg = deg < dm ? deg : dm;
  if (c->deg < 0) c->deg = 0;
  if (c->deg > 3) c->deg = 3;
  c->gx = (W + TILE - 1) / TILE; c->gy = (H + TILE - 1) / TILE;
  c->means = means; c->scales = scales; c->rots = rots; c->opac = opac; c->shs = shs;
  c->colors = colors; c->cov3p = cov3p;
  c->mod = (real)mod; c->tanx = (real)tanx; c->tany = (real)tany;
  c->fy = (real)((float)H / (2.0f * tany));
  c->fx = (real)((float)W / (2.0f * tanx));
  load_vec(view, c->view, 16); load_vec(proj, c->proj, 16); load_vec(campos, c->campos, 3); load_vec(bg, c->bg, 3);
  return 0;
}

/* pair statistics of the last forward (diagnostics): [0] pairs iterated, [1] pairs blended,
 * [2] pixels inside the image */
static long g_stats[4];

/* Worker threads of the forward / backward loops (OpenMP).  1 (the default, what the parity tests use)
 * runs the serial loops in the order written; n > 1 is for the CPU baseline timing (bench.py): the
 * tiles are blended in parallel and the backward sums per-thread partial gradients, so the gradients
 * differ from the serial build in the last bits (summation order).  Shared by the fp32 / fp64 builds. */
#ifdef _OPENMP
#include <omp.h>
#endif
#if !defined(ORACLE_F64) && !defined(ORACLE_F32C)
int g_oracle_threads = 1;
void oracle_set_threads(int n) { g_oracle_threads = n > 0 ? n : 1; }
int oracle_get_threads(void) { return g_oracle_threads; }
/* Order in which the backward visits the pixels, i.e. in which every per-Gaussian gradient sum adds its
 * per-pixel terms: 0 = tiles and pixels in raster order; 1 = both reversed.  The reference accumulates these
 * sums with float atomicAdd from concurrently running pixel threads (BACKWARD::renderCUDA [EXT]), so its
 * summation order is unspecified and changes from run to run: order 1 is another equally faithful run of it
 * (tests/gsr_testutil.py uses the pair to measure how far the reference is from itself, row by row). */
int g_oracle_order = 0;
void oracle_set_order(int order) { g_oracle_order = order; }
/* DIAGNOSTIC ONLY (scripts/parity_sources.py; never set by a parity test): evaluate pieces of the per-pixel
 * arithmetic the way the HIP blends do, to attribute their differences from this restatement.
 *   1  exponent: conic pre-multiplied by -log2(e)/2, -log2(e) (rounded), exp2 (csrc/gsr_common.h gauss_power2)
 *   2  transmittance recovery T * (1 / (1 - alpha)) instead of T / (1 - alpha)
 *   4  dL/dalpha from one scalar S = sum_ch accum_ch dL/dpix_ch over colour and alpha, the depth channel as
 *      (depth - accumulated depth) dL/ddepth (csrc/gsr_render.hip k_render_bwd replay)
 *   8  dL/dmean2D from the first moments of u = G dL/dalpha and the pre-multiplied conic, as the blend's
 *      flush forms it: (o / log2 e) (W/2) (2 A m1 + B m2), A = -log2(e)/2 a, B = -log2(e) b (rounded) */
int g_oracle_variant = 0;
void oracle_set_variant(int v) { g_oracle_variant = v; }
#else
extern int g_oracle_threads;
extern int g_oracle_order;
extern int g_oracle_variant;
#endif
/* the exponent (and G) under the diagnostic variant bit 1: returns the exponent's sign test value, G in *G */
static real blend_G(const gstate* g, real dx, real dy, real* G) {
  if (g_oracle_variant & 1) {
    const float A = -0.72134752044448170f * (float)g->ca, B = -1.4426950408889634f * (float)g->cb,
                C = -0.72134752044448170f * (float)g->cc;
    const float p2 = fmaf((float)dx, fmaf(A, (float)dx, B * (float)dy), (C * (float)dy) * (float)dy);
    *G = (real)exp2f(p2);
    return (real)p2;
  }
  const real power = gauss_power(g->ca, g->cb, g->cc, dx, dy);
  *G = EXPR(power);
  return power;
}
void FN(oracle_last_stats)(long* out) { for (int i = 0; i < 4; ++i) out[i] = g_stats[i]; }

static void forward_core(const ctx_t* c, int* radii, fwd_t* f, real* out_color, real* out_depth, real* out_alpha) {
  g_stats[0] = g_stats[1] = g_stats[2] = g_stats[3] = 0;
  const int P = c->P, W = c->W, H = c->H, nt = c->gx * c->gy;
  f->gs = (gstate*)calloc((size_t)(P > 0 ? P : 1), sizeof(gstate));
  long K = 0;
  const int nth = g_oracle_threads;
#pragma omp parallel for num_threads(nth) schedule(static) reduction(+ : K) if (nth > 1)
  for (int i = 0; i < P; ++i) {
    preprocess(c, i, &f->gs[i], radii);
    K += f->gs[i].tiles;
  }
  f->K = K;
  f->inst = (inst_t*)malloc(sizeof(inst_t) * (size_t)(K > 0 ? K : 1));
  long o = 0;
  for (int i = 0; i < P; ++i) {
    const gstate* g = &f->gs[i];
    for (int y = g->ymin; y < g->ymax; ++y)
      for (int x = g->xmin; x < g->xmax; ++x) {
        f->inst[o].tile = (uint32_t)(y * c->gx + x);
        f->inst[o].depth = g->depth;
        f->inst[o].g = (uint32_t)i;
        ++o;
      }
  }
  qsort(f->inst, (size_t)K, sizeof(inst_t), inst_cmp);
  f->range = (uint32_t*)calloc((size_t)2 * nt, sizeof(uint32_t));
  for (long p = 0; p < K; ++p) {
    const uint32_t t = f->inst[p].tile;
    if (p == 0 || f->inst[p - 1].tile != t) f->range[2 * t] = (uint32_t)p;
    if (p == K - 1 || f->inst[p + 1].tile != t) f->range[2 * t + 1] = (uint32_t)(p + 1);
  }
  f->final_T = (real*)calloc((size_t)W * H, sizeof(real));
  f->n_contrib = (uint32_t*)calloc((size_t)W * H, sizeof(uint32_t));
  const size_t HW = (size_t)W * H;
  long st0 = 0, st1 = 0, st2 = 0;
#pragma omp parallel for num_threads(nth) schedule(dynamic, 1) reduction(+ : st0, st1, st2) if (nth > 1)
  for (int tt = 0; tt < nt; ++tt) {
      const int ty = tt / c->gx, tx = tt - ty * c->gx;
      const uint32_t t = (uint32_t)tt;
      const uint32_t s = f->range[2 * t], e = f->range[2 * t + 1];
      for (int ly = 0; ly < TILE; ++ly)
        for (int lx = 0; lx < TILE; ++lx) {
          const int px = tx * TILE + lx, py = ty * TILE + ly;
          if (px >= W || py >= H) continue;
          real T = 1, C[3] = {0, 0, 0}, D = 0;
          uint32_t contributor = 0, last = 0;
          st2++;
          for (uint32_t p = s; p < e; ++p) {
            ++contributor;
            st0++;
            const gstate* g = &f->gs[f->inst[p].g];
            const real dx = g->px - (real)px, dy = g->py - (real)py;
            real Gv;
            const real power = blend_G(g, dx, dy, &Gv);
            if (power > 0) continue;
            const real alpha = rmin(RL(0.99), g->op * Gv);
            if (alpha < RL(1.0) / RL(255.0)) continue;
            const real test_T = T * (RL(1) - alpha);
            if (test_T < RL(0.0001)) break;
            for (int ch = 0; ch < 3; ++ch) C[ch] += g->rgb[ch] * alpha * T;
            D += g->depth * alpha * T;
            T = test_T;
            last = contributor;
            st1++;
          }
          const size_t pid = (size_t)py * W + px;
          f->final_T[pid] = T;
          f->n_contrib[pid] = last;
          if (out_color)
            for (int ch = 0; ch < 3; ++ch) out_color[ch * HW + pid] = C[ch] + T * c->bg[ch];
          if (out_depth) out_depth[pid] = D;
          if (out_alpha) out_alpha[pid] = RL(1) - T;
        }
  }
  g_stats[0] = st0; g_stats[1] = st1; g_stats[2] = st2;
}

static void free_fwd(fwd_t* f) {
  free(f->gs); free(f->inst); free(f->range); free(f->final_T); free(f->n_contrib);
}

/* Forward.  Outputs are REAL arrays: color (3,H,W), depth (H,W), alpha (H,W); radii int (P).
 * Returns K (number of instances). */
long FN(oracle_forward)(int P, int deg, int M, const float* means, const float* scales, float mod,
                        const float* rots, const float* opac, const float* shs, const float* colors,
                        const float* cov3p, const float* view, const float* proj, const float* campos,
                        int W, int H, float tanx, float tany, const float* bg, real* out_color,
                        real* out_depth, real* out_alpha, int* radii) {
  ctx_t c;
  setup(&c, P, deg, M, means, scales, mod, rots, opac, shs, colors, cov3p, view, proj, campos, W, H, tanx, tany, bg);
  fwd_t f;
  forward_core(&c, radii, &f, out_color, out_depth, out_alpha);
  const long K = f.K;
  free_fwd(&f);
  return K;
}

/* Per-Gaussian preprocess values for the parity tests (no blending): aux (P, 16) doubles = (pixel x,
 * pixel y, 3 sqrt(max eigenvalue) before the ceil, rectangle tiles, conic a, b, c, opacity, view depth,
 * r, g, b, tile rect xmin, ymin, xmax, ymax); rad3 = -1 for Gaussians culled before the radius (near
 * plane, singular cov2D); fields after px, py stay 0 for culled Gaussians.  With the fp64 build, a GPU radius that differs
 * from the fp32 oracle's is a legitimate fp32 rounding flip only when rad3 lies within a few ulp of an
 * integer; the rectangle tile count of any radius follows from (px, py) with the getRect formula. */
void FN(oracle_gauss_aux)(int P, int deg, int M, const float* means, const float* scales, float mod,
                          const float* rots, const float* opac, const float* shs, const float* colors,
                          const float* cov3p, const float* view, const float* proj, const float* campos,
                          int W, int H, float tanx, float tany, double* aux) {
  ctx_t c;
  const float bg0[3] = {0, 0, 0};
  setup(&c, P, deg, M, means, scales, mod, rots, opac, shs, colors, cov3p, view, proj, campos, W, H, tanx, tany, bg0);
  int* radii = (int*)calloc((size_t)(P > 0 ? P : 1), sizeof(int));
  for (int i = 0; i < P; ++i) {
    gstate g;
    preprocess(&c, i, &g, radii);
    double* o = aux + 16 * (size_t)i;
    o[0] = (double)g.px; o[1] = (double)g.py; o[2] = (double)g.rad3; o[3] = (double)g.tiles;
    o[4] = (double)g.ca; o[5] = (double)g.cb; o[6] = (double)g.cc; o[7] = (double)g.op; o[8] = (double)g.depth;
    o[9] = (double)g.rgb[0]; o[10] = (double)g.rgb[1]; o[11] = (double)g.rgb[2];
    o[12] = g.xmin; o[13] = g.ymin; o[14] = g.xmax; o[15] = g.ymax;
  }
  free(radii);
}

/* Backward (re-runs the forward).  Gradient outputs (REAL): dmeans2D (P,3), dcolors (P,3),
 * dopacity (P), dmeans3D (P,3), dcov3D (P,6), dsh (P,M,3) [if shs], dscales (P,3), drots (P,4)
 * [if scales].  dL_ddepth / dL_dalpha may be NULL. */
void FN(oracle_backward)(int P, int deg, int M, const float* means, const float* scales, float mod,
                         const float* rots, const float* opac, const float* shs, const float* colors,
                         const float* cov3p, const float* view, const float* proj, const float* campos,
                         int W, int H, float tanx, float tany, const float* bg, const float* dL_dcolor,
                         const float* dL_ddepth, const float* dL_dalpha, real* dmeans2D, real* dcolors,
                         real* dopacity, real* dmeans3D, real* dcov3D, real* dsh, real* dscales,
                         real* drots) {
  ctx_t c;
  setup(&c, P, deg, M, means, scales, mod, rots, opac, shs, colors, cov3p, view, proj, campos, W, H, tanx, tany, bg);
  int* radii = (int*)calloc((size_t)(P > 0 ? P : 1), sizeof(int));
  fwd_t f;
  forward_core(&c, radii, &f, NULL, NULL, NULL);
  const size_t HW = (size_t)W * H;
  /* per-Gaussian accumulators: m2x, m2y, ca, cb, cc, op, r, g, b, depth (one set per worker thread) */
  const int nth = g_oracle_threads;
  const size_t nacc = (size_t)10 * (P > 0 ? P : 1);
  real* acc_all = (real*)calloc(nacc * (size_t)nth, sizeof(real));
  real* acc = acc_all;
  const real ddelx_dx = RL(0.5) * W, ddely_dy = RL(0.5) * H;
  const int ntiles = c.gx * c.gy;
#pragma omp parallel for num_threads(nth) schedule(dynamic, 1) if (nth > 1)
  for (int tt0 = 0; tt0 < ntiles; ++tt0) {
      const int rev = g_oracle_order == 1;
      const int tt = rev ? ntiles - 1 - tt0 : tt0;
      const int ty = tt / c.gx, tx = tt - ty * c.gx;
      int me = 0;
#ifdef _OPENMP
      if (nth > 1) me = omp_get_thread_num();
#endif
      real* tacc = acc_all + nacc * (size_t)me;
      const uint32_t t = (uint32_t)tt;
      const uint32_t s = f.range[2 * t];
      for (int ly0 = 0; ly0 < TILE; ++ly0)
        for (int lx0 = 0; lx0 < TILE; ++lx0) {
          const int ly = rev ? TILE - 1 - ly0 : ly0, lx = rev ? TILE - 1 - lx0 : lx0;
          const int px = tx * TILE + lx, py = ty * TILE + ly;
          if (px >= W || py >= H) continue;
          const size_t pid = (size_t)py * W + px;
          const real T_final = f.final_T[pid];
          real T = T_final;
          const uint32_t last = f.n_contrib[pid];
          const real dpix[3] = {(real)dL_dcolor[pid], (real)dL_dcolor[HW + pid], (real)dL_dcolor[2 * HW + pid]};
          const real dpd = dL_ddepth ? (real)dL_ddepth[pid] : 0;
          const real dpa = dL_dalpha ? (real)dL_dalpha[pid] : 0;
          const real bg_dot = c.bg[0] * dpix[0] + c.bg[1] * dpix[1] + c.bg[2] * dpix[2];
          real accr[3] = {0, 0, 0}, accd = 0, acca = 0, last_alpha = 0, last_c[3] = {0, 0, 0}, last_d = 0;
          real S = 0, Sd = 0;  /* diagnostic variant 4 */
          for (long rel = (long)last - 1; rel >= 0; --rel) {
            const uint32_t gi = f.inst[s + rel].g;
            const gstate* g = &f.gs[gi];
            const real dx = g->px - (real)px, dy = g->py - (real)py;
            real G;
            const real power = blend_G(g, dx, dy, &G);
            if (power > 0) continue;
            const real alpha = rmin(RL(0.99), g->op * G);
            if (alpha < RL(1.0) / RL(255.0)) continue;
            if (g_oracle_variant & 2)
              T = T * (RL(1) / (RL(1) - alpha));
            else
              T = T / (RL(1) - alpha);
            const real dcd = alpha * T;
            real dL_dalpha = 0;
            real* a = tacc + (size_t)10 * gi;
            if (g_oracle_variant & 4) {
              const real cd = FMAR(g->rgb[0], dpix[0], FMAR(g->rgb[1], dpix[1], FMAR(g->rgb[2], dpix[2], dpa)));
              dL_dalpha = FMAR(T, FMAR(g->depth - Sd, dpd, cd - S), (RL(1) / (RL(1) - alpha)) * (-T_final * bg_dot));
              S = FMAR(alpha, cd, (RL(1) - alpha) * S);
              Sd = FMAR(alpha, g->depth, (RL(1) - alpha) * Sd);
              for (int ch = 0; ch < 3; ++ch) a[6 + ch] += dcd * dpix[ch];
              a[9] += dcd * dpd;
            } else {
            for (int ch = 0; ch < 3; ++ch) {
              accr[ch] = last_alpha * last_c[ch] + (RL(1) - last_alpha) * accr[ch];
              last_c[ch] = g->rgb[ch];
              dL_dalpha += (g->rgb[ch] - accr[ch]) * dpix[ch];
              a[6 + ch] += dcd * dpix[ch];
            }
            accd = last_alpha * last_d + (RL(1) - last_alpha) * accd;
            last_d = g->depth;
            dL_dalpha += (g->depth - accd) * dpd;
            a[9] += dcd * dpd;
            acca = last_alpha * RL(1) + (RL(1) - last_alpha) * acca;
            dL_dalpha += (RL(1) - acca) * dpa;
            dL_dalpha *= T;
            last_alpha = alpha;
            dL_dalpha += (-T_final / (RL(1) - alpha)) * bg_dot;
            }
            const real dL_dG = g->op * dL_dalpha;
            const real gdx = G * dx, gdy = G * dy;
            const real dG_ddelx = -gdx * g->ca - gdy * g->cb;
            const real dG_ddely = -gdy * g->cc - gdx * g->cb;
            if (g_oracle_variant & 8) {  /* first moments of u (finished after the loop) */
              a[0] += G * dL_dalpha * dx;
              a[1] += G * dL_dalpha * dy;
            } else {
            a[0] += dL_dG * dG_ddelx * ddelx_dx;
            a[1] += dL_dG * dG_ddely * ddely_dy;
            }
            a[2] += RL(-0.5) * gdx * dx * dL_dG;
            a[3] += RL(-0.5) * gdx * dy * dL_dG;
            a[4] += RL(-0.5) * gdy * dy * dL_dG;
            a[5] += G * dL_dalpha;
          }
        }
  }
  for (int th = 1; th < nth; ++th)
    for (size_t k = 0; k < nacc; ++k) acc[k] += acc_all[nacc * (size_t)th + k];
  if (g_oracle_variant & 8)
    for (int i = 0; i < P; ++i) {
      real* a = acc + (size_t)10 * i;
      const gstate* g = &f.gs[i];
      const float A = -0.72134752044448170f * (float)g->ca, B = -1.4426950408889634f * (float)g->cb,
                  C = -0.72134752044448170f * (float)g->cc;
      const float k = (float)g->op * (1.0f / 1.4426950408889634f);
      const float m1 = (float)a[0], m2 = (float)a[1];
      a[0] = (real)(k * (0.5f * W) * (2.0f * A * m1 + B * m2));
      a[1] = (real)(k * (0.5f * H) * (2.0f * C * m2 + B * m1));
    }

#pragma omp parallel for num_threads(nth) schedule(static) if (nth > 1)
  for (int i = 0; i < P; ++i) {
    const real* a = acc + (size_t)10 * i;
    dmeans2D[3 * i] = a[0]; dmeans2D[3 * i + 1] = a[1]; dmeans2D[3 * i + 2] = 0;
    dopacity[i] = a[5];
    dcolors[3 * i] = a[6]; dcolors[3 * i + 1] = a[7]; dcolors[3 * i + 2] = a[8];
    for (int k = 0; k < 3; ++k) dmeans3D[3 * i + k] = 0;
    if (dcov3D) for (int k = 0; k < 6; ++k) dcov3D[6 * i + k] = 0;
    if (shs && dsh) for (int k = 0; k < 3 * M; ++k) dsh[(size_t)3 * M * i + k] = 0;
    if (!cov3p && dscales) { for (int k = 0; k < 3; ++k) dscales[3 * i + k] = 0; for (int k = 0; k < 4; ++k) drots[4 * i + k] = 0; }
    if (radii[i] <= 0) continue;

    real mean[3];
    load_vec(means + 3 * i, mean, 3);
    real cov3[6], cv[3];
    get_cov3(&c, i, cov3);
    cov2d_state st;
    cov2d(mean, c.fx, c.fy, c.tanx, c.tany, cov3, c.view, &st, cv);
    const real xg = (st.txtz < -st.limx || st.txtz > st.limx) ? 0 : 1;
    const real yg = (st.tytz < -st.limy || st.tytz > st.limy) ? 0 : 1;
    const real ca = cv[0], cb = cv[1], cc = cv[2];
    const real dca = a[2], dcb = a[3], dcc = a[4];
    const real denom = ca * cc - cb * cb;
    real dL_da = 0, dL_db = 0, dL_dc = 0;
    const real denom2inv = RL(1) / ((denom * denom) + RL(0.0000001));
    real dcov[6] = {0, 0, 0, 0, 0, 0};
    real (*T)[3] = st.T;
    if (denom2inv != 0) {
      dL_da = denom2inv * (-cc * cc * dca + 2 * cb * cc * dcb + (denom - ca * cc) * dcc);
      dL_dc = denom2inv * (-ca * ca * dcc + 2 * ca * cb * dcb + (denom - ca * cc) * dca);
      dL_db = denom2inv * 2 * (cb * cc * dca - (denom + 2 * cb * cb) * dcb + ca * cb * dcc);
      dcov[0] = (T[0][0] * T[0][0] * dL_da + T[0][0] * T[1][0] * dL_db + T[1][0] * T[1][0] * dL_dc);
      dcov[3] = (T[0][1] * T[0][1] * dL_da + T[0][1] * T[1][1] * dL_db + T[1][1] * T[1][1] * dL_dc);
      dcov[5] = (T[0][2] * T[0][2] * dL_da + T[0][2] * T[1][2] * dL_db + T[1][2] * T[1][2] * dL_dc);
      dcov[1] = 2 * T[0][0] * T[0][1] * dL_da + (T[0][0] * T[1][1] + T[0][1] * T[1][0]) * dL_db + 2 * T[1][0] * T[1][1] * dL_dc;
      dcov[2] = 2 * T[0][0] * T[0][2] * dL_da + (T[0][0] * T[1][2] + T[0][2] * T[1][0]) * dL_db + 2 * T[1][0] * T[1][2] * dL_dc;
      dcov[4] = 2 * T[0][2] * T[0][1] * dL_da + (T[0][1] * T[1][2] + T[0][2] * T[1][1]) * dL_db + 2 * T[1][1] * T[1][2] * dL_dc;
    }
    const real V[3][3] = {{cov3[0], cov3[1], cov3[2]}, {cov3[1], cov3[3], cov3[4]}, {cov3[2], cov3[4], cov3[5]}};
    real dT0[3], dT1[3];
    for (int k = 0; k < 3; ++k) {
      const real tv0 = T[0][0] * V[k][0] + T[0][1] * V[k][1] + T[0][2] * V[k][2];
      const real tv1 = T[1][0] * V[k][0] + T[1][1] * V[k][1] + T[1][2] * V[k][2];
      dT0[k] = 2 * tv0 * dL_da + tv1 * dL_db;
      dT1[k] = 2 * tv1 * dL_dc + tv0 * dL_db;
    }
    real (*Wm)[3] = st.W;
    const real dJ00 = Wm[0][0] * dT0[0] + Wm[0][1] * dT0[1] + Wm[0][2] * dT0[2];
    const real dJ02 = Wm[2][0] * dT0[0] + Wm[2][1] * dT0[1] + Wm[2][2] * dT0[2];
    const real dJ11 = Wm[1][0] * dT1[0] + Wm[1][1] * dT1[1] + Wm[1][2] * dT1[2];
    const real dJ12 = Wm[2][0] * dT1[0] + Wm[2][1] * dT1[1] + Wm[2][2] * dT1[2];
    const real tz = RL(1) / st.t[2], tz2 = tz * tz, tz3 = tz2 * tz;
    const real hx = c.fx, hy = c.fy;
    const real dtx = xg * -hx * tz2 * dJ02;
    const real dty = yg * -hy * tz2 * dJ12;
    const real dtz = -hx * tz2 * dJ00 - hy * tz2 * dJ11 + (2 * hx * st.t[0]) * tz3 * dJ02 + (2 * hy * st.t[1]) * tz3 * dJ12;
    const real* vm = c.view;
    real dm[3] = {vm[0] * dtx + vm[1] * dty + vm[2] * dtz, vm[4] * dtx + vm[5] * dty + vm[6] * dtz,
                  vm[8] * dtx + vm[9] * dty + vm[10] * dtz};
    /* projection */
    const real* pm = c.proj;
    real mh[4];
    xform4x4(mean, pm, mh);
    const real mw = RL(1) / (mh[3] + RL(0.0000001));
    const real mul1 = (pm[0] * mean[0] + pm[4] * mean[1] + pm[8] * mean[2] + pm[12]) * mw * mw;
    const real mul2 = (pm[1] * mean[0] + pm[5] * mean[1] + pm[9] * mean[2] + pm[13]) * mw * mw;
    dm[0] += (pm[0] * mw - pm[3] * mul1) * a[0] + (pm[1] * mw - pm[3] * mul2) * a[1];
    dm[1] += (pm[4] * mw - pm[7] * mul1) * a[0] + (pm[5] * mw - pm[7] * mul2) * a[1];
    dm[2] += (pm[8] * mw - pm[11] * mul1) * a[0] + (pm[9] * mw - pm[11] * mul2) * a[1];
    /* view depth */
    dm[0] += vm[2] * a[9]; dm[1] += vm[6] * a[9]; dm[2] += vm[10] * a[9];
    /* SH */
    if (shs) {
      const uint32_t cl = f.gs[i].clamp;
      const real dRGB[3] = {(cl & 1u) ? 0 : a[6], (cl & 2u) ? 0 : a[7], (cl & 4u) ? 0 : a[8]};
      const real v[3] = {mean[0] - c.campos[0], mean[1] - c.campos[1], mean[2] - c.campos[2]};
      const real len = SQRTR(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
      real b[16], bx[16], by[16], bz[16];
      sh_basis(c.deg, v[0] / len, v[1] / len, v[2] / len, b, bx, by, bz);
      const int nc = (c.deg + 1) * (c.deg + 1);
      real* dshi = dsh + (size_t)3 * M * i;
      for (int k = 0; k < nc && k < M; ++k)
        for (int ch = 0; ch < 3; ++ch) dshi[3 * k + ch] = b[k] * dRGB[ch];
      real ddx[3] = {0, 0, 0}, ddy[3] = {0, 0, 0}, ddz[3] = {0, 0, 0};
      const float* shi = shs + (size_t)3 * M * i;
      for (int k = 1; k < nc && k < M; ++k)
        for (int ch = 0; ch < 3; ++ch) {
          const real s = (real)shi[3 * k + ch];
          ddx[ch] += bx[k] * s; ddy[ch] += by[k] * s; ddz[ch] += bz[k] * s;
        }
      const real dd[3] = {ddx[0] * dRGB[0] + ddx[1] * dRGB[1] + ddx[2] * dRGB[2],
                          ddy[0] * dRGB[0] + ddy[1] * dRGB[1] + ddy[2] * dRGB[2],
                          ddz[0] * dRGB[0] + ddz[1] * dRGB[1] + ddz[2] * dRGB[2]};
      const real sum2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
      const real inv32 = RL(1) / SQRTR(sum2 * sum2 * sum2);
      dm[0] += ((sum2 - v[0] * v[0]) * dd[0] - v[1] * v[0] * dd[1] - v[2] * v[0] * dd[2]) * inv32;
      dm[1] += (-v[0] * v[1] * dd[0] + (sum2 - v[1] * v[1]) * dd[1] - v[2] * v[1] * dd[2]) * inv32;
      dm[2] += (-v[0] * v[2] * dd[0] - v[1] * v[2] * dd[1] + (sum2 - v[2] * v[2]) * dd[2]) * inv32;
    }
    for (int k = 0; k < 3; ++k) dmeans3D[3 * i + k] = dm[k];
    if (dcov3D) for (int k = 0; k < 6; ++k) dcov3D[6 * i + k] = dcov[k];
    if (!cov3p && dscales) {
      real sc[3], q[4], R[3][3];
      load_vec(scales + 3 * i, sc, 3);
      load_vec(rots + 4 * i, q, 4);
      rot_from_quat(q, R);
      const real s[3] = {c.mod * sc[0], c.mod * sc[1], c.mod * sc[2]};
      const real Gm[3][3] = {{dcov[0], RL(0.5) * dcov[1], RL(0.5) * dcov[2]},
                             {RL(0.5) * dcov[1], dcov[3], RL(0.5) * dcov[4]},
                             {RL(0.5) * dcov[2], RL(0.5) * dcov[4], dcov[5]}};
      real dE[3][3], dR[3][3];
      for (int aa = 0; aa < 3; ++aa)
        for (int k = 0; k < 3; ++k)
          dE[aa][k] = 2 * (Gm[aa][0] * s[k] * R[0][k] + Gm[aa][1] * s[k] * R[1][k] + Gm[aa][2] * s[k] * R[2][k]);
      for (int k = 0; k < 3; ++k) {
        dscales[3 * i + k] = dE[0][k] * R[0][k] + dE[1][k] * R[1][k] + dE[2][k] * R[2][k];
        for (int aa = 0; aa < 3; ++aa) dR[aa][k] = dE[aa][k] * s[k];
      }
      const real r = q[0], x = q[1], y = q[2], z = q[3];
      drots[4 * i] = -2 * z * dR[0][1] + 2 * y * dR[0][2] + 2 * z * dR[1][0] - 2 * x * dR[1][2] - 2 * y * dR[2][0] + 2 * x * dR[2][1];
      drots[4 * i + 1] = 2 * y * dR[0][1] + 2 * z * dR[0][2] + 2 * y * dR[1][0] - 4 * x * dR[1][1] - 2 * r * dR[1][2] + 2 * z * dR[2][0] + 2 * r * dR[2][1] - 4 * x * dR[2][2];
      drots[4 * i + 2] = -4 * y * dR[0][0] + 2 * x * dR[0][1] + 2 * r * dR[0][2] + 2 * x * dR[1][0] + 2 * z * dR[1][2] - 2 * r * dR[2][0] + 2 * z * dR[2][1] - 4 * y * dR[2][2];
      drots[4 * i + 3] = -4 * z * dR[0][0] - 2 * r * dR[0][1] + 2 * x * dR[0][2] + 2 * r * dR[1][0] - 4 * z * dR[1][1] + 2 * y * dR[1][2] + 2 * x * dR[2][0] + 2 * y * dR[2][1];
    }
  }
  free(acc_all);
  free(radii);
  free_fwd(&f);
}

/*
 * simple_knn.distCUDA2 restated (external package graphdeco-inria/simple-knn, unpinned, not in the
 * reference tree; called at geometry/gaussian_base.py:434-437): for every point the mean of the squared
 * distances to its 3 nearest other points.  Brute force over all pairs (test sizes only), the published
 * updateKBest swap-insertion into best[3] initialised to FLT_MAX, mean (best0 + best1 + best2) / 3.
 * Per-pair distance fma(dz, dz, fma(dy, dy, dx * dx)) with d = other - point.  qidx (nq entries) selects
 * the query points (NULL: all P, nq = P).
 */
#include <float.h>
void FN(oracle_knn_mean_dist)(int P, const float* pts, int nq, const int* qidx, double* out) {
  for (int qi = 0; qi < nq; ++qi) {
    const int i = qidx ? qidx[qi] : qi;
    real best[3] = {RL(FLT_MAX), RL(FLT_MAX), RL(FLT_MAX)};
    const real qx = (real)pts[3 * i], qy = (real)pts[3 * i + 1], qz = (real)pts[3 * i + 2];
    for (int j = 0; j < P; ++j) {
      if (j == i) continue;
      const real dx = (real)pts[3 * j] - qx, dy = (real)pts[3 * j + 1] - qy, dz = (real)pts[3 * j + 2] - qz;
      real d = FMAR(dz, dz, FMAR(dy, dy, dx * dx));
      for (int k = 0; k < 3; ++k) {
        if (best[k] > d) {
          const real t = best[k];
          best[k] = d;
          d = t;
        }
      }
    }
    out[qi] = (double)((best[0] + best[1] + best[2]) / RL(3.0));
  }
}

/*
 * mpm_oracle.c -- scalar C restatement of the reference MPM substep.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Every function cites the
 * reference file:line it restates.  f32 throughout, -ffp-contract=off,
 * operation order as written in the Taichi source.
 *
 * Out-of-range grid indices are undefined behaviour in the reference (Taichi
 * debug=False, main.py:28); both this oracle and the HIP path skip them.
 */
#include "oracle.h"
#include <math.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <stdlib.h>

static inline float fmaxf_(float a, float b) { return a > b ? a : b; }
static inline float fminf_(float a, float b) { return a < b ? a : b; }

/* Host debug build (make asan / make debug: -DOM_DEBUG).  The
 * reference runs Taichi without debug=True (main.py:28), so an out-of-range
 * grid index there is undefined behaviour that nothing reports; Taichi's
 * debug mode would stop at it.  Here every grid access goes through OM_NODE,
 * which in the debug build aborts on an index outside [0, ng)^3, and every
 * stencil node that the restatement skips because it lies outside the grid
 * (the documented choice above) is counted (om_debug_skipped); with the
 * environment variable GSMPM_ORACLE_STRICT=1 a skip aborts too, as Taichi's
 * debug mode would. */
#ifdef OM_DEBUG
#include <stdio.h>
static long om_dbg_skipped = 0;
static int om_dbg_strict = -1;
static size_t om_node_checked(int ng, int ix, int iy, int iz, const char* where) {
  if (ix < 0 || iy < 0 || iz < 0 || ix >= ng || iy >= ng || iz >= ng) {
    fprintf(stderr, "oracle %s: grid node (%d, %d, %d) outside the %d^3 grid\n", where, ix, iy, iz, ng);
    abort();
  }
  return ((size_t)ix * ng + iy) * ng + iz;
}
static void om_skip(int ng, int ix, int iy, int iz, const char* where) {
  __atomic_add_fetch(&om_dbg_skipped, 1, __ATOMIC_RELAXED);
  if (om_dbg_strict < 0) {
    const char* e = getenv("GSMPM_ORACLE_STRICT");
    om_dbg_strict = e && e[0] == '1';
  }
  if (om_dbg_strict) {
    fprintf(stderr, "oracle %s: stencil node (%d, %d, %d) outside the %d^3 grid (strict)\n", where, ix, iy, iz, ng);
    abort();
  }
}
#define OM_NODE(ng, ix, iy, iz, where) om_node_checked((ng), (ix), (iy), (iz), (where))
#define OM_SKIP(ng, ix, iy, iz, where) om_skip((ng), (ix), (iy), (iz), (where))
long om_debug_skipped(void) { return __atomic_load_n(&om_dbg_skipped, __ATOMIC_RELAXED); }
int om_debug_build(void) { return 1; }
#else
#define OM_NODE(ng, ix, iy, iz, where) (((size_t)(ix) * (ng) + (iy)) * (ng) + (iz))
#define OM_SKIP(ng, ix, iy, iz, where) ((void)0)
long om_debug_skipped(void) { return -1; }
int om_debug_build(void) { return 0; }
#endif

/* ------------------------------------------------------------------ 3x3 -- */
static void mm3(const float A[9], const float B[9], float C[9]) {
  float T[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      T[i * 3 + j] = A[i * 3 + 0] * B[0 * 3 + j] + A[i * 3 + 1] * B[1 * 3 + j] + A[i * 3 + 2] * B[2 * 3 + j];
  memcpy(C, T, sizeof T);
}
static void mmT3(const float A[9], const float B[9], float C[9]) { /* A @ B^T */
  float T[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      T[i * 3 + j] = A[i * 3 + 0] * B[j * 3 + 0] + A[i * 3 + 1] * B[j * 3 + 1] + A[i * 3 + 2] * B[j * 3 + 2];
  memcpy(C, T, sizeof T);
}
static float det3(const float A[9]) {
  /* Taichi Matrix.determinant for 3x3 (cofactor expansion along row 0) */
  return A[0] * (A[4] * A[8] - A[5] * A[7]) - A[1] * (A[3] * A[8] - A[5] * A[6]) +
         A[2] * (A[3] * A[7] - A[4] * A[6]);
}

/* ------------------------------------------------------------------ SVD --
 * ti.svd (f32) is the McAdams et al. 2011 "minimal branching" 3x3 SVD:
 * Jacobi eigen-analysis of A^T A with approximate Givens rotations
 * (5 sweeps for f32), column sort by norm with sign fix-up, Givens QR.
 * U, V are proper rotations; sig = diag(R) so sig3 carries sign(det A).
 * (Taichi intrinsic, called at utils.py:33,385; constitutive_models.py:64,107,218.)
 */
#define SVD_GAMMA 5.828427124746190f /* 3 + 2*sqrt(2) */
#define SVD_CSTAR 0.923879532511287f /* cos(pi/8) */
#define SVD_SSTAR 0.382683432365090f /* sin(pi/8) */
#define SVD_EPS 1.0e-12f
#define SVD_SWEEPS 5

static void jacobi_conj(int p, int q, float S[9], float qv[4]) {
  float ch = 2.0f * (S[p * 3 + p] - S[q * 3 + q]);
  float sh = S[q * 3 + p];
  int b = (SVD_GAMMA * sh * sh) < (ch * ch);
  float w = 1.0f / sqrtf(ch * ch + sh * sh);
  ch = b ? w * ch : SVD_CSTAR;
  sh = b ? w * sh : SVD_SSTAR;
  float c = ch * ch - sh * sh, s = 2.0f * sh * ch;
  /* R = I with R[p][p]=c, R[p][q]=-s, R[q][p]=s, R[q][q]=c ; S <- R^T S R */
  float R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  R[p * 3 + p] = c; R[p * 3 + q] = -s; R[q * 3 + p] = s; R[q * 3 + q] = c;
  float T[9], Rt[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Rt[i * 3 + j] = R[j * 3 + i];
  mm3(S, R, T);
  mm3(Rt, T, S);
  /* quaternion of R: rotation about axis k (the index not in {p,q}); the
   * (p,q) plane orientation gives +sh on that axis for (0,1),(1,2),(2,0). */
  int k = 3 - p - q;
  float r[4] = {ch, 0.f, 0.f, 0.f};
  r[1 + k] = sh;
  /* qv <- qv * r */
  float a0 = qv[0], a1 = qv[1], a2 = qv[2], a3 = qv[3];
  float b0 = r[0], b1 = r[1], b2 = r[2], b3 = r[3];
  qv[0] = a0 * b0 - a1 * b1 - a2 * b2 - a3 * b3;
  qv[1] = a0 * b1 + a1 * b0 + a2 * b3 - a3 * b2;
  qv[2] = a0 * b2 - a1 * b3 + a2 * b0 + a3 * b1;
  qv[3] = a0 * b3 + a1 * b2 - a2 * b1 + a3 * b0;
}

static void quat_to_mat(const float q[4], float M[9]) {
  float w = q[0], x = q[1], y = q[2], z = q[3];
  M[0] = 1.f - 2.f * (y * y + z * z); M[1] = 2.f * (x * y - w * z); M[2] = 2.f * (x * z + w * y);
  M[3] = 2.f * (x * y + w * z); M[4] = 1.f - 2.f * (x * x + z * z); M[5] = 2.f * (y * z - w * x);
  M[6] = 2.f * (x * z - w * y); M[7] = 2.f * (y * z + w * x); M[8] = 1.f - 2.f * (x * x + y * y);
}

static void swap_cols(float M[9], int i, int j, int negate_j) {
  for (int r = 0; r < 3; ++r) {
    float t = M[r * 3 + i];
    M[r * 3 + i] = M[r * 3 + j];
    M[r * 3 + j] = negate_j ? -t : t;
  }
}

/* QR Givens on rows (p,q): zero B[q][p] using pivot B[p][p]; U <- U G. */
static void qr_givens(int p, int q, float B[9], float U[9]) {
  float a1 = B[p * 3 + p], a2 = B[q * 3 + p];
  float rho = sqrtf(a1 * a1 + a2 * a2);
  float sh = rho > SVD_EPS ? a2 : 0.0f;
  float ch = fabsf(a1) + fmaxf_(rho, SVD_EPS);
  if (a1 < 0.0f) { float t = sh; sh = ch; ch = t; }
  float w = 1.0f / sqrtf(ch * ch + sh * sh);
  ch *= w; sh *= w;
  float c = ch * ch - sh * sh, s = 2.0f * sh * ch;
  /* G = I, G[p][p]=c, G[p][q]=-s, G[q][p]=s, G[q][q]=c ; B <- G^T B, U <- U G */
  for (int j = 0; j < 3; ++j) {
    float bp = B[p * 3 + j], bq = B[q * 3 + j];
    B[p * 3 + j] = c * bp + s * bq;
    B[q * 3 + j] = -s * bp + c * bq;
  }
  for (int r = 0; r < 3; ++r) {
    float up = U[r * 3 + p], uq = U[r * 3 + q];
    U[r * 3 + p] = c * up + s * uq;
    U[r * 3 + q] = -s * up + c * uq;
  }
}

void om_svd3(const float A[9], float U[9], float sig[3], float V[9]) {
  float S[9];
  /* S = A^T A */
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      S[i * 3 + j] = A[0 * 3 + i] * A[0 * 3 + j] + A[1 * 3 + i] * A[1 * 3 + j] + A[2 * 3 + i] * A[2 * 3 + j];
  float qv[4] = {1.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < SVD_SWEEPS; ++it) {
    jacobi_conj(0, 1, S, qv);
    jacobi_conj(1, 2, S, qv);
    jacobi_conj(2, 0, S, qv);
  }
  float qn = 1.0f / sqrtf(qv[0] * qv[0] + qv[1] * qv[1] + qv[2] * qv[2] + qv[3] * qv[3]);
  for (int i = 0; i < 4; ++i) qv[i] *= qn;
  quat_to_mat(qv, V);
  float B[9];
  mm3(A, V, B);
  /* sort columns by decreasing norm; swapped-in column j is negated to keep det V = +1 */
  float rho[3];
  for (int c = 0; c < 3; ++c) rho[c] = B[c] * B[c] + B[3 + c] * B[3 + c] + B[6 + c] * B[6 + c];
  const int pairs[3][2] = {{0, 1}, {0, 2}, {1, 2}};
  for (int k = 0; k < 3; ++k) {
    int i = pairs[k][0], j = pairs[k][1];
    if (rho[i] < rho[j]) {
      swap_cols(B, i, j, 1);
      swap_cols(V, i, j, 1);
      float t = rho[i]; rho[i] = rho[j]; rho[j] = t;
    }
  }
  float Uq[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  qr_givens(0, 1, B, Uq);
  qr_givens(0, 2, B, Uq);
  qr_givens(1, 2, B, Uq);
  memcpy(U, Uq, sizeof Uq);
  sig[0] = B[0]; sig[1] = B[4]; sig[2] = B[8];
}

/* --------------------------------------------------- init (model.py) -- */
/* compute_mu_lam_from_E_nu, utils.py:349-362 */
void om_mu_lam(int n, const float* logE, const float* y, float* mu, float* lam) {
  for (int p = 0; p < n; ++p) {
    float E = powf(10.0f, logE[p]);
    float nu = 0.49f / (1.0f + expf(-y[p]));
    mu[p] = E / (2.0f * (1.0f + nu));
    lam[p] = E * nu / ((1.0f + nu) * (1.0f - 2.0f * nu));
  }
}

/* get_particle_volume, internel_filling/filling.py:11-24 (floor, i32 counts) */
void om_particle_volume(int n, const float* x, int ng, float grid_dx, int32_t* cnt, float* vol) {
  memset(cnt, 0, sizeof(int32_t) * (size_t)ng * ng * ng);
  for (int p = 0; p < n; ++p) {
    int c[3];
    for (int d = 0; d < 3; ++d) c[d] = (int)floorf(x[p * 3 + d] / grid_dx);
    if (c[0] < 0 || c[1] < 0 || c[2] < 0 || c[0] >= ng || c[1] >= ng || c[2] >= ng) {
      OM_SKIP(ng, c[0], c[1], c[2], "particle_volume");
      continue;
    }
    cnt[OM_NODE(ng, c[0], c[1], c[2], "particle_volume")] += 1;
  }
  float dx3 = grid_dx * grid_dx * grid_dx; /* Taichi lowers `grid_dx ** 3` (int exponent) to products */
  for (int p = 0; p < n; ++p) {
    int c[3];
    for (int d = 0; d < 3; ++d) c[d] = (int)floorf(x[p * 3 + d] / grid_dx);
    if (c[0] < 0 || c[1] < 0 || c[2] < 0 || c[0] >= ng || c[1] >= ng || c[2] >= ng) { vol[p] = 0.f; continue; }
    vol[p] = dx3 / (float)cnt[OM_NODE(ng, c[0], c[1], c[2], "particle_volume")];
  }
}

/* ------------------------------------- constitutive_models.py restated -- */
static void diag_sandwich(const float U[9], const float d[3], const float V[9], float out[9]) {
  /* U @ diag(d) @ V^T */
  float T[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T[i * 3 + j] = U[i * 3 + j] * d[j];
  mmT3(T, V, out);
}

/* von_mises_return_mapping, constitutive_models.py:62-103 */
static void von_mises(const float Ft[9], float mu, float lam, float* yield, float hardening, float xi, float Fout[9]) {
  float U[9], V[9], s[3];
  om_svd3(Ft, U, s, V);
  float sg[3] = {fmaxf_(s[0], 0.01f), fmaxf_(s[1], 0.01f), fmaxf_(s[2], 0.01f)};
  float eps[3] = {logf(sg[0]), logf(sg[1]), logf(sg[2])};
  float temp = (eps[0] + eps[1] + eps[2]) / 3.0f;
  float tr = eps[0] + eps[1] + eps[2];
  float tau[3];
  for (int d = 0; d < 3; ++d) tau[d] = 2.0f * mu * eps[d] + lam * tr * 1.0f;
  float sum_tau = tau[0] + tau[1] + tau[2];
  float cond[3];
  for (int d = 0; d < 3; ++d) cond[d] = tau[d] - sum_tau / 3.0f;
  float cn = sqrtf(cond[0] * cond[0] + cond[1] * cond[1] + cond[2] * cond[2]);
  if (cn > *yield) {
    float eh[3];
    for (int d = 0; d < 3; ++d) eh[d] = eps[d] - temp;
    float ehn = sqrtf(eh[0] * eh[0] + eh[1] * eh[1] + eh[2] * eh[2]) + 1e-6f;
    float dg = ehn - *yield / (2.0f * mu);
    for (int d = 0; d < 3; ++d) eps[d] -= (dg / ehn) * eh[d];
    float se[3] = {expf(eps[0]), expf(eps[1]), expf(eps[2])};
    diag_sandwich(U, se, V, Fout);
    if (hardening == 1.0f) *yield += 2.0f * mu * xi * dg;
  } else {
    memcpy(Fout, Ft, 36);
  }
}

/* sand_return_mapping, constitutive_models.py:105-140 */
static void sand(const float Ft[9], float mu, float lam, float alpha, float Fout[9]) {
  float U[9], V[9], s[3];
  om_svd3(Ft, U, s, V);
  float eps[3];
  for (int d = 0; d < 3; ++d) eps[d] = logf(fmaxf_(fabsf(s[d]), 1e-14f));
  float tr = eps[0] + eps[1] + eps[2];
  float eh[3];
  for (int d = 0; d < 3; ++d) eh[d] = eps[d] - tr / 3.0f;
  float ehn = sqrtf(eh[0] * eh[0] + eh[1] * eh[1] + eh[2] * eh[2]);
  float dg = ehn + (3.0f * lam + 2.0f * mu) / (2.0f * mu) * tr * alpha;
  if (dg <= 0.0f) {
    memcpy(Fout, Ft, 36);
  } else if (tr > 0.0f) {
    mmT3(U, V, Fout);
  } else {
    float H[3], sn[3];
    for (int d = 0; d < 3; ++d) H[d] = eps[d] - eh[d] * (dg / ehn);
    for (int d = 0; d < 3; ++d) sn[d] = expf(H[d]);
    diag_sandwich(U, sn, V, Fout);
  }
}

/* viscoplasticity_return_mapping_with_StVK, constitutive_models.py:216-259
 * NOTE: `U * sig_elastic * V.transpose()` is element-wise in Taichi (:256),
 * so only the diagonal U_ii e_i V_ii survives. */
static void viscoplastic(const float Ft[9], float mu, float yield, float pvisc, float dt, float Fout[9]) {
  float U[9], V[9], s[3];
  om_svd3(Ft, U, s, V);
  float sg[3] = {fmaxf_(s[0], 0.01f), fmaxf_(s[1], 0.01f), fmaxf_(s[2], 0.01f)};
  float b[3] = {sg[0] * sg[0], sg[1] * sg[1], sg[2] * sg[2]};
  float eps[3] = {logf(sg[0]), logf(sg[1]), logf(sg[2])};
  float tr = eps[0] + eps[1] + eps[2];
  float eh[3];
  for (int d = 0; d < 3; ++d) eh[d] = eps[d] - tr / 3.0f;
  float st[3];
  for (int d = 0; d < 3; ++d) st[d] = 2.0f * mu * eh[d];
  float stn = sqrtf(st[0] * st[0] + st[1] * st[1] + st[2] * st[2]);
  float y = stn - 0.8f * sqrtf(2.0f / 3.0f) * yield;
  if (y > 0.0f) {
    float mu_hat = mu * (b[0] + b[1] + b[2]) / 3.0f;
    float snn = stn - y / (1.0f + pvisc * 2.0f / (2.0f * mu_hat * dt));
    float en[3];
    for (int d = 0; d < 3; ++d) {
      float sn = (snn / stn) * st[d];
      en[d] = 1.0f / (2.0f * mu) * sn + tr / 3.0f;
    }
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        float se = (i == j) ? expf(en[i]) : 0.0f;
        Fout[i * 3 + j] = U[i * 3 + j] * se * V[j * 3 + i];
      }
  } else {
    memcpy(Fout, Ft, 36);
  }
}

/* kirchoff_stress_StVK, constitutive_models.py:23-38 */
static void stress_stvk(const float F[9], const float U[9], const float V[9], const float s[3], float mu, float lam, float out[9]) {
  float sv[3] = {fmaxf_(s[0], 0.01f), fmaxf_(s[1], 0.01f), fmaxf_(s[2], 0.01f)};
  float eps[3] = {logf(sv[0]), logf(sv[1]), logf(sv[2])};
  float lss = logf(sv[0]) + logf(sv[1]) + logf(sv[2]);
  float tau[3];
  for (int d = 0; d < 3; ++d) tau[d] = 2.0f * mu * eps[d] + lam * lss * 1.0f;
  float T[9];
  diag_sandwich(U, tau, V, T);
  mmT3(T, F, out); /* (U tau V^T) F^T */
}

/* kirchoff_stress_Drucker_Prager, constitutive_models.py:41-58 */
static void stress_dp(const float F[9], const float U[9], const float V[9], const float s[3], float mu, float lam, float out[9]) {
  float lss = logf(s[0]) + logf(s[1]) + logf(s[2]);
  float c[3];
  for (int d = 0; d < 3; ++d) c[d] = 2.0f * mu * logf(s[d]) / s[d] + lam * lss / s[d];
  float T[9];
  diag_sandwich(U, c, V, T);
  mmT3(T, F, out);
}

/* kirchoff_stress_FCR, constitutive_models.py:10-20 (only reached with the F3 quirk off) */
static void stress_fcr(const float F[9], const float U[9], const float V[9], float J, float mu, float lam, float out[9]) {
  float R[9];
  mmT3(U, V, R);
  float D[9];
  for (int i = 0; i < 9; ++i) D[i] = 2.0f * mu * (F[i] - R[i]);
  mmT3(D, F, out);
  float l = lam * J * (J - 1.0f);
  out[0] += l; out[4] += l; out[8] += l;
}

/* fluid_return_mapping, constitutive_models.py:142-213.  Defined by the
 * reference but dispatched nowhere (utils.py:13-54 has no branch for it); the
 * GPU build pairs it with kirchoff_stress_StVK (as material 3), so om_fluid
 * returns that stress too (symmetrised, utils.py:52).  Unlike :256 the
 * product at :205 is a true matrix product U @ diag @ V^T. */
void om_fluid(int n, const float* Ft_all, const float* mu_all, const float* lam_all, const float* yield_all,
              float pvisc, float dt, float* Fout_all, float* tau_all) {
  for (int p = 0; p < n; ++p) {
    const float* Ft = Ft_all + p * 9;
    float* Fo = Fout_all + p * 9;
    const float mu = mu_all[p], lam = lam_all[p];
    float U[9], V[9], sig[3];
    om_svd3(Ft, U, sig, V);
    float eps[3];
    for (int d = 0; d < 3; ++d) eps[d] = logf(fmaxf_(fabsf(sig[d]), 0.01f));   /* :163-167 */
    float tr = eps[0] + eps[1] + eps[2];
    float eh[3];
    for (int d = 0; d < 3; ++d) eh[d] = eps[d] - tr / 3.0f;                       /* :169 */
    float st[3];
    for (int d = 0; d < 3; ++d) st[d] = 2.0f * mu * eh[d];                        /* :172 */
    float stn = sqrtf(st[0] * st[0] + st[1] * st[1] + st[2] * st[2]);
    float yv = stn - sqrtf(2.0f / 3.0f) * yield_all[p];                           /* :177 */
    if (yv > 0.0f) {
      float mu_hat = mu * (sig[0] * sig[0] + sig[1] * sig[1] + sig[2] * sig[2]) / 3.0f;  /* :185 */
      float pf = 1.0f + pvisc / (2.0f * mu_hat * dt);                            /* :186 */
      float snn = stn - yv / pf;                                                  /* :189 */
      float se[3];
      for (int d = 0; d < 3; ++d) {
        float sn = (snn / stn) * st[d];                                           /* :190 */
        se[d] = expf((1.0f / (2.0f * mu)) * sn + tr / 3.0f);                      /* :193 */
      }
      diag_sandwich(U, se, V, Fo);                                                /* :205 */
    } else {
      memcpy(Fo, Ft, 36);                                                         /* :210 */
    }
    float U2[9], V2[9], s2[3], T[9];
    om_svd3(Fo, U2, s2, V2);
    stress_stvk(Fo, U2, V2, s2, mu, lam, T);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) tau_all[p * 9 + i * 3 + j] = (T[i * 3 + j] + T[j * 3 + i]) / 2.0f;
  }
}

/* compute_stress_from_F_trial, utils.py:13-54 */
void om_stress(om_state* s, float dt) {
  const int mat = s->material;
#pragma omp parallel for schedule(static)
  for (int p = 0; p < s->n; ++p) {
    float* Ft = s->F_trial + p * 9;
    float* F = s->F + p * 9;
    if (mat == 1) von_mises(Ft, s->mu[p], s->lam[p], &s->yield_stress[p], s->hardening, s->xi, F);
    else if (mat == 2) sand(Ft, s->mu[p], s->lam[p], s->alpha, F);
    else if (mat == 3) viscoplastic(Ft, s->mu[p], s->yield_stress[p], s->plastic_viscosity, dt, F);
    else memcpy(F, Ft, 36);
    float st[9] = {0};
    float out9[9];
    float* out = s->stress + p * 9;
    if (mat == 0 && s->jelly_quirk) {
      /* as written the FCR branch never fires: J/U/S/V are dead */
      memset(out, 0, sizeof out9);
      continue;
    }
    float J = det3(F);
    float U[9], V[9], sg[3];
    om_svd3(F, U, sg, V);
    if (mat == 0) {
      if (!s->jelly_quirk) stress_fcr(F, U, V, J, s->mu[p], s->lam[p], st);
    } else if (mat == 1 || mat == 3) {
      stress_stvk(F, U, V, sg, s->mu[p], s->lam[p], st);
    } else if (mat == 2) {
      stress_dp(F, U, V, sg, s->mu[p], s->lam[p], st);
    }
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) out[i * 3 + j] = (st[i * 3 + j] + st[j * 3 + i]) / 2.0f;
  }
}

/* quadratic B-spline weights, utils.py:93-109 / 221-246 */
static void bspline(const float xp[3], float inv_dx, int base[3], float fx[3], float w[3][3], float dw[3][3]) {
  for (int d = 0; d < 3; ++d) {
    float gp = xp[d] * inv_dx;
    base[d] = (int)(gp - 0.5f); /* .cast(int): truncation toward zero */
    fx[d] = gp - (float)base[d];
    float wa = 1.5f - fx[d], wb = fx[d] - 1.0f, wc = fx[d] - 0.5f;
    w[d][0] = wa * wa * 0.5f;
    w[d][1] = 0.75f - wb * wb;
    w[d][2] = wc * wc * 0.5f;
    dw[d][0] = fx[d] - 1.5f;
    dw[d][1] = -2.0f * (fx[d] - 1.0f);
    dw[d][2] = fx[d] - 0.5f;
  }
}

/* p2g, utils.py:89-134: the scatter of one particle */
static void p2g_particle(om_state* s, int p, float dt) {
  const int ng = s->ng;
  const float dx = s->dx, inv_dx = s->inv_dx;
  {
    const float* st = s->stress + p * 9;
    int base[3]; float fx[3], w[3][3], dw[3][3];
    bspline(s->x + p * 3, inv_dx, base, fx, w, dw);
    const float* C = s->C + p * 9;
    const float* vp = s->v + p * 3;
    const float m = s->mass[p], vol = s->vol[p];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        for (int k = 0; k < 3; ++k) {
          int o[3] = {i, j, k};
          float dpos[3];
          for (int d = 0; d < 3; ++d) dpos[d] = ((float)o[d] - fx[d]) * dx;
          int ix = base[0] + i, iy = base[1] + j, iz = base[2] + k;
          float weight = w[0][i] * w[1][j] * w[2][k];
          float dwt[3] = {dw[0][i] * w[1][j] * w[2][k] * inv_dx, w[0][i] * dw[1][j] * w[2][k] * inv_dx,
                          w[0][i] * w[1][j] * dw[2][k] * inv_dx};
          float ef[3], add[3];
          for (int r = 0; r < 3; ++r) {
            /* ((-vol) * stress) @ dweight */
            ef[r] = (-vol * st[r * 3 + 0]) * dwt[0] + (-vol * st[r * 3 + 1]) * dwt[1] + (-vol * st[r * 3 + 2]) * dwt[2];
          }
          for (int r = 0; r < 3; ++r) {
            float cd = C[r * 3 + 0] * dpos[0] + C[r * 3 + 1] * dpos[1] + C[r * 3 + 2] * dpos[2];
            add[r] = weight * m * (vp[r] + cd) + dt * ef[r];
          }
          if (ix < 0 || iy < 0 || iz < 0 || ix >= ng || iy >= ng || iz >= ng) {
            OM_SKIP(ng, ix, iy, iz, "p2g");
            continue;
          }
          size_t g = OM_NODE(ng, ix, iy, iz, "p2g");
          s->gv_in[g * 3 + 0] += add[0];
          s->gv_in[g * 3 + 1] += add[1];
          s->gv_in[g * 3 + 2] += add[2];
          s->gm[g] += weight * m;
        }
  }
}

void om_p2g(om_state* s, float dt) {
#ifndef _OPENMP
  /* the checker: particles in index order, exactly the reference's serial sum */
  for (int p = 0; p < s->n; ++p) p2g_particle(s, p, dt);
#else
  /* CPU-baseline build only (liboracle_omp.so): particles bucketed by x-slabs
   * of 4 cells (stable, index order inside a slab); even slabs then odd slabs
   * run in parallel -- a particle writes nodes base..base+2, so slabs two
   * apart never touch the same node.  Same math, different summation order. */
  const int W = 4, ng = s->ng, ns = (ng + W - 1) / W;
  int* cnt = (int*)calloc((size_t)ns + 1, sizeof(int));
  int* order = (int*)malloc(sizeof(int) * (size_t)(s->n > 0 ? s->n : 1));
  int* slab = (int*)malloc(sizeof(int) * (size_t)(s->n > 0 ? s->n : 1));
  for (int p = 0; p < s->n; ++p) {
    int b = (int)(s->x[p * 3] * s->inv_dx - 0.5f);
    b = b < 0 ? 0 : (b >= ng ? ng - 1 : b);
    slab[p] = b / W;
    cnt[slab[p] + 1]++;
  }
  for (int i = 0; i < ns; ++i) cnt[i + 1] += cnt[i];
  int* pos = (int*)malloc(sizeof(int) * (size_t)ns);
  memcpy(pos, cnt, sizeof(int) * (size_t)ns);
  for (int p = 0; p < s->n; ++p) order[pos[slab[p]]++] = p;
  for (int parity = 0; parity < 2; ++parity) {
#pragma omp parallel for schedule(dynamic, 1)
    for (int sl = parity; sl < ns; sl += 2)
      for (int q = cnt[sl]; q < cnt[sl + 1]; ++q) p2g_particle(s, order[q], dt);
  }
  free(pos);
  free(slab);
  free(order);
  free(cnt);
#endif
}

/* grid_normalization_and_gravity, utils.py:177-183 */
void om_grid_normalize(om_state* s, float dt) {
  const long nn = (long)s->ng * s->ng * s->ng;
#pragma omp parallel for schedule(static)
  for (long g = 0; g < nn; ++g) {
    if (s->gm[g] > 1e-15f) {
      for (int d = 0; d < 3; ++d) s->gv_out[g * 3 + d] = s->gv_in[g * 3 + d] / s->gm[g] + dt * s->gravity[d];
    }
  }
}

/* BasicBC.apply (boundary_conditions.py:23-27) and MPM_Collider.collide
 * (collider.py:13-44), in list order (solver.py:41-46). */
void om_grid_ops(om_state* s, int n_ops, const om_gridop* ops, const int32_t* active) {
  const int ng = s->ng;
  const float dx = s->dx;
  for (int o = 0; o < n_ops; ++o) {
    const om_gridop* op = &ops[o];
    if (op->kind == 0 && !active[o]) continue;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < ng; ++i)
      for (int j = 0; j < ng; ++j)
        for (int k = 0; k < ng; ++k) {
          size_t g = OM_NODE(ng, i, j, k, "grid_ops");
          float* v = s->gv_out + g * 3;
          if (op->kind == 0) {
            float px[3] = {(float)i * dx, (float)j * dx, (float)k * dx};
            int in = 1;
            for (int d = 0; d < 3; ++d) in &= fabsf(px[d] - op->a[d]) < op->b[d];
            if (in) { v[0] = 0.f; v[1] = 0.f; v[2] = 0.f; }
          } else {
            float off[3] = {(float)i * dx - op->a[0], (float)j * dx - op->a[1], (float)k * dx - op->a[2]};
            const float* n = op->b;
            float dot = off[0] * n[0] + off[1] * n[1] + off[2] * n[2];
            if (dot < 0.0f) {
              float vv[3] = {v[0], v[1], v[2]};
              float nc = vv[0] * n[0] + vv[1] * n[1] + vv[2] * n[2];
              float mn = fminf_(nc, 0.0f);
              for (int d = 0; d < 3; ++d) vv[d] = vv[d] - mn * n[d];
              float len = sqrtf(vv[0] * vv[0] + vv[1] * vv[1] + vv[2] * vv[2]);
              if (nc < 0.0f && len > 1e-20f) {
                float sc = fmaxf_(0.0f, len + nc * op->friction);
                float nv[3] = {vv[0] / len, vv[1] / len, vv[2] / len};
                for (int d = 0; d < 3; ++d) vv[d] = sc * nv[d];
              }
              for (int d = 0; d < 3; ++d) v[d] = vv[d] * 0.99f;
            }
          }
        }
  }
}

/* g2p, utils.py:218-282 (the dead update_cov at :282 is omitted) */
void om_g2p(om_state* s, float dt) {
  const int ng = s->ng;
  const float inv_dx = s->inv_dx;
#pragma omp parallel for schedule(static)
  for (int p = 0; p < s->n; ++p) {
    int base[3]; float fx[3], w[3][3], dw[3][3];
    bspline(s->x + p * 3, inv_dx, base, fx, w, dw);
    float nv[3] = {0, 0, 0}, nC[9] = {0}, nF[9] = {0};
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        for (int k = 0; k < 3; ++k) {
          int o[3] = {i, j, k};
          float dpos[3];
          for (int d = 0; d < 3; ++d) dpos[d] = (float)o[d] - fx[d];
          int ix = base[0] + i, iy = base[1] + j, iz = base[2] + k;
          float weight = w[0][i] * w[1][j] * w[2][k];
          float gv[3] = {0, 0, 0};
          if (ix < 0 || iy < 0 || iz < 0 || ix >= ng || iy >= ng || iz >= ng) {
            OM_SKIP(ng, ix, iy, iz, "g2p");
          } else {
            size_t g = OM_NODE(ng, ix, iy, iz, "g2p");
            gv[0] = s->gv_out[g * 3]; gv[1] = s->gv_out[g * 3 + 1]; gv[2] = s->gv_out[g * 3 + 2];
          }
          for (int d = 0; d < 3; ++d) nv[d] += gv[d] * weight;
          float cw = weight * inv_dx * 4.0f;
          for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) nC[r * 3 + c] += gv[r] * dpos[c] * cw;
          float dwt[3] = {dw[0][i] * w[1][j] * w[2][k] * inv_dx, w[0][i] * dw[1][j] * w[2][k] * inv_dx,
                          w[0][i] * w[1][j] * dw[2][k] * inv_dx};
          for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) nF[r * 3 + c] += gv[r] * dwt[c];
        }
    for (int d = 0; d < 3; ++d) {
      s->v[p * 3 + d] = nv[d];
      s->x[p * 3 + d] += dt * nv[d];
    }
    memcpy(s->C + p * 9, nC, 36);
    float A[9];
    for (int i = 0; i < 9; ++i) A[i] = ((i % 4) == 0 ? 1.0f : 0.0f) + nF[i] * dt;
    mm3(A, s->F + p * 9, s->F_trial + p * 9);
  }
}

/* ImpulseBC.apply, boundary_conditions.py:41-45 */
void om_impulses(om_state* s, int n_imp, const om_impulse* imp, const int32_t* active) {
  for (int b = 0; b < n_imp; ++b) {
    if (!active[b]) continue;
    const om_impulse* im = &imp[b];
#pragma omp parallel for schedule(static)
    for (int p = 0; p < s->n; ++p) {
      int in = 1;
      for (int d = 0; d < 3; ++d) in &= fabsf(s->x[p * 3 + d] - im->center[d]) < im->size[d];
      if (in)
        for (int d = 0; d < 3; ++d) s->v[p * 3 + d] = s->v[p * 3 + d] + im->force[d] / s->mass[p] * im->substep_dt;
    }
  }
}

/* threads the substep uses (1 in the serial checker build) */
int om_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* MPM_Simulator.p2g2p, solver.py:27-52 */
void om_substep(om_state* s, float dt, int n_imp, const om_impulse* imp, const int32_t* imp_active,
                int n_ops, const om_gridop* ops, const int32_t* op_active) {
  size_t nn = (size_t)s->ng * s->ng * s->ng;
  memset(s->gm, 0, nn * sizeof(float));
  memset(s->gv_in, 0, nn * 3 * sizeof(float));
  memset(s->gv_out, 0, nn * 3 * sizeof(float));
  om_impulses(s, n_imp, imp, imp_active);
  om_stress(s, dt);
  om_p2g(s, dt);
  om_grid_normalize(s, dt);
  om_grid_ops(s, n_ops, ops, op_active);
  om_g2p(s, dt);
}

/* MPM_Simulator.postprocess, solver.py:135-137 -> utils.py:376-433 */
void om_postprocess(om_state* s) {
  for (int p = 0; p < s->n; ++p) {
    const float* F = s->F_trial + p * 9;
    const float* a = s->init_cov + p * 6;
    float A[9] = {a[0], a[1], a[2], a[1], a[3], a[4], a[2], a[4], a[5]};
    float T[9], Cv[9];
    mm3(F, A, T);
    mmT3(T, F, Cv);
    float* c = s->cov + p * 6;
    c[0] = Cv[0]; c[1] = Cv[1]; c[2] = Cv[2]; c[3] = Cv[4]; c[4] = Cv[5]; c[5] = Cv[8];
    float U[9], V[9], sg[3];
    om_svd3(F, U, sg, V);
    if (det3(U) < 0.f) { U[2] = -U[2]; U[5] = -U[5]; U[8] = -U[8]; }
    if (det3(V) < 0.f) { V[2] = -V[2]; V[5] = -V[5]; V[8] = -V[8]; }
    float R[9];
    mmT3(U, V, R);
    float* Ro = s->R + p * 9;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Ro[i * 3 + j] = R[j * 3 + i];
  }
}

/*
 * diff_oracle.c -- CPU restatement of the reference's differentiable MPM path
 * (TEST INFRASTRUCTURE ONLY; see oracle.h).
 *
 * Forward (MPM_Simulator.p2g2p_forward, solver.py:54-69):
 *   compute_stress_from_F_opt  utils.py:56-76   (StVK on Green strain, J clamp)
 *   p2g_opt                    utils.py:136-174
 *   grid_normalization_and_gravity utils.py:177-183
 *   grid_postprocess[0].apply  boundary_conditions.py:23-27 (sticky ground /
 *                              first fixed cube; only entry 0, unconditionally)
 *   g2p_opt                    utils.py:284-347
 *   compute_cov_from_F_opt     utils.py:435-467 (from level 30)
 * State levels s = 0..L-1 (MPM_state_opt, model.py:135-167).
 *
 * Backward (p2g2p_backward, solver.py:71-90; postprocess_backward :170-171;
 * learn :92-108) restates what Taichi 1.5's reverse-mode autodiff computes for
 * those kernels, including the reference's accumulation behaviour:
 *   - adjoints accumulate (+=) and are cleared only by clear_grads;
 *   - the grid adjoints (v_in, v_out) are NOT cleared between substeps, so a
 *     substep's backward also carries the grid adjoints of later substeps;
 *   - grid_mass has no adjoint (the m-path of p2g/normalisation is dropped);
 *   - BasicBC.apply.grad is a no-op (the store of a constant has no input) and
 *     runs after the normalisation adjoint anyway;
 *   - compute_mu_lam_from_E_nu.grad runs every substep on the accumulated mu/lam
 *     adjoints (logE/y adjoints grow triangularly over the 30 substeps).
 * Math is the analytic chain rule of the forward expressions in f32.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static inline float* lv(float* base, int s, int n, int width) { return base + (size_t)s * n * width; }

static void bsp(const float x[3], float inv_dx, int base[3], float fx[3], float w[3][3], float dw[3][3]) {
  for (int d = 0; d < 3; ++d) {
    float gp = x[d] * inv_dx;
    base[d] = (int)(gp - 0.5f);
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
static const float kDDW[3] = {1.0f, -2.0f, 1.0f}; /* d(dw)/dfx */

/* The reference's _opt kernels index the grid without a range check
 * (utils.py:57-76, Taichi debug=False, main.py:28): an index outside the grid
 * is undefined behaviour there.  The debug build (-DOM_DEBUG: make asan /
 * make debug) stops at one, as Taichi's debug mode would. */
#ifdef OM_DEBUG
#include <stdio.h>
static inline size_t node(int ng, int ix, int iy, int iz) {
  if (ix < 0 || iy < 0 || iz < 0 || ix >= ng || iy >= ng || iz >= ng) {
    fprintf(stderr, "diff oracle: grid node (%d, %d, %d) outside the %d^3 grid\n", ix, iy, iz, ng);
    abort();
  }
  return ((size_t)ix * ng + iy) * ng + iz;
}
#else
static inline size_t node(int ng, int ix, int iy, int iz) { return ((size_t)ix * ng + iy) * ng + iz; }
#endif

/* compute_mu_lam_from_E_nu, utils.py:349-362 */
void od_mu_lam(od_state* s) {
  for (int p = 0; p < s->n; ++p) {
    float E = powf(10.0f, s->logE[p]);
    float nu = 0.49f / (1.0f + expf(-s->y[p]));
    s->mu[p] = E / (2.0f * (1.0f + nu));
    s->lam[p] = E * nu / ((1.0f + nu) * (1.0f - 2.0f * nu));
  }
}

/* ------------------------------------------------------------- forward --- */
static void stress_opt(od_state* st, int s) {
  for (int p = 0; p < st->n; ++p) {
    const float* F = lv(st->F, s, st->n, 9) + p * 9;
    float J = F[0] * (F[4] * F[8] - F[5] * F[7]) - F[1] * (F[3] * F[8] - F[5] * F[6]) + F[2] * (F[3] * F[7] - F[4] * F[6]);
    if (fabsf(J) < 1e-2f) J = 1e-2f * (J > 0.f ? 1.f : (J < 0.f ? -1.f : 0.f));
    float E[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        float ftf = F[0 * 3 + i] * F[0 * 3 + j] + F[1 * 3 + i] * F[1 * 3 + j] + F[2 * 3 + i] * F[2 * 3 + j];
        E[i * 3 + j] = 0.5f * (ftf - (i == j ? 1.f : 0.f));
      }
    const float mu = st->mu[p], lam = st->lam[p];
    const float tr = E[0] + E[4] + E[8];
    float S[9];
    for (int i = 0; i < 9; ++i) S[i] = 2.0f * mu * E[i] + ((i % 4) == 0 ? lam * tr : 0.f);
    float FS[9], sig[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) FS[i * 3 + j] = F[i * 3 + 0] * S[0 * 3 + j] + F[i * 3 + 1] * S[1 * 3 + j] + F[i * 3 + 2] * S[2 * 3 + j];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        sig[i * 3 + j] = (FS[i * 3 + 0] * F[j * 3 + 0] + FS[i * 3 + 1] * F[j * 3 + 1] + FS[i * 3 + 2] * F[j * 3 + 2]) / J;
    memcpy(lv(st->stress, s, st->n, 9) + p * 9, sig, sizeof sig);
  }
}

static void p2g_opt(od_state* st, float dt, int s) {
  const int ng = st->ng;
  for (int p = 0; p < st->n; ++p) {
    const float* x = lv(st->x, s, st->n, 3) + p * 3;
    const float* v = lv(st->v, s, st->n, 3) + p * 3;
    const float* C = lv(st->C, s, st->n, 9) + p * 9;
    const float* sg = lv(st->stress, s, st->n, 9) + p * 9;
    int base[3];
    float fx[3], w[3][3], dw[3][3];
    bsp(x, st->inv_dx, base, fx, w, dw);
    const float m = st->mass[p], vol = st->vol[p];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        for (int k = 0; k < 3; ++k) {
          const int o[3] = {i, j, k};
          float dpos[3];
          for (int d = 0; d < 3; ++d) dpos[d] = ((float)o[d] - fx[d]) * st->dx;
          const float weight = w[0][i] * w[1][j] * w[2][k];
          const float gw[3] = {st->inv_dx * dw[0][i] * w[1][j] * w[2][k], st->inv_dx * w[0][i] * dw[1][j] * w[2][k],
                               st->inv_dx * w[0][i] * w[1][j] * dw[2][k]};
          const size_t g = node(ng, base[0] + i, base[1] + j, base[2] + k);
          for (int r = 0; r < 3; ++r) {
            const float cd = C[r * 3 + 0] * dpos[0] + C[r * 3 + 1] * dpos[1] + C[r * 3 + 2] * dpos[2];
            const float ef = -vol * (sg[r * 3 + 0] * gw[0] + sg[r * 3 + 1] * gw[1] + sg[r * 3 + 2] * gw[2]);
            st->gv_in[g * 3 + r] += weight * m * (v[r] + cd) + dt * ef;
          }
          st->gm[g] += weight * m;
        }
  }
}

static void grid_update(od_state* st, float dt) {
  const int ng = st->ng;
  const size_t nn = (size_t)ng * ng * ng;
  for (size_t g = 0; g < nn; ++g)
    if (st->gm[g] > 1e-15f)
      for (int d = 0; d < 3; ++d) st->gv_out[g * 3 + d] = st->gv_in[g * 3 + d] / st->gm[g] + dt * st->gravity[d];
  if (st->n_box > 0) { /* grid_postprocess[0].apply: BasicBC.apply, unconditionally */
    for (int i = 0; i < ng; ++i)
      for (int j = 0; j < ng; ++j)
        for (int k = 0; k < ng; ++k) {
          const float px[3] = {(float)i * st->dx, (float)j * st->dx, (float)k * st->dx};
          int in = 1;
          for (int d = 0; d < 3; ++d) in &= fabsf(px[d] - st->box_c[d]) < st->box_s[d];
          if (in) {
            const size_t g = node(ng, i, j, k);
            st->gv_out[g * 3 + 0] = st->gv_out[g * 3 + 1] = st->gv_out[g * 3 + 2] = 0.f;
          }
        }
  }
}

static void g2p_opt(od_state* st, float dt, int s) {
  const int ng = st->ng, n = st->n;
  for (int p = 0; p < n; ++p) {
    const float* x = lv(st->x, s, n, 3) + p * 3;
    const float* F = lv(st->F, s, n, 9) + p * 9;
    int base[3];
    float fx[3], w[3][3], dw[3][3];
    bsp(x, st->inv_dx, base, fx, w, dw);
    float nv[3] = {0}, nC[9] = {0}, nF[9] = {0};
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        for (int k = 0; k < 3; ++k) {
          const int o[3] = {i, j, k};
          float dpos[3];
          for (int d = 0; d < 3; ++d) dpos[d] = (float)o[d] - fx[d];
          const float weight = w[0][i] * w[1][j] * w[2][k];
          const float* gv = st->gv_out + node(ng, base[0] + i, base[1] + j, base[2] + k) * 3;
          const float gw[3] = {st->inv_dx * dw[0][i] * w[1][j] * w[2][k], st->inv_dx * w[0][i] * dw[1][j] * w[2][k],
                               st->inv_dx * w[0][i] * w[1][j] * dw[2][k]};
          for (int r = 0; r < 3; ++r) {
            nv[r] += gv[r] * weight;
            for (int c = 0; c < 3; ++c) {
              nC[r * 3 + c] += gv[r] * dpos[c] * (weight * st->inv_dx * 4.0f);
              nF[r * 3 + c] += gv[r] * gw[c];
            }
          }
        }
    float* x1 = lv(st->x, s + 1, n, 3) + p * 3;
    for (int d = 0; d < 3; ++d) {
      lv(st->v, s + 1, n, 3)[p * 3 + d] = nv[d];
      x1[d] = x[d] + dt * nv[d];
    }
    memcpy(lv(st->C, s + 1, n, 9) + p * 9, nC, sizeof nC);
    float* F1 = lv(st->F, s + 1, n, 9) + p * 9;
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        float acc = 0.f;
        for (int q = 0; q < 3; ++q) acc += ((r == q ? 1.f : 0.f) + nF[r * 3 + q] * dt) * F[q * 3 + c];
        F1[r * 3 + c] = acc;
      }
  }
}

static void reset_grid(od_state* st) {
  const size_t nn = (size_t)st->ng * st->ng * st->ng;
  memset(st->gm, 0, nn * sizeof(float));
  memset(st->gv_in, 0, nn * 3 * sizeof(float));
  memset(st->gv_out, 0, nn * 3 * sizeof(float));
}

void od_substep_forward(od_state* st, float dt, int s) {
  reset_grid(st);
  stress_opt(st, s);
  p2g_opt(st, dt, s);
  grid_update(st, dt);
  g2p_opt(st, dt, s);
}

void od_cov_forward(od_state* st) {
  const int n = st->n;
  for (int p = 0; p < n; ++p) {
    const float* F = lv(st->F, st->L - 1, n, 9) + p * 9;
    const float* a = st->init_cov + p * 6;
    const float A[9] = {a[0], a[1], a[2], a[1], a[3], a[4], a[2], a[4], a[5]};
    float FA[9], M[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) FA[i * 3 + j] = F[i * 3 + 0] * A[0 * 3 + j] + F[i * 3 + 1] * A[1 * 3 + j] + F[i * 3 + 2] * A[2 * 3 + j];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) M[i * 3 + j] = FA[i * 3 + 0] * F[j * 3 + 0] + FA[i * 3 + 1] * F[j * 3 + 1] + FA[i * 3 + 2] * F[j * 3 + 2];
    float* c = st->cov + p * 6;
    c[0] = M[0]; c[1] = M[1]; c[2] = M[2]; c[3] = M[4]; c[4] = M[5]; c[5] = M[8];
  }
}

/* ------------------------------------------------------------ backward --- */
/* compute_cov_from_F_opt.grad: cov (upper 6 of F A F^T) -> F[L-1] */
void od_cov_backward(od_state* st) {
  const int n = st->n;
  for (int p = 0; p < n; ++p) {
    const float* F = lv(st->F, st->L - 1, n, 9) + p * 9;
    float* gF = lv(st->gF, st->L - 1, n, 9) + p * 9;
    const float* a = st->init_cov + p * 6;
    const float A[9] = {a[0], a[1], a[2], a[1], a[3], a[4], a[2], a[4], a[5]};
    const float* gc = st->gcov + p * 6;
    /* only the upper entries were stored: their adjoint, lower ones 0 */
    const float G[9] = {gc[0], gc[1], gc[2], 0.f, gc[3], gc[4], 0.f, 0.f, gc[5]};
    /* M = F A F^T: dF = G F A^T + G^T F A */
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        float acc = 0.f;
        for (int k = 0; k < 3; ++k)
          for (int l = 0; l < 3; ++l) acc += G[i * 3 + k] * F[k * 3 + l] * A[j * 3 + l] + G[k * 3 + i] * F[k * 3 + l] * A[l * 3 + j];
        gF[i * 3 + j] += acc;
      }
  }
}

/* adjoint of weight / grad-weight w.r.t. fx (d = axis) */
static void weight_fx_adjoint(const float w[3][3], const float dw[3][3], int i, int j, int k, float inv_dx,
                              float g_weight, const float g_gw[3], float gfx[3]) {
  const int o[3] = {i, j, k};
  /* weight = w0 w1 w2 ; gw_c = inv_dx * prod_d (c == d ? dw_d : w_d) */
  for (int d = 0; d < 3; ++d) {
    float dweight = 1.f;
    for (int e = 0; e < 3; ++e) dweight *= (e == d) ? dw[e][o[e]] : w[e][o[e]];
    float acc = g_weight * dweight;
    for (int c = 0; c < 3; ++c) {
      float t = inv_dx;
      for (int e = 0; e < 3; ++e) {
        if (e == c && e == d) t *= kDDW[o[e]];
        else if (e == c || e == d) t *= dw[e][o[e]];
        else t *= w[e][o[e]];
      }
      acc += g_gw[c] * t;
    }
    gfx[d] += acc;
  }
}

static void g2p_opt_bwd(od_state* st, float dt, int s) {
  const int ng = st->ng, n = st->n;
  for (int p = 0; p < n; ++p) {
    const float* x = lv(st->x, s, n, 3) + p * 3;
    const float* F = lv(st->F, s, n, 9) + p * 9;
    int base[3];
    float fx[3], w[3][3], dw[3][3];
    bsp(x, st->inv_dx, base, fx, w, dw);
    /* recompute new_F (needed for the F adjoint) */
    float nF[9] = {0};
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        for (int k = 0; k < 3; ++k) {
          const float* gv = st->gv_out + node(ng, base[0] + i, base[1] + j, base[2] + k) * 3;
          const float gw[3] = {st->inv_dx * dw[0][i] * w[1][j] * w[2][k], st->inv_dx * w[0][i] * dw[1][j] * w[2][k],
                               st->inv_dx * w[0][i] * w[1][j] * dw[2][k]};
          for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) nF[r * 3 + c] += gv[r] * gw[c];
        }
    const float* gx1 = lv(st->gx, s + 1, n, 3) + p * 3;
    const float* gv1 = lv(st->gv, s + 1, n, 3) + p * 3;
    const float* gC1 = lv(st->gC, s + 1, n, 9) + p * 9;
    const float* gF1 = lv(st->gF, s + 1, n, 9) + p * 9;
    float* gx0 = lv(st->gx, s, n, 3) + p * 3;
    float* gF0 = lv(st->gF, s, n, 9) + p * 9;
    /* x1 = x0 + dt nv ; v1 = nv */
    float g_nv[3];
    for (int d = 0; d < 3; ++d) {
      gx0[d] += gx1[d];
      g_nv[d] = gv1[d] + dt * gx1[d];
    }
    /* F1 = (I + dt nF) F0 */
    float g_nF[9];
    for (int r = 0; r < 3; ++r)
      for (int q = 0; q < 3; ++q) {
        float acc = 0.f;
        for (int c = 0; c < 3; ++c) acc += gF1[r * 3 + c] * F[q * 3 + c];
        g_nF[r * 3 + q] = dt * acc;
      }
    for (int q = 0; q < 3; ++q)
      for (int c = 0; c < 3; ++c) {
        float acc = 0.f;
        for (int r = 0; r < 3; ++r) acc += ((r == q ? 1.f : 0.f) + nF[r * 3 + q] * dt) * gF1[r * 3 + c];
        gF0[q * 3 + c] += acc;
      }
    float gfx[3] = {0.f, 0.f, 0.f};
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        for (int k = 0; k < 3; ++k) {
          const int o[3] = {i, j, k};
          float dpos[3];
          for (int d = 0; d < 3; ++d) dpos[d] = (float)o[d] - fx[d];
          const float weight = w[0][i] * w[1][j] * w[2][k];
          const float gw[3] = {st->inv_dx * dw[0][i] * w[1][j] * w[2][k], st->inv_dx * w[0][i] * dw[1][j] * w[2][k],
                               st->inv_dx * w[0][i] * w[1][j] * dw[2][k]};
          const size_t g = node(ng, base[0] + i, base[1] + j, base[2] + k);
          const float* gv = st->gv_out + g * 3;
          const float cw = weight * st->inv_dx * 4.0f;
          float g_weight = 0.f, g_dpos[3] = {0.f, 0.f, 0.f}, g_gw[3] = {0.f, 0.f, 0.f};
          for (int r = 0; r < 3; ++r) {
            float g_g = g_nv[r] * weight;
            g_weight += g_nv[r] * gv[r];
            for (int c = 0; c < 3; ++c) {
              g_g += gC1[r * 3 + c] * dpos[c] * cw + g_nF[r * 3 + c] * gw[c];
              g_weight += gC1[r * 3 + c] * gv[r] * dpos[c] * st->inv_dx * 4.0f;
              g_dpos[c] += gC1[r * 3 + c] * gv[r] * cw;
              g_gw[c] += g_nF[r * 3 + c] * gv[r];
            }
            st->g_gv_out[g * 3 + r] += g_g;
          }
          weight_fx_adjoint(w, dw, i, j, k, st->inv_dx, g_weight, g_gw, gfx);
          for (int d = 0; d < 3; ++d) gfx[d] -= g_dpos[d];
        }
    for (int d = 0; d < 3; ++d) gx0[d] += gfx[d] * st->inv_dx;
  }
}

static void grid_update_bwd(od_state* st) {
  const size_t nn = (size_t)st->ng * st->ng * st->ng;
  for (size_t g = 0; g < nn; ++g)
    if (st->gm[g] > 1e-15f)
      for (int d = 0; d < 3; ++d) st->g_gv_in[g * 3 + d] += st->g_gv_out[g * 3 + d] / st->gm[g];
  if (st->g_gm) /* test-only exact mass adjoint of v_out = v_in / m */
    for (size_t g = 0; g < nn; ++g) {
      float acc = 0.f;
      if (st->gm[g] > 1e-15f)
        for (int d = 0; d < 3; ++d) acc -= st->g_gv_out[g * 3 + d] * st->gv_in[g * 3 + d] / (st->gm[g] * st->gm[g]);
      st->g_gm[g] = acc;
    }
  /* BasicBC.apply.grad: adjoint of storing a constant -- nothing */
}

static void p2g_opt_bwd(od_state* st, float dt, int s) {
  const int ng = st->ng, n = st->n;
  for (int p = 0; p < n; ++p) {
    const float* x = lv(st->x, s, n, 3) + p * 3;
    const float* v = lv(st->v, s, n, 3) + p * 3;
    const float* C = lv(st->C, s, n, 9) + p * 9;
    const float* sg = lv(st->stress, s, n, 9) + p * 9;
    float* gx = lv(st->gx, s, n, 3) + p * 3;
    float* gvp = lv(st->gv, s, n, 3) + p * 3;
    float* gC = lv(st->gC, s, n, 9) + p * 9;
    float* gS = lv(st->gstress, s, n, 9) + p * 9;
    int base[3];
    float fx[3], w[3][3], dw[3][3];
    bsp(x, st->inv_dx, base, fx, w, dw);
    const float m = st->mass[p], vol = st->vol[p];
    float gfx[3] = {0.f, 0.f, 0.f};
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        for (int k = 0; k < 3; ++k) {
          const int o[3] = {i, j, k};
          float dpos[3];
          for (int d = 0; d < 3; ++d) dpos[d] = ((float)o[d] - fx[d]) * st->dx;
          const float weight = w[0][i] * w[1][j] * w[2][k];
          const float gw[3] = {st->inv_dx * dw[0][i] * w[1][j] * w[2][k], st->inv_dx * w[0][i] * dw[1][j] * w[2][k],
                               st->inv_dx * w[0][i] * w[1][j] * dw[2][k]};
          const size_t gi = node(ng, base[0] + i, base[1] + j, base[2] + k);
          const float* G = st->g_gv_in + gi * 3;
          float g_weight = st->g_gm ? st->g_gm[gi] * m : 0.f, g_dpos[3] = {0.f, 0.f, 0.f}, g_gw[3] = {0.f, 0.f, 0.f};
          for (int r = 0; r < 3; ++r) {
            const float cd = C[r * 3 + 0] * dpos[0] + C[r * 3 + 1] * dpos[1] + C[r * 3 + 2] * dpos[2];
            gvp[r] += weight * m * G[r];
            g_weight += m * G[r] * (v[r] + cd);
            for (int c = 0; c < 3; ++c) {
              gC[r * 3 + c] += weight * m * G[r] * dpos[c];
              g_dpos[c] += weight * m * G[r] * C[r * 3 + c];
              gS[r * 3 + c] += -dt * vol * G[r] * gw[c];
              g_gw[c] += -dt * vol * G[r] * sg[r * 3 + c];
            }
          }
          weight_fx_adjoint(w, dw, i, j, k, st->inv_dx, g_weight, g_gw, gfx);
          for (int d = 0; d < 3; ++d) gfx[d] -= st->dx * g_dpos[d];
        }
    for (int d = 0; d < 3; ++d) gx[d] += gfx[d] * st->inv_dx;
  }
}

static void stress_opt_bwd(od_state* st, int s) {
  const int n = st->n;
  for (int p = 0; p < n; ++p) {
    const float* F = lv(st->F, s, n, 9) + p * 9;
    const float* G = lv(st->gstress, s, n, 9) + p * 9;
    float* gF = lv(st->gF, s, n, 9) + p * 9;
    float J = F[0] * (F[4] * F[8] - F[5] * F[7]) - F[1] * (F[3] * F[8] - F[5] * F[6]) + F[2] * (F[3] * F[7] - F[4] * F[6]);
    const int clamped = fabsf(J) < 1e-2f;
    if (clamped) J = 1e-2f * (J > 0.f ? 1.f : (J < 0.f ? -1.f : 0.f));
    float E[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        float ftf = F[0 * 3 + i] * F[0 * 3 + j] + F[1 * 3 + i] * F[1 * 3 + j] + F[2 * 3 + i] * F[2 * 3 + j];
        E[i * 3 + j] = 0.5f * (ftf - (i == j ? 1.f : 0.f));
      }
    const float mu = st->mu[p], lam = st->lam[p];
    const float tr = E[0] + E[4] + E[8];
    float S[9];
    for (int i = 0; i < 9; ++i) S[i] = 2.0f * mu * E[i] + ((i % 4) == 0 ? lam * tr : 0.f);
    /* A = F S F^T ; sigma = A / J */
    float A[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        float acc = 0.f;
        for (int k = 0; k < 3; ++k)
          for (int l = 0; l < 3; ++l) acc += F[i * 3 + k] * S[k * 3 + l] * F[j * 3 + l];
        A[i * 3 + j] = acc;
      }
    float GA[9], gJ = 0.f;
    for (int i = 0; i < 9; ++i) {
      GA[i] = G[i] / J;
      gJ -= G[i] * A[i] / (J * J);
    }
    /* dA = dF S F^T + F dS F^T + F S dF^T */
    float GS[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        float a1 = 0.f, a2 = 0.f;
        for (int k = 0; k < 3; ++k)
          for (int l = 0; l < 3; ++l) {
            a1 += GA[i * 3 + k] * F[k * 3 + l] * S[j * 3 + l];  /* (G_A F S^T)_ij */
            a2 += GA[k * 3 + i] * F[k * 3 + l] * S[l * 3 + j];  /* (G_A^T F S)_ij */
          }
        gF[i * 3 + j] += a1 + a2;
        float s3 = 0.f;
        for (int k = 0; k < 3; ++k)
          for (int l = 0; l < 3; ++l) s3 += F[k * 3 + i] * GA[k * 3 + l] * F[l * 3 + j]; /* (F^T G_A F)_ij */
        GS[i * 3 + j] = s3;
      }
    /* S = 2 mu E + lam tr(E) I */
    float trGS = GS[0] + GS[4] + GS[8], gE[9];
    float gmu = 0.f;
    for (int i = 0; i < 9; ++i) {
      gE[i] = 2.0f * mu * GS[i] + ((i % 4) == 0 ? lam * trGS : 0.f);
      gmu += 2.0f * GS[i] * E[i];
    }
    st->gmu[p] += gmu;
    st->glam[p] += tr * trGS;
    /* E = (F^T F - I)/2: dF = F (gE + gE^T) / 2 */
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        float acc = 0.f;
        for (int k = 0; k < 3; ++k) acc += F[i * 3 + k] * 0.5f * (gE[k * 3 + j] + gE[j * 3 + k]);
        gF[i * 3 + j] += acc;
      }
    if (!clamped) { /* dJ/dF = cofactor(F) */
      const float cof[9] = {F[4] * F[8] - F[5] * F[7], F[5] * F[6] - F[3] * F[8], F[3] * F[7] - F[4] * F[6],
                            F[2] * F[7] - F[1] * F[8], F[0] * F[8] - F[2] * F[6], F[1] * F[6] - F[0] * F[7],
                            F[1] * F[5] - F[2] * F[4], F[2] * F[3] - F[0] * F[5], F[0] * F[4] - F[1] * F[3]};
      for (int i = 0; i < 9; ++i) gF[i] += gJ * cof[i];
    }
  }
}

/* compute_mu_lam_from_E_nu.grad on the accumulated mu/lam adjoints */
static void mu_lam_bwd(od_state* st) {
  for (int p = 0; p < st->n; ++p) {
    const float E = powf(10.0f, st->logE[p]);
    const float ey = expf(-st->y[p]);
    const float nu = 0.49f / (1.0f + ey);
    const float dnu_dy = 0.49f * ey / ((1.0f + ey) * (1.0f + ey));
    const float D = (1.0f + nu) * (1.0f - 2.0f * nu);
    const float dmu_dE = 1.0f / (2.0f * (1.0f + nu));
    const float dmu_dnu = -E / (2.0f * (1.0f + nu) * (1.0f + nu));
    const float dlam_dE = nu / D;
    const float dlam_dnu = E * (1.0f + 2.0f * nu * nu) / (D * D);
    const float gE = st->gmu[p] * dmu_dE + st->glam[p] * dlam_dE;
    const float gnu = st->gmu[p] * dmu_dnu + st->glam[p] * dlam_dnu;
    st->glogE[p] += gE * E * 2.302585092994046f;
    st->gy[p] += gnu * dnu_dy;
  }
}

void od_substep_backward(od_state* st, float dt, int s) {
  /* recompute the grid of substep s (the history is not stored) */
  reset_grid(st);
  p2g_opt(st, dt, s);
  grid_update(st, dt);
  g2p_opt_bwd(st, dt, s);
  grid_update_bwd(st);
  p2g_opt_bwd(st, dt, s);
  stress_opt_bwd(st, s);
  mu_lam_bwd(st);
}

/* learn, solver.py:92-108: clipped SGD */
void od_learn(od_state* st) {
  for (int p = 0; p < st->n; ++p) {
    float a = st->glogE[p], b = st->gy[p];
    if (fabsf(a) > 1.0f) a = a > 0.f ? 1.0f : -1.0f;
    if (fabsf(b) > 1.0f) b = b > 0.f ? 1.0f : -1.0f;
    st->logE[p] -= 0.8f * a;
    st->y[p] -= 1.6f * b;
  }
}

/* cycle_init, model.py:216-223 */
void od_cycle_init(od_state* st) {
  const int n = st->n, L = st->L;
  memcpy(st->x, lv(st->x, L - 1, n, 3), sizeof(float) * 3 * n);
  memcpy(st->v, lv(st->v, L - 1, n, 3), sizeof(float) * 3 * n);
  memcpy(st->F, lv(st->F, L - 1, n, 9), sizeof(float) * 9 * n);
  memcpy(st->stress, lv(st->stress, L - 1, n, 9), sizeof(float) * 9 * n);
  memcpy(st->C, lv(st->C, L - 1, n, 9), sizeof(float) * 9 * n);
}

/* clear_grads: MPM_model.clear_grad + MPM_state_opt.clear_grad */
void od_clear_grads(od_state* st) {
  const int n = st->n, L = st->L;
  const size_t nn = (size_t)st->ng * st->ng * st->ng;
  memset(st->glogE, 0, sizeof(float) * n);
  memset(st->gy, 0, sizeof(float) * n);
  memset(st->gmu, 0, sizeof(float) * n);
  memset(st->glam, 0, sizeof(float) * n);
  memset(st->gx, 0, sizeof(float) * 3 * n * L);
  memset(st->gv, 0, sizeof(float) * 3 * n * L);
  memset(st->gF, 0, sizeof(float) * 9 * n * L);
  memset(st->gstress, 0, sizeof(float) * 9 * n * L);
  memset(st->gC, 0, sizeof(float) * 9 * n * L);
  memset(st->gcov, 0, sizeof(float) * 6 * n);
  memset(st->g_gv_in, 0, sizeof(float) * 3 * nn);
  memset(st->g_gv_out, 0, sizeof(float) * 3 * nn);
}

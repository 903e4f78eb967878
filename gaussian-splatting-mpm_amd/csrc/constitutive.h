// constitutive.h -- return mapping + Kirchhoff stress per material
// (mpm_solver/constitutive_models.py, dispatched as utils.py:13-54).
#pragma once
#include "mpm_common.h"
#include "svd3.h"

namespace gsmpm {

// ---------------------------------------------------- constitutive models --
// Material codes as template: 0 = jelly as written (zero stress),
// 1 metal, 2 sand, 3 foam, 4 = jelly with FCR (F3 fixed), 5 = the cohesive
// fluid of fluid_return_mapping (constitutive_models.py:142-213), which the
// reference defines but never dispatches (utils.py:13-54 has no branch for
// it); here it is paired with the StVK Kirchhoff stress its viscoplastic
// sibling (material 3) uses.
//
// The stress needs the SVD of the returned F (utils.py:32-52 takes a second
// ti.svd).  Where the return map left F unchanged that is the SVD it already
// took (the same input, so the same factors, bit for bit); where it set
// F = U diag(se) V^T the factors are U, se, V, and the stresses below are
// isotropic functions of F (any SVD of it gives the same U f(s) V^T), so the
// second SVD is skipped on both branches.  The difference from a fresh SVD of
// the rounded product is rounding-level.  Foam (material 3) forms its new F
// element-wise, which is no SVD of anything, so its plastic lanes
// take the second SVD.  GSMPM_SVD_REUSE=0 at build time: always two SVDs.
#ifndef GSMPM_SVD_REUSE
#define GSMPM_SVD_REUSE 1
#endif
// GSMPM_LOG_REUSE=0 (A/B): metal's stress takes its three logs again even
// where the return map kept F
#ifndef GSMPM_LOG_REUSE
#define GSMPM_LOG_REUSE 1
#endif
template <int MAT>
__device__ __forceinline__ void return_map_and_stress(float (&F)[3][3], float mu, float lam, float& yld, float dt,
                                                      const MatConsts& mc, float (&tau)[3][3]) {
  float U[3][3], V[3][3], s[3];
  bool fresh = false;  // F changed in a way U, s, V do not describe: take its SVD
  // metal whose F the return map left unchanged: the stress's log(max(s, 0.01))
  // and its StVK diagonal are the return map's eps and t3 (the same f32
  // operations on the same s, utils.py:23-38 vs constitutive_models.py:62-75)
  bool kept = false;
  float t3_k[3] = {0.f, 0.f, 0.f};
  constexpr bool kFast = MAT != 3;  // foam's plastic F depends on the SVD basis (svd3.h)
  if constexpr (MAT == 1) {
    // von_mises_return_mapping, constitutive_models.py:62-103
    svd3<kFast>(F, U, s, V);
    float eps[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) eps[d] = logf(fmaxf(s[d], 0.01f));
    const float tr = eps[0] + eps[1] + eps[2];
    const float temp = tr / 3.0f;
    float t3[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) t3[d] = 2.0f * mu * eps[d] + lam * tr * 1.0f;
    const float st = t3[0] + t3[1] + t3[2];
    float cond[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) cond[d] = t3[d] - st / 3.0f;
    const float cn = sqrtf(cond[0] * cond[0] + cond[1] * cond[1] + cond[2] * cond[2]);
    kept = !(cn > yld);
#pragma unroll
    for (int d = 0; d < 3; ++d) t3_k[d] = t3[d];
    if (cn > yld) {
      float eh[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) eh[d] = eps[d] - temp;
      const float ehn = sqrtf(eh[0] * eh[0] + eh[1] * eh[1] + eh[2] * eh[2]) + 1e-6f;
      const float dg = ehn - yld / (2.0f * mu);
      float se[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) se[d] = expf(eps[d] - (dg / ehn) * eh[d]);
      usv(U, se, V, F);
#pragma unroll
      for (int d = 0; d < 3; ++d) s[d] = se[d];
      if (mc.hardening == 1.0f) yld += 2.0f * mu * mc.xi * dg;
    }
  } else if constexpr (MAT == 2) {
    // sand_return_mapping, constitutive_models.py:105-140
    svd3<kFast>(F, U, s, V);
    float eps[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) eps[d] = logf(fmaxf(fabsf(s[d]), 1e-14f));
    const float tr = eps[0] + eps[1] + eps[2];
    float eh[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) eh[d] = eps[d] - tr / 3.0f;
    const float ehn = sqrtf(eh[0] * eh[0] + eh[1] * eh[1] + eh[2] * eh[2]);
    const float dg = ehn + (3.0f * lam + 2.0f * mu) / (2.0f * mu) * tr * mc.alpha;
    if (dg > 0.0f) {
      if (tr > 0.0f) {
        mmT(U, V, F);
#pragma unroll
        for (int d = 0; d < 3; ++d) s[d] = 1.0f;
      } else {
        float sn[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) sn[d] = expf(eps[d] - eh[d] * (dg / ehn));
        usv(U, sn, V, F);
#pragma unroll
        for (int d = 0; d < 3; ++d) s[d] = sn[d];
      }
    }
  } else if constexpr (MAT == 3) {
    // viscoplasticity_return_mapping_with_StVK, constitutive_models.py:216-259
    svd3<kFast>(F, U, s, V);
    float sg[3], eps[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      sg[d] = fmaxf(s[d], 0.01f);
      eps[d] = logf(sg[d]);
    }
    const float tr = eps[0] + eps[1] + eps[2];
    float stv[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) stv[d] = 2.0f * mu * (eps[d] - tr / 3.0f);
    const float stn = sqrtf(stv[0] * stv[0] + stv[1] * stv[1] + stv[2] * stv[2]);
    const float y = stn - 0.8f * sqrtf(2.0f / 3.0f) * yld;
    if (y > 0.0f) {
      const float mu_hat = mu * (sg[0] * sg[0] + sg[1] * sg[1] + sg[2] * sg[2]) / 3.0f;
      const float snn = stn - y / (1.0f + mc.pvisc * 2.0f / (2.0f * mu_hat * dt));
      // element-wise U * diag * V^T (constitutive_models.py:256)
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const float en = 1.0f / (2.0f * mu) * ((snn / stn) * stv[i]) + tr / 3.0f;
          const float se = (i == j) ? expf(en) : 0.0f;
          F[i][j] = U[i][j] * se * V[j][i];
        }
      fresh = true;
    }
  }
  else if constexpr (MAT == 5) {
    // fluid_return_mapping, constitutive_models.py:142-213
    svd3<kFast>(F, U, s, V);
    float eps[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) eps[d] = logf(fmaxf(fabsf(s[d]), 0.01f));
    const float tr = eps[0] + eps[1] + eps[2];
    float stv[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) stv[d] = 2.0f * mu * (eps[d] - tr / 3.0f);
    const float stn = sqrtf(stv[0] * stv[0] + stv[1] * stv[1] + stv[2] * stv[2]);
    const float y = stn - sqrtf(2.0f / 3.0f) * yld;
    if (y > 0.0f) {
      const float mu_hat = mu * (s[0] * s[0] + s[1] * s[1] + s[2] * s[2]) / 3.0f;
      const float pf = 1.0f + mc.pvisc / (2.0f * mu_hat * dt);
      const float snn = stn - y / pf;
      float se[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) se[d] = expf(1.0f / (2.0f * mu) * ((snn / stn) * stv[d]) + tr / 3.0f);
      usv(U, se, V, F);  // a true matrix product here (U @ sig_elastic @ V^T, :205)
#pragma unroll
      for (int d = 0; d < 3; ++d) s[d] = se[d];
    }
  }
  // Kirchhoff stress of the (returned) F, utils.py:32-52
  float T[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) T[i][j] = 0.0f;
  if constexpr (MAT != 0) {
    if (MAT == 4 || !GSMPM_SVD_REUSE || fresh) svd3<kFast>(F, U, s, V);
    if constexpr (MAT == 1 || MAT == 3 || MAT == 5) {
      // kirchoff_stress_StVK, constitutive_models.py:23-38
      float tv[3];
      if (MAT == 1 && GSMPM_SVD_REUSE && GSMPM_LOG_REUSE && kept) {
#pragma unroll
        for (int d = 0; d < 3; ++d) tv[d] = t3_k[d];
      } else {
        float ls[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) ls[d] = logf(fmaxf(s[d], 0.01f));
        const float lss = ls[0] + ls[1] + ls[2];
#pragma unroll
        for (int d = 0; d < 3; ++d) tv[d] = 2.0f * mu * ls[d] + lam * lss * 1.0f;
      }
      float W[3][3];
      usv(U, tv, V, W);
      mmT(W, F, T);
    } else if constexpr (MAT == 2) {
      // kirchoff_stress_Drucker_Prager, constitutive_models.py:41-58
      const float lss = logf(s[0]) + logf(s[1]) + logf(s[2]);
      float cv[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) cv[d] = 2.0f * mu * logf(s[d]) / s[d] + lam * lss / s[d];
      float W[3][3];
      usv(U, cv, V, W);
      mmT(W, F, T);
    } else if constexpr (MAT == 4) {
      // kirchoff_stress_FCR, constitutive_models.py:10-20
      const float J = det3(F);
      float R[3][3], D[3][3];
      mmT(U, V, R);
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) D[i][j] = 2.0f * mu * (F[i][j] - R[i][j]);
      mmT(D, F, T);
      const float l = lam * J * (J - 1.0f);
      T[0][0] += l;
      T[1][1] += l;
      T[2][2] += l;
    }
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) tau[i][j] = (T[i][j] + T[j][i]) / 2.0f;
}

}  // namespace gsmpm

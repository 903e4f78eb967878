// svd3.h -- 3x3 f32 SVD for the constitutive kernels, register-resident.
//
// Same published algorithm as Taichi's ti.svd for f32 (McAdams, Selle, Tamstorf,
// Teran, Sifakis 2011, "Computing the SVD of 3x3 matrices with minimal branching
// and elementary floating point operations"), which the reference calls at
// mpm_solver/utils.py:33,385 and constitutive_models.py:64,107,218:
//   1. Jacobi eigen-analysis of S = A^T A with approximate Givens quaternions,
//      5 sweeps of the (0,1),(1,2),(2,0) pivots (f32 setting);
//   2. V from the accumulated quaternion, B = A V;
//   3. sort B's columns by decreasing norm, negating the swapped-in column so
//      V stays a rotation;
//   4. Givens QR of B: U = G1 G2 G3, sigma = diag(R) (sigma3 carries sign(det A)).
// Written branch-free for the wavefront: every select is a v_cndmask.
#pragma once
#include <hip/hip_runtime.h>

namespace gsmpm {

// FAST: reciprocal square roots and square roots by the hardware
// instructions (v_rsq_f32 / v_sqrt_f32, ~1 ulp) instead of the correctly
// rounded sequences (27 / 18 VALU each, 25 per SVD).  The bare instructions
// are not used (round 3): at the BASELINE sizes the ~1 ulp per SVD put the plastic materials ~10x
// further from the oracle than the oracle is from itself under a reordered
// P2G sum (metal, 100k / 128^3, substep 100: F_trial 1.2e-4 with it, 1.7e-5
// without, reorder spread 1.5e-5; sand v 2.3e-3 vs 4.3e-4 vs 4.4e-4;
// tests/test_gpu_parity_long.py), for 2.3 us of k_fused<metal>.  Where a
// result depends on the SVD basis itself (foam's element-wise U * diag * V^T,
// SURVEY F13) the correctly rounded form is used regardless.
// GSMPM_SVD_FAST (build time) selects the FAST form:
//   2 (default, round 4): the hardware rsqrt refined by one Newton-Raphson
//     step (y (3 - x y^2) / 2, ~0.5 ulp) and sqrt as x * rsqrt plus one Heron
//     correction: 6 / 8 VALU instead of 27 / 18.  Not bit-identical to the
//     oracle's 1 / sqrtf, but metal and sand stay inside the long-horizon
//     spread; metal k_fused 25.7 -> 24.3 us, sim 3.86 -> 3.71 ms/frame
//     (tools/ab_libs.sh, profiles/r04/).
//   1: the bare hardware instructions (A/B; ~10x outside the spread, above).
//   0: the correctly rounded sequences (round 3's default; A/B).
#ifndef GSMPM_SVD_FAST
#define GSMPM_SVD_FAST 2
#endif
// The refined forms run for x in [2^-100, 2^100], where y0^2 and x y0^2 stay
// normal; anything else (0, subnormal, huge, inf, NaN, negative) takes the
// correctly rounded form on a branch the wave skips when no lane needs it:
// v_rsq_f32 flushes a subnormal input (rsq -> inf where 1 / sqrtf gives
// ~1e20), at 0 / inf the step's x y0^2 is NaN, and near FLT_MAX y0^2 is
// subnormal.  Foam's degenerate F reaches these in the Jacobi sweeps (its R
// came out NaN with the unguarded step).
constexpr float kNrLo = 7.88860905e-31f, kNrHi = 1.26765060e30f;  // 2^-100, 2^100
__device__ __forceinline__ float svd_rsqrt_nr(float x) {
  if (x >= kNrLo && x <= kNrHi) {
    const float y0 = __builtin_amdgcn_rsqf(x);
    return y0 * fmaf(-0.5f * x, y0 * y0, 1.5f);
  }
  return 1.0f / sqrtf(x);
}
__device__ __forceinline__ float svd_sqrt_nr(float x) {
  if (x >= kNrLo && x <= kNrHi) {
    const float y0 = __builtin_amdgcn_rsqf(x);
    const float y = y0 * fmaf(-0.5f * x, y0 * y0, 1.5f);
    const float s = x * y;
    return fmaf(0.5f * y, fmaf(-s, s, x), s);
  }
  return sqrtf(x);
}
template <bool FAST>
__device__ __forceinline__ float svd_rsqrt(float x) {
  if constexpr (FAST && GSMPM_SVD_FAST == 1) return __builtin_amdgcn_rsqf(x);
  if constexpr (FAST && GSMPM_SVD_FAST == 2) return svd_rsqrt_nr(x);
  return 1.0f / sqrtf(x);
}
template <bool FAST>
__device__ __forceinline__ float svd_sqrt(float x) {
  if constexpr (FAST && GSMPM_SVD_FAST == 1) return __builtin_amdgcn_sqrtf(x);
  if constexpr (FAST && GSMPM_SVD_FAST == 2) return svd_sqrt_nr(x);
  return sqrtf(x);
}

// GSMPM_SVD_TRIM (default 1, round 6): the quaternion and U updates skip the
// products with the zeros of their rotation or of the identity they start
// from.  Same operands and order for every non-zero term, so the same f32
// results for finite input (0: the plain forms, A/B).
#ifndef GSMPM_SVD_TRIM
#define GSMPM_SVD_TRIM 1
#endif

struct M3 {
  float m[3][3];
};

template <bool FAST>
__device__ __forceinline__ void svd_jacobi(float (&S)[3][3], float (&q)[4], int p, int r, bool first = false) {
  constexpr float kGamma = 5.828427124746190f;  // 3 + 2 sqrt(2)
  constexpr float kCStar = 0.923879532511287f;  // cos(pi/8)
  constexpr float kSStar = 0.382683432365090f;  // sin(pi/8)
  float ch = 2.0f * (S[p][p] - S[r][r]);
  float sh = S[r][p];
  const bool b = (kGamma * sh * sh) < (ch * ch);
  const float w = svd_rsqrt<FAST>(ch * ch + sh * sh);
  ch = b ? w * ch : kCStar;
  sh = b ? w * sh : kSStar;
  const float c = ch * ch - sh * sh, s = 2.0f * sh * ch;
  // S <- R^T S R with R the (p,r)-plane rotation [[c,-s],[s,c]]
  const int k = 3 - p - r;
  const float spp = S[p][p], srr = S[r][r], spr = S[p][r], spk = S[p][k], srk = S[r][k];
  const float npp = c * (c * spp + s * spr) + s * (c * spr + s * srr);
  const float nrr = -s * (-s * spp + c * spr) + c * (-s * spr + c * srr);
  const float npr = c * (-s * spp + c * spr) + s * (-s * spr + c * srr);
  const float npk = c * spk + s * srk;
  const float nrk = -s * spk + c * srk;
  S[p][p] = npp; S[r][r] = nrr;
  S[p][r] = npr; S[r][p] = npr;
  S[p][k] = npk; S[k][p] = npk;
  S[r][k] = nrk; S[k][r] = nrk;
  // q <- q * (ch, sh e_k)
  const float a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3];
  if constexpr (GSMPM_SVD_TRIM) {
    // The Hamilton product with the two zero components of (ch, sh e_k)
    // dropped: the full form's a * 0 terms are +-0, and x +- 0 = x, so for
    // finite q each component is the same two products and one add, rounded
    // identically.  The full form spends 16 mul + 12 add a rotation, the
    // compiler cannot fold a * 0 under IEEE semantics; this one 8 + 4.
    if (first) {  // q = (1, 0, 0, 0): the product is (ch, sh e_k) exactly
      q[0] = ch;
      q[1] = k == 0 ? sh : 0.f;
      q[2] = k == 1 ? sh : 0.f;
      q[3] = k == 2 ? sh : 0.f;
    } else if (k == 0) {
      q[0] = a0 * ch - a1 * sh;
      q[1] = a0 * sh + a1 * ch;
      q[2] = a2 * ch + a3 * sh;
      q[3] = -(a2 * sh) + a3 * ch;
    } else if (k == 1) {
      q[0] = a0 * ch - a2 * sh;
      q[1] = a1 * ch - a3 * sh;
      q[2] = a0 * sh + a2 * ch;
      q[3] = a1 * sh + a3 * ch;
    } else {
      q[0] = a0 * ch - a3 * sh;
      q[1] = a1 * ch + a2 * sh;
      q[2] = -(a1 * sh) + a2 * ch;
      q[3] = a0 * sh + a3 * ch;
    }
    return;
  }
  float rq[4] = {ch, 0.f, 0.f, 0.f};
  rq[1 + k] = sh;
  q[0] = a0 * rq[0] - a1 * rq[1] - a2 * rq[2] - a3 * rq[3];
  q[1] = a0 * rq[1] + a1 * rq[0] + a2 * rq[3] - a3 * rq[2];
  q[2] = a0 * rq[2] - a1 * rq[3] + a2 * rq[0] + a3 * rq[1];
  q[3] = a0 * rq[3] + a1 * rq[2] - a2 * rq[1] + a3 * rq[0];
}

__device__ __forceinline__ void svd_cond_swap(bool c, float (&B)[3][3], float (&V)[3][3], float (&rho)[3], int i, int j) {
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const float bi = B[r][i], bj = B[r][j];
    B[r][i] = c ? bj : bi;
    B[r][j] = c ? -bi : bj;
    const float vi = V[r][i], vj = V[r][j];
    V[r][i] = c ? vj : vi;
    V[r][j] = c ? -vi : vj;
  }
  const float ri = rho[i], rj = rho[j];
  rho[i] = c ? rj : ri;
  rho[j] = c ? ri : rj;
}

// one Givens step of the QR: rotates B's rows p, r and returns the rotation
template <bool FAST>
__device__ __forceinline__ void svd_qr_rot(float (&B)[3][3], int p, int r, float& c, float& s) {
  constexpr float kEps = 1.0e-12f;
  const float a1 = B[p][p], a2 = B[r][p];
  const float rho = svd_sqrt<FAST>(a1 * a1 + a2 * a2);
  float sh = rho > kEps ? a2 : 0.0f;
  float ch = fabsf(a1) + fmaxf(rho, kEps);
  const bool neg = a1 < 0.0f;
  const float t = sh;
  sh = neg ? ch : sh;
  ch = neg ? t : ch;
  const float w = svd_rsqrt<FAST>(ch * ch + sh * sh);
  ch *= w;
  sh *= w;
  c = ch * ch - sh * sh;
  s = 2.0f * sh * ch;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const float bp = B[p][j], br = B[r][j];
    B[p][j] = c * bp + s * br;
    B[r][j] = -s * bp + c * br;
  }
}
// U <- U G(p, r)
__device__ __forceinline__ void svd_qr_acc(float (&U)[3][3], int p, int r, float c, float s) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float up = U[i][p], ur = U[i][r];
    U[i][p] = c * up + s * ur;
    U[i][r] = -s * up + c * ur;
  }
}

// A = U diag(sig) V^T
template <bool FAST = true>
__device__ __forceinline__ void svd3(const float (&A)[3][3], float (&U)[3][3], float (&sig)[3], float (&V)[3][3]) {
  float S[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) S[i][j] = A[0][i] * A[0][j] + A[1][i] * A[1][j] + A[2][i] * A[2][j];
  float q[4] = {1.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int it = 0; it < 5; ++it) {
    svd_jacobi<FAST>(S, q, 0, 1, it == 0);
    svd_jacobi<FAST>(S, q, 1, 2);
    svd_jacobi<FAST>(S, q, 2, 0);
  }
  const float qn = svd_rsqrt<FAST>(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  const float w = q[0] * qn, x = q[1] * qn, y = q[2] * qn, z = q[3] * qn;
  V[0][0] = 1.f - 2.f * (y * y + z * z); V[0][1] = 2.f * (x * y - w * z); V[0][2] = 2.f * (x * z + w * y);
  V[1][0] = 2.f * (x * y + w * z); V[1][1] = 1.f - 2.f * (x * x + z * z); V[1][2] = 2.f * (y * z - w * x);
  V[2][0] = 2.f * (x * z - w * y); V[2][1] = 2.f * (y * z + w * x); V[2][2] = 1.f - 2.f * (x * x + y * y);
  float B[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) B[i][j] = A[i][0] * V[0][j] + A[i][1] * V[1][j] + A[i][2] * V[2][j];
  float rho[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) rho[c] = B[0][c] * B[0][c] + B[1][c] * B[1][c] + B[2][c] * B[2][c];
  svd_cond_swap(rho[0] < rho[1], B, V, rho, 0, 1);
  svd_cond_swap(rho[0] < rho[2], B, V, rho, 0, 2);
  svd_cond_swap(rho[1] < rho[2], B, V, rho, 1, 2);
  float c1, s1, c2, s2, c3, s3;
  svd_qr_rot<FAST>(B, 0, 1, c1, s1);
  svd_qr_rot<FAST>(B, 0, 2, c2, s2);
  svd_qr_rot<FAST>(B, 1, 2, c3, s3);
  if constexpr (GSMPM_SVD_TRIM) {
    // U = I G(0,1) G(0,2) with the identity's zeros and ones folded (each
    // entry the one product the plain form rounds; the rest are +-0 or x*1)
    U[0][0] = c2 * c1;  U[0][1] = -s1;  U[0][2] = -s2 * c1;
    U[1][0] = c2 * s1;  U[1][1] = c1;   U[1][2] = -s2 * s1;
    U[2][0] = s2;
    // G(1,2) on the rows with U[i][1] = -s1, c1 and row 2's (s2, 0, c2)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float up = U[i][1], ur = U[i][2];
      U[i][1] = c3 * up + s3 * ur;
      U[i][2] = -s3 * up + c3 * ur;
    }
    U[2][1] = s3 * c2;
    U[2][2] = c3 * c2;
  } else {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) U[i][j] = (i == j) ? 1.f : 0.f;
    svd_qr_acc(U, 0, 1, c1, s1);
    svd_qr_acc(U, 0, 2, c2, s2);
    svd_qr_acc(U, 1, 2, c3, s3);
  }
  sig[0] = B[0][0];
  sig[1] = B[1][1];
  sig[2] = B[2][2];
}

}  // namespace gsmpm

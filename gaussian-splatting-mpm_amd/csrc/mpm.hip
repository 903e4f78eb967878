// mpm.hip -- MI355X (gfx950) MLS-MPM substep for the PhysGaussian loop.
//
// Replaces the Taichi kernels the reference launches from
// MPM_Simulator.p2g2p (mpm_solver/solver.py:27-52): reset_grid_state,
// ImpulseBC.apply, compute_stress_from_F_trial, p2g, grid_normalization_and_gravity,
// BasicBC.apply / MPM_Collider.collide, g2p -- ~10 launches per substep -- by
// three fused kernels per substep, replayed from a cached hipGraph:
//
//   k_p2g   particle-parallel: impulse kick + return map + SVD stress +
//           APIC scatter of (m*v, m) into the node accumulator (f32 atomics)
//   k_grid  node-parallel over the live node box: normalise + gravity + the
//           grid BC list in order, writes v_out, and re-zeroes the accumulator
//           (that re-zero replaces reset_grid_state's three full fills)
//   k_g2p   particle-parallel: 27-node gather, v/x/C/F_trial update, and the
//           live-node box for the next substep (wave-reduced atomics)
//
// Layout in HBM: particle state is SoA (one f32 plane per scalar component,
// stride np = N rounded to 256) so every particle-parallel load/store is a
// coalesced dword per lane; particles are stored in Morton order of their cell
// (rows map back to the caller's order through `orig`).  The grid is a dense
// n^3 array of float4 {m*v, m} plus a float4 {v_out} array: 32 B/node.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <numeric>
#include <vector>

#include "common.h"
#include "svd3.h"

namespace gsmpm {

// ------------------------------------------------------------------ layout --
enum Plane : int {
  PX = 0,      // x y z
  PV = 3,      // v
  PC = 6,      // C (row-major 3x3)
  PF = 15,     // F_trial between substeps; return-mapped F inside p2g
  PMASS = 24,
  PVOL = 25,
  PMU = 26,
  PLAM = 27,
  PYLD = 28,
  PICOV = 29,  // init cov (upper 6)
  PCOV = 35,   // cov (upper 6)
  PR = 41,     // particle_R
  NPLANES = 50
};

constexpr int kMaxBC = 32;

struct Impulse {
  float c[3], s[3], f[3], sdt;
  int bit;
};
struct GridOp {
  int kind;  // 0 fixed cube, 1 plane collider
  int bit;
  float a[3], b[3], friction;
};
struct BcTable {
  int n_imp, n_ops;
  Impulse imp[kMaxBC];
  GridOp op[kMaxBC];
};

struct Particles {
  float* P;
  int n, np;
  __device__ __forceinline__ float& at(int plane, int i) const { return P[(size_t)plane * np + i]; }
};

struct GridDims {
  int ng;
  float dx, inv_dx;
};

struct MatConsts {
  float alpha, hardening, xi, pvisc;
};

// live node box [lo, hi] of the last G2P (int x3 lo, x3 hi), used by k_grid
struct Box {
  int lo[3], hi[3];
};

// -------------------------------------------------------- device helpers --
__device__ __forceinline__ void bspline(const float x[3], float inv_dx, int base[3], float fx[3], float w[3][3],
                                        float dw[3][3]) {
  // utils.py:92-109: base = (x*inv_dx - 0.5).cast(int) (truncation), quadratic B-spline
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const float gp = x[d] * inv_dx;
    base[d] = (int)(gp - 0.5f);
    fx[d] = gp - (float)base[d];
    const float wa = 1.5f - fx[d], wb = fx[d] - 1.0f, wc = fx[d] - 0.5f;
    w[d][0] = wa * wa * 0.5f;
    w[d][1] = 0.75f - wb * wb;
    w[d][2] = wc * wc * 0.5f;
    dw[d][0] = fx[d] - 1.5f;
    dw[d][1] = -2.0f * (fx[d] - 1.0f);
    dw[d][2] = fx[d] - 0.5f;
  }
}

__device__ __forceinline__ float det3(const float (&A)[3][3]) {
  return A[0][0] * (A[1][1] * A[2][2] - A[1][2] * A[2][1]) - A[0][1] * (A[1][0] * A[2][2] - A[1][2] * A[2][0]) +
         A[0][2] * (A[1][0] * A[2][1] - A[1][1] * A[2][0]);
}

// U diag(d) V^T
__device__ __forceinline__ void usv(const float (&U)[3][3], const float (&d)[3], const float (&V)[3][3],
                                    float (&O)[3][3]) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) O[i][j] = (U[i][0] * d[0]) * V[j][0] + (U[i][1] * d[1]) * V[j][1] + (U[i][2] * d[2]) * V[j][2];
}

// A B^T
__device__ __forceinline__ void mmT(const float (&A)[3][3], const float (&B)[3][3], float (&O)[3][3]) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) O[i][j] = A[i][0] * B[j][0] + A[i][1] * B[j][1] + A[i][2] * B[j][2];
}

// ---------------------------------------------------- constitutive models --
// Material codes as template: 0 = jelly as written (zero stress),
// 1 metal, 2 sand, 3 foam, 4 = jelly with FCR (F3 fixed).
template <int MAT>
__device__ __forceinline__ void return_map_and_stress(float (&F)[3][3], float mu, float lam, float& yld, float dt,
                                                      const MatConsts& mc, float (&tau)[3][3]) {
  float U[3][3], V[3][3], s[3];
  if constexpr (MAT == 1) {
    // von_mises_return_mapping, constitutive_models.py:62-103
    svd3(F, U, s, V);
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
      if (mc.hardening == 1.0f) yld += 2.0f * mu * mc.xi * dg;
    }
  } else if constexpr (MAT == 2) {
    // sand_return_mapping, constitutive_models.py:105-140
    svd3(F, U, s, V);
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
      } else {
        float sn[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) sn[d] = expf(eps[d] - eh[d] * (dg / ehn));
        usv(U, sn, V, F);
      }
    }
  } else if constexpr (MAT == 3) {
    // viscoplasticity_return_mapping_with_StVK, constitutive_models.py:216-259
    svd3(F, U, s, V);
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
    }
  }
  // Kirchhoff stress of the (returned) F, utils.py:32-52
  float T[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) T[i][j] = 0.0f;
  if constexpr (MAT != 0) {
    svd3(F, U, s, V);
    if constexpr (MAT == 1 || MAT == 3) {
      // kirchoff_stress_StVK, constitutive_models.py:23-38
      float tv[3];
      float ls[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) ls[d] = logf(fmaxf(s[d], 0.01f));
      const float lss = ls[0] + ls[1] + ls[2];
#pragma unroll
      for (int d = 0; d < 3; ++d) tv[d] = 2.0f * mu * ls[d] + lam * lss * 1.0f;
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

// ------------------------------------------------------------------- P2G --
template <int MAT>
__global__ __launch_bounds__(256) void k_p2g(Particles ps, GridDims g, const BcTable* __restrict__ bct,
                                             uint32_t mask, float dt, MatConsts mc, float4* __restrict__ gacc) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ps.n) return;
  float x[3], v[3], C[3][3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    x[d] = ps.at(PX + d, p);
    v[d] = ps.at(PV + d, p);
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) C[i / 3][i % 3] = ps.at(PC + i, p);
  const float m = ps.at(PMASS, p);

  // ImpulseBC.apply (boundary_conditions.py:41-45), host-decided activity.
  // G2P overwrites particle_vel, so the kick only needs to live in registers.
  if (mask) {
    const int ni = bct->n_imp;
    for (int b = 0; b < ni; ++b) {
      const Impulse& im = bct->imp[b];
      if (!((mask >> im.bit) & 1u)) continue;
      const bool in = fabsf(x[0] - im.c[0]) < im.s[0] && fabsf(x[1] - im.c[1]) < im.s[1] &&
                      fabsf(x[2] - im.c[2]) < im.s[2];
      if (in) {
#pragma unroll
        for (int d = 0; d < 3; ++d) v[d] = v[d] + im.f[d] / m * im.sdt;
      }
    }
  }

  // compute_stress_from_F_trial (utils.py:13-54), fused: stress never leaves registers
  float nvt[3][3];  // -vol * tau
  if constexpr (MAT != 0) {
    float F[3][3], tau[3][3];
#pragma unroll
    for (int i = 0; i < 9; ++i) F[i / 3][i % 3] = ps.at(PF + i, p);
    float yld = ps.at(PYLD, p);
    const float mu = ps.at(PMU, p), lam = ps.at(PLAM, p);
    return_map_and_stress<MAT>(F, mu, lam, yld, dt, mc, tau);
    if constexpr (MAT == 1 || MAT == 2 || MAT == 3) {
#pragma unroll
      for (int i = 0; i < 9; ++i) ps.at(PF + i, p) = F[i / 3][i % 3];
    }
    if constexpr (MAT == 1) ps.at(PYLD, p) = yld;
    const float nvol = -ps.at(PVOL, p);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) nvt[i][j] = nvol * tau[i][j];
  }

  int base[3];
  float fx[3], w[3][3], dw[3][3];
  bspline(x, g.inv_dx, base, fx, w, dw);
  const int ng = g.ng;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int ix = base[0] + i, iy = base[1] + j, iz = base[2] + k;
        const float dpos0 = ((float)i - fx[0]) * g.dx;
        const float dpos1 = ((float)j - fx[1]) * g.dx;
        const float dpos2 = ((float)k - fx[2]) * g.dx;
        const float weight = w[0][i] * w[1][j] * w[2][k];
        const float wm = weight * m;
        float add[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) add[r] = wm * (v[r] + (C[r][0] * dpos0 + C[r][1] * dpos1 + C[r][2] * dpos2));
        if constexpr (MAT != 0) {
          const float dw0 = dw[0][i] * w[1][j] * w[2][k] * g.inv_dx;
          const float dw1 = w[0][i] * dw[1][j] * w[2][k] * g.inv_dx;
          const float dw2 = w[0][i] * w[1][j] * dw[2][k] * g.inv_dx;
#pragma unroll
          for (int r = 0; r < 3; ++r) add[r] = add[r] + dt * (nvt[r][0] * dw0 + nvt[r][1] * dw1 + nvt[r][2] * dw2);
        }
        if ((unsigned)ix < (unsigned)ng && (unsigned)iy < (unsigned)ng && (unsigned)iz < (unsigned)ng) {
          float* cell = reinterpret_cast<float*>(gacc + (((size_t)ix * ng + iy) * ng + iz));
          unsafeAtomicAdd(cell + 0, add[0]);
          unsafeAtomicAdd(cell + 1, add[1]);
          unsafeAtomicAdd(cell + 2, add[2]);
          unsafeAtomicAdd(cell + 3, wm);
        }
      }
    }
  }
}

// ------------------------------------------------------------------ grid --
// grid_normalization_and_gravity (utils.py:177-183) + grid_postprocess list
// (solver.py:41-46): BasicBC.apply (boundary_conditions.py:23-27) and
// MPM_Collider.collide (collider.py:13-44), pointwise, in list order.
__global__ __launch_bounds__(256) void k_grid(float4* __restrict__ gacc, float4* __restrict__ gvel, GridDims g,
                                              const BcTable* __restrict__ bct, uint32_t mask, float dt, float gx,
                                              float gy, float gz, int keep, const Box* __restrict__ box,
                                              Box* __restrict__ next_box) {
  // reset the box the following G2P accumulates into (stream order makes this safe)
  if (blockIdx.x == 0 && threadIdx.x < 3) {
    next_box->lo[threadIdx.x] = INT_MAX;
    next_box->hi[threadIdx.x] = INT_MIN;
  }
  const int ng = g.ng;
  const int lo0 = box->lo[0], lo1 = box->lo[1], lo2 = box->lo[2];
  const int e0 = box->hi[0] - lo0 + 1, e1 = box->hi[1] - lo1 + 1, e2 = box->hi[2] - lo2 + 1;
  if (e0 <= 0 || e1 <= 0 || e2 <= 0) return;
  const long total = (long)e0 * e1 * e2;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int k = lo2 + (int)(t % e2);
    const long t2 = t / e2;
    const int j = lo1 + (int)(t2 % e1);
    const int i = lo0 + (int)(t2 / e1);
    const size_t idx = ((size_t)i * ng + j) * ng + k;
    const float4 a = gacc[idx];
    if (!keep) gacc[idx] = make_float4(0.f, 0.f, 0.f, 0.f);
    float v[3] = {0.f, 0.f, 0.f};
    if (a.w > 1e-15f) {
      v[0] = a.x / a.w + dt * gx;
      v[1] = a.y / a.w + dt * gy;
      v[2] = a.z / a.w + dt * gz;
      const int nops = bct->n_ops;
      for (int o = 0; o < nops; ++o) {
        const GridOp& op = bct->op[o];
        const float p0 = (float)i * g.dx, p1 = (float)j * g.dx, p2 = (float)k * g.dx;
        if (op.kind == 0) {
          if (!((mask >> op.bit) & 1u)) continue;
          if (fabsf(p0 - op.a[0]) < op.b[0] && fabsf(p1 - op.a[1]) < op.b[1] && fabsf(p2 - op.a[2]) < op.b[2]) {
            v[0] = 0.f;
            v[1] = 0.f;
            v[2] = 0.f;
          }
        } else {
          const float o0 = p0 - op.a[0], o1 = p1 - op.a[1], o2 = p2 - op.a[2];
          const float dot = o0 * op.b[0] + o1 * op.b[1] + o2 * op.b[2];
          if (dot < 0.0f) {
            const float nc = v[0] * op.b[0] + v[1] * op.b[1] + v[2] * op.b[2];
            const float mn = fminf(nc, 0.0f);
#pragma unroll
            for (int d = 0; d < 3; ++d) v[d] = v[d] - mn * op.b[d];
            const float len = sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
            if (nc < 0.0f && len > 1e-20f) {
              const float sc = fmaxf(0.0f, len + nc * op.friction);
#pragma unroll
              for (int d = 0; d < 3; ++d) v[d] = sc * (v[d] / len);
            }
#pragma unroll
            for (int d = 0; d < 3; ++d) v[d] = v[d] * 0.99f;
          }
        }
      }
    }
    gvel[idx] = make_float4(v[0], v[1], v[2], 0.f);
  }
}

// ------------------------------------------------------------------- G2P --
__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}

// g2p (utils.py:218-282) without the dead update_cov
__global__ __launch_bounds__(256) void k_g2p(Particles ps, GridDims g, const float4* __restrict__ gvel, float dt,
                                             Box* __restrict__ next_box) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = p < ps.n;
  int blo[3] = {INT_MAX, INT_MAX, INT_MAX}, bhi[3] = {INT_MIN, INT_MIN, INT_MIN};
  if (live) {
    float x[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) x[d] = ps.at(PX + d, p);
    int base[3];
    float fx[3], w[3][3], dw[3][3];
    bspline(x, g.inv_dx, base, fx, w, dw);
    const int ng = g.ng;
    float nv[3] = {0.f, 0.f, 0.f}, nC[3][3], nF[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        nC[r][c] = 0.f;
        nF[r][c] = 0.f;
      }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int ix = base[0] + i, iy = base[1] + j, iz = base[2] + k;
          float4 gv = make_float4(0.f, 0.f, 0.f, 0.f);
          if ((unsigned)ix < (unsigned)ng && (unsigned)iy < (unsigned)ng && (unsigned)iz < (unsigned)ng)
            gv = gvel[((size_t)ix * ng + iy) * ng + iz];
          const float gvv[3] = {gv.x, gv.y, gv.z};
          const float dpos[3] = {(float)i - fx[0], (float)j - fx[1], (float)k - fx[2]};
          const float weight = w[0][i] * w[1][j] * w[2][k];
          const float cw = weight * g.inv_dx * 4.0f;
          const float dwt[3] = {dw[0][i] * w[1][j] * w[2][k] * g.inv_dx, w[0][i] * dw[1][j] * w[2][k] * g.inv_dx,
                                w[0][i] * w[1][j] * dw[2][k] * g.inv_dx};
#pragma unroll
          for (int r = 0; r < 3; ++r) {
            nv[r] += gvv[r] * weight;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              nC[r][c] += gvv[r] * dpos[c] * cw;
              nF[r][c] += gvv[r] * dwt[c];
            }
          }
        }
      }
    }
    float F[3][3];
#pragma unroll
    for (int i = 0; i < 9; ++i) F[i / 3][i % 3] = ps.at(PF + i, p);
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      ps.at(PV + d, p) = nv[d];
      x[d] += dt * nv[d];
      ps.at(PX + d, p) = x[d];
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) ps.at(PC + i, p) = nC[i / 3][i % 3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float a0 = (r == 0 ? 1.0f : 0.0f) + nF[r][0] * dt;
        const float a1 = (r == 1 ? 1.0f : 0.0f) + nF[r][1] * dt;
        const float a2 = (r == 2 ? 1.0f : 0.0f) + nF[r][2] * dt;
        ps.at(PF + r * 3 + c, p) = a0 * F[0][c] + a1 * F[1][c] + a2 * F[2][c];
      }
    // node box touched by the next P2G (base..base+2 of the new position)
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const int b = (int)(x[d] * g.inv_dx - 0.5f);
      blo[d] = max(0, b);
      bhi[d] = min(g.ng - 1, b + 2);
    }
  }
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const int lo = wave_min(blo[d]);
    const int hi = wave_max(bhi[d]);
    if ((threadIdx.x & 63) == 0 && lo <= hi) {
      atomicMin(&next_box->lo[d], lo);
      atomicMax(&next_box->hi[d], hi);
    }
  }
}

// box ping-pong: the box written by G2P of substep s is read by k_grid of s+1
__global__ void k_box_reset(Box* b) {
  if (threadIdx.x < 3) {
    b->lo[threadIdx.x] = INT_MAX;
    b->hi[threadIdx.x] = INT_MIN;
  }
}

__global__ void k_box_full(Box* b, int ng) {
  if (threadIdx.x < 3) {
    b->lo[threadIdx.x] = 0;
    b->hi[threadIdx.x] = ng - 1;
  }
}

// particle box from the current positions (used after set/set_field)
__global__ __launch_bounds__(256) void k_box_from_x(Particles ps, GridDims g, Box* box) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  int blo[3] = {INT_MAX, INT_MAX, INT_MAX}, bhi[3] = {INT_MIN, INT_MIN, INT_MIN};
  if (p < ps.n) {
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const int b = (int)(ps.at(PX + d, p) * g.inv_dx - 0.5f);
      blo[d] = max(0, b);
      bhi[d] = min(g.ng - 1, b + 2);
    }
  }
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const int lo = wave_min(blo[d]);
    const int hi = wave_max(bhi[d]);
    if ((threadIdx.x & 63) == 0 && lo <= hi) {
      atomicMin(&box->lo[d], lo);
      atomicMax(&box->hi[d], hi);
    }
  }
}

// ------------------------------------------------------------ postprocess --
// compute_cov_from_F (utils.py:401-433) + compute_R_from_F (utils.py:376-398)
__global__ __launch_bounds__(256) void k_postprocess(Particles ps) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ps.n) return;
  float F[3][3];
#pragma unroll
  for (int i = 0; i < 9; ++i) F[i / 3][i % 3] = ps.at(PF + i, p);
  const float a0 = ps.at(PICOV + 0, p), a1 = ps.at(PICOV + 1, p), a2 = ps.at(PICOV + 2, p);
  const float a3 = ps.at(PICOV + 3, p), a4 = ps.at(PICOV + 4, p), a5 = ps.at(PICOV + 5, p);
  const float A[3][3] = {{a0, a1, a2}, {a1, a3, a4}, {a2, a4, a5}};
  float T[3][3], Cv[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) T[i][j] = F[i][0] * A[0][j] + F[i][1] * A[1][j] + F[i][2] * A[2][j];
  mmT(T, F, Cv);
  ps.at(PCOV + 0, p) = Cv[0][0];
  ps.at(PCOV + 1, p) = Cv[0][1];
  ps.at(PCOV + 2, p) = Cv[0][2];
  ps.at(PCOV + 3, p) = Cv[1][1];
  ps.at(PCOV + 4, p) = Cv[1][2];
  ps.at(PCOV + 5, p) = Cv[2][2];
  float U[3][3], V[3][3], s[3];
  svd3(F, U, s, V);
  if (det3(U) < 0.f) {
    U[0][2] = -U[0][2];
    U[1][2] = -U[1][2];
    U[2][2] = -U[2][2];
  }
  if (det3(V) < 0.f) {
    V[0][2] = -V[0][2];
    V[1][2] = -V[1][2];
    V[2][2] = -V[2][2];
  }
  float R[3][3];
  mmT(U, V, R);
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) ps.at(PR + i * 3 + j, p) = R[j][i];  // particle_R = (U V^T)^T
}

// ------------------------------------------------------------ init / io --
struct InitArgs {
  const float *x, *cov6, *vol, *v;
  const int* orig;
  float density, logE, y, yield0;
};

// MPM_state.__init__ (model.py:100-116) + compute_mu_lam_from_E_nu + mass
__global__ __launch_bounds__(256) void k_init(Particles ps, InitArgs a) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ps.n) return;
  const int o = a.orig[p];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    ps.at(PX + d, p) = a.x[(size_t)o * 3 + d];
    ps.at(PV + d, p) = a.v ? a.v[(size_t)o * 3 + d] : 0.0f;
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    ps.at(PC + i, p) = 0.0f;
    ps.at(PF + i, p) = (i % 4 == 0) ? 1.0f : 0.0f;
    ps.at(PR + i, p) = 0.0f;
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const float c = a.cov6[(size_t)o * 6 + i];
    ps.at(PICOV + i, p) = c;
    ps.at(PCOV + i, p) = c;
  }
  const float vol = a.vol[o];
  ps.at(PVOL, p) = vol;
  ps.at(PMASS, p) = a.density * vol;
  // utils.py:349-362 in f32
  const float E = powf(10.0f, a.logE);
  const float nu = 0.49f / (1.0f + expf(-a.y));
  ps.at(PMU, p) = E / (2.0f * (1.0f + nu));
  ps.at(PLAM, p) = E * nu / ((1.0f + nu) * (1.0f - 2.0f * nu));
  ps.at(PYLD, p) = a.yield0;
}

__global__ __launch_bounds__(256) void k_get(Particles ps, const int* __restrict__ orig, int plane0, int width,
                                             float* __restrict__ out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ps.n) return;
  const size_t o = (size_t)orig[p] * width;
  for (int j = 0; j < width; ++j) out[o + j] = ps.at(plane0 + j, p);
}

__global__ __launch_bounds__(256) void k_set(Particles ps, const int* __restrict__ orig, int plane0, int width,
                                             const float* __restrict__ in) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ps.n) return;
  const size_t o = (size_t)orig[p] * width;
  for (int j = 0; j < width; ++j) ps.at(plane0 + j, p) = in[o + j];
}

__global__ __launch_bounds__(256) void k_world_out(Particles ps, const int* __restrict__ orig, float half, float s,
                                                   float c0, float c1, float c2, int render, float* __restrict__ mo,
                                                   float* __restrict__ co) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ps.n) return;
  const size_t o = (size_t)orig[p];
  const float c[3] = {c0, c1, c2};
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    float w = (ps.at(PX + d, p) - half) / s + c[d];  // grid2world, transform_utils.py:19
    if (render) w = c[d] + (w - 1.0f) / 1.0f;        // render_frame, main.py:139-144 (scale 1.0)
    mo[o * 3 + d] = w;
  }
  const float ss = s * s;
#pragma unroll
  for (int i = 0; i < 6; ++i) co[o * 6 + i] = ps.at(PCOV + i, p) / ss;  // transform_utils.py:20
}

__global__ void k_grid_get(const float4* __restrict__ src, size_t nn, int which, float* __restrict__ out) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nn; i += (size_t)gridDim.x * blockDim.x) {
    const float4 a = src[i];
    if (which == 0) {
      out[i] = a.w;
    } else {
      out[i * 3 + 0] = a.x;
      out[i * 3 + 1] = a.y;
      out[i * 3 + 2] = a.z;
    }
  }
}

__global__ __launch_bounds__(256) void k_svd3(const float* __restrict__ A, int n, float* __restrict__ U,
                                              float* __restrict__ S, float* __restrict__ V) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float a[3][3], u[3][3], v[3][3], s[3];
#pragma unroll
  for (int k = 0; k < 9; ++k) a[k / 3][k % 3] = A[(size_t)i * 9 + k];
  svd3(a, u, s, v);
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    U[(size_t)i * 9 + k] = u[k / 3][k % 3];
    V[(size_t)i * 9 + k] = v[k / 3][k % 3];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) S[(size_t)i * 3 + k] = s[k];
}

template <int MAT>
__global__ __launch_bounds__(256) void k_constitutive(const float* __restrict__ Ft, int n, const float* __restrict__ mu,
                                                      const float* __restrict__ lam, float* __restrict__ yld, float dt,
                                                      MatConsts mc, float* __restrict__ Fo, float* __restrict__ To) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float F[3][3], tau[3][3];
#pragma unroll
  for (int k = 0; k < 9; ++k) F[k / 3][k % 3] = Ft[(size_t)i * 9 + k];
  float y = yld[i];
  return_map_and_stress<MAT>(F, mu[i], lam[i], y, dt, mc, tau);
  yld[i] = y;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    Fo[(size_t)i * 9 + k] = F[k / 3][k % 3];
    To[(size_t)i * 9 + k] = tau[k / 3][k % 3];
  }
}

// filling.py:11-24: floor(x / dx) cell counts (i32 atomics), vol = dx^3 / count
__global__ __launch_bounds__(256) void k_fill_count(const float* __restrict__ x, int n, int ng, float gdx,
                                                    int* __restrict__ cnt) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  int c[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) c[d] = (int)floorf(x[(size_t)p * 3 + d] / gdx);
  if ((unsigned)c[0] >= (unsigned)ng || (unsigned)c[1] >= (unsigned)ng || (unsigned)c[2] >= (unsigned)ng) return;
  atomicAdd(&cnt[((size_t)c[0] * ng + c[1]) * ng + c[2]], 1);
}

__global__ __launch_bounds__(256) void k_fill_vol(const float* __restrict__ x, int n, int ng, float gdx,
                                                  const int* __restrict__ cnt, float* __restrict__ vol) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  int c[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) c[d] = (int)floorf(x[(size_t)p * 3 + d] / gdx);
  if ((unsigned)c[0] >= (unsigned)ng || (unsigned)c[1] >= (unsigned)ng || (unsigned)c[2] >= (unsigned)ng) {
    vol[p] = 0.0f;
    return;
  }
  const float dx3 = gdx * gdx * gdx;
  vol[p] = dx3 / (float)cnt[((size_t)c[0] * ng + c[1]) * ng + c[2]];
}

}  // namespace gsmpm

// =================================================================== host ==
using namespace gsmpm;

struct gsmpm_mpm {
  gsmpm_mpm_params prm{};
  GridDims g{};
  MatConsts mc{};
  int mat_kernel = 0;  // template code of k_p2g
  int n = 0, np = 0;
  float* planes = nullptr;
  int* orig = nullptr;
  float4* gacc = nullptr;
  float4* gvel = nullptr;
  Box* boxes = nullptr;  // [0],[1] ping-pong live-node boxes, [2] whole grid
  int cur_box = 0;
  BcTable host_bc{};
  BcTable* dev_bc = nullptr;
  int n_bc = 0;
  bool has_particles = false;
  hipStream_t cap = nullptr;
  std::map<std::vector<uint32_t>, hipGraphExec_t> graphs;
  std::map<std::vector<uint32_t>, int> graph_box_parity;
};

namespace gsmpm {
static thread_local std::string g_err;
void set_error(const std::string& m) { g_err = m; }

static Particles particles_of(gsmpm_mpm* h) { return Particles{h->planes, h->n, h->np}; }

template <int MAT>
static void launch_p2g(gsmpm_mpm* h, uint32_t mask, float dt, hipStream_t st) {
  const int blocks = div_up(h->n, 256);
  hipLaunchKernelGGL(k_p2g<MAT>, dim3(blocks), dim3(256), 0, st, particles_of(h), h->g, h->dev_bc, mask, dt, h->mc,
                     h->gacc);
}

static int launch_substeps(gsmpm_mpm* h, float dt, int nsub, const uint32_t* bc, hipStream_t st, int& box_parity,
                           hipEvent_t* ev = nullptr, float* kernel_ms = nullptr) {
  const size_t nn = (size_t)h->g.ng * h->g.ng * h->g.ng;
  const bool keep = (h->prm.flags & GSMPM_FLAG_KEEP_GRID) != 0;
  const float gx = (float)h->prm.gravity[0], gy = (float)h->prm.gravity[1], gz = (float)h->prm.gravity[2];
  const int pblocks = div_up(h->n, 256);
  // the node box is small in practice; cap the grid-stride launch at 8 blocks/CU
  const int gblocks = (int)std::min<long>(div_up((long)nn, 256), 2048);
  for (int s = 0; s < nsub; ++s) {
    const uint32_t mask = bc ? bc[s] : 0xffffffffu;
    Box* cur = h->boxes + box_parity;
    Box* nxt = h->boxes + (box_parity ^ 1);
    if (keep) GSMPM_HIP(hipMemsetAsync(h->gacc, 0, nn * sizeof(float4), st));
    if (ev) GSMPM_HIP(hipEventRecord(ev[0], st));
    switch (h->mat_kernel) {
      case 0: launch_p2g<0>(h, mask, dt, st); break;
      case 1: launch_p2g<1>(h, mask, dt, st); break;
      case 2: launch_p2g<2>(h, mask, dt, st); break;
      case 3: launch_p2g<3>(h, mask, dt, st); break;
      default: launch_p2g<4>(h, mask, dt, st); break;
    }
    GSMPM_LAUNCH_CHECK();
    if (ev) GSMPM_HIP(hipEventRecord(ev[1], st));
    hipLaunchKernelGGL(k_grid, dim3(gblocks), dim3(256), 0, st, h->gacc, h->gvel, h->g, h->dev_bc, mask, dt, gx, gy,
                       gz, keep ? 1 : 0, keep ? h->boxes + 2 : cur, nxt);
    GSMPM_LAUNCH_CHECK();
    if (ev) GSMPM_HIP(hipEventRecord(ev[2], st));
    hipLaunchKernelGGL(k_g2p, dim3(pblocks), dim3(256), 0, st, particles_of(h), h->g, h->gvel, dt, nxt);
    GSMPM_LAUNCH_CHECK();
    if (ev) {
      GSMPM_HIP(hipEventRecord(ev[3], st));
      GSMPM_HIP(hipEventSynchronize(ev[3]));
      for (int k = 0; k < 3; ++k) {
        float ms = 0.f;
        GSMPM_HIP(hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
        kernel_ms[k] += ms;
      }
    }
    box_parity ^= 1;
  }
  return GSMPM_OK;
}

static void drop_graphs(gsmpm_mpm* h) {
  for (auto& kv : h->graphs) hipGraphExecDestroy(kv.second);
  h->graphs.clear();
  h->graph_box_parity.clear();
}

static int upload_bc(gsmpm_mpm* h) {
  GSMPM_HIP(hipMemcpy(h->dev_bc, &h->host_bc, sizeof(BcTable), hipMemcpyHostToDevice));
  drop_graphs(h);
  return GSMPM_OK;
}

static int plane_of(int field, int* width) {
  switch (field) {
    case GSMPM_FIELD_X: *width = 3; return PX;
    case GSMPM_FIELD_V: *width = 3; return PV;
    case GSMPM_FIELD_C: *width = 9; return PC;
    case GSMPM_FIELD_F_TRIAL: *width = 9; return PF;
    case GSMPM_FIELD_COV: *width = 6; return PCOV;
    case GSMPM_FIELD_INIT_COV: *width = 6; return PICOV;
    case GSMPM_FIELD_R: *width = 9; return PR;
    case GSMPM_FIELD_MASS: *width = 1; return PMASS;
    case GSMPM_FIELD_VOL: *width = 1; return PVOL;
    case GSMPM_FIELD_MU: *width = 1; return PMU;
    case GSMPM_FIELD_LAM: *width = 1; return PLAM;
    case GSMPM_FIELD_YIELD: *width = 1; return PYLD;
    default: *width = 0; return -1;
  }
}

static uint64_t morton3(uint32_t a, uint32_t b, uint32_t c) {
  auto spread = [](uint64_t v) {
    v &= 0x1fffff;
    v = (v | v << 32) & 0x1f00000000ffffull;
    v = (v | v << 16) & 0x1f0000ff0000ffull;
    v = (v | v << 8) & 0x100f00f00f00f00full;
    v = (v | v << 4) & 0x10c30c30c30c30c3ull;
    v = (v | v << 2) & 0x1249249249249249ull;
    return v;
  };
  return (spread(a) << 2) | (spread(b) << 1) | spread(c);
}

static int refresh_box(gsmpm_mpm* h, hipStream_t st) {
  Box* cur = h->boxes + h->cur_box;
  hipLaunchKernelGGL(k_box_reset, dim3(1), dim3(64), 0, st, cur);
  hipLaunchKernelGGL(k_box_from_x, dim3(div_up(h->n, 256)), dim3(256), 0, st, particles_of(h), h->g, cur);
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}

}  // namespace gsmpm

extern "C" {

const char* gsmpm_last_error(void) { return g_err.c_str(); }
int gsmpm_version(void) { return 1; }

int gsmpm_mpm_create(const gsmpm_mpm_params* prm, gsmpm_mpm** out) {
  GSMPM_REQUIRE(prm && out, "gsmpm_mpm_create: null argument");
  GSMPM_REQUIRE(prm->n_particles > 0, "gsmpm_mpm_create: n_particles must be > 0");
  GSMPM_REQUIRE(prm->n_grid > 0 && prm->n_grid <= 2048, "gsmpm_mpm_create: n_grid out of range");
  GSMPM_REQUIRE(prm->grid_extent > 0, "gsmpm_mpm_create: grid_extent must be > 0");
  // model.py:27-30: anything but jelly/metal/sand/foam raises TypeError
  if (prm->material < 0 || prm->material > 3) {
    set_error("Material not supported yet");
    return GSMPM_EINVAL;
  }
  auto* h = new gsmpm_mpm();
  h->prm = *prm;
  h->n = prm->n_particles;
  h->np = (h->n + 255) / 256 * 256;
  h->g.ng = prm->n_grid;
  h->g.dx = (float)(prm->grid_extent / prm->n_grid);      // model.py:14
  h->g.inv_dx = (float)(prm->n_grid / prm->grid_extent);  // model.py:15
  const double sin_phi = std::sin(prm->friction_angle_deg / 180.0 * 3.141592653589793);
  h->mc.alpha = (float)(std::sqrt(2.0 / 3.0) * 2.0 * sin_phi / (3.0 - sin_phi));  // model.py:48-51
  h->mc.hardening = (float)prm->hardening;
  h->mc.xi = (float)prm->xi;
  h->mc.pvisc = (float)prm->plastic_viscosity;
  h->mat_kernel = prm->material;
  if (prm->material == 0 && (prm->flags & GSMPM_FLAG_JELLY_FCR)) h->mat_kernel = 4;
  const size_t nn = (size_t)h->g.ng * h->g.ng * h->g.ng;
  auto fail = [&](hipError_t e, const char* what) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    gsmpm_mpm_destroy(h);
    return GSMPM_EHIP;
  };
  hipError_t e;
  if ((e = hipMalloc(&h->planes, sizeof(float) * (size_t)NPLANES * h->np)) != hipSuccess) return fail(e, "hipMalloc planes");
  if ((e = hipMalloc(&h->orig, sizeof(int) * (size_t)h->np)) != hipSuccess) return fail(e, "hipMalloc orig");
  if ((e = hipMalloc(&h->gacc, sizeof(float4) * nn)) != hipSuccess) return fail(e, "hipMalloc grid acc");
  if ((e = hipMalloc(&h->gvel, sizeof(float4) * nn)) != hipSuccess) return fail(e, "hipMalloc grid vel");
  if ((e = hipMalloc(&h->boxes, sizeof(Box) * 3)) != hipSuccess) return fail(e, "hipMalloc boxes");
  if ((e = hipMalloc(&h->dev_bc, sizeof(BcTable))) != hipSuccess) return fail(e, "hipMalloc bc table");
  if ((e = hipMemset(h->gacc, 0, sizeof(float4) * nn)) != hipSuccess) return fail(e, "hipMemset");
  if ((e = hipMemset(h->gvel, 0, sizeof(float4) * nn)) != hipSuccess) return fail(e, "hipMemset");
  if ((e = hipMemset(h->planes, 0, sizeof(float) * (size_t)NPLANES * h->np)) != hipSuccess) return fail(e, "hipMemset");
  if ((e = hipStreamCreateWithFlags(&h->cap, hipStreamNonBlocking)) != hipSuccess) return fail(e, "hipStreamCreate");
  h->host_bc = BcTable{};
  if ((e = hipMemcpy(h->dev_bc, &h->host_bc, sizeof(BcTable), hipMemcpyHostToDevice)) != hipSuccess)
    return fail(e, "hipMemcpy bc");
  // the live-node box starts as the whole grid
  hipLaunchKernelGGL(k_box_full, dim3(1), dim3(64), 0, 0, h->boxes, h->g.ng);
  hipLaunchKernelGGL(k_box_full, dim3(1), dim3(64), 0, 0, h->boxes + 1, h->g.ng);
  hipLaunchKernelGGL(k_box_full, dim3(1), dim3(64), 0, 0, h->boxes + 2, h->g.ng);
  if ((e = hipDeviceSynchronize()) != hipSuccess) return fail(e, "init");
  *out = h;
  return GSMPM_OK;
}

int gsmpm_mpm_destroy(gsmpm_mpm* h) {
  if (!h) return GSMPM_OK;
  drop_graphs(h);
  if (h->cap) hipStreamDestroy(h->cap);
  hipFree(h->planes);
  hipFree(h->orig);
  hipFree(h->gacc);
  hipFree(h->gvel);
  hipFree(h->boxes);
  hipFree(h->dev_bc);
  delete h;
  return GSMPM_OK;
}

int gsmpm_mpm_set_particles(gsmpm_mpm* h, const float* x, const float* cov6, const float* vol, const float* v,
                            void* stream) {
  GSMPM_REQUIRE(h && x && cov6 && vol, "gsmpm_mpm_set_particles: null argument");
  hipStream_t st = (hipStream_t)stream;
  // spatial order: Morton code of the base cell, computed on the host once at
  // init (the sort only changes float-atomic order, never the math)
  std::vector<int> perm(h->n);
  std::iota(perm.begin(), perm.end(), 0);
  if (!(h->prm.flags & GSMPM_FLAG_NO_SORT)) {
    std::vector<float> hx((size_t)h->n * 3);
    GSMPM_HIP(hipMemcpyAsync(hx.data(), x, hx.size() * sizeof(float), hipMemcpyDeviceToHost, st));
    GSMPM_HIP(hipStreamSynchronize(st));
    std::vector<uint64_t> key(h->n);
    for (int p = 0; p < h->n; ++p) {
      uint32_t c[3];
      for (int d = 0; d < 3; ++d) {
        float gp = hx[(size_t)p * 3 + d] * h->g.inv_dx;
        int b = std::isfinite(gp) ? (int)std::min(std::max(gp, 0.0f), 2097151.0f) : 0;
        c[d] = (uint32_t)b;
      }
      key[p] = morton3(c[0], c[1], c[2]);
    }
    std::stable_sort(perm.begin(), perm.end(), [&](int a, int b) { return key[a] < key[b]; });
  }
  GSMPM_HIP(hipMemcpyAsync(h->orig, perm.data(), sizeof(int) * h->n, hipMemcpyHostToDevice, st));
  InitArgs a;
  a.x = x;
  a.cov6 = cov6;
  a.vol = vol;
  a.v = v;
  a.orig = h->orig;
  a.density = (float)h->prm.density;
  a.logE = (float)std::log10(h->prm.E);                   // model.py:42
  a.y = (float)(-std::log(0.49 / h->prm.nu - 1.0));       // model.py:43
  a.yield0 = (float)h->prm.yield_stress;                  // model.py:56
  hipLaunchKernelGGL(k_init, dim3(div_up(h->n, 256)), dim3(256), 0, st, particles_of(h), a);
  GSMPM_LAUNCH_CHECK();
  const size_t nn = (size_t)h->g.ng * h->g.ng * h->g.ng;
  GSMPM_HIP(hipMemsetAsync(h->gacc, 0, nn * sizeof(float4), st));
  GSMPM_HIP(hipMemsetAsync(h->gvel, 0, nn * sizeof(float4), st));
  int rc = refresh_box(h, st);
  if (rc) return rc;
  GSMPM_HIP(hipStreamSynchronize(st));
  h->has_particles = true;
  return GSMPM_OK;
}

static int add_bc_common(gsmpm_mpm* h) {
  if (h->n_bc >= kMaxBC) {
    set_error("too many boundary conditions (max 32)");
    return -1;
  }
  return h->n_bc++;
}

int gsmpm_mpm_add_fixed_cube(gsmpm_mpm* h, const double c[3], const double s[3]) {
  GSMPM_REQUIRE(h && c && s, "gsmpm_mpm_add_fixed_cube: null argument");
  const int id = add_bc_common(h);
  if (id < 0) return GSMPM_EINVAL;
  GridOp& op = h->host_bc.op[h->host_bc.n_ops++];
  op.kind = 0;
  op.bit = id;
  for (int d = 0; d < 3; ++d) {
    op.a[d] = (float)c[d];
    op.b[d] = (float)s[d];
  }
  op.friction = 0.f;
  int rc = upload_bc(h);
  return rc ? rc : id;
}

int gsmpm_mpm_add_impulse(gsmpm_mpm* h, const double c[3], const double s[3], const double f[3], double sdt) {
  GSMPM_REQUIRE(h && c && s && f, "gsmpm_mpm_add_impulse: null argument");
  const int id = add_bc_common(h);
  if (id < 0) return GSMPM_EINVAL;
  Impulse& im = h->host_bc.imp[h->host_bc.n_imp++];
  im.bit = id;
  for (int d = 0; d < 3; ++d) {
    im.c[d] = (float)c[d];
    im.s[d] = (float)s[d];
    im.f[d] = (float)f[d];
  }
  im.sdt = (float)sdt;
  int rc = upload_bc(h);
  return rc ? rc : id;
}

int gsmpm_mpm_add_plane_collider(gsmpm_mpm* h, const double p[3], const double n[3], double friction) {
  GSMPM_REQUIRE(h && p && n, "gsmpm_mpm_add_plane_collider: null argument");
  const double nn = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
  GSMPM_REQUIRE(nn > 0, "gsmpm_mpm_add_plane_collider: zero normal");
  const int id = add_bc_common(h);
  if (id < 0) return GSMPM_EINVAL;
  GridOp& op = h->host_bc.op[h->host_bc.n_ops++];
  op.kind = 1;
  op.bit = id;
  const double sc = 1.0 / std::sqrt(nn);  // solver.py:153-154 (f64)
  for (int d = 0; d < 3; ++d) {
    op.a[d] = (float)p[d];
    op.b[d] = (float)(sc * n[d]);
  }
  op.friction = (float)friction;
  int rc = upload_bc(h);
  return rc ? rc : id;
}

int gsmpm_mpm_step(gsmpm_mpm* h, float dt, int32_t nsub, const uint32_t* bc, void* stream) {
  GSMPM_REQUIRE(h, "gsmpm_mpm_step: null handle");
  if (!h->has_particles) {
    set_error("gsmpm_mpm_step: particles not set");
    return GSMPM_ESTATE;
  }
  GSMPM_REQUIRE(nsub >= 0, "gsmpm_mpm_step: n_substeps < 0");
  if (nsub == 0) return GSMPM_OK;
  hipStream_t st = (hipStream_t)stream;
  const bool use_graph = !(h->prm.flags & GSMPM_FLAG_NO_GRAPH) && nsub >= 2;
  if (!use_graph) {
    int parity = h->cur_box;
    int rc = launch_substeps(h, dt, nsub, bc, st, parity);
    h->cur_box = parity;
    return rc;
  }
  std::vector<uint32_t> key;
  key.reserve(nsub + 3);
  uint32_t dtb;
  std::memcpy(&dtb, &dt, 4);
  key.push_back(dtb);
  key.push_back((uint32_t)nsub);
  key.push_back((uint32_t)h->cur_box);
  for (int s = 0; s < nsub; ++s) key.push_back(bc ? bc[s] : 0xffffffffu);
  auto it = h->graphs.find(key);
  if (it == h->graphs.end()) {
    if (h->graphs.size() >= 16) drop_graphs(h);
    hipGraph_t graph;
    int parity = h->cur_box;
    GSMPM_HIP(hipStreamBeginCapture(h->cap, hipStreamCaptureModeRelaxed));
    int rc = launch_substeps(h, dt, nsub, bc, h->cap, parity);
    hipError_t e = hipStreamEndCapture(h->cap, &graph);
    if (rc) return rc;
    if (e != hipSuccess) {
      set_error(std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
      return GSMPM_EHIP;
    }
    hipGraphExec_t exec;
    e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    hipGraphDestroy(graph);
    if (e != hipSuccess) {
      set_error(std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
      return GSMPM_EHIP;
    }
    it = h->graphs.emplace(key, exec).first;
    h->graph_box_parity[key] = parity;
  }
  GSMPM_HIP(hipGraphLaunch(it->second, st));
  h->cur_box = h->graph_box_parity[key];
  return GSMPM_OK;
}

int gsmpm_mpm_postprocess(gsmpm_mpm* h, void* stream) {
  GSMPM_REQUIRE(h, "gsmpm_mpm_postprocess: null handle");
  hipLaunchKernelGGL(k_postprocess, dim3(div_up(h->n, 256)), dim3(256), 0, (hipStream_t)stream, particles_of(h));
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}

int gsmpm_mpm_field_width(int32_t field) {
  int w;
  if (plane_of(field, &w) < 0) return GSMPM_EINVAL;
  return w;
}

int gsmpm_mpm_get(gsmpm_mpm* h, int32_t field, float* out, void* stream) {
  GSMPM_REQUIRE(h && out, "gsmpm_mpm_get: null argument");
  int w;
  const int p0 = plane_of(field, &w);
  GSMPM_REQUIRE(p0 >= 0, "gsmpm_mpm_get: unknown field");
  hipLaunchKernelGGL(k_get, dim3(div_up(h->n, 256)), dim3(256), 0, (hipStream_t)stream, particles_of(h), h->orig, p0,
                     w, out);
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}

int gsmpm_mpm_set(gsmpm_mpm* h, int32_t field, const float* in, void* stream) {
  GSMPM_REQUIRE(h && in, "gsmpm_mpm_set: null argument");
  int w;
  const int p0 = plane_of(field, &w);
  GSMPM_REQUIRE(p0 >= 0, "gsmpm_mpm_set: unknown field");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_set, dim3(div_up(h->n, 256)), dim3(256), 0, st, particles_of(h), h->orig, p0, w, in);
  GSMPM_LAUNCH_CHECK();
  if (field == GSMPM_FIELD_X) return refresh_box(h, st);
  return GSMPM_OK;
}

int gsmpm_mpm_get_grid(gsmpm_mpm* h, int32_t which, float* out, void* stream) {
  GSMPM_REQUIRE(h && out, "gsmpm_mpm_get_grid: null argument");
  GSMPM_REQUIRE(which >= 0 && which <= 2, "gsmpm_mpm_get_grid: unknown grid field");
  if (!(h->prm.flags & GSMPM_FLAG_KEEP_GRID)) {
    // without it only the live node box is maintained (see k_grid)
    set_error("gsmpm_mpm_get_grid: grid readback needs GSMPM_FLAG_KEEP_GRID");
    return GSMPM_ESTATE;
  }
  const size_t nn = (size_t)h->g.ng * h->g.ng * h->g.ng;
  const float4* src = which == GSMPM_GRID_V_OUT ? h->gvel : h->gacc;
  hipLaunchKernelGGL(k_grid_get, dim3(2048), dim3(256), 0, (hipStream_t)stream, src, nn, which == 0 ? 0 : 1, out);
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}

int gsmpm_mpm_world_outputs(gsmpm_mpm* h, float scale, const float c[3], int32_t render, float* mo, float* co,
                            void* stream) {
  GSMPM_REQUIRE(h && c && mo && co, "gsmpm_mpm_world_outputs: null argument");
  const float half = (float)(1.0f * (float)h->prm.grid_extent / 2.0f);
  hipLaunchKernelGGL(k_world_out, dim3(div_up(h->n, 256)), dim3(256), 0, (hipStream_t)stream, particles_of(h),
                     h->orig, half, scale, c[0], c[1], c[2], render, mo, co);
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}

int gsmpm_mpm_profile_substeps(gsmpm_mpm* h, float dt, int32_t nsub, const uint32_t* bc, float* kernel_ms,
                               void* stream) {
  GSMPM_REQUIRE(h && kernel_ms && nsub >= 0, "gsmpm_mpm_profile_substeps: bad argument");
  if (!h->has_particles) {
    set_error("gsmpm_mpm_profile_substeps: particles not set");
    return GSMPM_ESTATE;
  }
  hipStream_t st = (hipStream_t)stream;
  hipEvent_t ev[4];
  for (int k = 0; k < 4; ++k) GSMPM_HIP(hipEventCreate(&ev[k]));
  kernel_ms[0] = kernel_ms[1] = kernel_ms[2] = 0.f;
  int parity = h->cur_box;
  int rc = launch_substeps(h, dt, nsub, bc, st, parity, ev, kernel_ms);
  h->cur_box = parity;
  for (int k = 0; k < 4; ++k) hipEventDestroy(ev[k]);
  return rc;
}

int gsmpm_mpm_live_box(gsmpm_mpm* h, int32_t* box6, void* stream) {
  GSMPM_REQUIRE(h && box6, "gsmpm_mpm_live_box: null argument");
  Box b;
  GSMPM_HIP(hipMemcpyAsync(&b, h->boxes + h->cur_box, sizeof(Box), hipMemcpyDeviceToHost, (hipStream_t)stream));
  GSMPM_HIP(hipStreamSynchronize((hipStream_t)stream));
  for (int d = 0; d < 3; ++d) {
    box6[d] = b.lo[d];
    box6[3 + d] = b.hi[d];
  }
  return GSMPM_OK;
}

int gsmpm_constitutive(int32_t material, const float* Ft, int32_t n, const float* mu, const float* lam, float* yld,
                       float dt, float* Fo, float* To, void* stream) {
  GSMPM_REQUIRE(Ft && mu && lam && yld && Fo && To && n >= 0, "gsmpm_constitutive: bad argument");
  GSMPM_REQUIRE(material >= 0 && material <= 4, "gsmpm_constitutive: material must be 0..4");
  if (n == 0) return GSMPM_OK;
  MatConsts mc;
  const double sin_phi = std::sin(25.0 / 180.0 * 3.141592653589793);
  mc.alpha = (float)(std::sqrt(2.0 / 3.0) * 2.0 * sin_phi / (3.0 - sin_phi));
  mc.hardening = 1.0f;
  mc.xi = 1.0f;
  mc.pvisc = 0.008f;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(div_up(n, 256)), b(256);
  switch (material) {
    case 0: hipLaunchKernelGGL(k_constitutive<0>, g, b, 0, st, Ft, n, mu, lam, yld, dt, mc, Fo, To); break;
    case 1: hipLaunchKernelGGL(k_constitutive<1>, g, b, 0, st, Ft, n, mu, lam, yld, dt, mc, Fo, To); break;
    case 2: hipLaunchKernelGGL(k_constitutive<2>, g, b, 0, st, Ft, n, mu, lam, yld, dt, mc, Fo, To); break;
    case 3: hipLaunchKernelGGL(k_constitutive<3>, g, b, 0, st, Ft, n, mu, lam, yld, dt, mc, Fo, To); break;
    default: hipLaunchKernelGGL(k_constitutive<4>, g, b, 0, st, Ft, n, mu, lam, yld, dt, mc, Fo, To); break;
  }
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}

int gsmpm_svd3(const float* A, int32_t n, float* U, float* sig, float* V, void* stream) {
  GSMPM_REQUIRE(A && U && sig && V && n >= 0, "gsmpm_svd3: bad argument");
  if (n == 0) return GSMPM_OK;
  hipLaunchKernelGGL(k_svd3, dim3(div_up(n, 256)), dim3(256), 0, (hipStream_t)stream, A, n, U, sig, V);
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}

int gsmpm_particle_volume(const float* x, int32_t n, int32_t ng, double extent, int32_t* scratch, float* vol,
                          void* stream) {
  GSMPM_REQUIRE(x && scratch && vol && n >= 0 && ng > 0, "gsmpm_particle_volume: bad argument");
  hipStream_t st = (hipStream_t)stream;
  const float gdx = (float)(extent / ng);  // filling.py:35 (f64) -> f32 kernel arg
  GSMPM_HIP(hipMemsetAsync(scratch, 0, sizeof(int32_t) * (size_t)ng * ng * ng, st));
  if (n == 0) return GSMPM_OK;
  hipLaunchKernelGGL(k_fill_count, dim3(div_up(n, 256)), dim3(256), 0, st, x, n, ng, gdx, scratch);
  hipLaunchKernelGGL(k_fill_vol, dim3(div_up(n, 256)), dim3(256), 0, st, x, n, ng, gdx, scratch, vol);
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}

}  // extern "C"

// mpm_common.h -- particle/grid layout, BC tables and small device helpers
// shared by the MPM kernels (mpm.hip) and the constitutive models.
#pragma once
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "common.h"

namespace gsmpm {

// ------------------------------------------------------------------ layout --
// Hot planes: what a substep reads and writes, in STORAGE order (re-sorted /
// permuted into bin order with the particles).
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
  NPLANES = 29
};
// Cold planes: only touched at init and by the per-frame postprocess /
// readback, kept in CALLER order (row = orig[storage row]) so re-sorting and
// re-binning never move them.
enum ColdPlane : int {
  PICOV = 0,   // init cov (upper 6)
  PCOV = 6,    // cov (upper 6)
  PR = 12,     // particle_R
  NCOLD = 21
};

constexpr int kMaxBC = 32;

// Tiles: the grid is cut into kTile^3-cell tiles; a particle belongs to the
// tile of its base cell, so its 3x3x3 stencil lies in the tile's
// (kTile+2)^3-node window.
constexpr int kTile = 8;  // k_grid decodes node offsets with 3-bit shifts
constexpr int kTW = kTile + 2;          // window edge
constexpr int kWin = kTW * kTW * kTW;   // window nodes (1000)

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

#ifndef GSMPM_PSTORE
#define GSMPM_PSTORE 2
#endif
struct Particles {
  float* P;
  int n, np;
  float* cold;          // [NCOLD][np], caller order
  const int* nlive;     // slab: the live count on the device (migration changes it inside a captured frame), else null
  // particles live now: kernels of a slab's step read it from the device and
  // run on a capacity-sized grid (the host learns n at the end of the step)
  __device__ __forceinline__ int count() const { return nlive ? *nlive : n; }
  // Plane access through a buffer resource: SGPR descriptor + SGPR plane
  // offset + ONE 32-bit VGPR lane offset for all hot planes (a flat access
  // holds a 64-bit VGPR address per plane, which costs the transfer kernels
  // ~48 VGPRs).  Requires NPLANES * np * 4 < 2^31, checked on the host.
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const {
    return __builtin_amdgcn_make_buffer_rsrc(P, (short)0, NPLANES * np * 4, 0x00020000);
  }
  __device__ __forceinline__ float ld(int plane, int i) const {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc(), i * 4, plane * np * 4, 0));
  }
  // GSMPM_PSTORE: the hot-plane stores' cache policy (buffer aux bits: 2 nt,
  // 16 sc1 write-through, 18 both)
  __device__ __forceinline__ void st(int plane, int i, float v) const {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rsrc(), i * 4, plane * np * 4, GSMPM_PSTORE);
  }
  // cold planes, by caller row
  __device__ __forceinline__ float ldc(int plane, int row) const { return cold[(size_t)plane * np + row]; }
  __device__ __forceinline__ void stc(int plane, int row, float v) const { cold[(size_t)plane * np + row] = v; }
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

// Whole-wave reductions through DPP (no LDS crossbar: a __shfl_xor compiles to
// ds_bpermute_b32): within each 16-lane row by quad swaps and the two row
// mirrors, then the four rows' results read out as uniform values.  Every lane
// of the wave must be active.
template <typename Op>
__device__ __forceinline__ int dpp_row_reduce(int v, Op op) {
  v = op(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
  v = op(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
  v = op(v, __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false));  // row_half_mirror
  v = op(v, __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false));  // row_mirror
  return v;
}
__device__ __forceinline__ int wave_or_dpp(int v) {
  v = dpp_row_reduce(v, [](int a, int b) { return a | b; });
  return __builtin_amdgcn_readlane(v, 0) | __builtin_amdgcn_readlane(v, 16) | __builtin_amdgcn_readlane(v, 32) |
         __builtin_amdgcn_readlane(v, 48);
}
// max of non-negative floats (their bit patterns order as integers)
__device__ __forceinline__ float wave_max_nonneg_dpp(float x) {
  int v = dpp_row_reduce(__float_as_int(x), [](int a, int b) { return max(a, b); });
  v = max(max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
          max(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
  return __int_as_float(v);
}

}  // namespace gsmpm

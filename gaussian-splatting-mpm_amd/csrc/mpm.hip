// mpm.hip -- MI355X (gfx950) MLS-MPM substep for the PhysGaussian loop.
//
// Replaces the Taichi kernels the reference launches from
// MPM_Simulator.p2g2p (mpm_solver/solver.py:27-52): reset_grid_state,
// ImpulseBC.apply, compute_stress_from_F_trial, p2g, grid_normalization_and_gravity,
// BasicBC.apply / MPM_Collider.collide, g2p -- ~10 launches per substep -- by
// three fused kernels per substep, replayed from a cached hipGraph:
//
//   k_p2g   one workgroup per 8^3-cell tile: impulse kick, return map + SVD
//           stress, APIC scatter of (m*v, m) into the tile's 10^3-node window
//           with LDS float atomics; the window is written to the tile's slot
//           with plain coalesced stores (no global atomics)
//   k_grid  node-parallel over the live node box: pulls the <= 8 tile windows
//           covering each node in a fixed order (deterministic sum), then
//           normalise + gravity + the grid BC list in order -> v_out
//   k_g2p   one workgroup per tile: stage the tile window of v_out in LDS,
//           gather the 27-node stencil, update v / x / C / F_trial, and
//           re-bucket every particle into its next tile (LDS-aggregated
//           counters: <= 27 global atomics per workgroup)
//
// Layout in HBM: particle state is SoA (one f32 plane per scalar component,
// stride np = N rounded up to 256), stored in Morton order of the particles'
// cells and re-sorted every `resort_interval` substeps for locality (rows map
// back to the caller's order through `orig`).  Grid: v_out dense float4 n^3;
// tile slots float4[ntiles][1000]; per-tile buckets int[2][ntiles][cap].
#include <hip/hip_runtime.h>
#include <dlfcn.h>


#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <map>
#include <numeric>
#include <vector>

#include "common.h"
#include "constitutive.h"
#include <hip/hip_ext.h>

#include "mpm_common.h"
#include "svd3.h"

namespace gsmpm {

#ifndef GSMPM_REBIN_SF
#define GSMPM_REBIN_SF 20
#endif
constexpr int kRebinStressFree = GSMPM_REBIN_SF;  // default re-binning interval, stress-free materials
// ... stress-bearing ones: 25 since round 6 (lego-fracture metal has no
// escapes at 20-40 and the frame is 0.8 % shorter at 25-40 than at 20,
// profiles/r06/rebin_sweep_r06i.txt; round 5 took 10 -> 20, frame 3.80 ->
// 3.74 ms, profiles/r05/ab/ab_rebin_interval_metal_r05ax.txt); a call of
// 100 substeps re-bins 4 times
#ifndef GSMPM_REBIN_STRESS
#define GSMPM_REBIN_STRESS 25
#endif
constexpr int kRebinStress = GSMPM_REBIN_STRESS;
constexpr int kChunk = 256;  // particles per work chunk (one per lane of a 256-lane workgroup)

// Workgroup timeline stamps (diagnostics): [kernel][wg][start, end] in
// s_memrealtime ticks (100 MHz), written by lane 0 of the first kStampWGs workgroups.
// Compiled in only with -DGSMPM_STAMPS (tools/wg_timeline*.py builds); the
// production library carries no diagnostic stores in its kernels.
#ifdef GSMPM_STAMPS
constexpr int kStampWGs = 8192;
__device__ unsigned long long g_stamps[4][kStampWGs][8];
__device__ __forceinline__ void stamp(int kern, int slot) {
  if (threadIdx.x == 0 && blockIdx.x < kStampWGs) g_stamps[kern][blockIdx.x][slot] = __builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ void stamp_val(int kern, int slot, unsigned long long v) {
  if (threadIdx.x == 0 && blockIdx.x < kStampWGs) g_stamps[kern][blockIdx.x][slot] = v;
}
#define GSMPM_HWREG(r) __builtin_amdgcn_s_getreg((r) | (0 << 6) | (31 << 11))
#else
__device__ __forceinline__ void stamp(int, int) {}
__device__ __forceinline__ void stamp_val(int, int, unsigned long long) {}
#define GSMPM_HWREG(r) 0
#endif

// Chunk work lists (one set per parity).  Every substep G2P re-bins each
// particle into the tile of its new base cell (LDS-aggregated counters), a
// one-workgroup scan turns the per-tile counts into list offsets and a list of
// <= 256-particle chunks, and a scatter writes the per-tile particle lists.
// Particles whose base leaves the grid go to the extra pseudo-tile `ntiles`
// (their transfers take the global, bounds-checked path).
struct Tiles {
  int td;      // tiles per axis
  int ntiles;  // td^3 (the pseudo-tile "outside" is index ntiles)
  int max_chunks;
};
struct ChunkIn {
  const int* count;    // [ntiles + 1] particles per tile
  const int* cbase;    // [ntiles + 1] first chunk of each tile
  const int4* chunk;   // [max_chunks] {tile, first list entry, particles, 0}
  const int* nchunk;   // [2] {chunks, touched tiles}
  const int* list;     // [n] particle (storage) indices grouped by tile
  const int* touched;  // [ntiles] tiles whose nodes the next grid update owns
  // fused pipeline (fused.h k_grid_f): per touched position, the 27 neighbour
  // tiles' {first chunk, chunks} ([27].x = 1: no record, use the tile tables)
  // and their stencil boxes of this substep; null: the tile tables only
  const int2* rcov = nullptr;
  const int* rbox = nullptr;
};
struct BinOut {
  int* count;    // [ntiles + 1], zeroed before G2P
  int* ptile;    // [n] next tile of each particle (storage index)
  int* pslot;    // [n] rank of the particle inside that tile
  int* tflag;    // [ntiles] tile owned by the next grid update (zeroed before G2P)
  int td, ntiles;
};

// A tile's nodes must be updated by the grid step when the tile or one of its
// 7 lower neighbours holds particles (the 10^3 P2G window of tile t covers the
// owned nodes of t + {0,1}^3).  The first reservation in a tile flags them
// (idempotent plain stores); the scan compacts the flags into a list.
__device__ __noinline__ void mark_window(const BinOut& bo, int t) {
  const int td = bo.td;
  const int ti = t / (td * td), tj = (t / td) % td, tk = t % td;
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int c = 0; c < 2; ++c)
        if (ti + a < td && tj + b < td && tk + c < td) bo.tflag[t + (a * td + b) * td + c] = 1;
}
__device__ __forceinline__ int reserve(const BinOut& bo, int t, int c) {
  const int old = atomicAdd(&bo.count[t], c);
  if (old == 0 && t < bo.ntiles) mark_window(bo, t);
  return old;
}

__device__ __forceinline__ int tile_of(const float (&x)[3], const GridDims& g, const Tiles& tl, int (&tc)[3]) {
  bool ok = true;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const float gp = x[d] * g.inv_dx - 0.5f;
    ok = ok && (gp >= 0.0f) && (gp < (float)g.ng);  // false for NaN
    const int b = ok ? (int)gp : 0;
    tc[d] = b / kTile;
  }
  return ok ? (tc[0] * tl.td + tc[1]) * tl.td + tc[2] : tl.ntiles;
}

// ------------------------------------------------------- particle front --
// loads + ImpulseBC.apply + compute_stress_from_F_trial for one particle
template <int MAT>
__device__ __forceinline__ void particle_front(const Particles& ps, int p, const BcTable* __restrict__ bct,
                                               uint32_t mask, float dt, const MatConsts& mc, float (&x)[3],
                                               float (&v)[3], float (&C)[3][3], float& m, float (&nvt)[3][3]) {
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    x[d] = ps.ld(PX + d, p);
    v[d] = ps.ld(PV + d, p);
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) C[i / 3][i % 3] = ps.ld(PC + i, p);
  m = ps.ld(PMASS, p);
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
#pragma unroll
  for (int i = 0; i < 9; ++i) nvt[i / 3][i % 3] = 0.f;
  if constexpr (MAT != 0) {
    float F[3][3], tau[3][3];
#pragma unroll
    for (int i = 0; i < 9; ++i) F[i / 3][i % 3] = ps.ld(PF + i, p);
    float yld = ps.ld(PYLD, p);
    const float mu = ps.ld(PMU, p), lam = ps.ld(PLAM, p);
    return_map_and_stress<MAT>(F, mu, lam, yld, dt, mc, tau);
    if constexpr (MAT == 1 || MAT == 2 || MAT == 3) {
#pragma unroll
      for (int i = 0; i < 9; ++i) ps.st(PF + i, p, F[i / 3][i % 3]);
    }
    if constexpr (MAT == 1) ps.st(PYLD, p, yld);
    const float nvol = -ps.ld(PVOL, p);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) nvt[i][j] = nvol * tau[i][j];
  }
}

// One P2G contribution (utils.py:110-134) of a particle to the stencil node at
// offset (i,j,k): the reference's expression, in its operation order.
template <int MAT>
__device__ __forceinline__ void p2g_term(int i, int j, int k, const float (&fx)[3], const float (&v)[3],
                                         const float (&C)[3][3], float m, const float (&nvt)[3][3], const GridDims& g,
                                         float dt, float4& acc) {
  float w[3], dw[3];
  const int o[3] = {i, j, k};
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const float f = fx[d];
    const float wa = 1.5f - f, wb = f - 1.0f, wc = f - 0.5f;
    w[d] = o[d] == 0 ? wa * wa * 0.5f : (o[d] == 1 ? 0.75f - wb * wb : wc * wc * 0.5f);
    dw[d] = o[d] == 0 ? f - 1.5f : (o[d] == 1 ? -2.0f * (f - 1.0f) : f - 0.5f);
  }
  const float dpos0 = ((float)i - fx[0]) * g.dx;
  const float dpos1 = ((float)j - fx[1]) * g.dx;
  const float dpos2 = ((float)k - fx[2]) * g.dx;
  const float weight = w[0] * w[1] * w[2];
  const float wm = weight * m;
  float add[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) add[r] = wm * (v[r] + (C[r][0] * dpos0 + C[r][1] * dpos1 + C[r][2] * dpos2));
  if constexpr (MAT != 0) {
    const float dw0 = dw[0] * w[1] * w[2] * g.inv_dx;
    const float dw1 = w[0] * dw[1] * w[2] * g.inv_dx;
    const float dw2 = w[0] * w[1] * dw[2] * g.inv_dx;
#pragma unroll
    for (int r = 0; r < 3; ++r) add[r] = add[r] + dt * (nvt[r][0] * dw0 + nvt[r][1] * dw1 + nvt[r][2] * dw2);
  }
  acc.x += add[0];
  acc.y += add[1];
  acc.z += add[2];
  acc.w += wm;
}

// Bounds-checked scatter of one particle into the dense accumulator with f32
// global atomics: the path of particles outside the grid (the reference's
// out-of-range writes are undefined; here they are dropped) and of
// particles that left their chunk's window.
template <int MAT>
__device__ __forceinline__ void p2g_global(const float (&x)[3], const float (&v)[3], const float (&C)[3][3], float m,
                                           const float (&nvt)[3][3], const GridDims& g, float dt,
                                           float4* __restrict__ gacc) {
  const int ng = g.ng;
  int base[3];
  float fx[3], ww[3][3], dw[3][3];
  bspline(x, g.inv_dx, base, fx, ww, dw);
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int kk = 0; kk < 3; ++kk) {
        const int ix = base[0] + i, iy = base[1] + j, iz = base[2] + kk;
        if ((unsigned)ix < (unsigned)ng && (unsigned)iy < (unsigned)ng && (unsigned)iz < (unsigned)ng) {
          float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
          p2g_term<MAT>(i, j, kk, fx, v, C, m, nvt, g, dt, a);
          float* cell = reinterpret_cast<float*>(gacc + (((size_t)ix * ng + iy) * ng + iz));
          unsafeAtomicAdd(cell + 0, a.x);
          unsafeAtomicAdd(cell + 1, a.y);
          unsafeAtomicAdd(cell + 2, a.z);
          unsafeAtomicAdd(cell + 3, a.w);
        }
      }
}

// ------------------------------------------------------------------- P2G --
// One workgroup per <= 256-particle chunk of one tile, one particle per lane.
// Contributions are accumulated into the tile's 10^3-node window in LDS as
// 64-bit fixed point with ds_add_u64: on gfx950 an f32 LDS atomic to distinct
// addresses costs ~192 cycles per wave-instruction, the u64 integer add ~9
// (tools/ubench/lds_atomics.hip).  The scale 2^S is chosen per chunk from a
// bound on its contributions so that no node sum can overflow and every
// contribution keeps >= 2^53 relative resolution; integer sums are exact and
// order-independent.  The window is converted back to f32 once and written to
// the chunk's slot with plain coalesced stores (no global atomics); k_grid sums
// the <= 8 windows covering each node.
// v * scale rounded to an integer, as two's complement int64, for
// |v * scale| < 2^51: adding 1.5 * 2^52 in f64 leaves the integer in the low
// mantissa bits (scale is a power of two, so the product is exact).
__device__ __forceinline__ unsigned long long to_fixed(float v, double scale) {
  const double d = __builtin_fma((double)v, scale, 6755399441055744.0);
  return (unsigned long long)__double_as_longlong(d) - 0x4338000000000000ull;
}

// fixed point -> f32 from the two 32-bit halves (full-rate f32 converts; the
// f64 path rounds once, this one at most twice: <= 1 ulp)
__device__ __forceinline__ float from_fixed32(unsigned long long a, int S) {
  const float hi = (float)(int)(a >> 32), lo = (float)(unsigned)a;
  return ldexpf(__builtin_fmaf(hi, 4294967296.0f, lo), -S);
}

__device__ __forceinline__ void lds_add(unsigned long long* a, unsigned long long v) {
  __hip_atomic_fetch_add(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The 27 contributions of one particle (utils.py:110-134), evaluated in
// separable form: with dd_c[o] = (o - fx_c) dx the APIC momentum
// v + C dpos is accumulated axis by axis (one FMA per component per node) and
// the stress term dt nvt . dweight, whose dweight factors are products of
// per-axis weights, collapses to two FMAs per component per node.  Same
// quantities as the reference's per-node expression, different rounding (a
// few ulp).
// GSMPM_P2G_PK=1 (A/B): components 0 and 1 of the momentum and stress terms
// as packed f32 pairs (v_pk_fma_f32 / v_pk_mul_f32: the same IEEE operation
// per element, two per instruction), component 2 scalar -- the same values
// bit for bit as the scalar form.  Measured slower (5 interleaved rounds,
// profiles/r05/ab/ab_rare_args_pk_r05k.txt): k_fused 16.68 against 16.07 us
// steady, sim 3.095 against 3.075 ms/frame -- the pairs have to be built
// (v_mov into aligned register pairs) and the scatter is not issue-bound
#ifndef GSMPM_P2G_PK
#define GSMPM_P2G_PK 0
#endif
typedef float pkf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pkf2 pk2(float a, float b) { return pkf2{a, b}; }
__device__ __forceinline__ pkf2 pk_fma(pkf2 a, pkf2 b, pkf2 c) { return __builtin_elementwise_fma(a, b, c); }

template <int MAT, int WY = kTW, int WZ = kTW, int WN = kWin>
__device__ __forceinline__ void p2g_scatter(unsigned long long* cell0, const float (&fx)[3], const float (&w)[3][3],
                                            const float (&dw)[3][3], const float (&v)[3], const float (&C)[3][3],
                                            float m, const float (&nvt)[3][3], const GridDims& g, float dt,
                                            double scale) {
#if GSMPM_P2G_PK
  float dd[3][3];
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int o = 0; o < 3; ++o) dd[c][o] = ((float)o - fx[c]) * g.dx;
  const pkf2 C0 = pk2(C[0][0], C[1][0]), C1 = pk2(C[0][1], C[1][1]), C2 = pk2(C[0][2], C[1][2]);
  const pkf2 v01 = pk2(v[0], v[1]);
  pkf2 G0 = pk2(0.f, 0.f), G1 = G0, G2 = G0;  // dt * inv_dx * nvt, rows 0 and 1
  float g20 = 0.f, g21 = 0.f, g22 = 0.f;       // row 2
  if constexpr (MAT != 0) {
    const float f = dt * g.inv_dx;
    G0 = pk2(f * nvt[0][0], f * nvt[1][0]);
    G1 = pk2(f * nvt[0][1], f * nvt[1][1]);
    G2 = pk2(f * nvt[0][2], f * nvt[1][2]);
    g20 = f * nvt[2][0];
    g21 = f * nvt[2][1];
    g22 = f * nvt[2][2];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const pkf2 qi = pk_fma(C0, pk2(dd[0][i], dd[0][i]), v01);
    const float qi2 = __builtin_fmaf(C[2][0], dd[0][i], v[2]);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const pkf2 qij = pk_fma(C1, pk2(dd[1][j], dd[1][j]), qi);
      const float qij2 = __builtin_fmaf(C[2][1], dd[1][j], qi2);
      const float wij = w[0][i] * w[1][j];
      const float mij = wij * m;
      pkf2 sa = pk2(0.f, 0.f), sc = sa;
      float sa2 = 0.f, sc2 = 0.f;
      if constexpr (MAT != 0) {
        const float a0 = dw[0][i] * w[1][j], a1 = w[0][i] * dw[1][j];
        sa = pk_fma(G0, pk2(a0, a0), G1 * pk2(a1, a1));
        sc = G2 * pk2(wij, wij);
        sa2 = __builtin_fmaf(g20, a0, g21 * a1);
        sc2 = g22 * wij;
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float wm = mij * w[2][k];
        const pkf2 q = pk_fma(C2, pk2(dd[2][k], dd[2][k]), qij);
        const float q2 = __builtin_fmaf(C[2][2], dd[2][k], qij2);
        pkf2 add = pk2(wm, wm) * q;
        float add2 = wm * q2;
        if constexpr (MAT != 0) {
          add = pk_fma(sa, pk2(w[2][k], w[2][k]), pk_fma(sc, pk2(dw[2][k], dw[2][k]), add));
          add2 = __builtin_fmaf(sa2, w[2][k], __builtin_fmaf(sc2, dw[2][k], add2));
        }
        unsigned long long* cell = cell0 + (i * WY + j) * WZ + k;
        lds_add(cell + 0 * WN, to_fixed(add.x, scale));
        lds_add(cell + 1 * WN, to_fixed(add.y, scale));
        lds_add(cell + 2 * WN, to_fixed(add2, scale));
        lds_add(cell + 3 * WN, to_fixed(wm, scale));
      }
    }
  }
#else
  float dd[3][3];
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int o = 0; o < 3; ++o) dd[c][o] = ((float)o - fx[c]) * g.dx;
  float G[3][3];  // dt * inv_dx * nvt
  if constexpr (MAT != 0) {
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) G[r][c] = dt * g.inv_dx * nvt[r][c];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    float qi[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) qi[r] = __builtin_fmaf(C[r][0], dd[0][i], v[r]);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float qij[3], sa[3], sc[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) qij[r] = __builtin_fmaf(C[r][1], dd[1][j], qi[r]);
      const float wij = w[0][i] * w[1][j];
      const float mij = wij * m;
      if constexpr (MAT != 0) {
        const float a0 = dw[0][i] * w[1][j], a1 = w[0][i] * dw[1][j];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          sa[r] = __builtin_fmaf(G[r][0], a0, G[r][1] * a1);
          sc[r] = G[r][2] * wij;
        }
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float wm = mij * w[2][k];
        float add[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const float q = __builtin_fmaf(C[r][2], dd[2][k], qij[r]);
          add[r] = wm * q;
          if constexpr (MAT != 0) add[r] = __builtin_fmaf(sa[r], w[2][k], __builtin_fmaf(sc[r], dw[2][k], add[r]));
        }
        unsigned long long* cell = cell0 + (i * WY + j) * WZ + k;
        lds_add(cell + 0 * WN, to_fixed(add[0], scale));
        lds_add(cell + 1 * WN, to_fixed(add[1], scale));
        lds_add(cell + 2 * WN, to_fixed(add[2], scale));
        lds_add(cell + 3 * WN, to_fixed(wm, scale));
      }
    }
  }
#endif
}

template <int MAT>
__global__ __launch_bounds__(256) void k_p2g(Particles ps, GridDims g, Tiles tl, ChunkIn ck,
                                             const BcTable* __restrict__ bct, uint32_t mask, float dt, MatConsts mc,
                                             float4* __restrict__ slots, float4* __restrict__ gacc,
                                             int* __restrict__ nonfin) {
  // channel-planar window: a wave's 8-byte atomics to random nodes of one
  // channel spread over all 64 banks (the node-interleaved float4 layout put
  // every channel on 16 of them: 75 % of LDS cycles were bank conflicts)
  __shared__ unsigned long long s_acc[4 * kWin];
  __shared__ float s_max[4];
  stamp(0, 0);
  const int nch = ck.nchunk[0];
  for (int w = blockIdx.x; w < nch; w += gridDim.x) {
    const int4 cr = ck.chunk[w];
    const int t = cr.x, first = cr.y, cnt = cr.z;
    const int k = threadIdx.x;
    if (t == tl.ntiles) {
      // particles outside the grid: bounds-checked global f32 atomics (reference UB region)
      if (k < cnt) {
        const int p = ck.list[first + k];
        float x[3], v[3], C[3][3], m, nvt[3][3];
        particle_front<MAT>(ps, p, bct, mask, dt, mc, x, v, C, m, nvt);
        p2g_global<MAT>(x, v, C, m, nvt, g, dt, gacc);
      }
      continue;  // workgroup-uniform
    }
    const int tx = t / (tl.td * tl.td), ty = (t / tl.td) % tl.td, tz = t % tl.td;
    for (int q = k; q < kWin * 4; q += kChunk) s_acc[q] = 0ull;
    float x[3], v[3], C[3][3], m = 0.f, nvt[3][3];
    int base[3] = {0, 0, 0};
    float fx[3] = {1.f, 1.f, 1.f}, ww[3][3], dw[3][3];
    float bound = 0.f;
    if (k < cnt) {
      const int p = ck.list[first + k];
      particle_front<MAT>(ps, p, bct, mask, dt, mc, x, v, C, m, nvt);
      bspline(x, g.inv_dx, base, fx, ww, dw);
      {  // non-finite scatter inputs (the fixed-point conversion would hide them; fused.h)
        float chk = m + v[0] + v[1] + v[2];
#pragma unroll
        for (int i = 0; i < 9; ++i) chk += nvt[i / 3][i % 3] + C[i / 3][i % 3];
        if (!__builtin_isfinite(chk)) *nonfin = 1;
      }
      float vm = 0.f, cm = 0.f, sm = 0.f;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        vm = fmaxf(vm, fabsf(v[r]));
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          cm = fmaxf(cm, fabsf(C[r][c]));
          sm = fmaxf(sm, fabsf(nvt[r][c]));
        }
      }
      // |m v + m C dpos| <= m (|v| + 3 * 1.5 dx |C|), |dt nvt dweight| <= dt * 3 * 1.5 inv_dx |nvt|
      bound = fmaxf(m, m * (vm + 4.5f * g.dx * cm) + dt * 4.5f * g.inv_dx * sm) * 1.01f;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) bound = fmaxf(bound, __shfl_xor(bound, o));
    if ((k & 63) == 0) s_max[k >> 6] = bound;
    __syncthreads();  // also orders the window zeroing before the adds
    if (w == (int)blockIdx.x) {
      stamp(0, 2);
      stamp_val(0, 5, cnt);
      stamp_val(0, 6, GSMPM_HWREG(4));  // HW_ID
    }
    const float bmax = fmaxf(fmaxf(s_max[0], s_max[1]), fmaxf(s_max[2], s_max[3]));
    int ebits;
    frexpf(bmax, &ebits);                     // bmax < 2^ebits
    // every contribution below 2^50 (to_fixed needs < 2^51); a node sums <= 256 of them
    const int S = bmax > 0.f ? 50 - ebits : 0;
    if (k < cnt) {
      const int l0 = base[0] - tx * kTile, l1 = base[1] - ty * kTile, l2 = base[2] - tz * kTile;
      p2g_scatter<MAT>(s_acc + ((l0 * kTW + l1) * kTW + l2), fx, ww, dw, v, C, m, nvt, g, dt, ldexp(1.0, S));
    }
    __syncthreads();
    if (w == (int)blockIdx.x) stamp(0, 3);
    float* dst = reinterpret_cast<float*>(slots + (size_t)w * kWin);
    for (int q = k; q < kWin * 4; q += kChunk)
      dst[q] = (float)ldexp((double)(long long)s_acc[(q & 3) * kWin + (q >> 2)], -S);
    __syncthreads();  // LDS reuse by the next chunk
    if (w == (int)blockIdx.x) stamp(0, 4);
  }
  stamp(0, 1);
}

// ------------------------------------------------------------------ grid --
// Sum of the chunk windows covering each node (fixed order: deterministic),
// then grid_normalization_and_gravity (utils.py:177-183) and the
// grid_postprocess list (solver.py:41-46): BasicBC.apply
// (boundary_conditions.py:23-27) / MPM_Collider.collide (collider.py:13-44),
// pointwise, in list order.
struct GridStep {
  // dgx..dgz: dt * gravity, the f32 product formed on the host (the same
  // rounding as the device multiply; as three uniform VALU products hoisted
  // out of k_grid_f's tile loop they held three VGPRs it needs)
  float dt, dgx, dgy, dgz;
  uint32_t mask;
  int keep;
};

// grid_normalization_and_gravity (utils.py:177-183) and the grid_postprocess
// list (solver.py:41-46) of one node: BasicBC.apply (boundary_conditions.py:
// 23-27) / MPM_Collider.collide (collider.py:13-44), pointwise, in list order.
__device__ __forceinline__ float4 node_update(const float4& a, int i, int j, int k, const GridDims& g,
                                              const GridStep& gs, const BcTable* __restrict__ bct) {
  float v[3] = {0.f, 0.f, 0.f};
  if (a.w > 1e-15f) {
    v[0] = a.x / a.w + gs.dgx;
    v[1] = a.y / a.w + gs.dgy;
    v[2] = a.z / a.w + gs.dgz;
    const int nops = bct->n_ops;
    for (int o = 0; o < nops; ++o) {
      const GridOp& op = bct->op[o];
      const float p0 = (float)i * g.dx, p1 = (float)j * g.dx, p2 = (float)k * g.dx;
      if (op.kind == 0) {
        if (!((gs.mask >> op.bit) & 1u)) continue;
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
  return make_float4(v[0], v[1], v[2], 0.f);
}

// Chunk ranges of the <= 8 tiles whose 10^3 windows cover the owned nodes of
// tile (ti, tj, tk) -> LDS (lanes 0..7; caller syncs).
__device__ __forceinline__ void load_cover(const ChunkIn& ck, int td, int ti, int tj, int tk, int* s_c0, int* s_nc) {
  if (threadIdx.x < 8) {
    const int a = threadIdx.x >> 2, b = (threadIdx.x >> 1) & 1, c = threadIdx.x & 1;
    int c0 = 0, nc = 0;
    if (ti >= a && tj >= b && tk >= c) {
      const int t = ((ti - a) * td + (tj - b)) * td + (tk - c);
      nc = (ck.count[t] + kChunk - 1) / kChunk;
      c0 = ck.cbase[t];
    }
    s_c0[threadIdx.x] = c0;
    s_nc[threadIdx.x] = nc;
  }
}

// Sum of the chunk windows covering owned node (li, lj, lk) of a tile: the
// first chunk of each covering tile as 8 unconditional loads in flight
// (inapplicable ones read the all-zero slot max_chunks), then the rare extra
// chunks of tiles holding > 256 particles.
__device__ __forceinline__ float4 node_sum(const float4* __restrict__ slots, int max_chunks, const int* s_c0,
                                           const int* s_nc, int li, int lj, int lk) {
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 s8[8];
  int extra = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int ax = e >> 2, ay = (e >> 1) & 1, az = e & 1;
    const int nc = s_nc[e];
    const bool on = (!ax || li < 2) && (!ay || lj < 2) && (!az || lk < 2) && nc > 0;
    const int loc = ((li + kTile * ax) * kTW + (lj + kTile * ay)) * kTW + (lk + kTile * az);
    const size_t off = on ? (size_t)s_c0[e] * kWin + loc : (size_t)max_chunks * kWin;
    s8[e] = slots[off];
    extra |= (on && nc > 1) ? (1 << e) : 0;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    a.x += s8[e].x;
    a.y += s8[e].y;
    a.z += s8[e].z;
    a.w += s8[e].w;
  }
  while (extra) {
    const int e = __builtin_ctz(extra);
    extra &= extra - 1;
    const int ax = e >> 2, ay = (e >> 1) & 1, az = e & 1;
    const int loc = ((li + kTile * ax) * kTW + (lj + kTile * ay)) * kTW + (lk + kTile * az);
    for (int w = s_c0[e] + 1; w < s_c0[e] + s_nc[e]; ++w) {
      const float4 sv = slots[(size_t)w * kWin + loc];
      a.x += sv.x;
      a.y += sv.y;
      a.z += sv.z;
      a.w += sv.w;
    }
  }
  return a;
}

__global__ __launch_bounds__(512) void k_grid(GridDims g, Tiles tl, ChunkIn ck, const float4* __restrict__ slots,
                                              float4* __restrict__ gacc, float4* __restrict__ gvel,
                                              const BcTable* __restrict__ bct, GridStep gs,
                                              BinOut nb) {
  // housekeeping for the G2P that follows (stream order makes this safe)
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t <= tl.ntiles; t += gridDim.x * blockDim.x) {
    nb.count[t] = 0;
    if (t < tl.ntiles) nb.tflag[t] = 0;
  }

  const int ng = g.ng, td = tl.td;
  const bool outside = ck.count[tl.ntiles] > 0;
  // particles outside the grid scatter through gacc anywhere on the boundary,
  // and KEEP_GRID wants the dense grid: then every tile is updated
  const bool all = outside || gs.keep;
  const int ntouch = all ? tl.ntiles : ck.nchunk[1];
  // one touched tile (8^3 owned nodes) per workgroup iteration, one node per lane (512 lanes: one round of window loads)
  __shared__ int s_c0[8], s_nc[8];
  for (int wt = blockIdx.x; wt < ntouch; wt += gridDim.x) {
    const int T = all ? wt : ck.touched[wt];
    const int ti = T / (td * td), tj = (T / td) % td, tk = T % td;
    __syncthreads();  // readers of the previous tile's ranges are done
    load_cover(ck, td, ti, tj, tk, s_c0, s_nc);
    __syncthreads();
    for (int q = threadIdx.x; q < kTile * kTile * kTile; q += blockDim.x) {
      const int li = q >> 6, lj = (q >> 3) & 7, lk = q & 7;
      const int i = ti * kTile + li, j = tj * kTile + lj, k = tk * kTile + lk;
      if (i >= ng || j >= ng || k >= ng) continue;
      const size_t idx = ((size_t)i * ng + j) * ng + k;
      float4 a = node_sum(slots, tl.max_chunks, s_c0, s_nc, li, lj, lk);
      if (outside || gs.keep) {
        const float4 o = gacc[idx];
        a.x += o.x;
        a.y += o.y;
        a.z += o.z;
        a.w += o.w;
        gacc[idx] = gs.keep ? a : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      gvel[idx] = node_update(a, i, j, k, g, gs, bct);
    }
  }
}

// ------------------------------------------------------------------- G2P --
// g2p (utils.py:218-282) without the dead update_cov; the gather
// reads through `fetch(base, i, j, k)` (LDS window or global v_out).
// x of a particle (loaded early by the callers, so its latency overlaps the
// grid window staging)
__device__ __forceinline__ void load_x(const Particles& ps, int p, float (&x)[3]) {
#pragma unroll
  for (int d = 0; d < 3; ++d) x[d] = ps.ld(PX + d, p);
}

// KEEPW: every fetched node's .w is kept live (an empty asm reads the nine of a
// slab once they are all fetched), so an LDS gather stays one ds_read_b128 a
// node -- 4 LDS cycles a wave -- instead of the ds_read_b96 of .xyz the
// compiler would pick (8 cycles a wave, CDNA4 LDS table)
template <bool KEEPW = false, typename Fetch>
__device__ __forceinline__ void g2p_gather(const float (&x)[3], const GridDims& g, Fetch fetch, float (&nv)[3],
                                           float (&nC)[3][3], float (&nF)[3][3]) {
  int base[3];
  float fx[3], w[3][3], dw[3][3];
  bspline(x, g.inv_dx, base, fx, w, dw);
  // Separable form of the reference's per-node sums: along k accumulate
  // P = sum w2 g, K = sum (k - fx2) w2 g, R = sum dw2 g (9 FMAs per node), then
  // fold each (i, j) row in with its w0/w1 factors.  With dpos = o - fx the
  // sums are v = sum w g, C = 4 inv_dx sum w g dpos^T, grad v = sum g dweight^T
  // -- the same quantities, accumulated in a different order (a few ulp).
  // The i loop stays rolled (weights picked by select) so only one slab of
  // gathers is live.
  float M[3][3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    nv[r] = 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      M[r][c] = 0.f;
      nF[r][c] = 0.f;
    }
  }
  float dk[3], ej[3];
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    dk[o] = ((float)o - fx[2]) * w[2][o];
    ej[o] = ((float)o - fx[1]) * w[1][o];
  }
#pragma unroll 1
  for (int i = 0; i < 3; ++i) {
    const float a = i == 0 ? w[0][0] : (i == 1 ? w[0][1] : w[0][2]);
    const float da = i == 0 ? dw[0][0] : (i == 1 ? dw[0][1] : dw[0][2]);
    const float di = ((float)i - fx[0]) * a;
    float4 gs[3][3];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int k = 0; k < 3; ++k) gs[j][k] = fetch(base, i, j, k);
    if constexpr (KEEPW)
      asm volatile("" ::"v"(gs[0][0].w), "v"(gs[0][1].w), "v"(gs[0][2].w), "v"(gs[1][0].w), "v"(gs[1][1].w),
                   "v"(gs[1][2].w), "v"(gs[2][0].w), "v"(gs[2][1].w), "v"(gs[2][2].w));
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float P[3] = {0.f, 0.f, 0.f}, K[3] = {0.f, 0.f, 0.f}, R[3] = {0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float4 gv = gs[j][k];
        const float gg[3] = {gv.x, gv.y, gv.z};
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          P[r] = __builtin_fmaf(w[2][k], gg[r], P[r]);
          K[r] = __builtin_fmaf(dk[k], gg[r], K[r]);
          R[r] = __builtin_fmaf(dw[2][k], gg[r], R[r]);
        }
      }
      const float b = w[1][j], ab = a * b;
      const float f0 = di * b, f1 = a * ej[j], g0 = da * b, g1 = a * dw[1][j];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        nv[r] = __builtin_fmaf(ab, P[r], nv[r]);
        M[r][0] = __builtin_fmaf(f0, P[r], M[r][0]);
        M[r][1] = __builtin_fmaf(f1, P[r], M[r][1]);
        M[r][2] = __builtin_fmaf(ab, K[r], M[r][2]);
        nF[r][0] = __builtin_fmaf(g0, P[r], nF[r][0]);
        nF[r][1] = __builtin_fmaf(g1, P[r], nF[r][1]);
        nF[r][2] = __builtin_fmaf(ab, R[r], nF[r][2]);
      }
    }
  }
  const float c4 = 4.0f * g.inv_dx;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      nC[r][c] = M[r][c] * c4;
      nF[r][c] = nF[r][c] * g.inv_dx;
    }
}

// F_trial = (I + dt grad v) F (utils.py:275-282), the reference's operation order
__device__ __forceinline__ void f_trial(const float (&gv)[3][3], const float (&F)[3][3], float dt, float (&Fn)[3][3]) {
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float a0 = (r == 0 ? 1.0f : 0.0f) + gv[r][0] * dt;
      const float a1 = (r == 1 ? 1.0f : 0.0f) + gv[r][1] * dt;
      const float a2 = (r == 2 ? 1.0f : 0.0f) + gv[r][2] * dt;
      Fn[r][c] = a0 * F[0][c] + a1 * F[1][c] + a2 * F[2][c];
    }
}

template <typename Fetch>
__device__ __forceinline__ void g2p_particle(const Particles& ps, int p, const float (&x)[3], const GridDims& g,
                                             float dt, Fetch fetch, float (&xn)[3], const float* Fpre = nullptr) {
  float nv[3], nC[3][3], nF[3][3];
  g2p_gather(x, g, fetch, nv, nC, nF);
  float F[3][3];
#pragma unroll
  for (int i = 0; i < 9; ++i) F[i / 3][i % 3] = Fpre ? Fpre[i] : ps.ld(PF + i, p);
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    ps.st(PV + d, p, nv[d]);
    xn[d] = x[d] + dt * nv[d];
    ps.st(PX + d, p, xn[d]);
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) ps.st(PC + i, p, nC[i / 3][i % 3]);
  float Fn[3][3];
  f_trial(nF, F, dt, Fn);
#pragma unroll
  for (int i = 0; i < 9; ++i) ps.st(PF + i, p, Fn[i / 3][i % 3]);
}

// SURVEY 5's per-frame NaN / Inf check of x for the per-phase pipeline
__global__ __launch_bounds__(256) void k_check_finite(Particles ps, int* __restrict__ flag) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < ps.count()) {
    const float a = ps.ld(PX, p), b = ps.ld(PX + 1, p), c = ps.ld(PX + 2, p);
    if (!(__builtin_isfinite(a) && __builtin_isfinite(b) && __builtin_isfinite(c))) *flag = 1;
  }
}

// One workgroup per chunk: stage the tile's 10^3 window of v_out in LDS,
// gather, update the particle, and bin it into the tile of its new base cell.
// Moves to the 27 neighbour tiles are counted in LDS and reserved with <= 27
// global atomics per chunk; farther moves / leaving the grid use one atomic.
__global__ __launch_bounds__(256) void k_g2p(Particles ps, GridDims g, Tiles tl, ChunkIn ck, BinOut bo,
                                                const float4* __restrict__ gvel, float dt) {
  __shared__ float4 s_win[kWin];
  __shared__ int s_cnt[27];
  __shared__ int s_base[27];
  const int ng = g.ng;
  stamp(1, 0);
  const int nch = ck.nchunk[0];
  for (int w = blockIdx.x; w < nch; w += gridDim.x) {
    const int4 cr = ck.chunk[w];
    const int t = cr.x, first = cr.y, cnt = cr.z;
    const int k = threadIdx.x;
    if (t == tl.ntiles) {
      if (k < cnt) {
        const int p = ck.list[first + k];
        float x0[3], xn[3];
        load_x(ps, p, x0);
        g2p_particle(ps, p, x0, g, dt,
                     [&](const int (&base)[3], int i, int j, int kk) {
                       const int ix = base[0] + i, iy = base[1] + j, iz = base[2] + kk;
                       float4 gv = make_float4(0.f, 0.f, 0.f, 0.f);
                       if ((unsigned)ix < (unsigned)ng && (unsigned)iy < (unsigned)ng && (unsigned)iz < (unsigned)ng)
                         gv = gvel[((size_t)ix * ng + iy) * ng + iz];
                       return gv;
                     },
                     xn);
        int tc[3];
        const int nt = tile_of(xn, g, tl, tc);
        bo.ptile[p] = nt;
        bo.pslot[p] = reserve(bo, nt, 1);
      }
      continue;  // workgroup-uniform
    }
    const int tx = t / (tl.td * tl.td), ty = (t / tl.td) % tl.td, tz = t % tl.td;
    const int lo0 = tx * kTile, lo1 = ty * kTile, lo2 = tz * kTile;
    // the particle's list entry and x are requested first so their round
    // trips overlap the window staging below
    int p = -1;
    float x0[3] = {0.f, 0.f, 0.f}, F0[9];
    if (k < cnt) {
      p = ck.list[first + k];
      load_x(ps, p, x0);
#pragma unroll
      for (int i = 0; i < 9; ++i) F0[i] = ps.ld(PF + i, p);  // F in flight with x (latency-bound phase)
    }
    {
      // all four loads in flight before the first LDS store (a guarded load
      // per iteration compiles to one round trip each)
      float4 gv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = min(k + u * kChunk, kWin - 1);
        const int a = q / (kTW * kTW), b = (q / kTW) % kTW, c = q % kTW;
        const int ix = lo0 + a, iy = lo1 + b, iz = lo2 + c;
        const bool in = ix < ng && iy < ng && iz < ng;
        gv[u] = gvel[in ? ((size_t)ix * ng + iy) * ng + iz : 0];
        if (!in) gv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (k + u * kChunk < kWin) s_win[k + u * kChunk] = gv[u];
    }
    if (k < 27) s_cnt[k] = 0;
    __syncthreads();
    if (w == (int)blockIdx.x) {
      stamp(1, 2);
      stamp_val(1, 5, cnt);
      stamp_val(1, 6, t);
      stamp_val(1, 7, GSMPM_HWREG(4));  // HW_ID
    }
    int code = -1, lslot = 0, nt = -1;
    if (k < cnt) {
      float xn[3];
      g2p_particle(ps, p, x0, g, dt,
                   [&](const int (&base)[3], int i, int j, int kk) {
                     const float4* wb = s_win + ((base[0] - lo0) * kTW + (base[1] - lo1)) * kTW + (base[2] - lo2);
                     return wb[(i * kTW + j) * kTW + kk];
                   },
                   xn, F0);
      int tc[3];
      nt = tile_of(xn, g, tl, tc);
      if (nt < tl.ntiles) {
        const int d0 = tc[0] - tx, d1 = tc[1] - ty, d2 = tc[2] - tz;
        if (abs(d0) <= 1 && abs(d1) <= 1 && abs(d2) <= 1) {
          code = (d0 + 1) * 9 + (d1 + 1) * 3 + (d2 + 1);
          lslot = atomicAdd(&s_cnt[code], 1);
        }
      }
    }
    __syncthreads();
    if (w == (int)blockIdx.x) stamp(1, 3);
    if (k < 27) {
      const int c = s_cnt[k];
      if (c > 0) {
        const int ntile = ((tx + k / 9 - 1) * tl.td + (ty + (k / 3) % 3 - 1)) * tl.td + (tz + k % 3 - 1);
        s_base[k] = reserve(bo, ntile, c);
      }
    }
    __syncthreads();
    if (w == (int)blockIdx.x) stamp(1, 4);
    if (p >= 0) {
      bo.ptile[p] = nt;
      bo.pslot[p] = code >= 0 ? s_base[code] + lslot : reserve(bo, nt, 1);
    }
    __syncthreads();  // LDS reuse by the next chunk
  }
  stamp(1, 1);
}

// ------------------------------------------------------- binning passes --
// bin every particle by its current x (set_particles / resort / set x)
__global__ __launch_bounds__(256) void k_bin_all(Particles ps, GridDims g, Tiles tl, BinOut bo) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < ps.n) {
    float x[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) x[d] = ps.ld(PX + d, p);
    int tc[3];
    const int t = tile_of(x, g, tl, tc);
    bo.ptile[p] = t;
    bo.pslot[p] = reserve(bo, t, 1);
  }
}

// Per-tile counts -> list offsets (exclusive scan) and chunk records
// (ceil(count/256) per tile, pseudo-tile last).
struct ChunkOut {
  int* cstart;         // [ntiles + 1] first list entry of each tile
  int* cbase;          // [ntiles + 1] first chunk of each tile
  int4* chunk;         // [max_chunks]
  int* nchunk;         // [2] {chunks, touched tiles}
  const int* tflag;    // [ntiles] touched flags from the binning
  int* touched;        // [ntiles] compacted touched tiles
  int2* rcov = nullptr;  // fused pipeline: [ntiles][32] cover records per touched position (ChunkIn)
  int* tpos = nullptr;   // [ntiles] touched position of each tile, -1: none
  int td1 = 0, td2 = 0;  // tile grid (fused tiles: td0 = ntiles / (td1 td2))
};

constexpr int kRecStride = 32;  // cover-record entries per touched position (27 neighbours + the flag)
// the cover record of touched tile t (position rk) from the binning's per-tile
// first chunks / offsets in LDS (k_finish_bins)
__device__ __forceinline__ void write_cover_record(const ChunkOut& co, int ntiles, int E, int t, int rk,
                                                   const int* s_off, const int* s_aux, int total) {
  const int td12 = co.td1 * co.td2, td0 = ntiles / td12;
  const int tz = t % co.td2, ty = (t / co.td2) % co.td1, tx = t / td12;
  for (int e = 0; e < 27; ++e) {
    const int x = tx + e / 9 - 1, y = ty + (e / 3) % 3 - 1, z = tz + e % 3 - 1;
    int2 r = make_int2(0, 0);
    if ((unsigned)x < (unsigned)td0 && (unsigned)y < (unsigned)co.td1 && (unsigned)z < (unsigned)co.td2) {
      const int u = (x * co.td1 + y) * co.td2 + z;
      const int cnt = (u + 1 < E ? s_off[u + 1] : total) - s_off[u];
      r = make_int2(s_aux[u] & 0xffff, (cnt + kChunk - 1) / kChunk);
    }
    co.rcov[(size_t)rk * kRecStride + e] = r;
  }
  co.rcov[(size_t)rk * kRecStride + 27] = make_int2(0, 0);
}

__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(v, o);
    if (lane >= o) v += y;
  }
  return v;
}

// Exclusive scan of three values over a 256-lane workgroup -> per-lane offsets and totals.
__device__ __forceinline__ void block_scan3(const int (&v)[3], int (&o)[3], int (&tot)[3]) {
  __shared__ int s_ws[3][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const int inc = wave_incl_scan(v[r]);
    if (lane == 63) s_ws[r][wave] = inc;
    o[r] = inc - v[r];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    tot[r] = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      if (w < wave) o[r] += s_ws[r][w];
      tot[r] += s_ws[r][w];
    }
  }
  __syncthreads();  // s_ws reusable
}

// Fused scan + scatter for grids with <= kFuseTiles tiles: every workgroup
// scans the (L2-resident) tile counts itself -- a 4097-entry scan is a few
// microseconds on one CU, so doing it redundantly on all CUs beats a
// one-workgroup scan kernel followed by a scatter launch.  Workgroup b writes
// the chunk records of its slice of tiles, then each lane places one particle.
constexpr int kFuseTiles = 8192;
// Permute (optional, fused pipeline): instead of the list entry, the lane's
// particle itself moves to its bin-order row -- every hot plane and its
// caller row (orig) -- which spares the separate k_permute launch.
struct BinPermute {
  const float* src;
  float* dst;
  int np;
  const int* osrc;
  int* odst;
  int skip_vc;  // v and C are dead (a re-binning between G2P + P2G launches, fused.h): not moved
};
__global__ __launch_bounds__(256) void k_finish_bins(Tiles tl, const int* __restrict__ count, ChunkOut co, int n,
                                                     const int* __restrict__ nlive, const int* __restrict__ ptile,
                                                     const int* __restrict__ pslot, int* __restrict__ list,
                                                     BinPermute bp) {
  __shared__ int s_off[kFuseTiles];  // count | touched << 31, then list offsets
  __shared__ int s_aux[kFuseTiles];  // first chunk (low 16 bits) | touched-list rank (high 16 bits)
  const int E = tl.ntiles + 1;
  if (nlive) n = *nlive;  // a slab: the live count, on a capacity-sized grid
  stamp(2, 0);
  // this lane's particle bin, requested first (independent of the scan)
  const int p = blockIdx.x * 256 + threadIdx.x;
  const int pq = max(0, min(p, n - 1));  // n may be 0 (an empty slab)
  const int pt = ptile[pq], psl = pslot[pq];
  // tile counts / flags: 16 + 16 unguarded loads in flight per lane per batch
  // (written by other XCDs just before, so each batch is one far round trip)
  for (int q0 = 0; q0 < E; q0 += 256 * 16) {
    int cv[16], fv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int q = q0 + u * 256 + threadIdx.x;
      cv[u] = count[min(q, E - 1)];
      fv[u] = co.tflag[min(q, tl.ntiles - 1)];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int q = q0 + u * 256 + threadIdx.x;
      if (q < E) s_off[q] = cv[u] | ((q < tl.ntiles && fv[u]) ? INT_MIN : 0);
    }
  }
  __syncthreads();
  const int per = ((E + 255) / 256) | 1;  // odd: lane-strided LDS segments hit distinct banks
  const int t0 = min(E, threadIdx.x * per), t1 = min(E, t0 + per);
  stamp(2, 2);
  int v[3] = {0, 0, 0};
  for (int t = t0; t < t1; ++t) {
    const int e = s_off[t], c = e & INT_MAX;
    v[0] += c;
    v[1] += (c + kChunk - 1) / kChunk;
    v[2] += e < 0;
  }
  int o[3], tot[3];
  block_scan3(v, o, tot);
  stamp(2, 3);
  // exclusive offsets per tile back into LDS (each lane its own contiguous tiles)
  for (int t = t0; t < t1; ++t) {
    const int e = s_off[t], c = e & INT_MAX;
    s_off[t] = o[0];
    s_aux[t] = o[1] | (o[2] << 16);
    o[0] += c;
    o[1] += (c + kChunk - 1) / kChunk;
    o[2] += e < 0;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    co.nchunk[0] = tot[1];
    co.nchunk[1] = tot[2];
  }
  __syncthreads();
  stamp(2, 4);
  // this workgroup's slice of tiles: one lane per tile writes its chunk
  // records, first chunk and touched-list entry
  const int R = (E + gridDim.x - 1) / gridDim.x;
  for (int t = blockIdx.x * R + threadIdx.x; t < min(E, (int)(blockIdx.x + 1) * R); t += 256) {
    const int off = s_off[t], aux = s_aux[t];
    const int c = (t + 1 < E ? s_off[t + 1] : tot[0]) - off;
    const int cb = aux & 0xffff, rk = aux >> 16;
    const bool touched = (t + 1 < E ? (s_aux[t + 1] >> 16) : tot[2]) > rk;
    co.cbase[t] = cb;
    // .w bit 3: the tile has several chunks (the fused pipeline's k_fused keeps
    // the lower-neighbour axes it added in bits 0..2)
    for (int k = 0; k * kChunk < c; ++k)
      co.chunk[cb + k] = make_int4(t, off + k * kChunk, min(kChunk, c - k * kChunk), c > kChunk ? 8 : 0);
    if (touched) co.touched[rk] = t;
    if (co.tpos && t < tl.ntiles) {
      co.tpos[t] = touched ? rk : -1;
      if (touched) write_cover_record(co, tl.ntiles, E, t, rk, s_off, s_aux, tot[0]);
    }
  }
  if (p < n) {
    const int d = s_off[pt] + psl;
    if (bp.dst) {
      float v[NPLANES];
      const bool skip = bp.skip_vc != 0;
#pragma unroll
      for (int q = 0; q < NPLANES; ++q)
        if (!(skip && q >= PV && q < PF)) v[q] = bp.src[(size_t)q * bp.np + p];
      const int o = bp.osrc[p];
#pragma unroll
      for (int q = 0; q < NPLANES; ++q)
        if (!(skip && q >= PV && q < PF)) bp.dst[(size_t)q * bp.np + d] = v[q];
      bp.odst[d] = o;
    } else {
      list[d] = p;
    }
  }
  stamp(2, 1);
}

// General path (any number of tiles), three launches: per-1024-tile block
// sums, then one workgroup per block adds the sums of the blocks before it and
// scans its own tiles (stores lane-contiguous), then k_scatter.
__device__ __forceinline__ void tile_values(const Tiles& tl, const int* __restrict__ count, const int* __restrict__ tflag,
                                            int t, int (&v)[3]) {
  const int E = tl.ntiles + 1;
  v[0] = t < E ? count[min(t, E - 1)] : 0;
  v[1] = (v[0] + kChunk - 1) / kChunk;
  v[2] = (t < tl.ntiles && tflag[min(t, tl.ntiles - 1)]) ? 1 : 0;
}

// sum of three values over a 1024-lane workgroup (all lanes get the totals)
__device__ __forceinline__ void block_sum3_1024(int (&v)[3]) {
  __shared__ int s_w[3][16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    int x = v[r];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if (lane == 0) s_w[r][wave] = x;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    int x = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) x += s_w[r][w];
    v[r] = x;
  }
  __syncthreads();
}

__global__ __launch_bounds__(1024) void k_scan_partials(Tiles tl, const int* __restrict__ count,
                                                        const int* __restrict__ tflag, int4* __restrict__ part) {
  int v[3];
  tile_values(tl, count, tflag, blockIdx.x * 1024 + threadIdx.x, v);
  block_sum3_1024(v);
  if (threadIdx.x == 0) part[blockIdx.x] = make_int4(v[0], v[1], v[2], 0);
}

__global__ __launch_bounds__(1024) void k_scan_tiles(Tiles tl, const int* __restrict__ count, ChunkOut co,
                                                     const int4* __restrict__ part) {
  __shared__ int s_wsum[3][16];
  const int E = tl.ntiles + 1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // offsets of this block = sums of the blocks before it
  int carry[3] = {0, 0, 0};
  for (int q = threadIdx.x; q < (int)blockIdx.x; q += 1024) {
    const int4 pq = part[q];
    carry[0] += pq.x;
    carry[1] += pq.y;
    carry[2] += pq.z;
  }
  block_sum3_1024(carry);
  const int t = blockIdx.x * 1024 + threadIdx.x;
  int v[3];
  tile_values(tl, count, co.tflag, t, v);
  int inc[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    inc[r] = wave_incl_scan(v[r]);
    if (lane == 63) s_wsum[r][wave] = inc[r];
  }
  __syncthreads();
  if (threadIdx.x < 64) {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int x = lane < 16 ? s_wsum[r][lane] : 0;
      const int xi = wave_incl_scan(x);
      if (lane < 16) s_wsum[r][lane] = xi - x;
    }
  }
  __syncthreads();
  int o[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) o[r] = carry[r] + s_wsum[r][wave] + inc[r] - v[r];
  if (t < E) {
    co.cstart[t] = o[0];
    co.cbase[t] = o[1];
    for (int k = 0; k < v[1]; ++k)
      co.chunk[o[1] + k] = make_int4(t, o[0] + k * kChunk, min(kChunk, v[0] - k * kChunk), v[0] > kChunk ? 8 : 0);
    if (v[2]) co.touched[o[2]] = t;
    // no cover records on this path (k_grid_f reads the tile tables)
    if (co.tpos && t < tl.ntiles) co.tpos[t] = -1;
    if (v[2] && co.rcov) co.rcov[(size_t)o[2] * kRecStride + 27] = make_int2(1, 0);
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 1023) {
    co.nchunk[0] = o[1] + v[1];
    co.nchunk[1] = o[2] + v[2];
  }
}

__global__ __launch_bounds__(256) void k_scatter(int n, const int* __restrict__ nlive, const int* __restrict__ ptile,
                                                 const int* __restrict__ pslot, const int* __restrict__ cstart,
                                                 int* __restrict__ list) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= (nlive ? *nlive : n)) return;
  list[cstart[ptile[p]] + pslot[p]] = p;
}


#include "fused.h"
#include "slab.h"
#include "lsd.h"

// ------------------------------------------------------------ postprocess --
// compute_cov_from_F (utils.py:401-433) + compute_R_from_F (utils.py:376-398)
__global__ __launch_bounds__(256) void k_postprocess(Particles ps, const int* __restrict__ orig) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ps.n) return;
  const int o = orig[p];  // the cold planes' row
  float F[3][3];
#pragma unroll
  for (int i = 0; i < 9; ++i) F[i / 3][i % 3] = ps.ld(PF + i, p);
  const float a0 = ps.ldc(PICOV + 0, o), a1 = ps.ldc(PICOV + 1, o), a2 = ps.ldc(PICOV + 2, o);
  const float a3 = ps.ldc(PICOV + 3, o), a4 = ps.ldc(PICOV + 4, o), a5 = ps.ldc(PICOV + 5, o);
  const float A[3][3] = {{a0, a1, a2}, {a1, a3, a4}, {a2, a4, a5}};
  float T[3][3], Cv[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) T[i][j] = F[i][0] * A[0][j] + F[i][1] * A[1][j] + F[i][2] * A[2][j];
  mmT(T, F, Cv);
  ps.stc(PCOV + 0, o, Cv[0][0]);
  ps.stc(PCOV + 1, o, Cv[0][1]);
  ps.stc(PCOV + 2, o, Cv[0][2]);
  ps.stc(PCOV + 3, o, Cv[1][1]);
  ps.stc(PCOV + 4, o, Cv[1][2]);
  ps.stc(PCOV + 5, o, Cv[2][2]);
  float U[3][3], V[3][3], s[3];
  // R is an output, once per frame: the correctly rounded SVD (the substep's
  // refined rsqrt differs from 1 / sqrtf by < 1 ulp, which a degenerate F --
  // foam's -- can turn into a different rotation)
  svd3<false>(F, U, s, V);
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
    for (int j = 0; j < 3; ++j) ps.stc(PR + i * 3 + j, o, R[j][i]);  // particle_R = (U V^T)^T
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
    ps.st(PX + d, p, a.x[(size_t)o * 3 + d]);
    ps.st(PV + d, p, a.v ? a.v[(size_t)o * 3 + d] : 0.0f);
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    ps.st(PC + i, p, 0.0f);
    ps.st(PF + i, p, (i % 4 == 0) ? 1.0f : 0.0f);
    ps.stc(PR + i, o, 0.0f);
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const float c = a.cov6[(size_t)o * 6 + i];
    ps.stc(PICOV + i, o, c);
    ps.stc(PCOV + i, o, c);
  }
  const float vol = a.vol[o];
  ps.st(PVOL, p, vol);
  ps.st(PMASS, p, a.density * vol);
  // utils.py:349-362 in f32
  const float E = powf(10.0f, a.logE);
  const float nu = 0.49f / (1.0f + expf(-a.y));
  ps.st(PMU, p, E / (2.0f * (1.0f + nu)));
  ps.st(PLAM, p, E * nu / ((1.0f + nu) * (1.0f - 2.0f * nu)));
  ps.st(PYLD, p, a.yield0);
}

__global__ __launch_bounds__(256) void k_get(Particles ps, const int* __restrict__ orig, int plane0, int width,
                                             int cold, float* __restrict__ out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ps.n) return;
  const int r = orig[p];
  const size_t o = (size_t)r * width;
  for (int j = 0; j < width; ++j) out[o + j] = cold ? ps.ldc(plane0 + j, r) : ps.ld(plane0 + j, p);
}

__global__ __launch_bounds__(256) void k_set(Particles ps, const int* __restrict__ orig, int plane0, int width,
                                             int cold, const float* __restrict__ in) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ps.n) return;
  const int r = orig[p];
  const size_t o = (size_t)r * width;
  for (int j = 0; j < width; ++j) {
    if (cold)
      ps.stc(plane0 + j, r, in[o + j]);
    else
      ps.st(plane0 + j, p, in[o + j]);
  }
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
    float w = (ps.ld(PX + d, p) - half) / s + c[d];  // grid2world, transform_utils.py:19
    if (render) w = c[d] + (w - 1.0f) / 1.0f;        // render_frame, main.py:139-144 (scale 1.0)
    mo[o * 3 + d] = w;
  }
  const float ss = s * s;
#pragma unroll
  for (int i = 0; i < 6; ++i) co[o * 6 + i] = ps.ldc(PCOV + i, (int)o) / ss;  // transform_utils.py:20
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

// ------------------------------------------------------- spatial resort --
__device__ __forceinline__ uint32_t spread10(uint32_t v) {
  v &= 0x3ffu;
  v = (v | (v << 16)) & 0x030000ffu;
  v = (v | (v << 8)) & 0x0300f00fu;
  v = (v | (v << 4)) & 0x030c30c3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

// 30-bit Morton key of each particle's base cell (clamped to [0, 1023]^3)
__global__ __launch_bounds__(256) void k_morton(Particles ps, float inv_dx, uint32_t* __restrict__ keys,
                                                int* __restrict__ idx) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ps.n) return;
  uint32_t c[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const float gp = ps.ld(PX + d, p) * inv_dx - 0.5f;
    c[d] = (uint32_t)min(1023.0f, fmaxf(0.0f, gp));  // NaN -> 0
  }
  keys[p] = (spread10(c[0]) << 2) | (spread10(c[1]) << 1) | spread10(c[2]);
  idx[p] = p;
}

// dst[plane][i] = src[plane][perm[i]] for every hot plane (blockIdx.y =
// plane), and the same for the orig map (blockIdx.y = NPLANES)
__global__ __launch_bounds__(256) void k_permute(const float* __restrict__ src, float* __restrict__ dst, int n,
                                                 const int* __restrict__ nlive, int np, const int* __restrict__ perm,
                                                 const int* __restrict__ osrc, int* __restrict__ odst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (nlive ? *nlive : n)) return;
  if (blockIdx.y == NPLANES) {
    odst[i] = osrc[perm[i]];
    return;
  }
  const size_t off = (size_t)blockIdx.y * np;
  dst[off + i] = src[off + perm[i]];
}

__global__ __launch_bounds__(256) void k_permute_i(const int* __restrict__ src, int* __restrict__ dst, int n,
                                                   const int* __restrict__ perm) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  dst[i] = src[perm[i]];
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
  Tiles tl{};
  int mat_kernel = 0;  // template code of k_p2g
  int n = 0, np = 0;
  float* planes = nullptr;
  float* cold = nullptr;  // [NCOLD][np] init_cov, cov, R in caller order
  int* orig = nullptr;
  float4* gacc = nullptr;   // dense accumulator: outside-grid particles + KEEP_GRID readback
  float4* gvel = nullptr;   // dense v_out
  float4* slots = nullptr;  // [max_chunks][kWin] per-chunk P2G windows
  // chunk work lists, one set per parity
  int* count[2] = {nullptr, nullptr};   // [ntiles + 1]
  int* cstart[2] = {nullptr, nullptr};  // [ntiles + 1]
  int* cbase[2] = {nullptr, nullptr};   // [ntiles + 1]
  int4* chunk[2] = {nullptr, nullptr};  // [max_chunks] chunk records
  int* nchunk[2] = {nullptr, nullptr};  // [2] {chunks, touched tiles}
  int* touched[2] = {nullptr, nullptr}; // [ntiles] tiles the grid update owns
  int* tflag[2] = {nullptr, nullptr};   // [ntiles] membership flags of `touched`
  int* list[2] = {nullptr, nullptr};    // [np]
  int4* scan_part = nullptr;            // [ceil((ntiles + 1) / 1024)] block sums (large-grid binning)
  int* ptile = nullptr;                 // [np]
  int* pslot = nullptr;                 // [np]
  int cur_box = 0;       // parity of the boxes / buckets the next substep reads
  BcTable host_bc{};
  BcTable* dev_bc = nullptr;
  int n_bc = 0;
  bool has_particles = false;
  hipStream_t cap = nullptr;
  // spatial resort (Morton order of the current cells), every resort_interval substeps
  int resort_interval = 100;
  long since_sort = 0;
  float* planes_tmp = nullptr;
  int* orig_tmp = nullptr;
  uint32_t* sort_keys = nullptr;  // [2][np]
  int* sort_idx = nullptr;        // [2][np]
  void* sort_tmp = nullptr;
  size_t sort_tmp_bytes = 0;
  // fused G2P2G pipeline (fused.h): its own tiling, chunk lists and slots
  bool fused = true;                      // chosen at create (GSMPM_FLAG_PHASED / KEEP_GRID select the per-phase one)
  FTiles ftl{};
  float4* fslots = nullptr;               // [max_chunks + 1][kFWin]
  int* fcount[2] = {nullptr, nullptr};
  int* fcstart[2] = {nullptr, nullptr};
  int* fcbase[2] = {nullptr, nullptr};
  int4* fchunk[2] = {nullptr, nullptr};
  int* fnchunk[2] = {nullptr, nullptr};
  int* ftouched[2] = {nullptr, nullptr};
  int* ftflag[2] = {nullptr, nullptr};
  int* flist[2] = {nullptr, nullptr};
  int* fesc = nullptr;                    // [2] escape flags (alternating per grid update), then the FOLD
                                          // rotation's [12] (one per phase) and one scratch word
  // the folded grid update (fused.h FOLD): launch r of a step call writes slot
  // buffer r % 2, tile-box buffer r % 2 and escape accumulator r % 3
  // GSMPM_FOLD=1 at create (A/B, off by default): measured and rejected in
  // round 6 -- the folded staging costs k_fused more than k_grid_f + its
  // boundary
  bool fold = false;
  float4* fslots2 = nullptr;              // the second slot buffer [max_chunks + 1][kFWin]
  float4* gacc_f[3] = {nullptr, nullptr, nullptr};  // escape accumulators ([0] = gacc)
  int* ftbox2[2] = {nullptr, nullptr};    // the second tile-box buffer per bins parity
  float4* fesc_nodes = nullptr;           // [np][27] stencil values of particles outside their window
  // adaptive re-binning (round 6): the re-binnings of a step call are chosen
  // from the particles' fastest velocity at the end of the call before
  // (vmax_dev, copied to vmax_host without a sync), so that no particle
  // moves more than ~0.8 of a cell between two re-binnings -- the moves that
  // leave a chunk's window and make the next grid update sweep every tile
  // (DESIGN.md §3.4).  rebin_interval is then the longest spacing allowed.
  // GSMPM_REBIN_AUTO=1 at create (A/B, off by default): it removes the
  // escape storms of long intervals (lego R = 50: 3.95 -> 3.26 ms/frame) but
  // at the default interval the extra re-binnings of the fall cost the
  // 20-frame bench 2-3 %
  bool rebin_auto = false;
  unsigned* vmax_dev = nullptr;           // [1] max |v| component of the last G2P-only launch (f32 bits)
  float* vmax_host = nullptr;             // pinned copy, read by the next call
  int rebin_m = 0;                        // re-binnings of the current call (0: from rebin_interval)
  int* fcbox[2] = {nullptr, nullptr};     // [max_chunks] per-chunk stencil boxes (fused.h)
  int* ftbox[2] = {nullptr, nullptr};     // [ntiles] per-tile stencil boxes
  int2* frcov[2] = {nullptr, nullptr};    // [ntiles][kRecStride] cover records per touched position (k_grid_f)
  int* frbox[2] = {nullptr, nullptr};     // [ntiles][kRecStride] their neighbours' stencil boxes (k_fused writes)
  int* ftpos[2] = {nullptr, nullptr};     // [ntiles] touched position of each tile
  unsigned char* fperm[2] = {nullptr, nullptr};  // [max_chunks][256] lane balance (fused.h); null: off
  bool lane_balance = true;               // GSMPM_LANE_BALANCE=0 turns it off (A/B)
  bool fuse_permute = true;               // GSMPM_FUSE_PERMUTE=0: separate k_permute (A/B)
  bool cover_records = true;              // GSMPM_COVER_RECORDS=0: k_grid_f reads the tile tables only (A/B)
  int fused_wgs = 1024;                   // k_fused grid cap: the workgroups resident at once x rounds of full chunks, <= 6 (init)
  // Chunk order (k_chunk_order): k_fused's workgroup b takes the chunk at
  // position b of a size-balanced order instead of chunk b, so the
  // workgroups that share a CU carry about equal particle counts.
  // On for one resident round of workgroups (init); GSMPM_CHUNK_ORDER=0 / 1
  // forces tile order / the balanced order (A/B)
  bool chunk_order = true;
  bool chunk_xcd_seq = false;             // multi-round grids: k_chunk_order_xcd_seq (XCD placement, tile order)
  int ncu = 256;                          // CUs of the device (the order's tier width)
  int4* fpchunk[2] = {nullptr, nullptr};  // [max_chunks] chunk records in that order (k_fused reads these)
  float* planes_alt = nullptr;            // the other particle-plane buffer: every binning permutes
  int* orig_alt = nullptr;                //   storage into bin order, alternating planes / planes_alt
  int fbpar = 0;                          // parity of the bins the next k_fused reads
  int fep = 0;                            // escape flag the next P2G raises
  int rebin_interval = 10;                // substeps between re-binnings (fused pipeline; set by material at create)
  std::map<std::vector<uint32_t>, hipGraphExec_t> graphs;
  // GSMPM_GRAPH_COPIES=2 (A/B): a second instance of each (non-slab) graph,
  // launched on alternate calls.  Under rocprofv3's kernel trace the bench
  // frame showed ~100 us of idle GPU before each frame's graph (the graph's
  // launch reaching the queue only after the previous frame drained); two
  // instances removed that idle in the trace (109 -> 15 us a frame) but
  // changed nothing in the untraced bench (3 rounds: 2.978 vs 2.980e9), so
  // one instance is the default
  std::map<std::vector<uint32_t>, hipGraphExec_t> graphs_alt;
  std::map<std::vector<uint32_t>, int> graph_turn;
  int graph_copies = 1;
  std::map<std::vector<uint32_t>, int> graph_box_parity;
  struct FState {
    int bpar, ep;
    float* planes;
    float* planes_alt;
    int* orig;
    int* orig_alt;
    // slabs: migrations swap these too, and count on the host
    float* cold;
    float* cold_alt;
    int* gid;
    int* gid_alt;
    long since, migrations;
  };
  std::map<std::vector<uint32_t>, FState> graph_fstate;  // fused-pipeline state after the graph
  // ---- multi-GPU slab (slab.h, slab_host.inc): n varies with migration, np is the capacity ----
  // A step call runs on the device end to end (one captured graph with the
  // RCCL transport): migrations keep the live count in d_n and raise sticky
  // flags; the host learns n, the errors and the boxes from one record
  // exchange at the end of the call (slab_records / slab_check).
  bool slab = false;
  int s_lo = 0, s_hi = 0, s_margin = 2, s_interval = 10, s_rank = 0, s_world = 1;
  int s_has[2] = {0, 0};
  SlabWin sw{};                              // windows + this rank's partial buffers
  float4* s_recv[2] = {nullptr, nullptr};    // the neighbours' partials
  int* d_n = nullptr;                        // [1] live particle count (device)
  int* s_drift = nullptr;                    // [kSlabFlags] sticky device flags (slab.h SlabFlag): drift past the
                                             // margin (k_fused), window mass outside the rect (k_grid_f),
                                             // send / capacity overflow and statistics (k_mig_*)
  bool s_synced = false;                     // the records have been exchanged since the particles were set
  bool s_rect_set = false;                   // the windows' rects have been agreed once (they never shrink after)
  int* gid = nullptr;                        // [np] global particle ids, caller order
  int* gid_alt = nullptr;
  float* cold_alt = nullptr;
  int* mig_bcnt = nullptr;                   // [nblk][3] per-block destination counts
  int* mig_boff = nullptr;                   // [nblk][3] their exclusive scan
  int* mig_tot = nullptr;                    // [3] leavers to lower, stayers, leavers to upper
  int* s_rec = nullptr;                      // [world][rec_ints_of(ng)] every rank's record (slab_records)
  std::vector<int> s_bounds;                 // every rank's planes: [world + 1] (from the records)
  float* s_wdev = nullptr;                   // this rank's re-cut share weight (device: the record reads it)
  float s_weight = 1.0f;
  bool s_rebal_on = true;                    // re-cut the slabs at call boundaries when unbalanced
  float s_rebal_tol = 0.05f;                 // ... by more than this (max count / mean - 1)
  bool s_rebal_pending = false;              // the next call starts with the migration to new bounds
  long s_rebalances = 0;
  int* s_rec_host = nullptr;                 // pinned copy
  int* nonfin_host = nullptr;                // non-finite particle state seen: x, or P2G's m / v / C / stress
                                             // (pinned, device-mapped; sticky)
  int* nonfin_dev = nullptr;                 // its device address
  // k_fused's rare arguments (fused.h): [2 bins parities][kRareSlots], slots
  // 0 / 1 the escape flags of the unfolded pipeline, 2 + r the FOLD phase r
  FusedRare* frare_dev = nullptr;
  FusedRare frare_host[2 * 14] = {};         // what frare_dev holds
  float* mig_send[2] = {nullptr, nullptr};   // fixed-size payloads: header + [NMIG][mig_cap]
  float* mig_recv[2] = {nullptr, nullptr};
  int mig_cap = 0;                           // leavers one migration may send one way (all ranks agree)
  hipStream_t s_comm = nullptr;              // RCCL exchanges run here, overlapping the interior grid update
  hipEvent_t s_ev_pack = nullptr, s_ev_x = nullptr;
  hipEvent_t s_ev_join = nullptr;            // the event the last exchange's join waits on
  bool capturing = false;                    // a graph capture of this handle is open (graph_substeps)
  long s_migrations = 0, s_migrated = 0;     // counters (gsmpm_mpm_slab_stats)
  long s_deferred = 0;
  long s_host_syncs = 0, s_calls = 0;        // host syncs inside gsmpm_mpm_slab_step, step calls
  long s_since = 0;                          // substeps since the last migration
  bool s_graph = true;                       // capture RCCL step calls in hipGraphs (GSMPM_SLAB_GRAPH=0: eager)
  float* x_host = nullptr;                   // CALLBACK transport: pinned staging of the exchanged buffers
  size_t x_host_cap = 0;
};

namespace gsmpm {
static thread_local std::string g_err;
void set_error(const std::string& m) { g_err = m; }

static Particles particles_of(gsmpm_mpm* h) {
  return Particles{h->planes, h->n, h->np, h->cold, h->slab ? h->d_n : nullptr};
}
// rows a per-particle launch covers: the live count, or a slab's capacity
// (its kernels read the live count from the device, ps.count())
static int live_rows(const gsmpm_mpm* h) { return h->slab ? h->np : h->n; }
static const int* nlive_of(const gsmpm_mpm* h) { return h->slab ? h->d_n : nullptr; }

static ChunkIn chunk_in(gsmpm_mpm* h, int c) {
  return ChunkIn{h->count[c], h->cbase[c], h->chunk[c], h->nchunk[c], h->list[c], h->touched[c]};
}
static ChunkOut chunk_out(gsmpm_mpm* h, int c) {
  return ChunkOut{h->cstart[c], h->cbase[c], h->chunk[c], h->nchunk[c], h->tflag[c], h->touched[c]};
}
static BinOut bin_out(gsmpm_mpm* h, int c) {
  return BinOut{h->count[c], h->ptile, h->pslot, h->tflag[c], h->tl.td, h->tl.ntiles};
}

static bool use_fused(const gsmpm_mpm* h) { return h->fused; }

// the chunk records k_fused walks: the balanced order (k_chunk_order) or tile order
// the multi-round XCD placement (k_chunk_order_xcd_seq): its grid must be a multiple of 8
static bool xcd_seq_on(const gsmpm_mpm* h) {
  return !h->chunk_order && h->chunk_xcd_seq && std::min(h->ftl.max_chunks, h->fused_wgs) % 8 == 0;
}
static int4* fused_records(gsmpm_mpm* h, int c) {
  return (h->chunk_order || xcd_seq_on(h)) ? h->fpchunk[c] : h->fchunk[c];
}
static ChunkIn chunk_in_f(gsmpm_mpm* h, int c) {
  ChunkIn ci{h->fcount[c], h->fcbase[c], fused_records(h, c), h->fnchunk[c], h->flist[c], h->ftouched[c]};
  if (h->cover_records) {
    ci.rcov = h->frcov[c];
    ci.rbox = h->frbox[c];
  }
  return ci;
}
static ChunkOut chunk_out_f(gsmpm_mpm* h, int c) {
  ChunkOut co{h->fcstart[c], h->fcbase[c], h->fchunk[c], h->fnchunk[c], h->ftflag[c], h->ftouched[c]};
  co.rcov = h->frcov[c];
  co.tpos = h->ftpos[c];
  co.td1 = h->ftl.td1;
  co.td2 = h->ftl.td2;
  return co;
}
static Touch touch_f(gsmpm_mpm* h, int c) {
  return Touch{h->ftflag[c], h->ftouched[c], h->fnchunk[c], h->fchunk[c], h->fcbox[c], h->ftbox[c],
               h->lane_balance ? h->fperm[c] : nullptr, h->frcov[c],
               h->cover_records ? h->ftpos[c] : nullptr, h->frbox[c]};
}
static BinOutF bin_out_f(gsmpm_mpm* h, int c) { return BinOutF{h->fcount[c], h->ptile, h->pslot, h->ftflag[c], h->ftl}; }
// k_finish_bins / the scan kernels only use ntiles and max_chunks of a Tiles
static Tiles ftiles_flat(const gsmpm_mpm* h) { return Tiles{h->ftl.td0, h->ftl.ntiles, h->ftl.max_chunks}; }

static int p2g_grid(gsmpm_mpm* h) { return std::min(h->tl.max_chunks, 1024); }
static int g2p_grid(gsmpm_mpm* h) { return std::min(h->tl.max_chunks, 1024); }
static int grid_grid(gsmpm_mpm* h) { return std::min(h->tl.ntiles, 1024); }

// Kernel launch; with ev = {start, stop} the dispatch packet itself stamps the
// two events (hipExtLaunchKernel), i.e. the kernel's own begin/end -- the same
// interval rocprofv3's kernel trace reports.
template <typename F, typename... Args>
static void launch(const hipEvent_t* ev, F kernel, dim3 grid, dim3 block, hipStream_t st, Args... args) {
  if (ev)
    hipExtLaunchKernelGGL(kernel, grid, block, 0, st, ev[0], ev[1], 0, args...);
  else
    hipLaunchKernelGGL(kernel, grid, block, 0, st, args...);
}

template <int MAT>
static void launch_p2g(gsmpm_mpm* h, int c, uint32_t mask, float dt, hipStream_t st, const hipEvent_t* ev) {
  launch(ev, k_p2g<MAT>, dim3(p2g_grid(h)), dim3(kChunk), st, particles_of(h), h->g, h->tl, chunk_in(h, c),
         (const BcTable*)h->dev_bc, mask, dt, h->mc, h->slots, h->gacc, h->nonfin_dev);
}

// counts -> list offsets + chunk list, then the per-tile lists
// fused path of the binning: tile table fits LDS, first-chunk indices fit 16 bits (s_aux)
static bool bins_fused(const Tiles& tl) { return tl.ntiles + 1 <= kFuseTiles && tl.max_chunks < 65536; }
// bp.dst non-null (fused path only): the particles are permuted into bin order by the same launch
static int finish_bins_on(gsmpm_mpm* h, const Tiles& tl, const int* count, const ChunkOut& co, int* list,
                          hipStream_t st, const hipEvent_t* ev, const BinPermute& bp = BinPermute{}) {
  if (bins_fused(tl)) {
    launch(ev, k_finish_bins, dim3(std::max(1, div_up(live_rows(h), 256))), dim3(256), st, tl, count, co, h->n,
           nlive_of(h), (const int*)h->ptile, (const int*)h->pslot, list, bp);
  } else {
    const hipEvent_t e0[2] = {ev ? ev[0] : nullptr, nullptr}, e1[2] = {nullptr, ev ? ev[1] : nullptr};
    const int nblk = div_up(tl.ntiles + 1, 1024);
    launch(ev ? e0 : nullptr, k_scan_partials, dim3(nblk), dim3(1024), st, tl, count, (const int*)co.tflag,
           h->scan_part);
    launch(nullptr, k_scan_tiles, dim3(nblk), dim3(1024), st, tl, count, co, (const int4*)h->scan_part);
    launch(ev ? e1 : nullptr, k_scatter, dim3(std::max(1, div_up(live_rows(h), 256))), dim3(256), st, h->n,
           nlive_of(h), (const int*)h->ptile, (const int*)h->pslot, (const int*)co.cstart, list);
  }
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}
static int finish_binning(gsmpm_mpm* h, int c, hipStream_t st, const hipEvent_t* ev = nullptr) {
  return finish_bins_on(h, h->tl, h->count[c], chunk_out(h, c), h->list[c], st, ev);
}
// Chunk order (the fused bins of parity c): one workgroup ranks the chunks by
// particle count, largest first, and lays the ranks out in tiers of ncu
// positions, every other complete tier reversed.  The k_fused grid is a
// multiple of the CU count, and the dispatcher puts workgroups b, b + ncu,
// b + 2 ncu, ... on one CU (tools/wg_timeline_f.py: "WG sets sharing a CU"),
// so a CU that gets one of the largest chunks gets one of the smallest of the
// next tier.  In tile order (round 5) the lego frame's CUs carried 392
// particles at the median and up to 667, and the launch ended with the
// most loaded CU's workgroups (profiles/r06/k_fused_wg_timeline_nofold_r06h.txt:
// max workgroup 13.7 us on CUs under 300 particles, 17.2 us over 600).  The
// order changes no arithmetic: a chunk's work is the same on any workgroup.
// Records keep their tile-order id in .w (bit 4 set, id << 5), which indexes
// the chunk's window slot (k_grid_f finds slots by tile chunk ranges); the
// per-chunk state k_fused keeps between launches (stencil box, lane order)
// is indexed by position.
__device__ __forceinline__ void order_by_size(const int4* __restrict__ chunk, int nch, int4* __restrict__ pchunk,
                                              int ncu) {
  __shared__ int s_h[kChunk];  // chunks of kChunk - b particles, then the first rank of each
  for (int i = threadIdx.x; i < kChunk; i += blockDim.x) s_h[i] = 0;
  __syncthreads();
  for (int c = threadIdx.x; c < nch; c += blockDim.x) atomicAdd(&s_h[kChunk - chunk[c].z], 1);
  __syncthreads();
  if (threadIdx.x < 64) {  // exclusive scan of the 256 bins: 4 a lane
    int v[kChunk / 64], t = 0;
#pragma unroll
    for (int u = 0; u < kChunk / 64; ++u) {
      v[u] = s_h[threadIdx.x * (kChunk / 64) + u];
      t += v[u];
    }
    int o = wave_incl_scan(t) - t;
#pragma unroll
    for (int u = 0; u < kChunk / 64; ++u) {
      s_h[threadIdx.x * (kChunk / 64) + u] = o;
      o += v[u];
    }
  }
  __syncthreads();
  const int full = nch / ncu;  // complete tiers (the last, partial tier runs forward)
  for (int c = threadIdx.x; c < nch; c += blockDim.x) {
    const int4 r = chunk[c];
    const int rank = atomicAdd(&s_h[kChunk - r.z], 1);
    const int tier = rank / ncu, i = rank - tier * ncu;
    const int pos = tier * ncu + (((tier & 1) && tier < full) ? ncu - 1 - i : i);
    pchunk[pos] = make_int4(r.x, r.y, r.z, r.w | 16 | (c << 5));
  }
}
__global__ __launch_bounds__(1024) void k_chunk_order(const int4* __restrict__ chunk, const int* __restrict__ nchunk,
                                                      int4* __restrict__ pchunk, int ncu) {
  order_by_size(chunk, *nchunk, pchunk, ncu);
}
// The same order made XCD-affine (round 6): k_fused's workgroup b runs on XCD
// b % 8 (its grid is a multiple of 8), and k_grid_f updates touched tile P on
// XCD (P / kGridGroup) % 8 (fused.h grid_work).  Here chunk c goes to a
// position on the XCD that updates its tile, so the v_out box it stages was
// stored from that XCD's L2 and its neighbour chunks' boxes share lines there.
// Each XCD takes exactly its share of positions (cap: ceil or floor of nch /
// 8, positions 0..nch-1 all filled): chunks past their XCD's share move to
// XCDs short of theirs.  Within an XCD the size tiers of k_chunk_order, 32
// positions (its CUs) a tier.  GSMPM_CHUNK_XCD=0: the size order alone (A/B).
constexpr int kOrdMax = 4096;  // chunks the XCD order handles (one-round grids: <= 3 x 256 workgroups' worth)
__global__ __launch_bounds__(1024) void k_chunk_order_xcd(const int4* __restrict__ chunk, const int* __restrict__ nchunk,
                                                          const int* __restrict__ tpos, int ntiles,
                                                          int4* __restrict__ pchunk, int ncu) {
  __shared__ int s_h[8][kChunk];      // per XCD: chunks of kChunk - b particles, then the first rank of each
  __shared__ unsigned char s_x[kOrdMax];
  __shared__ unsigned short s_r[kOrdMax];
  __shared__ int s_n[8], s_cap[8], s_def[9], s_ovf;
  const int nch = *nchunk;
  if (nch > kOrdMax) {  // more chunks than the tables hold: the size order alone
    order_by_size(chunk, nch, pchunk, ncu);
    return;
  }
  for (int i = threadIdx.x; i < 8 * kChunk; i += blockDim.x) (&s_h[0][0])[i] = 0;
  if (threadIdx.x < 8) s_n[threadIdx.x] = 0;
  if (threadIdx.x == 0) s_ovf = 0;
  __syncthreads();
  const int T = (nch + 7) / 8, rem = nch - 8 * (T - 1);  // XCD x takes T positions if x < rem, else T - 1
  for (int c = threadIdx.x; c < nch; c += blockDim.x) {
    const int t = chunk[c].x;
    const int P = t < ntiles ? tpos[t] : -1;
    const int x = P >= 0 ? (P / kGridGroup) & 7 : c & 7;
    s_x[c] = (unsigned char)x;
    s_r[c] = (unsigned short)atomicAdd(&s_n[x], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int d = 0;
    for (int x = 0; x < 8; ++x) {
      s_cap[x] = x < rem ? T : T - 1;
      s_def[x] = d;
      d += max(0, s_cap[x] - s_n[x]);
    }
    s_def[8] = d;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < nch; c += blockDim.x) {
    if (s_r[c] >= s_cap[s_x[c]]) {  // past its XCD's share: to the next free place of an XCD short of its share
      const int k = atomicAdd(&s_ovf, 1);
      int x = 0;
      while (x < 7 && s_def[x + 1] <= k) ++x;
      s_x[c] = (unsigned char)x;
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < nch; c += blockDim.x) atomicAdd(&s_h[s_x[c]][kChunk - chunk[c].z], 1);
  __syncthreads();
  if (threadIdx.x < 8 * 64) {  // one wave per XCD: exclusive scan of its 256 bins, 4 a lane
    const int x = threadIdx.x >> 6, l = threadIdx.x & 63;
    int v[kChunk / 64], t = 0;
#pragma unroll
    for (int u = 0; u < kChunk / 64; ++u) {
      v[u] = s_h[x][l * (kChunk / 64) + u];
      t += v[u];
    }
    int o = wave_incl_scan(t) - t;
#pragma unroll
    for (int u = 0; u < kChunk / 64; ++u) {
      s_h[x][l * (kChunk / 64) + u] = o;
      o += v[u];
    }
  }
  __syncthreads();
  const int cpx = max(1, ncu / 8);  // CUs an XCD
  for (int c = threadIdx.x; c < nch; c += blockDim.x) {
    const int4 r = chunk[c];
    const int x = s_x[c];
    const int rank = atomicAdd(&s_h[x][kChunk - r.z], 1);
    const int tier = rank / cpx, i = rank - tier * cpx, full = s_cap[x] / cpx;
    const int j = tier * cpx + (((tier & 1) && tier < full) ? cpx - 1 - i : i);
    pchunk[j * 8 + x] = make_int4(r.x, r.y, r.z, r.w | 16 | (c << 5));
  }
}
// Multi-round grids (bicycle's 1M: ~30,000 chunks over 6 rounds): no size
// tiers (later rounds are placed as CUs free up), only the XCD: each XCD's
// chunks in tile order at positions 8 j + x, so a round's workgroups on one
// XCD take consecutive groups of its tiles; the same equal shares as above.
// One workgroup, each lane a contiguous run of chunks; block scans of the 8
// per-XCD counts give every chunk its rank.
__device__ __forceinline__ void block_scan_n(int (&v)[8], int (&o)[8], int (&tot)[8], int nv) {
  __shared__ int s_ws[8][16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int r = 0; r < nv; ++r) {
    const int inc = wave_incl_scan(v[r]);
    if (lane == 63) s_ws[r][wave] = inc;
    o[r] = inc - v[r];
  }
  __syncthreads();
  for (int r = 0; r < nv; ++r) {
    tot[r] = 0;
    for (int w = 0; w < nw; ++w) {
      if (w < wave) o[r] += s_ws[r][w];
      tot[r] += s_ws[r][w];
    }
  }
  __syncthreads();
}
__device__ __forceinline__ int chunk_xcd(const int4* __restrict__ chunk, const int* __restrict__ tpos, int ntiles, int c) {
  const int t = chunk[c].x;
  const int P = t < ntiles ? tpos[t] : -1;
  return P >= 0 ? (P / kGridGroup) & 7 : c & 7;
}
__global__ __launch_bounds__(1024) void k_chunk_order_xcd_seq(const int4* __restrict__ chunk,
                                                              const int* __restrict__ nchunk,
                                                              const int* __restrict__ tpos, int ntiles,
                                                              int4* __restrict__ pchunk) {
  __shared__ int s_def[9], s_n[8];
  const int nch = *nchunk;
  const int S = (nch + (int)blockDim.x - 1) / (int)blockDim.x;
  const int c0 = min(nch, (int)threadIdx.x * S), c1 = min(nch, c0 + S);
  int v[8], o[8], tot[8];
#pragma unroll
  for (int x = 0; x < 8; ++x) v[x] = 0;
  for (int c = c0; c < c1; ++c) {
    const int x = chunk_xcd(chunk, tpos, ntiles, c);
#pragma unroll
    for (int y = 0; y < 8; ++y) v[y] += x == y;
  }
  block_scan_n(v, o, tot, 8);
  const int T = (nch + 7) / 8, rem = nch - 8 * (T - 1);
  int cap[8];
#pragma unroll
  for (int x = 0; x < 8; ++x) cap[x] = x < rem ? T : T - 1;
  if (threadIdx.x == 0) {
    int d = 0;
    for (int x = 0; x < 8; ++x) {
      s_def[x] = d;
      s_n[x] = tot[x];
      d += max(0, cap[x] - tot[x]);
    }
    s_def[8] = d;
  }
  // overflow chunks (past their XCD's share) of this lane's run, in tile order
  int ov[8] = {0, 0, 0, 0, 0, 0, 0, 0}, oo[8], ot[8];
  {
    int r[8];
#pragma unroll
    for (int x = 0; x < 8; ++x) r[x] = o[x];
    for (int c = c0; c < c1; ++c) {
      const int x = chunk_xcd(chunk, tpos, ntiles, c);
      int rk = 0;
#pragma unroll
      for (int y = 0; y < 8; ++y)
        if (x == y) rk = r[y]++;
      ov[0] += rk >= cap[x];
    }
  }
  block_scan_n(ov, oo, ot, 1);  // (also orders s_def / s_n before their reads)
  int k = oo[0];
  for (int c = c0; c < c1; ++c) {
    const int x = chunk_xcd(chunk, tpos, ntiles, c);
    int rk = 0;
#pragma unroll
    for (int y = 0; y < 8; ++y)
      if (x == y) rk = o[y]++;
    int px = x, pr = rk;
    if (rk >= cap[x]) {  // the k-th overflow chunk: the next free rank of an XCD short of its share
      int y = 0;
      while (y < 7 && s_def[y + 1] <= k) ++y;
      px = y;
      pr = s_n[y] + (k - s_def[y]);
      ++k;
    }
    const int4 rc = chunk[c];
    pchunk[pr * 8 + px] = make_int4(rc.x, rc.y, rc.z, rc.w | 16 | (c << 5));
  }
}
#ifndef GSMPM_CHUNK_XCD
#define GSMPM_CHUNK_XCD 1
#endif
// GSMPM_CHUNK_XCD_SEQ=1 (A/B, off): the multi-round placement above.  Measured
// on bicycle D (profiles/r06/ab_chunk_xcd_seq_r06z.txt): k_fused unchanged
// (98.2 against 98.5 us) and the frame 1.3 % slower -- the one-workgroup
// ordering pass over ~30,000 chunks at every re-binning costs more than the
// placement returns -- so multi-round grids keep the tile order.
#ifndef GSMPM_CHUNK_XCD_SEQ
#define GSMPM_CHUNK_XCD_SEQ 0
#endif
static int order_chunks_f(gsmpm_mpm* h, int c, hipStream_t st) {
  if (!h->chunk_order) {
    // multi-round grids: the XCD placement alone (tile order within each XCD)
    if (xcd_seq_on(h)) {
      launch(nullptr, k_chunk_order_xcd_seq, dim3(1), dim3(1024), st, (const int4*)h->fchunk[c],
             (const int*)h->fnchunk[c], (const int*)h->ftpos[c], h->ftl.ntiles, h->fpchunk[c]);
      GSMPM_LAUNCH_CHECK();
    }
    return GSMPM_OK;
  }
  // the XCD form where k_fused's grid is a multiple of 8 and the chunks fit its LDS tables
  if (GSMPM_CHUNK_XCD && kGridGroup > 0 && std::min(h->ftl.max_chunks, h->fused_wgs) % 8 == 0)
    launch(nullptr, k_chunk_order_xcd, dim3(1), dim3(1024), st, (const int4*)h->fchunk[c], (const int*)h->fnchunk[c],
           (const int*)h->ftpos[c], h->ftl.ntiles, h->fpchunk[c], h->ncu);
  else
    launch(nullptr, k_chunk_order, dim3(1), dim3(1024), st, (const int4*)h->fchunk[c], (const int*)h->fnchunk[c],
           h->fpchunk[c], h->ncu);
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}
static int finish_binning_f(gsmpm_mpm* h, int c, hipStream_t st, const hipEvent_t* ev = nullptr) {
  const int rc = finish_bins_on(h, ftiles_flat(h), h->fcount[c], chunk_out_f(h, c), h->flist[c], st, ev);
  return rc ? rc : order_chunks_f(h, c, st);
}
// the binning of parity c and the storage permutation into its order: one
// launch on the fused path (k_finish_bins moves the particles), else the
// list kernels followed by k_permute
static int permute_to_bins(gsmpm_mpm* h, int c, hipStream_t st, const hipEvent_t* ev);
static int rebin_permute_f(gsmpm_mpm* h, int c, hipStream_t st, const hipEvent_t* ev = nullptr, bool vc_live = true) {
  if (bins_fused(ftiles_flat(h)) && h->fuse_permute) {
    const BinPermute bp{h->planes, h->planes_alt, h->np, h->orig, h->orig_alt, (vc_live || GSMPM_STORE_VC) ? 0 : 1};
    int rc = finish_bins_on(h, ftiles_flat(h), h->fcount[c], chunk_out_f(h, c), h->flist[c], st, ev, bp);
    if (!rc) rc = order_chunks_f(h, c, st);
    if (rc) return rc;
    if (ev) {  // the permute's timing pair: nothing left to time
      GSMPM_HIP(hipEventRecord(ev[2], st));
      GSMPM_HIP(hipEventRecord(ev[3], st));
    }
    std::swap(h->planes, h->planes_alt);
    std::swap(h->orig, h->orig_alt);
    return GSMPM_OK;
  }
  int rc = finish_binning_f(h, c, st, ev);
  return rc ? rc : permute_to_bins(h, c, st, ev ? ev + 2 : nullptr);
}

// Storage into the bin order of parity c (list[c]: storage rows grouped by
// tile): planes / orig gathered into the other buffer, which becomes current.
static int permute_to_bins(gsmpm_mpm* h, int c, hipStream_t st, const hipEvent_t* ev) {
  launch(ev, k_permute, dim3(std::max(1, div_up(live_rows(h), 256)), NPLANES + 1), dim3(256), st,
         (const float*)h->planes, h->planes_alt, h->n, nlive_of(h), h->np, (const int*)h->flist[c],
         (const int*)h->orig, h->orig_alt);
  GSMPM_LAUNCH_CHECK();
  std::swap(h->planes, h->planes_alt);
  std::swap(h->orig, h->orig_alt);
  return GSMPM_OK;
}

// (Re)build the fused pipeline's chunk lists of parity `fbpar` from the current
// x and permute storage into that bin order.
static int rebin_f(gsmpm_mpm* h, hipStream_t st) {
  const int c = h->fbpar;
  GSMPM_HIP(hipMemsetAsync(h->fcount[c], 0, sizeof(int) * (h->ftl.ntiles + 1), st));
  GSMPM_HIP(hipMemsetAsync(h->ftflag[c], 0, sizeof(int) * h->ftl.ntiles, st));
  GSMPM_HIP(hipMemsetAsync(h->fnchunk[c], 0, sizeof(int) * 2, st));
  hipLaunchKernelGGL(k_bin_all_f, dim3(std::max(1, div_up(live_rows(h), 256))), dim3(256), 0, st, particles_of(h), h->g,
                     bin_out_f(h, c));
  GSMPM_LAUNCH_CHECK();
  return rebin_permute_f(h, c, st);
}

// (Re)build the per-phase pipeline's chunk lists of parity `cur_box` from the current x.
static int rebin_phased(gsmpm_mpm* h, hipStream_t st) {
  const int c = h->cur_box;
  GSMPM_HIP(hipMemsetAsync(h->count[c], 0, sizeof(int) * (h->tl.ntiles + 1), st));
  GSMPM_HIP(hipMemsetAsync(h->tflag[c], 0, sizeof(int) * h->tl.ntiles, st));
  GSMPM_HIP(hipMemsetAsync(h->nchunk[c], 0, sizeof(int) * 2, st));
  hipLaunchKernelGGL(k_bin_all, dim3(div_up(h->n, 256)), dim3(256), 0, st, particles_of(h), h->g, h->tl,
                     bin_out(h, c));
  GSMPM_LAUNCH_CHECK();
  return finish_binning(h, c, st);
}

static int rebin(gsmpm_mpm* h, hipStream_t st) { return use_fused(h) ? rebin_f(h, st) : rebin_phased(h, st); }

static GridStep grid_step(gsmpm_mpm* h, float dt, uint32_t mask) {
  GridStep gs;
  gs.dt = dt;
  gs.dgx = dt * (float)h->prm.gravity[0];
  gs.dgy = dt * (float)h->prm.gravity[1];
  gs.dgz = dt * (float)h->prm.gravity[2];
  gs.keep = (h->prm.flags & GSMPM_FLAG_KEEP_GRID) ? 1 : 0;
  gs.mask = mask;
  return gs;
}

// First half of a per-phase substep (parity c): P2G.
static int substep_begin(gsmpm_mpm* h, float dt, uint32_t mask, int c, hipStream_t st, const hipEvent_t* e8) {
  const bool keep = (h->prm.flags & GSMPM_FLAG_KEEP_GRID) != 0;
  if (keep) {
    const size_t nn = (size_t)h->g.ng * h->g.ng * h->g.ng;
    GSMPM_HIP(hipMemsetAsync(h->gacc, 0, nn * sizeof(float4), st));
  }
  switch (h->mat_kernel) {
    case 0: launch_p2g<0>(h, c, mask, dt, st, e8); break;
    case 1: launch_p2g<1>(h, c, mask, dt, st, e8); break;
    case 2: launch_p2g<2>(h, c, mask, dt, st, e8); break;
    case 3: launch_p2g<3>(h, c, mask, dt, st, e8); break;
    default: launch_p2g<4>(h, c, mask, dt, st, e8); break;
  }
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}

// Second half: grid update, G2P, binning of parity nx.
static int substep_end(gsmpm_mpm* h, float dt, uint32_t mask, int c, hipStream_t st, const hipEvent_t* e8) {
  const int nx = c ^ 1;
  launch(e8 ? e8 + 2 : nullptr, k_grid, dim3(grid_grid(h)), dim3(512), st, h->g, h->tl, chunk_in(h, c),
         (const float4*)h->slots, h->gacc, h->gvel, (const BcTable*)h->dev_bc, grid_step(h, dt, mask), bin_out(h, nx));
  GSMPM_LAUNCH_CHECK();
  launch(e8 ? e8 + 4 : nullptr, k_g2p, dim3(g2p_grid(h)), dim3(kChunk), st, particles_of(h), h->g, h->tl,
         chunk_in(h, c), bin_out(h, nx), (const float4*)h->gvel, dt);
  GSMPM_LAUNCH_CHECK();
  return finish_binning(h, nx, st, e8 ? e8 + 6 : nullptr);
}

static int launch_substeps(gsmpm_mpm* h, float dt, int nsub, const uint32_t* bc, hipStream_t st, int& parity,
                           hipEvent_t* ev = nullptr, float* kernel_ms = nullptr) {
  for (int s = 0; s < nsub; ++s) {
    const uint32_t mask = bc ? bc[s] : 0xffffffffu;
    const hipEvent_t* e8 = ev ? ev + 8 * s : nullptr;
    int rc = substep_begin(h, dt, mask, parity, st, e8);
    if (!rc) rc = substep_end(h, dt, mask, parity, st, e8);
    if (rc) return rc;
    parity ^= 1;
  }
  // the per-phase pipeline's non-finite check: one pass over x per call (the
  // fused pipeline checks inside k_fused)
  hipLaunchKernelGGL(k_check_finite, dim3(div_up(h->n, 256)), dim3(256), 0, st, particles_of(h), h->nonfin_dev);
  GSMPM_LAUNCH_CHECK();
  if (ev) {
    GSMPM_HIP(hipStreamSynchronize(st));
    for (int s = 0; s < nsub; ++s)
      for (int k = 0; k < 4; ++k) {
        float ms = 0.f;
        GSMPM_HIP(hipEventElapsedTime(&ms, ev[8 * s + 2 * k], ev[8 * s + 2 * k + 1]));
        kernel_ms[k] += ms;
      }
  }
  return GSMPM_OK;
}

// ------------------------------------------------------ fused pipeline --
// Chunks are dealt w, w + grid, ... to the workgroups, so a grid larger than
// the workgroups resident at once (LDS: 3 per CU) leaves the surplus to start
// only when a resident one has finished ALL its chunks; capped at residency,
// every workgroup starts at once and the chunks of a scene that needs several
// rounds (config D) are spread evenly.
static int fused_grid(gsmpm_mpm* h) { return std::min(h->ftl.max_chunks, h->fused_wgs); }

constexpr int kRareSlots = 14;  // per bins parity: 2 unfolded escape flags + 12 FOLD phases
constexpr int kFoldPhases = 12;
// FOLD phase r's buffers (launch r of a step call, fused.h FusedRare)
static float4* fold_slots(gsmpm_mpm* h, int r) { return (r & 1) ? h->fslots2 : h->fslots; }
static int* fold_tbox(gsmpm_mpm* h, int c, int r) { return (r & 1) ? h->ftbox2[c] : h->ftbox[c]; }
static int* fold_flag(gsmpm_mpm* h, int r) { return h->fesc + 2 + ((r % kFoldPhases) + kFoldPhases) % kFoldPhases; }
static float4* fold_gacc(gsmpm_mpm* h, int r) { return h->gacc_f[((r % 3) + 3) % 3]; }
static int* fold_scratch(gsmpm_mpm* h) { return h->fesc + 2 + kFoldPhases; }

// rare slot: 0 / 1 the unfolded pipeline's escape flag e; 2 + r the FOLD phase r
static FusedRare rare_of(gsmpm_mpm* h, int c, int slot) {
  FusedRare r{};
  const bool fold = slot >= 2;
  const int ph = slot - 2;
  r.bo = bin_out_f(h, c ^ 1);
  r.gacc = fold ? fold_gacc(h, ph) : h->gacc;
  r.esc = fold ? fold_flag(h, ph) : h->fesc + slot;
  r.drift = h->slab ? h->s_drift : nullptr;
  r.nonfin = h->slab ? h->s_drift + SF_NONFIN : h->nonfin_dev;
  r.bct = h->dev_bc;
  r.tflag = h->ftflag[c];
  r.touched = h->ftouched[c];
  r.nchunk = h->fnchunk[c];
  r.chunk = fused_records(h, c);
  r.rcov = h->frcov[c];
  r.tbox = fold ? fold_tbox(h, c, ph) : h->ftbox[c];
  r.tpos = h->cover_records ? h->ftpos[c] : nullptr;
  r.rbox = h->frbox[c];
  if (fold) {
    r.slots_prev = fold_slots(h, ph + 1);  // (r - 1) mod 2
    r.tbox_prev = fold_tbox(h, c, ph + 1);
    r.gacc_prev = fold_gacc(h, ph - 1);
    r.esc_prev = fold_flag(h, ph - 1);
    r.esc_old = fold_flag(h, ph - 2);
    r.gacc_old = fold_gacc(h, ph - 2);
    r.esc_clr = fold_flag(h, ph - 3);
  }
  for (int d = 0; d < 3; ++d) r.grav[d] = (float)h->prm.gravity[d];
  r.esc_count = reinterpret_cast<unsigned*>(h->fesc + 3 + kFoldPhases);
  r.esc_nodes = h->fesc_nodes;
  r.vmax = h->slab ? nullptr : h->vmax_dev;
  return r;
}
// k_fused's rare arguments in device memory, rewritten (outside captures,
// ordered on `st`) whenever one changes; graph_substeps calls it before it
// captures, so a captured launch never finds them stale
static int sync_rare(gsmpm_mpm* h, hipStream_t st) {
  bool dirty = false;
  for (int i = 0; i < 2 * kRareSlots; ++i) {
    const FusedRare r = rare_of(h, i / kRareSlots, i % kRareSlots);
    if (std::memcmp(&r, &h->frare_host[i], sizeof(r)) != 0) {
      h->frare_host[i] = r;
      dirty = true;
    }
  }
  if (!dirty) return GSMPM_OK;
  GSMPM_REQUIRE(!h->capturing, "k_fused's rare arguments changed inside a capture");
  GSMPM_HIP(hipMemcpyAsync(h->frare_dev, h->frare_host, sizeof(h->frare_host), hipMemcpyHostToDevice, st));
  return GSMPM_OK;
}
// one k_fused launch: bins parity c, rare slot `slot`, chunk windows stored to
// `slots`; mask_prev: the BC mask of the previous substep (a FOLD launch's grid step)
struct FusedLaunch {
  int c, bin, use_box, slot;
  uint32_t mask, mask_prev;
  float dt;
  float4* slots;
};
template <int MAT, int MODE>
static void launch_fused_t(gsmpm_mpm* h, const FusedLaunch& f, hipStream_t st, const hipEvent_t* ev) {
  const int xlo = h->slab ? h->s_lo - h->s_margin : INT_MIN, xhi = h->slab ? h->s_hi + h->s_margin : INT_MAX;
  launch(ev, k_fused<MAT, MODE>, dim3(fused_grid(h)), dim3(256), st, particles_of(h), h->g, h->ftl, chunk_in_f(h, f.c),
         touch_f(h, f.c), f.bin, f.use_box, (const float4*)h->gvel, f.mask, f.dt, h->mc, f.slots, xlo, xhi,
         (const FusedRare*)(h->frare_dev + f.c * kRareSlots + f.slot), f.mask_prev);
}
template <int MODE>
static void launch_fused_m(gsmpm_mpm* h, const FusedLaunch& f, hipStream_t st, const hipEvent_t* ev) {
  switch (h->mat_kernel) {
    case 0: launch_fused_t<0, MODE>(h, f, st, ev); break;
    case 1: launch_fused_t<1, MODE>(h, f, st, ev); break;
    case 2: launch_fused_t<2, MODE>(h, f, st, ev); break;
    case 3: launch_fused_t<3, MODE>(h, f, st, ev); break;
    default: launch_fused_t<4, MODE>(h, f, st, ev); break;
  }
}
// mode 1: G2P only, 2: P2G only, 3: G2P of the last grid update + P2G; + 4:
// FOLD (the G2P stages the previous substep's grid update from its chunk
// windows, fused.h).  use_box: the previous k_fused launch did the P2G of
// these same bins, so its per-chunk stencil boxes bound this launch's G2P.
static int launch_fused(gsmpm_mpm* h, int mode, const FusedLaunch& f, hipStream_t st, const hipEvent_t* ev) {
  if (!h->capturing) {
    const int rc = sync_rare(h, st);
    if (rc) return rc;
  }
  switch (mode) {
    case 1: launch_fused_t<0, 1>(h, f, st, ev); break;  // G2P does not depend on the material
    case 5: launch_fused_t<0, 5>(h, f, st, ev); break;
    case 2: launch_fused_m<2>(h, f, st, ev); break;
    case 7: launch_fused_m<7>(h, f, st, ev); break;
    default: launch_fused_m<3>(h, f, st, ev); break;
  }
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}
// the unfolded pipeline's launch: escape flag ep, slot buffer fslots
static int launch_fused(gsmpm_mpm* h, int mode, int c, bool bin, bool use_box, uint32_t mask, float dt, int ep,
                        hipStream_t st, const hipEvent_t* ev) {
  const FusedLaunch f{c, bin ? 1 : 0, use_box ? 1 : 0, ep, mask, mask, dt, h->fslots};
  return launch_fused(h, mode, f, st, ev);
}

// k_grid_f's buffers: the unfolded pipeline's (fslots, ftbox[wp], gacc, escape
// flag ep read, ep ^ 1 cleared), or a FOLD phase's (fold_grid_bufs)
struct GridBufs {
  const float4* slots;
  const int* tbox;
  float4* gacc;
  const int* esc_in;
  int* esc_clear;
};
static GridBufs grid_bufs(gsmpm_mpm* h, int wp, int ep) {
  return GridBufs{h->fslots, h->ftbox[wp], h->gacc, h->fesc + ep, h->fesc + (ep ^ 1)};
}
// after FOLD launch r (the re-binning one): its windows, boxes and escapes; the
// rotation clears the flags, so the grid's own clear goes to a scratch word
static GridBufs fold_grid_bufs(gsmpm_mpm* h, int wp, int r) {
  return GridBufs{fold_slots(h, r), fold_tbox(h, wp, r), fold_gacc(h, r), fold_flag(h, r), fold_scratch(h)};
}
static int launch_grid_f(gsmpm_mpm* h, int wp, float dt, uint32_t mask, const GridBufs& gb, int* zc, int* zf,
                         hipStream_t st, const hipEvent_t* ev, const SlabWin* swp = nullptr) {
  const SlabWin sw = swp ? *swp : SlabWin{};
  // a multiple of 8 workgroups: grid_work's XCD grouping takes b % 8 as the XCD
  const dim3 grid((std::min(kGridParts * h->ftl.ntiles, 1024 * kGridParts) + 7) / 8 * 8);
  if (swp)
    launch(ev, k_grid_f<true>, grid, dim3(kGridT), st, h->g, h->ftl, chunk_in_f(h, wp), gb.tbox, gb.slots, gb.gacc,
           h->gvel, (const BcTable*)h->dev_bc, grid_step(h, dt, mask), gb.esc_in, gb.esc_clear, zc, zf, sw);
  else
    launch(ev, k_grid_f<false>, grid, dim3(kGridT), st, h->g, h->ftl, chunk_in_f(h, wp), gb.tbox, gb.slots, gb.gacc,
           h->gvel, (const BcTable*)h->dev_bc, grid_step(h, dt, mask), gb.esc_in, gb.esc_clear, zc, zf, sw);
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}
static int launch_grid_f(gsmpm_mpm* h, int wp, float dt, uint32_t mask, int ep, int* zc, int* zf, hipStream_t st,
                         const hipEvent_t* ev, const SlabWin* swp = nullptr) {
  return launch_grid_f(h, wp, dt, mask, grid_bufs(h, wp, ep), zc, zf, st, ev, swp);
}

// nsub substeps = nsub + 1 k_fused launches (P2G, nsub - 1 x G2P+P2G, G2P)
// and nsub grid updates; the particles are re-binned by the G2P half every
// rebin_interval substeps and at the end, so the bins are fresh for the next
// call.  bp / ep: bins parity / escape flag, updated.  ev: 8 events per
// k_fused launch ({K, grid, binning} pairs), summed into kernel_ms[0..2].
static int slab_grid_phase(gsmpm_mpm* h, int wp, float dt, uint32_t mask, int ep, int* zc, int* zf, hipStream_t st,
                           const gsmpm_transport* xp);  // slab_host.inc
static bool fold_on(const gsmpm_mpm* h) { return h->fold && !h->slab; }
static int launch_substeps_f(gsmpm_mpm* h, float dt, int nsub, const uint32_t* bc, hipStream_t st, int& bp, int& ep,
                             hipEvent_t* ev = nullptr, float* kernel_ms = nullptr,
                             const gsmpm_transport* xp = nullptr) {
  const int R = std::max(1, h->rebin_interval);
  // m re-binnings, evenly spread (spacing <= R), the last at the end.  Each one
  // flips the bins parity and the particle buffer, which key the captured
  // graphs, so outside slabs m is made even: an odd m alternates two graphs
  // per BC-mask sequence from call to call (a capture inside a timed frame).
  // Slabs re-bin every R substeps, in step with their migrations.
  int m = std::max(1, (nsub + R - 1) / R);
  if (!h->slab && h->rebin_m > 0) m = std::min(std::max(m, h->rebin_m), nsub);  // the call's chosen count
  if (!h->slab && (m & 1) && m < nsub) ++m;
  auto bin_at = [&](int s) {
    if (s == nsub) return true;
    if (s <= 0) return false;
    return h->slab ? s % R == 0 : (long)s * m / nsub > (long)(s - 1) * m / nsub;
  };
  // FOLD (fused.h): launch s stages the grid update of substep s - 1 itself
  // whenever launch s - 1 did its P2G on the same bins; a k_grid_f launch
  // remains only after a re-binning launch (the next launch's chunks are new)
  const bool fold = fold_on(h);
  std::vector<char> grid_at(nsub + 1, 0);
  int wp = bp;
  bool zeroed = false;  // counts / flags of parity bp ^ 1 zeroed by a grid launch since the last binning
  bool boxed = false;   // the last k_fused launch did P2G on the bins parity bp
  for (int s = 0; s <= nsub; ++s) {
    const int mode = s == 0 ? 2 : (s == nsub ? 1 : 3);
    const bool bin = bin_at(s);
    const uint32_t mask = s < nsub ? (bc ? bc[s] : 0xffffffffu) : 0u;
    const uint32_t mask_prev = s > 0 ? (bc ? bc[s - 1] : 0xffffffffu) : 0u;
    hipEvent_t* e8 = ev ? ev + 8 * s : nullptr;
    if (bin && !zeroed) {
      GSMPM_HIP(hipMemsetAsync(h->fcount[bp ^ 1], 0, sizeof(int) * (h->ftl.ntiles + 1), st));
      GSMPM_HIP(hipMemsetAsync(h->ftflag[bp ^ 1], 0, sizeof(int) * h->ftl.ntiles, st));
    }
    if (mode == 1 && !h->slab && h->vmax_dev) GSMPM_HIP(hipMemsetAsync(h->vmax_dev, 0, sizeof(unsigned), st));
    // FOLD: the launch before a re-binning one zeroes its counts (no grid launch between them)
    const bool zero_next = fold && !bin && s < nsub && bin_at(s + 1);
    const bool fl = fold && boxed && (mode & 1);
    const FusedLaunch f{bp, bin ? 1 : (zero_next ? 2 : 0), boxed ? 1 : 0, fold ? 2 + s % kFoldPhases : ep,
                        mask, mask_prev, dt, fold ? fold_slots(h, s) : h->fslots};
    int rc = launch_fused(h, fl ? mode + 4 : mode, f, st, e8);
    if (rc) return rc;
    if (zero_next) zeroed = true;
    if (mode & 2) wp = bp;
    boxed = (mode & 2) && !bin;
    if (bin) {
      rc = rebin_permute_f(h, bp ^ 1, st, e8 ? e8 + 4 : nullptr, /*vc_live=*/mode != 3);
      if (rc) return rc;
      bp ^= 1;
      zeroed = false;
    }
    if (s < nsub && (!fold || bin)) {
      const bool next_bin = bin_at(s + 1);
      int *zc = nullptr, *zf = nullptr;
      if (next_bin && wp == bp) {  // this grid launch does not read parity bp ^ 1
        zc = h->fcount[bp ^ 1];
        zf = h->ftflag[bp ^ 1];
        zeroed = true;
      }
      rc = h->slab ? slab_grid_phase(h, wp, dt, mask, ep, zc, zf, st, xp)
                   : launch_grid_f(h, wp, dt, mask, fold ? fold_grid_bufs(h, wp, s) : grid_bufs(h, wp, ep), zc, zf, st,
                                   e8 ? e8 + 2 : nullptr);
      if (rc) return rc;
      if (!fold) ep ^= 1;
      grid_at[s] = 1;
    }
  }
  if (fold) {  // escape accumulators the call's last launches left dirty, and the rotation's flags
    hipLaunchKernelGGL(k_fold_tail, dim3(1), dim3(1024), 0, st, h->fesc + 2, h->gacc_f[0], h->gacc_f[1], h->gacc_f[2],
                       h->g.ng);
    GSMPM_LAUNCH_CHECK();
  }
  if (ev) {
    // kernel_ms: {k_fused, k_grid_f, binning (+ permute), grid launches}
    GSMPM_HIP(hipStreamSynchronize(st));
    for (int s = 0; s <= nsub; ++s) {
      const bool bin = bin_at(s);
      for (int k = 0; k < 4; ++k) {
        if ((k == 1 && !grid_at[s]) || (k >= 2 && !bin)) continue;
        float ms = 0.f;
        GSMPM_HIP(hipEventElapsedTime(&ms, ev[8 * s + 2 * k], ev[8 * s + 2 * k + 1]));
        kernel_ms[k < 3 ? k : 2] += ms;
      }
      if (grid_at[s]) kernel_ms[3] += 1.f;
    }
  }
  return GSMPM_OK;
}

static void drop_graphs(gsmpm_mpm* h) {
  for (auto& kv : h->graphs) (void)hipGraphExecDestroy(kv.second);
  for (auto& kv : h->graphs_alt) (void)hipGraphExecDestroy(kv.second);
  h->graphs.clear();
  h->graphs_alt.clear();
  h->graph_turn.clear();
  h->graph_box_parity.clear();
  h->graph_fstate.clear();
}

static int upload_bc(gsmpm_mpm* h) {
  GSMPM_HIP(hipMemcpy(h->dev_bc, &h->host_bc, sizeof(BcTable), hipMemcpyHostToDevice));
  drop_graphs(h);
  return GSMPM_OK;
}

// plane of a field; *cold: a cold plane (caller order)
static int plane_of(int field, int* width, int* cold = nullptr) {
  int dummy;
  if (!cold) cold = &dummy;
  *cold = field == GSMPM_FIELD_COV || field == GSMPM_FIELD_INIT_COV || field == GSMPM_FIELD_R;
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

// Re-establish Morton order of the particles' current cells so the transfer
// kernels' per-workgroup windows stay compact.  Only the storage order (and so
// the float-atomic summation order) changes; `orig` keeps rows in caller order.
// The sort: 30-bit Morton keys with the particle index as value, stable LSD
// by 8-bit digits (lsd.h, four passes between the two halves of sort_keys /
// sort_idx: the result lands back in the first halves).
static int resort(gsmpm_mpm* h, hipStream_t st) {
  const int n = h->n, np = h->np;
  const int nch = std::max(1, div_up(np, kLsdChunk));
  if (!h->planes_tmp) {
    GSMPM_HIP(hipMalloc(&h->planes_tmp, sizeof(float) * (size_t)NPLANES * np));
    GSMPM_HIP(hipMalloc(&h->orig_tmp, sizeof(int) * (size_t)np));
    GSMPM_HIP(hipMalloc(&h->sort_keys, sizeof(uint32_t) * 2 * (size_t)np));
    GSMPM_HIP(hipMalloc(&h->sort_idx, sizeof(int) * 2 * (size_t)np));
    // digit histograms and their row prefixes [2][256][nch], digit totals [256]
    GSMPM_HIP(hipMalloc(&h->sort_tmp, sizeof(unsigned) * (2 * 256 * (size_t)nch + 256)));
    h->sort_tmp_bytes = sizeof(unsigned) * (2 * 256 * (size_t)nch + 256);
  }
  const dim3 pb(div_up(n, 256));
  hipLaunchKernelGGL(k_morton, pb, dim3(256), 0, st, particles_of(h), h->g.inv_dx, h->sort_keys, h->sort_idx);
  GSMPM_LAUNCH_CHECK();
  if (n > 0) {
    const int nc = div_up(n, kLsdChunk);
    unsigned* H = reinterpret_cast<unsigned*>(h->sort_tmp);
    unsigned* Hs = H + 256 * (size_t)nc;
    unsigned* tot = H + 2 * 256 * (size_t)nch;
    unsigned* kb[2] = {h->sort_keys, h->sort_keys + np};
    unsigned* vb[2] = {reinterpret_cast<unsigned*>(h->sort_idx), reinterpret_cast<unsigned*>(h->sort_idx) + np};
    for (int p = 0; p < 4; ++p) {
      const unsigned* sk = kb[p & 1];
      const unsigned* sv = vb[p & 1];
      hipLaunchKernelGGL(k_lsd_hist, dim3(nc), dim3(kLsdT), 0, st, n, nc, 8 * p, sk, H);
      hipLaunchKernelGGL(k_tile_rows, dim3(64), dim3(256), 0, st, 255, nc, (const unsigned*)H, Hs, tot);
      hipLaunchKernelGGL(k_lsd_scatter, dim3(nc), dim3(kLsdT), 0, st, n, nc, 8 * p, sk, sv, (const unsigned*)Hs,
                         (const unsigned*)tot, kb[(p + 1) & 1], vb[(p + 1) & 1]);
    }
    GSMPM_LAUNCH_CHECK();
  }
  const int* perm = h->sort_idx;
  hipLaunchKernelGGL(k_permute, dim3(div_up(n, 256), NPLANES + 1), dim3(256), 0, st, h->planes, h->planes_tmp, n,
                     (const int*)nullptr, np, perm, (const int*)h->orig, h->orig_tmp);
  GSMPM_LAUNCH_CHECK();
  // copy back so pointers baked into cached graphs stay valid
  GSMPM_HIP(hipMemcpyAsync(h->planes, h->planes_tmp, sizeof(float) * (size_t)NPLANES * np, hipMemcpyDeviceToDevice, st));
  GSMPM_HIP(hipMemcpyAsync(h->orig, h->orig_tmp, sizeof(int) * (size_t)n, hipMemcpyDeviceToDevice, st));
  h->since_sort = 0;
  return rebin(h, st);  // list entries are storage indices
}

}  // namespace gsmpm

namespace gsmpm {
static int slab_body(gsmpm_mpm* h, float dt, int nsub, const uint32_t* bc, hipStream_t st,
                     const gsmpm_transport* xp);  // slab_host.inc

static gsmpm_mpm::FState fstate_of(const gsmpm_mpm* h, int bp, int ep) {
  return gsmpm_mpm::FState{bp,      ep,          h->planes, h->planes_alt, h->orig, h->orig_alt, h->cold,
                           h->cold_alt, h->gid, h->gid_alt, h->s_since, h->s_migrations};
}
static void set_fstate(gsmpm_mpm* h, const gsmpm_mpm::FState& f) {
  h->planes = f.planes;
  h->planes_alt = f.planes_alt;
  h->orig = f.orig;
  h->orig_alt = f.orig_alt;
  h->cold = f.cold;
  h->cold_alt = f.cold_alt;
  h->gid = f.gid;
  h->gid_alt = f.gid_alt;
  h->s_since = f.since;
  h->s_migrations = f.migrations;
}

// nsub substeps through a cached hipGraph: captured once per (dt, BC masks,
// bins / escape / buffer parities, transport) key and replayed.  A slab with
// the RCCL transport captures its whole step call: the window exchanges
// (grouped ncclSend/ncclRecv on the comm stream, joined into the capture by
// events) and the migrations between chunks, whose counts stay on the device.
// GSMPM_GRAPH_TRACE=1: one stderr line per stage of a capture / replay (diagnostics)
static void gtrace(const char* what) {
  static const bool on = std::getenv("GSMPM_GRAPH_TRACE") && std::getenv("GSMPM_GRAPH_TRACE")[0] == '1';
  if (on) std::fprintf(stderr, "[gsmpm graph] %s\n", what), std::fflush(stderr);
}
static int graph_substeps(gsmpm_mpm* h, float dt, int nsub, const uint32_t* bc, hipStream_t st,
                          const gsmpm_transport* xp) {
  const bool fz = use_fused(h);
  std::vector<uint32_t> key;
  key.reserve(nsub + 14);
  uint32_t dtb;
  std::memcpy(&dtb, &dt, 4);
  key.push_back(dtb);
  key.push_back((uint32_t)nsub);
  key.push_back((uint32_t)h->cur_box);
  key.push_back(fz ? 1u : 0u);
  key.push_back((uint32_t)h->fbpar);
  key.push_back((uint32_t)h->fep);
  key.push_back((uint32_t)h->rebin_interval);
  key.push_back(fold_on(h) ? 1u : 0u);
  key.push_back((uint32_t)h->rebin_m);
  key.push_back(h->planes_alt && h->planes > h->planes_alt ? 1u : 0u);  // which particle buffer is current
  key.push_back(xp ? (uint32_t)(((uintptr_t)xp->comm >> 4) ^ (uint32_t)xp->kind) : 0u);
  if (h->slab) {  // where the migrations fall, and the buffers they swap (rects / capacity changes drop graphs)
    key.push_back((uint32_t)(h->s_since % h->s_interval));
    key.push_back(h->cold_alt && h->cold > h->cold_alt ? 1u : 0u);
    key.push_back(h->gid_alt && h->gid > h->gid_alt ? 1u : 0u);
    key.push_back((uint32_t)h->mig_cap);
    key.push_back(h->s_rebal_pending ? 1u : 0u);  // the call opens with the re-cut's migration
  }
  for (int s = 0; s < nsub; ++s) key.push_back(bc ? bc[s] : 0xffffffffu);
  auto it = h->graphs.find(key);
  if (it == h->graphs.end()) {
    if (h->graphs.size() >= 16) drop_graphs(h);
    hipGraph_t graph;
    int parity = h->cur_box, bp = h->fbpar, ep = h->fep;
    const gsmpm_mpm::FState start = fstate_of(h, bp, ep);
    if (fz) {
      const int rr = sync_rare(h, st);  // k_fused's rare arguments are current before the capture
      if (rr) return rr;
      GSMPM_HIP(hipStreamSynchronize(st));
    }
    gtrace("begin capture");
    GSMPM_HIP(hipStreamBeginCapture(h->cap, hipStreamCaptureModeRelaxed));
    h->capturing = true;
    int rc;
    if (h->slab) {
      rc = slab_body(h, dt, nsub, bc, h->cap, xp);
      gtrace("slab body captured");
      bp = h->fbpar;
      ep = h->fep;
      h->fbpar = start.bpar;
      h->fep = start.ep;
    } else {
      rc = fz ? launch_substeps_f(h, dt, nsub, bc, h->cap, bp, ep, nullptr, nullptr, xp)
              : launch_substeps(h, dt, nsub, bc, h->cap, parity);
    }
    h->capturing = false;
    hipError_t e = hipStreamEndCapture(h->cap, &graph);
    gtrace(e == hipSuccess ? "end capture ok" : "end capture FAILED");
    // capture swapped the particle buffers on the host: keep the end state for
    // the key and start the replay below from the key's state
    gsmpm_mpm::FState end = fstate_of(h, bp, ep);
    end.since -= start.since;  // the counters advance by the graph's own substeps / migrations
    end.migrations -= start.migrations;
    set_fstate(h, start);
    if (rc) {
      if (e == hipSuccess) (void)hipGraphDestroy(graph);
      return rc;
    }
    if (e != hipSuccess) {
      set_error(std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
      return GSMPM_EHIP;
    }
    hipGraphExec_t exec, exec2 = nullptr;
    e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    gtrace(e == hipSuccess ? "instantiated" : "instantiate FAILED");
    if (e == hipSuccess && !h->slab && h->graph_copies > 1) {
      e = hipGraphInstantiate(&exec2, graph, nullptr, nullptr, 0);
      if (e != hipSuccess) (void)hipGraphExecDestroy(exec);
    }
    (void)hipGraphDestroy(graph);
    if (e != hipSuccess) {
      set_error(std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
      return GSMPM_EHIP;
    }
    it = h->graphs.emplace(key, exec).first;
    if (exec2) h->graphs_alt.emplace(key, exec2);
    h->graph_box_parity[key] = parity;
    h->graph_fstate[key] = end;
  }
  gtrace("launch");
  hipGraphExec_t run = it->second;
  auto alt = h->graphs_alt.find(key);
  if (alt != h->graphs_alt.end()) {
    int& turn = h->graph_turn[key];
    if (turn) run = alt->second;
    turn ^= 1;
  }
  GSMPM_HIP(hipGraphLaunch(run, st));
  gtrace("launched");
  h->cur_box = h->graph_box_parity[key];
  const gsmpm_mpm::FState& fs = h->graph_fstate[key];
  h->fbpar = fs.bpar;
  h->fep = fs.ep;
  const long since = h->s_since, migrations = h->s_migrations;
  set_fstate(h, fs);
  h->s_since = since + fs.since;
  h->s_migrations = migrations + fs.migrations;
  return GSMPM_OK;
}
}  // namespace gsmpm

extern "C" {

const char* gsmpm_last_error(void) { return g_err.c_str(); }
int gsmpm_version(void) { return 1; }

int gsmpm_mpm_create(const gsmpm_mpm_params* prm, gsmpm_mpm** out) {
  GSMPM_REQUIRE(prm && out, "gsmpm_mpm_create: null argument");
  GSMPM_REQUIRE(prm->n_particles > 0, "gsmpm_mpm_create: n_particles must be > 0");
  // particle planes are addressed with 32-bit buffer offsets (mpm_common.h)
  GSMPM_REQUIRE((long long)NPLANES * ((prm->n_particles + 255) / 256 * 256) * 4 < (1LL << 31),
                "gsmpm_mpm_create: n_particles too large for one domain (use slabs, < 10.7M)");
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
  // re-binning interval: stress-free jelly every kRebinStressFree substeps; a
  // stress-bearing material's plastic flow amplifies the change of summation
  // order a longer interval brings (metal F_trial 1.22e-4 at 15)
  h->rebin_interval = h->mat_kernel == 0 ? kRebinStressFree : kRebinStress;
  const size_t nn = (size_t)h->g.ng * h->g.ng * h->g.ng;
  auto fail = [&](hipError_t e, const char* what) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    gsmpm_mpm_destroy(h);
    return GSMPM_EHIP;
  };
  hipError_t e;
  if ((e = hipMalloc(&h->planes, sizeof(float) * (size_t)NPLANES * h->np)) != hipSuccess) return fail(e, "hipMalloc planes");
  if ((e = hipMalloc(&h->cold, sizeof(float) * (size_t)NCOLD * h->np)) != hipSuccess) return fail(e, "hipMalloc planes");
  if ((e = hipMemset(h->cold, 0, sizeof(float) * (size_t)NCOLD * h->np)) != hipSuccess) return fail(e, "hipMemset");
  if ((e = hipMalloc(&h->orig, sizeof(int) * (size_t)h->np)) != hipSuccess) return fail(e, "hipMalloc orig");
  if ((e = hipMalloc(&h->gacc, sizeof(float4) * nn)) != hipSuccess) return fail(e, "hipMalloc grid acc");
  if ((e = hipMalloc(&h->gvel, sizeof(float4) * nn)) != hipSuccess) return fail(e, "hipMalloc grid vel");
  h->tl.td = (h->g.ng + kTile - 1) / kTile;
  h->tl.ntiles = h->tl.td * h->tl.td * h->tl.td;
  // every chunk but the last of each tile is full: <= n/256 + occupied tiles
  h->tl.max_chunks = h->n / kChunk + std::min(h->tl.ntiles + 1, h->n) + 1;
  // + one all-zero slot (index max_chunks) that k_grid reads for absent tiles
  if ((e = hipMalloc(&h->slots, sizeof(float4) * (size_t)(h->tl.max_chunks + 1) * kWin)) != hipSuccess)
    return fail(e, "hipMalloc chunk slots");
  if ((e = hipMemset(h->slots + (size_t)h->tl.max_chunks * kWin, 0, sizeof(float4) * kWin)) != hipSuccess)
    return fail(e, "hipMemset");
  for (int c = 0; c < 2; ++c) {
    const size_t E = (size_t)h->tl.ntiles + 1;
    if ((e = hipMalloc(&h->count[c], sizeof(int) * E)) != hipSuccess) return fail(e, "hipMalloc count");
    if ((e = hipMalloc(&h->cstart[c], sizeof(int) * E)) != hipSuccess) return fail(e, "hipMalloc cstart");
    if ((e = hipMalloc(&h->cbase[c], sizeof(int) * E)) != hipSuccess) return fail(e, "hipMalloc cbase");
    if ((e = hipMalloc(&h->chunk[c], sizeof(int4) * (size_t)h->tl.max_chunks)) != hipSuccess) return fail(e, "hipMalloc chunk");
    if ((e = hipMalloc(&h->touched[c], sizeof(int) * (size_t)h->tl.ntiles)) != hipSuccess) return fail(e, "hipMalloc touched");
    if ((e = hipMalloc(&h->tflag[c], sizeof(int) * (size_t)h->tl.ntiles)) != hipSuccess) return fail(e, "hipMalloc tflag");
    if ((e = hipMemset(h->tflag[c], 0, sizeof(int) * (size_t)h->tl.ntiles)) != hipSuccess) return fail(e, "hipMemset");
    if ((e = hipMalloc(&h->nchunk[c], sizeof(int) * 2)) != hipSuccess) return fail(e, "hipMalloc nchunk");
    if ((e = hipMalloc(&h->list[c], sizeof(int) * (size_t)h->np)) != hipSuccess) return fail(e, "hipMalloc list");
    if ((e = hipMemset(h->count[c], 0, sizeof(int) * E)) != hipSuccess) return fail(e, "hipMemset");
    if ((e = hipMemset(h->nchunk[c], 0, sizeof(int) * 2)) != hipSuccess) return fail(e, "hipMemset");
  }
  // fused pipeline: 8 x 8 x 7-cell tiles (fused.h)
  h->fused = !(prm->flags & (GSMPM_FLAG_PHASED | GSMPM_FLAG_KEEP_GRID));
  if (const char* lb = std::getenv("GSMPM_LANE_BALANCE")) h->lane_balance = lb[0] != '0';
  if (const char* gc = std::getenv("GSMPM_GRAPH_COPIES")) h->graph_copies = std::max(1, std::atoi(gc));
  if (const char* fp = std::getenv("GSMPM_FUSE_PERMUTE")) h->fuse_permute = fp[0] != '0';
  if (const char* cr = std::getenv("GSMPM_COVER_RECORDS")) h->cover_records = cr[0] != '0';
  {
    int dev = 0, ncu = 0, per_cu = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_fused<0, 3>, 256, 0) == hipSuccess && ncu > 0 &&
        per_cu > 0) {
      // one round of resident workgroups, or -- a scene of several rounds of
      // full chunks (bicycle's 1M: ~30,000 chunks of ~33 particles) -- up to
      // 6 rounds' worth, so workgroups own fewer chunks each and the
      // dispatcher refills CUs as chunks finish.  Bicycle's k_fused (A/B,
      // GSMPM_FUSED_WGS): 100.8 us at 1 round, 99.2 at 2, 96.7 at 3, 94.4 at 6,
      // 98.5 at one workgroup a chunk; B' (240,549, 1.2 rounds) lost frame
      // time at 2 rounds, so the factor is the floor of the rounds
      h->ncu = ncu;
      const int resident = ncu * per_cu;
      const int rounds = (int)std::min<long long>(6, std::max<long long>(1, (long long)h->n / ((long long)resident * kChunk)));
      h->fused_wgs = resident * rounds;
      // the balanced order only where the workgroups are one resident round
      // (later rounds are placed as CUs free up, not by position): lego and B'
      // gain, bicycle's 5 rounds lost 1 % (profiles/r06/ab_chunk_order_r06n.txt)
      h->chunk_order = rounds == 1;
      h->chunk_xcd_seq = GSMPM_CHUNK_XCD_SEQ && rounds > 1 && GSMPM_CHUNK_XCD && kGridGroup > 0 && h->fused_wgs % 8 == 0;
    }
    if (const char* fw = std::getenv("GSMPM_FUSED_WGS")) h->fused_wgs = std::max(1, std::atoi(fw));
    if (const char* co = std::getenv("GSMPM_CHUNK_ORDER")) h->chunk_order = co[0] != '0';
    if (h->chunk_order) h->chunk_xcd_seq = false;
  }
  h->ftl.td0 = (h->g.ng + kFT0 - 1) / kFT0;
  h->ftl.td1 = (h->g.ng + kFT1 - 1) / kFT1;
  h->ftl.td2 = (h->g.ng + kFT2 - 1) / kFT2;
  h->ftl.ntiles = h->ftl.td0 * h->ftl.td1 * h->ftl.td2;
  h->ftl.max_chunks = h->n / kChunk + std::min(h->ftl.ntiles + 1, h->n) + 1;
  // k_grid_f addresses the window slots with 32-bit byte offsets (fused.h
  // ld_slot): a rank whose slot array would pass 4 GiB (~40M particles) runs
  // the per-phase pipeline instead
  if (h->fused && sizeof(float4) * (size_t)(h->ftl.max_chunks + 1) * kFWin > 0xffffffffull) h->fused = false;
  if (h->fused) {
    const size_t E = (size_t)h->ftl.ntiles + 1;
    if ((e = hipMalloc(&h->fslots, sizeof(float4) * (size_t)(h->ftl.max_chunks + 1) * kFWin)) != hipSuccess)
      return fail(e, "hipMalloc fused slots");
    if ((e = hipMemset(h->fslots + (size_t)h->ftl.max_chunks * kFWin, 0, sizeof(float4) * kFWin)) != hipSuccess)
      return fail(e, "hipMemset");
    for (int c = 0; c < 2; ++c) {
      if ((e = hipMalloc(&h->fcount[c], sizeof(int) * E)) != hipSuccess) return fail(e, "hipMalloc count");
      if ((e = hipMalloc(&h->fcstart[c], sizeof(int) * E)) != hipSuccess) return fail(e, "hipMalloc cstart");
      if ((e = hipMalloc(&h->fcbase[c], sizeof(int) * E)) != hipSuccess) return fail(e, "hipMalloc cbase");
      if ((e = hipMalloc(&h->fchunk[c], sizeof(int4) * (size_t)h->ftl.max_chunks)) != hipSuccess)
        return fail(e, "hipMalloc chunk");
      if ((e = hipMalloc(&h->ftouched[c], sizeof(int) * (size_t)h->ftl.ntiles)) != hipSuccess)
        return fail(e, "hipMalloc touched");
      // entries past the live count are never used, but a read of one must see a valid tile (round 3's
      // uncommitted three-tiles-per-workgroup k_grid_f read past the count: hipErrorIllegalAddress)
      if ((e = hipMemset(h->ftouched[c], 0, sizeof(int) * (size_t)h->ftl.ntiles)) != hipSuccess)
        return fail(e, "hipMemset touched");
      if ((e = hipMalloc(&h->ftflag[c], sizeof(int) * (size_t)h->ftl.ntiles)) != hipSuccess)
        return fail(e, "hipMalloc tflag");
      if ((e = hipMalloc(&h->fnchunk[c], sizeof(int) * 2)) != hipSuccess) return fail(e, "hipMalloc nchunk");
      if ((e = hipMalloc(&h->flist[c], sizeof(int) * (size_t)h->np)) != hipSuccess) return fail(e, "hipMalloc list");
      if ((e = hipMalloc(&h->fcbox[c], sizeof(int) * (size_t)h->ftl.max_chunks)) != hipSuccess)
        return fail(e, "hipMalloc boxes");
      if ((e = hipMalloc(&h->fpchunk[c], sizeof(int4) * (size_t)h->ftl.max_chunks)) != hipSuccess ||
          (e = hipMemset(h->fpchunk[c], 0, sizeof(int4) * (size_t)h->ftl.max_chunks)) != hipSuccess)
        return fail(e, "hipMalloc ordered chunks");
      if ((e = hipMalloc(&h->ftbox[c], sizeof(int) * (size_t)h->ftl.ntiles)) != hipSuccess)
        return fail(e, "hipMalloc boxes");
      if ((e = hipMalloc(&h->frcov[c], sizeof(int2) * kRecStride * (size_t)h->ftl.ntiles)) != hipSuccess ||
          (e = hipMemset(h->frcov[c], 0, sizeof(int2) * kRecStride * (size_t)h->ftl.ntiles)) != hipSuccess)
        return fail(e, "hipMalloc cover records");
      if ((e = hipMalloc(&h->frbox[c], sizeof(int) * kRecStride * (size_t)h->ftl.ntiles)) != hipSuccess ||
          (e = hipMemset(h->frbox[c], 0, sizeof(int) * kRecStride * (size_t)h->ftl.ntiles)) != hipSuccess)
        return fail(e, "hipMalloc cover boxes");
      if ((e = hipMalloc(&h->ftpos[c], sizeof(int) * (size_t)h->ftl.ntiles)) != hipSuccess ||
          (e = hipMemset(h->ftpos[c], 0xff, sizeof(int) * (size_t)h->ftl.ntiles)) != hipSuccess)
        return fail(e, "hipMalloc touched positions");
      if ((e = hipMalloc(&h->fperm[c], (size_t)h->ftl.max_chunks * 256)) != hipSuccess)
        return fail(e, "hipMalloc lane balance");
      if ((e = hipMemset(h->fperm[c], 0, (size_t)h->ftl.max_chunks * 256)) != hipSuccess) return fail(e, "hipMemset");
      if ((e = hipMemset(h->fcount[c], 0, sizeof(int) * E)) != hipSuccess) return fail(e, "hipMemset");
      if ((e = hipMemset(h->ftflag[c], 0, sizeof(int) * (size_t)h->ftl.ntiles)) != hipSuccess) return fail(e, "hipMemset");
      if ((e = hipMemset(h->fnchunk[c], 0, sizeof(int) * 2)) != hipSuccess) return fail(e, "hipMemset");
    }
    if ((e = hipMalloc(&h->planes_alt, sizeof(float) * (size_t)NPLANES * h->np)) != hipSuccess)
      return fail(e, "hipMalloc planes");
    if ((e = hipMemset(h->planes_alt, 0, sizeof(float) * (size_t)NPLANES * h->np)) != hipSuccess)
      return fail(e, "hipMemset");
    if ((e = hipMalloc(&h->orig_alt, sizeof(int) * (size_t)h->np)) != hipSuccess) return fail(e, "hipMalloc orig");
    if ((e = hipMalloc(&h->fesc, sizeof(int) * (4 + kFoldPhases))) != hipSuccess) return fail(e, "hipMalloc escape flags");
    if ((e = hipMemset(h->fesc, 0, sizeof(int) * (4 + kFoldPhases))) != hipSuccess) return fail(e, "hipMemset");
    // FOLD (fused.h): the second slot and tile-box buffers, two more escape accumulators
    if (const char* fo = std::getenv("GSMPM_FOLD")) h->fold = fo[0] != '0';
    if ((e = hipMalloc(&h->fslots2, sizeof(float4) * (size_t)(h->ftl.max_chunks + 1) * kFWin)) != hipSuccess)
      return fail(e, "hipMalloc fused slots");
    if ((e = hipMemset(h->fslots2 + (size_t)h->ftl.max_chunks * kFWin, 0, sizeof(float4) * kFWin)) != hipSuccess)
      return fail(e, "hipMemset");
    h->gacc_f[0] = h->gacc;
    for (int b = 1; b < 3; ++b) {
      if ((e = hipMalloc(&h->gacc_f[b], sizeof(float4) * nn)) != hipSuccess) return fail(e, "hipMalloc grid acc");
      if ((e = hipMemset(h->gacc_f[b], 0, sizeof(float4) * nn)) != hipSuccess) return fail(e, "hipMemset");
    }
    if ((e = hipMalloc(&h->fesc_nodes, sizeof(float4) * 27 * (size_t)h->np)) != hipSuccess)
      return fail(e, "hipMalloc escape nodes");
    if ((e = hipMalloc(&h->vmax_dev, sizeof(unsigned))) != hipSuccess ||
        (e = hipMemset(h->vmax_dev, 0, sizeof(unsigned))) != hipSuccess)
      return fail(e, "hipMalloc vmax");
    if ((e = hipHostMalloc((void**)&h->vmax_host, sizeof(float), hipHostMallocDefault)) != hipSuccess)
      return fail(e, "hipHostMalloc vmax");
    *h->vmax_host = 0.f;
    if (const char* ra = std::getenv("GSMPM_REBIN_AUTO")) h->rebin_auto = ra[0] != '0';
    for (int c = 0; c < 2; ++c) {
      if ((e = hipMalloc(&h->ftbox2[c], sizeof(int) * (size_t)h->ftl.ntiles)) != hipSuccess)
        return fail(e, "hipMalloc boxes");
      if ((e = hipMemset(h->ftbox2[c], 0, sizeof(int) * (size_t)h->ftl.ntiles)) != hipSuccess) return fail(e, "hipMemset");
    }
    if ((e = hipMalloc(&h->frare_dev, sizeof(h->frare_host))) != hipSuccess) return fail(e, "hipMalloc rare args");
  }
  const int scan_tiles = std::max(h->tl.ntiles, h->ftl.ntiles) + 1;
  if ((e = hipMalloc(&h->scan_part, sizeof(int4) * (size_t)div_up(scan_tiles, 1024))) != hipSuccess)
    return fail(e, "hipMalloc scan partials");
  if ((e = hipMalloc(&h->ptile, sizeof(int) * (size_t)h->np)) != hipSuccess) return fail(e, "hipMalloc ptile");
  if ((e = hipMalloc(&h->pslot, sizeof(int) * (size_t)h->np)) != hipSuccess) return fail(e, "hipMalloc pslot");
  if ((e = hipMalloc(&h->dev_bc, sizeof(BcTable))) != hipSuccess) return fail(e, "hipMalloc bc table");
  if ((e = hipMemset(h->gacc, 0, sizeof(float4) * nn)) != hipSuccess) return fail(e, "hipMemset");
  if ((e = hipMemset(h->gvel, 0, sizeof(float4) * nn)) != hipSuccess) return fail(e, "hipMemset");
  if ((e = hipMemset(h->planes, 0, sizeof(float) * (size_t)NPLANES * h->np)) != hipSuccess) return fail(e, "hipMemset");
  if ((e = hipStreamCreateWithFlags(&h->cap, hipStreamNonBlocking)) != hipSuccess) return fail(e, "hipStreamCreate");
  // the non-finite word: written by the kernels only when a position is NaN / Inf,
  // read by the host without a sync (step reports it at its next call)
  if ((e = hipHostMalloc((void**)&h->nonfin_host, 64, hipHostMallocMapped)) != hipSuccess)
    return fail(e, "hipHostMalloc");
  *(volatile int*)h->nonfin_host = 0;
  if ((e = hipHostGetDevicePointer((void**)&h->nonfin_dev, h->nonfin_host, 0)) != hipSuccess)
    return fail(e, "hipHostGetDevicePointer");
  h->host_bc = BcTable{};
  if ((e = hipMemcpy(h->dev_bc, &h->host_bc, sizeof(BcTable), hipMemcpyHostToDevice)) != hipSuccess)
    return fail(e, "hipMemcpy bc");
  if ((e = hipDeviceSynchronize()) != hipSuccess) return fail(e, "init");
  *out = h;
  return GSMPM_OK;
}

int gsmpm_mpm_destroy(gsmpm_mpm* h) {
  if (!h) return GSMPM_OK;
  drop_graphs(h);
  if (h->cap) (void)hipStreamDestroy(h->cap);
  (void)hipFree(h->planes);
  (void)hipFree(h->cold);
  (void)hipFree(h->orig);
  (void)hipFree(h->gacc);
  (void)hipFree(h->gvel);
  (void)hipFree(h->dev_bc);
  (void)hipFree(h->slots);
  for (int c = 0; c < 2; ++c) {
    (void)hipFree(h->count[c]);
    (void)hipFree(h->cstart[c]);
    (void)hipFree(h->cbase[c]);
    (void)hipFree(h->chunk[c]);
    (void)hipFree(h->touched[c]);
    (void)hipFree(h->tflag[c]);
    (void)hipFree(h->nchunk[c]);
    (void)hipFree(h->list[c]);
  }
  for (int c = 0; c < 2; ++c) {
    (void)hipFree(h->fcount[c]);
    (void)hipFree(h->fcstart[c]);
    (void)hipFree(h->fcbase[c]);
    (void)hipFree(h->fchunk[c]);
    (void)hipFree(h->ftouched[c]);
    (void)hipFree(h->ftflag[c]);
    (void)hipFree(h->fnchunk[c]);
    (void)hipFree(h->flist[c]);
    (void)hipFree(h->fcbox[c]);
    (void)hipFree(h->fpchunk[c]);
    (void)hipFree(h->ftbox[c]);
    (void)hipFree(h->fperm[c]);
    (void)hipFree(h->frcov[c]);
    (void)hipFree(h->frbox[c]);
    (void)hipFree(h->ftpos[c]);
  }
  (void)hipFree(h->fslots);
  (void)hipFree(h->fslots2);
  (void)hipFree(h->gacc_f[1]);
  (void)hipFree(h->gacc_f[2]);
  for (int c = 0; c < 2; ++c) (void)hipFree(h->ftbox2[c]);
  (void)hipFree(h->fesc_nodes);
  (void)hipFree(h->vmax_dev);
  if (h->vmax_host) (void)hipHostFree(h->vmax_host);
  (void)hipFree(h->fesc);
  (void)hipFree(h->frare_dev);
  (void)hipFree(h->planes_alt);
  (void)hipFree(h->orig_alt);
  (void)hipFree(h->ptile);
  (void)hipFree(h->scan_part);
  (void)hipFree(h->pslot);
  (void)hipFree(h->planes_tmp);
  (void)hipFree(h->orig_tmp);
  (void)hipFree(h->sort_keys);
  (void)hipFree(h->sort_idx);
  (void)hipFree(h->sort_tmp);
  for (int w = 0; w < 2; ++w) {
    (void)hipFree(h->sw.part[w]);
    (void)hipFree(h->s_recv[w]);
    (void)hipFree(h->mig_send[w]);
    (void)hipFree(h->mig_recv[w]);
  }
  (void)hipFree(h->s_drift);
  (void)hipFree(h->s_wdev);
  (void)hipFree(h->d_n);
  (void)hipFree(h->gid);
  (void)hipFree(h->gid_alt);
  (void)hipFree(h->cold_alt);
  (void)hipFree(h->mig_bcnt);
  (void)hipFree(h->mig_boff);
  (void)hipFree(h->mig_tot);
  (void)hipFree(h->s_rec);
  if (h->s_rec_host) (void)hipHostFree(h->s_rec_host);
  if (h->nonfin_host) (void)hipHostFree(h->nonfin_host);
  if (h->x_host) (void)hipHostFree(h->x_host);
  if (h->s_ev_pack) (void)hipEventDestroy(h->s_ev_pack);
  if (h->s_ev_x) (void)hipEventDestroy(h->s_ev_x);
  if (h->s_comm) (void)hipStreamDestroy(h->s_comm);
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
  if (h->fesc) {  // the fused pipeline's escape flags and the FOLD accumulators: a new state
    GSMPM_HIP(hipMemsetAsync(h->fesc, 0, sizeof(int) * (4 + kFoldPhases), st));
    for (int b = 1; b < 3; ++b) GSMPM_HIP(hipMemsetAsync(h->gacc_f[b], 0, nn * sizeof(float4), st));
  }
  int rc = rebin(h, st);
  if (rc) return rc;
  GSMPM_HIP(hipStreamSynchronize(st));
  *(volatile int*)h->nonfin_host = 0;  // a new state
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

namespace gsmpm {
// The re-binnings of the next step call (fused pipeline, one domain): enough
// that no particle moves more than 0.8 cell between two of them, from the
// fastest velocity component the previous call ended with (read from pinned
// memory without a sync: one or two calls old) plus the velocity gravity can
// add over two calls; at least the count rebin_interval asks for; a call with
// an active impulse (boundary_conditions.py:41-45: an unbounded kick)
// re-bins every 5 substeps.  A spacing that turns out too long only costs
// time: the particles that leave their window take the escape path.
static void choose_rebins(gsmpm_mpm* h, float dt, int nsub, const uint32_t* bc) {
  h->rebin_m = 0;
  if (!h->rebin_auto || h->slab || !h->vmax_host || nsub < 2) return;
  const float vprev = *(volatile float*)h->vmax_host;
  const double g = std::sqrt(h->prm.gravity[0] * h->prm.gravity[0] + h->prm.gravity[1] * h->prm.gravity[1] +
                             h->prm.gravity[2] * h->prm.gravity[2]);
  const double v = (std::isfinite(vprev) ? (double)vprev : 0.0) + 2.0 * g * (double)nsub * dt;
  const double cells = v * (double)nsub * dt * h->g.inv_dx;  // cells the fastest particle crosses in the call
  int m = (int)std::ceil(cells / 0.8);
  bool imp = false;
  for (int b = 0; b < h->host_bc.n_imp && !imp; ++b)
    for (int s = 0; s < nsub && !imp; ++s) imp = !bc || ((bc[s] >> h->host_bc.imp[b].bit) & 1u);
  if (imp) m = std::max(m, (nsub + 4) / 5);
  h->rebin_m = std::min(std::max(m, 0), nsub);
}
}  // namespace gsmpm

int gsmpm_mpm_step(gsmpm_mpm* h, float dt, int32_t nsub, const uint32_t* bc, void* stream) {
  GSMPM_REQUIRE(h, "gsmpm_mpm_step: null handle");
  if (!h->has_particles) {
    set_error("gsmpm_mpm_step: particles not set");
    return GSMPM_ESTATE;
  }
  GSMPM_REQUIRE(nsub >= 0, "gsmpm_mpm_step: n_substeps < 0");
  if (h->slab) {
    set_error("gsmpm_mpm_step: this simulator is one slab of a multi-GPU domain; step it with gsmpm_mpm_slab_step");
    return GSMPM_ESTATE;
  }
  if (*(volatile int*)h->nonfin_host) {
    set_error("gsmpm_mpm_step: particle state (position, mass, velocity, C or stress) became non-finite (NaN / Inf) "
              "in an earlier step; the state is invalid");
    return GSMPM_ESTATE;
  }
  if (nsub == 0) return GSMPM_OK;
  hipStream_t st = (hipStream_t)stream;
  // the fused pipeline keeps storage in bin order; the per-phase one re-sorts
  if (!use_fused(h) && !(h->prm.flags & GSMPM_FLAG_NO_SORT) && h->resort_interval > 0 &&
      h->since_sort >= h->resort_interval) {
    int rc = resort(h, st);
    if (rc) return rc;
  }
  h->since_sort += nsub;
  if (use_fused(h)) choose_rebins(h, dt, nsub, bc);
  const bool use_graph = !(h->prm.flags & GSMPM_FLAG_NO_GRAPH) && nsub >= 2;
  int rc;
  if (!use_graph) {
    int parity = h->cur_box;
    rc = use_fused(h) ? launch_substeps_f(h, dt, nsub, bc, st, h->fbpar, h->fep)
                      : launch_substeps(h, dt, nsub, bc, st, parity);
    h->cur_box = parity;
  } else {
    rc = graph_substeps(h, dt, nsub, bc, st, nullptr);
  }
  // the call's fastest velocity, for the next call's re-binnings (no sync)
  if (!rc && use_fused(h) && h->vmax_host && h->rebin_auto)
    GSMPM_HIP(hipMemcpyAsync(h->vmax_host, h->vmax_dev, sizeof(unsigned), hipMemcpyDeviceToHost, st));
  return rc;
}

int gsmpm_mpm_check_finite(gsmpm_mpm* h, int32_t clear, void* stream) {
  GSMPM_REQUIRE(h, "gsmpm_mpm_check_finite: null handle");
  GSMPM_HIP(hipStreamSynchronize((hipStream_t)stream));
  if (h->slab && h->s_drift) {  // a slab's word is one of its device flags
    int f = 0;
    GSMPM_HIP(hipMemcpy(&f, h->s_drift + SF_NONFIN, sizeof(int), hipMemcpyDeviceToHost));
    if (f) *(volatile int*)h->nonfin_host = 1;
  }
  const int f = *(volatile int*)h->nonfin_host;
  if (clear) {
    *(volatile int*)h->nonfin_host = 0;
    if (h->slab && h->s_drift) GSMPM_HIP(hipMemset(h->s_drift + SF_NONFIN, 0, sizeof(int)));
  }
  if (f) {
    set_error("non-finite (NaN / Inf) particle state (position, mass, velocity, C or stress)");
    return GSMPM_ESTATE;
  }
  return GSMPM_OK;
}

int gsmpm_mpm_set_rebin_interval(gsmpm_mpm* h, int32_t substeps) {
  GSMPM_REQUIRE(h, "gsmpm_mpm_set_rebin_interval: null handle");
  GSMPM_REQUIRE(substeps >= 1, "gsmpm_mpm_set_rebin_interval: substeps must be >= 1");
  h->rebin_interval = substeps;
  h->rebin_auto = false;  // a fixed spacing, as asked
  h->rebin_m = 0;
  return GSMPM_OK;
}

int gsmpm_mpm_pipeline(gsmpm_mpm* h) {
  GSMPM_REQUIRE(h, "gsmpm_mpm_pipeline: null handle");
  return use_fused(h) ? GSMPM_PIPE_FUSED : GSMPM_PIPE_PHASED;
}

int gsmpm_mpm_escapes(gsmpm_mpm* h, int32_t clear, int64_t* out, void* stream) {
  GSMPM_REQUIRE(h && out, "gsmpm_mpm_escapes: null argument");
  *out = 0;
  if (!use_fused(h)) return GSMPM_OK;
  hipStream_t st = (hipStream_t)stream;
  unsigned v = 0;
  unsigned* d = reinterpret_cast<unsigned*>(h->fesc + 3 + kFoldPhases);
  GSMPM_HIP(hipMemcpyAsync(&v, d, sizeof(v), hipMemcpyDeviceToHost, st));
  GSMPM_HIP(hipStreamSynchronize(st));
  if (clear) GSMPM_HIP(hipMemsetAsync(d, 0, sizeof(unsigned), st));
  *out = (int64_t)v;
  return GSMPM_OK;
}

int gsmpm_mpm_rebin_state(gsmpm_mpm* h, int32_t* out3, float* vmax) {
  GSMPM_REQUIRE(h && out3, "gsmpm_mpm_rebin_state: null argument");
  out3[0] = h->rebin_interval;
  out3[1] = h->rebin_auto ? 1 : 0;
  out3[2] = h->rebin_m;
  if (vmax) *vmax = h->vmax_host ? *(volatile float*)h->vmax_host : 0.f;
  return GSMPM_OK;
}

int gsmpm_mpm_folded(gsmpm_mpm* h) {
  GSMPM_REQUIRE(h, "gsmpm_mpm_folded: null handle");
  return use_fused(h) && fold_on(h) ? 1 : 0;
}

int gsmpm_mpm_resort(gsmpm_mpm* h, int32_t interval, void* stream) {
  GSMPM_REQUIRE(h, "gsmpm_mpm_resort: null handle");
  if (interval >= 0) h->resort_interval = interval;
  if (!h->has_particles || (h->prm.flags & GSMPM_FLAG_NO_SORT)) return GSMPM_OK;
  if (use_fused(h)) return rebin_f(h, (hipStream_t)stream);  // storage follows the tile bins
  return resort(h, (hipStream_t)stream);
}

int gsmpm_mpm_postprocess(gsmpm_mpm* h, void* stream) {
  GSMPM_REQUIRE(h, "gsmpm_mpm_postprocess: null handle");
  hipLaunchKernelGGL(k_postprocess, dim3(div_up(h->n, 256)), dim3(256), 0, (hipStream_t)stream, particles_of(h),
                     (const int*)h->orig);
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
  int w, cold;
  const int p0 = plane_of(field, &w, &cold);
  GSMPM_REQUIRE(p0 >= 0, "gsmpm_mpm_get: unknown field");
  hipLaunchKernelGGL(k_get, dim3(div_up(h->n, 256)), dim3(256), 0, (hipStream_t)stream, particles_of(h), h->orig, p0,
                     w, cold, out);
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}

int gsmpm_mpm_set(gsmpm_mpm* h, int32_t field, const float* in, void* stream) {
  GSMPM_REQUIRE(h && in, "gsmpm_mpm_set: null argument");
  int w, cold;
  const int p0 = plane_of(field, &w, &cold);
  GSMPM_REQUIRE(p0 >= 0, "gsmpm_mpm_set: unknown field");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_set, dim3(div_up(h->n, 256)), dim3(256), 0, st, particles_of(h), h->orig, p0, w, cold, in);
  GSMPM_LAUNCH_CHECK();
  if (field == GSMPM_FIELD_X) return rebin(h, st);
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
  for (int k = 0; k < 4; ++k) kernel_ms[k] = 0.f;
  if (nsub == 0) return GSMPM_OK;
  if (use_fused(h)) {
    std::vector<hipEvent_t> ev(8 * (size_t)(nsub + 1));
    for (auto& e : ev) GSMPM_HIP(hipEventCreate(&e));
    int rc = launch_substeps_f(h, dt, nsub, bc, st, h->fbpar, h->fep, ev.data(), kernel_ms);
    for (auto& e : ev) (void)hipEventDestroy(e);
    return rc;
  }
  std::vector<hipEvent_t> ev(8 * (size_t)nsub);
  for (auto& e : ev) GSMPM_HIP(hipEventCreate(&e));
  int parity = h->cur_box;
  int rc = launch_substeps(h, dt, nsub, bc, st, parity, ev.data(), kernel_ms);
  h->cur_box = parity;
  for (auto& e : ev) (void)hipEventDestroy(e);
  return rc;
}

// fused pipeline: ms4 = {k_fused (G2P + P2G), k_grid_f, binning, 0}; state restored afterwards
static int time_kernels_f(gsmpm_mpm* h, float dt, uint32_t mask, int reps, float* ms4, hipStream_t st, size_t pbytes) {
  const int c = h->fbpar, ep = h->fep;
  const size_t nn = (size_t)h->g.ng * h->g.ng * h->g.ng;
  hipEvent_t e[2];
  GSMPM_HIP(hipEventCreate(&e[0]));
  GSMPM_HIP(hipEventCreate(&e[1]));
  auto timed = [&](int k, auto&& body) -> int {
    GSMPM_HIP(hipEventRecord(e[0], st));
    for (int r = 0; r < reps; ++r) {
      int rc = body();
      if (rc) return rc;
    }
    GSMPM_HIP(hipEventRecord(e[1], st));
    GSMPM_HIP(hipEventSynchronize(e[1]));
    float ms = 0.f;
    GSMPM_HIP(hipEventElapsedTime(&ms, e[0], e[1]));
    ms4[k] = ms / reps;
    return GSMPM_OK;
  };
  ms4[3] = 0.f;
  int rc = launch_fused(h, 2, c, false, false, mask, dt, ep, st, nullptr);  // windows of the current x
  if (!rc) rc = launch_grid_f(h, c, dt, mask, ep, nullptr, nullptr, st, nullptr);
  if (!rc) rc = timed(0, [&]() { return launch_fused(h, 3, c, false, true, mask, dt, ep, st, nullptr); });
  if (!rc) {
    GSMPM_HIP(hipMemsetAsync(h->fesc, 0, 2 * sizeof(int), st));  // time the touched-tile update
    rc = timed(1, [&]() { return launch_grid_f(h, c, dt, mask, ep, nullptr, nullptr, st, nullptr); });
  }
  if (!rc) {
    GSMPM_HIP(hipMemsetAsync(h->fcount[c ^ 1], 0, sizeof(int) * (h->ftl.ntiles + 1), st));
    GSMPM_HIP(hipMemsetAsync(h->ftflag[c ^ 1], 0, sizeof(int) * h->ftl.ntiles, st));
    rc = launch_fused(h, 1, c, true, true, mask, dt, ep, st, nullptr);
    if (!rc) rc = timed(2, [&]() { return finish_binning_f(h, c ^ 1, st); });
  }
  (void)hipEventDestroy(e[0]);
  (void)hipEventDestroy(e[1]);
  if (rc) return rc;
  GSMPM_HIP(hipMemcpyAsync(h->planes, h->planes_tmp, pbytes, hipMemcpyDeviceToDevice, st));
  GSMPM_HIP(hipMemsetAsync(h->fesc, 0, 2 * sizeof(int), st));
  GSMPM_HIP(hipMemsetAsync(h->gacc, 0, nn * sizeof(float4), st));
  return rebin(h, st);
}

int gsmpm_mpm_time_kernels(gsmpm_mpm* h, float dt, uint32_t bc_active, int32_t reps, float* ms4, void* stream) {
  GSMPM_REQUIRE(h && ms4 && reps > 0, "gsmpm_mpm_time_kernels: bad argument");
  if (!h->has_particles) {
    set_error("gsmpm_mpm_time_kernels: particles not set");
    return GSMPM_ESTATE;
  }
  hipStream_t st = (hipStream_t)stream;
  const size_t pbytes = sizeof(float) * (size_t)NPLANES * h->np;
  if (!h->planes_tmp) GSMPM_HIP(hipMalloc(&h->planes_tmp, pbytes));
  GSMPM_HIP(hipMemcpyAsync(h->planes_tmp, h->planes, pbytes, hipMemcpyDeviceToDevice, st));
  if (use_fused(h)) return time_kernels_f(h, dt, bc_active, reps, ms4, st, pbytes);
  const int c = h->cur_box, nx = c ^ 1;
  const GridStep gs = grid_step(h, dt, bc_active);
  hipEvent_t e[2];
  GSMPM_HIP(hipEventCreate(&e[0]));
  GSMPM_HIP(hipEventCreate(&e[1]));
  auto grid = [&]() {
    launch(nullptr, k_grid, dim3(grid_grid(h)), dim3(512), st, h->g, h->tl, chunk_in(h, c), (const float4*)h->slots,
           h->gacc, h->gvel, (const BcTable*)h->dev_bc, gs, bin_out(h, nx));
  };
  auto g2p = [&]() {
    launch(nullptr, k_g2p, dim3(g2p_grid(h)), dim3(kChunk), st, particles_of(h), h->g, h->tl, chunk_in(h, c),
           bin_out(h, nx), (const float4*)h->gvel, dt);
  };
  auto timed = [&](int k, auto&& body) -> int {
    GSMPM_HIP(hipEventRecord(e[0], st));
    for (int r = 0; r < reps; ++r) body();
    GSMPM_HIP(hipEventRecord(e[1], st));
    GSMPM_HIP(hipEventSynchronize(e[1]));
    float ms = 0.f;
    GSMPM_HIP(hipEventElapsedTime(&ms, e[0], e[1]));
    ms4[k] = ms / reps;
    return GSMPM_OK;
  };
  int rc = timed(0, [&]() {
    switch (h->mat_kernel) {
      case 0: launch_p2g<0>(h, c, bc_active, dt, st, nullptr); break;
      case 1: launch_p2g<1>(h, c, bc_active, dt, st, nullptr); break;
      case 2: launch_p2g<2>(h, c, bc_active, dt, st, nullptr); break;
      case 3: launch_p2g<3>(h, c, bc_active, dt, st, nullptr); break;
      default: launch_p2g<4>(h, c, bc_active, dt, st, nullptr); break;
    }
  });
  if (!rc) rc = timed(1, grid);
  if (!rc) rc = timed(2, g2p);
  if (!rc) {
    grid();  // fresh bins of parity nx from one G2P, then time the binning on them
    g2p();
    rc = timed(3, [&]() { finish_binning(h, nx, st); });
  }
  (void)hipEventDestroy(e[0]);
  (void)hipEventDestroy(e[1]);
  if (rc) return rc;
  // restore the state: the repeated G2P launches advanced the particles
  GSMPM_HIP(hipMemcpyAsync(h->planes, h->planes_tmp, pbytes, hipMemcpyDeviceToDevice, st));
  return rebin(h, st);
}

int gsmpm_mpm_debug_stats(gsmpm_mpm* h, int32_t* out8, void* stream) {
  GSMPM_REQUIRE(h && out8, "gsmpm_mpm_debug_stats: null argument");
  hipStream_t st = (hipStream_t)stream;
  const bool fz = use_fused(h);
  const int ntiles = fz ? h->ftl.ntiles : h->tl.ntiles, par = fz ? h->fbpar : h->cur_box;
  std::vector<int> hc(ntiles + 1);
  int nch[2] = {0, 0};
  GSMPM_HIP(hipMemcpyAsync(hc.data(), fz ? h->fcount[par] : h->count[par], sizeof(int) * hc.size(),
                           hipMemcpyDeviceToHost, st));
  GSMPM_HIP(hipMemcpyAsync(nch, fz ? h->fnchunk[par] : h->nchunk[par], sizeof(int) * 2, hipMemcpyDeviceToHost, st));
  GSMPM_HIP(hipStreamSynchronize(st));
  int active = 0, mx = 0;
  long tot = 0;
  for (int t = 0; t < ntiles; ++t) {
    active += hc[t] > 0;
    mx = std::max(mx, hc[t]);
    tot += hc[t];
  }
  out8[0] = active;
  out8[1] = mx;
  out8[2] = hc[ntiles];  // particles outside the grid
  out8[3] = nch[0];
  out8[4] = nch[1];  // tiles owned by the next grid update
  out8[5] = (int)tot;
  out8[6] = par;
  out8[7] = (int)h->since_sort;
  return GSMPM_OK;
}

int gsmpm_debug_stamps(uint64_t* out, void* stream) {
  GSMPM_REQUIRE(out, "gsmpm_debug_stamps: null argument");
#ifdef GSMPM_STAMPS
  GSMPM_HIP(hipStreamSynchronize((hipStream_t)stream));
  GSMPM_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 4 * kStampWGs * 8));
  return GSMPM_OK;
#else
  (void)stream;
  GSMPM_REQUIRE(false, "gsmpm_debug_stamps: library built without -DGSMPM_STAMPS");
#endif
}

int gsmpm_mpm_live_box(gsmpm_mpm* h, int32_t* box6, void* stream) {
  GSMPM_REQUIRE(h && box6, "gsmpm_mpm_live_box: null argument");
  // node box of the tiles the next grid update owns
  hipStream_t st = (hipStream_t)stream;
  const bool fz = use_fused(h);
  const int c = fz ? h->fbpar : h->cur_box, td = h->tl.td;
  int nch[2] = {0, 0};
  GSMPM_HIP(hipMemcpyAsync(nch, fz ? h->fnchunk[c] : h->nchunk[c], sizeof(int) * 2, hipMemcpyDeviceToHost, st));
  GSMPM_HIP(hipStreamSynchronize(st));
  std::vector<int> tl(nch[1]);
  if (nch[1] > 0) {
    GSMPM_HIP(hipMemcpyAsync(tl.data(), fz ? h->ftouched[c] : h->touched[c], sizeof(int) * nch[1],
                             hipMemcpyDeviceToHost, st));
    GSMPM_HIP(hipStreamSynchronize(st));
  }
  for (int d = 0; d < 3; ++d) {
    box6[d] = INT_MAX;
    box6[3 + d] = INT_MIN;
  }
  const int fT[3] = {kFT0, kFT1, kFT2};
  for (int t : tl) {
    int tc[3], T[3];
    if (fz) {
      tc[2] = t % h->ftl.td2;
      tc[1] = (t / h->ftl.td2) % h->ftl.td1;
      tc[0] = t / (h->ftl.td1 * h->ftl.td2);
      for (int d = 0; d < 3; ++d) T[d] = fT[d];
    } else {
      tc[0] = t / (td * td);
      tc[1] = (t / td) % td;
      tc[2] = t % td;
      for (int d = 0; d < 3; ++d) T[d] = kTile;
    }
    for (int d = 0; d < 3; ++d) {
      box6[d] = std::min(box6[d], tc[d] * T[d]);
      box6[3 + d] = std::max(box6[3 + d], std::min(h->g.ng - 1, tc[d] * T[d] + T[d] - 1));
    }
  }
  return GSMPM_OK;
}

int gsmpm_constitutive(int32_t material, const float* Ft, int32_t n, const float* mu, const float* lam, float* yld,
                       float dt, float* Fo, float* To, void* stream) {
  GSMPM_REQUIRE(Ft && mu && lam && yld && Fo && To && n >= 0, "gsmpm_constitutive: bad argument");
  GSMPM_REQUIRE(material >= 0 && material <= 5, "gsmpm_constitutive: material must be 0..5");
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
    case 4: hipLaunchKernelGGL(k_constitutive<4>, g, b, 0, st, Ft, n, mu, lam, yld, dt, mc, Fo, To); break;
    default: hipLaunchKernelGGL(k_constitutive<5>, g, b, 0, st, Ft, n, mu, lam, yld, dt, mc, Fo, To); break;
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

#include "slab_host.inc"

// fit.hip -- differentiable MPM (the reference's args.fitting=True path) for gfx950.
//
// Reference: MPM_Simulator.p2g2p_forward / p2g2p_backward / learn /
// postprocess_forward / _backward / clear_grads (mpm_solver/solver.py:54-108,
// 167-177), MPM_state_opt (model.py:135-223) and the _opt kernels
// (utils.py:56-76 compute_stress_from_F_opt, 136-174 p2g_opt, 177-183
// grid_normalization_and_gravity, 284-347 g2p_opt, 349-362
// compute_mu_lam_from_E_nu, 435-467 compute_cov_from_F_opt).  The reference
// differentiates those kernels with Taichi's reverse mode; the adjoints here are
// the analytic chain rule of the same f32 expressions with Taichi's accumulation
// behaviour (oracle/diff_oracle.c states it and is checked by finite
// differences):
//   * adjoints accumulate and are cleared only by clear_grads;
//   * the grid adjoints are not cleared between substeps;
//   * grid_mass has no adjoint;
//   * the BC store has no adjoint (the grid adjoint passes through it);
//   * the mu/lam -> logE/y adjoint runs every substep on the accumulated
//     mu/lam adjoints.
//
// Layout (HBM): every per-particle quantity is a plane of np floats
// (np = N rounded up to 256) in an internal, tile-sorted particle order (fixed
// at set_particles, so a workgroup's particles share grid nodes); leveled
// fields are [L][width][np].  The dense grid (n^3 nodes, (ix*n+iy)*n+iz) is
// planar too: m | v_in xyz | v_out xyz | v_in.grad xyz | v_out.grad xyz.
//
// Scatters (P2G, and the G2P adjoint into v_out.grad) bin the level's
// particles into 8^3-cell tiles (count / scan / place, cached per level),
// accumulate each chunk of <= 256 same-tile particles into a 10^3-node LDS
// window as 64-bit fixed point (ds_add_u64: ~9 cycles per wave-instruction on
// gfx950 against ~192 for ds_add_f32, tools/ubench/lds_atomics.hip; per-chunk,
// per-channel power-of-two scales chosen from a bound on the contributions),
// and store the window to the chunk's slot with plain stores.  The grid
// kernels then sum the chunk windows covering each node in a fixed order; no
// global float atomic is used (scattered ones run ~17x below the atomic byte
// rate, MI355X_MICROARCH.md "Global float atomics").  Sums inside a window are
// exact; which particles share a chunk follows the binning's atomic ranks, so
// results can still differ in the last bits from run to run.  Gathers (G2P, the P2G adjoint) read the grid planes directly,
// one thread per particle.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"

namespace gsmpm {
namespace fit {

constexpr int kTile = 8;
constexpr int kWin = 10;
constexpr int kWin3 = kWin * kWin * kWin;
constexpr int kChunk = 256;

struct View {
  int n, np, ng, L, nta, ntiles, max_chunks;
  long nn;
  float dx, inv_dx, gx_, gy_, gz_;
  int has_box;
  float bc0, bc1, bc2, bs0, bs1, bs2;
  float *x, *v, *F, *C, *S;           // [L][w][np]
  float *gx, *gv, *gF, *gC, *gS;      // adjoints
  float *vol, *mass, *logE, *y, *mu, *lam, *glogE, *gy, *gmu, *glam;  // [np]
  float *icov, *cov, *gcov;           // [6][np]
  float *gm, *vin, *vout, *gvin, *gvout;  // grid planes
  long gstride;  // level stride of gm | vin | vout (7 nn: one grid per level), or 0 (one grid)
  int *count, *cbase, *cstart, *tl, *rk, *perm, *nchunks;  // count, cbase: [L][ntiles]
  int4* chunks;
  float4* slots;  // [max_chunks + 1][kWin3] chunk windows; slot max_chunks stays 0
};

// the (m | v_in | v_out) planes of level s
__device__ __forceinline__ float* glv(float* base, const View& V, int s) { return base + (size_t)s * V.gstride; }

__device__ __forceinline__ float* pl(float* base, const View& V, int s, int w, int c) {
  return base + ((size_t)s * w + c) * V.np;
}

__device__ __forceinline__ void bsp(const float x[3], float inv_dx, int base[3], float fx[3], float w[3][3],
                                    float dw[3][3]) {
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

__device__ __forceinline__ int tile_axis(int b, const View& V) { return min(max(b, 0), V.ng - 3) >> 3; }

__device__ __forceinline__ void load_x(const View& V, int s, int p, float x[3]) {
  for (int d = 0; d < 3; ++d) x[d] = pl(V.x, V, s, 3, d)[p];
}
__device__ __forceinline__ void load9(float* base, const View& V, int s, int p, float m[9]) {
  for (int c = 0; c < 9; ++c) m[c] = pl(base, V, s, 9, c)[p];
}
__device__ __forceinline__ void store9(float* base, const View& V, int s, int p, const float m[9]) {
  for (int c = 0; c < 9; ++c) pl(base, V, s, 9, c)[p] = m[c];
}
__device__ __forceinline__ float det3(const float F[9]) {
  return F[0] * (F[4] * F[8] - F[5] * F[7]) - F[1] * (F[3] * F[8] - F[5] * F[6]) + F[2] * (F[3] * F[7] - F[4] * F[6]);
}

// ------------------------------------------------------------- binning ---
__device__ __forceinline__ int tile_of_x(const float x[3], const View& V) {
  int t[3];
  for (int d = 0; d < 3; ++d) t[d] = tile_axis((int)(x[d] * V.inv_dx - 0.5f), V);
  return (t[0] * V.nta + t[1]) * V.nta + t[2];
}
// Rank of each active lane's particle inside its tile (count: that level's
// per-tile counters, zero before the level's first call).  Lanes of a wave
// that share a tile (the common case: particles are stored tile-sorted) take
// their ranks from ONE returning atomic per distinct tile.
__device__ __forceinline__ void count_rank(const View& V, int* count, int p, bool on, int tile) {
  const int lane = __lane_id();
  const unsigned long long below = (1ull << lane) - 1ull;
  unsigned long long pending = __ballot(on);
  int rank = 0;
  while (pending) {
    const int leader = __ffsll((long long)pending) - 1;
    const int key = __shfl(tile, leader);
    const unsigned long long m = __ballot(tile == key) & pending;
    int base = 0;
    if (lane == leader) base = atomicAdd(&count[key], __popcll(m));
    base = __shfl(base, leader);
    if ((m >> lane) & 1ull) rank = base + __popcll(m & below);
    pending &= ~m;
  }
  if (on) {
    V.tl[p] = tile;
    V.rk[p] = rank;
  }
}

// Tile of every particle of level s and its rank inside the tile.
__global__ __launch_bounds__(256) void k_count(View V, int s) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const bool on = p < V.n;
  int tile = -1;
  if (on) {
    float x[3];
    load_x(V, s, p, x);
    tile = tile_of_x(x, V);
  }
  count_rank(V, V.count + (size_t)s * V.ntiles, p, on, tile);
}

// inclusive scan of one value per thread over a 1024-thread block
__device__ __forceinline__ int block_incl_scan(int v, int* s_w) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(v, o);
    if (lane >= o) v += y;
  }
  if (lane == 63) s_w[wid] = v;
  __syncthreads();
  if (wid == 0) {
    int t = lane < 16 ? s_w[lane] : 0;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const int y = __shfl_up(t, o);
      if (lane >= o) t += y;
    }
    if (lane < 16) s_w[lane] = t;
  }
  __syncthreads();
  const int r = v + (wid ? s_w[wid - 1] : 0);
  __syncthreads();
  return r;
}

// One workgroup: tile starts and the <=256-particle chunk records of level s.
__global__ __launch_bounds__(1024) void k_scan(View V, int s) {
  __shared__ int s_w[16];
  __shared__ int s_carry[2];
  if (threadIdx.x == 0) s_carry[0] = s_carry[1] = 0;
  __syncthreads();
  int4* chunks = V.chunks + (size_t)s * V.max_chunks;
  const int* count = V.count + (size_t)s * V.ntiles;
  int* cbase = V.cbase + (size_t)s * V.ntiles;
  for (int b = 0; b < V.ntiles; b += 1024) {
    const int t = b + threadIdx.x;
    const int cnt = t < V.ntiles ? count[t] : 0;
    const int nch = (cnt + kChunk - 1) / kChunk;
    const int ci = block_incl_scan(cnt, s_w);
    const int hi = block_incl_scan(nch, s_w);
    const int c0 = s_carry[0], h0 = s_carry[1];
    if (t < V.ntiles) {
      const int start = c0 + ci - cnt, cb = h0 + hi - nch;
      V.cstart[t] = start;
      cbase[t] = cb;
      for (int j = 0; j < nch; ++j) chunks[cb + j] = make_int4(t, start + j * kChunk, min(kChunk, cnt - j * kChunk), 0);
    }
    __syncthreads();
    if (threadIdx.x == 1023) {
      s_carry[0] = c0 + ci;
      s_carry[1] = h0 + hi;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) V.nchunks[s] = s_carry[1];
}

__global__ __launch_bounds__(256) void k_place(View V, int s) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= V.n) return;
  V.perm[(size_t)s * V.np + V.cstart[V.tl[p]] + V.rk[p]] = p;
}

// k_scan + k_place in one launch for grids of <= kScanTiles tiles: every
// workgroup scans the (L2-resident) tile counts itself, workgroup 0 writes the
// chunk records; then each lane places its particle.  zero_next: zero the
// next level's counters (the G2P that produces that level counts into them).
constexpr int kScanTiles = 8192;
__global__ __launch_bounds__(256) void k_scanplace(View V, int s, int zero_next) {
  __shared__ int s_start[kScanTiles];
  __shared__ int s_w[8];
  const int* count = V.count + (size_t)s * V.ntiles;
  const int nt = V.ntiles, per = (nt + 255) / 256;
  const int t0 = min((int)threadIdx.x * per, nt), t1 = min(t0 + per, nt);
  int sc = 0, sh = 0;
  for (int t = t0; t < t1; ++t) {
    const int c = count[t];
    sc += c;
    sh += (c + kChunk - 1) / kChunk;
  }
  // exclusive scans of (particles, chunks) over the 256 segments
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int ic = sc, ih = sh;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int yc = __shfl_up(ic, o), yh = __shfl_up(ih, o);
    if (lane >= o) {
      ic += yc;
      ih += yh;
    }
  }
  if (lane == 63) {
    s_w[wid] = ic;
    s_w[4 + wid] = ih;
  }
  __syncthreads();
  int bc = 0, bh = 0;
  for (int q = 0; q < wid; ++q) {
    bc += s_w[q];
    bh += s_w[4 + q];
  }
  int c0 = bc + ic - sc, h0 = bh + ih - sh;
  int4* chunks = V.chunks + (size_t)s * V.max_chunks;
  int* cbase = V.cbase + (size_t)s * V.ntiles;
  for (int t = t0; t < t1; ++t) {
    const int c = count[t], nch = (c + kChunk - 1) / kChunk;
    s_start[t] = c0;
    if (blockIdx.x == 0) {
      cbase[t] = h0;
      for (int j = 0; j < nch; ++j) chunks[h0 + j] = make_int4(t, c0 + j * kChunk, min(kChunk, c - j * kChunk), 0);
    }
    c0 += c;
    h0 += nch;
  }
  if (blockIdx.x == 0 && threadIdx.x == 255) V.nchunks[s] = h0;
  __syncthreads();
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < V.n) V.perm[(size_t)s * V.np + s_start[V.tl[p]] + V.rk[p]] = p;
  if (zero_next) {
    int* cn = V.count + (size_t)(s + 1) * V.ntiles;
    for (int t = p; t < nt; t += gridDim.x * blockDim.x) cn[t] = 0;
  }
}

// ------------------------------------------------------------- forward ---
// compute_stress_from_F_opt (utils.py:56-76): StVK on the Green strain,
// sigma = F S F^T / J with |J| clamped to >= 1e-2.
__device__ __forceinline__ void stvk_stress(const float F[9], float mu, float lam, float sig[9]) {
  float J = det3(F);
  if (fabsf(J) < 1e-2f) J = 1e-2f * (J > 0.f ? 1.f : (J < 0.f ? -1.f : 0.f));
  float E[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      const float ftf = F[0 * 3 + i] * F[0 * 3 + j] + F[1 * 3 + i] * F[1 * 3 + j] + F[2 * 3 + i] * F[2 * 3 + j];
      E[i * 3 + j] = 0.5f * (ftf - (i == j ? 1.f : 0.f));
    }
  const float tr = E[0] + E[4] + E[8];
  float Sm[9], FS[9];
  for (int i = 0; i < 9; ++i) Sm[i] = 2.0f * mu * E[i] + ((i % 4) == 0 ? lam * tr : 0.f);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      FS[i * 3 + j] = F[i * 3 + 0] * Sm[0 * 3 + j] + F[i * 3 + 1] * Sm[1 * 3 + j] + F[i * 3 + 2] * Sm[2 * 3 + j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      sig[i * 3 + j] = (FS[i * 3 + 0] * F[j * 3 + 0] + FS[i * 3 + 1] * F[j * 3 + 1] + FS[i * 3 + 2] * F[j * 3 + 2]) / J;
}

// ------------------------------------------------ fixed-point LDS windows ---
// v * 2^S rounded to an integer as two's complement int64 (|v * 2^S| < 2^51):
// adding 1.5 * 2^52 in f64 leaves the integer in the low mantissa bits.
__device__ __forceinline__ unsigned long long to_fixed(float v, double scale) {
  const double d = __builtin_fma((double)v, scale, 6755399441055744.0);
  return (unsigned long long)__double_as_longlong(d) - 0x4338000000000000ull;
}
__device__ __forceinline__ void lds_add(unsigned long long* a, unsigned long long v) {
  __hip_atomic_fetch_add(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Workgroup max of a per-lane bound on |contribution| -> scale 2^S with every
// scaled contribution below 2^50 (to_fixed needs < 2^51); a node sums <= 256
// of them, < 2^58: no int64 overflow.  Resolution: 2^-50 of the chunk's bound.
__device__ __forceinline__ int chunk_exponent(float bound, float* s_max, int slot) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) bound = fmaxf(bound, __shfl_xor(bound, o));
  if ((threadIdx.x & 63) == 0) s_max[slot * 4 + (threadIdx.x >> 6)] = bound;
  __syncthreads();
  const float* m = s_max + slot * 4;
  const float b = fmaxf(fmaxf(m[0], m[1]), fmaxf(m[2], m[3]));
  int e;
  frexpf(b, &e);  // b < 2^e
  return b > 0.f ? 50 - e : 0;
}

// Window (nch u64 planes) -> the chunk's slot: float4 per node, channel c -> .x/.y/.z/.w
__device__ __forceinline__ void store_window(const View& V, const unsigned long long* win, int nch, const int* S,
                                             int chunk) {
  float4* dst = V.slots + (size_t)chunk * kWin3;
  for (int l = threadIdx.x; l < kWin3; l += kChunk) {
    float c[4] = {0.f, 0.f, 0.f, 0.f};
    for (int ch = 0; ch < nch; ++ch) c[ch] = (float)ldexp((double)(long long)win[ch * kWin3 + l], -S[ch]);
    // write-through: the grid kernels read the slots from other XCDs (common.h)
    wt_store4(dst + l, make_float4(c[0], c[1], c[2], c[3]));
  }
}

// p2g_opt (utils.py:136-174), one workgroup per chunk of same-tile particles.
// RECOMPUTE: the backward pass's redo of P2G (solver.py:75-78) reads
// stress[s]; the forward pass computes and stores it (fused stress kernel).
// Slot layout: (m v_in x, y, z, m).
template <bool RECOMPUTE>
__global__ __launch_bounds__(kChunk) void k_p2g(View V, int s, float dt) {
  __shared__ unsigned long long win[4 * kWin3];
  __shared__ float s_max[8];
  const int c = blockIdx.x;
  if (c >= V.nchunks[s]) return;
  const int4 rec = V.chunks[(size_t)s * V.max_chunks + c];
  for (int l = threadIdx.x; l < 4 * kWin3; l += kChunk) win[l] = 0ull;
  const int tz = rec.x % V.nta, ty = (rec.x / V.nta) % V.nta, tx = rec.x / (V.nta * V.nta);
  const int ox = tx * kTile, oy = ty * kTile, oz = tz * kTile;
  const bool on = (int)threadIdx.x < rec.z;
  float x[3] = {0.f, 0.f, 0.f}, vv[3] = {0.f, 0.f, 0.f}, Cm[9] = {0.f}, sg[9] = {0.f}, m = 0.f, vol = 0.f;
  float bm = 0.f, bv = 0.f;
  if (on) {
    const int p = V.perm[(size_t)s * V.np + rec.y + threadIdx.x];
    load_x(V, s, p, x);
    for (int d = 0; d < 3; ++d) vv[d] = pl(V.v, V, s, 3, d)[p];
    load9(V.C, V, s, p, Cm);
    if (RECOMPUTE) {
      load9(V.S, V, s, p, sg);
    } else {
      float Fm[9];
      load9(V.F, V, s, p, Fm);
      stvk_stress(Fm, V.mu[p], V.lam[p], sg);
      store9(V.S, V, s, p, sg);
    }
    m = V.mass[p];
    vol = V.vol[p];
    float vm = 0.f, cm = 0.f, sm = 0.f;
    for (int r = 0; r < 3; ++r) vm = fmaxf(vm, fabsf(vv[r]));
    for (int i = 0; i < 9; ++i) {
      cm = fmaxf(cm, fabsf(Cm[i]));
      sm = fmaxf(sm, fabsf(sg[i]));
    }
    // |weight| <= 1, |dpos| <= 1.5 dx, |gw| <= inv_dx per component
    bm = m * 1.01f;
    bv = (m * (vm + 4.5f * V.dx * cm) + fabsf(dt) * vol * 3.0f * V.inv_dx * sm) * 1.01f;
  }
  int S[4];
  S[3] = chunk_exponent(bm, s_max, 0);
  S[0] = S[1] = S[2] = chunk_exponent(bv, s_max, 1);  // its barrier also orders the zeroing
  if (on) {
    const double sc_v = ldexp(1.0, S[0]), sc_m = ldexp(1.0, S[3]);
    int base[3];
    float fx[3], w[3][3], dw[3][3];
    bsp(x, V.inv_dx, base, fx, w, dw);
    const int lb0 = base[0] - ox, lb1 = base[1] - oy, lb2 = base[2] - oz;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        for (int k = 0; k < 3; ++k) {
          const int a = lb0 + i, b = lb1 + j, cc = lb2 + k;
          if ((unsigned)a >= (unsigned)kWin || (unsigned)b >= (unsigned)kWin || (unsigned)cc >= (unsigned)kWin) continue;
          const int o[3] = {i, j, k};
          float dpos[3];
          for (int d = 0; d < 3; ++d) dpos[d] = ((float)o[d] - fx[d]) * V.dx;
          const float weight = w[0][i] * w[1][j] * w[2][k];
          const float gw[3] = {V.inv_dx * dw[0][i] * w[1][j] * w[2][k], V.inv_dx * w[0][i] * dw[1][j] * w[2][k],
                               V.inv_dx * w[0][i] * w[1][j] * dw[2][k]};
          const int l = (a * kWin + b) * kWin + cc;
          for (int r = 0; r < 3; ++r) {
            const float cd = Cm[r * 3 + 0] * dpos[0] + Cm[r * 3 + 1] * dpos[1] + Cm[r * 3 + 2] * dpos[2];
            const float ef = -vol * (sg[r * 3 + 0] * gw[0] + sg[r * 3 + 1] * gw[1] + sg[r * 3 + 2] * gw[2]);
            lds_add(&win[r * kWin3 + l], to_fixed(weight * m * (vv[r] + cd) + dt * ef, sc_v));
          }
          lds_add(&win[3 * kWin3 + l], to_fixed(weight * m, sc_m));
        }
  }
  __syncthreads();
  store_window(V, win, 4, S, c);
}

// Grid kernels run one 512-thread workgroup per 8^3 block of owned nodes
// (ceil(n/8)^3 blocks; nodes past the particle tiles' range are owned by the
// last blocks).  Lanes 0..7 first fetch the chunk range of the <= 8 particle
// tiles whose 10^3 windows cover the block; each thread then sums its node's
// windows in a fixed order (covering tile, then chunk).
constexpr int kGridWG = kTile * kTile * kTile;

__device__ __forceinline__ void load_cover(const View& V, int s, int bx, int by, int bz, int* s_c0, int* s_nc) {
  if (threadIdx.x < 8) {
    const int a = threadIdx.x >> 2, b = (threadIdx.x >> 1) & 1, c = threadIdx.x & 1;
    const int tx = bx - a, ty = by - b, tz = bz - c;
    int c0 = 0, nc = 0;
    if (tx >= 0 && ty >= 0 && tz >= 0 && tx < V.nta && ty < V.nta && tz < V.nta) {
      const int t = (tx * V.nta + ty) * V.nta + tz;
      nc = (V.count[(size_t)s * V.ntiles + t] + kChunk - 1) / kChunk;
      c0 = V.cbase[(size_t)s * V.ntiles + t];
    }
    s_c0[threadIdx.x] = c0;
    s_nc[threadIdx.x] = nc;
  }
}

__device__ __forceinline__ float4 window_sum(const View& V, const int* s_c0, const int* s_nc, int li, int lj, int lk) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int e = 0; e < 8; ++e) {
    const int ax = e >> 2, ay = (e >> 1) & 1, az = e & 1;
    const int nc = s_nc[e];
    if (!nc || (ax && li >= 2) || (ay && lj >= 2) || (az && lk >= 2)) continue;
    const int loc = ((li + kTile * ax) * kWin + (lj + kTile * ay)) * kWin + (lk + kTile * az);
    const float4* src = V.slots + (size_t)s_c0[e] * kWin3 + loc;
    int c = 0;
    for (; c + 4 <= nc; c += 4) {  // four window loads in flight
      const float4 v0 = src[(size_t)(c + 0) * kWin3], v1 = src[(size_t)(c + 1) * kWin3];
      const float4 v2 = src[(size_t)(c + 2) * kWin3], v3 = src[(size_t)(c + 3) * kWin3];
      acc.x += v0.x; acc.y += v0.y; acc.z += v0.z; acc.w += v0.w;
      acc.x += v1.x; acc.y += v1.y; acc.z += v1.z; acc.w += v1.w;
      acc.x += v2.x; acc.y += v2.y; acc.z += v2.z; acc.w += v2.w;
      acc.x += v3.x; acc.y += v3.y; acc.z += v3.z; acc.w += v3.w;
    }
    for (; c < nc; ++c) {
      const float4 v = src[(size_t)c * kWin3];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  return acc;
}

// window sums -> (m, v_in) planes, then grid_normalization_and_gravity
// (utils.py:177-183) + grid_postprocess[0] (BasicBC.apply,
// boundary_conditions.py:23-27).  v_out is 0 where m <= 1e-15 (the reset).
__global__ __launch_bounds__(kGridWG) void k_grid(View V, int s, float dt) {
  __shared__ int s_c0[8], s_nc[8];
  const int nb = (V.ng + kTile - 1) / kTile;
  const int bz = blockIdx.x % nb, by = (blockIdx.x / nb) % nb, bx = blockIdx.x / (nb * nb);
  load_cover(V, s, bx, by, bz, s_c0, s_nc);
  __syncthreads();
  const int li = threadIdx.x >> 6, lj = (threadIdx.x >> 3) & 7, lk = threadIdx.x & 7;
  const int ix = bx * kTile + li, iy = by * kTile + lj, iz = bz * kTile + lk;
  if (ix >= V.ng || iy >= V.ng || iz >= V.ng) return;
  const long g = ((long)ix * V.ng + iy) * V.ng + iz;
  const float4 a = window_sum(V, s_c0, s_nc, li, lj, lk);
  const float m = a.w;
  float* const gm = glv(V.gm, V, s);
  float* const vin = glv(V.vin, V, s);
  float* const vout = glv(V.vout, V, s);
  gm[g] = m;
  vin[g] = a.x;
  vin[V.nn + g] = a.y;
  vin[2 * V.nn + g] = a.z;
  float o[3] = {0.f, 0.f, 0.f};
  if (m > 1e-15f) {
    const float gr[3] = {V.gx_, V.gy_, V.gz_};
    const float vi[3] = {a.x, a.y, a.z};
    for (int d = 0; d < 3; ++d) o[d] = vi[d] / m + dt * gr[d];
  }
  if (V.has_box) {
    const float px = (float)ix * V.dx, py = (float)iy * V.dx, pz = (float)iz * V.dx;
    if (fabsf(px - V.bc0) < V.bs0 && fabsf(py - V.bc1) < V.bs1 && fabsf(pz - V.bc2) < V.bs2) o[0] = o[1] = o[2] = 0.f;
  }
  for (int d = 0; d < 3; ++d) vout[d * V.nn + g] = o[d];
}

__device__ __forceinline__ long node_of(const View& V, const int base[3], int i, int j, int k) {
  const int a = base[0] + i, b = base[1] + j, c = base[2] + k;
  if ((unsigned)a >= (unsigned)V.ng || (unsigned)b >= (unsigned)V.ng || (unsigned)c >= (unsigned)V.ng) return -1;
  return ((long)a * V.ng + b) * V.ng + c;
}
// The 3 planes of a grid vector at node g, 0 off the grid (g < 0).  The loads
// are unconditional (clamped index), so a stencil loop's 27 gathers are not
// each behind a branch (one round trip apiece); a node off the grid then adds
// zeros where the reference skips it.
__device__ __forceinline__ void grid3(const float* b, const View& V, long g, float out[3]) {
  const long gg = g < 0 ? 0 : g;
  const float a0 = b[gg], a1 = b[V.nn + gg], a2 = b[2 * V.nn + gg];
  out[0] = g < 0 ? 0.f : a0;
  out[1] = g < 0 ? 0.f : a1;
  out[2] = g < 0 ? 0.f : a2;
}

// g2p_opt (utils.py:284-347): level s -> s+1 (v, x, C, F; no cov update).
// count_next: also count level s+1's particles into its (zeroed) tile
// counters, k_count's work for the next binning.
__global__ __launch_bounds__(256) void k_g2p(View V, int s, float dt, int count_next) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= V.n) return;
  const float* const vout = glv(V.vout, V, s);
  float x[3], Fm[9];
  load_x(V, s, p, x);
  load9(V.F, V, s, p, Fm);
  int base[3];
  float fx[3], w[3][3], dw[3][3];
  bsp(x, V.inv_dx, base, fx, w, dw);
  float nv[3] = {0.f, 0.f, 0.f}, nC[9] = {0.f}, nF[9] = {0.f};
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const long g = node_of(V, base, i, j, k);
        const int o[3] = {i, j, k};
        float dpos[3];
        for (int d = 0; d < 3; ++d) dpos[d] = (float)o[d] - fx[d];
        const float weight = w[0][i] * w[1][j] * w[2][k];
        float gv[3];
        grid3(vout, V, g, gv);
        const float gw[3] = {V.inv_dx * dw[0][i] * w[1][j] * w[2][k], V.inv_dx * w[0][i] * dw[1][j] * w[2][k],
                             V.inv_dx * w[0][i] * w[1][j] * dw[2][k]};
        for (int r = 0; r < 3; ++r) {
          nv[r] += gv[r] * weight;
          for (int c = 0; c < 3; ++c) {
            nC[r * 3 + c] += gv[r] * dpos[c] * (weight * V.inv_dx * 4.0f);
            nF[r * 3 + c] += gv[r] * gw[c];
          }
        }
      }
  float x1[3];
  for (int d = 0; d < 3; ++d) {
    x1[d] = x[d] + dt * nv[d];
    pl(V.v, V, s + 1, 3, d)[p] = nv[d];
    pl(V.x, V, s + 1, 3, d)[p] = x1[d];
  }
  if (count_next) count_rank(V, V.count + (size_t)(s + 1) * V.ntiles, p, true, tile_of_x(x1, V));
  store9(V.C, V, s + 1, p, nC);
  float F1[9];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      float acc = 0.f;
      for (int q = 0; q < 3; ++q) acc += ((r == q ? 1.f : 0.f) + nF[r * 3 + q] * dt) * Fm[q * 3 + c];
      F1[r * 3 + c] = acc;
    }
  store9(V.F, V, s + 1, p, F1);
}

// ------------------------------------------------------------ backward ---
// d(weight)/d(fx) and d(grad weight)/d(fx) contracted with their adjoints.
__device__ __forceinline__ void weight_fx_adjoint(const float w[3][3], const float dw[3][3], int i, int j, int k,
                                                  float inv_dx, float g_weight, const float g_gw[3], float gfx[3]) {
  const int o[3] = {i, j, k};
  const float ddw[3] = {1.0f, -2.0f, 1.0f};
  for (int d = 0; d < 3; ++d) {
    float dweight = 1.f;
    for (int e = 0; e < 3; ++e) dweight *= (e == d) ? dw[e][o[e]] : w[e][o[e]];
    float acc = g_weight * dweight;
    for (int c = 0; c < 3; ++c) {
      float t = inv_dx;
      for (int e = 0; e < 3; ++e) {
        if (e == c && e == d) t *= ddw[o[e]];
        else if (e == c || e == d) t *= dw[e][o[e]];
        else t *= w[e][o[e]];
      }
      acc += g_gw[c] * t;
    }
    gfx[d] += acc;
  }
}

// g2p_opt.grad: adjoints of level s+1 -> x[s], F[s], and the v_out.grad
// contributions scattered through the chunk's fixed-point window to its slot.
__global__ __launch_bounds__(kChunk) void k_g2p_bwd(View V, int s, float dt) {
  __shared__ unsigned long long win[3 * kWin3];
  __shared__ float s_max[4];
  const float* const vout = glv(V.vout, V, s);
  const int c = blockIdx.x;
  if (c >= V.nchunks[s]) return;
  const int4 rec = V.chunks[(size_t)s * V.max_chunks + c];
  for (int l = threadIdx.x; l < 3 * kWin3; l += kChunk) win[l] = 0ull;
  const int tz = rec.x % V.nta, ty = (rec.x / V.nta) % V.nta, tx = rec.x / (V.nta * V.nta);
  const int ox = tx * kTile, oy = ty * kTile, oz = tz * kTile;
  const bool on = (int)threadIdx.x < rec.z;
  int p = 0, base[3] = {0, 0, 0};
  float fx[3] = {1.f, 1.f, 1.f}, w[3][3], dw[3][3], gC1[9] = {0.f}, g_nv[3] = {0.f, 0.f, 0.f}, g_nF[9] = {0.f};
  float bound = 0.f;
  if (on) {
    p = V.perm[(size_t)s * V.np + rec.y + threadIdx.x];
    float x[3], Fm[9];
    load_x(V, s, p, x);
    load9(V.F, V, s, p, Fm);
    bsp(x, V.inv_dx, base, fx, w, dw);
    float nF[9] = {0.f};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const long g = node_of(V, base, i, j, k);
          float gv[3];
          grid3(vout, V, g, gv);
          const float gw[3] = {V.inv_dx * dw[0][i] * w[1][j] * w[2][k], V.inv_dx * w[0][i] * dw[1][j] * w[2][k],
                               V.inv_dx * w[0][i] * w[1][j] * dw[2][k]};
          for (int r = 0; r < 3; ++r)
            for (int cc = 0; cc < 3; ++cc) nF[r * 3 + cc] += gv[r] * gw[cc];
        }
    float gx1[3], gv1[3], gF1[9];
    for (int d = 0; d < 3; ++d) {
      gx1[d] = pl(V.gx, V, s + 1, 3, d)[p];
      gv1[d] = pl(V.gv, V, s + 1, 3, d)[p];
    }
    load9(V.gC, V, s + 1, p, gC1);
    load9(V.gF, V, s + 1, p, gF1);
    // x1 = x0 + dt nv ; v1 = nv
    for (int d = 0; d < 3; ++d) {
      pl(V.gx, V, s, 3, d)[p] += gx1[d];
      g_nv[d] = gv1[d] + dt * gx1[d];
    }
    // F1 = (I + dt nF) F0
    float gF0[9];
    load9(V.gF, V, s, p, gF0);
    for (int r = 0; r < 3; ++r)
      for (int q = 0; q < 3; ++q) {
        float acc = 0.f;
        for (int cc = 0; cc < 3; ++cc) acc += gF1[r * 3 + cc] * Fm[q * 3 + cc];
        g_nF[r * 3 + q] = dt * acc;
      }
    for (int q = 0; q < 3; ++q)
      for (int cc = 0; cc < 3; ++cc) {
        float acc = 0.f;
        for (int r = 0; r < 3; ++r) acc += ((r == q ? 1.f : 0.f) + nF[r * 3 + q] * dt) * gF1[r * 3 + cc];
        gF0[q * 3 + cc] += acc;
      }
    store9(V.gF, V, s, p, gF0);
    // |g_g| <= |g_nv| + 3 |gC1| 1.5 (4 inv_dx) + 3 |g_nF| inv_dx
    float a = 0.f, b = 0.f, e = 0.f;
    for (int r = 0; r < 3; ++r) a = fmaxf(a, fabsf(g_nv[r]));
    for (int i = 0; i < 9; ++i) {
      b = fmaxf(b, fabsf(gC1[i]));
      e = fmaxf(e, fabsf(g_nF[i]));
    }
    bound = (a + 18.0f * V.inv_dx * b + 3.0f * V.inv_dx * e) * 1.01f;
  }
  int S[3];
  S[0] = S[1] = S[2] = chunk_exponent(bound, s_max, 0);  // its barrier also orders the zeroing
  if (on) {
    const double sc = ldexp(1.0, S[0]);
    const int lb0 = base[0] - ox, lb1 = base[1] - oy, lb2 = base[2] - oz;
    float gfx[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const long g = node_of(V, base, i, j, k);
          const int o[3] = {i, j, k};
          float dpos[3];
          for (int d = 0; d < 3; ++d) dpos[d] = (float)o[d] - fx[d];
          const float weight = w[0][i] * w[1][j] * w[2][k];
          const float gw[3] = {V.inv_dx * dw[0][i] * w[1][j] * w[2][k], V.inv_dx * w[0][i] * dw[1][j] * w[2][k],
                               V.inv_dx * w[0][i] * w[1][j] * dw[2][k]};
          float gv[3];
          grid3(vout, V, g, gv);
          const float cw = weight * V.inv_dx * 4.0f;
          float g_weight = 0.f, g_dpos[3] = {0.f, 0.f, 0.f}, g_gw[3] = {0.f, 0.f, 0.f};
          const int a = lb0 + i, b = lb1 + j, c3 = lb2 + k;
          const bool in_win = g >= 0 && (unsigned)a < (unsigned)kWin && (unsigned)b < (unsigned)kWin &&
                              (unsigned)c3 < (unsigned)kWin;
          const int l = (a * kWin + b) * kWin + c3;
          for (int r = 0; r < 3; ++r) {
            float g_g = g_nv[r] * weight;
            g_weight += g_nv[r] * gv[r];
            for (int cc = 0; cc < 3; ++cc) {
              g_g += gC1[r * 3 + cc] * dpos[cc] * cw + g_nF[r * 3 + cc] * gw[cc];
              g_weight += gC1[r * 3 + cc] * gv[r] * dpos[cc] * V.inv_dx * 4.0f;
              g_dpos[cc] += gC1[r * 3 + cc] * gv[r] * cw;
              g_gw[cc] += g_nF[r * 3 + cc] * gv[r];
            }
            if (in_win) lds_add(&win[r * kWin3 + l], to_fixed(g_g, sc));
          }
          weight_fx_adjoint(w, dw, i, j, k, V.inv_dx, g_weight, g_gw, gfx);
          for (int d = 0; d < 3; ++d) gfx[d] -= g_dpos[d];
        }
    for (int d = 0; d < 3; ++d) pl(V.gx, V, s, 3, d)[p] += gfx[d] * V.inv_dx;
  }
  __syncthreads();
  store_window(V, win, 3, S, c);
}

// grid_normalization_and_gravity.grad: v_out.grad += this substep's window
// sums (the grid adjoints persist across substeps), then
// v_in.grad += v_out.grad / m (no m adjoint); the BC's .grad is a no-op.
__global__ __launch_bounds__(kGridWG) void k_grid_bwd(View V, int s) {
  __shared__ int s_c0[8], s_nc[8];
  const int nb = (V.ng + kTile - 1) / kTile;
  const int bz = blockIdx.x % nb, by = (blockIdx.x / nb) % nb, bx = blockIdx.x / (nb * nb);
  load_cover(V, s, bx, by, bz, s_c0, s_nc);
  __syncthreads();
  if (!(s_nc[0] | s_nc[1] | s_nc[2] | s_nc[3] | s_nc[4] | s_nc[5] | s_nc[6] | s_nc[7])) return;  // m = 0 here
  const int li = threadIdx.x >> 6, lj = (threadIdx.x >> 3) & 7, lk = threadIdx.x & 7;
  const int ix = bx * kTile + li, iy = by * kTile + lj, iz = bz * kTile + lk;
  if (ix >= V.ng || iy >= V.ng || iz >= V.ng) return;
  const long g = ((long)ix * V.ng + iy) * V.ng + iz;
  const float4 a = window_sum(V, s_c0, s_nc, li, lj, lk);
  const float add[3] = {a.x, a.y, a.z};
  const float m = glv(V.gm, V, s)[g];
  for (int d = 0; d < 3; ++d) {
    const float go = V.gvout[d * V.nn + g] + add[d];
    V.gvout[d * V.nn + g] = go;
    if (m > 1e-15f) V.gvin[d * V.nn + g] += go / m;
  }
}

// p2g_opt.grad + compute_stress_from_F_opt.grad + compute_mu_lam_from_E_nu.grad
// for one particle per thread (all three are per-particle after the grid gather).
__global__ __launch_bounds__(256) void k_p2g_bwd(View V, int s, float dt) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= V.n) return;
  float x[3], vv[3], Cm[9], sg[9];
  load_x(V, s, p, x);
  for (int d = 0; d < 3; ++d) vv[d] = pl(V.v, V, s, 3, d)[p];
  load9(V.C, V, s, p, Cm);
  load9(V.S, V, s, p, sg);
  float gvp[3], gCp[9], gSp[9];
  for (int d = 0; d < 3; ++d) gvp[d] = pl(V.gv, V, s, 3, d)[p];
  load9(V.gC, V, s, p, gCp);
  load9(V.gS, V, s, p, gSp);
  int base[3];
  float fx[3], w[3][3], dw[3][3];
  bsp(x, V.inv_dx, base, fx, w, dw);
  const float m = V.mass[p], vol = V.vol[p];
  float gfx[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const long g = node_of(V, base, i, j, k);
        const int o[3] = {i, j, k};
        float dpos[3];
        for (int d = 0; d < 3; ++d) dpos[d] = ((float)o[d] - fx[d]) * V.dx;
        const float weight = w[0][i] * w[1][j] * w[2][k];
        const float gw[3] = {V.inv_dx * dw[0][i] * w[1][j] * w[2][k], V.inv_dx * w[0][i] * dw[1][j] * w[2][k],
                             V.inv_dx * w[0][i] * w[1][j] * dw[2][k]};
        float G[3];
        grid3(V.gvin, V, g, G);
        float g_weight = 0.f, g_dpos[3] = {0.f, 0.f, 0.f}, g_gw[3] = {0.f, 0.f, 0.f};
        for (int r = 0; r < 3; ++r) {
          const float cd = Cm[r * 3 + 0] * dpos[0] + Cm[r * 3 + 1] * dpos[1] + Cm[r * 3 + 2] * dpos[2];
          gvp[r] += weight * m * G[r];
          g_weight += m * G[r] * (vv[r] + cd);
          for (int c = 0; c < 3; ++c) {
            gCp[r * 3 + c] += weight * m * G[r] * dpos[c];
            g_dpos[c] += weight * m * G[r] * Cm[r * 3 + c];
            gSp[r * 3 + c] += -dt * vol * G[r] * gw[c];
            g_gw[c] += -dt * vol * G[r] * sg[r * 3 + c];
          }
        }
        weight_fx_adjoint(w, dw, i, j, k, V.inv_dx, g_weight, g_gw, gfx);
        for (int d = 0; d < 3; ++d) gfx[d] -= V.dx * g_dpos[d];
      }
  for (int d = 0; d < 3; ++d) {
    pl(V.gv, V, s, 3, d)[p] = gvp[d];
    pl(V.gx, V, s, 3, d)[p] += gfx[d] * V.inv_dx;
  }
  store9(V.gC, V, s, p, gCp);
  store9(V.gS, V, s, p, gSp);

  // ---- compute_stress_from_F_opt.grad (utils.py:56-76)
  float F[9], gF[9];
  load9(V.F, V, s, p, F);
  load9(V.gF, V, s, p, gF);
  float J = det3(F);
  const bool clamped = fabsf(J) < 1e-2f;
  if (clamped) J = 1e-2f * (J > 0.f ? 1.f : (J < 0.f ? -1.f : 0.f));
  float E[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      const float ftf = F[0 * 3 + i] * F[0 * 3 + j] + F[1 * 3 + i] * F[1 * 3 + j] + F[2 * 3 + i] * F[2 * 3 + j];
      E[i * 3 + j] = 0.5f * (ftf - (i == j ? 1.f : 0.f));
    }
  const float mu = V.mu[p], lam = V.lam[p];
  const float tr = E[0] + E[4] + E[8];
  float Sm[9];
  for (int i = 0; i < 9; ++i) Sm[i] = 2.0f * mu * E[i] + ((i % 4) == 0 ? lam * tr : 0.f);
  float A[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      float acc = 0.f;
      for (int k = 0; k < 3; ++k)
        for (int l = 0; l < 3; ++l) acc += F[i * 3 + k] * Sm[k * 3 + l] * F[j * 3 + l];
      A[i * 3 + j] = acc;
    }
  float GA[9], gJ = 0.f;
  for (int i = 0; i < 9; ++i) {
    GA[i] = gSp[i] / J;
    gJ -= gSp[i] * A[i] / (J * J);
  }
  float GS[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      float a1 = 0.f, a2 = 0.f;
      for (int k = 0; k < 3; ++k)
        for (int l = 0; l < 3; ++l) {
          a1 += GA[i * 3 + k] * F[k * 3 + l] * Sm[j * 3 + l];
          a2 += GA[k * 3 + i] * F[k * 3 + l] * Sm[l * 3 + j];
        }
      gF[i * 3 + j] += a1 + a2;
      float s3 = 0.f;
      for (int k = 0; k < 3; ++k)
        for (int l = 0; l < 3; ++l) s3 += F[k * 3 + i] * GA[k * 3 + l] * F[l * 3 + j];
      GS[i * 3 + j] = s3;
    }
  const float trGS = GS[0] + GS[4] + GS[8];
  float gE[9], gmu = 0.f;
  for (int i = 0; i < 9; ++i) {
    gE[i] = 2.0f * mu * GS[i] + ((i % 4) == 0 ? lam * trGS : 0.f);
    gmu += 2.0f * GS[i] * E[i];
  }
  const float gmu_t = V.gmu[p] + gmu, glam_t = V.glam[p] + tr * trGS;
  V.gmu[p] = gmu_t;
  V.glam[p] = glam_t;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      float acc = 0.f;
      for (int k = 0; k < 3; ++k) acc += F[i * 3 + k] * 0.5f * (gE[k * 3 + j] + gE[j * 3 + k]);
      gF[i * 3 + j] += acc;
    }
  if (!clamped) {
    const float cof[9] = {F[4] * F[8] - F[5] * F[7], F[5] * F[6] - F[3] * F[8], F[3] * F[7] - F[4] * F[6],
                          F[2] * F[7] - F[1] * F[8], F[0] * F[8] - F[2] * F[6], F[1] * F[6] - F[0] * F[7],
                          F[1] * F[5] - F[2] * F[4], F[2] * F[3] - F[0] * F[5], F[0] * F[4] - F[1] * F[3]};
    for (int i = 0; i < 9; ++i) gF[i] += gJ * cof[i];
  }
  store9(V.gF, V, s, p, gF);

  // ---- compute_mu_lam_from_E_nu.grad on the accumulated mu/lam adjoints
  const float Ey = powf(10.0f, V.logE[p]);
  const float ey = expf(-V.y[p]);
  const float nu = 0.49f / (1.0f + ey);
  const float dnu_dy = 0.49f * ey / ((1.0f + ey) * (1.0f + ey));
  const float D = (1.0f + nu) * (1.0f - 2.0f * nu);
  const float gEy = gmu_t * (1.0f / (2.0f * (1.0f + nu))) + glam_t * (nu / D);
  const float gnu = gmu_t * (-Ey / (2.0f * (1.0f + nu) * (1.0f + nu))) + glam_t * (Ey * (1.0f + 2.0f * nu * nu) / (D * D));
  V.glogE[p] += gEy * Ey * 2.302585092994046f;
  V.gy[p] += gnu * dnu_dy;
}

// ------------------------------------------------------ per-particle misc ---
__global__ __launch_bounds__(256) void k_mu_lam(View V) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= V.n) return;
  const float E = powf(10.0f, V.logE[p]);
  const float nu = 0.49f / (1.0f + expf(-V.y[p]));
  V.mu[p] = E / (2.0f * (1.0f + nu));
  V.lam[p] = E * nu / ((1.0f + nu) * (1.0f - 2.0f * nu));
}

// compute_cov_from_F_opt (utils.py:435-467): cov = upper 6 of F[L-1] A F[L-1]^T
__global__ __launch_bounds__(256) void k_cov(View V) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= V.n) return;
  float F[9], a[6];
  load9(V.F, V, V.L - 1, p, F);
  for (int c = 0; c < 6; ++c) a[c] = V.icov[(size_t)c * V.np + p];
  const float A[9] = {a[0], a[1], a[2], a[1], a[3], a[4], a[2], a[4], a[5]};
  float FA[9], M[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) FA[i * 3 + j] = F[i * 3 + 0] * A[0 * 3 + j] + F[i * 3 + 1] * A[1 * 3 + j] + F[i * 3 + 2] * A[2 * 3 + j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) M[i * 3 + j] = FA[i * 3 + 0] * F[j * 3 + 0] + FA[i * 3 + 1] * F[j * 3 + 1] + FA[i * 3 + 2] * F[j * 3 + 2];
  const float o[6] = {M[0], M[1], M[2], M[4], M[5], M[8]};
  for (int c = 0; c < 6; ++c) V.cov[(size_t)c * V.np + p] = o[c];
}

__global__ __launch_bounds__(256) void k_cov_bwd(View V) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= V.n) return;
  float F[9], gF[9], a[6], gc[6];
  load9(V.F, V, V.L - 1, p, F);
  load9(V.gF, V, V.L - 1, p, gF);
  for (int c = 0; c < 6; ++c) {
    a[c] = V.icov[(size_t)c * V.np + p];
    gc[c] = V.gcov[(size_t)c * V.np + p];
  }
  const float A[9] = {a[0], a[1], a[2], a[1], a[3], a[4], a[2], a[4], a[5]};
  const float G[9] = {gc[0], gc[1], gc[2], 0.f, gc[3], gc[4], 0.f, 0.f, gc[5]};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      float acc = 0.f;
      for (int k = 0; k < 3; ++k)
        for (int l = 0; l < 3; ++l) acc += G[i * 3 + k] * F[k * 3 + l] * A[j * 3 + l] + G[k * 3 + i] * F[k * 3 + l] * A[l * 3 + j];
      gF[i * 3 + j] += acc;
    }
  store9(V.gF, V, V.L - 1, p, gF);
}

// learn (solver.py:92-108): clipped SGD, lr 0.8 on logE and 1.6 on y.
__global__ __launch_bounds__(256) void k_learn(View V) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= V.n) return;
  float a = V.glogE[p], b = V.gy[p];
  if (fabsf(a) > 1.0f) a = a > 0.f ? 1.0f : -1.0f;
  if (fabsf(b) > 1.0f) b = b > 0.f ? 1.0f : -1.0f;
  V.logE[p] -= 0.8f * a;
  V.y[p] -= 1.6f * b;
}

// external [n, w] <-> internal planes [w][np] through order[] (internal -> external)
__global__ void k_gather_out(const float* plane, int w, int n, int np, const int* order, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int e = order[i];
  for (int c = 0; c < w; ++c) out[(size_t)e * w + c] = plane[(size_t)c * np + i];
}
__global__ void k_scatter_in(float* plane, int w, int n, int np, const int* order, const float* in) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int e = order[i];
  for (int c = 0; c < w; ++c) plane[(size_t)c * np + i] = in ? in[(size_t)e * w + c] : 0.f;
}
__global__ void k_iota(int* a, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = i;
}
__global__ void k_init_level0(View V, float density, float logE, float y) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= V.n) return;
  for (int c = 0; c < 9; ++c) {
    pl(V.F, V, 0, 9, c)[p] = (c % 4) == 0 ? 1.f : 0.f;
    pl(V.C, V, 0, 9, c)[p] = 0.f;
    pl(V.S, V, 0, 9, c)[p] = 0.f;
  }
  V.mass[p] = density * V.vol[p];  // compute_mass_from_vol_density (utils.py:365-368)
  V.logE[p] = logE;
  V.y[p] = y;
}
__global__ void k_interleave(const float* planes, long nn, int w, float* out) {
  const long g = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nn) return;
  for (int c = 0; c < w; ++c) out[g * w + c] = planes[c * nn + g];
}

}  // namespace fit
}  // namespace gsmpm

using namespace gsmpm;
using namespace gsmpm::fit;

struct gsmpm_fit {
  gsmpm_fit_params p{};
  int n = 0, np = 0, ng = 0, L = 0, nta = 0, ntiles = 0, max_chunks = 0;
  long nn = 0;
  bool ready = false;
  int has_box = 0;
  float box_c[3] = {0, 0, 0}, box_s[3] = {0, 0, 0};
  std::vector<char> binned;  // per level: bins of x[level] are current
  // One grid per level (memory allowing): the backward pass then reads the
  // grid its forward pass computed instead of recomputing it (the reference's
  // P2G + grid update redo in p2g2p_backward gives the same values from the
  // same inputs).  gvalid[s]: level s's grid is that of the current x/v/C/S[s]
  // (forward(s) with dt gdt[s]); any state change through the API drops it.
  int glevels = 1;
  std::vector<char> gvalid;
  std::vector<float> gdt;
  int glast = 0;             // the level whose grid was computed last (get_grid)
  // Binning state: tl/rk (one set) and count[counted] are complete for level
  // `counted` (-1: none); czero[l]: count[l] is all zero.
  int counted = -1;
  std::vector<char> czero;
  void* mem = nullptr;       // one allocation for everything
  View V{};
  int* order = nullptr;
};

namespace {

hipStream_t S(void* s) { return (hipStream_t)s; }
int blocks(long n, int b = 256) { return (int)((n + b - 1) / b); }
int grid_blocks(const gsmpm_fit* h) {
  const int nb = (h->ng + kTile - 1) / kTile;
  return nb * nb * nb;
}

int require_ready(gsmpm_fit* h, const char* fn) {
  if (!h) {
    set_error(std::string(fn) + ": null handle");
    return GSMPM_EINVAL;
  }
  if (!h->ready) {
    set_error(std::string(fn) + ": particles not set");
    return GSMPM_ESTATE;
  }
  return GSMPM_OK;
}

void drop_grids(gsmpm_fit* h) { std::fill(h->gvalid.begin(), h->gvalid.end(), 0); }

// Bins of level s.  Its counts come from the G2P that produced the level when
// it counted (forward), else k_count; the scan and the placement are one launch
// on grids of <= kScanTiles tiles, which also zeroes level s+1's counters.
int bin_level(gsmpm_fit* h, int s, hipStream_t st) {
  if (h->counted != s) {
    if (!h->czero[s]) GSMPM_HIP(hipMemsetAsync(h->V.count + (size_t)s * h->ntiles, 0, sizeof(int) * h->ntiles, st));
    hipLaunchKernelGGL(k_count, dim3(blocks(h->n)), dim3(256), 0, st, h->V, s);
    h->counted = s;
    h->czero[s] = 0;
  }
  if (h->ntiles <= kScanTiles) {
    const int zn = s + 1 < h->L ? 1 : 0;
    hipLaunchKernelGGL(k_scanplace, dim3(blocks(h->n)), dim3(256), 0, st, h->V, s, zn);
    if (zn) {
      h->czero[s + 1] = 1;
      h->binned[s + 1] = 0;
    }
  } else {
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, h->V, s);
    hipLaunchKernelGGL(k_place, dim3(blocks(h->n)), dim3(256), 0, st, h->V, s);
  }
  GSMPM_LAUNCH_CHECK();
  h->binned[s] = 1;
  return GSMPM_OK;
}

// p2g (+ stress) into chunk windows + window sums and grid update of level s
// (the reset_grid_state of the reference is implicit: k_grid writes every node)
int grid_of_level(gsmpm_fit* h, int s, float dt, bool recompute, hipStream_t st) {
  h->glast = h->glevels > 1 ? s : 0;
  if (recompute && h->glevels > 1 && h->gvalid[s] && h->gdt[s] == dt && h->binned[s]) return GSMPM_OK;
  if (!h->binned[s]) {
    int rc = bin_level(h, s, st);
    if (rc) return rc;
  }
  if (recompute)
    hipLaunchKernelGGL(k_p2g<true>, dim3(h->max_chunks), dim3(kChunk), 0, st, h->V, s, dt);
  else
    hipLaunchKernelGGL(k_p2g<false>, dim3(h->max_chunks), dim3(kChunk), 0, st, h->V, s, dt);
  hipLaunchKernelGGL(k_grid, dim3(grid_blocks(h)), dim3(kGridWG), 0, st, h->V, s, dt);
  GSMPM_LAUNCH_CHECK();
  h->gvalid[s] = 1;
  h->gdt[s] = dt;
  return GSMPM_OK;
}

struct FieldDesc {
  float* base;
  int width;
  bool leveled;
};

FieldDesc field_desc(gsmpm_fit* h, int f) {
  View& V = h->V;
  switch (f) {
    case GSMPM_FIT_X: return {V.x, 3, true};
    case GSMPM_FIT_V: return {V.v, 3, true};
    case GSMPM_FIT_F: return {V.F, 9, true};
    case GSMPM_FIT_C: return {V.C, 9, true};
    case GSMPM_FIT_STRESS: return {V.S, 9, true};
    case GSMPM_FIT_GX: return {V.gx, 3, true};
    case GSMPM_FIT_GV: return {V.gv, 3, true};
    case GSMPM_FIT_GF: return {V.gF, 9, true};
    case GSMPM_FIT_GC: return {V.gC, 9, true};
    case GSMPM_FIT_GSTRESS: return {V.gS, 9, true};
    case GSMPM_FIT_LOGE: return {V.logE, 1, false};
    case GSMPM_FIT_Y: return {V.y, 1, false};
    case GSMPM_FIT_MU: return {V.mu, 1, false};
    case GSMPM_FIT_LAM: return {V.lam, 1, false};
    case GSMPM_FIT_GLOGE: return {V.glogE, 1, false};
    case GSMPM_FIT_GY: return {V.gy, 1, false};
    case GSMPM_FIT_GMU: return {V.gmu, 1, false};
    case GSMPM_FIT_GLAM: return {V.glam, 1, false};
    case GSMPM_FIT_COV: return {V.cov, 6, false};
    case GSMPM_FIT_GCOV: return {V.gcov, 6, false};
    case GSMPM_FIT_INIT_COV: return {V.icov, 6, false};
    case GSMPM_FIT_VOL: return {V.vol, 1, false};
    case GSMPM_FIT_MASS: return {V.mass, 1, false};
    default: return {nullptr, 0, false};
  }
}

}  // namespace

extern "C" {

int gsmpm_fit_create(const gsmpm_fit_params* p, gsmpm_fit** out) {
  GSMPM_REQUIRE(p && out, "gsmpm_fit_create: null argument");
  GSMPM_REQUIRE(p->n_particles > 0, "gsmpm_fit_create: n_particles must be > 0");
  GSMPM_REQUIRE(p->n_grid >= 4 && p->n_grid <= 1024, "gsmpm_fit_create: n_grid must be in [4, 1024]");
  GSMPM_REQUIRE(p->levels >= 2, "gsmpm_fit_create: levels must be >= 2");
  GSMPM_REQUIRE(p->grid_extent > 0, "gsmpm_fit_create: grid_extent must be > 0");
  GSMPM_REQUIRE(p->nu > 0 && p->nu < 0.49 && p->E > 0, "gsmpm_fit_create: need E > 0 and 0 < nu < 0.49");
  auto* h = new gsmpm_fit;
  h->p = *p;
  h->n = p->n_particles;
  h->np = div_up(h->n, 256) * 256;
  h->ng = p->n_grid;
  h->L = p->levels;
  h->nn = (long)h->ng * h->ng * h->ng;
  h->nta = (h->ng - 3) / kTile + 1;
  h->ntiles = h->nta * h->nta * h->nta;
  h->max_chunks = div_up(h->n, kChunk) + h->ntiles;
  h->binned.assign(h->L, 0);
  h->czero.assign(h->L, 0);
  const size_t np = h->np, L = h->L, nn = h->nn;
  // per-level grids up to 4 GiB (GSMPM_FIT_GRID_LEVELS=0: one grid, recomputed in the backward pass)
  const char* glenv = std::getenv("GSMPM_FIT_GRID_LEVELS");
  h->glevels = (glenv && glenv[0] == '0') || 7 * nn * 4 * L > (size_t(4) << 30) ? 1 : h->L;
  h->gvalid.assign(h->L, 0);
  h->gdt.assign(h->L, 0.f);
  const size_t nf = L * np * (3 + 3 + 9 + 9 + 9) * 2 + np * 10 + np * 6 * 3 + nn * (7 * (size_t)h->glevels + 6);
  const size_t ni = (size_t)h->ntiles * (2 * L + 1) + np * 3 + L * np + L + 64;
  const size_t nslot = (size_t)(h->max_chunks + 1) * kWin3;
  const size_t bytes = nf * 4 + ni * 4 + L * h->max_chunks * sizeof(int4) + nslot * sizeof(float4) + 64 * 256;  // + per-take alignment
  void* mem = nullptr;
  hipError_t e = hipMalloc(&mem, bytes);
  if (e != hipSuccess) {
    delete h;
    set_error(std::string("gsmpm_fit_create: hipMalloc: ") + hipGetErrorString(e));
    return GSMPM_EHIP;
  }
  h->mem = mem;
  char* cur = (char*)mem;
  auto take = [&](size_t b) {
    char* r = cur;
    cur += (b + 255) & ~size_t(255);
    return r;
  };
  View& V = h->V;
  V.chunks = (int4*)take(L * h->max_chunks * sizeof(int4));
  V.slots = (float4*)take(nslot * sizeof(float4));
  auto F = [&](size_t count) { return (float*)take(count * 4); };
  auto I = [&](size_t count) { return (int*)take(count * 4); };
  V.x = F(L * 3 * np); V.v = F(L * 3 * np); V.F = F(L * 9 * np); V.C = F(L * 9 * np); V.S = F(L * 9 * np);
  V.gx = F(L * 3 * np); V.gv = F(L * 3 * np); V.gF = F(L * 9 * np); V.gC = F(L * 9 * np); V.gS = F(L * 9 * np);
  V.vol = F(np); V.mass = F(np); V.logE = F(np); V.y = F(np); V.mu = F(np); V.lam = F(np);
  V.glogE = F(np); V.gy = F(np); V.gmu = F(np); V.glam = F(np);
  V.icov = F(6 * np); V.cov = F(6 * np); V.gcov = F(6 * np);
  V.gm = F(7 * nn * h->glevels);  // per level: m | v_in | v_out
  V.vin = V.gm + nn;
  V.vout = V.gm + 4 * nn;
  V.gstride = h->glevels > 1 ? 7 * (long)nn : 0;
  V.gvin = F(3 * nn); V.gvout = F(3 * nn);
  V.count = I(L * h->ntiles); V.cbase = I(L * h->ntiles); V.cstart = I(h->ntiles); V.tl = I(np); V.rk = I(np); V.perm = I(L * np);
  V.nchunks = I(L);
  h->order = I(np);
  if ((size_t)(cur - (char*)mem) > bytes) {
    (void)hipFree(mem);
    delete h;
    set_error("gsmpm_fit_create: internal layout overflow");
    return GSMPM_EINVAL;
  }
  V.n = h->n; V.np = h->np; V.ng = h->ng; V.L = h->L; V.nta = h->nta; V.ntiles = h->ntiles;
  V.max_chunks = h->max_chunks; V.nn = h->nn;
  V.dx = (float)(p->grid_extent / p->n_grid);
  V.inv_dx = (float)(p->n_grid / p->grid_extent);
  V.gx_ = (float)p->gravity[0]; V.gy_ = (float)p->gravity[1]; V.gz_ = (float)p->gravity[2];
  V.has_box = 0;
  *out = h;
  return GSMPM_OK;
}

int gsmpm_fit_destroy(gsmpm_fit* h) {
  if (!h) return GSMPM_OK;
  if (h->mem) (void)hipFree(h->mem);
  delete h;
  return GSMPM_OK;
}

int gsmpm_fit_set_particles(gsmpm_fit* h, const float* xyz, const float* cov6, const float* vol, const float* init_v,
                            void* stream) {
  GSMPM_REQUIRE(h && xyz && cov6 && vol, "gsmpm_fit_set_particles: null argument");
  hipStream_t st = S(stream);
  View& V = h->V;
  const int n = h->n, np = h->np;
  // zero every plane once (padding lanes stay 0), then level-0 bins in input
  // order define the internal (tile-sorted) order
  GSMPM_HIP(hipMemsetAsync(V.x, 0, (char*)(V.icov + 6 * (size_t)np * 3) - (char*)V.x, st));
  GSMPM_HIP(hipMemsetAsync(V.gm, 0, sizeof(float) * 7 * h->nn * h->glevels, st));
  for (float* g : {V.gvin, V.gvout}) GSMPM_HIP(hipMemsetAsync(g, 0, sizeof(float) * 3 * h->nn, st));
  drop_grids(h);
  hipLaunchKernelGGL(k_iota, dim3(blocks(n)), dim3(256), 0, st, h->order, n);
  hipLaunchKernelGGL(k_scatter_in, dim3(blocks(n)), dim3(256), 0, st, V.x, 3, n, np, (const int*)h->order, xyz);
  GSMPM_LAUNCH_CHECK();
  std::fill(h->binned.begin(), h->binned.end(), 0);
  std::fill(h->czero.begin(), h->czero.end(), 0);
  h->counted = -1;
  int rc = bin_level(h, 0, st);
  if (rc) return rc;
  GSMPM_HIP(hipMemcpyAsync(h->order, V.perm, sizeof(int) * n, hipMemcpyDeviceToDevice, st));
  h->counted = -1;  // the particles are re-stored in tile order below
  const int* ord = h->order;
  hipLaunchKernelGGL(k_scatter_in, dim3(blocks(n)), dim3(256), 0, st, V.x, 3, n, np, ord, xyz);
  hipLaunchKernelGGL(k_scatter_in, dim3(blocks(n)), dim3(256), 0, st, V.v, 3, n, np, ord, init_v);
  hipLaunchKernelGGL(k_scatter_in, dim3(blocks(n)), dim3(256), 0, st, V.icov, 6, n, np, ord, cov6);
  hipLaunchKernelGGL(k_scatter_in, dim3(blocks(n)), dim3(256), 0, st, V.cov, 6, n, np, ord, cov6);
  hipLaunchKernelGGL(k_scatter_in, dim3(blocks(n)), dim3(256), 0, st, V.vol, 1, n, np, ord, vol);
  // MPM_model.init_elasiticity_params (model.py:40-44): logE, y from the host in f64, stored f32
  const float logE = (float)std::log10(h->p.E), y = (float)(-std::log(0.49 / h->p.nu - 1.0));
  hipLaunchKernelGGL(k_init_level0, dim3(blocks(n)), dim3(256), 0, st, V, (float)h->p.density, logE, y);
  hipLaunchKernelGGL(k_mu_lam, dim3(blocks(n)), dim3(256), 0, st, V);
  GSMPM_LAUNCH_CHECK();
  std::fill(h->binned.begin(), h->binned.end(), 0);
  h->ready = true;
  return GSMPM_OK;
}

int gsmpm_fit_set_fixed_cube(gsmpm_fit* h, const double center[3], const double size[3]) {
  GSMPM_REQUIRE(h && center && size, "gsmpm_fit_set_fixed_cube: null argument");
  View& V = h->V;
  V.has_box = 1;
  V.bc0 = (float)center[0]; V.bc1 = (float)center[1]; V.bc2 = (float)center[2];
  V.bs0 = (float)size[0]; V.bs1 = (float)size[1]; V.bs2 = (float)size[2];
  drop_grids(h);
  return GSMPM_OK;
}

int gsmpm_fit_forward(gsmpm_fit* h, float dt, int32_t s, void* stream) {
  if (int rc = require_ready(h, "gsmpm_fit_forward")) return rc;
  GSMPM_REQUIRE(s >= 0 && s < h->L - 1, "gsmpm_fit_forward: level out of range");
  hipStream_t st = S(stream);
  if (int rc = grid_of_level(h, s, dt, false, st)) return rc;
  const int cn = h->czero[s + 1];  // count level s+1 on the way (its counters are zero)
  hipLaunchKernelGGL(k_g2p, dim3(blocks(h->n)), dim3(256), 0, st, h->V, (int)s, dt, cn);
  GSMPM_LAUNCH_CHECK();
  h->binned[s + 1] = 0;
  h->czero[s + 1] = 0;
  h->counted = cn ? s + 1 : (h->counted == s + 1 ? -1 : h->counted);
  std::fill(h->gvalid.begin() + s + 1, h->gvalid.end(), 0);  // x/v/C/F of the later levels change
  return GSMPM_OK;
}

int gsmpm_fit_backward(gsmpm_fit* h, float dt, int32_t s, void* stream) {
  if (int rc = require_ready(h, "gsmpm_fit_backward")) return rc;
  GSMPM_REQUIRE(s >= 0 && s < h->L - 1, "gsmpm_fit_backward: level out of range");
  hipStream_t st = S(stream);
  if (int rc = grid_of_level(h, s, dt, true, st)) return rc;
  hipLaunchKernelGGL(k_g2p_bwd, dim3(h->max_chunks), dim3(kChunk), 0, st, h->V, (int)s, dt);
  hipLaunchKernelGGL(k_grid_bwd, dim3(grid_blocks(h)), dim3(kGridWG), 0, st, h->V, (int)s);
  hipLaunchKernelGGL(k_p2g_bwd, dim3(blocks(h->n)), dim3(256), 0, st, h->V, (int)s, dt);
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}

int gsmpm_fit_postprocess_forward(gsmpm_fit* h, void* stream) {
  if (int rc = require_ready(h, "gsmpm_fit_postprocess_forward")) return rc;
  hipLaunchKernelGGL(k_cov, dim3(blocks(h->n)), dim3(256), 0, S(stream), h->V);
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}

int gsmpm_fit_postprocess_backward(gsmpm_fit* h, void* stream) {
  if (int rc = require_ready(h, "gsmpm_fit_postprocess_backward")) return rc;
  hipLaunchKernelGGL(k_cov_bwd, dim3(blocks(h->n)), dim3(256), 0, S(stream), h->V);
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}

int gsmpm_fit_set_grads(gsmpm_fit* h, const float* xyz_grad, const float* cov_grad, void* stream) {
  if (int rc = require_ready(h, "gsmpm_fit_set_grads")) return rc;
  GSMPM_REQUIRE(xyz_grad && cov_grad, "gsmpm_fit_set_grads: null argument");
  hipStream_t st = S(stream);
  View& V = h->V;
  hipLaunchKernelGGL(k_scatter_in, dim3(blocks(h->n)), dim3(256), 0, st, V.gx + (size_t)(h->L - 1) * 3 * h->np, 3, h->n,
                     h->np, (const int*)h->order, xyz_grad);
  hipLaunchKernelGGL(k_scatter_in, dim3(blocks(h->n)), dim3(256), 0, st, V.gcov, 6, h->n, h->np, (const int*)h->order,
                     cov_grad);
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}

int gsmpm_fit_learn(gsmpm_fit* h, void* stream) {
  if (int rc = require_ready(h, "gsmpm_fit_learn")) return rc;
  hipLaunchKernelGGL(k_learn, dim3(blocks(h->n)), dim3(256), 0, S(stream), h->V);
  GSMPM_LAUNCH_CHECK();
  drop_grids(h);
  return GSMPM_OK;
}

int gsmpm_fit_mu_lam(gsmpm_fit* h, void* stream) {
  if (int rc = require_ready(h, "gsmpm_fit_mu_lam")) return rc;
  hipLaunchKernelGGL(k_mu_lam, dim3(blocks(h->n)), dim3(256), 0, S(stream), h->V);
  GSMPM_LAUNCH_CHECK();
  drop_grids(h);
  return GSMPM_OK;
}

int gsmpm_fit_cycle_init(gsmpm_fit* h, void* stream) {
  if (int rc = require_ready(h, "gsmpm_fit_cycle_init")) return rc;
  hipStream_t st = S(stream);
  View& V = h->V;
  const size_t np = h->np, last = h->L - 1;
  float* const planes[5] = {V.x, V.v, V.F, V.S, V.C};
  const int widths[5] = {3, 3, 9, 9, 9};
  for (int i = 0; i < 5; ++i)
    GSMPM_HIP(hipMemcpyAsync(planes[i], planes[i] + last * widths[i] * np, sizeof(float) * widths[i] * np,
                             hipMemcpyDeviceToDevice, st));
  h->binned[0] = 0;
  if (h->counted == 0) h->counted = -1;
  drop_grids(h);
  return GSMPM_OK;
}

int gsmpm_fit_clear_grads(gsmpm_fit* h, void* stream) {
  if (int rc = require_ready(h, "gsmpm_fit_clear_grads")) return rc;
  hipStream_t st = S(stream);
  View& V = h->V;
  const size_t np = h->np, L = h->L;
  // gx..gS are contiguous; so are glogE..glam; gcov; v_in.grad | v_out.grad
  GSMPM_HIP(hipMemsetAsync(V.gx, 0, (char*)(V.gS + L * 9 * np) - (char*)V.gx, st));
  GSMPM_HIP(hipMemsetAsync(V.glogE, 0, (char*)(V.glam + np) - (char*)V.glogE, st));
  GSMPM_HIP(hipMemsetAsync(V.gcov, 0, sizeof(float) * 6 * np, st));
  GSMPM_HIP(hipMemsetAsync(V.gvin, 0, sizeof(float) * 3 * h->nn, st));
  GSMPM_HIP(hipMemsetAsync(V.gvout, 0, sizeof(float) * 3 * h->nn, st));
  return GSMPM_OK;
}

int gsmpm_fit_field_width(int32_t field) {
  static const int w[GSMPM_FIT_FIELD_COUNT] = {3, 3, 9, 9, 9, 3, 3, 9, 9, 9, 1, 1, 1, 1, 1, 1, 1, 1, 6, 6, 6, 1, 1};
  if (field < 0 || field >= GSMPM_FIT_FIELD_COUNT) {
    set_error("gsmpm_fit_field_width: unknown field");
    return GSMPM_EINVAL;
  }
  return w[field];
}

static int fit_io(gsmpm_fit* h, int32_t field, int32_t level, float* out, const float* in, void* stream) {
  FieldDesc d = field_desc(h, field);
  GSMPM_REQUIRE(d.base, "gsmpm_fit_get/set: unknown field");
  GSMPM_REQUIRE(!d.leveled || (level >= 0 && level < h->L), "gsmpm_fit_get/set: level out of range");
  float* plane = d.base + (d.leveled ? (size_t)level * d.width * h->np : 0);
  hipStream_t st = S(stream);
  if (out)
    hipLaunchKernelGGL(k_gather_out, dim3(blocks(h->n)), dim3(256), 0, st, (const float*)plane, d.width, h->n, h->np,
                       (const int*)h->order, out);
  else
    hipLaunchKernelGGL(k_scatter_in, dim3(blocks(h->n)), dim3(256), 0, st, plane, d.width, h->n, h->np,
                       (const int*)h->order, in);
  GSMPM_LAUNCH_CHECK();
  if (in && field == GSMPM_FIT_X) {
    h->binned[level] = 0;
    if (h->counted == level) h->counted = -1;
  }
  if (in) drop_grids(h);
  return GSMPM_OK;
}

int gsmpm_fit_get(gsmpm_fit* h, int32_t field, int32_t level, float* out, void* stream) {
  if (int rc = require_ready(h, "gsmpm_fit_get")) return rc;
  GSMPM_REQUIRE(out, "gsmpm_fit_get: null output");
  return fit_io(h, field, level, out, nullptr, stream);
}

int gsmpm_fit_set(gsmpm_fit* h, int32_t field, int32_t level, const float* in, void* stream) {
  if (int rc = require_ready(h, "gsmpm_fit_set")) return rc;
  GSMPM_REQUIRE(in, "gsmpm_fit_set: null input");
  return fit_io(h, field, level, nullptr, in, stream);
}

int gsmpm_fit_get_grid(gsmpm_fit* h, int32_t which, float* out, void* stream) {
  if (int rc = require_ready(h, "gsmpm_fit_get_grid")) return rc;
  GSMPM_REQUIRE(out && which >= 0 && which <= 4, "gsmpm_fit_get_grid: bad argument");
  hipStream_t st = S(stream);
  View& V = h->V;
  const size_t lo = (size_t)h->glast * V.gstride;  // the grid computed last
  if (which == GSMPM_GRID_MASS) {
    GSMPM_HIP(hipMemcpyAsync(out, V.gm + lo, sizeof(float) * h->nn, hipMemcpyDeviceToDevice, st));
    return GSMPM_OK;
  }
  const float* src = which == GSMPM_GRID_V_IN ? V.vin + lo : which == GSMPM_GRID_V_OUT ? V.vout + lo : which == 3 ? V.gvin : V.gvout;
  hipLaunchKernelGGL(k_interleave, dim3(blocks(h->nn)), dim3(256), 0, st, src, h->nn, 3, out);
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}

}  // extern "C"

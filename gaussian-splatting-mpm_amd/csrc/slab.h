// slab.h -- multi-GPU spatial slabs on the fused pipeline (included by
// mpm.hip inside namespace gsmpm, after fused.h).  SURVEY.md 8(e).
//
// The reference is one device (mpm_solver/solver.py:27-52).  Here a scene is
// cut along grid axis 0 into slabs, one per rank (one GPU each):
//
//  * rank r owns the grid planes [lo, hi) and the particles whose base plane
//    (trunc(x0 * inv_dx - 0.5), utils.py:95) was in [lo, hi) at the last
//    migration.  Between migrations (every `interval` substeps) a particle may
//    drift M planes (the margin), so its stencil reaches planes
//    [lo - M, hi + M + 2).
//  * The planes two neighbours can both scatter into are the window
//    [b - M, b + M + 2) around each shared bound b (W = 2M + 2 planes).  After
//    P2G each rank writes its PARTIAL (m v, m) of every window node
//    (k_grid_f, SlabWin), the two ranks swap partials (RCCL send/recv over
//    the xGMI link between them, SlabXport in mpm.hip), and both compute the
//    node's total as lower-rank partial + upper-rank partial -- the same f32
//    sum on both sides -- and the grid update of it (k_win_update): the
//    pairwise "all-reduce of boundary grid nodes".  Nodes outside the windows
//    receive contributions from one rank only and are updated locally.
//  * G2P of rank r reads v_out on [lo - M, hi + M + 2): interior nodes from
//    its own grid update, window nodes from k_win_update.
//  * Migration (k_mig_*): particles whose base plane left [lo, hi) are
//    compacted (wave ballot + prefix sum, stable) into per-neighbour send
//    buffers, stayers into a compacted storage; arrivals are appended.  A
//    particle that drifts past the margin between migrations raises a flag
//    (k_fused, SlabK) -- the window exchange would have missed its
//    contributions -- and the host reports it.

constexpr int NMIG = NPLANES + NCOLD + 1;  // migration payload per particle: hot + cold planes + global id

// SlabWin / SlabK (the hooks in k_fused and k_grid_f) are declared in fused.h.

// Window totals and their grid update.  One lane per window node; the lower
// rank's partial is always the left operand, so both ranks of a bound compute
// bit-identical totals (and v_out).  The partial is zeroed for the next P2G.
__global__ __launch_bounds__(256) void k_win_update(GridDims g, SlabWin sw, const float4* __restrict__ recv0,
                                                   const float4* __restrict__ recv1, float4* __restrict__ gvel,
                                                   const BcTable* __restrict__ bct, GridStep gs) {
  const int ng = g.ng;
  const size_t per0 = sw.on[0] ? (size_t)sw.W * sw.ny[0] * sw.nz[0] : 0;
  const size_t per1 = sw.on[1] ? (size_t)sw.W * sw.ny[1] * sw.nz[1] : 0;
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < per0 + per1;
       q += (size_t)gridDim.x * blockDim.x) {
    const int w = q < per0 ? 0 : 1;
    const size_t r = q - (w ? per0 : 0);
    const int ny = sw.ny[w], nz = sw.nz[w];
    const int pl = (int)(r / ((size_t)ny * nz));
    const int i = sw.a[w] + pl;
    if (i < 0 || i >= ng) continue;
    const int j = sw.y0[w] + (int)((r / nz) % ny), k = sw.z0[w] + (int)(r % nz);
    const float4 mine = sw.part[w][r];
    const float4 other = w == 0 ? recv0[r] : recv1[r];
    float4 a = w == 0 ? other : mine;  // lower rank's partial first
    const float4 b = w == 0 ? mine : other;
    a.x += b.x;
    a.y += b.y;
    a.z += b.z;
    a.w += b.w;
    gvel[((size_t)i * ng + j) * ng + k] = node_update(a, i, j, k, g, gs, bct);
    sw.part[w][r] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// yz box of the particles' base nodes (trunc(x * inv_dx - 0.5), utils.py:95)
// -> out4 {min y, max y, min z, max z} (initialised to INT_MAX / INT_MIN).
__global__ __launch_bounds__(256) void k_slab_bbox(Particles ps, float inv_dx, int* __restrict__ out4) {
  int v[4] = {INT_MAX, INT_MIN, INT_MAX, INT_MIN};
  for (int p = blockIdx.x * 256 + threadIdx.x; p < ps.n; p += gridDim.x * 256) {
    const int by = (int)(ps.ld(PX + 1, p) * inv_dx - 0.5f), bz = (int)(ps.ld(PX + 2, p) * inv_dx - 0.5f);
    v[0] = min(v[0], by);
    v[1] = max(v[1], by);
    v[2] = min(v[2], bz);
    v[3] = max(v[3], bz);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v[0] = min(v[0], __shfl_xor(v[0], o));
    v[1] = max(v[1], __shfl_xor(v[1], o));
    v[2] = min(v[2], __shfl_xor(v[2], o));
    v[3] = max(v[3], __shfl_xor(v[3], o));
  }
  if ((threadIdx.x & 63) == 0 && v[0] <= v[1]) {
    atomicMin(out4 + 0, v[0]);
    atomicMax(out4 + 1, v[1]);
    atomicMin(out4 + 2, v[2]);
    atomicMax(out4 + 3, v[3]);
  }
}

// ------------------------------------------------------------- migration --
// Destination of a particle: 0 the lower neighbour, 1 stay, 2 the upper one.
struct MigGeom {
  float inv_dx;
  int lo, hi;      // owned planes
  int has_lo, has_hi;
};
__device__ __forceinline__ int mig_dest(const MigGeom& mg, float x0) {
  const int b = (int)(x0 * mg.inv_dx - 0.5f);  // utils.py:95 (trunc), as every kernel computes it
  if (mg.has_lo && b < mg.lo) return 0;
  if (mg.has_hi && b >= mg.hi) return 2;
  return 1;
}

// Per-block counts of the three destinations (wave ballots), blocks of 256.
__global__ __launch_bounds__(256) void k_mig_count(Particles ps, MigGeom mg, int* __restrict__ bcnt) {
  __shared__ int s_c[4][3];
  const int p = blockIdx.x * 256 + threadIdx.x;
  const int d = p < ps.n ? mig_dest(mg, ps.ld(PX, p)) : -1;
  const int wv = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const unsigned long long bal = __ballot(d == c);
    if ((threadIdx.x & 63) == 0) s_c[wv][c] = __popcll(bal);
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int c = threadIdx.x;
    bcnt[(size_t)blockIdx.x * 3 + c] = s_c[0][c] + s_c[1][c] + s_c[2][c] + s_c[3][c];
  }
}

// Exclusive scan of the per-block counts (one workgroup of 1024; nblk is a
// few thousand at most): boff[b][c] and the totals tot[c].
__global__ __launch_bounds__(1024) void k_mig_scan(int nblk, const int* __restrict__ bcnt, int* __restrict__ boff,
                                                   int* __restrict__ tot) {
  __shared__ int s_w[16][3];
  __shared__ int s_carry[3];
  if (threadIdx.x < 3) s_carry[threadIdx.x] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int base = 0; base < nblk; base += 1024) {
    const int b = base + threadIdx.x;
    int v[3], incl[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      v[c] = b < nblk ? bcnt[(size_t)b * 3 + c] : 0;
      incl[c] = v[c];
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl[c], o);
        if (lane >= o) incl[c] += t;
      }
      if (lane == 63) s_w[wv][c] = incl[c];
    }
    __syncthreads();
    if (threadIdx.x < 3) {  // wave sums -> exclusive wave offsets
      int run = s_carry[threadIdx.x];
      for (int w = 0; w < 16; ++w) {
        const int t = s_w[w][threadIdx.x];
        s_w[w][threadIdx.x] = run;
        run += t;
      }
      s_carry[threadIdx.x] = run;
    }
    __syncthreads();
    if (b < nblk) {
#pragma unroll
      for (int c = 0; c < 3; ++c) boff[(size_t)b * 3 + c] = s_w[wv][c] + incl[c] - v[c];
    }
    __syncthreads();
  }
  if (threadIdx.x < 3) tot[threadIdx.x] = s_carry[threadIdx.x];
}

// Stable scatter: stayers to rows [0, n_stay) of the new storage (hot planes,
// and the cold planes / global id read through orig, which become caller
// order = the new storage order); leavers to their send buffer, SoA
// [NMIG][count] (hot planes, cold planes, id as float bits).
struct MigOut {
  float* planes;   // new hot planes [NPLANES][np]
  float* cold;     // new cold planes [NCOLD][np]
  int* gid;        // new global ids [np]
  float* send[2];  // lower / upper payloads
};
__global__ __launch_bounds__(256) void k_mig_scatter(Particles ps, const int* __restrict__ orig,
                                                     const int* __restrict__ gid, MigGeom mg,
                                                     const int* __restrict__ boff, const int* __restrict__ tot,
                                                     MigOut mo) {
  __shared__ int s_c[4][3];
  const int p = blockIdx.x * 256 + threadIdx.x;
  const int d = p < ps.n ? mig_dest(mg, ps.ld(PX, p)) : -1;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int rank_in_wave = 0;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const unsigned long long bal = __ballot(d == c);
    if (lane == 0) s_c[wv][c] = __popcll(bal);
    if (d == c) rank_in_wave = __popcll(bal & ((1ull << lane) - 1ull));  // mbcnt
  }
  __syncthreads();
  if (d < 0) return;
  int row = boff[(size_t)blockIdx.x * 3 + d] + rank_in_wave;
  for (int w = 0; w < wv; ++w) row += s_c[w][d];
  const int src = orig[p];  // caller row of the cold planes / id
  if (d == 1) {
    for (int q = 0; q < NPLANES; ++q) mo.planes[(size_t)q * ps.np + row] = ps.ld(q, p);
    for (int q = 0; q < NCOLD; ++q) mo.cold[(size_t)q * ps.np + row] = ps.ldc(q, src);
    mo.gid[row] = gid[src];
  } else {
    float* out = mo.send[d >> 1];
    const size_t cnt = (size_t)tot[d];
    for (int q = 0; q < NPLANES; ++q) out[(size_t)q * cnt + row] = ps.ld(q, p);
    for (int q = 0; q < NCOLD; ++q) out[(size_t)(NPLANES + q) * cnt + row] = ps.ldc(q, src);
    out[(size_t)(NPLANES + NCOLD) * cnt + row] = __int_as_float(gid[src]);
  }
}

// Arrivals: payload rows -> storage rows [row0, row0 + cnt) (hot + cold + id).
__global__ __launch_bounds__(256) void k_mig_unpack(const float* __restrict__ in, int cnt, int row0, float* planes,
                                                    float* cold, int* gid, int np) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= cnt) return;
  const size_t c = (size_t)cnt;
  for (int q = 0; q < NPLANES; ++q) planes[(size_t)q * np + row0 + r] = in[(size_t)q * c + r];
  for (int q = 0; q < NCOLD; ++q) cold[(size_t)q * np + row0 + r] = in[(size_t)(NPLANES + q) * c + r];
  gid[row0 + r] = __float_as_int(in[(size_t)(NPLANES + NCOLD) * c + r]);
}

__global__ __launch_bounds__(256) void k_iota(int* __restrict__ a, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) a[i] = i;
}

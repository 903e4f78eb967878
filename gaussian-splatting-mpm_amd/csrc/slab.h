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
//    (k_fused's xlo / xhi check) -- the window exchange would have missed its
//    contributions -- and the host reports it.

constexpr int NMIG = NPLANES + NCOLD + 1;  // migration payload per particle: hot + cold planes + global id

// SlabWin and k_fused's xlo / xhi / FusedRare::drift (the hooks in k_grid_f and k_fused) are declared in fused.h.

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

// ------------------------------------------------------------ slab record --
// Every slab's state after a step call, exchanged with every rank (one round,
// 64 bytes a peer) so all ranks see the same errors, counts and boxes.
enum SlabRec : int {
  RF_FLAGS = 0,   // bit 0 drift past the margin, 1 window mass outside the rect, 3 over capacity,
                  // 4 a non-finite particle position
  RF_N = 1,       // live particles
  RF_NWANT = 2,   // the most particles a migration tried to hold (capacity overflow)
  RF_SENDMAX = 3, // the most leavers one migration sent one way (send capacity)
  RF_MIGRATED = 4,
  RF_YLO = 5, RF_YHI = 6, RF_ZLO = 7, RF_ZHI = 8,  // yz box of the particles' base nodes
  RF_VY = 9, RF_VZ = 10,                            // max |v_y|, |v_z| (f32 bits)
  RF_BAND_LO = 11, RF_BAND_HI = 12,                 // particles within `margin` planes of the lower / upper bound
  RF_DEFERRED = 13,                                 // leavers kept for a later migration (payload full)
  RF_CAP = 14,                                      // the slab's particle capacity
  RF_MMIN = 15,                                     // min particle mass (f32 bits; INT_MAX: no particle)
  RF_SLO = 16, RF_SHI = 17,                         // this rank's slab planes [lo, hi)
  RF_WEIGHT = 18,                                   // this rank's share weight of the re-cut (f32 bits; 1: even)
  kRecHdr = 20                                      // then ng ints: the particles' base-plane histogram
};
// ints of one rank's record: the header and the base-plane histogram (the
// load every rank needs to re-cut the slabs, slab_host.inc slab_rebalance)
__host__ __device__ constexpr int rec_ints_of(int ng) { return kRecHdr + ng; }
// Device flags of a slab (s_flags): sticky until the handle is reset.
enum SlabFlag : int {
  SF_DRIFT = 0, SF_OOB = 1, SF_DEFERRED = 2, SF_NWANT_OVER = 3, SF_SENDMAX = 4, SF_MIGRATED = 5, SF_NONFIN = 6,
  kSlabFlags = 8
};

struct MigGeom {
  float inv_dx;
  int lo, hi;      // owned planes
  int has_lo, has_hi;
};

__global__ void k_rec_init(const int* __restrict__ flags, const int* __restrict__ nlive, int capacity, int lo, int hi,
                           int nrec, int* __restrict__ rec, const float* __restrict__ weight) {
  for (int i = kRecHdr + threadIdx.x; i < nrec; i += blockDim.x) rec[i] = 0;  // the histogram
  if (threadIdx.x != 0) return;
  rec[RF_FLAGS] = (flags[SF_DRIFT] ? 1 : 0) | (flags[SF_OOB] ? 2 : 0) | (flags[SF_NWANT_OVER] ? 8 : 0) |
                  (flags[SF_NONFIN] ? 16 : 0);
  rec[RF_N] = *nlive;
  rec[RF_NWANT] = flags[SF_NWANT_OVER];
  rec[RF_SENDMAX] = flags[SF_SENDMAX];
  rec[RF_MIGRATED] = flags[SF_MIGRATED];
  rec[RF_YLO] = INT_MAX;
  rec[RF_YHI] = INT_MIN;
  rec[RF_ZLO] = INT_MAX;
  rec[RF_ZHI] = INT_MIN;
  rec[RF_VY] = 0;
  rec[RF_VZ] = 0;
  rec[RF_BAND_LO] = 0;
  rec[RF_BAND_HI] = 0;
  rec[RF_DEFERRED] = flags[SF_DEFERRED];
  rec[RF_CAP] = capacity;
  rec[RF_MMIN] = INT_MAX;
  rec[RF_SLO] = lo;
  rec[RF_SHI] = hi;
  rec[RF_WEIGHT] = __float_as_int(*weight);
  for (int i = RF_WEIGHT + 1; i < kRecHdr; ++i) rec[i] = 0;
}

// yz box of the particles' base nodes (trunc(x * inv_dx - 0.5), utils.py:95),
// max |v_y|, |v_z| and the particles within `margin` planes of each bound (the
// most that can leave by the next migration) -> rec (after k_rec_init).
constexpr int kRecMaxNg = 4096;  // the LDS histogram of k_slab_record
__global__ __launch_bounds__(256) void k_slab_record(Particles ps, MigGeom mg, int margin, int ng,
                                                     int* __restrict__ rec) {
  __shared__ int s_h[kRecMaxNg];
  for (int i = threadIdx.x; i < ng; i += 256) s_h[i] = 0;
  __syncthreads();
  int v[4] = {INT_MAX, INT_MIN, INT_MAX, INT_MIN};
  float vy = 0.f, vz = 0.f, mmin = __int_as_float(INT_MAX);  // INT_MAX bits: a NaN above every finite mass
  int blo = 0, bhi = 0;
  const int n = ps.count();
  for (int p = blockIdx.x * 256 + threadIdx.x; p < n; p += gridDim.x * 256) {
    const int bx = (int)(ps.ld(PX, p) * mg.inv_dx - 0.5f);
    const int by = (int)(ps.ld(PX + 1, p) * mg.inv_dx - 0.5f), bz = (int)(ps.ld(PX + 2, p) * mg.inv_dx - 0.5f);
    v[0] = min(v[0], by);
    v[1] = max(v[1], by);
    v[2] = min(v[2], bz);
    v[3] = max(v[3], bz);
    vy = fmaxf(vy, fabsf(ps.ld(PV + 1, p)));
    vz = fmaxf(vz, fabsf(ps.ld(PV + 2, p)));
    mmin = __int_as_float(min(__float_as_int(mmin), __float_as_int(ps.ld(PMASS, p))));
    blo += (bx < mg.lo + margin) ? 1 : 0;
    bhi += (bx >= mg.hi - margin) ? 1 : 0;
    atomicAdd(&s_h[min(max(bx, 0), ng - 1)], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < ng; i += 256)
    if (s_h[i]) atomicAdd(rec + kRecHdr + i, s_h[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v[0] = min(v[0], __shfl_xor(v[0], o));
    v[1] = max(v[1], __shfl_xor(v[1], o));
    v[2] = min(v[2], __shfl_xor(v[2], o));
    v[3] = max(v[3], __shfl_xor(v[3], o));
    vy = fmaxf(vy, __shfl_xor(vy, o));
    vz = fmaxf(vz, __shfl_xor(vz, o));
    mmin = __int_as_float(min(__float_as_int(mmin), __float_as_int(__shfl_xor(mmin, o))));
    blo += __shfl_xor(blo, o);
    bhi += __shfl_xor(bhi, o);
  }
  if ((threadIdx.x & 63) == 0) {
    if (v[0] <= v[1]) {
      atomicMin(rec + RF_YLO, v[0]);
      atomicMax(rec + RF_YHI, v[1]);
      atomicMin(rec + RF_ZLO, v[2]);
      atomicMax(rec + RF_ZHI, v[3]);
    }
    // non-negative floats order as their bit patterns (NaN: all bits set, wins)
    atomicMax(rec + RF_VY, __float_as_int(vy));
    atomicMax(rec + RF_VZ, __float_as_int(vz));
    atomicMin(rec + RF_MMIN, __float_as_int(mmin));  // masses are positive: bit order is value order
    if (blo) atomicAdd(rec + RF_BAND_LO, blo);
    if (bhi) atomicAdd(rec + RF_BAND_HI, bhi);
  }
}

// ------------------------------------------------------------- migration --
// Runs on the device between two chunks of substeps, inside the captured
// frame: the counts never visit the host.  The payload to each neighbour has
// a FIXED size (RCCL send/recv sizes are baked into the graph): a header of
// kMigHdr ints (the leaver count first) and [NMIG][cap] floats.  Leavers
// beyond `cap` stay for a later migration (SF_DEFERRED): ownership does not
// change the physics while a particle stays within the margin, which k_fused
// checks, and the host grows `cap` after the call.
constexpr int kMigHdr = 16;
__host__ __device__ constexpr size_t mig_payload_floats(int cap) { return (size_t)kMigHdr + (size_t)NMIG * cap; }

// Destination of a particle: 0 the lower neighbour, 1 stay, 2 the upper one.
__device__ __forceinline__ int mig_dest(const MigGeom& mg, float x0) {
  const int b = (int)(x0 * mg.inv_dx - 0.5f);  // utils.py:95 (trunc), as every kernel computes it
  if (mg.has_lo && b < mg.lo) return 0;
  if (mg.has_hi && b >= mg.hi) return 2;
  return 1;
}

// Per-block counts of the three destinations (wave ballots), blocks of 256
// over the capacity (rows past the live count count nowhere).
__global__ __launch_bounds__(256) void k_mig_count(Particles ps, MigGeom mg, int* __restrict__ bcnt) {
  __shared__ int s_c[4][3];
  const int p = blockIdx.x * 256 + threadIdx.x;
  const int d = p < ps.count() ? mig_dest(mg, ps.ld(PX, p)) : -1;
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
// few thousand at most): boff[b][c] and the totals tot = {leavers down,
// stayers, leavers up, rows kept (stayers + deferred leavers)}; then the send
// headers and the statistics flags.
struct MigSend {
  float* buf[2];  // lower / upper payloads (null: no neighbour)
  int cap;
  int* flags;     // s_flags
};
__global__ __launch_bounds__(1024) void k_mig_scan(int nblk, const int* __restrict__ bcnt, int* __restrict__ boff,
                                                   int* __restrict__ tot, MigSend ms) {
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
  if (threadIdx.x == 0) {
    const int c_lo = s_carry[0], n_stay = s_carry[1], c_hi = s_carry[2];
    const int d_lo = max(0, c_lo - ms.cap), d_hi = max(0, c_hi - ms.cap);
    tot[0] = c_lo;
    tot[1] = n_stay;
    tot[2] = c_hi;
    tot[3] = n_stay + d_lo + d_hi;
    if (ms.buf[0]) reinterpret_cast<int*>(ms.buf[0])[0] = c_lo - d_lo;
    if (ms.buf[1]) reinterpret_cast<int*>(ms.buf[1])[0] = c_hi - d_hi;
    atomicMax(ms.flags + SF_SENDMAX, max(c_lo, c_hi));
    if (d_lo + d_hi) atomicAdd(ms.flags + SF_DEFERRED, d_lo + d_hi);
    atomicAdd(ms.flags + SF_MIGRATED, c_lo - d_lo + c_hi - d_hi);
  }
}

// Stable scatter: stayers to rows [0, n_stay) of the new storage (hot planes,
// and the cold planes / global id read through orig, which become caller
// order = the new storage order), deferred leavers after them; leavers to
// their payload, SoA [NMIG][cap] after the header (hot planes, cold planes,
// id as float bits).
struct MigOut {
  float* planes;   // new hot planes [NPLANES][np]
  float* cold;     // new cold planes [NCOLD][np]
  int* gid;        // new global ids [np]
};
__global__ __launch_bounds__(256) void k_mig_scatter(Particles ps, const int* __restrict__ orig,
                                                     const int* __restrict__ gid, MigGeom mg,
                                                     const int* __restrict__ boff, const int* __restrict__ tot,
                                                     MigOut mo, MigSend ms) {
  __shared__ int s_c[4][3];
  const int p = blockIdx.x * 256 + threadIdx.x;
  int d = p < ps.count() ? mig_dest(mg, ps.ld(PX, p)) : -1;
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
  if (d != 1 && row >= ms.cap) {  // payload full: stays, after the stayers
    row = tot[1] + (d == 0 ? 0 : max(0, tot[0] - ms.cap)) + row - ms.cap;
    d = 1;
  }
  if (d == 1) {
    for (int q = 0; q < NPLANES; ++q) mo.planes[(size_t)q * ps.np + row] = ps.ld(q, p);
    for (int q = 0; q < NCOLD; ++q) mo.cold[(size_t)q * ps.np + row] = ps.ldc(q, src);
    mo.gid[row] = gid[src];
  } else {
    float* out = ms.buf[d >> 1] + kMigHdr;
    const size_t cap = (size_t)ms.cap;
    for (int q = 0; q < NPLANES; ++q) out[(size_t)q * cap + row] = ps.ld(q, p);
    for (int q = 0; q < NCOLD; ++q) out[(size_t)(NPLANES + q) * cap + row] = ps.ldc(q, src);
    out[(size_t)(NPLANES + NCOLD) * cap + row] = __int_as_float(gid[src]);
  }
}

// Arrivals: payload rows -> storage rows after the kept rows (blockIdx.y =
// the side: the lower neighbour's first), hot + cold + id; rows past the capacity
// raise SF_NWANT_OVER and are dropped (the state is invalid).
struct MigRecv {
  const float* buf[2];  // null: no neighbour on that side
  int cap;
};
__device__ __forceinline__ int mig_arrivals(const MigRecv& mr, int w) {
  return mr.buf[w] ? reinterpret_cast<const int*>(mr.buf[w])[0] : 0;
}
__global__ __launch_bounds__(256) void k_mig_unpack(MigRecv mr, const int* __restrict__ tot, float* planes,
                                                    float* cold, int* gid, int np, int capacity) {
  const int w = blockIdx.y;
  const int cnt = mig_arrivals(mr, w);
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= cnt) return;
  const int row = tot[3] + (w ? mig_arrivals(mr, 0) : 0) + r;
  if (row >= capacity) return;
  const float* in = mr.buf[w] + kMigHdr;
  const size_t c = (size_t)mr.cap;
  for (int q = 0; q < NPLANES; ++q) planes[(size_t)q * np + row] = in[(size_t)q * c + r];
  for (int q = 0; q < NCOLD; ++q) cold[(size_t)q * np + row] = in[(size_t)(NPLANES + q) * c + r];
  gid[row] = __float_as_int(in[(size_t)(NPLANES + NCOLD) * c + r]);
}

// The new live count (kept rows + arrivals, capped at the slab's capacity:
// the chunk tables are sized for it), and the caller order := the new
// storage order.
__global__ __launch_bounds__(256) void k_mig_finish(MigRecv mr, const int* __restrict__ tot, int capacity,
                                                    int* __restrict__ nlive, int* __restrict__ orig,
                                                    int* __restrict__ flags) {
  const int want = tot[3] + mig_arrivals(mr, 0) + mig_arrivals(mr, 1);
  const int n = min(want, capacity);
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i == 0) {
    *nlive = n;
    if (want > capacity) atomicMax(flags + SF_NWANT_OVER, want);
  }
  if (i < n) orig[i] = i;
}

__global__ void k_set_int(int* __restrict__ p, int v) {
  if (threadIdx.x == 0) *p = v;
}

// dsort.h -- the rasterizer's depth order, hand-written (included by
// raster.hip inside namespace gsmpm).
//
// The forward needs the Gaussians in (depth, index) order and, in that order,
// the inclusive scan of their tiles words ((3-sigma count << 32) | binned
// count): the scan gives every Gaussian's emission offset, and its last entry
// K and num_rendered (upstream: the stable radix sort of (tile << 32 | depth
// bits) keys, duplicateWithKeys' offsets).  Depths of visible Gaussians are
// > 0.2 (k_preprocess culls nearer ones), so their f32 bit patterns order as
// the depths do.
//
// Instead of a device-wide radix sort, the visible Gaussians are bucketed on
// their depth bits and each bucket is sorted where it lies:
//   k_preprocess     also reduces the visible depth bits' min and max into 8
//                    shards each (one atomic per wave)
//   k_dsort_hist     bucket b = (bits - lo) >> shift (NB buckets spanning
//                    [lo, hi]): count and tiles-word sum per bucket
//                    (returnless global atomics)
//   k_dsort_scan     one workgroup: exclusive scans of the bucket counts and
//                    sums, the list of occupied buckets (small and big ones)
//   k_dsort_scatter  every visible Gaussian to its bucket's run (returning
//                    atomic cursor: any order inside the run); culled ones to
//                    the tail [Pv, P) (they carry no pair)
//   k_dsort_small    a wave per occupied bucket of <= kDsSmall: rank every
//                    entry by the unique composite (bits << 32 | index), write
//                    the order and the scan of its tiles words (bucket prefix
//                    + in-bucket inclusive scan)
//   k_dsort_big      a 1,024-lane workgroup per bucket of (kDsSmall, kDsBig]:
//                    bitonic sort of the composites in LDS, the same outputs
// The result is exactly the order a stable sort of the depth bits gives (ties
// keep index order) -- bit-identical emission, tile lists and images.  A
// bucket of more than kDsBig entries (a degenerate depth distribution: tens
// of thousands of Gaussians within a few ulps) raises a flag the host reads
// with the pair count; the forward then takes the library sort instead
// (raster.hip; tested with a scene of equal depths).
//
// State (dstate, bucket arrays) is zero when idle: every forward leaves it
// zeroed for the next one (the min shards hold the complement of the bits so
// that zero is their identity), so a caller-owned workspace only needs to be
// zero-filled once, when it is created.

constexpr int kDsNBMax = 65536;   // buckets, at most
constexpr int kDsSmall = 256;     // entries a wave sorts
constexpr int kDsBig = 8192;      // entries a workgroup sorts
constexpr int kDsScanT = 1024;
// dstate words
enum : int {
  DS_MIN = 0,      // [8] shards: max of ~bits (zero = identity)
  DS_MAX = 8,      // [8] shards: max of bits
  DS_CULL = 16,    // culled cursor
  DS_NLIST = 17,   // occupied buckets of <= kDsSmall
  DS_NBIG = 18,    // occupied buckets above
  DS_OVER = 19,    // a bucket above kDsBig (host fallback)
  DS_PV = 20,      // visible Gaussians
  DS_LO = 21, DS_SHIFT = 22, DS_NB = 23,
  DS_TOT = 24,     // [2] u64 total of the tiles words (K | num_rendered << 32)
  DS_MAXN = 26,    // the largest bucket (diagnostics)
  kDsWords = 32
};

// bytes of the depth-order state (fixed layout at the start of a workspace)
constexpr size_t kDsStateBytes = kDsWords * 4 + (size_t)kDsNBMax * (4 + 8);  // dstate, bcount, bsum

struct DsortBufs {
  unsigned* st;                // dstate [kDsWords]
  unsigned* bcount;            // [kDsNBMax]  (zero when idle)
  unsigned long long* bsum;    // [kDsNBMax]  (zero when idle)
  unsigned* bbase;             // [kDsNBMax]  run start of an occupied bucket
  unsigned* bcur;              // [kDsNBMax]  scatter cursor
  unsigned long long* bpre;    // [kDsNBMax]  exclusive prefix of the tiles words
  unsigned* blist;             // [kDsNBMax]  occupied buckets <= kDsSmall
  unsigned* bbig;              // [kDsNBMax]  occupied buckets above
  unsigned* dkey;              // [P] depth bits by bucket run
  unsigned* dval;              // [P] Gaussian index by bucket run
};

__device__ __forceinline__ int ds_log2(int nb) { return 31 - __clz(nb); }

// the bucket map: lo and shift from the shards
__device__ __forceinline__ void ds_range(const unsigned* st, int nb, unsigned& lo, int& shift) {
  unsigned nlo = 0, hi = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    nlo = max(nlo, __hip_atomic_load(st + DS_MIN + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    hi = max(hi, __hip_atomic_load(st + DS_MAX + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
  lo = ~nlo;
  const unsigned span = hi >= lo ? hi - lo : 0u;
  const int nbits = span ? 32 - __clz(span) : 0;
  shift = max(0, nbits - ds_log2(nb));
}

// k_preprocess's contribution: min / max of the visible depth bits, per wave
__device__ __forceinline__ void ds_minmax(unsigned* st, bool vis, unsigned bits) {
  unsigned nlo = vis ? ~bits : 0u, hi = vis ? bits : 0u;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    nlo = max(nlo, (unsigned)__shfl_xor((int)nlo, o));
    hi = max(hi, (unsigned)__shfl_xor((int)hi, o));
  }
  if ((threadIdx.x & 63) == 0 && hi != 0u) {
    const int sh = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & 7;
    __hip_atomic_fetch_max(st + DS_MIN + sh, nlo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_max(st + DS_MAX + sh, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(256) void k_dsort_hist(int P, int nb, const float* __restrict__ depth,
                                                    const unsigned long long* __restrict__ tiles, DsortBufs d) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= P) return;
  const unsigned long long tw = tiles[i];
  if (tw == 0ull) return;  // culled (k_preprocess wrote no depth)
  unsigned lo;
  int shift;
  ds_range(d.st, nb, lo, shift);
  const unsigned b = (__float_as_uint(depth[i]) - lo) >> shift;
  __hip_atomic_fetch_add(d.bcount + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_add(d.bsum + b, tw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one workgroup: exclusive scans of counts and sums over the nb buckets, in
// coalesced passes of 1,024 buckets (a bucket per lane: wave scans, then the
// 16 wave totals through LDS, a running carry across passes)
__global__ __launch_bounds__(kDsScanT) void k_dsort_scan(int nb, DsortBufs d) {
  __shared__ unsigned s_wc[kDsScanT / 64];
  __shared__ unsigned long long s_ws[kDsScanT / 64];
  __shared__ unsigned s_nl, s_nb, s_over, s_maxn;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t == 0) s_nl = s_nb = s_over = s_maxn = 0;
  unsigned carry_c = 0;
  unsigned long long carry_s = 0;
  for (int b0 = 0; b0 < nb; b0 += kDsScanT) {  // workgroup-uniform
    const int b = b0 + t;
    const unsigned n = d.bcount[b];
    const unsigned long long sm = d.bsum[b];
    unsigned ic = n;
    unsigned long long is = sm;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned uc = (unsigned)__shfl_up((int)ic, o);
      const unsigned long long us = __shfl_up(is, o);
      if (lane >= o) {
        ic += uc;
        is += us;
      }
    }
    if (lane == 63) {
      s_wc[wv] = ic;
      s_ws[wv] = is;
    }
    __syncthreads();
    unsigned pc = carry_c, tc = 0;
    unsigned long long ps = carry_s, ts = 0;
#pragma unroll
    for (int q = 0; q < kDsScanT / 64; ++q) {
      const unsigned xc = s_wc[q];
      const unsigned long long xs = s_ws[q];
      if (q < wv) {
        pc += xc;
        ps += xs;
      }
      tc += xc;
      ts += xs;
    }
    if (n) {
      d.bbase[b] = pc + ic - n;
      d.bcur[b] = pc + ic - n;
      d.bpre[b] = ps + is - sm;
      if (n <= (unsigned)kDsSmall) {
        d.blist[atomicAdd(&s_nl, 1u)] = (unsigned)b;
      } else {
        d.bbig[atomicAdd(&s_nb, 1u)] = (unsigned)b;
        if (n > (unsigned)kDsBig) s_over = 1u;
      }
      atomicMax(&s_maxn, n);
    }
    carry_c += tc;
    carry_s += ts;
    __syncthreads();  // s_wc / s_ws reused by the next pass
  }
  if (t == 0) {
    unsigned lo;
    int shift;
    ds_range(d.st, nb, lo, shift);
    d.st[DS_LO] = lo;
    d.st[DS_SHIFT] = (unsigned)shift;
    d.st[DS_NB] = (unsigned)nb;
    d.st[DS_NLIST] = s_nl;
    d.st[DS_NBIG] = s_nb;
    d.st[DS_OVER] = s_over;
    d.st[DS_MAXN] = s_maxn;
    d.st[DS_PV] = carry_c;
    d.st[DS_CULL] = 0;
    d.st[DS_TOT] = (unsigned)carry_s;
    d.st[DS_TOT + 1] = (unsigned)(carry_s >> 32);
  }
}

__global__ __launch_bounds__(256) void k_dsort_scatter(int P, const float* __restrict__ depth,
                                                       const unsigned long long* __restrict__ tiles, DsortBufs d,
                                                       unsigned* __restrict__ order,
                                                       unsigned long long* __restrict__ offr) {
  if (blockIdx.x == 0 && threadIdx.x < 16) d.st[DS_MIN + threadIdx.x] = 0u;  // the shards: read for the last time by k_dsort_scan
  const int i = blockIdx.x * 256 + threadIdx.x;
  const unsigned lo = d.st[DS_LO], shift = d.st[DS_SHIFT], pv = d.st[DS_PV];
  const bool in = i < P;
  const unsigned long long tw = in ? tiles[i] : 1ull;
  const bool culled = in && tw == 0ull;
  // culled: one returning atomic per wave, the tail [Pv, P) in any order (no pairs: no output depends on it)
  const unsigned long long m = __ballot(culled);
  if (m) {
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)m) - 1;
    unsigned base = 0;
    if (lane == leader) base = atomicAdd(d.st + DS_CULL, (unsigned)__popcll(m));
    base = (unsigned)__shfl((int)base, leader);
    if (culled) {
      const unsigned pos = pv + base + (unsigned)__popcll(m & ((1ull << lane) - 1ull));
      order[pos] = (unsigned)i;
      offr[pos] = ((unsigned long long)d.st[DS_TOT + 1] << 32) | d.st[DS_TOT];
    }
  }
  if (!in || culled) return;
  const unsigned bits = __float_as_uint(depth[i]);
  const unsigned b = (bits - lo) >> shift;
  const unsigned pos = atomicAdd(d.bcur + b, 1u);
  d.dkey[pos] = bits;
  d.dval[pos] = (unsigned)i;
}

// inclusive u64 scan over the wave
__device__ __forceinline__ unsigned long long ds_wave_scan(unsigned long long v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  return v;
}

// a wave per occupied bucket of <= kDsSmall entries; 4 waves per workgroup,
// the workgroup's waves move through the list together (barriers are uniform)
__global__ __launch_bounds__(256) void k_dsort_small(const unsigned long long* __restrict__ tiles, DsortBufs d,
                                                     unsigned* __restrict__ order,
                                                     unsigned long long* __restrict__ offr) {
  __shared__ unsigned long long s_c[4][kDsSmall];
  __shared__ unsigned s_id[4][kDsSmall];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nl = (int)d.st[DS_NLIST];
  for (int base = blockIdx.x * 4; base < nl; base += gridDim.x * 4) {  // workgroup-uniform
    const int li = base + wv;
    const bool act = li < nl;
    const unsigned b = act ? d.blist[li] : 0u;
    const int n = act ? (int)d.bcount[b] : 0;
    const unsigned s = act ? d.bbase[b] : 0u;
    for (int j = lane; j < n; j += 64)
      s_c[wv][j] = ((unsigned long long)d.dkey[s + j] << 32) | d.dval[s + j];
    __syncthreads();
    // rank = number of smaller composites (all distinct: the index is in the low word)
    for (int j = lane; j < n; j += 64) {
      const unsigned long long c = s_c[wv][j];
      int r = 0;
      for (int k = 0; k < n; ++k) r += s_c[wv][k] < c ? 1 : 0;
      s_id[wv][r] = (unsigned)c;
    }
    __syncthreads();
    unsigned long long carry = act ? d.bpre[b] : 0ull;
    for (int j0 = 0; j0 < n; j0 += 64) {
      const int j = j0 + lane;
      const unsigned g = j < n ? s_id[wv][j] : 0u;
      const unsigned long long tw = j < n ? tiles[g] : 0ull;
      const unsigned long long inc = ds_wave_scan(tw);
      if (j < n) {
        order[s + j] = g;
        offr[s + j] = carry + inc;
      }
      carry += __shfl(inc, 63);
    }
    if (act && lane == 0) {  // idle state for the next forward
      d.bcount[b] = 0u;
      d.bsum[b] = 0ull;
    }
    __syncthreads();
  }
}

// a workgroup per bucket of (kDsSmall, kDsBig] entries: bitonic sort in LDS
__global__ __launch_bounds__(1024) void k_dsort_big(const unsigned long long* __restrict__ tiles, DsortBufs d,
                                                    unsigned* __restrict__ order,
                                                    unsigned long long* __restrict__ offr) {
  __shared__ unsigned long long s_c[kDsBig];
  __shared__ unsigned long long s_w[16];
  const int nbg = (int)d.st[DS_NBIG];
  for (int w = blockIdx.x; w < nbg; w += gridDim.x) {
    const unsigned b = d.bbig[w];
    const int n = (int)d.bcount[b];
    const unsigned s = d.bbase[b];
    if (n <= kDsBig) {  // larger: the host falls back (DS_OVER)
      int m = 1;
      while (m < n) m <<= 1;
      for (int j = threadIdx.x; j < m; j += 1024)
        s_c[j] = j < n ? ((unsigned long long)d.dkey[s + j] << 32) | d.dval[s + j] : ~0ull;
      __syncthreads();
      for (int k = 2; k <= m; k <<= 1)
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
          for (int i = threadIdx.x; i < m; i += 1024) {
            const int p = i ^ jj;
            if (p > i) {
              const unsigned long long a = s_c[i], c = s_c[p];
              const bool up = (i & k) == 0;
              if ((a > c) == up) {
                s_c[i] = c;
                s_c[p] = a;
              }
            }
          }
          __syncthreads();
        }
      unsigned long long carry = d.bpre[b];
      for (int j0 = 0; j0 < n; j0 += 1024) {
        const int j = j0 + (int)threadIdx.x;
        const unsigned g = j < n ? (unsigned)s_c[j] : 0u;
        const unsigned long long tw = j < n ? tiles[g] : 0ull;
        unsigned long long inc = ds_wave_scan(tw);
        if ((threadIdx.x & 63) == 63) s_w[threadIdx.x >> 6] = inc;
        __syncthreads();
        unsigned long long wpre = 0, tot = 0;
        for (int q = 0; q < 16; ++q) {
          const unsigned long long x = s_w[q];
          wpre += q < (int)(threadIdx.x >> 6) ? x : 0ull;
          tot += x;
        }
        if (j < n) {
          order[s + j] = g;
          offr[s + j] = carry + wpre + inc;
        }
        carry += tot;
        __syncthreads();
      }
    }
    if (threadIdx.x == 0) {
      d.bcount[b] = 0u;
      d.bsum[b] = 0ull;
    }
    __syncthreads();
  }
}

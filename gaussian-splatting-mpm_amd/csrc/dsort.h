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
//   k_preprocess     also reduces the visible depth bits' min and max into 64
//                    shards (one atomic pair per workgroup)
//   k_dsort_hist     bucket b = (bits - lo) >> shift (NB buckets spanning
//                    [lo, hi]): count and tiles-word sum per bucket
//                    (returnless global atomics)
//   k_dsort_scan1/2  exclusive scans of the bucket counts and sums (block
//                    totals, then each block's scan), the lists of occupied
//                    buckets (small and big ones)
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
  DS_CULL = 16,    // culled cursor
  DS_NLIST = 17,   // occupied buckets of <= kDsSmall
  DS_NBIG = 18,    // occupied buckets above
  DS_OVER = 19,    // a bucket above kDsBig (host fallback): set by k_dsort_scan1, reset by k_dsort_scatter
  DS_PV = 20,      // visible Gaussians
  DS_LO = 21, DS_SHIFT = 22, DS_NB = 23,
  DS_TOT = 24,     // [2] u64 total of the tiles words (K | num_rendered << 32)
  DS_MAXN = 26,    // the largest bucket (diagnostics)
  DS_OVERD = 29,   // the overflow flag the last bucket-form forward published (diagnostics)
  DS_BIGANY = 30,  // a bucket above kDsSmall (k_dsort_big has work): set by k_dsort_scan1, reset by k_dsort_scatter
  kDsWords = 32
};

// The visible depth bits' min / max: 64 shards, one 256-byte line each (word 0:
// max of ~bits, zero = identity; word 1: max of bits).  Round 4's first form
// had 8 shards in one line and an atomic pair per wave: 2,000 device-scope
// atomics on each word of one line (bicycle, 1M Gaussians) took k_preprocess
// from 65 to 373 us.  Device-scope atomics resolve past the XCDs' L2s, and
// those on one address are serialized there.
constexpr int kDsShards = 64, kDsShardWords = 64;
// bytes of the depth-order state (fixed layout at the start of a workspace)
constexpr size_t kDsShardOff =  // dstate, bcount, bsum, the block totals (scratch), then the shards
    ((kDsWords * 4 + (size_t)kDsNBMax * (4 + 8) + (size_t)(kDsNBMax / 1024) * (4 + 8)) + 255) / 256 * 256;
constexpr size_t kDsStateBytes = kDsShardOff + (size_t)kDsShards * kDsShardWords * 4;

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
  unsigned* btc;               // [kDsNBMax / kDsBlk] block totals of the counts
  unsigned long long* bts;     // [kDsNBMax / kDsBlk] ... of the tiles-word sums
  unsigned* shard;             // [kDsShards][kDsShardWords] min / max shards (zero when idle)
};

__device__ __forceinline__ int ds_log2(int nb) { return 31 - __clz(nb); }

// The pair counts to the host (pinned, coherent; the host spins on pub[0]):
// pub[3] = a bucket above kDsSmall exists, pub[2] = the overflow flag, pub[1]
// = num_rendered, then pub[0] = K.  The
// depth order publishes them itself as soon as they are known -- the bucket
// form from k_dsort_scan2 (the total of the tiles words), before its scatter
// and in-bucket sorts run, the LSD form from the last element of its scan --
// so the host queues the post-count launches while the order is finished.
__device__ __forceinline__ void ds_publish(unsigned* pub, unsigned long long v, unsigned over, unsigned big = 1u) {
  __hip_atomic_store(pub + 3, big, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(pub + 2, over, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(pub + 1, (unsigned)(v >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(pub, (unsigned)v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the bucket map: lo and shift from the shards, by one whole wave (lane l
// reads shard l; every lane gets the result)
__device__ __forceinline__ void ds_range_wave(const unsigned* shard, int nb, unsigned& lo, int& shift) {
  const int lane = threadIdx.x & 63;
  unsigned nlo = __hip_atomic_load(shard + lane * kDsShardWords, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned hi = __hip_atomic_load(shard + lane * kDsShardWords + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    nlo = max(nlo, (unsigned)__shfl_xor((int)nlo, o));
    hi = max(hi, (unsigned)__shfl_xor((int)hi, o));
  }
  lo = ~nlo;
  const unsigned span = hi >= lo ? hi - lo : 0u;
  const int nbits = span ? 32 - __clz(span) : 0;
  shift = max(0, nbits - ds_log2(nb));
}

// k_preprocess's contribution: min / max of the visible depth bits, reduced
// over the workgroup (shuffles, then LDS), one atomic pair per workgroup into
// shard blockIdx mod 64.  Every thread of the workgroup calls it.
__device__ __forceinline__ void ds_minmax(unsigned* shard, bool vis, unsigned bits) {
  __shared__ unsigned s_mm[2][8];
  unsigned nlo = vis ? ~bits : 0u, hi = vis ? bits : 0u;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    nlo = max(nlo, (unsigned)__shfl_xor((int)nlo, o));
    hi = max(hi, (unsigned)__shfl_xor((int)hi, o));
  }
  const int nw = (int)(blockDim.x >> 6), wv = (int)(threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0) {
    s_mm[0][wv] = nlo;
    s_mm[1][wv] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < nw; ++w) {
      nlo = max(nlo, s_mm[0][w]);
      hi = max(hi, s_mm[1][w]);
    }
    if (hi != 0u) {
      unsigned* sh = shard + (blockIdx.x & (kDsShards - 1)) * kDsShardWords;
      __hip_atomic_fetch_max(sh, nlo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_max(sh + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ __launch_bounds__(256) void k_dsort_hist(int P, int nb, const float* __restrict__ depth,
                                                    const unsigned long long* __restrict__ tiles, DsortBufs d) {
  __shared__ unsigned s_lo;
  __shared__ int s_shift;
  if (threadIdx.x < 64) {
    unsigned lo;
    int shift;
    ds_range_wave(d.shard, nb, lo, shift);
    if (threadIdx.x == 0) {
      s_lo = lo;
      s_shift = shift;
    }
  }
  __syncthreads();
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= P) return;
  const unsigned long long tw = tiles[i];
  if (tw == 0ull) return;  // culled (k_preprocess wrote no depth)
  const unsigned b = (__float_as_uint(depth[i]) - s_lo) >> s_shift;
  __hip_atomic_fetch_add(d.bcount + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_add(d.bsum + b, tw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Exclusive scans of the bucket counts and tiles-word sums over the nb
// buckets, in two launches of nb / 1,024 workgroups (a block of 1,024 buckets
// each, 4 per lane, coalesced): k_dsort_scan1 writes every block's totals,
// k_dsort_scan2 adds the totals of the blocks before its own (<= 64 values)
// to its block's scan and lists the occupied buckets (one list reservation
// per workgroup).  Round 4's first form scanned in one workgroup and cost
// ~50 us on the lego frame (latency-bound passes over 16k buckets).
constexpr int kDsBlk = 1024;
__device__ __forceinline__ unsigned ds_block_sum_u32(unsigned v, unsigned* s_tmp) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (unsigned)__shfl_xor((int)v, o);
  if ((threadIdx.x & 63) == 0) s_tmp[threadIdx.x >> 6] = v;
  __syncthreads();
  v = s_tmp[0] + s_tmp[1] + s_tmp[2] + s_tmp[3];
  __syncthreads();
  return v;
}
__device__ __forceinline__ unsigned long long ds_block_sum_u64(unsigned long long v, unsigned long long* s_tmp) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) s_tmp[threadIdx.x >> 6] = v;
  __syncthreads();
  v = s_tmp[0] + s_tmp[1] + s_tmp[2] + s_tmp[3];
  __syncthreads();
  return v;
}
__global__ __launch_bounds__(256) void k_dsort_scan1(DsortBufs d, unsigned* __restrict__ btc,
                                                     unsigned long long* __restrict__ bts) {
  __shared__ unsigned s_c[4];
  __shared__ unsigned long long s_s[4];
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // the list counters k_dsort_scan2 reserves from
    d.st[DS_NLIST] = 0;
    d.st[DS_NBIG] = 0;
    d.st[DS_MAXN] = 0;
  }
  const int b = blockIdx.x * kDsBlk + 4 * threadIdx.x;
  const uint4 c4 = *reinterpret_cast<const uint4*>(d.bcount + b);
  // a bucket above kDsBig: the flag k_dsort_scan2 publishes (zero here: k_dsort_scatter resets it)
  const unsigned cmax = max(max(c4.x, c4.y), max(c4.z, c4.w));
  if (cmax > (unsigned)kDsBig) d.st[DS_OVER] = 1u;
  if (cmax > (unsigned)kDsSmall) d.st[DS_BIGANY] = 1u;  // the host skips k_dsort_big without it
  const ulonglong2 s01 = *reinterpret_cast<const ulonglong2*>(d.bsum + b);
  const ulonglong2 s23 = *reinterpret_cast<const ulonglong2*>(d.bsum + b + 2);
  const unsigned c = ds_block_sum_u32(c4.x + c4.y + c4.z + c4.w, s_c);
  const unsigned long long sm = ds_block_sum_u64(s01.x + s01.y + s23.x + s23.y, s_s);
  if (threadIdx.x == 0) {
    btc[blockIdx.x] = c;
    bts[blockIdx.x] = sm;
  }
}
__global__ __launch_bounds__(256) void k_dsort_scan2(int nb, DsortBufs d, const unsigned* __restrict__ btc,
                                                     const unsigned long long* __restrict__ bts,
                                                     unsigned* __restrict__ pub) {
  __shared__ unsigned s_c[4], s_f[4], s_wf[4], s_base[2];
  __shared__ unsigned long long s_s[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, g = blockIdx.x, ng = nb / kDsBlk;
  // the totals of the blocks before this one (and of all, for the last block)
  unsigned pc = 0, ac = 0;
  unsigned long long ps = 0, as = 0;
  for (int q = lane; q < ng; q += 64) {  // every wave alike: no LDS needed
    const unsigned xc = btc[q];
    const unsigned long long xs = bts[q];
    if (q < g) {
      pc += xc;
      ps += xs;
    }
    ac += xc;
    as += xs;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    pc += (unsigned)__shfl_xor((int)pc, o);
    ac += (unsigned)__shfl_xor((int)ac, o);
    ps += __shfl_xor(ps, o);
    as += __shfl_xor(as, o);
  }
  const int b = g * kDsBlk + 4 * t;
  const uint4 c4 = *reinterpret_cast<const uint4*>(d.bcount + b);
  const ulonglong2 s01 = *reinterpret_cast<const ulonglong2*>(d.bsum + b);
  const ulonglong2 s23 = *reinterpret_cast<const ulonglong2*>(d.bsum + b + 2);
  const unsigned n[4] = {c4.x, c4.y, c4.z, c4.w};
  const unsigned long long sm[4] = {s01.x, s01.y, s23.x, s23.y};
  unsigned lc = n[0] + n[1] + n[2] + n[3];
  unsigned long long ls = sm[0] + sm[1] + sm[2] + sm[3];
  unsigned fl = (n[0] != 0) + (n[1] != 0) + (n[2] != 0) + (n[3] != 0);  // occupied small
  unsigned fb = 0, mx = max(max(n[0], n[1]), max(n[2], n[3]));
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    fl -= n[q] > (unsigned)kDsSmall ? 1u : 0u;
    fb += n[q] > (unsigned)kDsSmall ? 1u : 0u;
  }
  // workgroup exclusive scans of (count, sum, small flags, big flags)
  unsigned ic = lc, ifl = fl, ifb = fb;
  unsigned long long is = ls;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned uc = (unsigned)__shfl_up((int)ic, o), uf = (unsigned)__shfl_up((int)ifl, o),
                   ub = (unsigned)__shfl_up((int)ifb, o);
    const unsigned long long us = __shfl_up(is, o);
    if (lane >= o) {
      ic += uc;
      ifl += uf;
      ifb += ub;
      is += us;
    }
  }
  if (lane == 63) {
    s_c[wv] = ic;
    s_s[wv] = is;
    s_f[wv] = ifl;
    s_wf[wv] = ifb;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, (unsigned)__shfl_xor((int)mx, o));
  __syncthreads();
  unsigned wc = 0, wfl = 0, wfb = 0, tfl = 0, tfb = 0;
  unsigned long long ws = 0;
  for (int q = 0; q < 4; ++q) {
    if (q < wv) {
      wc += s_c[q];
      ws += s_s[q];
      wfl += s_f[q];
      wfb += s_wf[q];
    }
    tfl += s_f[q];
    tfb += s_wf[q];
  }
  if (t == 0) {
    s_base[0] = tfl ? atomicAdd(d.st + DS_NLIST, tfl) : 0u;
    s_base[1] = tfb ? atomicAdd(d.st + DS_NBIG, tfb) : 0u;
  }
  if (lane == 0 && mx) atomicMax(d.st + DS_MAXN, mx);
  __syncthreads();
  unsigned run = pc + wc + ic - lc;
  unsigned long long pre = ps + ws + is - ls;
  unsigned li = s_base[0] + wfl + ifl - fl, bi = s_base[1] + wfb + ifb - fb;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (n[q]) {
      const int bb = b + q;
      d.bbase[bb] = run;
      d.bcur[bb] = run;
      d.bpre[bb] = pre;
      if (n[q] <= (unsigned)kDsSmall) {
        d.blist[li++] = (unsigned)bb;
      } else {
        d.bbig[bi++] = (unsigned)bb;
      }
      run += n[q];
      pre += sm[q];
    }
  }
  if (g == ng - 1 && wv == 0) {
    unsigned lo;
    int shift;
    ds_range_wave(d.shard, nb, lo, shift);
    if (lane == 0) {
      d.st[DS_LO] = lo;
      d.st[DS_SHIFT] = (unsigned)shift;
      d.st[DS_NB] = (unsigned)nb;
      d.st[DS_PV] = ac;
      d.st[DS_CULL] = 0;
      d.st[DS_TOT] = (unsigned)as;
      d.st[DS_TOT + 1] = (unsigned)(as >> 32);
      const unsigned over = d.st[DS_OVER];
      d.st[DS_OVERD] = over;
      if (pub) ds_publish(pub, as, over, d.st[DS_BIGANY]);  // K and num_rendered: the total of the tiles words
    }
  }
}

__global__ __launch_bounds__(256) void k_dsort_scatter(int P, const float* __restrict__ depth,
                                                       const unsigned long long* __restrict__ tiles, DsortBufs d,
                                                       unsigned* __restrict__ order,
                                                       unsigned long long* __restrict__ offr) {
  if (blockIdx.x == 0 && threadIdx.x < 2 * kDsShards)  // the shards: read for the last time by k_dsort_scan2
    d.shard[(threadIdx.x >> 1) * kDsShardWords + (threadIdx.x & 1)] = 0u;
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // published by k_dsort_scan2
    d.st[DS_OVER] = 0u;
    d.st[DS_BIGANY] = 0u;
  }
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

// ---------------------------------------------------------------------------
// The LSD form of the depth order (the default above kDlMin Gaussians; the
// bucket form's histogram and scatter take a device-scope atomic per
// Gaussian, which resolves past the XCDs' L2s: 87 + 71 us for bicycle's 1M).
//
// Keys: key = bits - lo for a visible Gaussian (lo: the smallest visible
// depth bits, from the shards), all ones for a culled one.  A stable LSD sort
// over 8-bit digits from index order gives exactly the (bits, index) order,
// culled ones last.  Only R = ceil(nb1 / 8) passes can move anything, nb1 the
// bit length of (span + 1): every visible key is then below 2^(8R) - 1, the
// low 8R bits of a culled key, so after R passes the order is final and the
// remaining passes are identities.  The host launches all 4 passes (it does
// not know the span); a pass at or beyond R returns at once, and the final
// scan reads the buffer the last real pass wrote.  Each pass is
// reduce-then-scan without look-back or atomics on global memory:
//   k_dl_hist     per 2,048-key chunk its 256 digit counts (LDS), digit-major
//   k_dl_rows     a wave per digit: the chunk prefix of that digit + its total
//   k_dl_scatter  per chunk: wave-ballot digit ranks (in order: stable), the
//                 chunk staged sorted in LDS, striped coalesced stores
// Pass 0 reads the depth bits and tiles words itself (no key-building pass).
// Then k_dl_scan_blocks / k_dl_scan_apply: the inclusive scan of the tiles
// words in that order (gathered through it), writing the order and offr.
constexpr int kDlI = 8, kDlChunk = 256 * kDlI, kDlPasses = 4;
constexpr int kDlMin = 262144;  // below: the bucket form
enum : int { DS_DL_LO = 27, DS_DL_NB1 = 28 };

struct DlBufs {
  unsigned* st;
  unsigned* shard;
  unsigned *k0, *v0, *k1, *v1;  // pass p writes (k, v)[p & 1]
  unsigned *H, *Hs, *tot;       // [256][nch] digit-major counts, their row prefixes, [256] digit totals
};

// lo and nb1 from the shards, by one whole wave
__device__ __forceinline__ void dl_span_wave(const unsigned* shard, unsigned& lo, int& nb1) {
  const int lane = threadIdx.x & 63;
  unsigned nlo = __hip_atomic_load(shard + lane * kDsShardWords, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned hi = __hip_atomic_load(shard + lane * kDsShardWords + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    nlo = max(nlo, (unsigned)__shfl_xor((int)nlo, o));
    hi = max(hi, (unsigned)__shfl_xor((int)hi, o));
  }
  lo = ~nlo;
  const unsigned span = hi >= lo ? hi - lo : 0u;  // < 0x7F800000: span + 1 does not wrap
  nb1 = 32 - __clz(span + 1u);
}
__device__ __forceinline__ bool dl_trivial(const unsigned* st, int pass) {
  return pass > 0 && (unsigned)(8 * pass) >= st[DS_DL_NB1];
}
__device__ __forceinline__ unsigned dl_key0(const float* depth, const unsigned long long* tiles, int e,
                                            unsigned lo) {
  return tiles[e] ? __float_as_uint(depth[e]) - lo : 0xFFFFFFFFu;  // culled: no depth was written
}

// lo and nb1 of pass 0.  from_state: the overflow fallback of the bucket form
// (raster.hip), which has already read (and zeroed) the shards: lo from the
// state it left (DS_LO) and all four passes (nb1 = 32: any span fits)
__device__ __forceinline__ void dl_span0(const DlBufs& b, int from_state, unsigned& lo, int& nb1) {
  if (from_state) {
    lo = b.st[DS_LO];
    nb1 = 32;
  } else {
    dl_span_wave(b.shard, lo, nb1);
  }
}

template <bool FIRST>
__global__ __launch_bounds__(256) void k_dl_hist(int P, int nch, int pass, const float* __restrict__ depth,
                                                 const unsigned long long* __restrict__ tiles, DlBufs b,
                                                 int from_state) {
  __shared__ unsigned s_h[256];
  __shared__ unsigned s_lo;
  __shared__ int s_skip;
  const int t = threadIdx.x, c = blockIdx.x;
  s_h[t] = 0;
  if (FIRST) {
    if (t < 64) {
      unsigned lo;
      int nb1;
      dl_span0(b, from_state, lo, nb1);
      if (t == 0) s_lo = lo;
    }
  } else {
    if (t == 0) s_skip = dl_trivial(b.st, pass) ? 1 : 0;
    if (pass == 1 && c == 0 && t < 2 * kDsShards)  // idle state: pass 0 read the shards for the last time
      b.shard[(t >> 1) * kDsShardWords + (t & 1)] = 0u;
  }
  __syncthreads();
  if (!FIRST && s_skip) return;  // workgroup-uniform
  const unsigned* keys = (pass & 1) ? b.k0 : b.k1;
  const int sh = 8 * pass;
#pragma unroll
  for (int i = 0; i < kDlI; ++i) {
    const int e = c * kDlChunk + i * 256 + t;
    if (e < P) {
      const unsigned k = FIRST ? dl_key0(depth, tiles, e, s_lo) : keys[e];
      atomicAdd(&s_h[(k >> sh) & 255u], 1u);
    }
  }
  __syncthreads();
  b.H[(size_t)t * nch + c] = s_h[t];
}

// 64 workgroups of 4 waves: wave d = digit d's row
__global__ __launch_bounds__(256) void k_dl_rows(int nch, int pass, DlBufs b) {
  if (dl_trivial(b.st, pass)) return;
  const int d = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const unsigned* h = b.H + (size_t)d * nch;
  unsigned* o = b.Hs + (size_t)d * nch;
  unsigned carry = 0;
  for (int c0 = 0; c0 < nch; c0 += 64) {
    const int c = c0 + lane;
    const unsigned v = c < nch ? h[c] : 0u;
    unsigned inc = v;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
      const unsigned u = (unsigned)__shfl_up((int)inc, s);
      if (lane >= s) inc += u;
    }
    if (c < nch) o[c] = carry + inc - v;
    carry += (unsigned)__shfl((int)inc, 63);
  }
  if (lane == 0) b.tot[d] = carry;
}

template <bool FIRST>
__global__ __launch_bounds__(256) void k_dl_scatter(int P, int nch, int pass, const float* __restrict__ depth,
                                                    const unsigned long long* __restrict__ tiles, DlBufs b,
                                                    int from_state) {
  __shared__ unsigned s_k[kDlChunk], s_v[kDlChunk];
  __shared__ unsigned s_wrun[4][256];  // per wave: running count of each digit, then its offset
  __shared__ unsigned s_doff[256];     // chunk-local start of each digit's run
  __shared__ unsigned s_gbase[256];    // global position of this chunk's run of each digit
  __shared__ unsigned s_part[4][2];
  __shared__ unsigned s_lo;
  __shared__ int s_skip;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, c = blockIdx.x;
  if (FIRST) {
    if (t < 64) {
      unsigned lo;
      int nb1;
      dl_span0(b, from_state, lo, nb1);
      if (t == 0) {
        s_lo = lo;
        if (c == 0) {
          b.st[DS_DL_LO] = lo;
          b.st[DS_DL_NB1] = (unsigned)nb1;
        }
      }
    }
  } else if (t == 0) {
    s_skip = dl_trivial(b.st, pass) ? 1 : 0;
  }
#pragma unroll
  for (int w = 0; w < 4; ++w) s_wrun[w][t] = 0;
  __syncthreads();
  if (!FIRST && s_skip) return;  // workgroup-uniform
  const unsigned* keys = (pass & 1) ? b.k0 : b.k1;
  const unsigned* vals = (pass & 1) ? b.v0 : b.v1;
  unsigned* keys_out = (pass & 1) ? b.k1 : b.k0;
  unsigned* vals_out = (pass & 1) ? b.v1 : b.v0;
  const int sh = 8 * pass;
  // where each digit's run starts overall: exclusive scan of the 256 digit totals (thread t: digit t)
  const unsigned dt = b.tot[t];
  unsigned inc = dt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned u = (unsigned)__shfl_up((int)inc, o);
    if (lane >= o) inc += u;
  }
  if (lane == 63) s_part[wv][0] = inc;
  __syncthreads();
  unsigned dstart = inc - dt;
  for (int w = 0; w < wv; ++w) dstart += s_part[w][0];
  s_gbase[t] = dstart + b.Hs[(size_t)t * nch + c];
  // wave wv ranks keys [c * 2048 + wv * 512, +512) in 8 slots of 64, in order
  const int e0 = c * kDlChunk + wv * (kDlChunk / 4);
  unsigned k[kDlI], v[kDlI], r[kDlI];
#pragma unroll
  for (int j = 0; j < kDlI; ++j) {
    const int e = e0 + j * 64 + lane;
    if (FIRST) {
      k[j] = e < P ? dl_key0(depth, tiles, e, s_lo) : 0u;
      v[j] = (unsigned)e;
    } else {
      k[j] = e < P ? keys[e] : 0u;
      v[j] = e < P ? vals[e] : 0u;
    }
  }
  const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
  for (int j = 0; j < kDlI; ++j) {
    const bool ok = e0 + j * 64 + lane < P;
    const unsigned d = ok ? (k[j] >> sh) & 255u : 256u;
    unsigned long long peers = ~0ull;
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      const unsigned long long bal = __ballot((d >> q) & 1u);
      peers &= ((d >> q) & 1u) ? bal : ~bal;
    }
    const unsigned rk = (unsigned)__popcll(peers & below);
    const unsigned base = ok ? s_wrun[wv][d & 255u] : 0u;
    r[j] = base + rk;
    // the digit's lowest lane moves the count on; the wave's LDS operations
    // execute in order, so the next slot's read sees it
    if (ok && rk == 0) s_wrun[wv][d] = base + (unsigned)__popcll(peers);
  }
  __syncthreads();
  {  // thread t = digit t: the four waves' counts -> the run start and each wave's offset in it
    const unsigned c0 = s_wrun[0][t], c1 = s_wrun[1][t], c2 = s_wrun[2][t], c3 = s_wrun[3][t];
    const unsigned n = c0 + c1 + c2 + c3;
    unsigned inc2 = n;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned u = (unsigned)__shfl_up((int)inc2, o);
      if (lane >= o) inc2 += u;
    }
    if (lane == 63) s_part[wv][1] = inc2;
    __syncthreads();
    unsigned off = inc2 - n;
    for (int w = 0; w < wv; ++w) off += s_part[w][1];
    s_doff[t] = off;
    s_wrun[0][t] = off;
    s_wrun[1][t] = off + c0;
    s_wrun[2][t] = off + c0 + c1;
    s_wrun[3][t] = off + c0 + c1 + c2;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kDlI; ++j) {
    if (e0 + j * 64 + lane < P) {
      const unsigned idx = s_wrun[wv][(k[j] >> sh) & 255u] + r[j];
      s_k[idx] = k[j];
      s_v[idx] = v[j];
    }
  }
  __syncthreads();
  const int nv = min(kDlChunk, P - c * kDlChunk);
#pragma unroll
  for (int i = 0; i < kDlI; ++i) {  // striped: each digit run leaves as coalesced stores
    const int sp = i * 256 + t;
    if (sp < nv) {
      const unsigned kk = s_k[sp], d = (kk >> sh) & 255u;
      const unsigned pos = s_gbase[d] + (unsigned)sp - s_doff[d];
      keys_out[pos] = kk;
      vals_out[pos] = s_v[sp];
    }
  }
}

// the order the last real pass wrote
__device__ __forceinline__ const unsigned* dl_final(const DlBufs& b) {
  const int R = ((int)b.st[DS_DL_NB1] + 7) >> 3;
  return (R & 1) ? b.v0 : b.v1;
}
// the inclusive scan of the tiles words in that order (scan.h's two launches, gathered)
__global__ __launch_bounds__(256) void k_dl_scan_blocks(int P, const unsigned long long* __restrict__ tiles, DlBufs b,
                                                        unsigned long long* __restrict__ btot) {
  __shared__ unsigned long long s_w[4];
  const unsigned* ord = dl_final(b);
  const int i0 = blockIdx.x * kScanBlk + 4 * threadIdx.x;
  unsigned long long v = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (i0 + q < P) v += tiles[ord[i0 + q]];
  v = scan_block_sum(v, s_w);
  if (threadIdx.x == 0) btot[blockIdx.x] = v;
}
__global__ __launch_bounds__(256) void k_dl_scan_apply(int P, const unsigned long long* __restrict__ tiles, DlBufs b,
                                                       const unsigned long long* __restrict__ btot,
                                                       unsigned* __restrict__ order,
                                                       unsigned long long* __restrict__ offr,
                                                       unsigned* __restrict__ pub) {
  __shared__ unsigned long long s_w[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = blockIdx.x;
  const unsigned* ord = dl_final(b);
  unsigned long long pb = 0;
  for (int q = threadIdx.x; q < g; q += 256) pb += btot[q];
  pb = scan_block_sum(pb, s_w);
  const int i0 = g * kScanBlk + 4 * threadIdx.x;
  unsigned o[4];
  unsigned long long e[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    o[q] = i0 + q < P ? ord[i0 + q] : 0u;
    e[q] = i0 + q < P ? tiles[o[q]] : 0ull;
  }
  const unsigned long long lt = e[0] + e[1] + e[2] + e[3];
  unsigned long long inc = lt;
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const unsigned long long u = __shfl_up(inc, s);
    if (lane >= s) inc += u;
  }
  if (lane == 63) s_w[wv] = inc;
  __syncthreads();
  unsigned long long run = pb + inc - lt;
  for (int w = 0; w < wv; ++w) run += s_w[w];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    run += e[q];
    if (i0 + q < P) {
      order[i0 + q] = o[q];
      offr[i0 + q] = run;
      if (pub && i0 + q == P - 1) ds_publish(pub, run, 0u);  // the total: K, num_rendered
    }
  }
}

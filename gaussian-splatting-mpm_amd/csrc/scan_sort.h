// scan_sort.h -- hand-written single-pass device scan and LSD radix sort for
// the rasterizer (included by raster.hip inside namespace gsmpm).
//
// Both are chained ("decoupled look-back") single-pass algorithms in the form
// CDNA's 64-lane waves make cheap:
//
//   k_scan_u32   inclusive / exclusive sum of n u32.  A workgroup takes a
//                4096-element tile (256 lanes x 16, striped loads staged in
//                LDS), scans it (wave prefix sums + a cross-wave pass), then
//                publishes its aggregate and, once its predecessors' are
//                known, its inclusive prefix in one 64-bit status word per
//                tile: {epoch, flag, value}.  The epoch tags a call, so the
//                status array is never cleared.
//   k_rs_hist +  stable LSD radix sort of (u32 key, u32 value) pairs, 8-bit
//   k_rs_pass    digits: one histogram launch for every pass, then one launch
//                per digit (onesweep).  A workgroup ranks its 2048 items per
//                digit with wave ballots (the 8 digit-bit ballots give the
//                lanes holding the same digit; rank = popcount below the
//                lane), in (slot, wave, lane) order -- the items' own order
//                with striped loads -- then looks back per digit (lane d owns
//                digit d) for the items of that digit in earlier tiles and
//                scatters.  Stable, so the passes compose into the sort.
//
// Tiles are claimed through a ticket counter (atomicAdd), so a tile's
// predecessors have all started before it waits on them.  Every wait is
// bounded (~50 ms of s_memrealtime): on expiry the kernel raises *err and
// carries on, and the host turns that into an error instead of a hang.

constexpr int kScanT = 256, kScanI = 16, kScanTile = kScanT * kScanI;  // 4096 elements per scan tile
constexpr int kRsT = 256, kRsI = 8, kRsTile = kRsT * kRsI;              // 2048 pairs per sort tile
constexpr unsigned long long kLbFlagA = 1ull << 32, kLbFlagP = 2ull << 32;
constexpr unsigned long long kLbTimeout = 5000000ull;                   // 50 ms at 100 MHz

__device__ __forceinline__ unsigned long long lb_load(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long lb_word(unsigned epoch, unsigned long long flag, unsigned value) {
  return ((unsigned long long)epoch << 34) | flag | value;
}

// Exclusive prefix of tile `blk` for one chain (status[(blk - 1) * stride] ...):
// the predecessors' aggregates down to the nearest inclusive prefix, read
// kLbBatch words at a time (all tiles of a launch start together, so the
// nearest prefix is often many tiles back: one dependent load per tile cost
// ~0.7 us each).
constexpr int kLbBatch = 16;
__device__ __forceinline__ unsigned lookback(const unsigned long long* __restrict__ status, int blk, int stride,
                                             unsigned epoch, unsigned* __restrict__ err) {
  unsigned sum = 0;
  const unsigned ep = epoch & 0x3fffffffu;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  int p = blk - 1;
  while (p >= 0) {
    unsigned long long w[kLbBatch];
#pragma unroll
    for (int j = 0; j < kLbBatch; ++j) w[j] = p - j >= 0 ? lb_load(status + (size_t)(p - j) * stride) : 0ull;
    bool done = false, stalled = false;
#pragma unroll
    for (int j = 0; j < kLbBatch; ++j) {
      if (done || stalled || p < 0) continue;
      if ((unsigned)(w[j] >> 34) == ep && (w[j] & (3ull << 32))) {
        sum += (unsigned)w[j];
        if (w[j] & kLbFlagP) done = true;
        --p;
      } else {
        stalled = true;  // not published yet: reload from here
      }
    }
    if (done) break;
    if (stalled) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > kLbTimeout) {
        atomicOr(err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  return sum;
}

__device__ __forceinline__ unsigned wave_incl_sum(unsigned v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned y = __shfl_up(v, o);
    if (lane >= o) v += y;
  }
  return v;
}

// ------------------------------------------------------------------ scan --
__global__ __launch_bounds__(kScanT) void k_scan_u32(const unsigned* __restrict__ in, unsigned* __restrict__ out, int n,
                                                     int inclusive, unsigned long long* __restrict__ status,
                                                     unsigned* __restrict__ ticket, unsigned tbase, unsigned epoch,
                                                     unsigned* __restrict__ err) {
  __shared__ unsigned s_v[kScanTile];
  __shared__ unsigned s_w[kScanT / 64];
  __shared__ int s_blk;
  __shared__ unsigned s_prefix;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (t == 0) s_blk = (int)(atomicAdd(ticket, 1u) - tbase);
  __syncthreads();
  const int blk = s_blk;
  const size_t base = (size_t)blk * kScanTile;
  // striped (coalesced) loads staged in LDS, then each lane scans 16 consecutive elements
  unsigned v[kScanI];
#pragma unroll
  for (int u = 0; u < kScanI; ++u) {
    const size_t e = base + (size_t)u * kScanT + t;
    v[u] = e < (size_t)n ? in[e] : 0u;
  }
#pragma unroll
  for (int u = 0; u < kScanI; ++u) s_v[u * kScanT + t] = v[u];
  __syncthreads();
  unsigned run = 0;
#pragma unroll
  for (int u = 0; u < kScanI; ++u) {
    run += s_v[t * kScanI + u];
    v[u] = run;  // inclusive within the lane
  }
  const unsigned incl = wave_incl_sum(run);
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  unsigned wpre = 0, agg = 0;
#pragma unroll
  for (int w = 0; w < kScanT / 64; ++w) {
    wpre += w < wave ? s_w[w] : 0u;
    agg += s_w[w];
  }
  const unsigned lane_pre = wpre + incl - run;  // exclusive prefix of this lane's 16 within the tile
  if (t == 0) {
    unsigned prefix = 0;
    if (blk == 0) {
      lb_store(status, lb_word(epoch, kLbFlagP, agg));
    } else {
      lb_store(status + blk, lb_word(epoch, kLbFlagA, agg));
      prefix = lookback(status, blk, 1, epoch, err);
      lb_store(status + blk, lb_word(epoch, kLbFlagP, prefix + agg));
    }
    s_prefix = prefix;
  }
  __syncthreads();
  const unsigned pre = s_prefix + lane_pre;
#pragma unroll
  for (int u = 0; u < kScanI; ++u) {
    const unsigned x = s_v[t * kScanI + u];
    s_v[t * kScanI + u] = pre + (inclusive ? v[u] : v[u] - x);
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kScanI; ++u) {
    const size_t e = base + (size_t)u * kScanT + t;
    if (e < (size_t)n) out[e] = s_v[u * kScanT + t];
  }
}

// ------------------------------------------------------------------ sort --
// hist[pass][256]: digit counts of every pass (zeroed by the caller)
__global__ __launch_bounds__(kRsT) void k_rs_hist(const unsigned* __restrict__ keys, int n, int npass,
                                                  unsigned* __restrict__ hist) {
  __shared__ unsigned s_h[4][256];
  const int t = threadIdx.x;
  for (int p = 0; p < 4; ++p) s_h[p][t] = 0;
  __syncthreads();
  for (size_t e = (size_t)blockIdx.x * kRsTile + t; e < (size_t)min((size_t)n, (size_t)(blockIdx.x + 1) * kRsTile);
       e += kRsT) {
    const unsigned k = keys[e];
    for (int p = 0; p < npass; ++p) atomicAdd(&s_h[p][(k >> (8 * p)) & 255u], 1u);
  }
  __syncthreads();
  for (int p = 0; p < npass; ++p)
    if (s_h[p][t]) atomicAdd(&hist[p * 256 + t], s_h[p][t]);
}

// One stable 8-bit digit pass (digit = (key >> shift) & 255).  vals_in null:
// the values are the item indices (counting iterator).
__global__ __launch_bounds__(kRsT) void k_rs_pass(const unsigned* __restrict__ keys_in, const unsigned* __restrict__ vals_in,
                                                  unsigned* __restrict__ keys_out, unsigned* __restrict__ vals_out, int n,
                                                  int shift, const unsigned* __restrict__ hist,
                                                  unsigned long long* __restrict__ status, unsigned* __restrict__ ticket,
                                                  unsigned tbase, unsigned epoch, unsigned* __restrict__ err) {
  __shared__ unsigned s_run[256];        // items of each digit in earlier slots of this tile
  __shared__ unsigned s_wc[kRsT / 64][256];
  __shared__ unsigned s_gbase[256];      // global position of the digit's first item of this tile
  __shared__ int s_blk;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (t == 0) s_blk = (int)(atomicAdd(ticket, 1u) - tbase);
  s_run[t] = 0;
#pragma unroll
  for (int w = 0; w < kRsT / 64; ++w) s_wc[w][t] = 0;
  __syncthreads();
  const int blk = s_blk;
  const size_t base = (size_t)blk * kRsTile;
  unsigned k[kRsI], v[kRsI], d[kRsI], rank[kRsI];
#pragma unroll
  for (int u = 0; u < kRsI; ++u) {  // striped: item u * 256 + t of the tile
    const size_t e = base + (size_t)u * kRsT + t;
    const bool ok = e < (size_t)n;
    k[u] = ok ? keys_in[e] : 0u;
    v[u] = ok ? (vals_in ? vals_in[e] : (unsigned)e) : 0u;
    d[u] = ok ? (k[u] >> shift) & 255u : 256u;  // 256: no item
  }
  // a digit every item shares leaves the order as it is: copy (every tile
  // decides alike from the pass histogram; no ranking, no look-back)
  __shared__ int s_trivial;
  if (t == 0) s_trivial = 0;
  __syncthreads();
  if (hist[t] == (unsigned)n) s_trivial = 1;
  __syncthreads();
  if (s_trivial) {
#pragma unroll
    for (int u = 0; u < kRsI; ++u) {
      const size_t e = base + (size_t)u * kRsT + t;
      if (e < (size_t)n) {
        keys_out[e] = k[u];
        vals_out[e] = v[u];
      }
    }
    return;
  }
  const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
  for (int u = 0; u < kRsI; ++u) {
    // lanes of this wave holding the same digit (bit 8 set for "no item")
    unsigned long long peers = ~0ull;
#pragma unroll
    for (int b = 0; b < 9; ++b) {
      const unsigned long long bal = __ballot((d[u] >> b) & 1u);
      peers &= ((d[u] >> b) & 1u) ? bal : ~bal;
    }
    const unsigned r = (unsigned)__popcll(peers & below);
    if (d[u] < 256u && r == 0) s_wc[wave][d[u]] = (unsigned)__popcll(peers);
    __syncthreads();
    if (d[u] < 256u) {
      unsigned off = s_run[d[u]];
      for (int w = 0; w < wave; ++w) off += s_wc[w][d[u]];
      rank[u] = off + r;
    }
    __syncthreads();
    {  // lane t owns digit t: fold this slot's counts in, clear them
      unsigned c = 0;
#pragma unroll
      for (int w = 0; w < kRsT / 64; ++w) {
        c += s_wc[w][t];
        s_wc[w][t] = 0;
      }
      s_run[t] += c;
    }
    __syncthreads();
  }
  // digit t of this tile: publish its count, look back over earlier tiles
  {
    const unsigned cnt = s_run[t];
    unsigned long long* st = status + t;  // status[tile][256]
    unsigned prefix = 0;
    if (blk == 0) {
      lb_store(st, lb_word(epoch, kLbFlagP, cnt));
    } else {
      lb_store(st + (size_t)blk * 256, lb_word(epoch, kLbFlagA, cnt));
      prefix = lookback(st, blk, 256, epoch, err);
      lb_store(st + (size_t)blk * 256, lb_word(epoch, kLbFlagP, prefix + cnt));
    }
    // exclusive scan of the pass histogram: where digit t starts overall
    const unsigned hv = hist[t];
    const unsigned hi = wave_incl_sum(hv);
    __shared__ unsigned s_hw[kRsT / 64];
    if (lane == 63) s_hw[wave] = hi;
    __syncthreads();
    unsigned hpre = hi - hv;
    for (int w = 0; w < wave; ++w) hpre += s_hw[w];
    s_gbase[t] = hpre + prefix;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kRsI; ++u) {
    if (d[u] < 256u) {
      const unsigned pos = s_gbase[d[u]] + rank[u];
      keys_out[pos] = k[u];
      vals_out[pos] = v[u];
    }
  }
}

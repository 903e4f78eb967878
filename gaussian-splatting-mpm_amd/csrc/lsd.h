// lsd.h -- row scans and a stable LSD radix sort of (u32 key, u32 value)
// pairs by 8-bit digits, hand-written (included by raster.hip and mpm.hip
// inside namespace gsmpm; the kernels are static: each library object keeps
// its own copy).  The rasterizer sorts its (Gaussian, tile) pairs by tile with
// it above 4,096 tiles; the simulator sorts particles by their Morton code
// (resort) with it.
#pragma once

// The chunk histograms' positions, without a device-wide scan: a wave per
// tile row (H is tile-major, [tile][chunk]) writes the row's exclusive prefix
// (the chunk's offset inside the tile's run) into Hs and the row total into
// tot[tile]; k_tile_scatter's workgroups each scan the <= 4,097 totals in LDS
// (redundantly: cheaper than one more launch and a look-back chain).
static __global__ __launch_bounds__(256) void k_tile_rows(int ntiles, int nch, const unsigned* __restrict__ H,
                                                   unsigned* __restrict__ Hs, unsigned* __restrict__ tot) {
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (t > ntiles) return;  // wave-uniform
  const unsigned* h = H + (size_t)t * nch;
  unsigned* o = Hs + (size_t)t * nch;
  unsigned carry = 0;
  for (int c0 = 0; c0 < nch; c0 += 64) {
    const int c = c0 + lane;
    const unsigned v = c < nch ? h[c] : 0u;
    unsigned inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned u = (unsigned)__shfl_up((int)inc, d);
      if (lane >= d) inc += u;
    }
    if (c < nch) o[c] = carry + inc - v;
    carry += (unsigned)__shfl((int)inc, 63);
  }
  if (lane == 0) tot[t] = carry;
}

// The same row prefixes for long rows (many chunks): a workgroup per row.
// The row is read into LDS with coalesced loads, each thread scans a
// contiguous segment of it, the 256 segment sums are scanned across the
// workgroup, and the prefixes leave with coalesced stores.  k_tile_rows' wave
// walks a row of 7,275 chunks (bicycle's 29.8M pairs) in 114 dependent steps:
// 63.5 us per digit pass.  skip (optional): the row pass is a no-op when
// *skip <= skip_at (the LSD depth order's passes past the span, dsort.h).
constexpr int kRowsWideMin = 512, kRowsWideMax = 16000;  // chunks (dynamic LDS: 4 B each, under 64 KB with s_w)
static __global__ __launch_bounds__(256) void k_rows_wide(int nch, const unsigned* __restrict__ H,
                                                   unsigned* __restrict__ Hs, unsigned* __restrict__ tot,
                                                   const unsigned* __restrict__ skip, unsigned skip_at) {
  extern __shared__ unsigned s_row[];
  __shared__ unsigned s_w[4];
  if (skip && *skip <= skip_at) return;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const unsigned* h = H + (size_t)blockIdx.x * nch;
  unsigned* o = Hs + (size_t)blockIdx.x * nch;
  for (int c = t; c < nch; c += 1024) {
    unsigned v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = c + 256 * q < nch ? h[c + 256 * q] : 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (c + 256 * q < nch) s_row[c + 256 * q] = v[q];
  }
  __syncthreads();
  const int S = (nch + 255) / 256, c0 = min(nch, t * S), c1 = min(nch, c0 + S);
  unsigned sum = 0;
  for (int c = c0; c < c1; ++c) sum += s_row[c];
  unsigned inc = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned u = (unsigned)__shfl_up((int)inc, d);
    if (lane >= d) inc += u;
  }
  if (lane == 63) s_w[wv] = inc;
  __syncthreads();
  unsigned run = inc - sum;
  for (int w = 0; w < wv; ++w) run += s_w[w];
  for (int c = c0; c < c1; ++c) {
    const unsigned v = s_row[c];
    s_row[c] = run;
    run += v;
  }
  __syncthreads();
  for (int c = t; c < nch; c += 256) o[c] = s_row[c];
  if (t == 0) tot[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

// Above kMaxTiles tiles: a stable LSD radix sort over 8-bit digits of the
// tile index (two passes up to 65,535 tiles, three above), each pass
// reduce-then-scan with no look-back chain and no library call:
//   k_lsd_hist     per 4,096-pair chunk, its 256 digit counts (LDS atomics),
//                  stored digit-major H[d][chunk]
//   k_tile_rows    (256 rows) each digit's row prefix over the chunks + totals
//   k_lsd_scatter  per chunk: every wave ranks its 1,024 pairs (16 slots of
//                  64, in order) by digit with 8 ballots per slot and a
//                  wave-private running count per digit -- no barrier between
//                  slots; the four waves' counts then give each pair its
//                  chunk-local sorted index; the chunk is staged sorted in LDS
//                  and stored striped, so each digit run leaves as coalesced
//                  stores at digit start + the run's row prefix.
// Stable: a pair's rank follows (wave, slot, lane) = its chunk order.  Culled
// keys (tile field all ones) carry digit 255 in every pass, so they sort after
// every real tile (ntiles <= 256^passes - 1).  Round 3's form (2,048-pair
// chunks, the library's block radix sort for the local ranks, the library's
// device scan) ran 1.41 ms per bicycle render against 1.31 with the library's
// onesweep.
// I: keys per thread (chunk = 256 I); 16 by default (the simulator's
// re-sort).  The rasterizer's tile sort takes 32: 8,192-pair chunks, digit
// runs of 32 pairs on average instead of 16 (128-byte store runs), half the
// chunk histograms, 2 workgroups per CU (68 KB of LDS); GSMPM_RASTER_LSD_I=16
// restores 16 there (A/B).
constexpr int kLsdT = 256, kLsdI = 16, kLsdChunk = kLsdT * kLsdI;
template <int I = kLsdI>
static __global__ __launch_bounds__(kLsdT) void k_lsd_hist(int K, int nch, int shift, const unsigned* __restrict__ keys,
                                                    unsigned* __restrict__ H) {
  constexpr int kChunkI = kLsdT * I;
  __shared__ unsigned s_h[256];
  s_h[threadIdx.x] = 0;
  __syncthreads();
  const int c = blockIdx.x;
  unsigned k[I];
#pragma unroll
  for (int i = 0; i < I; ++i) {
    const int e = c * kChunkI + i * kLsdT + threadIdx.x;
    k[i] = e < K ? keys[e] : 0u;
  }
#pragma unroll
  for (int i = 0; i < I; ++i)
    if (c * kChunkI + i * kLsdT + (int)threadIdx.x < K) atomicAdd(&s_h[(k[i] >> shift) & 255u], 1u);
  __syncthreads();
  H[(size_t)threadIdx.x * nch + c] = s_h[threadIdx.x];
}
template <int I = kLsdI>
static __global__ __launch_bounds__(kLsdT) void k_lsd_scatter(int K, int nch, int shift, const unsigned* __restrict__ keys,
                                                       const unsigned* __restrict__ vals,
                                                       const unsigned* __restrict__ Hs, const unsigned* __restrict__ tot,
                                                       unsigned* __restrict__ keys_out,
                                                       unsigned* __restrict__ vals_out) {
  constexpr int kChunkI = kLsdT * I;
  __shared__ unsigned s_k[kChunkI], s_v[kChunkI];
  __shared__ unsigned s_wrun[4][256];  // per wave: running count of each digit, then its offset
  __shared__ unsigned s_doff[256];     // chunk-local start of each digit's run
  __shared__ unsigned s_gbase[256];    // global position of this chunk's run of each digit
  __shared__ unsigned s_part[4][2];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, c = blockIdx.x;
#pragma unroll
  for (int w = 0; w < 4; ++w) s_wrun[w][t] = 0;
  // where each digit's run starts overall: exclusive scan of the 256 digit totals (thread t: digit t)
  const unsigned dt = tot[t];
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
  s_gbase[t] = dstart + Hs[(size_t)t * nch + c];
  // wave wv ranks pairs [c * 256 I + wv * 64 I, + 64 I) in I slots of 64, in order
  const int e0 = c * kChunkI + wv * (kChunkI / 4);
  unsigned k[I], v[I], r[I];
#pragma unroll
  for (int j = 0; j < I; ++j) {
    const int e = e0 + j * 64 + lane;
    k[j] = e < K ? keys[e] : 0u;
    v[j] = e < K ? vals[e] : 0u;
  }
  const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
  for (int j = 0; j < I; ++j) {
    const bool ok = e0 + j * 64 + lane < K;
    const unsigned d = ok ? (k[j] >> shift) & 255u : 256u;
    unsigned long long peers = ~0ull;
#pragma unroll
    for (int b = 0; b < 9; ++b) {
      const unsigned long long bal = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? bal : ~bal;
    }
    const unsigned rk = (unsigned)__popcll(peers & below);
    const unsigned base = ok ? s_wrun[wv][d] : 0u;
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
  for (int j = 0; j < I; ++j) {
    if (e0 + j * 64 + lane < K) {
      const unsigned idx = s_wrun[wv][(k[j] >> shift) & 255u] + r[j];
      s_k[idx] = k[j];
      s_v[idx] = v[j];
    }
  }
  __syncthreads();
  const int nv = min(kChunkI, K - c * kChunkI);
#pragma unroll
  for (int i = 0; i < I; ++i) {  // striped: each digit run leaves as coalesced stores
    const int sp = i * kLsdT + t;
    if (sp < nv) {
      const unsigned kk = s_k[sp], d = (kk >> shift) & 255u;
      const unsigned pos = s_gbase[d] + (unsigned)sp - s_doff[d];
      keys_out[pos] = kk;
      vals_out[pos] = s_v[sp];
    }
  }
}


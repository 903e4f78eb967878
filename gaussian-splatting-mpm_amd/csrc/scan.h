// scan.h -- the rasterizer's index-order inclusive scans, hand-written
// (included by raster.hip inside namespace gsmpm, after dsort.h).
//
// Two launches of n / 1,024 workgroups, no look-back chain: k_scan_blocks
// writes each 1,024-element block's total; k_scan_apply scans its block (4
// consecutive elements a lane, wave scans, the 4 wave totals through LDS) and
// adds the totals of the blocks before it, which every workgroup sums for
// itself (<= n / 1,024 values, L2-resident).  Used for the tiles-touched
// offsets in Gaussian-index order: the backward's record slots (binned count,
// u32) and the upstream-keyed / per-tile-depth-sort emission (both counts,
// u64).

constexpr int kScanBlk = 1024;

// element i of the scanned sequence: the binned count (low word) or the whole tiles word
template <typename T>
__device__ __forceinline__ T scan_elem(const unsigned long long* __restrict__ tiles, int i, int n) {
  if (i >= n) return T(0);
  if constexpr (sizeof(T) == 4) return (T)(unsigned)tiles[i];
  else return (T)tiles[i];
}

template <typename T>
__device__ __forceinline__ T scan_block_sum(T v, T* s_w) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = v;
  __syncthreads();
  v = s_w[0] + s_w[1] + s_w[2] + s_w[3];
  __syncthreads();
  return v;
}

template <typename T>
__global__ __launch_bounds__(256) void k_scan_blocks(const unsigned long long* __restrict__ tiles, int n,
                                                     T* __restrict__ btot) {
  __shared__ T s_w[4];
  const int i0 = blockIdx.x * kScanBlk + 4 * threadIdx.x;
  T v = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) v += scan_elem<T>(tiles, i0 + q, n);
  v = scan_block_sum(v, s_w);
  if (threadIdx.x == 0) btot[blockIdx.x] = v;
}

template <typename T>
__global__ __launch_bounds__(256) void k_scan_apply(const unsigned long long* __restrict__ tiles, int n,
                                                    const T* __restrict__ btot, T* __restrict__ out) {
  __shared__ T s_w[4], s_pre;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = blockIdx.x;
  // the blocks before this one
  T pb = 0;
  for (int q = threadIdx.x; q < g; q += 256) pb += btot[q];
  pb = scan_block_sum(pb, s_w);
  const int i0 = g * kScanBlk + 4 * threadIdx.x;
  T e[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) e[q] = scan_elem<T>(tiles, i0 + q, n);
  const T lt = e[0] + e[1] + e[2] + e[3];
  T inc = lt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T u = __shfl_up(inc, o);
    if (lane >= o) inc += u;
  }
  if (lane == 63) s_w[wv] = inc;
  __syncthreads();
  T run = pb + inc - lt;
  for (int w = 0; w < wv; ++w) run += s_w[w];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    run += e[q];
    if (i0 + q < n) out[i0 + q] = run;
  }
  (void)s_pre;
}

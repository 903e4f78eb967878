// Micro-benchmark: the lane groups and banking of ds_add_u64 (k_fused's P2G
// scatter) and ds_read_b128 (its G2P gather) on gfx950.  Each pattern gives
// every lane of a wave a node index n(l); the wave issues ITERS instructions
// to u64 element n (or float4 element n), shifted uniformly by a multiple of
// 128 elements per iteration (the same banks).  Cycles per wave-instruction
// with 4 waves per CU tell which lanes share a conflict group:
//   distinct     n = l                                (conflict-free)
//   res16        n = l % 16 + 64 (l / 16)             (lanes l, l+16 on one bank pair)
//   res32        n = l % 32 + 64 (l / 32)             (lanes l, l+32 on one bank pair)
//   res16x       n = l % 16 + 64 (l / 16), lanes 16..31 and 32..47 swapped in pairs
//   bank0        n = 32 l                             (every lane on banks 0-1: the worst case)
//   same         n = 0                                (one address)
//   pairs        n = l / 2                            (two lanes per address)
//   group0       n = l, lanes 0..15 active only       (are idle lane groups free?)
//   half         n = l, lanes with l % 16 < 8 active  (half of every group)
// The reads are inline-asm ds_read_b128 in batches of 8 behind one
// lgkmcnt wait (a plain C++ load was hoisted out of the loop).
// Build: hipcc -O3 --offload-arch=gfx950 lds_banks.hip -o lds_banks
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int ITERS = 4096;
enum Pat { DISTINCT = 0, RES16, RES32, RES16X, BANK0, SAME, PAIRS, GROUP0, HALF, NPAT };
static const char* kName[NPAT] = {"distinct", "res16", "res32", "res16x", "bank0", "same", "pairs", "group0", "half"};

__device__ __forceinline__ unsigned node_of(int pat, unsigned l) {
  switch (pat) {
    case DISTINCT: return l;
    case RES16: return (l % 16) + 64 * (l / 16);
    case RES32: return (l % 32) + 64 * (l / 32);
    case RES16X: {
      const unsigned g = l / 16, r = l % 16;
      const unsigned gg = g == 1 ? 2 : g == 2 ? 1 : g;
      return r + 64 * gg;
    }
    case BANK0: return 32 * l;
    case SAME: return 0;
    case PAIRS: return l / 2;
    default: return l;
  }
}

template <int OP>  // 0: ds_add_u64 (returnless), 1: ds_read_b128
__global__ __launch_bounds__(256) void kern(int pat, unsigned long long* out, float* sink) {
  __shared__ __attribute__((aligned(16))) unsigned long long s[4096];  // 32 KB
  for (int i = threadIdx.x; i < 4096; i += 256) s[i] = 0ull;
  __syncthreads();
  const unsigned l = threadIdx.x & 63;
  const unsigned n = node_of(pat, l) & 2047u;
  const bool on = pat == GROUP0 ? l < 16 : pat == HALF ? (l % 16) < 8 : true;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (on) {
    if constexpr (OP == 0) {
      for (int it = 0; it < ITERS; ++it) {
        const unsigned sh = (unsigned)(it & 7) * 128u;
        __hip_atomic_fetch_add(&s[(n + sh) & 2047u], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    } else {
      const unsigned base = (unsigned)(uintptr_t)s;  // LDS byte address
      for (int it = 0; it < ITERS; it += 8) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const unsigned a = base + 16u * ((n + (unsigned)u * 128u) & 2047u);
          asm volatile("ds_read_b128 %0, %1" : "=v"(v[u]) : "v"(a));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          acc.x += v[u].x;
          acc.y += v[u].y;
          acc.z += v[u].z;
          acc.w += v[u].w;
        }
      }
    }
  }
  __syncthreads();
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (acc.x + acc.y + acc.z + acc.w == 12345.f) sink[threadIdx.x] = acc.x;
}

template <int OP>
static void run(int pat) {
  const int blocks = 256;
  unsigned long long* d;
  float* sink;
  (void)hipMalloc(&d, sizeof(unsigned long long) * blocks);
  (void)hipMalloc(&sink, 1024);
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, pat, d, sink);
  (void)hipDeviceSynchronize();
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, pat, d, sink);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks);
  (void)hipMemcpy(h.data(), d, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
  double avg = 0;
  for (auto v : h) avg += (double)v;
  avg /= blocks;
  // s_memtime: the shader clock (the existing lds_atomics ubench reads it as cycles)
  printf("%-14s %-9s cycles/wave-instr (4 waves/CU) %.2f\n", OP == 0 ? "ds_add_u64" : "ds_read_b128",
         kName[pat], avg / ITERS / 4.0);
  (void)hipFree(d);
  (void)hipFree(sink);
}

int main() {
  for (int p = 0; p < NPAT; ++p) run<0>(p);
  for (int p = 0; p < NPAT; ++p) run<1>(p);
  return 0;
}

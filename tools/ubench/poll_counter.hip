// Micro-benchmark: how a workgroup can see a device-scope counter that
// workgroups on other XCDs add to inside the same launch (k_fused's grid
// phase, fused.h FusedGrid).  G workgroups of k_fused's geometry (256 lanes,
// 50.7 KB LDS: 3 per CU) each spin a random short time, add 1 to the counter
// shard blockIdx & 7, then wait until the 8 shards sum to G, polling with one
// of several load forms.  Every spin is bounded (a timeout is counted, the
// launch still ends).  Reports per form: launches that timed out, and the
// average launch time over 50 launches (parity-alternating counters, zeroed
// for the next launch as FusedGrid does).
//   hipcc -O3 --offload-arch=gfx950 poll_counter.hip -o poll_counter && ./poll_counter
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHECK(x)                                                          \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                           \
    }                                                                     \
  } while (0)

constexpr int kLds = 12672;  // floats: 50.7 KB
constexpr int kStride = 32;

template <int M>
__device__ __forceinline__ unsigned poll1(unsigned* p) {
  unsigned v;
  if constexpr (M == 0) {
    v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if constexpr (M == 1) {
    v = __hip_atomic_fetch_add(p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if constexpr (M == 2) {
    asm volatile("global_load_dword %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  } else if constexpr (M == 3) {
    asm volatile("global_load_dword %0, %1, off sc0 sc1 nt\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  } else {
    v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  return v;
}

template <int M>
__global__ __launch_bounds__(256) void k_wait(unsigned* done, int par, int G, int* timeouts, float* sink, int seed) {
  __shared__ float s[kLds];
  __shared__ int ok;
  s[threadIdx.x] = (float)threadIdx.x;
  float a = s[(threadIdx.x * 7) & 255];
  const int work = ((blockIdx.x * 2654435761u + seed * 40503u) >> 20) & 1023;  // 0..1023 dependent FMAs
  for (int w = 0; w < work; ++w) a = __builtin_fmaf(a, 0.999f, 0.5f);
  if (blockIdx.x == 0 && threadIdx.x < 8) done[((par ^ 1) * 8 + threadIdx.x) * kStride] = 0u;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(done + (par * 8 + (blockIdx.x & 7)) * kStride, 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    const long long t0 = clock64();
    int good = 1;
    for (;;) {
      unsigned sum = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) sum += poll1<M>(done + (par * 8 + k) * kStride);
      if ((int)sum >= G) break;
      if (clock64() - t0 > (1LL << 25)) {
        good = 0;
        atomicAdd(timeouts, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    ok = good;
  }
  __syncthreads();
  if (a == -1.f || !ok) sink[blockIdx.x] = a;
}

int main() {
  int dev = 0, ncu = 0, per_cu = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_wait<0>, 256, 0));
  if (per_cu > 3) per_cu = 3;
  unsigned* done;
  int* timeouts;
  float* sink;
  CHECK(hipMalloc(&done, sizeof(unsigned) * 16 * kStride));
  CHECK(hipMalloc(&timeouts, sizeof(int)));
  CHECK(hipMalloc(&sink, sizeof(float) * 4096));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const char* names[5] = {"sc1 load (agent atomic load)", "returning atomic add 0", "sc0 sc1 load",
                          "sc0 sc1 nt load", "system-scope atomic load"};
  std::printf("CUs %d, workgroups per CU %d\n", ncu, per_cu);
  for (int G : {ncu * per_cu - 128, ncu * per_cu}) {
    for (int M = 0; M < 5; ++M) {
      CHECK(hipMemsetAsync(done, 0, sizeof(unsigned) * 16 * kStride, st));
      CHECK(hipMemsetAsync(timeouts, 0, sizeof(int), st));
      CHECK(hipEventRecord(e0, st));
      for (int it = 0; it < 50; ++it) {
        switch (M) {
          case 0: hipLaunchKernelGGL(k_wait<0>, dim3(G), dim3(256), 0, st, done, it & 1, G, timeouts, sink, it); break;
          case 1: hipLaunchKernelGGL(k_wait<1>, dim3(G), dim3(256), 0, st, done, it & 1, G, timeouts, sink, it); break;
          case 2: hipLaunchKernelGGL(k_wait<2>, dim3(G), dim3(256), 0, st, done, it & 1, G, timeouts, sink, it); break;
          case 3: hipLaunchKernelGGL(k_wait<3>, dim3(G), dim3(256), 0, st, done, it & 1, G, timeouts, sink, it); break;
          default: hipLaunchKernelGGL(k_wait<4>, dim3(G), dim3(256), 0, st, done, it & 1, G, timeouts, sink, it); break;
        }
      }
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(e1, st));
      CHECK(hipStreamSynchronize(st));
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      int to = 0;
      CHECK(hipMemcpy(&to, timeouts, sizeof(int), hipMemcpyDeviceToHost));
      std::printf("G %4d  %-30s  timed-out waits %5d   %.2f us per launch\n", G, names[M], to, ms * 1e3f / 50);
    }
  }
  return 0;
}

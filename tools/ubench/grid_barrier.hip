// Micro-benchmark: what a persistent substep kernel would pay per grid
// barrier, against the kernel boundary it would remove (DESIGN.md §3,
// "Rejected: a persistent k_fused + k_grid_f").
//
// Geometry of k_fused: 256-thread workgroups, 50.7 KB of LDS each (3 per CU),
// one workgroup per resident slot (3 x CUs).  Two barrier forms:
//   counter  one monotonic device counter, lane 0 of each workgroup adds
//            after a release fence and polls with relaxed agent loads
//   xcd      per-XCD counters (workgroup j is dispatched to XCD j mod 8);
//            the last arriver of an XCD adds to a top counter; the last
//            arriver there publishes the epoch to every XCD's word
// and the boundary: B dependent launches of the same empty grid, replayed
// from a hipGraph (what the simulator runs).  Every spin is bounded: a
// barrier that does not complete within ~0.2 s sets a flag and the kernel
// exits, so a mis-sized grid cannot hang the GPU.
//
//   hipcc -O3 --offload-arch=gfx950 grid_barrier.hip -o grid_barrier && ./grid_barrier
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                         \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

constexpr int kLdsFloats = 12672;  // 50.7 KB: three workgroups per CU, as k_fused
constexpr int kLine = 32;          // ints per 128-B line

struct Bar {
  unsigned* words;  // [0]: counter / top; [kLine * (1 + x)]: XCD x counter; [kLine * (9 + x)]: XCD x epoch
  int* timeout;
  int nwg;
  int per_xcd[8];
};

__device__ __forceinline__ bool spin_until(unsigned* p, unsigned target, int* timeout) {
  const long long t0 = clock64();
  while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    __builtin_amdgcn_s_sleep(1);
    if (clock64() - t0 > 400000000LL) {  // ~0.2 s at 2.4 GHz
      atomicExch(timeout, 1);
      return false;
    }
  }
  return true;
}

template <int MODE>
__device__ __forceinline__ bool grid_barrier(const Bar& b, unsigned epoch) {
  __syncthreads();
  bool ok = true;
  if (threadIdx.x == 0) {
    __atomic_thread_fence(__ATOMIC_RELEASE);  // agent scope: this workgroup's stores before the arrival
    if (MODE == 0) {
      atomicAdd(b.words, 1u);
      ok = spin_until(b.words, epoch * (unsigned)b.nwg, b.timeout);
    } else {
      const int x = blockIdx.x & 7;
      const unsigned old = atomicAdd(b.words + kLine * (1 + x), 1u);
      if (old + 1 == epoch * (unsigned)b.per_xcd[x]) {
        int nx = 0;
        for (int i = 0; i < 8; ++i) nx += b.per_xcd[i] > 0;
        const unsigned o2 = atomicAdd(b.words, 1u);
        if (o2 + 1 == epoch * (unsigned)nx)
          for (int i = 0; i < 8; ++i)
            __hip_atomic_store(b.words + kLine * (9 + i), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      ok = spin_until(b.words + kLine * (9 + x), epoch, b.timeout);
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
  }
  __syncthreads();
  return ok;
}

// iters barriers; `work` iterations of dependent FMAs per lane between them
template <int MODE>
__global__ __launch_bounds__(256) void k_barriers(Bar b, int iters, int work, float* sink) {
  __shared__ float s[kLdsFloats];
  s[threadIdx.x] = (float)threadIdx.x;
  float a = s[(threadIdx.x * 7) & 255];
  for (int it = 1; it <= iters; ++it) {
    for (int w = 0; w < work; ++w) a = __builtin_fmaf(a, 0.999f, 0.5f);
    if (!grid_barrier<MODE>(b, (unsigned)it)) break;
  }
  if (a == -1.f) sink[blockIdx.x] = a;
}

__global__ __launch_bounds__(256) void k_empty(int work, float* sink) {
  __shared__ float s[kLdsFloats];
  s[threadIdx.x] = (float)threadIdx.x;
  float a = s[(threadIdx.x * 7) & 255];
  for (int w = 0; w < work; ++w) a = __builtin_fmaf(a, 0.999f, 0.5f);
  if (a == -1.f) sink[blockIdx.x] = a;
}

int main() {
  int dev = 0, ncu = 0, per_cu = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_barriers<1>, 256, 0));
  int per_cu0 = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu0, k_barriers<0>, 256, 0));
  per_cu = per_cu < per_cu0 ? per_cu : per_cu0;
  if (per_cu > 3) per_cu = 3;  // the LDS allows three; never more than k_fused holds
  std::printf("CUs %d, workgroups per CU %d\n", ncu, per_cu);
  unsigned* words;
  int* timeout;
  float* sink;
  CHECK(hipMalloc(&words, sizeof(unsigned) * kLine * 20));
  CHECK(hipMalloc(&timeout, sizeof(int)));
  CHECK(hipMalloc(&sink, sizeof(float) * 4096));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int iters = 200;
  for (int wpc : {1, 2, 3}) {
    if (wpc > per_cu) break;
    const int nwg = ncu * wpc;
    Bar b{words, timeout, nwg, {0}};
    for (int j = 0; j < nwg; ++j) b.per_xcd[j & 7]++;
    for (int work : {0, 2000}) {
      for (int mode = 0; mode < 2; ++mode) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
          CHECK(hipMemsetAsync(words, 0, sizeof(unsigned) * kLine * 20, st));
          CHECK(hipMemsetAsync(timeout, 0, sizeof(int), st));
          CHECK(hipEventRecord(e0, st));
          if (mode == 0)
            hipLaunchKernelGGL(k_barriers<0>, dim3(nwg), dim3(256), 0, st, b, iters, work, sink);
          else
            hipLaunchKernelGGL(k_barriers<1>, dim3(nwg), dim3(256), 0, st, b, iters, work, sink);
          CHECK(hipGetLastError());
          CHECK(hipEventRecord(e1, st));
          CHECK(hipStreamSynchronize(st));
          int to = 0;
          CHECK(hipMemcpy(&to, timeout, sizeof(int), hipMemcpyDeviceToHost));
          if (to) {
            std::printf("barrier timed out (mode %d, %d WG/CU): not co-resident\n", mode, wpc);
            return 2;
          }
          float ms = 0.f;
          CHECK(hipEventElapsedTime(&ms, e0, e1));
          best = ms < best ? ms : best;
        }
        // the same work as back-to-back dependent launches from a graph
        float best_k = 1e30f;
        hipGraph_t g;
        hipGraphExec_t ge;
        CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
        for (int it = 0; it < iters; ++it) hipLaunchKernelGGL(k_empty, dim3(nwg), dim3(256), 0, st, work, sink);
        CHECK(hipStreamEndCapture(st, &g));
        CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int rep = 0; rep < 3; ++rep) {
          CHECK(hipEventRecord(e0, st));
          CHECK(hipGraphLaunch(ge, st));
          CHECK(hipEventRecord(e1, st));
          CHECK(hipStreamSynchronize(st));
          float ms = 0.f;
          CHECK(hipEventElapsedTime(&ms, e0, e1));
          best_k = ms < best_k ? ms : best_k;
        }
        CHECK(hipGraphExecDestroy(ge));
        CHECK(hipGraphDestroy(g));
        std::printf("%d WG/CU (%d WGs), %4d FMA/lane per phase: %-7s barrier %.2f us/phase | graph of launches %.2f "
                    "us/phase\n",
                    wpc, nwg, work, mode ? "xcd" : "counter", best * 1e3f / iters, best_k * 1e3f / iters);
      }
    }
  }
  return 0;
}

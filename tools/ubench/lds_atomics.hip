// Micro-benchmark: LDS atomic flavours on gfx950 (cycles per wave-instruction).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

enum Mode { ADD_F32 = 0, ADD_U32, ADD_F32_SAME, ADD_U32_SAME, WRITE_B32, ADD_F32_RTN, ADD_U64, ADD_F32_STRIDE16 };
constexpr int ITERS = 2048;

template <int MODE>
__global__ __launch_bounds__(256) void kern(unsigned long long* out, float val) {
  __shared__ __attribute__((aligned(16))) float s[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) s[i] = 0.f;
  __syncthreads();
  unsigned lane = threadIdx.x;
  unsigned addr = (lane * 2654435761u) >> 20;  // pseudo-random in [0, 4096)
  addr &= 4095u;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  float acc = 0.f;
  for (int it = 0; it < ITERS; ++it) {
    unsigned a = (addr + it * 97u) & 4095u;
    if constexpr (MODE == ADD_F32) __hip_atomic_fetch_add(&s[a], val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if constexpr (MODE == ADD_U32)
      __hip_atomic_fetch_add(reinterpret_cast<unsigned*>(&s[a]), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if constexpr (MODE == ADD_F32_SAME)
      __hip_atomic_fetch_add(&s[it & 4095], val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if constexpr (MODE == ADD_U32_SAME)
      __hip_atomic_fetch_add(reinterpret_cast<unsigned*>(&s[it & 4095]), 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    if constexpr (MODE == WRITE_B32) {
      s[a] = val + it;
      asm volatile("" ::: "memory");
    }
    if constexpr (MODE == ADD_F32_RTN)
      acc += __hip_atomic_fetch_add(&s[a], val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if constexpr (MODE == ADD_U64) atomicAdd(reinterpret_cast<unsigned long long*>(&s[a & ~1u]), 1ull);
    if constexpr (MODE == ADD_F32_STRIDE16)
      __hip_atomic_fetch_add(&s[((lane * 4u) + it * 256u) & 4095u], val, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (acc == 12345.f) out[blockIdx.x] = 0;
}

template <int MODE>
double run(const char* name) {
  const int blocks = 256;
  unsigned long long* d;
  hipMalloc(&d, sizeof(unsigned long long) * blocks);
  hipLaunchKernelGGL(kern<MODE>, dim3(blocks), dim3(256), 0, 0, d, 1.0f);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern<MODE>, dim3(blocks), dim3(256), 0, 0, d, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(blocks);
  hipMemcpy(h.data(), d, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
  double avg = 0;
  for (auto v : h) avg += v;
  avg /= blocks;
  // 4 waves per block issue ITERS instructions each; cycles per wave-instruction per CU
  printf("%-18s kernel %.3f ms  cycles/wave-instr (4 waves/CU) %.1f\n", name, ms, avg / ITERS / 4.0);
  hipFree(d);
  return avg;
}

int main() {
  run<WRITE_B32>("ds_write_b32");
  run<ADD_U32>("ds_add_u32 rand");
  run<ADD_U64>("ds_add_u64 rand");
  run<ADD_F32>("ds_add_f32 rand");
  run<ADD_F32_RTN>("ds_add_rtn_f32");
  run<ADD_F32_STRIDE16>("ds_add_f32 stride16");
  run<ADD_U32_SAME>("ds_add_u32 same");
  run<ADD_F32_SAME>("ds_add_f32 same");
  return 0;
}

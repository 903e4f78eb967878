// Micro-benchmark: what it costs k_fused's P2G half to hand its chunk window
// to the grid, in the lego frame's geometry (100k particles, 128^3, tiles of
// 8x8x7 cells: ~650 chunks of one round, 3 workgroups of 50.7 KB LDS per CU,
// each chunk's stencil box ~10x10x9 nodes, neighbouring boxes overlapping by
// 2 node layers per face as real tiles do).
//
//   slot_sc1     the shipped form: write-through float4 stores of the box to
//                the chunk's private slot (k_grid_f then sums <= 8 slots a node)
//   atom_f32_n4  global_atomic_add_f32 into a dense float4 (m v, m) grid, one
//                lane per node, its 4 channels in turn (4 instructions)
//   atom_f32_c1  the same, one lane per (node, channel): consecutive lanes
//                cover a z-run's 16-B nodes contiguously
//   atom_u64_c1  global 64-bit integer atomic add into a dense [n^3][4] u64
//                fixed-point grid, one lane per (node, channel)
//   read_f4      plain float4 loads of the box from a dense grid (G2P staging)
//   read_u64     the box as 4 x u64 per node (32 B), lane per (node, channel)
//
// Reports the average launch time over 20 launches of each.
//   hipcc -O3 --offload-arch=gfx950 window_flush.hip -o window_flush && ./window_flush
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHECK(x)                                                          \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                           \
    }                                                                     \
  } while (0)

constexpr int N = 128, B0 = 10, B1 = 10, B2 = 9, BOX = B0 * B1 * B2, WIN = 1584;
constexpr int kLdsBytes = 50688;

struct Geo {
  const int4* org;  // per chunk: box origin node (x, y, z)
  int nch;
};

__device__ __forceinline__ int box_node(const Geo& g, int w, int q, int& ix, int& iy, int& iz) {
  const int4 o = g.org[w];
  const int a = q / (B1 * B2), r = q - a * (B1 * B2), b = r / B2, c = r - b * B2;
  ix = o.x + a;
  iy = o.y + b;
  iz = o.z + c;
  return (a * B1 + b) * B2 + c;
}

template <int MODE>
__global__ __launch_bounds__(256, 3) void k_flush(Geo g, float4* slots, float* grid_f, unsigned long long* grid_u,
                                                  float4* out) {
  extern __shared__ float4 lds[];
  const int w = blockIdx.x;
  const float val = 1.0f + (float)(threadIdx.x & 7) * 0.125f;
  if constexpr (MODE == 0) {  // slot_sc1
    for (int q = threadIdx.x; q < BOX; q += 256) {
      int ix, iy, iz;
      const int loc = box_node(g, w, q, ix, iy, iz);
      float4* p = slots + (size_t)w * WIN + loc;
      typedef float f4v __attribute__((ext_vector_type(4)));
      f4v t = {val, val, val, val};
      asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(t) : "memory");
    }
  } else if constexpr (MODE == 1) {  // atom_f32_n4
    for (int q = threadIdx.x; q < BOX; q += 256) {
      int ix, iy, iz;
      box_node(g, w, q, ix, iy, iz);
      float* p = grid_f + 4 * (((size_t)ix * N + iy) * N + iz);
#pragma unroll
      for (int ch = 0; ch < 4; ++ch) __hip_atomic_fetch_add(p + ch, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else if constexpr (MODE == 2) {  // atom_f32_c1
    for (int e = threadIdx.x; e < 4 * BOX; e += 256) {
      int ix, iy, iz;
      box_node(g, w, e >> 2, ix, iy, iz);
      float* p = grid_f + 4 * (((size_t)ix * N + iy) * N + iz) + (e & 3);
      __hip_atomic_fetch_add(p, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else if constexpr (MODE == 3) {  // atom_u64_c1
    for (int e = threadIdx.x; e < 4 * BOX; e += 256) {
      int ix, iy, iz;
      box_node(g, w, e >> 2, ix, iy, iz);
      unsigned long long* p = grid_u + 4 * (((size_t)ix * N + iy) * N + iz) + (e & 3);
      __hip_atomic_fetch_add(p, (unsigned long long)(val * 1024.0f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else if constexpr (MODE == 4) {  // read_f4
    for (int q = threadIdx.x; q < BOX; q += 256) {
      int ix, iy, iz;
      const int loc = box_node(g, w, q, ix, iy, iz);
      lds[loc] = reinterpret_cast<const float4*>(grid_f)[((size_t)ix * N + iy) * N + iz];
    }
    __syncthreads();
    if (threadIdx.x == 0 && lds[threadIdx.x + 5].x == 12345.f) out[w] = lds[0];
  } else {  // read_u64
    unsigned long long* l = reinterpret_cast<unsigned long long*>(lds);
    for (int e = threadIdx.x; e < 4 * BOX; e += 256) {
      int ix, iy, iz;
      const int loc = box_node(g, w, e >> 2, ix, iy, iz);
      l[(e & 3) * WIN + loc] = grid_u[4 * (((size_t)ix * N + iy) * N + iz) + (e & 3)];
    }
    __syncthreads();
    if (threadIdx.x == 0 && l[7] == 12345ull) out[w] = lds[0];
  }
}

int main() {
  // ~650 chunks: the tiles of a 8 x 8 x 9 blob (576) plus a second chunk in 74 of them
  std::vector<int4> org;
  for (int tx = 4; tx < 12; ++tx)
    for (int ty = 4; ty < 12; ++ty)
      for (int tz = 5; tz < 14; ++tz) org.push_back(make_int4(tx * 8, ty * 8, tz * 7, 0));
  for (int i = 0; i < 74; ++i) org.push_back(org[i * 7]);
  const int nch = (int)org.size();
  int4* d_org;
  float4 *slots, *out;
  float* grid_f;
  unsigned long long* grid_u;
  CHECK(hipMalloc(&d_org, sizeof(int4) * nch));
  CHECK(hipMemcpy(d_org, org.data(), sizeof(int4) * nch, hipMemcpyHostToDevice));
  CHECK(hipMalloc(&slots, sizeof(float4) * (size_t)nch * WIN));
  CHECK(hipMalloc(&grid_f, sizeof(float) * 4 * (size_t)N * N * N));
  CHECK(hipMalloc(&grid_u, sizeof(unsigned long long) * 4 * (size_t)N * N * N));
  CHECK(hipMalloc(&out, sizeof(float4) * nch));
  CHECK(hipMemset(grid_f, 0, sizeof(float) * 4 * (size_t)N * N * N));
  CHECK(hipMemset(grid_u, 0, sizeof(unsigned long long) * 4 * (size_t)N * N * N));
  Geo g{d_org, nch};
  const char* names[6] = {"slot_sc1", "atom_f32_n4", "atom_f32_c1", "atom_u64_c1", "read_f4", "read_u64"};
  void (*ks[6])(Geo, float4*, float*, unsigned long long*, float4*) = {k_flush<0>, k_flush<1>, k_flush<2>,
                                                                       k_flush<3>, k_flush<4>, k_flush<5>};
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::printf("chunks %d, box %d nodes\n", nch, BOX);
  for (int round = 0; round < 2; ++round)
    for (int m = 0; m < 6; ++m) {
      for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(ks[m], dim3(nch), dim3(256), kLdsBytes, 0, g, slots, grid_f, grid_u, out);
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0, 0));
      for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(ks[m], dim3(nch), dim3(256), kLdsBytes, 0, g, slots, grid_f, grid_u, out);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("%-12s %8.2f us per launch\n", names[m], ms * 1e3f / 20.f);
    }
  CHECK(hipGetLastError());
  return 0;
}

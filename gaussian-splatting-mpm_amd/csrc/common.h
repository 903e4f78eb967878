// common.h -- error plumbing and small device helpers shared by the HIP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <string>

#include "gsmpm.h"

namespace gsmpm {

void set_error(const std::string& msg);

#define GSMPM_HIP(call)                                                                   \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess) {                                                               \
      ::gsmpm::set_error(std::string(#call) + ": " + hipGetErrorString(e_));              \
      return GSMPM_EHIP;                                                                  \
    }                                                                                     \
  } while (0)

#define GSMPM_REQUIRE(cond, msg)                                                          \
  do {                                                                                    \
    if (!(cond)) {                                                                        \
      ::gsmpm::set_error(msg);                                                            \
      return GSMPM_EINVAL;                                                                \
    }                                                                                     \
  } while (0)

// Checks the launch that just happened (launch-configuration errors only; it
// does not synchronise).
#define GSMPM_LAUNCH_CHECK() GSMPM_HIP(hipGetLastError())

inline int div_up(long a, long b) { return (int)((a + b - 1) / b); }

typedef float nt_f4 __attribute__((ext_vector_type(4)));
// write-through vector store (sc1): the line leaves the XCD's L2 with the
// store, so the end-of-kernel release has no dirty line of it to write back.
// For data the next launch reads from other XCDs (chunk windows).
__device__ __forceinline__ void wt_store4(float4* p, const float4& v) {
  nt_f4 t = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(t) : "memory");
}
// streaming (non-temporal) vector store (nt): A/B form of the grid update's v_out store
__device__ __forceinline__ void nt_store4(float4* p, const float4& v) {
  nt_f4 t = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(t) : "memory");
}

}  // namespace gsmpm

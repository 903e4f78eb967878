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

}  // namespace gsmpm

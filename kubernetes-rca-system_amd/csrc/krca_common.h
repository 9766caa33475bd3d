// Shared helpers for the krca HIP translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string>

#include "../../include/krca.h"

namespace krca {

void set_error(const char* fmt, ...);

#define KRCA_CHECK_ARG(cond, ...)            \
  do {                                       \
    if (!(cond)) {                           \
      ::krca::set_error(__VA_ARGS__);        \
      return KRCA_EINVAL;                    \
    }                                        \
  } while (0)

#define KRCA_HIP(call)                                                              \
  do {                                                                              \
    hipError_t e_ = (call);                                                         \
    if (e_ != hipSuccess) {                                                         \
      ::krca::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_),      \
                        __FILE__, __LINE__);                                        \
      return KRCA_EDEVICE;                                                          \
    }                                                                               \
  } while (0)

#define KRCA_LAUNCH_CHECK() KRCA_HIP(hipGetLastError())

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int kWave = 64;

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// 2^60: fixed-point unit of the PageRank mass (krca_ppr)
constexpr double kFix = 1152921504606846976.0;

}  // namespace krca

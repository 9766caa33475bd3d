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
// a non-blocking stream of the calling thread's current device for work a launcher forks off its
// caller's stream (and joins back with events before returning); created once per thread and device
hipStream_t side_stream();

constexpr int kWave = 64;

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// 2^60: fixed-point unit of the PageRank mass (krca_ppr)
constexpr double kFix = 1152921504606846976.0;

// Kernel-development A/B switches (include/krca.h krca_tune_set).  Read from the environment
// once when the library loads, changed only through krca_tune_set; launchers read the struct,
// never the environment.
struct Tuning {
  int score_impl;   // KRCA_SCORE_IMPL: 0 pipelined chunks, 1 plain loads, 2 W-block buffer loads, 4 per-row descriptors
  int score_chunk;  // KRCA_SCORE_CHUNK: rows per pipelined chunk at W = 60 (10/12/15/20/30)
  int score_nt;     // KRCA_SCORE_NT: non-temporal metric loads
  int ppr_grid;     // KRCA_PPR_GRID: persistent PageRank grid (0 = occupancy API)
  int ppr_dict;     // KRCA_PPR_DICT: krca_ppr_pack builds dictionary blocks (0 = all direct)
  int log_impl;     // KRCA_LOG_IMPL: 0 line index + DFA lanes, 1 chunk-lane single pass
  int group_impl;   // KRCA_GROUP_IMPL: 0 peeled atomics, 1 one atomic per lane
  int corr_debug;   // KRCA_CORR_DEBUG: profiling aid (results wrong when != 0)
  int corr_rs_grid; // KRCA_CORR_RS_GRID: workgroups of the ambiguous-pair re-score (a multiple of 8)
};
const Tuning& tuning();
int tuning_ppr_dict();

}  // namespace krca

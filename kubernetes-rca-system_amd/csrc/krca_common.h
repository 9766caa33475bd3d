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
// a non-blocking stream on the device of `st` (the current device for the null stream) for work a
// launcher forks off its caller's stream (and joins back with events before returning); created
// once per thread and device
hipStream_t side_stream(hipStream_t st);
// workgroups of `kernel` (block size tpb, no dynamic LDS) that the device of `st` keeps resident:
// CU count x the occupancy API's blocks per CU (fallback_per_cu if the query fails).  Cached per
// (kernel, device), so a process driving several devices sizes each device's grid from that device
int64_t resident_workgroups(const void* kernel, int tpb, hipStream_t st, int fallback_per_cu);

// makes the device of `st` current for the guard's lifetime (events and side streams are created
// on the current device), restoring the caller's device afterwards
class DeviceGuard {
 public:
  explicit DeviceGuard(hipStream_t st) {
    if (hipGetDevice(&prev_) != hipSuccess) {
      rc_ = KRCA_EDEVICE;
      return;
    }
    int dev = prev_;
    if (st && hipStreamGetDevice(st, &dev) != hipSuccess) {
      rc_ = KRCA_EDEVICE;
      return;
    }
    if (dev != prev_) {
      if (hipSetDevice(dev) != hipSuccess) {
        rc_ = KRCA_EDEVICE;
        return;
      }
      switched_ = true;
    }
  }
  ~DeviceGuard() {
    if (switched_) (void)hipSetDevice(prev_);
  }
  int status() const {
    if (rc_) set_error("krca: cannot select the device of the caller's stream");
    return rc_;
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;

 private:
  int prev_ = 0, rc_ = 0;
  bool switched_ = false;
};

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
  int corr_batch;   // KRCA_CORR_BATCH: super-tiles per main-pass batch (0 = 8192)
  int corr_amb_tile;  // KRCA_CORR_AMB_TILE: ambiguous-list budget per tile of a batch (-1 = 512; 0 = every
                      // tile decides its pairs in place)
  int ppr_fuse;     // KRCA_PPR_FUSE: single device, the iteration's reduction in the step's last workgroup
                    // (0 = a ppr_reduce launch after each step)
  int ppr_nt;       // KRCA_PPR_NT: the step streams its plan / column / row arrays with non-temporal loads
  int ppr_xcd;      // KRCA_PPR_XCD: each XCD's workgroups take one contiguous eighth of the plan entries
  int log_fused;    // KRCA_LOG_FUSED: krca_log_scan walks the DFA inside the line-index pass (0 = index, then log_dfa)
  int corr_rs_group;  // KRCA_CORR_RS_GROUP: the ambiguous pairs re-scored grouped by row pod (row in LDS; 0 = per pair)
  int corr_side;      // KRCA_CORR_SIDE: where the exact-count re-scores run: 0 every batch's on a side stream beside
                      // the next batch's tiles, 1 each after its batch on the caller's stream, 2 those after their
                      // batch except the last (beside the merge chain)
  int corr_rs_q16;    // KRCA_CORR_RS_Q16: the grouped re-score reads int16 partner rows (row max / 32767 steps)
                      // and re-reads the fp32 row only within their error bound of tau (0 = fp32 rows)
  int corr_capc;      // KRCA_CORR_CAPC: candidate slots used per pod, 64 .. krca_corr_cand_cap() (0 = all; tests
                      // make buffers overflow with fewer)
  int corr_km_extra;  // KRCA_CORR_KM_EXTRA: candidates the merge re-scores in float64 past the k-th (1..8, default 6)
  int corr_rsg_grid;  // KRCA_CORR_RSG_GRID: workgroups of the grouped re-score (0 = 2048)
  int corr_proj;      // KRCA_CORR_PROJ: the grouped re-score tries the projection bound (DCT basis) before the
                      // partner's int16 row: 2 always (default), 1 when the main pass runs in several batches,
                      // 0 never (identical counts)
  int corr_persist;   // KRCA_CORR_PERSIST: the main pass as persistent workgroups that load the next tile's first
                      // K stage under the current one (1) or one workgroup per tile (0, default: R7a, the
                      // persistent form ran 2-5 % slower); same bits
};
const Tuning& tuning();
int tuning_ppr_dict();

}  // namespace krca

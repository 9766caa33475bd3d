// Pod status categorisation: ResourceAnalyzer._analyze_pods
// (ref:agents/resource_analyzer.py:264-380) with _is_pod_healthy (:856-895) as a columnar kernel.
//
// Input is the columnar pod status the host encodes once (krca/podstate.py):
//   pod_code  u8[P]   bits 0-2 phase (0 Pending, 1 Running, 2 Succeeded, 3 Failed, 4 Unknown or
//                     missing, 5 other), bit 3 first Ready condition has status "True", bit 4 some
//                     Ready condition has status != "True", bit 5 status.reason == "Evicted"
//   cont_off  i64[P+1] container records of pod p: [cont_off[p], cont_off[p+1]), in the order
//                     containerStatuses then initContainerStatuses (the reference's scan order)
//   cont_code u16[C]  bit 0 from initContainerStatuses, bit 1 ready, bit 2 state has "waiting",
//                     bit 3 state has "terminated", bits 4-6 waiting reason (1 CrashLoopBackOff,
//                     2 ImagePullBackOff, 3 ErrImagePull, 4 ContainerCreating, 0 other), bits 7-8
//                     terminated reason (1 Completed, 2 Error, 0 other), bit 9 name starts "init-"
// Output: mask u16[P], bit b = membership of the reference's status group b in its dict order
// (pending, running, succeeded, failed, unknown, crashloopbackoff, imagepullbackoff,
// containercreating, error, evicted, init_crashloopbackoff, not_ready) — a pod can sit in several,
// exactly as in the reference — and hist i32[12], the group sizes.
//
// One lane per pod (grid-stride); the group sizes are wave ballots summed in LDS, one atomic per
// group and workgroup (integer: order-free).  HBM-bound: 11 + 2*containers bytes per pod.
#include "krca_common.h"

namespace {

constexpr int TPB = 256;
constexpr int NGROUP = 12;
enum : uint32_t {
  G_PENDING = 1u << 0, G_RUNNING = 1u << 1, G_SUCCEEDED = 1u << 2, G_FAILED = 1u << 3, G_UNKNOWN = 1u << 4,
  G_CRASHLOOP = 1u << 5, G_IMAGEPULL = 1u << 6, G_CREATING = 1u << 7, G_ERROR = 1u << 8, G_EVICTED = 1u << 9,
  G_INIT_CRASHLOOP = 1u << 10, G_NOT_READY = 1u << 11
};

__device__ __forceinline__ uint32_t classify(uint8_t pc, const uint16_t* __restrict__ cc, int64_t c0, int64_t c1) {
  const int phase = pc & 7;
  uint32_t m = 0;
  if (phase == 0) {
    m |= G_PENDING;
  } else if (phase == 1) {
    // _is_pod_healthy: Running, first Ready condition "True", >= 1 container status, every one
    // ready, none waiting, none terminated for a reason other than Completed
    bool healthy = (pc & 8) != 0;
    int n_main = 0;
    for (int64_t c = c0; c < c1 && healthy; ++c) {
      const uint32_t x = cc[c];
      if (x & 1) break;  // init statuses come after the main ones
      ++n_main;
      healthy = (x & 2) && !(x & 4) && !((x & 8) && ((x >> 7) & 3) != 1);
    }
    healthy = healthy && n_main > 0;
    if (healthy) {
      m |= G_RUNNING;
    } else {
      for (int64_t c = c0; c < c1; ++c) {  // first waiting status with a recognised reason
        const uint32_t x = cc[c];
        if (!(x & 4)) continue;
        const uint32_t wr = (x >> 4) & 7;
        if (wr == 1) {
          m |= (x & 512) ? G_INIT_CRASHLOOP : G_CRASHLOOP;
          break;
        }
        if (wr == 2 || wr == 3) {
          m |= G_IMAGEPULL;
          break;
        }
        if (wr == 4) {
          m |= G_CREATING;
          break;
        }
      }
      if (pc & 16) m |= G_NOT_READY;
    }
  } else if (phase == 2) {
    m |= G_SUCCEEDED;
  } else if (phase == 3) {
    m |= G_FAILED;
  } else if (phase == 4) {
    m |= G_UNKNOWN;
  }
  if (pc & 32) m |= G_EVICTED;
  for (int64_t c = c0; c < c1; ++c) {  // a main container terminated with reason Error
    const uint32_t x = cc[c];
    if (x & 1) break;
    if ((x & 8) && ((x >> 7) & 3) == 2) {
      m |= G_ERROR;
      break;
    }
  }
  return m;
}

__global__ __launch_bounds__(TPB) void pod_classify(const uint8_t* __restrict__ pod_code,
                                                    const int64_t* __restrict__ cont_off,
                                                    const uint16_t* __restrict__ cont_code, int64_t P,
                                                    uint16_t* __restrict__ mask, int32_t* __restrict__ hist) {
  __shared__ int lh[NGROUP];
  if (threadIdx.x < NGROUP) lh[threadIdx.x] = 0;
  __syncthreads();
  int cnt[NGROUP];
#pragma unroll
  for (int b = 0; b < NGROUP; ++b) cnt[b] = 0;
  const int64_t stride = (int64_t)gridDim.x * TPB;
  for (int64_t base = (int64_t)blockIdx.x * TPB; base < P; base += stride) {  // wave-uniform trip count
    const int64_t p = base + threadIdx.x;
    uint32_t m = 0;
    if (p < P) {
      m = classify(pod_code[p], cont_code, cont_off[p], cont_off[p + 1]);
      mask[p] = (uint16_t)m;
    }
#pragma unroll
    for (int b = 0; b < NGROUP; ++b) cnt[b] += __popcll(__ballot((m >> b) & 1));  // wave-uniform
  }
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int b = 0; b < NGROUP; ++b)
      if (cnt[b]) atomicAdd(&lh[b], cnt[b]);
  }
  __syncthreads();
  if (threadIdx.x < NGROUP && lh[threadIdx.x]) atomicAdd(&hist[threadIdx.x], lh[threadIdx.x]);
}

}  // namespace

extern "C" {

int32_t krca_pod_groups(void) { return NGROUP; }

int krca_pod_classify(const uint8_t* pod_code, const int64_t* cont_off, const uint16_t* cont_code, int64_t P,
                      uint16_t* mask, int32_t* hist, void* stream) {
  KRCA_CHECK_ARG(P >= 0, "krca_pod_classify: P < 0");
  KRCA_CHECK_ARG(hist, "krca_pod_classify: null hist");
  hipStream_t st = krca::as_stream(stream);
  KRCA_HIP(hipMemsetAsync(hist, 0, NGROUP * sizeof(int32_t), st));
  if (P == 0) return KRCA_OK;
  KRCA_CHECK_ARG(pod_code && cont_off && cont_code && mask, "krca_pod_classify: null pointer");
  const unsigned blocks = (unsigned)std::min<int64_t>(krca::ceil_div(P, TPB), 4096);
  hipLaunchKernelGGL(pod_classify, dim3(blocks), dim3(TPB), 0, st, pod_code, cont_off, cont_code, P, mask, hist);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

}  // extern "C"

// Root-cause explanation pass (krca_rca_explain; DESIGN.md §3.2 "Ranking").
//
// The root-cause key of krca.rca.Config (key "explained") ranks a pod by the PageRank mass it
// received from its callers times the part of its own anomaly that no anomalous dependency explains.
// This pass finds, for each pod of a rank's range, the largest anomaly among the dependencies that
// explain it:
//   q_j   the quantised seed of krca_ppr_shard_init (2^32 per |z| unit above the floor; q > 0 =
//         anomalous);
//   A_k   per anomalous pod k: its edges from anomalous callers (row k of the pull-CSR), S_k the sum
//         of their q (128 bits; q <= 2^40, so every comparison below is exact for any row length);
//   an anomalous dependency k of an anomalous pod j (edge j -> k, j != k) explains j when it collects
//   at least as many anomalous callers besides j (A_k - 1 >= A_j: the symptoms converge on k) or is
//   at least twice as anomalous (q_k >= 2 q_j), AND j looks like k's other symptoms (A_k q_j <=
//   3 S_k: at most 3x their mean -- a pod far above them is a fault of its own that calls k);
//   d_j   the largest q_k over the dependencies that explain j (0: none).
// Integer counts and an integer max: the result is independent of the schedule and bit-identical to
// oracle/krca_oracle.c krco_rca_explain.
//
// Work and data: it needs the scores of EVERY pod and the whole pull-CSR (a rank's pods may be
// explained by, or call, pods of any rank), but only the anomalous pods' rows are walked -- a few
// thousand rows at C4 -- so every rank runs the pass on the full graph it keeps resident, with no
// collective beyond the scores (all-gathered once per step at G > 1).  Three launches, no host sync:
//   rca_anomalous        one pass over the N scores (4 B per pod): the anomalous pods' ids, compacted
//                        with a wave ballot and one atomic per wave (the order does not matter);
//   rca_caller_counts    a wave per anomalous pod: A_k and S_k over its row (lanes stride the callers);
//   rca_explain_scatter  a wave per anomalous pod k: for each anomalous caller j of the rank's range
//                        that k explains, a 64-bit atomicMax of q_k into d[j - lo].
#include <algorithm>

#include "krca_common.h"

namespace {

constexpr int TPB = 256;

// a seed's anomaly above the floor in 2^-32 units, clamped at 256 units (q <= 2^40: every product
// and sum of the explanation pass and the int64 seed total of N <= 2^23 pods stay exact; a NaN is 0)
__device__ __forceinline__ int64_t quantise(float s, float floor_) {  // == ppr.hip quantise
  const double v = (double)s - (double)floor_;
  return v > 0.0 ? (int64_t)(fmin(v, 256.0) * 4294967296.0) : 0;
}

__device__ __forceinline__ int wave_sum(int v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ __int128 wave_sum128(__int128 v) {  // exact: the lanes' sums of q <= 2^40 each
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t lo = (uint64_t)v, hi = (uint64_t)(v >> 64);
    const uint64_t olo = (uint64_t)__shfl_xor((long long)lo, off, 64), ohi = (uint64_t)__shfl_xor((long long)hi, off, 64);
    v += (__int128)(((unsigned __int128)ohi << 64) | olo);
  }
  return v;
}

__global__ __launch_bounds__(TPB) void rca_anomalous(const float* __restrict__ s, int64_t N, float fl,
                                                     int32_t* __restrict__ list, uint32_t* __restrict__ n_list) {
  const int lane = threadIdx.x & 63;
  // block-uniform trip count: every lane of a wave runs the same iterations (the ballot needs them)
  for (int64_t base = (int64_t)blockIdx.x * TPB; base < N; base += (int64_t)gridDim.x * TPB) {
    const int64_t i = base + threadIdx.x;
    const bool a = i < N && quantise(s[i], fl) > 0;
    const unsigned long long m = __ballot(a);
    if (m == 0ull) continue;  // wave-uniform
    const int leader = __ffsll(m) - 1;
    uint32_t off = 0;
    if (lane == leader) off = atomicAdd(n_list, (uint32_t)__popcll(m));
    off = __shfl(off, leader, 64);
    if (a) {
      const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      list[off + below] = (int32_t)i;
    }
  }
}

__global__ __launch_bounds__(TPB) void rca_caller_counts(const int32_t* __restrict__ list,
                                                         const uint32_t* __restrict__ n_list,
                                                         const float* __restrict__ s, float fl,
                                                         const int64_t* __restrict__ row_ptr,
                                                         const int32_t* __restrict__ col, int32_t* __restrict__ A,
                                                         __int128* __restrict__ S) {
  const int lane = threadIdx.x & 63;
  const int64_t n = *n_list;
  for (int64_t w = ((int64_t)blockIdx.x * TPB + threadIdx.x) >> 6; w < n; w += ((int64_t)gridDim.x * TPB) >> 6) {
    const int32_t k = list[w];
    const int64_t e1 = row_ptr[k + 1];
    int c = 0;
    __int128 sum = 0;
    for (int64_t e = row_ptr[k] + lane; e < e1; e += 64) {
      const int64_t qc = quantise(s[col[e]], fl);
      c += qc > 0;
      sum += qc;  // 0 for a caller at or below the floor
    }
    c = wave_sum(c);
    sum = wave_sum128(sum);
    if (lane == 0) {
      A[k] = c;
      S[k] = sum;
    }
  }
}

__global__ __launch_bounds__(TPB) void rca_explain_scatter(const int32_t* __restrict__ list,
                                                           const uint32_t* __restrict__ n_list,
                                                           const float* __restrict__ s, float fl,
                                                           const int64_t* __restrict__ row_ptr,
                                                           const int32_t* __restrict__ col,
                                                           const int32_t* __restrict__ A,
                                                           const __int128* __restrict__ S, int64_t lo, int64_t hi,
                                                           unsigned long long* __restrict__ d) {
  const int lane = threadIdx.x & 63;
  const int64_t n = *n_list;
  for (int64_t w = ((int64_t)blockIdx.x * TPB + threadIdx.x) >> 6; w < n; w += ((int64_t)gridDim.x * TPB) >> 6) {
    const int32_t k = list[w];
    const int64_t qk = quantise(s[k], fl);
    const int32_t ak = A[k];
    const __int128 sk3 = 3 * S[k];  // (128 bits: exact for any row length)
    const int64_t e1 = row_ptr[k + 1];
    for (int64_t e = row_ptr[k] + lane; e < e1; e += 64) {
      const int64_t j = col[e];
      if (j < lo || j >= hi || j == k) continue;
      const int64_t qj = quantise(s[j], fl);
      if (qj <= 0) continue;
      if ((ak - 1 >= A[j] || qk >= 2 * qj) && (__int128)ak * qj <= sk3) atomicMax(d + (j - lo), (unsigned long long)qk);
    }
  }
}

constexpr int64_t kListGrid = 1024;  // waves x 4 per workgroup walking the anomalous pods' rows

}  // namespace

extern "C" {

// workspace: S int128[N] | A int32[N] | list int32[N] | counter (256 B)
int64_t krca_rca_explain_ws_size(int64_t N) { return 24 * std::max<int64_t>(N, 1) + 256; }

int krca_rca_explain(const float* score_all, int64_t N, float seed_floor, const int64_t* row_ptr, const int32_t* col,
                     int64_t lo, int64_t hi, int64_t* d_local, void* ws, void* stream) {
  KRCA_CHECK_ARG(N > 0 && N < INT32_MAX && lo >= 0 && lo <= hi && hi <= N, "krca_rca_explain: bad sizes");
  KRCA_CHECK_ARG(score_all && row_ptr && col && ws && (hi == lo || d_local), "krca_rca_explain: null pointer");
  hipStream_t st = krca::as_stream(stream);
  char* p = reinterpret_cast<char*>(ws);
  KRCA_CHECK_ARG(((uintptr_t)ws & 15) == 0, "krca_rca_explain: workspace must be 16-byte aligned");
  __int128* S = reinterpret_cast<__int128*>(p);
  int32_t* A = reinterpret_cast<int32_t*>(p + 16 * N);
  int32_t* list = A + N;
  uint32_t* n_list = reinterpret_cast<uint32_t*>(p + 24 * N);
  KRCA_HIP(hipMemsetAsync(n_list, 0, sizeof(uint32_t), st));
  if (hi > lo) KRCA_HIP(hipMemsetAsync(d_local, 0, (hi - lo) * sizeof(int64_t), st));
  const unsigned g0 = (unsigned)std::min<int64_t>(krca::ceil_div(N, TPB), 2048);
  hipLaunchKernelGGL(rca_anomalous, dim3(g0), dim3(TPB), 0, st, score_all, N, seed_floor, list, n_list);
  KRCA_LAUNCH_CHECK();
  hipLaunchKernelGGL(rca_caller_counts, dim3((unsigned)kListGrid), dim3(TPB), 0, st, list, n_list, score_all,
                     seed_floor, row_ptr, col, A, S);
  KRCA_LAUNCH_CHECK();
  if (hi > lo) {
    hipLaunchKernelGGL(rca_explain_scatter, dim3((unsigned)kListGrid), dim3(TPB), 0, st, list, n_list, score_all,
                       seed_floor, row_ptr, col, A, S, lo, hi, reinterpret_cast<unsigned long long*>(d_local));
    KRCA_LAUNCH_CHECK();
  }
  return KRCA_OK;
}

}  // extern "C"

// krca_group_reduce — the group-bys of EventsAgent and Coordinator._correlate_findings.
//
// The reference builds Python dicts keyed by object / pod / component / node name
// (ref:agents/events_agent.py:105-133,169-228,230-290,330-375,377-446) and by finding component
// (ref:agents/coordinator.py:118-155), then takes per group: the group's first-seen position (dict
// insertion order), its size, the number of "selected" members (Warning events) and the latest
// member(s) by lastTimestamp (`max(...)`, `sorted(..., reverse=True)[:3]`) or the highest
// severity.  The host interns the group keys to dense slot ids and packs each member's sort key
// into a non-negative int64 that is unique per member ((rank << 32) | (2^31-1-index): larger rank
// wins, ties go to the earlier member, exactly like Python's max / stable reverse sort).
//
// Device work per membership record i (slot s, key k), into the slot's 64-byte record
// rec[s] = {first, (count << 32) | n_key, top[0], ..., top[R-1]} (int64 words):
//   first = min i,  count += 1,  n_key += (k >= 0),  top[0] = max k              (pass 0)
//   top[r] = max { k : 0 <= k < top[r-1] }, records i < n_ranked only            (pass r >= 1)
// One record per slot keeps every atomic of a group on one 128-byte L2 line: with millions of
// slots the output (64 B x S) does not fit the L2, and the scattered atomics are the cost (the
// SoA layout touched 4 lines per record in pass 0).  A wave folds the lanes that share a slot
// before touching memory ("peeling": the lowest active lane's slot is broadcast, the matching
// lanes reduce with ballots and shuffles, one lane issues the atomics), so a hot slot (4
// control-plane components over 1M events) costs one atomic per wave, not one per event.
// min / add / max are order-free: the result is deterministic.
#include "krca_common.h"

#include <algorithm>
#include <climits>
#include <cstdlib>

namespace {

constexpr int TPB = 256;

__device__ inline int64_t wave_max_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t w = __shfl_xor(v, o, 64);
    v = w > v ? w : v;
  }
  return v;
}

constexpr int REC = 8;  // int64 words per slot record (64 B)

__global__ __launch_bounds__(TPB) void group_init(int32_t S, int64_t* __restrict__ rec) {
  const int64_t stride = (int64_t)gridDim.x * TPB;
  for (int64_t w = (int64_t)blockIdx.x * TPB + threadIdx.x; w < (int64_t)S * REC; w += stride) {
    const int j = (int)(w & (REC - 1));
    rec[w] = j == 0 ? (int64_t)INT_MAX : (j == 1 ? 0 : -1);
  }
}

// PASS 0: first / count / n_key / top[0].  PASS r>0: top[r] below top[r-1].
template <bool PASS0, bool PEEL>
__global__ __launch_bounds__(TPB) void group_pass(const int32_t* __restrict__ slot, const int64_t* __restrict__ key,
                                                  int64_t N, int32_t S, int r, int64_t* __restrict__ rec) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * TPB;
  for (int64_t base = (int64_t)blockIdx.x * TPB; base < N; base += stride) {  // wave-uniform trip count
    const int64_t i = base + threadIdx.x;
    int32_t s = -1;
    int64_t k = -1;
    if (i < N) {
      s = __builtin_nontemporal_load(slot + i);
      k = __builtin_nontemporal_load(key + i);
      if (s >= S) s = -1;  // out-of-range slots are ignored (documented in krca.h)
      if (!PASS0 && s >= 0) {
        const int64_t lim = rec[(int64_t)s * REC + 1 + r];  // top[r-1]
        if (!(k >= 0 && k < lim)) s = -1;  // only keys strictly below the previous rank compete
      }
    }
    if (!PEEL) {  // A/B variant (KRCA_GROUP_IMPL=1): every lane issues its own atomics
      if (s >= 0) {
        int64_t* rp = rec + (int64_t)s * REC;
        if (PASS0) {
          atomicMin((long long*)rp, (long long)i);
          atomicAdd((unsigned long long*)(rp + 1), (1ull << 32) | (k >= 0 ? 1u : 0u));
        }
        if (k >= 0) atomicMax((long long*)(rp + 2 + r), (long long)k);
      }
      continue;
    }
    uint64_t act = __ballot(s >= 0);
    while (act) {  // wave-uniform: act is a ballot
      const int leader = __ffsll((unsigned long long)act) - 1;
      const int32_t ls = __shfl(s, leader, 64);
      const bool mine = (s == ls);
      const uint64_t m = __ballot(mine);
      const int64_t mx = wave_max_i64(mine ? k : -1);
      const uint64_t nk = PASS0 ? (uint64_t)__popcll(__ballot(mine && k >= 0)) : 0;  // whole wave votes
      if (lane == leader) {
        int64_t* rp = rec + (int64_t)ls * REC;
        if (PASS0) {
          // the leader is the lowest lane of the group: its i is the group's min
          atomicMin((long long*)rp, (long long)i);
          atomicAdd((unsigned long long*)(rp + 1), ((uint64_t)__popcll(m) << 32) | nk);
        }
        if (mx >= 0) atomicMax((long long*)(rp + 2 + r), (long long)mx);
      }
      act &= ~m;
      if (mine) s = -1;
    }
  }
}

unsigned grid_for(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>(krca::ceil_div(n, TPB), 8192)); }

}  // namespace

extern "C" {

int32_t krca_group_max_rank(void) { return REC - 2; }

int krca_group_reduce(const int32_t* slot, const int64_t* key, int64_t N, int64_t n_ranked, int32_t S, int32_t R,
                      int64_t* rec, void* stream) {
  KRCA_CHECK_ARG(N >= 0 && N < INT_MAX, "krca_group_reduce: N=%lld out of [0, 2^31-1)", (long long)N);
  KRCA_CHECK_ARG(n_ranked >= 0 && n_ranked <= N, "krca_group_reduce: n_ranked=%lld not in [0, N]",
                 (long long)n_ranked);
  KRCA_CHECK_ARG(S >= 0, "krca_group_reduce: S < 0");
  KRCA_CHECK_ARG(R >= 1 && R <= REC - 2, "krca_group_reduce: R=%d not in [1, %d]", R, REC - 2);
  if (S == 0) return KRCA_OK;
  KRCA_CHECK_ARG(rec, "krca_group_reduce: null output");
  hipStream_t st = krca::as_stream(stream);
  hipLaunchKernelGGL(group_init, dim3(grid_for((int64_t)S * REC)), dim3(TPB), 0, st, S, rec);
  KRCA_LAUNCH_CHECK();
  if (N == 0) return KRCA_OK;
  KRCA_CHECK_ARG(slot && key, "krca_group_reduce: null input");
  const int impl = krca::tuning().group_impl;
  if (impl == 1)
    hipLaunchKernelGGL((group_pass<true, false>), dim3(grid_for(N)), dim3(TPB), 0, st, slot, key, N, S, 0, rec);
  else
    hipLaunchKernelGGL((group_pass<true, true>), dim3(grid_for(N)), dim3(TPB), 0, st, slot, key, N, S, 0, rec);
  KRCA_LAUNCH_CHECK();
  for (int r = 1; r < R && n_ranked > 0; ++r) {
    if (impl == 1)
      hipLaunchKernelGGL((group_pass<false, false>), dim3(grid_for(n_ranked)), dim3(TPB), 0, st, slot, key, n_ranked,
                         S, r, rec);
    else
      hipLaunchKernelGGL((group_pass<false, true>), dim3(grid_for(n_ranked)), dim3(TPB), 0, st, slot, key, n_ranked,
                         S, r, rec);
    KRCA_LAUNCH_CHECK();
  }
  return KRCA_OK;
}

}  // extern "C"

// Service-graph construction from Kubernetes objects:
// TopologyAgent._build_service_graph (ref:agents/topology_agent.py:94-160) and
// _infer_dependencies_from_env (:228-260), plus the same selector test in
// ResourceAnalyzer._find_matching_pods (ref:agents/resource_analyzer.py:835-854, O(S*P)).  The
// all-pairs loops of those builds run here; the host replays the matches in the reference's
// insertion order (node / edge order and attribute overwrites are part of the result: cycle
// listings, path ties and `topology_data` follow it).
//
// 1. krca_selector_match — `all(item in labels.items() for item in selector.items())` for every
//    (object, selector) pair (:133; the network-policy coverage test :474-480 with the roles
//    swapped).  The host interns each (key, value) item to a dense int32 id, so a test is "every
//    selector id occurs in the object's id list" — exact, no hashing.  Output: a bit matrix
//    bits[d][ceil(S/64)] (u64), bit s of row d = match; an empty selector matches everything.
//    One wave per (object, 64 selectors): the object's ids are wave-uniform loads, each lane
//    checks its selector's ids against them; one ballot gives the 64-bit word.  No atomics.
//
// 2. krca_substr_match — `key in value` for every (env value, service DNS key) pair (:257).  Keys
//    are hashed once (FNV-1a 64) into an open-addressing table (krca_substr_prepare).  A wave
//    takes one value; its lanes take start positions, extend one FNV state byte by byte through
//    the distinct key lengths in ascending order and probe the table at each; a hit is verified
//    byte for byte (exact), then appended as v * K + k.  Python's `in` on str equals byte
//    containment on the UTF-8 encodings (UTF-8 is self-synchronising), so the host passes UTF-8.
//    Work: sum over values of len(value) * (longest key) byte steps, re-read from L1.
#include <stdint.h>

#include "krca_common.h"

namespace {

constexpr int TPB = 256;
constexpr uint64_t FNV_BASIS = 1469598103934665603ull;
constexpr uint64_t FNV_PRIME = 1099511628211ull;

__global__ __launch_bounds__(TPB) void selector_match(const int32_t* __restrict__ lab, const int64_t* __restrict__ lab_off,
                                                      int64_t D, const int32_t* __restrict__ sel,
                                                      const int64_t* __restrict__ sel_off, int64_t S, int64_t SW,
                                                      unsigned long long* __restrict__ bits) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * TPB + threadIdx.x) >> 6;
  if (wave >= D * SW) return;  // wave-uniform
  const int64_t d = wave / SW, w = wave % SW;
  const int64_t s = w * 64 + lane;
  const int64_t l0 = lab_off[d], l1 = lab_off[d + 1];
  bool ok = s < S;
  if (ok) {
    for (int64_t i = sel_off[s], i1 = sel_off[s + 1]; i < i1 && ok; ++i) {
      const int32_t want = sel[i];
      bool found = false;
      for (int64_t j = l0; j < l1; ++j) found |= (lab[j] == want);
      ok = found;
    }
  }
  const unsigned long long m = __ballot(ok);
  if (lane == 0) bits[d * SW + w] = m;
}

__device__ __forceinline__ uint64_t fnv_step(uint64_t h, uint8_t c) { return (h ^ c) * FNV_PRIME; }

__global__ __launch_bounds__(TPB) void substr_prepare(const uint8_t* __restrict__ pat, const int64_t* __restrict__ pat_off,
                                                      int64_t K, int32_t* __restrict__ table, uint64_t mask,
                                                      uint64_t* __restrict__ hash) {
  const int64_t k = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (k >= K) return;
  uint64_t h = FNV_BASIS;
  for (int64_t i = pat_off[k]; i < pat_off[k + 1]; ++i) h = fnv_step(h, pat[i]);
  hash[k] = h;
  for (uint64_t slot = h & mask;; slot = (slot + 1) & mask) {  // the table has >= 2K slots
    if (atomicCAS(&table[slot], -1, (int32_t)k) == -1) break;
  }
}

__global__ __launch_bounds__(TPB) void substr_match(const uint8_t* __restrict__ text, const int64_t* __restrict__ val_off,
                                                    int64_t V, const uint8_t* __restrict__ pat,
                                                    const int64_t* __restrict__ pat_off, int64_t K,
                                                    const int32_t* __restrict__ table, uint64_t mask,
                                                    const uint64_t* __restrict__ hash, const int32_t* __restrict__ lens,
                                                    int32_t n_lens, long long* __restrict__ out, int64_t cap,
                                                    unsigned long long* __restrict__ n_out) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (TPB / 64);
  for (int64_t v = ((int64_t)blockIdx.x * TPB + threadIdx.x) >> 6; v < V; v += nw) {  // wave-uniform
    const int64_t b0 = val_off[v], n = val_off[v + 1] - b0;
    for (int64_t i = lane; i < n; i += 64) {
      uint64_t h = FNV_BASIS;
      int64_t j = 0;
      for (int li = 0; li < n_lens; ++li) {
        const int32_t L = lens[li];
        if (i + L > n) break;
        for (; j < L; ++j) h = fnv_step(h, text[b0 + i + j]);
        for (uint64_t slot = h & mask;; slot = (slot + 1) & mask) {
          const int32_t k = table[slot];
          if (k < 0) break;
          if (hash[k] != h || pat_off[k + 1] - pat_off[k] != L) continue;
          const uint8_t* p = pat + pat_off[k];
          bool eq = true;
          for (int32_t q = 0; q < L && eq; ++q) eq = p[q] == text[b0 + i + q];
          if (eq) {
            const unsigned long long at = atomicAdd(n_out, 1ull);
            if ((int64_t)at < cap) out[at] = (long long)(v * K + k);
          }
        }
      }
    }
  }
}

}  // namespace

extern "C" {

int krca_selector_match(const int32_t* lab, const int64_t* lab_off, int64_t D, const int32_t* sel,
                        const int64_t* sel_off, int64_t S, uint64_t* bits, void* stream) {
  KRCA_CHECK_ARG(D >= 0 && S >= 0, "krca_selector_match: negative sizes");
  if (D == 0 || S == 0) return KRCA_OK;
  KRCA_CHECK_ARG(lab && lab_off && sel && sel_off && bits, "krca_selector_match: null pointer");
  hipStream_t st = krca::as_stream(stream);
  const int64_t SW = (S + 63) / 64;
  const int64_t waves = D * SW;
  KRCA_CHECK_ARG(krca::ceil_div(waves, TPB / 64) < INT32_MAX, "krca_selector_match: D*S too large");
  hipLaunchKernelGGL(selector_match, dim3((unsigned)krca::ceil_div(waves, TPB / 64)), dim3(TPB), 0, st, lab, lab_off,
                     D, sel, sel_off, S, SW, reinterpret_cast<unsigned long long*>(bits));
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int64_t krca_substr_table_size(int64_t K) {
  int64_t n = 64;
  while (n < 2 * K) n *= 2;
  return n;
}

int krca_substr_prepare(const uint8_t* pat, const int64_t* pat_off, int64_t K, int32_t* table, int64_t table_size,
                        uint64_t* hash, void* stream) {
  KRCA_CHECK_ARG(K >= 0 && table_size >= krca_substr_table_size(K) && (table_size & (table_size - 1)) == 0,
                 "krca_substr_prepare: table too small or not a power of two");
  KRCA_CHECK_ARG(table && (K == 0 || (pat && pat_off && hash)), "krca_substr_prepare: null pointer");
  hipStream_t st = krca::as_stream(stream);
  KRCA_HIP(hipMemsetAsync(table, 0xff, table_size * sizeof(int32_t), st));
  if (K == 0) return KRCA_OK;
  hipLaunchKernelGGL(substr_prepare, dim3((unsigned)krca::ceil_div(K, TPB)), dim3(TPB), 0, st, pat, pat_off, K, table,
                     (uint64_t)(table_size - 1), hash);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_substr_match(const uint8_t* text, const int64_t* val_off, int64_t V, const uint8_t* pat,
                      const int64_t* pat_off, int64_t K, const int32_t* table, int64_t table_size,
                      const uint64_t* hash, const int32_t* lens, int32_t n_lens, int64_t* out, int64_t cap,
                      uint64_t* n_out, void* stream) {
  KRCA_CHECK_ARG(V >= 0 && K >= 0 && n_lens >= 0 && cap >= 0, "krca_substr_match: negative sizes");
  KRCA_CHECK_ARG(n_out, "krca_substr_match: null n_out");
  hipStream_t st = krca::as_stream(stream);
  KRCA_HIP(hipMemsetAsync(n_out, 0, sizeof(uint64_t), st));
  if (V == 0 || K == 0 || n_lens == 0) return KRCA_OK;
  KRCA_CHECK_ARG(text && val_off && pat && pat_off && table && hash && lens && (cap == 0 || out),
                 "krca_substr_match: null pointer");
  KRCA_CHECK_ARG(table_size >= krca_substr_table_size(K) && (table_size & (table_size - 1)) == 0,
                 "krca_substr_match: bad table size");
  const int64_t blocks = std::min<int64_t>(krca::ceil_div(V, TPB / 64), 8192);
  hipLaunchKernelGGL(substr_match, dim3((unsigned)blocks), dim3(TPB), 0, st, text, val_off, V, pat, pat_off, K, table,
                     (uint64_t)(table_size - 1), hash, lens, n_lens, reinterpret_cast<long long*>(out), cap,
                     reinterpret_cast<unsigned long long*>(n_out));
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

}  // extern "C"

// Deterministic top-k (descending value, ties -> lower index) for float32 and int64 keys.
//
// Used for the anomaly ranking (a5) and the root-cause top-10 (a10).  Two launches:
//   stage 1: each lane keeps a sorted top-KM list in registers (KM = 10 for k <= 10, else 16;
//            unrolled insertion network, static register indices), then the workgroup extracts its top-k by k rounds of
//            a block-wide arg-max over the lanes' list heads (wave shuffles + LDS);
//   stage 2: one workgroup merges the G*k stage-1 candidates the same way.
// NaN keys are never selected: they are skipped like the sentinel, so with fewer than k
// non-NaN keys the missing slots come back as (idx -1, lowest()).  Bandwidth: one read of v.
#include <float.h>

#include "krca_common.h"

namespace {

constexpr int KMAX = 16;
constexpr int TPB = 256;
constexpr int BATCH = 8;  // keys loaded per lane before they are inserted

template <typename K>
struct Key;
template <>
struct Key<float> {
  __device__ static float lowest() { return -INFINITY; }
  __device__ static bool valid(float v) { return v == v; }
};
template <>
struct Key<int64_t> {
  __device__ static int64_t lowest() { return INT64_MIN; }
  __device__ static bool valid(int64_t) { return true; }
};

// a ranks before b
template <typename K>
__device__ __forceinline__ bool better(K va, int32_t ia, K vb, int32_t ib) {
  return va > vb || (va == vb && (uint32_t)ia < (uint32_t)ib);
}

template <typename K, int KM>
struct List {
  K v[KM];
  int32_t i[KM];
  __device__ void init() {
#pragma unroll
    for (int j = 0; j < KM; ++j) {
      v[j] = Key<K>::lowest();
      i[j] = -1;  // (uint32)-1 = loses every tie
    }
  }
  __device__ void insert(K nv, int32_t ni) {
    if (!better(nv, ni, v[KM - 1], i[KM - 1])) return;
#pragma unroll
    for (int j = KM - 1; j > 0; --j) {
      const bool up = better(nv, ni, v[j - 1], i[j - 1]);
      const bool here = better(nv, ni, v[j], i[j]);
      const K pv = v[j - 1];
      const int32_t pi = i[j - 1];
      v[j] = up ? pv : (here ? nv : v[j]);
      i[j] = up ? pi : (here ? ni : i[j]);
    }
    if (better(nv, ni, v[0], i[0])) {
      v[0] = nv;
      i[0] = ni;
    }
  }
  __device__ void pop() {
#pragma unroll
    for (int j = 0; j < KM - 1; ++j) {
      v[j] = v[j + 1];
      i[j] = i[j + 1];
    }
    v[KM - 1] = Key<K>::lowest();
    i[KM - 1] = -1;
  }
};

template <typename K>
__device__ __forceinline__ K shfl_xor_key(K v, int off);
template <>
__device__ __forceinline__ float shfl_xor_key<float>(float v, int off) {
  return __shfl_xor(v, off, 64);
}
template <>
__device__ __forceinline__ int64_t shfl_xor_key<int64_t>(int64_t v, int off) {
  return (int64_t)__shfl_xor((long long)v, off, 64);
}

// k rounds of block-wide arg-max over list heads; thread 0 writes (out_v, out_i)[0..k)
template <typename K, int KM>
__device__ void block_extract(List<K, KM>& L, int k, K* out_v, int32_t* out_i) {
  __shared__ K sv[TPB / 64];
  __shared__ int32_t si[TPB / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int r = 0; r < k; ++r) {
    K bv = L.v[0];
    int32_t bi = L.i[0];
    for (int off = 32; off > 0; off >>= 1) {
      const K ov = shfl_xor_key<K>(bv, off);
      const int32_t oi = __shfl_xor(bi, off, 64);
      if (better(ov, oi, bv, bi)) {
        bv = ov;
        bi = oi;
      }
    }
    if (lane == 0) {
      sv[wid] = bv;
      si[wid] = bi;
    }
    __syncthreads();
    K wv = sv[0];
    int32_t wi = si[0];
    for (int w = 1; w < TPB / 64; ++w)
      if (better(sv[w], si[w], wv, wi)) {
        wv = sv[w];
        wi = si[w];
      }
    __syncthreads();
    if (threadIdx.x == 0) {
      out_v[r] = wv;
      out_i[r] = wi;
    }
    // the unique owner of (wv, wi) pops it (indices are unique, sentinels are -1)
    if (wi != -1 && L.i[0] == wi && L.v[0] == wv) L.pop();
  }
}

template <typename K, int KM>
__global__ __launch_bounds__(TPB) void topk_stage1(const K* __restrict__ v, int64_t N, int k, K* __restrict__ cv,
                                                   int32_t* __restrict__ ci) {
  List<K, KM> L;
  L.init();
  const int64_t stride = (int64_t)gridDim.x * TPB;
  for (int64_t j0 = (int64_t)blockIdx.x * TPB + threadIdx.x; j0 < N; j0 += stride * BATCH) {
    K bv[BATCH];  // the batch's loads are issued together, not one per (branchy) insert
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const int64_t j = j0 + u * stride;
      bv[u] = j < N ? v[j] : Key<K>::lowest();
    }
#pragma unroll
    for (int u = 0; u < BATCH; ++u)
      if (j0 + u * stride < N && Key<K>::valid(bv[u])) L.insert(bv[u], (int32_t)(j0 + u * stride));
  }
  block_extract<K, KM>(L, k, cv + (int64_t)blockIdx.x * k, ci + (int64_t)blockIdx.x * k);
}

template <typename K, int KM>
__global__ __launch_bounds__(TPB) void topk_stage2(const K* __restrict__ cv, const int32_t* __restrict__ ci,
                                                   int64_t M, int k, int32_t* __restrict__ idx,
                                                   K* __restrict__ val) {
  List<K, KM> L;
  L.init();
  for (int64_t j0 = threadIdx.x; j0 < M; j0 += TPB * BATCH) {
    K bv[BATCH];
    int32_t bi[BATCH];
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const int64_t j = j0 + u * TPB;
      bi[u] = j < M ? ci[j] : -1;
      bv[u] = j < M ? cv[j] : Key<K>::lowest();
    }
#pragma unroll
    for (int u = 0; u < BATCH; ++u)
      if (bi[u] != -1) L.insert(bv[u], bi[u]);
  }
  block_extract<K, KM>(L, k, val, idx);
}

int64_t stage1_blocks(int64_t N) { return std::max<int64_t>(1, std::min<int64_t>(krca::ceil_div(N, TPB * 8), 1024)); }

template <typename K>
int topk_impl(const K* v, int64_t N, int32_t k, void* ws, int32_t* idx, K* val, void* stream) {
  KRCA_CHECK_ARG(N >= 0 && N < (int64_t)INT32_MAX, "krca_topk: N out of range");
  KRCA_CHECK_ARG(k >= 1 && k <= KMAX, "krca_topk: k=%d must be in [1, %d]", k, KMAX);
  KRCA_CHECK_ARG(v && ws && idx && val, "krca_topk: null pointer");
  const int64_t G = stage1_blocks(N);
  K* cv = reinterpret_cast<K*>(ws);
  int32_t* ci = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(ws) + G * k * sizeof(int64_t));
  hipStream_t st = krca::as_stream(stream);
  if (k <= 10) {  // the insertion network sized to k: the stages are instruction-bound on it
    hipLaunchKernelGGL((topk_stage1<K, 10>), dim3((unsigned)G), dim3(TPB), 0, st, v, N, k, cv, ci);
    KRCA_LAUNCH_CHECK();
    hipLaunchKernelGGL((topk_stage2<K, 10>), dim3(1), dim3(TPB), 0, st, cv, ci, G * k, k, idx, val);
  } else {
    hipLaunchKernelGGL((topk_stage1<K, KMAX>), dim3((unsigned)G), dim3(TPB), 0, st, v, N, k, cv, ci);
    KRCA_LAUNCH_CHECK();
    hipLaunchKernelGGL((topk_stage2<K, KMAX>), dim3(1), dim3(TPB), 0, st, cv, ci, G * k, k, idx, val);
  }
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

}  // namespace

extern "C" {

int64_t krca_topk_workspace_size(int64_t N, int32_t k) {
  return stage1_blocks(N) * (int64_t)std::max(k, 1) * (int64_t)(sizeof(int64_t) + sizeof(int32_t)) + 256;
}

int krca_topk_f32(const float* v, int64_t N, int32_t k, void* ws, int32_t* idx, float* val, void* stream) {
  return topk_impl<float>(v, N, k, ws, idx, val, stream);
}

int krca_topk_i64(const int64_t* v, int64_t N, int32_t k, void* ws, int32_t* idx, int64_t* val, void* stream) {
  return topk_impl<int64_t>(v, N, k, ws, idx, val, stream);
}

}  // extern "C"

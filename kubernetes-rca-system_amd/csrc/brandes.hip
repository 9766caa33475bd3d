// Betweenness centrality for the single-point-of-failure check:
// TopologyAgent._analyze_single_points_of_failure (ref:agents/topology_agent.py:322-356) calls
// networkx 3.4.2 betweenness_centrality(G) (unweighted Brandes, endpoints excluded, normalized by
// 1/((n-1)(n-2)) for a directed graph).  Same algorithm and float64 formulas as networkx
// (sigma as float counts, coeff = (1 + delta[w]) / sigma[w], delta[v] += sigma[v] * coeff); the
// order of the dependency sum differs (successors in CSR order instead of stack-pop order), so
// values agree to rounding, and exactly whenever the sums are exact (small integer-valued cases).
//
// Work: one workgroup per source, a batch of B sources at a time.  Per source a level-synchronous
// BFS over the out-edge CSR (frontier in the source's global order list, dist claimed with
// atomicCAS, sigma added with float64 atomics: the values are integers < 2^53, so the sum is
// exact in any order); then levels deepest-first, each vertex pulling its dependency from its
// successors one level deeper in CSR order (deterministic).  delta_s lands in row b of a [B][N]
// buffer; a reduction kernel adds the rows in source order into bc (deterministic) and zeroes
// them for the next batch.  Only visited vertices are touched per source (dist is reset through
// the order list), so a source costs O(reached vertices + their edges).
#include <stdint.h>

#include "krca_common.h"

namespace {

constexpr int TPB = 256;

struct SrcScratch {  // per workgroup, reused for every source it takes
  int32_t* dist;     // [N], -1 = unvisited (kept -1 between sources)
  double* sigma;     // [N]
  double* delta;     // [N]
  int32_t* order;    // [N] visit order (level by level)
  int32_t* lvl;      // [N + 1] level start offsets into order
};

__device__ __forceinline__ SrcScratch scratch_of(char* base, int64_t N, int64_t wg) {
  const int64_t per = N * (4 + 8 + 8 + 4) + (N + 2) * 4;
  char* p = base + wg * ((per + 255) / 256 * 256);
  SrcScratch s;
  s.sigma = reinterpret_cast<double*>(p);
  s.delta = s.sigma + N;
  s.dist = reinterpret_cast<int32_t*>(s.delta + N);
  s.order = s.dist + N;
  s.lvl = s.order + N;
  return s;
}

__global__ __launch_bounds__(TPB) void brandes_sources(const int64_t* __restrict__ row_ptr,
                                                       const int32_t* __restrict__ col, int64_t N, int64_t s0,
                                                       int64_t nsrc, char* __restrict__ scratch,
                                                       double* __restrict__ dep /*[B][N]*/) {
  __shared__ int tail;
  __shared__ int nlev;
  const int tid = threadIdx.x;
  SrcScratch S = scratch_of(scratch, N, blockIdx.x);
  for (int64_t b = blockIdx.x; b < nsrc; b += gridDim.x) {
    const int32_t s = (int32_t)(s0 + b);
    if (tid == 0) {
      S.dist[s] = 0;
      S.sigma[s] = 1.0;
      S.delta[s] = 0.0;
      S.order[0] = s;
      S.lvl[0] = 0;
      S.lvl[1] = 1;
      tail = 1;
      nlev = 1;
    }
    __syncthreads();
    // BFS, one level per round: frontier = order[lvl[d] .. lvl[d+1])
    for (int d = 0;; ++d) {
      const int f0 = S.lvl[d], f1 = S.lvl[d + 1];
      if (f0 == f1) break;
      for (int i = f0 + tid; i < f1; i += TPB) {
        const int32_t u = S.order[i];
        const double su = S.sigma[u];
        for (int64_t e = row_ptr[u]; e < row_ptr[u + 1]; ++e) {
          const int32_t w = col[e];
          const int32_t old = atomicCAS(&S.dist[w], -1, d + 1);
          if (old == -1) {
            const int pos = atomicAdd(&tail, 1);
            S.order[pos] = w;
            S.delta[w] = 0.0;
          }
          if (old == -1 || old == d + 1) atomicAdd(&S.sigma[w], su);  // sigma[w] = 0 before: see reset
        }
      }
      __syncthreads();
      if (tid == 0) {
        S.lvl[d + 2] = tail;
        nlev = d + 2;
      }
      __syncthreads();
    }
    // dependencies, deepest level first; each vertex pulls from its successors in CSR order
    for (int d = nlev - 2; d >= 0; --d) {
      const int f0 = S.lvl[d], f1 = S.lvl[d + 1];
      for (int i = f0 + tid; i < f1; i += TPB) {
        const int32_t v = S.order[i];
        const double sv = S.sigma[v];
        double dv = 0.0;
        for (int64_t e = row_ptr[v]; e < row_ptr[v + 1]; ++e) {
          const int32_t w = col[e];
          if (S.dist[w] == d + 1) {
            const double coeff = (1.0 + S.delta[w]) / S.sigma[w];
            dv += sv * coeff;
          }
        }
        S.delta[v] = dv;
      }
      __syncthreads();
    }
    // export delta_s (source excluded), reset the visited entries for the next source
    const int nvis = S.lvl[nlev - 1];
    double* row = dep + b * N;
    for (int i = tid; i < nvis; i += TPB) {
      const int32_t v = S.order[i];
      if (v != s) row[v] = S.delta[v];
      S.dist[v] = -1;
      S.sigma[v] = 0.0;
    }
    __syncthreads();
  }
}

// bc[v] += sum_b dep[b][v] in source order; dep rows are zeroed for the next batch
__global__ __launch_bounds__(TPB) void brandes_reduce(double* __restrict__ dep, int64_t N, int64_t nsrc,
                                                      double* __restrict__ bc) {
  const int64_t v = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (v >= N) return;
  double acc = bc[v];
  for (int64_t b = 0; b < nsrc; ++b) {
    double* p = dep + b * N + v;
    acc += *p;
    *p = 0.0;
  }
  bc[v] = acc;
}

__global__ __launch_bounds__(TPB) void brandes_scale(double* __restrict__ bc, int64_t N, double scale) {
  const int64_t v = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (v < N) bc[v] *= scale;
}

__global__ __launch_bounds__(TPB) void brandes_init(char* __restrict__ scratch, int64_t N, int64_t nwg) {
  // dist = -1, sigma = 0 in every workgroup's scratch
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= N * nwg) return;
  SrcScratch S = scratch_of(scratch, N, i / N);
  S.dist[i % N] = -1;
  S.sigma[i % N] = 0.0;
}

}  // namespace

extern "C" {

// workspace bytes for batches of up to `batch` sources (one workgroup each)
int64_t krca_betweenness_ws_size(int64_t N, int32_t batch) {
  const int64_t per = N * (4 + 8 + 8 + 4) + (N + 2) * 4;
  return (int64_t)batch * ((per + 255) / 256 * 256) + (int64_t)batch * N * 8 + 256;
}

int krca_betweenness(const int64_t* row_ptr, const int32_t* col, int64_t N, int32_t normalized, int32_t directed,
                     int32_t batch, void* ws, double* bc, void* stream) {
  KRCA_CHECK_ARG(N >= 0 && N < INT32_MAX && batch >= 1, "krca_betweenness: bad sizes");
  hipStream_t st = krca::as_stream(stream);
  if (N == 0) return KRCA_OK;
  KRCA_CHECK_ARG(row_ptr && col && ws && bc, "krca_betweenness: null pointer");
  const int64_t B = std::min<int64_t>(batch, N);
  const int64_t per = N * (4 + 8 + 8 + 4) + (N + 2) * 4;
  char* scratch = reinterpret_cast<char*>(ws);
  double* dep = reinterpret_cast<double*>(scratch + B * ((per + 255) / 256 * 256));
  KRCA_HIP(hipMemsetAsync(bc, 0, N * sizeof(double), st));
  KRCA_HIP(hipMemsetAsync(dep, 0, B * N * sizeof(double), st));
  hipLaunchKernelGGL(brandes_init, dim3((unsigned)krca::ceil_div(N * B, TPB)), dim3(TPB), 0, st, scratch, N, B);
  KRCA_LAUNCH_CHECK();
  for (int64_t s0 = 0; s0 < N; s0 += B) {
    const int64_t nsrc = std::min<int64_t>(B, N - s0);
    hipLaunchKernelGGL(brandes_sources, dim3((unsigned)nsrc), dim3(TPB), 0, st, row_ptr, col, N, s0, nsrc, scratch,
                       dep);
    KRCA_LAUNCH_CHECK();
    hipLaunchKernelGGL(brandes_reduce, dim3((unsigned)krca::ceil_div(N, TPB)), dim3(TPB), 0, st, dep, N, nsrc, bc);
    KRCA_LAUNCH_CHECK();
  }
  // networkx _rescale: normalized -> 1/((n-1)(n-2)) (n > 2); unnormalized undirected -> 1/2
  double scale = 1.0;
  bool do_scale = false;
  if (normalized) {
    if (N > 2) {
      scale = 1.0 / ((double)(N - 1) * (double)(N - 2));
      do_scale = true;
    }
  } else if (!directed) {
    scale = 0.5;
    do_scale = true;
  }
  if (do_scale) {
    hipLaunchKernelGGL(brandes_scale, dim3((unsigned)krca::ceil_div(N, TPB)), dim3(TPB), 0, st, bc, N, scale);
    KRCA_LAUNCH_CHECK();
  }
  return KRCA_OK;
}

}  // extern "C"

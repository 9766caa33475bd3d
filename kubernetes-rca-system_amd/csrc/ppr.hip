// Personalized PageRank root-cause propagation.
//
// Semantics: networkx 3.4.2 pagerank (_pagerank_scipy) — x <- alpha*(x·A + D(x)·p) + (1-alpha)*p,
// A row-normalised by out-degree, dangling mass D(x) redistributed along the personalization p,
// x0 = 1/N, stop when sum|x - x_prev| < N*tol (tol <= 0: exactly max_iter iterations).
// Personalization p_i ∝ max(seed_i - seed_floor, 0) (uniform if every seed is at the floor).
//
// Determinism: the rank mass is held in int64 fixed point (1.0 == 2^60).  Per-node quantities
// that need a product or quotient are formed in float64 with a fixed expression and truncated
// to int64; every SUM (SpMV rows, dangling mass, residual, seed total) is an integer sum, so the
// result does not depend on the summation order, on atomics or on the number of GPUs, and is
// bit-identical to oracle/krca_oracle.c.
//
// Sharding: rank g of G owns the contiguous node range [g*n_max, ...) and the
// pull-CSR rows of those nodes.  Each iteration ends with ONE exchange: every rank's slice
// [w_local (n_max int64) | residual | dangling mass | seed total] is all-gathered (RCCL over
// xGMI, driven by the host: krca/rca.py) into w_all[G][n_max+3]; the column indices are
// pre-remapped to that layout (col' = j + 3*(j / n_max)), so the SpMV gathers directly.
// G = 1 is the same code with no collective (krca_ppr).
//
// SpMV (pull CSR, HBM-bound): CSR-adaptive row blocks from krca_ppr_plan —
//   short-row blocks: <= 2048 edges and <= 256 rows; the block gathers w[col[e]] for its edge
//                     range into LDS (coalesced col reads, lane per edge), then lane r sums row r
//                     from LDS ("LDS-staged row segments");
//   long rows:        split into 2048-edge chunks, each chunk block-reduced and added with one
//                     int64 atomic (order-free integer add).
#include <vector>

#include "krca_common.h"

#pragma clang fp contract(off)

namespace {

constexpr int TPB = 256;
constexpr int EDGE_BUDGET = 2048;  // edges per short block == LDS slots
constexpr int ROW_BUDGET = TPB;    // rows per short block
constexpr int NSLOT = 3;           // residual, dangling, seed total

struct Ctl {        // device control block
  double tele;      // (1-alpha)*2^60 + alpha*D   for the next update
  int64_t q_total;  // sum of quantised seeds over all ranks
  int32_t converged;  // iteration count at convergence (0 = running)
  int32_t iter;       // iterations done
  uint32_t ticket;    // arrival counter of the last-block reduction (0 between kernels)
};
constexpr int MAX_BLOCKS = 2048;  // grid cap of the node-parallel kernels (partials array size)
constexpr int CTL_BYTES = 256;    // Ctl, then int64 partials[2 * MAX_BLOCKS]

__device__ __forceinline__ int64_t* partials(Ctl* ctl) {
  return reinterpret_cast<int64_t*>(reinterpret_cast<char*>(ctl) + CTL_BYTES);
}

__device__ __forceinline__ int64_t block_sum_i64(int64_t v, int64_t* red) {
  for (int off = 32; off > 0; off >>= 1) v += (int64_t)__shfl_xor((long long)v, off, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  int64_t s = 0;
  if (threadIdx.x == 0)
    for (int w = 0; w < TPB / 64; ++w) s += red[w];
  __syncthreads();
  return s;  // valid in thread 0
}

__device__ __forceinline__ void add_slot(int64_t* slot, int64_t v) {
  atomicAdd(reinterpret_cast<unsigned long long*>(slot), (unsigned long long)v);
}

// Two block sums (a, b) reduced over the grid without contended atomics and without an L2
// write-back per block: lane 0 stores the block's pair write-through (relaxed agent-scope atomic
// store = global_store ... sc1, straight to memory), drains it (vmcnt(0)) and arrives on ONE
// ticket; the last arriver reads every pair with agent-scope atomic loads (sc1: bypass the
// non-coherent L1/L2 copies) and stores the totals (cdna_hip_programming.md split-K recipe,
// write-through form; integer sums are order-free anyway).
__device__ void grid_sum2(int64_t a, int64_t b, Ctl* ctl, int64_t* out, int64_t* red) {
  __shared__ int is_last;
  a = block_sum_i64(a, red);
  b = block_sum_i64(b, red);
  int64_t* part = partials(ctl);
  if (threadIdx.x == 0) {
    __hip_atomic_store(&part[2 * blockIdx.x], a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&part[2 * blockIdx.x + 1], b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(&ctl->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = (t == gridDim.x - 1);
  }
  __syncthreads();
  if (!is_last) return;
  int64_t sa = 0, sb = 0;
  for (int i = threadIdx.x; i < (int)gridDim.x; i += TPB) {
    sa += __hip_atomic_load(&part[2 * i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sb += __hip_atomic_load(&part[2 * i + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  sa = block_sum_i64(sa, red);
  sb = block_sum_i64(sb, red);
  if (threadIdx.x == 0) {
    out[0] = sa;
    out[1] = sb;
    ctl->ticket = 0;
  }
}

// w_j for node j given its fixed-point rank rj
__device__ __forceinline__ int64_t edge_weight(int64_t rj, int32_t deg, double alpha) {
  if (deg == 0) return 0;
  const double coef = alpha / (double)deg;
  return (int64_t)((double)rj * coef);
}

__device__ __forceinline__ int64_t quantise(float s, float floor_) {
  const double v = (double)s - (double)floor_;
  return v > 0.0 ? (int64_t)(v * 4294967296.0) : 0;
}

// r0 = floor(2^60/N), w0, seeds, partial slots (dangling mass, seed total)
__global__ __launch_bounds__(TPB) void ppr_init(const float* __restrict__ seed, float seed_floor,
                                                const int32_t* __restrict__ outdeg, int64_t n, int64_t N,
                                                double alpha, int64_t* __restrict__ q, int64_t* __restrict__ r,
                                                int64_t* __restrict__ send, int64_t n_max, Ctl* ctl) {
  __shared__ int64_t red[TPB / 64];
  const int64_t r0 = (int64_t)(krca::kFix / (double)N);
  int64_t dang = 0, qs = 0;
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    const int32_t deg = outdeg[i];
    const int64_t qi = quantise(seed[i], seed_floor);
    q[i] = qi;
    qs += qi;
    r[i] = r0;
    send[i] = edge_weight(r0, deg, alpha);
    if (deg == 0) dang += r0;
  }
  grid_sum2(dang, qs, ctl, send + n_max + 1, red);
}

__global__ __launch_bounds__(TPB) void ppr_spmv(const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
                                                const int32_t* __restrict__ plan, const int64_t* __restrict__ w,
                                                int64_t* __restrict__ acc, const Ctl* __restrict__ ctl) {
  constexpr int K = EDGE_BUDGET / TPB;  // edges per lane: all col loads, then all gathers, in flight
  __shared__ int64_t lds[EDGE_BUDGET];
  __shared__ int64_t red[TPB / 64];
  if (ctl->converged) return;
  const int32_t rb = plan[2 * blockIdx.x];
  const int32_t code = plan[2 * blockIdx.x + 1];
  int64_t e0, e1;
  if (code > 0) {
    e0 = row_ptr[rb];
    e1 = row_ptr[code];
  } else {
    e0 = row_ptr[rb] + (int64_t)(-code) * EDGE_BUDGET;
    e1 = std::min<int64_t>(row_ptr[rb + 1], e0 + EDGE_BUDGET);
  }
  int32_t c[K];
  int64_t v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int64_t e = e0 + threadIdx.x + k * TPB;
    c[k] = e < e1 ? col[e] : -1;
  }
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = c[k] >= 0 ? w[c[k]] : 0;
  if (code > 0) {  // short rows [rb, code): stage the gathered segment in LDS, lane r sums row r
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t e = threadIdx.x + k * TPB;
      if (e0 + e < e1) lds[e] = v[k];
    }
    __syncthreads();
    const int32_t row = rb + (int32_t)threadIdx.x;
    if (row < code) {
      const int64_t a = row_ptr[row] - e0, b = row_ptr[row + 1] - e0;
      int64_t s = 0;
      for (int64_t e = a; e < b; ++e) s += lds[e];
      acc[row] = s;
    }
  } else {  // chunk of long row rb (acc[rb] was zeroed by the previous update)
    int64_t s = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += v[k];
    const int64_t tot = block_sum_i64(s, red);
    if (threadIdx.x == 0) add_slot(&acc[rb], tot);
  }
}

__global__ __launch_bounds__(TPB) void ppr_update(const int32_t* __restrict__ outdeg, const int64_t* __restrict__ q,
                                                  int64_t n, int64_t N, double alpha, int64_t* __restrict__ r,
                                                  int64_t* __restrict__ acc, int64_t* __restrict__ send,
                                                  int64_t n_max, Ctl* ctl) {
  __shared__ int64_t red[TPB / 64];
  if (ctl->converged) return;
  const double tele = ctl->tele;
  const int64_t qt = ctl->q_total;
  const double qtot = (double)qt;
  const double uni = 1.0 / (double)N;
  int64_t err = 0, dang = 0;
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    const double pd = qt > 0 ? (double)q[i] / qtot : uni;
    const int64_t t = (int64_t)(pd * tele);
    const int64_t rn = acc[i] + t;
    acc[i] = 0;
    const int64_t ro = r[i];
    r[i] = rn;
    err += rn > ro ? rn - ro : ro - rn;
    const int32_t deg = outdeg[i];
    if (deg == 0) dang += rn;
    send[i] = edge_weight(rn, deg, alpha);
  }
  grid_sum2(err, dang, ctl, send + n_max, red);
}

// one lane: sum the G gathered partial slots (integer -> order-free), decide convergence,
// set the teleport scale of the next update, zero this rank's send slots
__global__ void ppr_reduce(const int64_t* __restrict__ w_all, int32_t G, int64_t n_max, double alpha,
                           double err_limit, int first, Ctl* ctl, int64_t* __restrict__ send) {
  int64_t err = 0, dang = 0, qs = 0;
  for (int g = 0; g < G; ++g) {
    const int64_t* s = w_all + (int64_t)g * (n_max + NSLOT) + n_max;
    err += s[0];
    dang += s[1];
    qs += s[2];
  }
  send[n_max] = 0;
  send[n_max + 1] = 0;
  send[n_max + 2] = 0;
  if (ctl->converged) return;
  if (first) {
    ctl->q_total = qs;
  } else {
    ctl->iter += 1;
    if (err_limit > 0.0 && (double)err < err_limit) {
      ctl->converged = ctl->iter;
      return;
    }
  }
  ctl->tele = (1.0 - alpha) * krca::kFix + alpha * (double)dang;
}

__global__ __launch_bounds__(TPB) void ppr_to_float(const int64_t* __restrict__ r, int64_t n, float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB)
    out[i] = (float)((double)r[i] * (1.0 / krca::kFix));
}

// root-cause key: the bits of (double)r_i * (double)q_i (non-negative doubles order like int64)
__global__ __launch_bounds__(TPB) void ppr_rca_key(const int64_t* __restrict__ r, const int64_t* __restrict__ q,
                                                   int64_t n, int64_t* __restrict__ key) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    const double v = (double)r[i] * (double)q[i];
    key[i] = __double_as_longlong(v);
  }
}

__global__ __launch_bounds__(TPB) void remap_cols(const int32_t* __restrict__ col, int64_t E, int64_t n_max,
                                                  int32_t* __restrict__ out) {
  for (int64_t e = (int64_t)blockIdx.x * TPB + threadIdx.x; e < E; e += (int64_t)gridDim.x * TPB) {
    const int64_t j = col[e];
    out[e] = (int32_t)(j + NSLOT * (j / n_max));
  }
}

// host: CSR-adaptive row blocks; returns the number of int32 entries (2 per block)
int64_t build_plan(const int64_t* rp, int64_t N, int32_t* out) {
  int64_t n = 0;
  int64_t r = 0;
  while (r < N) {
    const int64_t deg = rp[r + 1] - rp[r];
    if (deg > EDGE_BUDGET) {
      const int64_t chunks = krca::ceil_div(deg, EDGE_BUDGET);
      for (int64_t c = 0; c < chunks; ++c) {
        if (out) {
          out[n] = (int32_t)r;
          out[n + 1] = (int32_t)(-c);  // chunk 0 encodes as 0 (<= 0 means long-row chunk)
        }
        n += 2;
      }
      r += 1;
      continue;
    }
    int64_t re = r + 1;
    while (re < N && re - r < ROW_BUDGET && rp[re + 1] - rp[r] <= EDGE_BUDGET) ++re;
    if (out) {
      out[n] = (int32_t)r;
      out[n + 1] = (int32_t)re;
    }
    n += 2;
    r = re;
  }
  return n;
}

unsigned grid_for(int64_t n) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(krca::ceil_div(n, TPB), MAX_BLOCKS));
}

}  // namespace

extern "C" {

int64_t krca_ppr_plan_size(const int64_t* row_ptr_host, int64_t N) {
  if (!row_ptr_host || N <= 0) return 0;
  return build_plan(row_ptr_host, N, nullptr);
}

int krca_ppr_plan(const int64_t* row_ptr_host, int64_t N, int32_t* plan_host, int64_t plan_len) {
  KRCA_CHECK_ARG(row_ptr_host && plan_host && N > 0 && N < INT32_MAX, "krca_ppr_plan: bad arguments");
  for (int64_t i = 0; i < N; ++i)
    KRCA_CHECK_ARG(row_ptr_host[i + 1] >= row_ptr_host[i], "krca_ppr_plan: row_ptr not monotone at %lld", (long long)i);
  const int64_t need = build_plan(row_ptr_host, N, nullptr);
  KRCA_CHECK_ARG(plan_len == need, "krca_ppr_plan: plan_len %lld != %lld", (long long)plan_len, (long long)need);
  build_plan(row_ptr_host, N, plan_host);
  return KRCA_OK;
}

int64_t krca_ppr_ctl_size(void) { return CTL_BYTES + 16 * MAX_BLOCKS; }

int krca_ppr_remap_cols(const int32_t* col, int64_t E, int64_t n_max, int32_t* out, void* stream) {
  KRCA_CHECK_ARG(E >= 0 && n_max > 0, "krca_ppr_remap_cols: bad sizes");
  if (E == 0) return KRCA_OK;
  KRCA_CHECK_ARG(col && out, "krca_ppr_remap_cols: null pointer");
  hipLaunchKernelGGL(remap_cols, dim3(grid_for(E)), dim3(TPB), 0, krca::as_stream(stream), col, E, n_max, out);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_ppr_shard_init(const float* seed, float seed_floor, const int32_t* outdeg, int64_t n_local, int64_t n_max,
                        int64_t N, double alpha, void* ctl, int64_t* q_local, int64_t* r_local, int64_t* send,
                        void* stream) {
  KRCA_CHECK_ARG(N > 0 && N < INT32_MAX && n_local >= 0 && n_local <= n_max, "krca_ppr_shard_init: bad sizes");
  KRCA_CHECK_ARG(alpha > 0.0 && alpha < 1.0, "krca_ppr_shard_init: alpha must be in (0, 1)");
  KRCA_CHECK_ARG(ctl && send && (n_local == 0 || (seed && outdeg && q_local && r_local)), "krca_ppr_shard_init: null pointer");
  hipStream_t st = krca::as_stream(stream);
  KRCA_HIP(hipMemsetAsync(ctl, 0, sizeof(Ctl), st));
  KRCA_HIP(hipMemsetAsync(send + n_max, 0, NSLOT * sizeof(int64_t), st));  // residual slot stays 0
  hipLaunchKernelGGL(ppr_init, dim3(grid_for(n_local)), dim3(TPB), 0, st, seed, seed_floor, outdeg, n_local, N, alpha,
                     q_local, r_local, send, n_max, reinterpret_cast<Ctl*>(ctl));
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_ppr_shard_spmv(const int64_t* row_ptr, const int32_t* col, const int32_t* plan, int64_t plan_len,
                        const int64_t* w_all, int64_t* acc, const void* ctl, void* stream) {
  KRCA_CHECK_ARG(plan_len >= 0 && plan_len % 2 == 0, "krca_ppr_shard_spmv: bad plan");
  if (plan_len == 0) return KRCA_OK;
  KRCA_CHECK_ARG(row_ptr && col && plan && w_all && acc && ctl, "krca_ppr_shard_spmv: null pointer");
  hipLaunchKernelGGL(ppr_spmv, dim3((unsigned)(plan_len / 2)), dim3(TPB), 0, krca::as_stream(stream), row_ptr, col,
                     plan, w_all, acc, reinterpret_cast<const Ctl*>(ctl));
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_ppr_shard_update(const int32_t* outdeg, const int64_t* q_local, int64_t n_local, int64_t n_max, int64_t N,
                          double alpha, int64_t* r_local, int64_t* acc, int64_t* send, void* ctl, void* stream) {
  KRCA_CHECK_ARG(n_local >= 0 && n_local <= n_max && N > 0, "krca_ppr_shard_update: bad sizes");
  KRCA_CHECK_ARG(send && ctl && (n_local == 0 || (outdeg && q_local && r_local && acc)), "krca_ppr_shard_update: null pointer");
  hipLaunchKernelGGL(ppr_update, dim3(grid_for(n_local)), dim3(TPB), 0, krca::as_stream(stream), outdeg, q_local,
                     n_local, N, alpha, r_local, acc, send, n_max, reinterpret_cast<Ctl*>(ctl));
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_ppr_shard_reduce(const int64_t* w_all, int32_t G, int64_t n_max, int64_t N, double alpha, double tol,
                          int32_t first, void* ctl, int64_t* send, void* stream) {
  KRCA_CHECK_ARG(G >= 1 && n_max > 0 && N > 0, "krca_ppr_shard_reduce: bad sizes");
  KRCA_CHECK_ARG(w_all && ctl && send, "krca_ppr_shard_reduce: null pointer");
  const double err_limit = tol > 0.0 ? (double)N * tol * krca::kFix : 0.0;
  hipLaunchKernelGGL(ppr_reduce, dim3(1), dim3(1), 0, krca::as_stream(stream), w_all, G, n_max, alpha, err_limit,
                     (int)first, reinterpret_cast<Ctl*>(ctl), send);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_ppr_ctl_read(const void* ctl, int32_t* iters_host, int32_t* converged_host, void* stream) {
  KRCA_CHECK_ARG(ctl && iters_host && converged_host, "krca_ppr_ctl_read: null pointer");
  Ctl h{};
  hipStream_t st = krca::as_stream(stream);
  KRCA_HIP(hipMemcpyAsync(&h, ctl, sizeof(Ctl), hipMemcpyDeviceToHost, st));
  KRCA_HIP(hipStreamSynchronize(st));
  *iters_host = h.converged ? h.converged : h.iter;
  *converged_host = h.converged;
  return KRCA_OK;
}

int krca_ppr_fixed_to_float(const int64_t* r, int64_t n, float* out, void* stream) {
  if (n <= 0) return KRCA_OK;
  KRCA_CHECK_ARG(r && out, "krca_ppr_fixed_to_float: null pointer");
  hipLaunchKernelGGL(ppr_to_float, dim3(grid_for(n)), dim3(TPB), 0, krca::as_stream(stream), r, n, out);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_ppr_rca_key(const int64_t* r, const int64_t* q, int64_t n, int64_t* key, void* stream) {
  if (n <= 0) return KRCA_OK;
  KRCA_CHECK_ARG(r && q && key, "krca_ppr_rca_key: null pointer");
  hipLaunchKernelGGL(ppr_rca_key, dim3(grid_for(n)), dim3(TPB), 0, krca::as_stream(stream), r, q, n, key);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

// workspace: ctl (krca_ppr_ctl_size) | q[N] | acc[N] | send/w_all[N+3] | r (if r_fixed == NULL) [N]
int64_t krca_ppr_workspace_size(int64_t N) { return krca_ppr_ctl_size() + (4 * N + NSLOT) * 8 + 256; }

int krca_ppr(const int64_t* row_ptr, const int32_t* col, const int32_t* outdeg, int64_t N, const int32_t* plan,
             int64_t plan_len, const float* seed, float seed_floor, double alpha, int32_t max_iter, double tol,
             void* workspace, float* r_out, int64_t* r_fixed, int64_t* q_out, int32_t* iters_host, void* stream) {
  KRCA_CHECK_ARG(N > 0 && N < INT32_MAX, "krca_ppr: N=%lld out of range", (long long)N);
  KRCA_CHECK_ARG(row_ptr && col && outdeg && plan && seed && workspace && r_out, "krca_ppr: null pointer");
  KRCA_CHECK_ARG(plan_len > 0 && plan_len % 2 == 0, "krca_ppr: bad plan");
  KRCA_CHECK_ARG(alpha > 0.0 && alpha < 1.0 && max_iter > 0, "krca_ppr: alpha in (0,1), max_iter > 0");
  char* ctl = reinterpret_cast<char*>(workspace);
  char* p = ctl + krca_ppr_ctl_size();
  int64_t* q = q_out ? q_out : reinterpret_cast<int64_t*>(p);
  int64_t* acc = reinterpret_cast<int64_t*>(p + N * 8);
  int64_t* w = reinterpret_cast<int64_t*>(p + 2 * N * 8);
  int64_t* r = r_fixed ? r_fixed : reinterpret_cast<int64_t*>(p + (3 * N + NSLOT) * 8);
  hipStream_t st = krca::as_stream(stream);
  KRCA_HIP(hipMemsetAsync(acc, 0, N * 8, st));
  int rc = krca_ppr_shard_init(seed, seed_floor, outdeg, N, N, N, alpha, ctl, q, r, w, stream);
  if (rc) return rc;
  if ((rc = krca_ppr_shard_reduce(w, 1, N, N, alpha, tol, 1, ctl, w, stream))) return rc;
  const int check_every = 8;
  int32_t iters = 0, conv = 0;
  for (int it = 0; it < max_iter; ++it) {
    if ((rc = krca_ppr_shard_spmv(row_ptr, col, plan, plan_len, w, acc, ctl, stream))) return rc;
    if ((rc = krca_ppr_shard_update(outdeg, q, N, N, N, alpha, r, acc, w, ctl, stream))) return rc;
    if ((rc = krca_ppr_shard_reduce(w, 1, N, N, alpha, tol, 0, ctl, w, stream))) return rc;
    if (tol > 0.0 && (it + 1) % check_every == 0 && it + 1 < max_iter) {
      if ((rc = krca_ppr_ctl_read(ctl, &iters, &conv, stream))) return rc;
      if (conv) break;
    }
  }
  if ((rc = krca_ppr_fixed_to_float(r, N, r_out, stream))) return rc;
  if ((rc = krca_ppr_ctl_read(ctl, &iters, &conv, stream))) return rc;
  if (iters_host) *iters_host = iters;
  if (tol > 0.0 && !conv) {
    krca::set_error("krca_ppr: no convergence in %d iterations", max_iter);
    return KRCA_ENOTCONV;
  }
  return KRCA_OK;
}

}  // extern "C"

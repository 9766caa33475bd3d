// Personalized PageRank root-cause propagation.
//
// Semantics: networkx 3.4.2 pagerank (_pagerank_scipy) — x <- alpha*(x·A + D(x)·p) + (1-alpha)*p,
// A row-normalised by out-degree, dangling mass D(x) redistributed along the personalization p,
// x0 = 1/N, stop when sum|x - x_prev| < N*tol (tol <= 0: exactly max_iter iterations).
//
// Determinism: the rank mass is held in int64 fixed point (1.0 == 2^60).  Per-node quantities
// that need a product or quotient are formed in float64 with a fixed expression and truncated
// to int64; every SUM (SpMV rows, dangling mass, residual, seed total) is an integer sum, so the
// result does not depend on the summation order, on atomics or on the number of GPUs, and is
// bit-identical to oracle/krca_oracle.c.
//
// SpMV (pull CSR, HBM-bound): CSR-adaptive row blocks from krca_ppr_plan —
//   short-row blocks: <= 2048 edges and <= 256 rows; the block gathers w[col[e]] for its edge
//                     range into LDS (coalesced col reads, lane per edge), then lane r sums row r
//                     from LDS ("LDS-staged row segments");
//   long rows:        split into 2048-edge chunks, each chunk block-reduced and added with one
//                     int64 atomic (order-free integer add).
// Per iteration: spmv -> update (r, residual, dangling mass, next w; fused) -> finalize (1 lane).
#include <vector>

#include "krca_common.h"

#pragma clang fp contract(off)

namespace {

constexpr int TPB = 256;
constexpr int EDGE_BUDGET = 2048;  // edges per short block == LDS slots
constexpr int ROW_BUDGET = TPB;    // rows per short block

struct Ctl {  // device control block (in the workspace)
  double tele;          // (1-alpha)*2^60 + alpha*D   for the current iteration
  int64_t acc_err;      // residual accumulator
  int64_t acc_dangle;   // dangling-mass accumulator
  int64_t q_total;      // sum of quantised seeds
  int32_t converged;    // iteration count at convergence (0 = running)
  int32_t iter;         // iterations done
};

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

// w_j for node j given its fixed-point rank rj
__device__ __forceinline__ int64_t edge_weight(int64_t rj, int32_t deg, double alpha) {
  if (deg == 0) return 0;
  const double coef = alpha / (double)deg;
  return (int64_t)((double)rj * coef);
}

__global__ __launch_bounds__(TPB) void ppr_seed_quant(const float* __restrict__ seed, int64_t N,
                                                      int64_t* __restrict__ q, Ctl* ctl) {
  __shared__ int64_t red[TPB / 64];
  int64_t local = 0;
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < N; i += (int64_t)gridDim.x * TPB) {
    const float s = seed[i];
    const int64_t qi = (s > 0.f) ? (int64_t)((double)s * 4294967296.0) : 0;
    q[i] = qi;
    local += qi;
  }
  const int64_t tot = block_sum_i64(local, red);
  if (threadIdx.x == 0) atomicAdd((unsigned long long*)&ctl->q_total, (unsigned long long)tot);
}

// r0 = floor(2^60/N) everywhere, w0, dangling mass D0
__global__ __launch_bounds__(TPB) void ppr_init(const int32_t* __restrict__ outdeg, int64_t N, double alpha,
                                                int64_t* __restrict__ r, int64_t* __restrict__ w,
                                                int64_t* __restrict__ acc, Ctl* ctl) {
  __shared__ int64_t red[TPB / 64];
  const int64_t r0 = (int64_t)(krca::kFix / (double)N);
  int64_t dang = 0;
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < N; i += (int64_t)gridDim.x * TPB) {
    const int32_t deg = outdeg[i];
    r[i] = r0;
    w[i] = edge_weight(r0, deg, alpha);
    acc[i] = 0;
    if (deg == 0) dang += r0;
  }
  const int64_t tot = block_sum_i64(dang, red);
  if (threadIdx.x == 0) atomicAdd((unsigned long long*)&ctl->acc_dangle, (unsigned long long)tot);
}

// one lane: consume accumulators, decide convergence, set the teleport scale of the next iteration
__global__ void ppr_finalize(Ctl* ctl, double alpha, double err_limit, int first) {
  if (ctl->converged) return;
  const int64_t err = ctl->acc_err;
  const int64_t dang = ctl->acc_dangle;
  ctl->acc_err = 0;
  ctl->acc_dangle = 0;
  if (!first) {
    ctl->iter += 1;
    if (err_limit > 0.0 && (double)err < err_limit) {
      ctl->converged = ctl->iter;
      return;
    }
  }
  ctl->tele = (1.0 - alpha) * krca::kFix + alpha * (double)dang;
}

__global__ __launch_bounds__(TPB) void ppr_spmv(const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
                                                const int32_t* __restrict__ plan, const int64_t* __restrict__ w,
                                                int64_t* __restrict__ acc, const Ctl* __restrict__ ctl) {
  __shared__ int64_t lds[EDGE_BUDGET];
  __shared__ int64_t red[TPB / 64];
  if (ctl->converged) return;
  const int32_t rb = plan[2 * blockIdx.x];
  const int32_t code = plan[2 * blockIdx.x + 1];
  if (code > 0) {  // short rows [rb, code)
    const int32_t re = code;
    const int64_t e0 = row_ptr[rb], e1 = row_ptr[re];
    for (int64_t e = e0 + threadIdx.x; e < e1; e += TPB) lds[e - e0] = w[col[e]];
    __syncthreads();
    const int32_t row = rb + (int32_t)threadIdx.x;
    if (row < re) {
      const int64_t a = row_ptr[row] - e0, b = row_ptr[row + 1] - e0;
      int64_t s = 0;
      for (int64_t e = a; e < b; ++e) s += lds[e];
      acc[row] = s;
    }
  } else {  // chunk -code of long row rb
    const int64_t c = -(int64_t)code;
    const int64_t r0 = row_ptr[rb], r1 = row_ptr[rb + 1];
    const int64_t e0 = r0 + c * EDGE_BUDGET;
    const int64_t e1 = std::min<int64_t>(r1, e0 + EDGE_BUDGET);
    int64_t s = 0;
    for (int64_t e = e0 + threadIdx.x; e < e1; e += TPB) s += w[col[e]];
    const int64_t tot = block_sum_i64(s, red);
    if (threadIdx.x == 0) atomicAdd((unsigned long long*)&acc[rb], (unsigned long long)tot);
  }
}

__global__ __launch_bounds__(TPB) void ppr_update(const int32_t* __restrict__ outdeg, const int64_t* __restrict__ q,
                                                  int64_t N, double alpha, int64_t* __restrict__ r,
                                                  int64_t* __restrict__ w, int64_t* __restrict__ acc, Ctl* ctl) {
  __shared__ int64_t red[TPB / 64];
  if (ctl->converged) return;
  const double tele = ctl->tele;
  const double qtot = (double)ctl->q_total;
  int64_t err = 0, dang = 0;
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < N; i += (int64_t)gridDim.x * TPB) {
    const double pd = (double)q[i] / qtot;
    const int64_t t = (int64_t)(pd * tele);
    const int64_t rn = acc[i] + t;
    acc[i] = 0;
    const int64_t ro = r[i];
    r[i] = rn;
    err += rn > ro ? rn - ro : ro - rn;
    const int32_t deg = outdeg[i];
    if (deg == 0) dang += rn;
    w[i] = edge_weight(rn, deg, alpha);
  }
  int64_t tot = block_sum_i64(err, red);
  if (threadIdx.x == 0) atomicAdd((unsigned long long*)&ctl->acc_err, (unsigned long long)tot);
  tot = block_sum_i64(dang, red);
  if (threadIdx.x == 0) atomicAdd((unsigned long long*)&ctl->acc_dangle, (unsigned long long)tot);
}

__global__ __launch_bounds__(TPB) void ppr_to_float(const int64_t* __restrict__ r, int64_t N, float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < N; i += (int64_t)gridDim.x * TPB)
    out[i] = (float)((double)r[i] * (1.0 / krca::kFix));
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

struct Workspace {
  Ctl* ctl;
  int64_t* q;
  int64_t* w;
  int64_t* acc;
  int64_t* rfix;
};

Workspace carve(void* ws, int64_t N) {
  char* p = reinterpret_cast<char*>(ws);
  Workspace W;
  W.ctl = reinterpret_cast<Ctl*>(p);
  p += 256;
  W.q = reinterpret_cast<int64_t*>(p);
  p += N * 8;
  W.w = reinterpret_cast<int64_t*>(p);
  p += N * 8;
  W.acc = reinterpret_cast<int64_t*>(p);
  p += N * 8;
  W.rfix = reinterpret_cast<int64_t*>(p);
  return W;
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

int64_t krca_ppr_workspace_size(int64_t N) { return 256 + 4 * N * 8 + 256; }

int krca_ppr(const int64_t* row_ptr, const int32_t* col, const int32_t* outdeg, int64_t N, const int32_t* plan,
             int64_t plan_len, const float* seed, double alpha, int32_t max_iter, double tol, void* workspace,
             float* r_out, int64_t* r_fixed, int32_t* iters_host, void* stream) {
  KRCA_CHECK_ARG(N > 0 && N < INT32_MAX, "krca_ppr: N=%lld out of range", (long long)N);
  KRCA_CHECK_ARG(row_ptr && col && outdeg && plan && seed && workspace && r_out, "krca_ppr: null pointer");
  KRCA_CHECK_ARG(plan_len > 0 && plan_len % 2 == 0, "krca_ppr: bad plan");
  KRCA_CHECK_ARG(alpha > 0.0 && alpha < 1.0 && max_iter > 0, "krca_ppr: alpha in (0,1), max_iter > 0");
  hipStream_t st = krca::as_stream(stream);
  Workspace W = carve(workspace, N);
  int64_t* r = r_fixed ? r_fixed : W.rfix;
  const unsigned gN = (unsigned)std::min<int64_t>(krca::ceil_div(N, TPB), 2048);
  const unsigned nblk = (unsigned)(plan_len / 2);
  const double err_limit = tol > 0.0 ? (double)N * tol * krca::kFix : 0.0;

  KRCA_HIP(hipMemsetAsync(W.ctl, 0, sizeof(Ctl), st));
  hipLaunchKernelGGL(ppr_seed_quant, dim3(gN), dim3(TPB), 0, st, seed, N, W.q, W.ctl);
  hipLaunchKernelGGL(ppr_init, dim3(gN), dim3(TPB), 0, st, outdeg, N, alpha, r, W.w, W.acc, W.ctl);
  hipLaunchKernelGGL(ppr_finalize, dim3(1), dim3(1), 0, st, W.ctl, alpha, err_limit, 1);
  KRCA_LAUNCH_CHECK();
  Ctl host{};
  const int check_every = 8;
  int it = 0;
  for (; it < max_iter; ++it) {
    hipLaunchKernelGGL(ppr_spmv, dim3(nblk), dim3(TPB), 0, st, row_ptr, col, plan, W.w, W.acc, W.ctl);
    hipLaunchKernelGGL(ppr_update, dim3(gN), dim3(TPB), 0, st, outdeg, W.q, N, alpha, r, W.w, W.acc, W.ctl);
    hipLaunchKernelGGL(ppr_finalize, dim3(1), dim3(1), 0, st, W.ctl, alpha, err_limit, 0);
    KRCA_LAUNCH_CHECK();
    if (err_limit > 0.0 && ((it + 1) % check_every == 0) && it + 1 < max_iter) {
      KRCA_HIP(hipMemcpyAsync(&host, W.ctl, sizeof(Ctl), hipMemcpyDeviceToHost, st));
      KRCA_HIP(hipStreamSynchronize(st));
      if (host.converged) break;
    }
  }
  hipLaunchKernelGGL(ppr_to_float, dim3(gN), dim3(TPB), 0, st, r, N, r_out);
  KRCA_LAUNCH_CHECK();
  KRCA_HIP(hipMemcpyAsync(&host, W.ctl, sizeof(Ctl), hipMemcpyDeviceToHost, st));
  KRCA_HIP(hipStreamSynchronize(st));
  if (iters_host) *iters_host = host.converged ? host.converged : host.iter;
  if (err_limit > 0.0 && !host.converged) {
    krca::set_error("krca_ppr: no convergence in %d iterations", max_iter);
    return KRCA_ENOTCONV;
  }
  return KRCA_OK;
}

}  // extern "C"

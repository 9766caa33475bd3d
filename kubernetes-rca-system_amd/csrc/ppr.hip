// Personalized PageRank root-cause propagation.
//
// Semantics: networkx 3.4.2 pagerank (_pagerank_scipy) — x <- alpha*(x·A + D(x)·p) + (1-alpha)*p,
// A row-normalised by out-degree, dangling mass D(x) redistributed along the personalization p,
// x0 = 1/N, stop when sum|x - x_prev| < N*tol (tol <= 0: exactly max_iter iterations).
// Personalization p_i ∝ max(seed_i - seed_floor, 0) (uniform if every seed is at the floor).
//
// Determinism: the rank mass is held in int64 fixed point (1.0 == 2^60).  Per-node quantities
// that need a product or quotient are formed in float64 with a fixed expression and truncated
// to int64; every SUM (pulled row mass, dangling mass, residual, seed total) is an integer sum,
// so the result does not depend on the summation order, on atomics or on the number of GPUs,
// and is bit-identical to oracle/krca_oracle.c.
//
// Gathered weights: w_j = floor(r_j * alpha / outdeg_j) is stored as a 32-bit code (wenc: 26
// significant bits and a 6-bit shift, truncating; wdec restores the int64 it stands for), so the
// table every row gathers from is 4 bytes per node: at C4 (1M pods) 4 MB, the size of one XCD's
// L2, instead of 8 MB.  The rank update still sums int64 (the decoded codes), so sums stay exact
// and order-free; oracle/krca_oracle.c applies the same code.  Relative rounding <= 2^-25 per
// weight (networkx parity is asserted at 1e-5).
//
// Sharding: rank g of G owns the contiguous node range [g*n_max, ...) and the
// pull-CSR rows of those nodes.  Each iteration ends with ONE exchange: every rank's slice of
// krca_ppr_slice_words(n_max) int64 words — [codes (n_max uint32, padded to 8 bytes) | NSLOT
// partial-sum slots] — is all-gathered (RCCL over xGMI, driven by the host: krca/rca.py) into
// w_all[G][slice]; the column indices are pre-remapped to that layout in uint32 units (col' = j +
// (j / n_max) * (2 * slice - n_max)), so the step kernel gathers directly.  At G = 1 the
// "exchange" is a swap of two such buffers (ping-pong), no copy.
//
// One iteration = ppr_step (pull SpMV fused with the rank update) + ppr_reduce (one block), or --
// the default of krca/rca.py -- one folded ppr_step that first does the previous step's reduction
// itself (Fold: every workgroup sums the previous slot set; three rotating sets in the payload).
//   ppr_step, short-row blocks (<= 2048 edges, <= 256 rows, from krca_ppr_plan): coalesced col
//     loads and 8 independent w[col] gathers per lane (lane-strided), staged in LDS; each lane
//     then sums 8 CONTIGUOUS staged edges as row segments (binary search of its first row in the
//     LDS row offsets, int64 LDS atomics at row boundaries), so a 1800-edge hub row costs no more
//     than 1800 one-edge rows; lane r then updates row r (teleport, residual, next w).
//   ppr_step, long rows (> 2048 edges): 2048-edge chunks, block sum, one agent-scope int64 atomic
//     into the row's accumulator and a per-row ticket; the last chunk to arrive updates the row.
//   Residual / dangling mass: one int64 atomic per block into NSPREAD slots of the send tail, so
//     the partial sums ride the same all-gather; ppr_reduce sums G*NSPREAD slots.
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "krca_common.h"
#include "ppr_layout.h"

#pragma clang fp contract(off)

namespace {
using namespace pprl;

constexpr int PPR_RESIDUAL = KRCA_PPR_RESIDUAL;
constexpr int PPR_WRITE_R = KRCA_PPR_WRITE_R;
constexpr int PPR_NT = 4;  // stream the plan / column / row arrays with non-temporal loads (KRCA_PPR_NT)

// a load of streamed data: non-temporal when NT, so it does not evict the gathered code table
// from the XCD's L2
template <bool NT, class T>
__device__ __forceinline__ T ld_stream(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

struct Ctl {          // device control block (header of the ctl buffer)
  double tele;        // (1-alpha)*2^60 + alpha*D   for the next step
  int64_t q_total;    // sum of quantised seeds over all ranks
  int32_t converged;  // iteration count at convergence (0 = running)
  int32_t iter;       // iterations done
  uint32_t done;      // single device, reduction fused: workgroups of the running step that finished
  double tele_used;   // the teleport scale of the last step that updated the rows (written by its
                      // workgroup 0): krca_rca_key_explained recovers each row's received mass as
                      // r_i - t_i with the same t_i
};
// ctl buffer: Ctl header (CTL_BYTES) | int64 acc_long[n] | uint32 ticket[n] (8-byte slots) | {double coef, double q}[n].  The long-row
// accumulators and tickets are zero when allocated and reset by the last chunk of each row.

__device__ __forceinline__ int64_t* acc_long_of(Ctl* ctl) {
  return reinterpret_cast<int64_t*>(reinterpret_cast<char*>(ctl) + CTL_BYTES);
}
__device__ __forceinline__ uint32_t* ticket_of(Ctl* ctl, int64_t n) {
  return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(ctl) + CTL_BYTES + 8 * n);
}
// per-row pair {edge coefficient alpha / outdeg (0 for a dangling row), seed q_i as a double},
// written by the solve's init: the step multiplies instead of dividing per row and iteration, and
// loads both with one 16-byte read and no int64 -> double conversion ((double)q_i is exact: q_i <
// 2^53)
static_assert(CTL_BYTES % 16 == 0, "16-byte row pairs");
__device__ __forceinline__ double* coef_of(Ctl* ctl, int64_t n) {
  return reinterpret_cast<double*>(reinterpret_cast<char*>(ctl) + CTL_BYTES + 16 * n);
}

__device__ __forceinline__ int64_t block_sum_i64(int64_t v, int64_t* red) {
  for (int off = 32; off > 0; off >>= 1) v += (int64_t)__shfl_xor((long long)v, off, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();  // red may still be read by a previous call
  if (lane == 0) red[wid] = v;
  __syncthreads();
  int64_t s = 0;
  if (threadIdx.x == 0)
    for (int w = 0; w < TPB / 64; ++w) s += red[w];
  return s;  // valid in thread 0
}

// one int64 atomic per block into one of NSPREAD slots (integer: order-free)
__device__ __forceinline__ void add_slot(int64_t* slots, int64_t v) {
  if (v)
    atomicAdd(reinterpret_cast<unsigned long long*>(slots + (blockIdx.x & (NSPREAD - 1))), (unsigned long long)v);
}

// w_j for node j given its fixed-point rank rj
__device__ __forceinline__ int64_t edge_weight(int64_t rj, int32_t deg, double alpha) {
  if (deg == 0) return 0;
  const double coef = alpha / (double)deg;
  return (int64_t)((double)rj * coef);
}
__device__ __forceinline__ double edge_coef(int32_t deg, double alpha) { return deg == 0 ? 0.0 : alpha / (double)deg; }
// the same weight from the row's coefficient (coef = alpha / deg exactly as above; 0: dangling)
__device__ __forceinline__ int64_t edge_weight_c(int64_t rj, double coef) {
  return coef == 0.0 ? 0 : (int64_t)((double)rj * coef);
}


constexpr int64_t kMaxSeedN = (int64_t)1 << 23;  // N x 2^40 (the largest q) fits the int64 seed total
// a seed's anomaly above the floor in 2^-32 units, clamped at 256 units (q <= 2^40: every product
// and sum of the explanation pass and the int64 seed total of N <= 2^23 pods stay exact; a NaN is 0)
__device__ __forceinline__ int64_t quantise(float s, float floor_) {
  const double v = (double)s - (double)floor_;
  return v > 0.0 ? (int64_t)(fmin(v, 256.0) * 4294967296.0) : 0;
}

// r0 = floor(2^60/N), w0, seeds; dangling mass and seed total into the send slots
__global__ __launch_bounds__(TPB) void ppr_init(const float* __restrict__ seed, float seed_floor,
                                                const int32_t* __restrict__ outdeg, int64_t n, int64_t N,
                                                double alpha, int64_t* __restrict__ q, int64_t* __restrict__ r,
                                                int64_t* __restrict__ send, int64_t n_max, double* __restrict__ coef) {
  __shared__ int64_t red[TPB / 64];
  const int64_t r0 = (int64_t)(krca::kFix / (double)N);
#ifdef KRCA_GRAPH_DEBUG
  if (blockIdx.x == 0 && threadIdx.x == 0)
    printf("KGD init seed=%p q=%p r=%p send=%p coef=%p n=%ld N=%ld alpha=%.4f floor=%.4f\n", (const void*)seed, (void*)q,
           (void*)r, (void*)send, (void*)coef, (long)n, (long)N, alpha, seed_floor);
#endif
  int64_t dang = 0, qs = 0;
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    const int32_t deg = outdeg[i];
    const int64_t qi = quantise(seed[i], seed_floor);
    q[i] = qi;
    qs += qi;
    r[i] = r0;
    coef[2 * i] = edge_coef(deg, alpha);
    coef[2 * i + 1] = (double)qi;
    reinterpret_cast<uint32_t*>(send)[i] = wenc(edge_weight(r0, deg, alpha));
    if (deg == 0) dang += r0;
  }
  dang = block_sum_i64(dang, red);
  qs = block_sum_i64(qs, red);
  if (threadIdx.x == 0) {
    add_slot(send + wslots(n_max) + NSPREAD, dang);
    add_slot(send + wslots(n_max) + 2 * NSPREAD, qs);
  }
}

// warm start (streaming re-ranking): keep r from the previous solve, new seeds, w and dangling
// mass from the kept r (networkx's nstart, taken as the fixed-point vector itself)
__global__ __launch_bounds__(TPB) void ppr_init_warm(const float* __restrict__ seed, float seed_floor,
                                                     const int32_t* __restrict__ outdeg, int64_t n, double alpha,
                                                     int64_t* __restrict__ q, const int64_t* __restrict__ r,
                                                     int64_t* __restrict__ send, int64_t n_max, double* __restrict__ coef) {
  __shared__ int64_t red[TPB / 64];
  int64_t dang = 0, qs = 0;
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    const int32_t deg = outdeg[i];
    const int64_t qi = quantise(seed[i], seed_floor);
    q[i] = qi;
    qs += qi;
    const int64_t ri = r[i];
    coef[2 * i] = edge_coef(deg, alpha);
    coef[2 * i + 1] = (double)qi;
    reinterpret_cast<uint32_t*>(send)[i] = wenc(edge_weight(ri, deg, alpha));
    if (deg == 0) dang += ri;
  }
  dang = block_sum_i64(dang, red);
  qs = block_sum_i64(qs, red);
  if (threadIdx.x == 0) {
    add_slot(send + wslots(n_max) + NSPREAD, dang);
    add_slot(send + wslots(n_max) + 2 * NSPREAD, qs);
  }
}

struct StepScalars {
  double tele, tq, alpha;  // tq = tele / q_total: t_i = q_i * tq (no per-row division)
  int64_t qt, tu;          // tu: the uniform share when every seed is at the floor
};

// Single device (G = 1): the iteration's reduction runs in the step kernel's last workgroup
// instead of a ppr_reduce launch (the exchange is a buffer swap, so nothing happens between them).
struct Fuse {
  int on;
  double err_limit;
  int64_t* w_next;  // the buffer the step gathered from = the next step's write target (slots zeroed)
};

// Folded iteration (krca_ppr_shard_step_folded): step `it` (1-based) does the reduction of step
// it - 1 itself -- every workgroup sums the G ranks' slot set (it - 1) % NSET of w_all (integers:
// every workgroup gets the same totals) and decides convergence / the teleport scale locally --
// writes its own partial sums into set it % NSET of send, and workgroup 0 zeroes set (it + 1) % NSET
// of the next step's write target.  No ppr_reduce launch between steps: one kernel and one
// exchange per iteration.
struct Fold {
  int on, it, G;
  double err_limit;
  int64_t* next;  // the next step's write target (G = 1: the buffer gathered from; G > 1: send)
};

// the reduction of ppr_reduce over ONE slice (G = 1), by a whole workgroup: residual / dangling
// sums of `slice` (atomically updated by this step's workgroups), convergence, next teleport scale,
// the next write target's slots zeroed; called by the step's last workgroup only
__device__ void reduce_single(const int64_t* slice_slots, int64_t* next_slots, double alpha, double err_limit,
                              Ctl* ctl, int64_t* red) {
  const int tid = threadIdx.x;
  int64_t e = 0, d = 0;
  if (tid < NSPREAD) {
    e = __hip_atomic_load(slice_slots + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    d = __hip_atomic_load(slice_slots + NSPREAD + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const int64_t err = block_sum_i64(e, red);
  const int64_t dang = block_sum_i64(d, red);
  if (tid < SET_WORDS) next_slots[tid] = 0;
  if (tid != 0) return;
  ctl->done = 0;
  if (ctl->converged) return;
  ctl->iter += 1;
  if (err_limit > 0.0 && (double)err < err_limit) {
    ctl->converged = ctl->iter;
    return;
  }
  ctl->tele = (1.0 - alpha) * krca::kFix + alpha * (double)dang;
}

// The reduction of folded step it - 1, done at the start of step it (krca_ppr_shard_step_folded):
// every wave sums the G x NSPREAD slots of set (it - 1) % NSET of each quantity on its own (a
// butterfly leaves the total in every lane: integers, so all waves and all workgroups get the same
// totals, with no LDS and no barrier -- three block sums cost 8 barriers, ~2 us per step at C4) and
// decides convergence / the teleport scale locally.  The `lead` workgroup also zeroes set
// (it + 1) % NSET of the next write target and records the decision in ctl.  Returns true when
// step it - 1 converged (the caller does nothing more).  ppr_fold_only runs just this for a rank
// that owns no plan entries, so every rank's ctl advances identically.
__device__ __forceinline__ bool fold_reduce(const Fold& fo, const int64_t* wall, int64_t n_max, double alpha, Ctl* ctl,
                                            bool lead, StepScalars& k) {
  const int tid = threadIdx.x;
  const int ps = (fo.it - 1) % NSET, zs = (fo.it + 1) % NSET;
  int64_t pe = 0, pd = 0, pq = 0;
  for (int i = tid & 63; i < fo.G * NSPREAD; i += 64) {
    const int64_t* sl = wall + (int64_t)(i / NSPREAD) * slice_words(n_max) + wslots(n_max) + ps * SET_WORDS + (i % NSPREAD);
    pe += sl[0];
    pd += sl[NSPREAD];
    pq += sl[2 * NSPREAD];
  }
  for (int off = 32; off > 0; off >>= 1) {
    pe += (int64_t)__shfl_xor((long long)pe, off, 64);
    pd += (int64_t)__shfl_xor((long long)pd, off, 64);
    pq += (int64_t)__shfl_xor((long long)pq, off, 64);
  }
  const bool stop = fo.it > 1 && fo.err_limit > 0.0 && (double)pe < fo.err_limit;  // step it-1 converged
  k.tele = (1.0 - alpha) * krca::kFix + alpha * (double)pd;
  k.qt = fo.it == 1 ? pq : ctl->q_total;  // written by step 1's lead workgroup (an earlier kernel)
  if (lead) {
    for (int i = tid; i < SET_WORDS; i += blockDim.x) fo.next[wslots(n_max) + zs * SET_WORDS + i] = 0;
    if (tid == 0) {
      if (fo.it == 1) ctl->q_total = pq;
      ctl->iter = fo.it - 1;
      if (stop) ctl->converged = fo.it - 1;
      else ctl->tele = k.tele;
    }
  }
  return stop;
}

// a folded step of a rank that owns no plan entries (no rows): the reduction only, one workgroup
__global__ __launch_bounds__(64) void ppr_fold_only(int64_t n_max, double alpha, Ctl* ctl, Fold fo,
                                                    const int64_t* __restrict__ w_all) {
  if (ctl->converged) return;
  StepScalars k;
  (void)fold_reduce(fo, w_all, n_max, alpha, ctl, true, k);
}

// r_i <- pulled mass + teleport share; next w_i; residual and dangling contributions
// (q_i, r_i, deg_i were loaded by the caller together with the row's edges).  flags: PPR_RESIDUAL
// = the L1 stop rule needs |r_new - r_old| (ro was loaded), PPR_WRITE_R = store r_new (every
// iteration under a tolerance; only the last one of a fixed-iteration solve).
template <int FLAGS>
__device__ __forceinline__ void update_row(int64_t i, int64_t pulled, double qd, int64_t ro, double coef,
                                           const StepScalars& k, int64_t* __restrict__ r,
                                           int64_t* __restrict__ send, int64_t& err, int64_t& dang) {
  const int64_t t = k.qt > 0 ? (int64_t)(qd * k.tq) : k.tu;  // qd = (double)q_i
  const int64_t rn = pulled + t;
  if (FLAGS & PPR_WRITE_R) r[i] = rn;
  if (FLAGS & PPR_RESIDUAL) err += rn > ro ? rn - ro : ro - rn;
  if (coef == 0.0) dang += rn;
  reinterpret_cast<uint32_t*>(send)[i] = wenc(edge_weight_c(rn, coef));
}

// One plan entry, loaded in two parts so that a prefetched value is never copied or computed on
// before it is used (that would make the compiler wait for it and, the vector memory counter
// being in order, for every load issued before it):
//   Head  the plan entry (wave-uniform, scalar loads) and the lane's columns to gather; loaded two
//         entries ahead of the one being summed;
//   Rows  what the sum and the update need; loaded one entry ahead, beside that entry's gathers.
// Plan entry {rb | nu << 32, code, e0, e1}: code > 0: short rows [rb, code) with edges [e0, e1);
// code <= 0: chunk -code of long row rb.  nu == 0 (direct block): pk[e0, e1) are the edges'
// remapped columns, gathered one per edge.  nu > 0 (dictionary block, krca_ppr_pack): pk[e0, e0+nu)
// are the block's DISTINCT columns (ascending, so neighbouring lanes gather neighbouring words) and
// from pk[e0 + pad(nu)] on, two uint16 per word, each edge's slot in that list.  Lane tid gathers
// slots / edges tid + j*TPB (coalesced) and sums the contiguous edges [8 tid, 8 tid + 8).
struct Meta {
  int32_t rb, code, nu;
  int64_t e0, e1;
};
struct Head {
  Meta m;
  uint32_t c[SEG];  // remapped columns (uint32 units of the exchange layout)
};
struct Rows {
  int64_t my_r;
  double my_coef, my_qd;  // alpha / outdeg and (double)q_i (coef_of)
  uint32_t li;  // krca_ppr_pack lane word: (sum slot of the row holding edge 8t) << 8 | head bits
  uint32_t rs;  // the sum slot of the lane's row (ROW_BUDGET: a row without edges)
  uint4 ix;     // dictionary blocks: the slots of edges 8t .. 8t+7 (uint16 pairs)
};

__device__ __forceinline__ int64_t dict_words(int64_t e0, int32_t nu) {  // pk offset of the slot words
  return ((e0 + nu + 3) & ~int64_t(3)) - e0;
}

// a bounds-checked buffer over [p, p + bytes): loads past the end return 0, so the lanes past a
// block's count need no clamped index (each clamp was a compare + select or min per load); the
// byte offsets tid * size are loop-invariant registers and the per-slot strides are immediates
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_over(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ int64_t buf_i64(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  const u32x2 v = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, (int)off, 0, 0));
  return (int64_t)(((uint64_t)v.y << 32) | v.x);
}

template <bool NT>
__device__ __forceinline__ void load_head(const int64_t* __restrict__ plan, int64_t b, const int32_t* __restrict__ pk,
                                          Head& H) {
  const int64_t* pe = plan + 4 * b;
  const int64_t h = pe[0];
  H.m.rb = (int32_t)(h & 0xFFFFFFFF);
  H.m.nu = (int32_t)(h >> 32);
  H.m.code = (int32_t)pe[1];
  H.m.e0 = pe[2];
  H.m.e1 = pe[3];
  const uint32_t tid = threadIdx.x;
  // every lane loads (a predicated default value would have to wait for whatever load last wrote
  // that register): slots past the block's count read 0 from the bounds-checked buffer, i.e.
  // column 0, a valid gather whose value no sum reads (dictionary slots >= nu and edges >= ne are
  // never summed; long-row chunks mask their sum)
  const uint32_t lim = (uint32_t)(H.m.nu > 0 ? (int64_t)H.m.nu : H.m.e1 - H.m.e0);
  const __amdgpu_buffer_rsrc_t rs = buf_over(pk + H.m.e0, 4 * lim);
  // the slot stride goes into the VGPR offset, never the SGPR one: the raw-buffer range check
  // covers VGPR + immediate offset only, so an SGPR stride would let a lane below `lim` read past
  // the block (and, for the last entry, past pk) instead of getting 0
#pragma unroll
  for (int j = 0; j < SEG; ++j) H.c[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(4 * (tid + j * TPB)), 0, 0);
}

template <int FLAGS>
__device__ __forceinline__ void load_rows(const Meta& m, int64_t b, const uint16_t* __restrict__ lane_info,
                                          const int32_t* __restrict__ pk,
                                          const double* __restrict__ coef, const int64_t* __restrict__ q,
                                          const int64_t* __restrict__ r, Rows& R) {
  const uint32_t tid = threadIdx.x;
  const uint32_t nrows = (uint32_t)(m.code > 0 ? m.code - m.rb : 1);
  constexpr bool NT = (FLAGS & PPR_NT) != 0;
  // the lane's row (lanes past the block's rows read 0 and update nothing)
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  R.my_r = (FLAGS & PPR_RESIDUAL) ? buf_i64(buf_over(r + m.rb, 8 * nrows), 8 * tid) : 0;
  const u32x4 cq = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(buf_over(coef + 2 * m.rb, 16 * nrows),
                                                                                    (int)(16 * tid), 0, 0));
  R.my_coef = __builtin_bit_cast(double, ((uint64_t)cq.y << 32) | cq.x);
  R.my_qd = __builtin_bit_cast(double, ((uint64_t)cq.w << 32) | cq.z);
  const uint16_t* lb = lane_info + b * 2 * TPB;  // zero / empty for long-row chunks
  R.li = ld_stream<NT>(lb + tid);
  R.rs = ld_stream<NT>(lb + TPB + tid);
  // the lane's 16 bytes of edge slots (used by dictionary blocks only; lanes past the edges read 0)
  const int64_t wb = m.nu > 0 ? m.e0 + dict_words(m.e0, m.nu) : (m.e0 & ~int64_t(3));
  const uint32_t nlane = (uint32_t)((m.e1 - m.e0 + SEG - 1) / SEG);
  const u32x4 ix = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(buf_over(pk + wb, 16 * nlane),
                                                                                    (int)(16 * tid), 0, 0));
  R.ix = make_uint4(ix.x, ix.y, ix.z, ix.w);
}

// every lane gathers all SEG columns (past the block's count load_head read column 0: a valid
// address whose value no sum reads), so the 8 loads issue back to back with no select
__device__ __forceinline__ void gather(const Head& H, const uint32_t* __restrict__ w, uint32_t (&v)[SEG]) {
#pragma unroll
  for (int j = 0; j < SEG; ++j)  // 32-bit byte offsets (krca_ppr_pack keeps remapped columns < 2^30)
    v[j] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(w) + (H.c[j] << 2));
}

// Persistent, software-pipelined step.  Workgroup g takes plan entries g, g + G, g + 2G, ...;
// while it sums entry i, the w gathers and row loads of entry i+1 and the plan / column loads of
// entry i+2 are in flight, so neither the gather latency nor the dependent plan -> column latency
// is paid per entry.  The loop is unrolled x2 over ping-pong Head / Rows slots (no copies of
// in-flight loads).  A short block in three barrier-separated phases:
//  stage   the gathered values (or distinct-column values) go to LDS;
//  sum     lane t sums its 8 contiguous edges [8t, 8t+8) as row segments: the host-built lane word
//          (krca_ppr_pack, 2 bytes) gives the sum slot of the row holding edge 8t and the edges that
//          start a row; the block's non-empty rows have consecutive slots, so each segment ends in
//          one no-return LDS atomic into the current slot and moves to the next; the 8 values are
//          independent LDS reads: no dependent LDS chain and no row offsets (round 1 searched the
//          row offsets and walked the row ends, ~25 dependent LDS round trips per lane; round 3
//          first staged each row's index at its first edge and loaded two row offsets per row,
//          then carried one row byte per edge: 8 bytes per lane);
//  update  lane r updates row r (teleport, residual, next w).
#ifdef PPR_TIMING
__device__ unsigned long long g_ppr_timing[4096 * 5];  // per workgroup: stage, sum, update, long, blocks
#endif
#ifndef PPR_WAVES
#define PPR_WAVES 5  // 96 VGPRs, 5 workgroups per CU: 38.1 -> 34.9 us per step at C4 (4: 104 VGPRs; 6 spills)
#endif

template <int FLAGS>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(PPR_WAVES, 8))) void ppr_step(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ pk, const int64_t* __restrict__ plan,
    const uint16_t* __restrict__ lane_info, int64_t nblk, const uint32_t* __restrict__ w,
    const int32_t* __restrict__ outdeg, const int64_t* __restrict__ q, int64_t n, int64_t N, double alpha,
    int64_t* __restrict__ r, int64_t* __restrict__ send, int64_t n_max, Ctl* ctl, Fuse fz, Fold fo, int xcd) {
  __shared__ __attribute__((aligned(16))) uint32_t vals[EDGE_BUDGET];  // staged codes: edge (direct) or slot (dictionary) i
  __shared__ unsigned long long rowsum[ROW_BUDGET + 1];  // + the zero slot of rows without edges
  __shared__ int64_t red[TPB / 64];
  // entries of this workgroup: b, b + stride, ... below lim.  xcd (the host sets it when the grid is
  // a multiple of 8 and nblk >= grid): workgroups g, g + 8, ... (one XCD, for speed only) share one
  // contiguous eighth of the plan, so the callers an XCD's L2 holds are those of neighbouring rows
#ifdef KRCA_GRAPH_DEBUG  // tools/graph_replay_probe.py (make gdbg): the kernel arguments and ctl header as seen
  if (blockIdx.x == 0 && threadIdx.x == 0)
    printf("KGD step fold=%d it=%d G=%d next=%p ctl=%p r=%p send=%p w=%p q=%p plan=%p n=%ld nblk=%ld alpha=%.4f"
           " | ctl iter=%d conv=%d qt=%ld tele=%.9e\n", fo.on, fo.it, fo.G, (void*)fo.next, (void*)ctl, (void*)r,
           (void*)send, (const void*)w, (const void*)q, (const void*)plan, (long)n, (long)nblk, alpha, ctl->iter,
           ctl->converged, (long)ctl->q_total, ctl->tele);
#endif
  int64_t b = blockIdx.x, lim = nblk, stride = gridDim.x;
  if (xcd) {
    const int64_t x = blockIdx.x & 7;
    stride = gridDim.x >> 3;
    b = x * nblk / 8 + (blockIdx.x >> 3);
    lim = (x + 1) * nblk / 8;
  }
  if (b >= lim) return;
  const int32_t conv = ctl->converged;
  if (conv) return;  // converged (tol > 0): no writes (uniform)
  const int tid = threadIdx.x;
  if (tid == 0) rowsum[ROW_BUDGET] = 0ull;  // never added to (the entries' barriers order it)
  Head H0, H1;
  Rows R0, R1;
  load_head<(FLAGS & PPR_NT) != 0>(plan, b, pk, H0);
  uint32_t v[SEG];  // codes: decoded where summed (a prefetched register is never computed on early)
  gather(H0, w, v);
  const double* coef = coef_of(ctl, n);
  load_rows<FLAGS>(H0.m, b, lane_info, pk, coef, q, r, R0);
  Meta cur = H0.m;
  int64_t b1 = b + stride;
  // prefetches past the workgroup's last entry load the grid's last entry again (clamped, results
  // unused): every path issues the same loads, so the compiler's vector-memory waits stay counted
  // (vmcnt(N)) instead of vmcnt(0) at the join of an `if (b1 < nblk)`, which made the sum phase
  // wait for the NEXT entry's gathers and rows and undid the software pipeline
  load_head<(FLAGS & PPR_NT) != 0>(plan, b1 < lim ? b1 : lim - 1, pk, H1);
  // the teleport scale of this step (after the first entry's loads are issued: a folded step's
  // reduction of the previous one overlaps them)
  StepScalars k;
  int64_t* my_slots = send + wslots(n_max);  // this step's partial-sum slots
  if (fo.on) {  // block-uniform
    if (fold_reduce(fo, reinterpret_cast<const int64_t*>(w), n_max, alpha, ctl, blockIdx.x == 0, k))
      return;  // step it - 1 converged: uniform, every workgroup decided the same
    my_slots += (fo.it % NSET) * SET_WORDS;
  } else {
    k.tele = ctl->tele;
    k.qt = ctl->q_total;
  }
  k.tq = k.tele / (double)k.qt;
  k.tu = (int64_t)((1.0 / (double)N) * k.tele);
  k.alpha = alpha;
  if (blockIdx.x == 0 && tid == 0) ctl->tele_used = k.tele;  // this step updates the rows with k.tele
  int64_t err = 0, dang = 0;
#ifdef PPR_TIMING
  uint64_t tacc[5] = {0, 0, 0, 0, 0};
  uint64_t tp = clock64();
#define PPR_T(i) do { const uint64_t tn = clock64(); tacc[i] += tn - tp; tp = tn; } while (0)
#else
#define PPR_T(i) do {} while (0)
#endif
  // one entry: stage `cur` (its values gathered last round, rows in rc), gather entry b1 (head hn)
  // and load its rows into rn, load the head of entry b2 into hl; sum and update `cur`.
  // False when `cur` was the workgroup's last entry.
  auto entry = [&](Head& hn, Head& hl, const Rows& rc, Rows& rn) -> bool {
    const bool shortb = cur.code > 0;
    const int ne = (int)(cur.e1 - cur.e0);
    const bool dict = cur.nu > 0;
    int64_t sacc_long = 0;
    if (shortb) {
      // every lane stores all SEG values (EDGE_BUDGET slots; the gathers past the block's staged
      // count returned 0 and the sum reads only slots / edges of the block): no divergent store
      // per value (each cost an exec-mask save / branch / restore: ~32 scalar + vector
      // instructions per entry)
#pragma unroll
      for (int j = 0; j < SEG; ++j) vals[tid + j * TPB] = v[j];
      rowsum[tid] = 0ull;
    } else {  // a chunk of a long row: its edges [0, ne) (the gathers past them read column 0)
#pragma unroll
      for (int j = 0; j < SEG; ++j) sacc_long += tid + j * TPB < ne ? wdec(v[j]) : 0;
    }
    // v is free: gathers and rows of the next entry, head of the one after
    const int64_t b2 = b1 + stride;
    const Meta next = hn.m;
    gather(hn, w, v);
    load_rows<FLAGS>(next, b1 < lim ? b1 : lim - 1, lane_info, pk, coef, q, r, rn);
    load_head<(FLAGS & PPR_NT) != 0>(plan, b2 < lim ? b2 : lim - 1, pk, hl);
    if (shortb) {
      const int nrows = cur.code - cur.rb;
      __syncthreads();
      PPR_T(0);
      const int a = tid * SEG;
      if (a < ne) {
        const uint32_t M = rc.li & 0xFFu;  // bits of the lane's edges that start a row
        // the 8 LDS reads are unconditional (a slot past the block's edges reads a value the
        // sum drops), so they issue back to back: a read under a per-edge branch was a branch
        // with its own lgkmcnt(0) wait, 8 dependent LDS round trips.  Direct blocks read the
        // lane's 8 staged edges as two 16-byte reads; dictionary blocks read one slot each (the
        // branch is block-uniform: no per-value select between the two addressings)
        uint32_t c[SEG];
        if (dict) {
          const uint4 sx = rc.ix;  // this lane's own slots (prefetched with the rows)
#pragma unroll
          for (int kk = 0; kk < SEG; ++kk) {
            const uint32_t wd = kk < 2 ? sx.x : kk < 4 ? sx.y : kk < 6 ? sx.z : sx.w;
            c[kk] = vals[(wd >> (16 * (kk & 1))) & (EDGE_BUDGET - 1)];
          }
        } else {
          const uint4 lo = *reinterpret_cast<const uint4*>(vals + a), hi = *reinterpret_cast<const uint4*>(vals + a + 4);
          c[0] = lo.x; c[1] = lo.y; c[2] = lo.z; c[3] = lo.w;
          c[4] = hi.x; c[5] = hi.y; c[6] = hi.z; c[7] = hi.w;
        }
        int64_t sacc = wdec(c[0]);
        // byte offset of the current row's sum slot; each head: the next slot
        uint32_t row8 = (rc.li >> 8) * (uint32_t)sizeof(unsigned long long);
        char* const rsb = reinterpret_cast<char*>(rowsum);
        auto flush = [&]() {
          atomicAdd(reinterpret_cast<unsigned long long*>(rsb + row8), (unsigned long long)sacc);  // no return: no wait
          sacc = 0;
          row8 += (uint32_t)sizeof(unsigned long long);
        };
        if (a + SEG <= ne) {  // every edge of the lane is the block's (all lanes but one per block)
#pragma unroll
          for (int kk = 1; kk < SEG; ++kk) {
            if ((M >> kk) & 1u) flush();  // edge a + kk starts the next row's segment
            sacc += wdec(c[kk]);
          }
        } else {
#pragma unroll
          for (int kk = 1; kk < SEG; ++kk) {
            if ((M >> kk) & 1u) flush();
            sacc += a + kk < ne ? wdec(c[kk]) : 0;
          }
        }
        atomicAdd(reinterpret_cast<unsigned long long*>(rsb + row8), (unsigned long long)sacc);
      }
      __syncthreads();
      PPR_T(1);
      if (tid < nrows)
        update_row<FLAGS>(cur.rb + tid, (int64_t)rowsum[rc.rs], rc.my_qd, rc.my_r, rc.my_coef, k, r, send, err, dang);
      __syncthreads();  // rowsum / vals are rewritten by the next entry
      PPR_T(2);
    } else {  // chunk of long row rb: block sum -> row accumulator; the last chunk updates the row
      const int64_t tot = block_sum_i64(sacc_long, red);
      if (tid == 0) {
        const int32_t rb = cur.rb;
        const int64_t deg_in = row_ptr[rb + 1] - row_ptr[rb];
        const uint32_t nch = (uint32_t)((deg_in + EDGE_BUDGET - 1) / EDGE_BUDGET);
        int64_t* acc = acc_long_of(ctl) + rb;
        uint32_t* tk = ticket_of(ctl, n) + rb;
        __hip_atomic_fetch_add(acc, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the add is performed before the ticket
        const uint32_t t = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == nch - 1) {
          const int64_t pulled = __hip_atomic_load(acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(acc, (int64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          update_row<FLAGS>(rb, pulled, rc.my_qd, rc.my_r, rc.my_coef, k, r, send, err, dang);
        }
      }
      PPR_T(3);
    }
#ifdef PPR_TIMING
    tacc[4] += 1;
#endif
    if (b1 >= lim) return false;
    cur = next;
    b = b1;
    b1 = b2;
    return true;
  };
  while (entry(H1, H0, R0, R1) && entry(H0, H1, R1, R0)) {
  }
#ifdef PPR_TIMING
  if (tid == 0 && blockIdx.x < 4096)
    for (int i = 0; i < 5; ++i) g_ppr_timing[blockIdx.x * 5 + i] += tacc[i];
#endif
  err = block_sum_i64(err, red);
  dang = block_sum_i64(dang, red);
  if (tid == 0) {
    add_slot(my_slots, err);
    add_slot(my_slots + NSPREAD, dang);
  }
  if (fz.on) {  // block-uniform
    __shared__ int last;
    if (tid == 0) {
      // this workgroup's slot adds are performed (at the memory side, device-scope atomics) before
      // its ticket; the last workgroup reads the slots with agent-scope atomic loads.  (A
      // __threadfence() here -- a release fence per workgroup -- doubled the step: 39 -> 77 us.)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      last = __hip_atomic_fetch_add(&ctl->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    }
    __syncthreads();
    if (last) reduce_single(send + wslots(n_max), fz.w_next + wslots(n_max), alpha, fz.err_limit, ctl, red);
  }
}

// one block: sum the G*NSPREAD gathered slots of each quantity (integer -> order-free), decide
// convergence, set the teleport scale of the next step, zero the next write target's slots
__global__ __launch_bounds__(TPB) void ppr_reduce(const int64_t* __restrict__ w_all, int32_t G, int64_t n_max,
                                                  double alpha, double err_limit, int first, Ctl* ctl,
                                                  int64_t* __restrict__ send_next) {
  __shared__ int64_t red[TPB / 64];
  int64_t part[3] = {0, 0, 0};
  for (int i = threadIdx.x; i < G * NSPREAD; i += TPB) {
    const int64_t* s = w_all + (int64_t)(i / NSPREAD) * slice_words(n_max) + wslots(n_max) + (i % NSPREAD);
    part[0] += s[0];
    part[1] += s[NSPREAD];
    part[2] += s[2 * NSPREAD];
  }
  const int64_t err = block_sum_i64(part[0], red);
  const int64_t dang = block_sum_i64(part[1], red);
  const int64_t qs = block_sum_i64(part[2], red);
  __syncthreads();
  if (threadIdx.x < SET_WORDS) send_next[wslots(n_max) + threadIdx.x] = 0;
  if (threadIdx.x != 0 || ctl->converged) return;
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

// the reduction of the last folded step (it): sums set it % NSET of the G slices, counts the
// iteration and decides convergence -- what ppr_reduce does after every unfolded step
__global__ __launch_bounds__(TPB) void ppr_finish(const int64_t* __restrict__ w_all, int32_t G, int64_t n_max,
                                                  double alpha, double err_limit, int it, Ctl* ctl) {
  __shared__ int64_t red[TPB / 64];
  int64_t pe = 0, pd = 0;
  for (int i = threadIdx.x; i < G * NSPREAD; i += TPB) {
    const int64_t* sl = w_all + (int64_t)(i / NSPREAD) * slice_words(n_max) + wslots(n_max) + (it % NSET) * SET_WORDS +
                        (i % NSPREAD);
    pe += sl[0];
    pd += sl[NSPREAD];
  }
  const int64_t err = block_sum_i64(pe, red);
  const int64_t dang = block_sum_i64(pd, red);
#ifdef KRCA_GRAPH_DEBUG
  if (threadIdx.x == 0)
    printf("KGD finish it=%d G=%d w_all=%p ctl=%p err=%ld dang=%ld | ctl iter=%d conv=%d qt=%ld tele=%.9e\n", it, G,
           (const void*)w_all, (void*)ctl, (long)err, (long)dang, ctl->iter, ctl->converged, (long)ctl->q_total,
           ctl->tele);
#endif
  if (threadIdx.x != 0 || ctl->converged) return;
  ctl->iter = it;
  if (err_limit > 0.0 && (double)err < err_limit) {
    ctl->converged = it;
    return;
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

// the default root-cause key (krca_rca_key_explained): u_i = q_i - d_i (the anomaly that no
// explaining dependency accounts for, d from krca_rca_explain), recv_i = r_i - t_i (the mass the row
// received from its callers in the last step: t_i is that step's teleport share, update_row's
// expression with the recorded scale), key = bits(((double)recv_i + (double)t_i / 32) * (double)u_i),
// 0 when u_i <= 0 (the own share at 1/32: a fault whose callers carry no anomaly still ranks by it)
__global__ __launch_bounds__(TPB) void rca_key_explained(const int64_t* __restrict__ r, const int64_t* __restrict__ q,
                                                         const int64_t* __restrict__ d, int64_t n, int64_t N,
                                                         const Ctl* __restrict__ ctl, int64_t* __restrict__ key) {
  const double tele = ctl->tele_used;
  const int64_t qt = ctl->q_total;
  const double tq = tele / (double)qt;
  const int64_t tu = (int64_t)((1.0 / (double)N) * tele);
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    const int64_t qi = q[i], u = qi - d[i];
    double v = 0.0;
    if (u > 0) {
      const int64_t t = qt > 0 ? (int64_t)((double)qi * tq) : tu;
      v = ((double)(r[i] - t) + (double)t * 0.03125) * (double)u;
    }
    key[i] = __double_as_longlong(v);
  }
}

__global__ __launch_bounds__(TPB) void remap_cols(const int32_t* __restrict__ col, int64_t E, int64_t n_max,
                                                  int32_t* __restrict__ out) {
  for (int64_t e = (int64_t)blockIdx.x * TPB + threadIdx.x; e < E; e += (int64_t)gridDim.x * TPB) {
    const int64_t j = col[e];
    out[e] = (int32_t)remap_col(j, n_max);
  }
}

double* host_coef(void* ctl, int64_t n) {  // coef_of on the host side of the ctl layout
  return reinterpret_cast<double*>(reinterpret_cast<char*>(ctl) + CTL_BYTES + 16 * n);
}

unsigned grid_for(int64_t n, int64_t cap = 2048) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(krca::ceil_div(n, TPB), cap));
}

}  // namespace

namespace {
// Zeroing on the solve path is done by kernels, never by hipMemsetAsync: a solve captured into a
// HIP graph with the runtime's graph packet capture on replayed its memset nodes with stale bytes
// once ~300 later eager launches had reused the runtime's staging memory (R6a,
// tools/graph_replay_probe.py: every captured kernel's arguments were intact at the bad replay, but
// the ctl header read back torch kernels' argument words), while kernel nodes replay exactly.
__global__ __launch_bounds__(TPB) void zero_words2(int64_t* __restrict__ a, int64_t na, int64_t* __restrict__ b,
                                                   int64_t nb) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < na + nb; i += (int64_t)gridDim.x * TPB) {
    if (i < na) a[i] = 0;
    else b[i - na] = 0;
  }
}
__global__ __launch_bounds__(TPB) void fill_words(int64_t* __restrict__ a, int64_t n, int64_t v) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) a[i] = v;
}
static_assert(sizeof(Ctl) % 8 == 0, "the ctl header is zeroed in int64 words");
// the ctl header and the send buffer's partial-sum slots, zeroed before an init adds into them
int zero_ctl_and_slots(void* ctl, int64_t* send_slots, hipStream_t st) {
  hipLaunchKernelGGL(zero_words2, dim3(1), dim3(TPB), 0, st, reinterpret_cast<int64_t*>(ctl), (int64_t)(sizeof(Ctl) / 8),
                     send_slots, (int64_t)NSLOT);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}
}  // namespace

extern "C" {


int64_t krca_ppr_ctl_size(int64_t n_local) { return CTL_BYTES + 32 * std::max<int64_t>(n_local, 1); }

int krca_ppr_remap_cols(const int32_t* col, int64_t E, int64_t n_max, int32_t* out, void* stream) {
  KRCA_CHECK_ARG(E >= 0 && n_max > 0, "krca_ppr_remap_cols: bad sizes");
  if (E == 0) return KRCA_OK;
  KRCA_CHECK_ARG(col && out, "krca_ppr_remap_cols: null pointer");
  hipLaunchKernelGGL(remap_cols, dim3(grid_for(E, 8192)), dim3(TPB), 0, krca::as_stream(stream), col, E, n_max, out);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_fill_i64(int64_t* p, int64_t n, int64_t value, void* stream) {
  KRCA_CHECK_ARG(n >= 0, "krca_fill_i64: bad size");
  if (n == 0) return KRCA_OK;
  KRCA_CHECK_ARG(p, "krca_fill_i64: null pointer");
  hipLaunchKernelGGL(fill_words, dim3((unsigned)std::min<int64_t>(krca::ceil_div(n, TPB), 1024)), dim3(TPB), 0,
                     krca::as_stream(stream), p, n, value);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_ppr_shard_init(const float* seed, float seed_floor, const int32_t* outdeg, int64_t n_local, int64_t n_max,
                        int64_t N, double alpha, void* ctl, int64_t* q_local, int64_t* r_local, int64_t* send,
                        void* stream) {
  KRCA_CHECK_ARG(N > 0 && N <= kMaxSeedN && n_local >= 0 && n_local <= n_max, "krca_ppr_shard_init: bad sizes");
  KRCA_CHECK_ARG(alpha > 0.0 && alpha < 1.0, "krca_ppr_shard_init: alpha must be in (0, 1)");
  KRCA_CHECK_ARG(ctl && send && (n_local == 0 || (seed && outdeg && q_local && r_local)), "krca_ppr_shard_init: null pointer");
  hipStream_t st = krca::as_stream(stream);
  if (int rc = zero_ctl_and_slots(ctl, send + wslots(n_max), st)) return rc;
  if (n_local > 0)
    hipLaunchKernelGGL(ppr_init, dim3(grid_for(n_local)), dim3(TPB), 0, st, seed, seed_floor, outdeg, n_local, N,
                       alpha, q_local, r_local, send, n_max, host_coef(ctl, n_local));
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_ppr_shard_init_warm(const float* seed, float seed_floor, const int32_t* outdeg, int64_t n_local,
                             int64_t n_max, int64_t N, double alpha, void* ctl, int64_t* q_local,
                             const int64_t* r_local, int64_t* send, void* stream) {
  KRCA_CHECK_ARG(N > 0 && N <= kMaxSeedN && n_local >= 0 && n_local <= n_max, "krca_ppr_shard_init_warm: bad sizes");
  KRCA_CHECK_ARG(alpha > 0.0 && alpha < 1.0, "krca_ppr_shard_init_warm: alpha must be in (0, 1)");
  KRCA_CHECK_ARG(ctl && send && (n_local == 0 || (seed && outdeg && q_local && r_local)),
                 "krca_ppr_shard_init_warm: null pointer");
  hipStream_t st = krca::as_stream(stream);
  if (int rc = zero_ctl_and_slots(ctl, send + wslots(n_max), st)) return rc;
  if (n_local > 0)
    hipLaunchKernelGGL(ppr_init_warm, dim3(grid_for(n_local)), dim3(TPB), 0, st, seed, seed_floor, outdeg, n_local,
                       alpha, q_local, r_local, send, n_max, host_coef(ctl, n_local));
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

namespace {
int launch_step(const int64_t* row_ptr, const int32_t* col, const int64_t* plan, int64_t plan_len, const uint16_t* lane,
                const int64_t* w_all, const int32_t* outdeg, const int64_t* q_local, int64_t n_local, int64_t n_max,
                int64_t N, double alpha, int32_t flags, int64_t* r_local, int64_t* send, void* ctl, Fuse fz,
                void* stream, Fold fo = Fold{0, 0, 1, 0.0, nullptr});
}

int krca_ppr_shard_step(const int64_t* row_ptr, const int32_t* col, const int64_t* plan, int64_t plan_len,
                        const uint16_t* lane, const int64_t* w_all, const int32_t* outdeg, const int64_t* q_local, int64_t n_local,
                        int64_t n_max, int64_t N, double alpha, int32_t flags, int64_t* r_local, int64_t* send,
                        void* ctl, void* stream) {
  return launch_step(row_ptr, col, plan, plan_len, lane, w_all, outdeg, q_local, n_local, n_max, N, alpha, flags, r_local,
                     send, ctl, Fuse{0, 0.0, nullptr}, stream);
}

int krca_ppr_shard_step_folded(const int64_t* row_ptr, const int32_t* col, const int64_t* plan, int64_t plan_len,
                               const uint16_t* lane, const int64_t* w_all, int32_t G, const int32_t* outdeg,
                               const int64_t* q_local, int64_t n_local, int64_t n_max, int64_t N, double alpha,
                               double tol, int32_t it, int32_t flags, int64_t* r_local, int64_t* send,
                               int64_t* next_target, void* ctl, void* stream) {
  KRCA_CHECK_ARG(G >= 1 && it >= 1 && n_max > 0 && N > 0, "krca_ppr_shard_step_folded: bad sizes");
  KRCA_CHECK_ARG(next_target && (next_target == send || (G == 1 && next_target == w_all)),
                 "krca_ppr_shard_step_folded: next_target is send, or w_all at G = 1 (swap exchange)");
  const double err_limit = tol > 0.0 ? (double)N * tol * krca::kFix : 0.0;
  const Fold fo{1, (int)it, (int)G, err_limit, next_target};
  if (plan_len == 0) {  // a rank without rows still does the step's reduction: its ctl (iteration
                        // count, convergence) and slot rotation advance with every other rank's
    KRCA_CHECK_ARG(w_all && ctl && n_local == 0, "krca_ppr_shard_step_folded: no plan for %lld rows",
                   (long long)n_local);
    hipLaunchKernelGGL(ppr_fold_only, dim3(1), dim3(64), 0, krca::as_stream(stream), n_max, alpha,
                       reinterpret_cast<Ctl*>(ctl), fo, w_all);
    KRCA_LAUNCH_CHECK();
    return KRCA_OK;
  }
  return launch_step(row_ptr, col, plan, plan_len, lane, w_all, outdeg, q_local, n_local, n_max, N, alpha, flags, r_local,
                     send, ctl, Fuse{0, 0.0, nullptr}, stream, fo);
}

int krca_ppr_shard_finish(const int64_t* w_all, int32_t G, int64_t n_max, int64_t N, double alpha, double tol,
                          int32_t it, void* ctl, void* stream) {
  KRCA_CHECK_ARG(G >= 1 && it >= 1 && n_max > 0 && N > 0, "krca_ppr_shard_finish: bad sizes");
  KRCA_CHECK_ARG(w_all && ctl, "krca_ppr_shard_finish: null pointer");
  const double err_limit = tol > 0.0 ? (double)N * tol * krca::kFix : 0.0;
  hipLaunchKernelGGL(ppr_finish, dim3(1), dim3(TPB), 0, krca::as_stream(stream), w_all, G, n_max, alpha, err_limit,
                     (int)it, reinterpret_cast<Ctl*>(ctl));
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_ppr_solo_step(const int64_t* row_ptr, const int32_t* col, const int64_t* plan, int64_t plan_len,
                       const uint16_t* lane, int64_t* w, const int32_t* outdeg, const int64_t* q, int64_t N, double alpha,
                       int32_t flags, double tol, int64_t* r, int64_t* send, void* ctl, void* stream) {
  KRCA_CHECK_ARG(plan_len > 0 && N > 0, "krca_ppr_solo_step: bad sizes");
  const double err_limit = tol > 0.0 ? (double)N * tol * krca::kFix : 0.0;
  if (krca::tuning().ppr_fuse)
    return launch_step(row_ptr, col, plan, plan_len, lane, w, outdeg, q, N, N, N, alpha, flags, r, send, ctl,
                       Fuse{1, err_limit, w}, stream);
  // the step, then the reduction over the slice it wrote (zeroing the slots of the buffer it
  // gathered from: the next step's write target)
  if (int rc = launch_step(row_ptr, col, plan, plan_len, lane, w, outdeg, q, N, N, N, alpha, flags, r, send, ctl,
                           Fuse{0, 0.0, nullptr}, stream))
    return rc;
  return krca_ppr_shard_reduce(send, 1, N, N, alpha, tol, 0, ctl, w, stream);
}
}  // extern "C"

namespace {
int launch_step(const int64_t* row_ptr, const int32_t* col, const int64_t* plan, int64_t plan_len, const uint16_t* lane,
                const int64_t* w_all, const int32_t* outdeg, const int64_t* q_local, int64_t n_local, int64_t n_max,
                int64_t N, double alpha, int32_t flags, int64_t* r_local, int64_t* send, void* ctl, Fuse fz,
                void* stream, Fold fo) {
  KRCA_CHECK_ARG(plan_len >= 0 && plan_len % 4 == 0 && n_local >= 0 && n_local <= n_max && N > 0,
                 "krca_ppr_shard_step: bad sizes");
  if (plan_len == 0) return KRCA_OK;
  KRCA_CHECK_ARG(row_ptr && col && plan && lane && w_all && outdeg && q_local && r_local && send && ctl,
                 "krca_ppr_shard_step: null pointer");
  KRCA_CHECK_ARG(w_all != send, "krca_ppr_shard_step: w_all and send must be distinct buffers (ping-pong)");
  const int64_t nblk = plan_len / 4;
  // workgroups the stream's device keeps resident (occupancy API, cached per device)
  const int64_t occupancy =
      krca::resident_workgroups(reinterpret_cast<const void*>(&ppr_step<0>), TPB, krca::as_stream(stream), 4);
  const int64_t resident = krca::tuning().ppr_grid > 0 ? (int64_t)krca::tuning().ppr_grid : occupancy;
  const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(nblk, resident));
  const bool nt = krca::tuning().ppr_nt != 0;
  const int xcd = krca::tuning().ppr_xcd != 0 && grid % 8 == 0 && nblk >= grid;
  auto kern = (flags & KRCA_PPR_RESIDUAL) ? (nt ? ppr_step<PPR_RESIDUAL | PPR_WRITE_R | PPR_NT> : ppr_step<PPR_RESIDUAL | PPR_WRITE_R>)
              : (flags & KRCA_PPR_WRITE_R) ? (nt ? ppr_step<PPR_WRITE_R | PPR_NT> : ppr_step<PPR_WRITE_R>)
                                           : (nt ? ppr_step<PPR_NT> : ppr_step<0>);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(TPB), 0, krca::as_stream(stream), row_ptr, col, plan, lane, nblk,
                     reinterpret_cast<const uint32_t*>(w_all), outdeg, q_local, n_local, N, alpha, r_local, send, n_max,
                     reinterpret_cast<Ctl*>(ctl), fz, fo, xcd);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}
}  // namespace

extern "C" {

int krca_ppr_shard_reduce(const int64_t* w_all, int32_t G, int64_t n_max, int64_t N, double alpha, double tol,
                          int32_t first, void* ctl, int64_t* send_next, void* stream) {
  KRCA_CHECK_ARG(G >= 1 && n_max > 0 && N > 0, "krca_ppr_shard_reduce: bad sizes");
  KRCA_CHECK_ARG(w_all && ctl && send_next, "krca_ppr_shard_reduce: null pointer");
  const double err_limit = tol > 0.0 ? (double)N * tol * krca::kFix : 0.0;
  hipLaunchKernelGGL(ppr_reduce, dim3(1), dim3(TPB), 0, krca::as_stream(stream), w_all, G, n_max, alpha, err_limit,
                     (int)first, reinterpret_cast<Ctl*>(ctl), send_next);
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

int krca_ppr_ctl_copy(const void* ctl, int32_t* host, void* stream) {
  KRCA_CHECK_ARG(ctl && host, "krca_ppr_ctl_copy: null pointer");
  static_assert(offsetof(Ctl, iter) == offsetof(Ctl, converged) + 4, "converged, iter adjacent");
  KRCA_HIP(hipMemcpyAsync(host, &reinterpret_cast<const Ctl*>(ctl)->converged, 2 * sizeof(int32_t),
                          hipMemcpyDeviceToHost, krca::as_stream(stream)));
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

int krca_rca_key_explained(const int64_t* r, const int64_t* q, const int64_t* d, int64_t n, int64_t N, const void* ctl,
                           int64_t* key, void* stream) {
  if (n <= 0) return KRCA_OK;
  KRCA_CHECK_ARG(n <= N && N < INT32_MAX, "krca_rca_key_explained: bad sizes");
  KRCA_CHECK_ARG(r && q && d && ctl && key, "krca_rca_key_explained: null pointer");
  hipLaunchKernelGGL(rca_key_explained, dim3(grid_for(n)), dim3(TPB), 0, krca::as_stream(stream), r, q, d, n, N,
                     reinterpret_cast<const Ctl*>(ctl), key);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

// workspace: ctl (krca_ppr_ctl_size(N), zeroed here once) | q[N] | w0[slice(N)] | w1[slice(N)] | r[N]
int64_t krca_ppr_workspace_size(int64_t N) {
  return krca::ceil_div(krca_ppr_ctl_size(N), 256) * 256 + (2 * N + 2 * slice_words(N)) * 8 + 256;
}

int krca_ppr(const int64_t* row_ptr, const int32_t* col, const int32_t* outdeg, int64_t N, const int64_t* plan,
             int64_t plan_len, const uint16_t* lane, const float* seed, float seed_floor, double alpha, int32_t max_iter, double tol,
             void* workspace, float* r_out, int64_t* r_fixed, int64_t* q_out, int32_t* iters_host, void* stream) {
  KRCA_CHECK_ARG(N > 0 && N <= kMaxSeedN, "krca_ppr: N=%lld out of range", (long long)N);
  KRCA_CHECK_ARG(row_ptr && col && outdeg && plan && lane && seed && workspace && r_out, "krca_ppr: null pointer");
  KRCA_CHECK_ARG(plan_len > 0 && plan_len % 4 == 0, "krca_ppr: bad plan");
  KRCA_CHECK_ARG(alpha > 0.0 && alpha < 1.0 && max_iter > 0, "krca_ppr: alpha in (0,1), max_iter > 0");
  char* ctl = reinterpret_cast<char*>(workspace);
  const int64_t ctl_bytes = krca::ceil_div(krca_ppr_ctl_size(N), 256) * 256;
  char* p = ctl + ctl_bytes;
  int64_t* q = q_out ? q_out : reinterpret_cast<int64_t*>(p);
  int64_t* wb[2] = {reinterpret_cast<int64_t*>(p + N * 8), reinterpret_cast<int64_t*>(p + (N + slice_words(N)) * 8)};
  int64_t* r = r_fixed ? r_fixed : reinterpret_cast<int64_t*>(p + (N + 2 * slice_words(N)) * 8);
  hipStream_t st = krca::as_stream(stream);
  KRCA_HIP(hipMemsetAsync(ctl, 0, ctl_bytes, st));
  int rc = krca_ppr_shard_init(seed, seed_floor, outdeg, N, N, N, alpha, ctl, q, r, wb[0], stream);
  if (rc) return rc;
  // folded iterations (one kernel each: step it reduces step it - 1 first); the first writes its
  // partial sums into the other buffer's slots, zeroed here
  KRCA_HIP(hipMemsetAsync(wb[1] + wslots(N), 0, NSLOT * sizeof(int64_t), st));
  const int check_every = 8;
  int32_t iters = 0, conv = 0;
  int cur = 0;  // w buffer the next step gathers from
  int it = 0;
  while (it < max_iter) {
    ++it;
    const int32_t flags = tol > 0.0 ? (KRCA_PPR_RESIDUAL | KRCA_PPR_WRITE_R) : (it == max_iter ? KRCA_PPR_WRITE_R : 0);
    if ((rc = krca_ppr_shard_step_folded(row_ptr, col, plan, plan_len, lane, wb[cur], 1, outdeg, q, N, N, N, alpha, tol,
                                         it, flags, r, wb[cur ^ 1], wb[cur], ctl, stream)))
      return rc;
    cur ^= 1;
    if (tol > 0.0 && it % check_every == 0 && it < max_iter) {  // step it's own test is in step it + 1
      if ((rc = krca_ppr_ctl_read(ctl, &iters, &conv, stream))) return rc;
      if (conv) break;
    }
  }
  if ((rc = krca_ppr_shard_finish(wb[cur], 1, N, N, alpha, tol, it, ctl, stream))) return rc;
  if ((rc = krca_ppr_fixed_to_float(r, N, r_out, stream))) return rc;
  if ((rc = krca_ppr_ctl_read(ctl, &iters, &conv, stream))) return rc;
  if (iters_host) *iters_host = iters;
  if (tol > 0.0 && !conv) {
    krca::set_error("krca_ppr: no convergence in %d iterations", max_iter);
    return KRCA_ENOTCONV;
  }
  return KRCA_OK;
}

#ifdef PPR_TIMING
int krca_ppr_debug_timing(unsigned long long* host, int reset) {
  KRCA_HIP(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ppr_timing), sizeof(g_ppr_timing)));
  if (reset) {
    static unsigned long long zero[4096 * 5];
    KRCA_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_ppr_timing), zero, sizeof(zero)));
  }
  return KRCA_OK;
}
#endif
}  // extern "C"

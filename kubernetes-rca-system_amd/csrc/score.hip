// Per-pod scoring kernels.
//
//  krca_usage_flags    — the instantaneous CPU / memory thresholds of
//                        ref:agents/metrics_agent.py:88-114 and :135-161 (x > 80 strict, high if > 90).
//  krca_rolling_score  — rolling-window z-scores over a time-major [T][P][M] float32 tensor.
//
// Design (MI355X): HBM-streaming, one lane per series s = p*M + m.  At every time step a wave
// reads 64 consecutive floats (256 B, fully coalesced) and the trailing window of W samples
// lives in registers (a W-entry ring indexed by the compile-time position inside an unrolled
// W-step block), so each input byte crosses HBM exactly once: 4*P*M*T bytes per call.  The
// window statistics are float64 sliding sums updated in a FIXED order, so the integer outputs
// (n_exceed, flags) are bit-identical to the C restatement in oracle/krca_oracle.c; the
// threshold test is |z| > thr  <=>  A^2 > thr^2*B (A = W*x - s1, B = W*s2 - s1^2), with no
// division or square root; all products that feed a decision are explicit fma()s.
// Pod-level reductions (max |z|, sum of exceedances, flag OR) are wave shuffles inside the
// aligned M-lane group of the pod.
#include "krca_common.h"

#pragma clang fp contract(off)

namespace {

constexpr double kVarEps = 1e-12;

__global__ __launch_bounds__(256) void usage_flags_kernel(const float2* __restrict__ usage, int64_t P,
                                                          uint8_t* __restrict__ flags) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < P; p += stride) {
    const float2 u = usage[p];
    flags[p] = (u.x > 80.f ? KRCA_F_CPU80 : 0u) | (u.x > 90.f ? KRCA_F_CPU90 : 0u) |
               (u.y > 80.f ? KRCA_F_MEM80 : 0u) | (u.y > 90.f ? KRCA_F_MEM90 : 0u);
  }
}

struct StepState {
  double s1, s2;  // window sum and sum of squares (float64, fixed order)
  int cnt;        // exceedances of this series
  double al, bl;  // A and B (below) at t = T-1
};

// One time step of the rolling statistics; `old` is x[t-W].  With A = W*x_t - s1 and
// B = W*s2 - s1^2 (= W^2 * var, ddof 0):  z = A / sqrt(B),  |z| > thr  <=>  A^2 > thr^2 * B,
// var > 1e-12  <=>  B > 1e-12 * W^2 — 13 float64 operations per sample, no division or sqrt.
// The fma()s are explicit (and mirrored in oracle/krca_oracle.c): one rounding each.
__device__ __forceinline__ void step(StepState& st, float v, float old, double Wd, double epsB, double thr2,
                                     bool last) {
  const double vd = (double)v;
  const double od = (double)old;
  const double A = fma(Wd, vd, -st.s1);
  const double B = fma(Wd, st.s2, -(st.s1 * st.s1));
  st.cnt += (B > epsB) && (fma(A, A, -(thr2 * B)) > 0.0);
  if (last) {
    st.al = A;
    st.bl = B;
  }
  st.s1 = (st.s1 + vd) - od;
  st.s2 = fma(-od, od, fma(vd, vd, st.s2));
}

// Pod epilogue shared by both kernels: z_last per series, pod max|z|, exceedance sum, flags.
__device__ __forceinline__ void pod_epilogue(const StepState& st, double epsB, int64_t s, bool active, int M, int T,
                                             const float* __restrict__ xs, int64_t S,
                                             float* __restrict__ z_last, float* __restrict__ score,
                                             int32_t* __restrict__ n_exceed, uint8_t* __restrict__ flags) {
  const bool has_z = st.bl > epsB;
  const float z = has_z ? (float)(st.al / sqrt(st.bl)) : 0.f;
  const int m = (int)(s & (M - 1));
  float vlast = (active && T > 0) ? xs[(int64_t)(T - 1) * S] : 0.f;
  unsigned f = 0;
  if (m == 0) f = (vlast > 80.f ? KRCA_F_CPU80 : 0u) | (vlast > 90.f ? KRCA_F_CPU90 : 0u);
  if (m == 1) f = (vlast > 80.f ? KRCA_F_MEM80 : 0u) | (vlast > 90.f ? KRCA_F_MEM90 : 0u);
  float az = fabsf(z);
  int cnt = st.cnt;
  for (int off = 1; off < M; off <<= 1) {  // the M lanes of a pod are aligned inside the wave
    az = fmaxf(az, __shfl_xor(az, off, 64));
    cnt += __shfl_xor(cnt, off, 64);
    f |= __shfl_xor(f, off, 64);
  }
  if (!active) return;
  z_last[s] = z;
  if (m == 0) {
    const int64_t p = s / M;
    score[p] = az;
    n_exceed[p] = cnt;
    flags[p] = (uint8_t)f;
  }
}

template <int W>
__global__ __launch_bounds__(256) void rolling_score_ring(const float* __restrict__ x, int64_t S, int T, int M,
                                                          double thr2, float* __restrict__ z_last,
                                                          float* __restrict__ score, int32_t* __restrict__ n_exceed,
                                                          uint8_t* __restrict__ flags) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = s < S;
  const float* xs = x + (active ? s : 0);
  const double Wd = (double)W, epsB = kVarEps * Wd * Wd;
  StepState st{0.0, 0.0, 0, 0.0, 0.0};
  float ring[W];
#pragma unroll
  for (int j = 0; j < W; ++j) {
    const float v = (j < T && active) ? xs[(int64_t)j * S] : 0.f;
    ring[j] = v;
    const double vd = (double)v;
    st.s1 = st.s1 + vd;
    st.s2 = fma(vd, vd, st.s2);
  }
  int t0 = W;
  for (; t0 + W <= T; t0 += W) {  // full W-step blocks: every ring slot index is static
    float nx[W];
#pragma unroll
    for (int j = 0; j < W; ++j) nx[j] = active ? xs[(int64_t)(t0 + j) * S] : 0.f;
#pragma unroll
    for (int j = 0; j < W; ++j) {
      step(st, nx[j], ring[j], Wd, epsB, thr2, t0 + j == T - 1);
      ring[j] = nx[j];
    }
  }
  if (t0 < T) {  // tail block
#pragma unroll
    for (int j = 0; j < W; ++j) {
      if (t0 + j < T) {
        const float v = active ? xs[(int64_t)(t0 + j) * S] : 0.f;
        step(st, v, ring[j], Wd, epsB, thr2, t0 + j == T - 1);
        ring[j] = v;
      }
    }
  }
  pod_epilogue(st, epsB, s, active, M, T, xs, S, z_last, score, n_exceed, flags);
}

// Same arithmetic as rolling_score_ring; addressing for gfx950 buffer loads: per W-step block a
// wave-uniform buffer descriptor on the block's first row, the lane's 32-bit byte offset in
// voffset and the row offset j*S*4 in soffset, so a load costs no per-lane address arithmetic
// (`buffer_load_dword v, v_off, s[rsrc], s_off offen`).  Requires 4*S*W < 2^31.
template <int AUX = 0>  // cache policy bits: 0 default, 2 = nt (streamed once)
__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, AUX));
}

template <int W>
__global__ __launch_bounds__(256) void rolling_score_ring_buf(const float* __restrict__ x, int64_t S, int T, int M,
                                                              double thr2, float* __restrict__ z_last,
                                                              float* __restrict__ score,
                                                              int32_t* __restrict__ n_exceed,
                                                              uint8_t* __restrict__ flags) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = s < S;
  const uint32_t voff = active ? (uint32_t)s * 4u : 0u;
  const uint32_t rowb = (uint32_t)(S * 4);  // bytes per time row
  const double Wd = (double)W, epsB = kVarEps * Wd * Wd;
  StepState st{0.0, 0.0, 0, 0.0, 0.0};
  float ring[W];
  const int Tw = T < W ? T : W;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, (int)(rowb * (uint32_t)Tw), 0x00020000);
#pragma unroll
  for (int j = 0; j < W; ++j) {
    const float v = j < T ? bload(rs, voff, rowb * j) : 0.f;
    ring[j] = v;
    const double vd = (double)v;
    st.s1 = st.s1 + vd;
    st.s2 = fma(vd, vd, st.s2);
  }
  int t0 = W;
  for (; t0 + W <= T; t0 += W) {
    rs = __builtin_amdgcn_make_buffer_rsrc((void*)(x + (int64_t)t0 * S), 0, (int)(rowb * (uint32_t)W), 0x00020000);
    float nx[W];
#pragma unroll
    for (int j = 0; j < W; ++j) nx[j] = bload(rs, voff, rowb * j);
#pragma unroll
    for (int j = 0; j < W; ++j) {
      step(st, nx[j], ring[j], Wd, epsB, thr2, t0 + j == T - 1);
      ring[j] = nx[j];
    }
  }
  if (t0 < T) {
    rs = __builtin_amdgcn_make_buffer_rsrc((void*)(x + (int64_t)t0 * S), 0, (int)(rowb * (uint32_t)(T - t0)),
                                           0x00020000);
#pragma unroll
    for (int j = 0; j < W; ++j) {
      if (t0 + j < T) {
        const float v = bload(rs, voff, rowb * j);
        step(st, v, ring[j], Wd, epsB, thr2, t0 + j == T - 1);
        ring[j] = v;
      }
    }
  }
  pod_epilogue(st, epsB, s, active, M, T, x + (active ? s : 0), S, z_last, score, n_exceed, flags);
}

// Software-pipelined form of rolling_score_ring_buf (same arithmetic, same bits).  The time axis
// is walked in C-row chunks (W % C == 0, so every ring slot index stays static); the loads of
// chunk c+1 are issued before chunk c is computed, so each wave keeps C rows (C*256 B) in flight
// through its whole compute phase instead of alternating load bursts and VALU bursts.  Only the
// final block (the one holding t = T-1) tracks the last-step A/B, so the steady-state loop has
// no per-sample select.  Buffer descriptors cover exactly the rows < T of a chunk: loads past the
// end return 0 and touch no memory, which lets the prefetch run ahead unconditionally.
template <int C>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t chunk_rsrc(const float* x, int64_t S, uint32_t rowb, int t,
                                                             int T) {
  int n = T - t;
  n = n < 0 ? 0 : (n > C ? C : n);
  n = __builtin_amdgcn_readfirstlane(n);  // wave-uniform: keeps the descriptor in SGPRs (no v_med3 waterfall)
  return __builtin_amdgcn_make_buffer_rsrc((void*)(x + (int64_t)(n ? t : 0) * S), 0, (int)(rowb * (uint32_t)n),
                                           0x00020000);
}

// Row sources of the pipelined kernel.  SpanRows: one descriptor per chunk spanning its C rows
// (needs 4*S*C < 2^31: up to ~3.3M pods x 8 metrics at C = 20).  BlockRows: one descriptor per
// row covering only the workgroup's 256 series (base = x + t*S + s0), so any S < 2^32 works; it
// costs a few scalar instructions per row, off the vector path.
struct SpanRows {
  const float* x;
  int64_t S;
  uint32_t rowb, voff;
  int T;
  __device__ __forceinline__ SpanRows(const float* x_, int64_t S_, int T_, int64_t s, bool active)
      : x(x_), S(S_), rowb((uint32_t)(S_ * 4)), voff(active ? (uint32_t)s * 4u : 0u), T(T_) {}
  template <int C, int AUX>
  __device__ __forceinline__ void load(int t, float (&out)[C]) const {
    const __amdgpu_buffer_rsrc_t rs = chunk_rsrc<C>(x, S, rowb, t, T);
#pragma unroll
    for (int j = 0; j < C; ++j) out[j] = bload<AUX>(rs, voff, rowb * j);
  }
};

struct BlockRows {
  const float* xb;  // x + s0, s0 = the workgroup's first series
  int64_t S;
  uint32_t voff;
  int nrec;  // bytes of the workgroup's series inside [0, S)
  int T;
  __device__ __forceinline__ BlockRows(const float* x_, int64_t S_, int T_, int64_t, bool)
      : S(S_), voff(threadIdx.x * 4u), T(T_) {
    const int64_t s0 = (int64_t)blockIdx.x * blockDim.x;
    xb = x_ + s0;
    const int64_t n = S_ - s0;
    nrec = __builtin_amdgcn_readfirstlane((int)(4 * (n < (int64_t)blockDim.x ? n : (int64_t)blockDim.x)));
  }
  template <int C, int AUX>
  __device__ __forceinline__ void load(int t, float (&out)[C]) const {
#pragma unroll
    for (int j = 0; j < C; ++j) {
      const int tt = t + j;
      const bool in = tt < T;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(xb + (int64_t)(in ? tt : 0) * S), 0, in ? nrec : 0, 0x00020000);
      out[j] = bload<AUX>(rs, voff, 0);
    }
  }
};

template <int W, int C, int AUX = 0, class Rows = SpanRows>
__global__ __launch_bounds__(256) void rolling_score_pipe(const float* __restrict__ x, int64_t S, int T, int M,
                                                          double thr2, float* __restrict__ z_last,
                                                          float* __restrict__ score, int32_t* __restrict__ n_exceed,
                                                          uint8_t* __restrict__ flags) {
  static_assert(W % C == 0, "chunk must divide the window");
  constexpr int NC = W / C;
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = s < S;
  const Rows rows(x, S, T, s, active);
  const double Wd = (double)W, epsB = kVarEps * Wd * Wd;
  StepState st{0.0, 0.0, 0, 0.0, 0.0};
  float ring[W];
  float cur[C];
  // prologue: rows [0, W) fill the window (requires T > W, checked by the launcher)
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    float tmp[C];
    rows.template load<C, AUX>(c * C, tmp);
#pragma unroll
    for (int j = 0; j < C; ++j) ring[c * C + j] = tmp[j];
  }
  rows.template load<C, AUX>(W, cur);
#pragma unroll
  for (int j = 0; j < W; ++j) {
    const double vd = (double)ring[j];
    st.s1 = st.s1 + vd;
    st.s2 = fma(vd, vd, st.s2);
  }
  int t0 = W;
  for (; t0 + W < T; t0 += W) {  // full blocks that do not contain t = T-1
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      float nxt[C];
      rows.template load<C, AUX>(t0 + (c + 1) * C, nxt);
#pragma unroll
      for (int j = 0; j < C; ++j) {
        step(st, cur[j], ring[c * C + j], Wd, epsB, thr2, false);
        ring[c * C + j] = cur[j];
      }
#pragma unroll
      for (int j = 0; j < C; ++j) cur[j] = nxt[j];
    }
  }
  // final block: rows [t0, T), 1..W of them; cur already holds rows [t0, t0 + C)
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (c > 0) rows.template load<C, AUX>(t0 + c * C, cur);
#pragma unroll
    for (int j = 0; j < C; ++j) {
      const int t = t0 + c * C + j;
      if (t < T) {
        step(st, cur[j], ring[c * C + j], Wd, epsB, thr2, t == T - 1);
        ring[c * C + j] = cur[j];
      }
    }
  }
  pod_epilogue(st, epsB, s, active, M, T, x + (active ? s : 0), S, z_last, score, n_exceed, flags);
}

// LDS-DMA form of rolling_score_pipe (KRCA_SCORE_IMPL=5, A/B; same steps in the same order, same
// bits).  The workgroup's 256 series of a time row are 1 KiB contiguous: ONE wave instruction
// (global_load_lds_dwordx4, 16 B per lane) lands a whole row in LDS, instead of four 256-B register
// loads; a C-row chunk is C / 4 such instructions per wave, double-buffered (2 x C KiB), the next
// chunk's in flight while the current one is stepped from LDS.  Needs S % 4 == 0 (16-B aligned rows);
// the last workgroup's lanes past S re-read its first piece (their values are never used).
template <int W, int C, int AUX>
__global__ __launch_bounds__(256) void rolling_score_lds(const float* __restrict__ x, int64_t S, int T, int M,
                                                         double thr2, float* __restrict__ z_last,
                                                         float* __restrict__ score, int32_t* __restrict__ n_exceed,
                                                         uint8_t* __restrict__ flags) {
  static_assert(W % C == 0 && C % 4 == 0, "chunk must divide the window and split over 4 waves");
  constexpr int NC = W / C;
  __shared__ float stage[2][C][256];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t s0 = (int64_t)blockIdx.x * 256;
  const int64_t s = s0 + tid;
  const bool active = s < S;
  const int64_t piece = s0 + 4 * lane < S ? s0 + 4 * lane : s0;
  // rows [t, t + C) of the workgroup's series into stage[buf]; rows >= T are not loaded (never read)
  auto dma = [&](int buf, int t) {
#pragma unroll
    for (int q = 0; q < C / 4; ++q) {
      const int j = wv + 4 * q;
      if (t + j < T)
        __builtin_amdgcn_global_load_lds(x + (int64_t)(t + j) * S + piece,
                                         (__attribute__((address_space(3))) void*)&stage[buf][j][0], 16, 0, AUX);
    }
  };
  auto landed = [&]() {  // this wave's DMA done, then every wave's
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  const double Wd = (double)W, epsB = kVarEps * Wd * Wd;
  StepState st{0.0, 0.0, 0, 0.0, 0.0};
  float ring[W];
  // prologue: chunks 0 .. NC-1 fill the window (requires T > W, checked by the launcher)
  dma(0, 0);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    landed();
    dma((c + 1) & 1, (c + 1) * C);  // the next chunk (chunk NC: the first rows past the window)
#pragma unroll
    for (int j = 0; j < C; ++j) ring[c * C + j] = stage[c & 1][j][tid];
  }
#pragma unroll
  for (int j = 0; j < W; ++j) {
    const double vd = (double)ring[j];
    st.s1 = st.s1 + vd;
    st.s2 = fma(vd, vd, st.s2);
  }
  int k = NC;  // chunk k = rows [k C, k C + C) is in flight into stage[k & 1]
  int t0 = W;
  for (; t0 + W < T; t0 += W) {  // full blocks that do not contain t = T-1
#pragma unroll
    for (int c = 0; c < NC; ++c, ++k) {
      landed();
      dma((k + 1) & 1, (k + 1) * C);
      const int b = k & 1;
#pragma unroll
      for (int j = 0; j < C; ++j) {
        const float v = stage[b][j][tid];
        step(st, v, ring[c * C + j], Wd, epsB, thr2, false);
        ring[c * C + j] = v;
      }
    }
  }
  // final block: rows [t0, T), 1..W of them
#pragma unroll
  for (int c = 0; c < NC; ++c, ++k) {
    landed();
    if (c + 1 < NC) dma((k + 1) & 1, (k + 1) * C);
    const int b = k & 1;
#pragma unroll
    for (int j = 0; j < C; ++j) {
      const int t = t0 + c * C + j;
      if (t < T) {
        const float v = stage[b][j][tid];
        step(st, v, ring[c * C + j], Wd, epsB, thr2, t == T - 1);
        ring[c * C + j] = v;
      }
    }
  }
  pod_epilogue(st, epsB, s, active, M, T, x + (active ? s : 0), S, z_last, score, n_exceed, flags);
}

// Any W: the outgoing sample x[t-W] is re-read (same values, same arithmetic -> same bits).
__global__ __launch_bounds__(256) void rolling_score_reread(const float* __restrict__ x, int64_t S, int T, int W,
                                                            int M, double thr2, float* __restrict__ z_last,
                                                            float* __restrict__ score,
                                                            int32_t* __restrict__ n_exceed,
                                                            uint8_t* __restrict__ flags) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = s < S;
  const float* xs = x + (active ? s : 0);
  const double Wd = (double)W, epsB = kVarEps * Wd * Wd;
  StepState st{0.0, 0.0, 0, 0.0, 0.0};
  for (int j = 0; j < W && j < T; ++j) {
    const double vd = active ? (double)xs[(int64_t)j * S] : 0.0;
    st.s1 = st.s1 + vd;
    st.s2 = fma(vd, vd, st.s2);
  }
  for (int t = W; t < T; ++t) {
    const float v = active ? xs[(int64_t)t * S] : 0.f;
    const float o = active ? xs[(int64_t)(t - W) * S] : 0.f;
    step(st, v, o, Wd, epsB, thr2, t == T - 1);
  }
  pod_epilogue(st, epsB, s, active, M, T, xs, S, z_last, score, n_exceed, flags);
}

// ---- streaming rescoring (BASELINE configs[4]) ----------------------------
// The batch scorer applied to an unbounded stream, carried forward window by window: state per
// series = the float64 window sums (s1, s2), the last W samples (ring [W][S]) and the exceedance
// bits of the last H evaluated steps (bits [ceil(H/32)][S]) with their count.  A window of delta
// new steps t0 .. t0+delta-1 runs exactly the batch kernel's operations for those steps (the
// prologue sums while t < W, step() after), so after any sequence of windows z_last / score /
// flags equal krca_rolling_score over the whole series so far, and n_exceed counts its
// exceedances over the last H evaluated steps (all of them while there are fewer than H).
// Per series and window: 20 B of state read + written, 12*delta B of samples (new, old, ring
// write) and 8*delta B of exceedance bits.
struct StreamState {
  double* s1;
  double* s2;
  int32_t* cnt;
  float* ring;
  uint32_t* bits;
};

__global__ __launch_bounds__(256) void stream_score(const float* __restrict__ xn, int64_t S, int delta, int64_t t0,
                                                    int W, int H, int M, double thr2, StreamState stt,
                                                    float* __restrict__ z_last, float* __restrict__ score,
                                                    int32_t* __restrict__ n_exceed, uint8_t* __restrict__ flags) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = s < S;
  const int64_t sl = active ? s : 0;
  const double Wd = (double)W, epsB = kVarEps * Wd * Wd;
  StepState st{0.0, 0.0, 0, 0.0, 0.0};
  int cnt = 0;
  if (t0 > 0) {
    st.s1 = stt.s1[sl];
    st.s2 = stt.s2[sl];
    cnt = stt.cnt[sl];
  }
  for (int j = 0; j < delta; ++j) {
    const int64_t t = t0 + j;
    const float v = xn[(int64_t)j * S + sl];
    float* rp = stt.ring + (t % W) * S + sl;
    if (t < W) {  // the batch prologue: window fill
      const double vd = (double)v;
      st.s1 = st.s1 + vd;
      st.s2 = fma(vd, vd, st.s2);
    } else {
      const float o = *rp;
      st.cnt = 0;
      step(st, v, o, Wd, epsB, thr2, j == delta - 1);
      const int64_t e = t - W;  // index among the evaluated steps
      uint32_t* wp = stt.bits + ((e % H) >> 5) * S + sl;
      const uint32_t bit = 1u << ((e % H) & 31);
      const uint32_t word = *wp;  // zeroed when the stream starts (t0 == 0)
      cnt += st.cnt - ((word & bit) ? 1 : 0);
      if (active) *wp = st.cnt ? (word | bit) : (word & ~bit);
    }
    if (active) *rp = v;
  }
  if (active) {
    stt.s1[sl] = st.s1;
    stt.s2[sl] = st.s2;
    stt.cnt[sl] = cnt;
  }
  st.cnt = cnt;
  if (t0 + delta - 1 < W) st.bl = 0.0;  // no evaluated step yet: z = 0
  pod_epilogue(st, epsB, s, active, M, delta, xn + sl, S, z_last, score, n_exceed, flags);
}

int rows_per_chunk(int W) {
  return W == 60 ? krca::tuning().score_chunk : (W == 30 ? 15 : (W == 20 ? 10 : W));
}
bool pipe_window(int W) { return W == 60 || W == 30 || W == 20 || W == 15 || W == 10; }
}  // namespace

extern "C" {

// state: s1, s2 f64 [S] | cnt i32 [S] | ring f32 [W][S] | bits u32 [ceil(H/32)][S]  (S = P*M)
int64_t krca_stream_state_size(int64_t P, int32_t M, int32_t W, int32_t H) {
  const int64_t S = P * M;
  return S * (8 + 8 + 4) + (int64_t)W * S * 4 + krca::ceil_div(H, 32) * S * 4 + 64;
}

int krca_stream_score(const float* x_new, int64_t P, int32_t M, int32_t delta, int64_t t0, int32_t W, int32_t H,
                      float z_thr, void* state, float* z_last, float* score, int32_t* n_exceed, uint8_t* flags,
                      void* stream) {
  KRCA_CHECK_ARG(P >= 0 && delta >= 1 && t0 >= 0 && W >= 1 && H >= 1, "krca_stream_score: bad sizes");
  KRCA_CHECK_ARG(M >= 1 && M <= 64 && (M & (M - 1)) == 0, "krca_stream_score: M=%d must be a power of two <= 64", M);
  if (P == 0) return KRCA_OK;
  KRCA_CHECK_ARG(x_new && state && z_last && score && n_exceed && flags, "krca_stream_score: null pointer");
  const int64_t S = P * (int64_t)M;
  char* b = reinterpret_cast<char*>(state);
  StreamState stt;
  stt.s1 = reinterpret_cast<double*>(b);
  stt.s2 = stt.s1 + S;
  stt.cnt = reinterpret_cast<int32_t*>(stt.s2 + S);
  stt.ring = reinterpret_cast<float*>(stt.cnt + S);
  stt.bits = reinterpret_cast<uint32_t*>(stt.ring + (int64_t)W * S);
  hipStream_t st = krca::as_stream(stream);
  if (t0 == 0) KRCA_HIP(hipMemsetAsync(stt.bits, 0, krca::ceil_div(H, 32) * S * 4, st));
  hipLaunchKernelGGL(stream_score, dim3((unsigned)krca::ceil_div(S, 256)), dim3(256), 0, st, x_new, S, delta, t0, W,
                     H, M, (double)z_thr * (double)z_thr, stt, z_last, score, n_exceed, flags);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_usage_flags(const float* usage, int64_t P, uint8_t* flags, void* stream) {
  KRCA_CHECK_ARG(P >= 0, "krca_usage_flags: P < 0");
  if (P == 0) return KRCA_OK;
  KRCA_CHECK_ARG(usage && flags, "krca_usage_flags: null pointer");
  const int64_t blocks = std::min<int64_t>(krca::ceil_div(P, 256), 4096);
  hipLaunchKernelGGL(usage_flags_kernel, dim3((unsigned)blocks), dim3(256), 0, krca::as_stream(stream),
                     reinterpret_cast<const float2*>(usage), P, flags);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_rolling_score_variant(int64_t P, int32_t M, int32_t T, int32_t W) {
  const krca::Tuning& tu = krca::tuning();
  const int64_t S = P * (int64_t)M;
  if (!pipe_window(W)) return KRCA_SCORE_REREAD;
  if (tu.score_impl == KRCA_SCORE_PIPE_ROWS && T > W) return KRCA_SCORE_PIPE_ROWS;  // A/B: forced
  if (tu.score_impl == KRCA_SCORE_LDS && T > W && W == 60 && S % 4 == 0) return KRCA_SCORE_LDS;  // A/B
  if (tu.score_impl == 0 && T > W) {
    return S * 4 * rows_per_chunk(W) < (int64_t(1) << 31) ? KRCA_SCORE_PIPE : KRCA_SCORE_PIPE_ROWS;
  }
  return tu.score_impl == 2 && S * 4 * W < (int64_t(1) << 31) ? KRCA_SCORE_RING_BUF : KRCA_SCORE_RING;
}

int krca_rolling_score(const float* x, int64_t P, int32_t M, int32_t T, int32_t W, float z_thr, float* z_last,
                       float* score, int32_t* n_exceed, uint8_t* flags, void* stream) {
  KRCA_CHECK_ARG(P >= 0 && T >= 0 && W >= 1, "krca_rolling_score: bad sizes P=%lld T=%d W=%d", (long long)P, T, W);
  KRCA_CHECK_ARG(M >= 1 && M <= 64 && (M & (M - 1)) == 0, "krca_rolling_score: M=%d must be a power of two <= 64", M);
  if (P == 0) return KRCA_OK;
  KRCA_CHECK_ARG(x && z_last && score && n_exceed && flags, "krca_rolling_score: null pointer");
  const int64_t S = P * (int64_t)M;
  KRCA_CHECK_ARG(S < (int64_t(1) << 32), "krca_rolling_score: P*M must be < 2^32");
  const double thr2 = (double)z_thr * (double)z_thr;
  const dim3 grid((unsigned)krca::ceil_div(S, 256)), block(256);
  hipStream_t st = krca::as_stream(stream);
  // the metric stream is read once: non-temporal loads (cache policy nt) by default, 6.17 -> 6.61 TB/s
  // at C4 (tools/score_ab.py); KRCA_SCORE_NT=0 restores the default policy
  const bool nt = krca::tuning().score_nt != 0;
  const int chunk = rows_per_chunk(W);
  const int variant = krca_rolling_score_variant(P, M, T, W);
#define KRCA_PIPE_AS(WV, CV, ROWS)                                                                               \
  if (nt)                                                                                                        \
    hipLaunchKernelGGL((rolling_score_pipe<WV, CV, 2, ROWS>), grid, block, 0, st, x, S, T, M, thr2, z_last, score, \
                       n_exceed, flags);                                                                         \
  else                                                                                                           \
    hipLaunchKernelGGL((rolling_score_pipe<WV, CV, 0, ROWS>), grid, block, 0, st, x, S, T, M, thr2, z_last, score, \
                       n_exceed, flags);
#define KRCA_PIPE(WV, CV)                                    \
  if (variant == KRCA_SCORE_PIPE) { KRCA_PIPE_AS(WV, CV, SpanRows) } \
  else { KRCA_PIPE_AS(WV, CV, BlockRows) }
#define KRCA_RING(WV)                                                                                         \
  if (variant == KRCA_SCORE_RING_BUF)                                                                         \
    hipLaunchKernelGGL(rolling_score_ring_buf<WV>, grid, block, 0, st, x, S, T, M, thr2, z_last, score,        \
                       n_exceed, flags);                                                                       \
  else                                                                                                         \
    hipLaunchKernelGGL(rolling_score_ring<WV>, grid, block, 0, st, x, S, T, M, thr2, z_last, score, n_exceed,  \
                       flags);
  const bool pipe = variant == KRCA_SCORE_PIPE || variant == KRCA_SCORE_PIPE_ROWS;
  if (variant == KRCA_SCORE_LDS) {  // W = 60, C = 20 only
    if (nt)
      hipLaunchKernelGGL((rolling_score_lds<60, 20, 2>), grid, block, 0, st, x, S, T, M, thr2, z_last, score, n_exceed,
                         flags);
    else
      hipLaunchKernelGGL((rolling_score_lds<60, 20, 0>), grid, block, 0, st, x, S, T, M, thr2, z_last, score, n_exceed,
                         flags);
  } else switch (W) {
    case 60:
      if (pipe && chunk == 10) { KRCA_PIPE(60, 10) }
      else if (pipe && chunk == 12) { KRCA_PIPE(60, 12) }
      else if (pipe && chunk == 15) { KRCA_PIPE(60, 15) }
      else if (pipe && chunk == 30) { KRCA_PIPE(60, 30) }
      else if (pipe) { KRCA_PIPE(60, 20) }
      else { KRCA_RING(60) }
      break;
    case 30:
      if (pipe) { KRCA_PIPE(30, 15) }
      else { KRCA_RING(30) }
      break;
    case 20:
      if (pipe) { KRCA_PIPE(20, 10) }
      else { KRCA_RING(20) }
      break;
    case 15:
      if (pipe) { KRCA_PIPE(15, 15) }
      else { KRCA_RING(15) }
      break;
    case 10:
      if (pipe) { KRCA_PIPE(10, 10) }
      else { KRCA_RING(10) }
      break;
    default:
      hipLaunchKernelGGL(rolling_score_reread, grid, block, 0, st, x, S, T, W, M, thr2, z_last, score, n_exceed,
                         flags);
  }
#undef KRCA_PIPE
#undef KRCA_PIPE_AS
#undef KRCA_RING
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

}  // extern "C"

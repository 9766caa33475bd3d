// Cross-pod Pearson correlation with per-row top-k (configs C3/C4).
//
// R = Z·Zᵀ where z[p,t] = (x[p,t] - mean_p) / (std_p * sqrt(T)) (population std over the T
// samples of one metric channel; a flat series gives z = 0).  Per pod: the k partners with the
// largest |R| (self excluded; ties -> lower index) and the number of partners with |R| > tau.
// The full P x P matrix is never materialised.
//
//   krca_corr_prepare  time-major x[T][P][M] -> per-pod mean/scale (one float64 pass, shifted
//                      sums), then an LDS-tiled transpose to pod-major rows: z32[P][T] (fp32,
//                      used for the exact re-scoring) and zh[Pp][Tp] = fp16(z) (zero padded to
//                      256 rows / 64 steps).  |z| <= 1 (unit-norm rows), so fp16 keeps 11 bits.
//   sample pass        every pod against the first NSB*128 pods and against its own 256-pod
//                      block (its likely group): phi[p] = (k-th best sampled |r|) - 2 eps, a lower
//                      bound every member of p's exact top-k clears on the screening product.
//   main pass          MFMA (v_mfma_f32_16x16x32_f16, fp32 accumulation) over the UPPER triangle
//                      of 256x256 tiles only (P(P+1)/2 pairs, the algorithmic flop count), one
//                      512-thread workgroup per tile (8 waves x 128x64), in an XCD-aware
//                      super-tile order, LDS double-buffered.  Epilogue straight from the
//                      accumulators: a value above phi of its row pod (column pod) is appended to
//                      that pod's candidate buffer (one atomic slot reservation per hit; hits are
//                      sparse by construction of phi); |r| > tau counts via LDS, one global add per
//                      row / column and tile.
//   merge              one workgroup per pod: selection of its best k+7 of (<= CAPC) candidates
//                      (per-wave register bitonic sorts of 64 and merges into a running best 32),
//                      the best k+6 re-scored in float64 from z32 (fixed-order wave reduction), final top-k;
//                      cert[p] = (k-th re-scored |r|) - max(phi, first unre-scored |r|) - eps:
//                      cert > 0 proves the reported set equals the exact top-k.  A pod whose buffer
//                      overflowed gets phi2 = (k-th best stored |r|) - 2 eps (any subset bounds the
//                      k-th from below) and a second main pass runs for those pods only.
//   flat pods          (z = 0, detected by a zero self product) correlate 0 with everything:
//                      their top-k is the k lowest other indices, exactly.
//
// Error bound of the screening product (eps, host-computed): fp16 rounding of unit-norm rows
// moves a dot product by <= 2^-10 (+ 2^-24 sqrt(T) from subnormals), fp32 accumulation of T
// terms of a unit-norm product by <= T 2^-24.  It bounds the candidate pool.  |r| > tau counts
// are exact: a screening value above tau + eps counts at once, one within eps of tau is appended
// to the AMBIGUOUS list and re-scored in float64 (corr_amb_rescore; grouped by row pod, from the
// partner's int16 row first and its fp32 row only within the int16 row's error bound of tau), one
// below tau - eps cannot count.  Reported r values are exact.  The sample and main passes run the same K loop, so a
// pair's screening value is the same bits in both.
//
//   deep merge         a pod whose certificate is <= 0 after the merge (near-ties around its k-th
//                      partner) has ALL its candidates re-scored in float64 (corr_merge_deep):
//                      everything outside the buffer is below phi, so the certificate becomes
//                      (k-th exact |r|) - phi - eps > 0.
#include <cmath>
#include <cstdlib>
#include <type_traits>
#include <utility>
#include <vector>

#include "krca_common.h"

namespace {

constexpr int TPB = 256;  // threads of the auxiliary kernels (the tile kernels: Geo<TC>::NTH = 512)
constexpr int BM = 128;   // half of a 256-pod tile: the sample pass's list granularity
constexpr int BK = 64;    // K step (time samples); zh rows are padded to a multiple of it
constexpr int SUPER = 8;  // super-tile edge (tiles) of the XCD-aware order
constexpr int KM = 24;    // candidates re-scored per pod in the merge (>= k + 6)
constexpr int KMAX = 16;  // largest k served
constexpr int NSB = 16;   // 128-pod column blocks in the threshold sample (2048 pods)
constexpr int NSL = NSB + 2;  // sample lists per pod: NSB sample blocks + the pod's own 256-block
#ifndef KRCA_CORR_CAPC_SLOTS
#define KRCA_CORR_CAPC_SLOTS 4096  // (an A/B build can set it: tools/build_variant.sh ... -DKRCA_CORR_CAPC_SLOTS=2048)
#endif
constexpr int CAPC = KRCA_CORR_CAPC_SLOTS;  // candidate buffer per pod (main pass appends; 1024 overflowed ~1 % of
                              // the pods at C3 / 1M, whose rectangle pass cost 1.8 ms / 123 ms, R5k;
                              // 2048 still overflowed at C3: rectangle pass 1.4-1.7 ms on the merge
                              // chain, R7a / R7d; 4096 since R7d: 32 GB of buffer at 1M pods)
// Ambiguous |r| ~ tau pairs (screening value within eps of tau, not settled by the pair's own
// bound) are re-scored in float64 for exact counts.  C3's random-walk series put ~130 partners per
// pod within eps of tau = 0.5 (~170 in EVERY 256 x 256 tile, about half settled in the tile), so the
// pairs scale with P^2: ~6.5M at 100k pods, ~6e8 at 1M.  The main pass therefore runs in batches of
// SB super-tiles, each batch appending to one of two lists of a fixed capacity that the re-score
// drains while the next batch runs; a tile that finds its batch's list full decides its ambiguous
// pairs itself (float64 from z32, in the epilogue), so no valid tau ever fails.
// (knobs KRCA_CORR_BATCH / KRCA_CORR_AMB_TILE, for tests: many batches, lists that fill early)
inline int64_t sb_batch() { return krca::tuning().corr_batch > 0 ? krca::tuning().corr_batch : 8192; }  // R9d/R9e: 1M pods 1.81 -> 1.77 s
inline int64_t amb_per_tile() {  // list budget per tile of a batch (C3 data: ~85 on average)
  return krca::tuning().corr_amb_tile >= 0 ? krca::tuning().corr_amb_tile : 512;
}
constexpr int32_t AMB_BOTH = 1 << 30;  // entry.y flag: credit the partner's count as well
// KC = candidates kept per (pod, sample block) in the sample pass: a template parameter >= k
// (8, 12 or 16), so the k best sampled partners of a pod survive their blocks' cuts

typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // (HIP's uint4 struct defeats SROA)

__device__ __forceinline__ uint16_t f16_bits(float f) {
  const _Float16 h = (_Float16)f;  // round to nearest even
  return __builtin_bit_cast(uint16_t, h);
}

template <int... Is, class F>
__device__ __forceinline__ void static_for_impl(std::integer_sequence<int, Is...>, F&& f) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {  // f(integral_constant<int, k>) for k = 0 .. N-1
  static_for_impl(std::make_integer_sequence<int, N>{}, f);
}

// ---- prepare -------------------------------------------------------------------------------
__global__ __launch_bounds__(TPB) void corr_stats(const float* __restrict__ x, int64_t P, int M, int T, int ch,
                                                  float* __restrict__ mean, float* __restrict__ scale) {
  const int64_t p = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (p >= P) return;
  const int64_t S = P * M;
  const float* xs = x + p * M + ch;
  const double x0 = (double)xs[0];
  double s1 = 0.0, s2 = 0.0;
  for (int t = 0; t < T; ++t) {
    const double d = (double)xs[(int64_t)t * S] - x0;
    s1 += d;
    s2 += d * d;
  }
  const double mu = s1 / T;
  const double var = s2 / T - mu * mu;
  mean[p] = (float)(x0 + mu);
  scale[p] = var > 1e-20 ? (float)(1.0 / sqrt(var * (double)T)) : 0.f;
}

// 64 pods x 64 steps per block: reads of the channel, LDS transpose, pod-major row writes
__global__ __launch_bounds__(TPB) void corr_transpose(const float* __restrict__ x, int64_t P, int M, int T, int Tp,
                                                      int ch, const float* __restrict__ mean,
                                                      const float* __restrict__ scale, float* __restrict__ z32,
                                                      uint16_t* __restrict__ zh) {
  __shared__ float tile[64][65];
  const int64_t p0 = (int64_t)blockIdx.x * 64;
  const int t0 = blockIdx.y * 64;
  const int64_t S = P * M;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t p = p0 + tx;
  const float mu = p < P ? mean[p] : 0.f;
  const float sc = p < P ? scale[p] : 0.f;
  for (int r = ty; r < 64; r += 4) {  // r = time offset
    const int t = t0 + r;
    float v = 0.f;
    if (p < P && t < T) v = (x[(int64_t)t * S + p * M + ch] - mu) * sc;
    tile[tx][r] = v;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {  // r = pod offset
    const int64_t pp = p0 + r;
    const int t = t0 + tx;
    const float z = tile[r][tx];
    zh[pp * Tp + t] = f16_bits(z);  // rows up to Pp (padding rows / steps are zero)
    if (pp < P && t < T) z32[pp * T + t] = z;
  }
}

// ---- tiles -----------------------------------------------------------------------------------
// Sorted candidate list of one row (or column) of a tile.  The scan visits partners in
// ascending index order, so a later partner with an equal |r| never displaces an earlier one:
// "better" is a strict |r| comparison and the index tie rule holds by construction.
template <int KC>
struct Cand {
  float k[KC];    // |r|, -1 = empty (below every |r|, so an empty slot takes any value)
  int32_t c[KC];  // partner << 1 | sign of r, -1 = empty (partner < 2^30)
  float thr;      // k[KC-1]: -1 while the list is not full
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      k[j] = -1.f;
      c[j] = -1;
    }
    thr = -1.f;
  }
  // one compare per slot (h[j] = the new value goes above slot j), then a shift of the slots below
  // the insertion point: 2 selects per slot for the key and the packed partner
  __device__ __forceinline__ void insert(float nv, int32_t ni) {
    const float a = fabsf(nv);
    const int32_t code = (ni << 1) | (int32_t)(__float_as_uint(nv) >> 31);
    bool h[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) h[j] = a > k[j];
#pragma unroll
    for (int j = KC - 1; j > 0; --j) {
      k[j] = h[j - 1] ? k[j - 1] : (h[j] ? a : k[j]);
      c[j] = h[j - 1] ? c[j - 1] : (h[j] ? code : c[j]);
    }
    if (h[0]) {
      k[0] = a;
      c[0] = code;
    }
    thr = k[KC - 1];
  }
  __device__ __forceinline__ float value(int j) const {
    return c[j] < 0 ? 0.f : ((c[j] & 1) ? -k[j] : k[j]);
  }
  __device__ __forceinline__ int32_t partner(int j) const { return c[j] < 0 ? -1 : c[j] >> 1; }
};

// float64 dot product of two fp32 rows by the 16 lanes of a group (sub = lane & 15; float4 loads
// when the rows are 16-B aligned), reduced over the group: every lane gets the sum
__device__ __forceinline__ double dot16_f64(const float* za, const float* zb, int T, int sub) {
  double acc = 0.0;
  if ((T & 3) == 0) {
    const float4* va = reinterpret_cast<const float4*>(za);
    const float4* vb = reinterpret_cast<const float4*>(zb);
    for (int t = sub; t < T / 4; t += 16) {
      const float4 x = va[t], y = vb[t];
      acc += (double)x.x * (double)y.x + (double)x.y * (double)y.y + (double)x.z * (double)y.z +
             (double)x.w * (double)y.w;
    }
  } else {
    for (int t = sub; t < T; t += 16) acc += (double)za[t] * (double)zb[t];
  }
  for (int off = 8; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 16);
  return acc;
}

// dot16_f64 with the row pod's row in LDS and the partner's loads issued eight steps at a time
// (corr_amb_rescore_grouped): per lane the same products added in the same order, so the same bits
__device__ __forceinline__ double dot16_f64_pf(const float* za_lds, const float* zb, int T, int sub) {
  double acc = 0.0;
  if ((T & 3) == 0) {
    const float4* va = reinterpret_cast<const float4*>(za_lds);
    const float4* vb = reinterpret_cast<const float4*>(zb);
    const int n4 = T / 4;
    for (int t0 = sub; t0 < n4; t0 += 16 * 8) {
      float4 y[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int t = t0 + 16 * j;
        y[j] = vb[t < n4 ? t : sub];  // in range: the tail reloads step 0 and adds nothing
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int t = t0 + 16 * j;
        if (t < n4) {
          const float4 x = va[t];
          acc += (double)x.x * (double)y[j].x + (double)x.y * (double)y[j].y + (double)x.z * (double)y[j].z +
                 (double)x.w * (double)y[j].w;
        }
      }
    }
  } else {
    for (int t = sub; t < T; t += 16) acc += (double)za_lds[t] * (double)zb[t];
  }
  for (int off = 8; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 16);
  return acc;
}

// za . zq_b in float64 over 16 lanes (za in LDS, Tq floats, zero past T; zq_b an int16 row of Tq,
// Tq % 8 == 0): 16-byte loads of 8 steps each, every product exact in float64
__device__ __forceinline__ double dot16_q16(const float* za_lds, const int16_t* qb, int Tq, int sub) {
  const float4* va = reinterpret_cast<const float4*>(za_lds);
  const uint4* vb = reinterpret_cast<const uint4*>(qb);
  const int n8 = Tq / 8;
  double acc = 0.0;
  for (int c0 = sub; c0 < n8; c0 += 16 * 4) {
    uint4 y[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = c0 + 16 * j;
      y[j] = vb[c < n8 ? c : sub];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = c0 + 16 * j;
      if (c < n8) {
        const float4 x0 = va[2 * c], x1 = va[2 * c + 1];
        const uint32_t w[4] = {y[j].x, y[j].y, y[j].z, y[j].w};
        const float xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          acc += (double)xs[2 * h] * (double)(int16_t)(w[h] & 0xffffu) +
                 (double)xs[2 * h + 1] * (double)(int16_t)(w[h] >> 16);
        }
      }
    }
  }
  for (int off = 8; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 16);
  return acc;
}

// Tile kernels.  Rows: 256-pod blocks of zA; columns: TC-pod blocks of zh (TC = 256 in every pass):
// 8 waves (2 row halves x 4 column quarters), each a 128 x 64 tile = 8 x 4 MFMA 16x16 blocks, K
// steps of 64 through a double-buffered LDS stage (130 KB with the sample pass's parking area: one
// workgroup per CU) fed by direct global->LDS loads.  (Measured and dropped: 256 x 128 tiles with
// 4 waves and two workgroups per CU hide most of the epilogue but stage 1.5x the bytes per flop;
// their product ran 1.57x slower.)  Every output accumulates its 32-deep K slices in ascending
// order, so a pair's screening value is the same bits in every pass.  Sample-pass lists keep a
// 128-pod block granularity (a row's list covers one 128-column half of a 256-column tile).
constexpr int TB = 256;                  // row block (pods); the unit of the upper-triangle order
constexpr int EPI_LD = TB + 4;           // padded row of the sample pass's parked half tile (16-B rows)
constexpr int EPI_LIST_OFF = 8192;       // main-pass epilogue: per-wave candidate lists start here
template <int TC>
struct Geo {
  static constexpr int NWC = TC / 64;                     // wave columns
  static constexpr int NW = 2 * NWC;                      // waves
  static constexpr int NTH = 64 * NW;                     // threads
  static constexpr int BKS = TC == 256 ? 64 : 32;         // K step (time samples)
  static constexpr int KS = BKS / 16;                     // MFMA slices per K step
  static constexpr int ROWB = BKS * 2;                    // bytes of one staged row (fp16)
  static constexpr int CPR = ROWB / 16;                   // 16-byte chunks per staged row
  static constexpr int RPP = 1024 / ROWB;                 // rows per 1 KiB LDS-DMA piece
  static constexpr int NPA = TB / RPP / NW, NPB = TC / RPP / NW;  // pieces per wave and K step
  static constexpr int STAGE = (TB + TC) * ROWB;          // A and B
  static constexpr int LDS_STAGE = 2 * STAGE;             // double buffered
  static constexpr int LDS_EPI = TC == 256 ? BM * EPI_LD * 4 : 0;  // sample pass: 128 x 256 fp32
  static constexpr int LDS_MAIN = LDS_STAGE > LDS_EPI ? LDS_STAGE : LDS_EPI;
  static constexpr int LDS_BYTES = LDS_MAIN;
  static constexpr int CAPL = (LDS_MAIN - EPI_LIST_OFF) / (NW * 8);  // epilogue list entries per wave
  // persistent main pass (corr_main_persist): the whole 160 KiB, the epilogue's arrays and lists past
  // the two stage buffers, so the next tile's first stage can land while this tile's epilogue runs
  static constexpr int LDS_PERSIST = 160 * 1024;
  static constexpr int CAPL_P = (LDS_PERSIST - LDS_STAGE - EPI_LIST_OFF) / (NW * 8);
  // 16-byte chunk c of staged row r, XOR-swizzled: the 256/ROWB rows of one 256-B bank row sit in
  // distinct granule groups and the key (r / (256/ROWB)) % CPR spreads the rest, so every 16-lane
  // ds_read_b128 phase of 16 rows hits 16 distinct 4-bank granules
  __device__ static __forceinline__ int key(int r) { return (r / (256 / ROWB)) & (CPR - 1); }
  __device__ static __forceinline__ int chunk_off(int r, int c) { return r * ROWB + ((c ^ key(r)) << 4); }
};

// MODE_MAIN:   the upper triangle of 256-blocks (all pairs), in TC-column tiles; hits above phi
//              appended to the per-pod candidate buffers (row and column side), |r| > tau counted.
// MODE_SAMPLE: rows x (the first nsb 128-column blocks, then the row's own 256-block): row lists
//              only (sample slots NSB, NSB+1 = own block), and each pod's self product.
// MODE_RECT:   the gathered rows zA = zh[rect_pods] x every column block (second pass of the pods
//              whose buffer overflowed): row-side appends only, against phi = phi2.
constexpr int MODE_MAIN = 0, MODE_SAMPLE = 1, MODE_RECT = 2;

// Pod-sharded runs: rank g of G takes every G-th super-tile of the upper triangle
// (MAIN), the row blocks [I0, ...) of its own pods (SAMPLE), and appends the candidates of its own
// pods [lo, lo + n_loc) into local buffers indexed g - lo (RECT, merge).  Single device: {0, 1, 0, 0}.
struct Shard {
  int64_t lo;
  int G, g;
  int64_t I0;
  int j0 = 0;        // SAMPLE: first 256-column block of this chunk of the sample
  int own = 0;       // SAMPLE: this chunk also runs each row block's own 256-block
  int nsb2_all = 0;  // SAMPLE: 256-blocks of the whole sample (an own block inside it is skipped)
};

struct TileArgs {
  const uint16_t* zA;  // row operand: zh, or the gathered rows of a rect pass
  const uint16_t* zh;
  int64_t P;
  int Tp, nb2;
  int64_t per_xcd;     // workgroup slots per XCD
  int64_t n_tiles;     // RECT / SAMPLE: tiles of the launch (slots past it exit at once)
  int nsb;
  float tau_hi;   // MAIN: tau + eps, every screening |r| above it is a hit
  float tau_lo;   // MAIN: tau - eps, none at or below it is
  double tau;     // MAIN: the caller's tau, float64 as the exact r it is compared with (the per-pair band in between)
  float acc_err;  // MAIN: the fp32 accumulation terms of eps
  const float* phi;  // MAIN: candidate bound per pod; RECT: phi2
  float* samp_v;
  int32_t* samp_i;
  const float* samp_run;  // SAMPLE, chunks after the first: the running top-k |r| (corr_theta), else null
  int k;
  float* selfd;
  int2* buf;
  int32_t* cnt;
  int capc;  // candidate slots used per pod (<= CAPC, the buffers' row stride; cand_cap())
  int32_t* count;
  const int32_t* rect_pods;
  int64_t n_rect;
  Shard sh;
  int debug;
  int2* amb;                  // MAIN: this batch's ambiguous-pair list
  unsigned long long* amb_n;  // MAIN: its fill (may pass amb_cap: the tiles past it decide in place)
  int64_t amb_cap;
  float* ambv;
  const float* dn;   // MAIN: fp16 rounding-error norm per pod (corr_dnorm)
  const float* z32;  // MAIN: fp32 rows for the in-tile re-score of a full list
  int T;
  int64_t st0, st_end;  // MAIN: this launch's batch [st0, st_end) of the rank's super-tiles
  unsigned* tick;       // MAIN, persistent: one ticket counter per XCD for this batch (zeroed)
};

// Persistent main pass: the state one workgroup carries from tile to tile.
struct PState {
  int b0;        // LDS stage buffer holding this tile's first K stage
  bool staged;   // that stage was loaded by the previous tile's last K step (no prologue wait)
  bool redo;     // a later window of the same tile (rare): product again, no ticket, no next-tile load
  int x;         // this workgroup's XCD (its ticket counter)
  int* tk_next;  // LDS words {I, J} of the next tile, written by thread 0 during this tile's K loop
};
constexpr int TK_OFF = 8176;  // ticket words in the epilogue area (past the epilogue's arrays)

// slot L2 of the main pass's XCD-aware order -> tile (I, J); false for slots below the diagonal or
// past this batch / the triangle.  Workgroups are dispatched round-robin over the 8 XCDs, so slot
// L2 = (b % 8) * per_xcd + b / 8 gives each XCD a contiguous run of slots; consecutive slots walk
// the upper triangle in SUPER x SUPER super-tiles, so the tiles an XCD has in flight share 2*SUPER
// row blocks through its L2.
__device__ __forceinline__ bool main_slot(const TileArgs& A, int64_t L, int64_t& I, int64_t& J) {
  const int64_t ns = (A.nb2 + SUPER - 1) / SUPER;
  const int64_t sl = A.st0 + L / (SUPER * SUPER);  // this batch's share of the rank's super-tiles
  if (sl >= A.st_end) return false;
  const int64_t st = sl * A.sh.G + A.sh.g;
  if (st >= ns * (ns + 1) / 2) return false;
  int64_t SJ = (int64_t)((sqrt(8.0 * (double)st + 1.0) - 1.0) * 0.5);
  while ((SJ + 1) * (SJ + 2) / 2 <= st) ++SJ;
  while (SJ * (SJ + 1) / 2 > st) --SJ;
  const int64_t SI = st - SJ * (SJ + 1) / 2;
  const int64_t in = L % (SUPER * SUPER);
  I = SI * SUPER + in / SUPER;
  J = SJ * SUPER + in % SUPER;
  return I <= J && J < A.nb2;
}

// thread 0 of a persistent workgroup: ticket t of XCD x (and more tickets past invalid slots) -> the
// next tile, or I = -1 when the XCD's run is used up
__device__ __forceinline__ void take_tile(const TileArgs& A, int x, unsigned t, int* out) {
  int64_t I = -1, J = -1;
  for (;;) {
    if ((int64_t)t >= A.per_xcd) {
      I = -1;
      break;
    }
    if (main_slot(A, (int64_t)x * A.per_xcd + t, I, J)) break;
    t = atomicAdd(&A.tick[x], 1u);
  }
  if (I >= 0 && A.debug == 4) I = J = x;  // profiling aid: product only, operands L2-resident
  out[0] = (int)I;
  out[1] = (int)J;
}

// One tile: row block I (256 pods), column block J (TC pods).  Main / rect passes: the epilogue takes
// the flagged values of list slots [win, win + CAPL) of each wave; returns whether some wave has
// more (rare: the caller runs the tile again for the next window; the counts of |r| > tau + eps are
// taken in window 0 only).
// PERSIST (main pass only, corr_main_persist): the first K stage may already be in LDS buffer
// ps->b0; the last K step loads the NEXT tile's first stage (ps->tk_next) into the idle buffer; the
// epilogue works past the stage buffers and runs every window itself (the accumulators stay live).
template <int KC, int MODE, int TC, bool PERSIST = false>
__device__ __forceinline__ bool tile_body(const TileArgs& A, const int64_t I, const int64_t J, const bool own,
                                          const int win, const PState* ps = nullptr) {
  static_assert(!PERSIST || (MODE == MODE_MAIN && TC == 256), "persistent: main pass, 256-column tiles");
  using G = Geo<TC>;
  constexpr bool SAMPLE = MODE == MODE_SAMPLE;
  static_assert(!SAMPLE || TC == 256, "the sample pass parks 256-column tiles");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int64_t P = A.P;
  const int Tp = A.Tp;
  const Shard& sh = A.sh;
  const int debug = A.debug;
  // persistent: the thread index made opaque per tile, so that nothing derived from it (epilogue
  // addresses, list codes) is hoisted out of the tile loop and kept live across it (spills)
  int tid_ = threadIdx.x;
  if constexpr (PERSIST) asm volatile("" : "+v"(tid_));
  const int tid = tid_, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w / G::NWC, wc = w % G::NWC;
  const int64_t rowA = I * TB, rowB = J * TC;
  // main / rect epilogue operands, loaded now so their latency hides behind the K loop: thread rq
  // (< 256) holds row pod rq of the tile, its phi and rounding-error norm; thread cq (in [0, TC))
  // column pod cq
  const int rq = tid;
  const int cq = G::NTH == 2 * TB ? tid - TB : tid;
  int r_pod = -1;
  float r_phi = 4.f, c_phi = 4.f;  // 4 = never a candidate owner (padding, or column side of a rect pass)
  float r_dn = 0.f, c_dn = 0.f;
  if (!SAMPLE) {
    if (rq < TB) {
      const int64_t g = MODE == MODE_RECT ? (rowA + rq < A.n_rect ? A.rect_pods[rowA + rq] : -1) : (rowA + rq < P ? rowA + rq : -1);
      r_pod = (int)g;
      if (g >= 0) {
        r_phi = A.phi[g];
        if (MODE == MODE_MAIN) r_dn = A.dn[g];
      }
    }
    if (MODE == MODE_MAIN && cq >= 0 && cq < TC && rowB + cq < P) {
      c_phi = A.phi[rowB + cq];
      c_dn = A.dn[rowB + cq];
    }
  }

  // 16x16x32 MFMA blocks: acc[i][j][e] = row wr*128 + i*16 + 4*(lane >> 4) + e, column
  // wc*64 + j*16 + (lane & 15) of the tile.  (The 32x32x16 form ran the same MACs in the same
  // cycles, 7-9 % slower in wall time: the chip holds a lower clock on it, MI355X_MICROARCH.md
  // 'DVFS give-back' item 7.)
  static_assert(G::BKS == 64, "the K loop runs two 32-deep sub-steps per stage");
  floatx4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[i][j][e] = 0.f;

  // Staging: global -> LDS direct (global_load_lds_dwordx4, no VGPR round trip).  One wave
  // instruction writes a lane-linear 1 KiB piece = RPP rows; lane l lands on row l / CPR, slot
  // l % CPR, so it fetches the global chunk (l % CPR) ^ key(row): the XOR swizzle is applied on the
  // SOURCE address.
  const uint16_t* gA = A.zA + rowA * Tp;
  const uint16_t* gB = A.zh + rowB * Tp;
  const int prow = lane / G::CPR, pslot = lane % G::CPR;
  auto glds_a = [&](int buf, const uint16_t* src, int k0) {
    char* sbase = smem + buf * G::STAGE;
#pragma unroll
    for (int q = 0; q < G::NPA; ++q) {
      const int piece = w + G::NW * q;
      const int row = G::RPP * piece + prow;
      __builtin_amdgcn_global_load_lds(src + (int64_t)row * Tp + k0 + ((pslot ^ G::key(row)) << 3),
                                       (__attribute__((address_space(3))) void*)(sbase + piece * 1024), 16, 0, 0);
    }
  };
  auto glds_b = [&](int buf, const uint16_t* src, int k0) {
    char* sbase = smem + buf * G::STAGE;
#pragma unroll
    for (int q = 0; q < G::NPB; ++q) {
      const int piece = w + G::NW * q;
      const int row = G::RPP * piece + prow;
      __builtin_amdgcn_global_load_lds(src + (int64_t)row * Tp + k0 + ((pslot ^ G::key(row)) << 3),
                                       (__attribute__((address_space(3))) void*)(sbase + TB * G::ROWB + piece * 1024),
                                       16, 0, 0);
    }
  };
  auto glds = [&](int buf, int k0) {
    glds_a(buf, gA, k0);
    glds_b(buf, gB, k0);
  };
  const int r16 = lane & 15, g4 = lane >> 4;
  // Fragments (16x16x32: lane l holds A[row l & 15][k = 8 (l >> 4) .. + 7] of a 16-row block, B the
  // same of a 16-column block): A row blocks 0-3 (alo) and 4-7 (ahi), B in two sets (one per
  // 32-deep sub-step).  Each phase runs 16 MFMAs with the reads of the next phase's operands pinned
  // between them, so no MFMA waits on a just-issued LDS read.
  halfx8 alo[4], ahi[4], bfr[2][4];
  auto chunk = [&](int kk) { return 4 * kk + g4; };
  auto ld_alo = [&](int buf, int kk) {
    const char* sA = smem + buf * G::STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      alo[i] = *reinterpret_cast<const halfx8*>(sA + G::chunk_off(wr * 128 + i * 16 + r16, chunk(kk)));
  };
  auto ld_ahi = [&](int buf, int kk) {
    const char* sA = smem + buf * G::STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      ahi[i] = *reinterpret_cast<const halfx8*>(sA + G::chunk_off(wr * 128 + (i + 4) * 16 + r16, chunk(kk)));
  };
  auto ld_b = [&](int set, int buf, int kk) {
    const char* sB = smem + buf * G::STAGE + TB * G::ROWB;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bfr[set][j] = *reinterpret_cast<const halfx8*>(sB + G::chunk_off(wc * 64 + j * 16 + r16, chunk(kk)));
  };
  auto mm_lo = [&](int set) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo[i], bfr[set][j], acc[i][j], 0, 0, 0);
  };
  auto mm_hi = [&](int set) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i + 4][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[i], bfr[set][j], acc[i + 4][j], 0, 0, 0);
  };
  const int nk = Tp / G::BKS;
  const int b0 = PERSIST ? ps->b0 : 0;
  if (!PERSIST || !ps->staged) {
    glds(b0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // persistent: thread 0 takes the next tile's ticket now and resolves it at step 1 (the atomic's
  // return lands under step 0); every wave reads the tile at the last step, after the barriers
  unsigned traw = 0;
  if constexpr (PERSIST) {
    if (!ps->redo && tid == 0) {
      traw = atomicAdd(&A.tick[ps->x], 1u);
      if (nk < 3) take_tile(A, ps->x, traw, ps->tk_next);
    }
    if (!ps->redo && nk < 3) __syncthreads();
  }
  ld_alo(b0, 0);
  ld_b(0, b0, 0);
  // Per stage (64 deep = sub-steps 0 and 1): A(0) alo x b0 while reading ahi(0); B(0) ahi x b0 while
  // reading alo(1), b1; A(1) alo x b1 while reading ahi(1); barrier; B(1) ahi x b1 while reading
  // alo(0), b0 of the next stage.
#define CORR_PIN(NM, ND)                                                                 \
  _Pragma("unroll") for (int q = 0; q < 16 / (NM); ++q) {                                 \
    __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);                                   \
    __builtin_amdgcn_sched_group_barrier(0x100, ND, 0);                                   \
  }                                                                                       \
  __builtin_amdgcn_sched_barrier(0);
  for (int s = 0; s < nk; ++s) {
    const int buf = (s & 1) ^ b0;
    // stage buf ^ 1 was last read in step s-1; every wave retired those reads (lgkmcnt(0)) before
    // the barrier that ended it.  The next stage's A pieces go out before the first MFMA phase, its
    // B pieces after it: issued together (or in three groups) they ran 4 % (2 %) slower.  The last
    // step re-loads its own stage into the idle buffer (never read), so the loop has no branch --
    // or, persistent, the next tile's first stage.
    // (An L2 prefetch of step s + 2 by 4-byte LDS-DMA loads, one per 128-B line, ran 7 % slower in
    // the 16x16x32 form: its issue slots and a lower clock cost more than the latency it hid;
    // without any staging in the loop the product ran 9.3 vs 12.8 ms, clock 1.97 vs 1.74 GHz.)
    int kn = (s + 1 < nk ? s + 1 : s) * G::BKS;
    const uint16_t* sa = gA;
    const uint16_t* sb = gB;
    if constexpr (PERSIST) {
      if (s == 1 && nk >= 3 && tid == 0 && !ps->redo) take_tile(A, ps->x, traw, ps->tk_next);
      if (s == nk - 1 && !ps->redo) {
        const int nI = ps->tk_next[0], nJ = ps->tk_next[1];
        if (nI >= 0) {
          sa = A.zA + (int64_t)nI * TB * Tp;
          sb = A.zh + (int64_t)nJ * TC * Tp;
          kn = 0;
        }
      }
    }
    glds_a(buf ^ 1, sa, kn);
    __builtin_amdgcn_sched_barrier(0);
    ld_ahi(buf, 0);
    mm_lo(0);
    CORR_PIN(4, 1)
    glds_b(buf ^ 1, sb, kn);
    __builtin_amdgcn_sched_barrier(0);
    ld_alo(buf, 1);
    ld_b(1, buf, 1);
    mm_hi(0);
    CORR_PIN(2, 1)
    ld_ahi(buf, 1);
    mm_lo(1);
    CORR_PIN(4, 1)
    // stage buf ^ 1 has landed for this wave and this
    // wave's reads of stage buf are retired; after the barrier, for every wave.  The last step
    // reads stage buf ^ 1 as well (stale bytes, never used): no branch in the loop.
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    ld_alo(buf ^ 1, 0);
    ld_b(0, buf ^ 1, 0);
    mm_hi(1);
    CORR_PIN(2, 1)
  }
#undef CORR_PIN
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // a diagonal 256-block: its tiles hold both orders of every pair (across the TC-column tiles of
  // the block), so counts and candidates go to the row side only
  const bool diag = MODE != MODE_RECT && rowB / TB == I;
  if (debug == 1 || debug == 4) {  // profiling aid (KRCA_CORR_DEBUG=1 / 4): product only, no epilogue
    if (tid == 0 && acc[0][0][0] == 12345.f) A.count[0] = 1;
    return false;
  }
  if constexpr (!SAMPLE) {
    // ---- main / rect epilogue, straight from the accumulators ---------------------------
    // lane holds rows wr*128 + i*16 + 4*(lane >> 4) + e and columns wc*64 + j*16 + (lane & 15).
    // Padding rows / columns have z = 0 (r = 0: never above tau >= 0) and phi = 4 (never a
    // candidate); the self products of a diagonal tile are zeroed first.
    //   1. per wave, branch-free over a lane's 128 values: |r| > tau + eps counted (a lane's own hit
    //      bits added per row e into byte e of a packed counter, summed over the 16 lanes of its row
    //      group per row block i; column counts per lane), and each
    //      value that may need anything (above phi of its row or column pod, or within eps of tau)
    //      appended RAW to the wave's LDS list {row | col << 8, r bits} (ballot + mbcnt, only when
    //      some lane has one: they are sparse)
    //   2. every thread takes list entries: classified (candidate of the row / column pod; within eps
    //      of tau: settled by the pair's own rounding-error bound, or ambiguous), settled pairs
    //      counted in LDS, ambiguous pairs ranked in the tile (one LDS atomic per wave and round)
    //   3. counts committed (one global add per row / column), ONE global atomic reserves the tile's
    //      range of the ambiguous-pair list, then the entries are written out (ambiguous list,
    //      candidate buffers)
    constexpr bool RECT = MODE == MODE_RECT;
    constexpr bool HITS = MODE == MODE_MAIN;    // |r| > tau + eps counted in step 1 (first window)
    constexpr bool SETTLE = MODE == MODE_MAIN;  // pairs settled by their bound counted in step 2
    constexpr int CAPL = PERSIST ? G::CAPL_P : G::CAPL;
    // an entry after classification: row | col << 8 | candidate bits << 16 | (ambiguous rank + 1) << 18
    static_assert(G::NW * CAPL < (1 << 14) - 1, "ambiguous ranks of a window fit 14 bits");
    char* const ebase = smem + (PERSIST ? G::LDS_STAGE : 0);  // persistent: past the stage buffers
    float* sphr = reinterpret_cast<float*>(ebase);  // phi of the 256 row pods
    float* sphc = sphr + TB;                        // phi of the TC column pods
    int* srcnt = reinterpret_cast<int*>(sphc + TC);  // |r| > tau counts per row / column
    int* sccnt = srcnt + TB;
    int* spod = sccnt + TC;    // row pod ids
    float* sdnr = reinterpret_cast<float*>(spod + TB);  // rounding-error norms of the rows / columns
    float* sdnc = sdnr + TB;
    int* wcount = reinterpret_cast<int*>(sdnc + TC);  // list length per wave
    int* sflag = wcount + G::NW;  // [0] a list passed its window, [1] ranked ambiguous pairs
    long long* sbase = reinterpret_cast<long long*>(sflag + 4);  // their base in the list (slots past amb_cap: decided here)
    int2* lists = reinterpret_cast<int2*>(ebase + EPI_LIST_OFF);
    static_assert(7 * 1024 + 64 <= TK_OFF && TK_OFF + 16 <= EPI_LIST_OFF, "epilogue arrays, ticket words, lists");
    if (diag) {
      const int doff = (int)(rowB - rowA);  // global row == global column <=> row - col == doff
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (wr * 128 + i * 16 + 4 * g4 + e == wc * 64 + j * 16 + r16 + doff) acc[i][j][e] = 0.f;
    }
    // one window of the lists (slots [win, win + CAPL) of each wave); returns whether one follows
    auto epi = [&](const int win) -> bool {
    {
      if (rq < TB) {
        sphr[rq] = r_phi;
        srcnt[rq] = 0;
        sdnr[rq] = r_dn;
        spod[rq] = r_pod;
      }
      if (cq >= 0 && cq < TC) {
        sphc[cq] = c_phi;
        sccnt[cq] = 0;
        sdnc[cq] = c_dn;
      }
      if (tid == 0) {
        sflag[0] = 0;
        sflag[1] = 0;
      }
    }
    __syncthreads();
    // classification of one flagged value: bit 0 candidate of the row pod, bit 1 of the column pod
    // (never in a diagonal tile: both orders are present), bit 2 ambiguous, bit 3 settled above tau
    auto classify = [&](int row, int col, float v) -> int {
      const float a = fabsf(v);
      const int gr = RECT ? spod[row] : (int)(rowA + row);
      const int gc = (int)(rowB + col);
      const bool pair = gc < P && gc != gr;  // padding partners / zeroed self: r = 0
      int tag = (a > sphr[row] && pair) ? 1 : 0;
      if (!RECT && !diag && a > sphc[col] && rowA + row < P) tag |= 2;
      if (!RECT && a > A.tau_lo && a <= A.tau_hi && pair && rowA + row < P) {
        // within eps of tau: the pair's own bound from the rows' rounding-error norms (corr_dnorm)
        // often settles it; otherwise it is listed for float64 re-scoring
        const double dr = (double)sdnr[row], dc = (double)sdnc[col];
        const double band = dr + dc + 3.0 * dr * dc + (double)A.acc_err + 1e-9;
        if ((double)a > (double)A.tau + band) {
          tag |= 8;
        } else if ((double)a > (double)A.tau - band) {
          tag |= 4;
        }
      }
      return tag;
    };
    // ---- 1. counts and raw lists (this window's CAPL slots per wave) --------------------------
    int2* wlist = lists + w * CAPL;
    const float tau_hi = A.tau_hi, tau_lo = A.tau_lo;
    {
      int nlist = 0;  // wave-uniform
      int colcnt[4] = {0, 0, 0, 0};
      const bool hits = HITS && win == 0;
      // the lane's 32 row bounds and 4 column bounds, read once (one LDS wait, not one per block)
      float4 prall[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) prall[i] = *reinterpret_cast<const float4*>(sphr + wr * 128 + i * 16 + 4 * g4);
      float pc[4];  // diagonal tile: both orders present, candidates on the row side only
#pragma unroll
      for (int j = 0; j < 4; ++j) pc[j] = diag ? 4.f : sphc[wc * 64 + j * 16 + r16];
      static_for<8>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const float pr[4] = {prall[i].x, prall[i].y, prall[i].z, prall[i].w};
        int rh[4] = {0, 0, 0, 0};  // this lane's hits in row e of block i (over its 4 columns)
        static_for<4>([&](auto ec) {
          constexpr int e = decltype(ec)::value;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float v = acc[i][j][e];
            const float a = fabsf(v);
            // the masks straight from the compares (no boolean round trip through a VGPR)
            const uint64_t mh = __builtin_amdgcn_ballot_w64(a > tau_hi);
            if (hits) {  // += own hit bit (v_addc on the mask), row and column counters
              int cr = rh[e], cc = colcnt[j];
              uint64_t co;
              asm volatile("v_addc_co_u32_e64 %0, %1, 0, %0, %2" : "+v"(cr), "=s"(co) : "s"(mh));
              asm volatile("v_addc_co_u32_e64 %0, %1, 0, %0, %2" : "+v"(cc), "=s"(co) : "s"(mh));
              rh[e] = cr;
              colcnt[j] = cc;
            }
            uint64_t fm = __builtin_amdgcn_ballot_w64(a > pr[e]) | __builtin_amdgcn_ballot_w64(a > pc[j]);
            if (!RECT) fm |= __builtin_amdgcn_ballot_w64(a > tau_lo) & ~mh;
            if (fm) {  // wave-uniform, rare
              const int slot = nlist - win + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32),
                                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u));
              if (((fm >> lane) & 1) && slot >= 0 && slot < CAPL) {
                const int row = wr * 128 + i * 16 + 4 * g4 + e;
                const int col = wc * 64 + j * 16 + r16;
                wlist[slot] = make_int2(row | (col << 8), __float_as_int(v));
              }
              nlist += __builtin_popcountll(fm);
            }
          }
        });
        if (hits) {  // rows of block i: packed (byte e <= 64), summed over the 16 lanes of the row group
          int pk = rh[0] | (rh[1] << 8) | (rh[2] << 16) | (rh[3] << 24);
#pragma unroll
          for (int d = 1; d < 16; d <<= 1) pk += __shfl_xor(pk, d, 16);
          const int c = (pk >> (8 * (r16 & 3))) & 0xFF;
          if (r16 < 4 && c) atomicAdd(&srcnt[wr * 128 + i * 16 + 4 * g4 + r16], c);
        }
      });
      if (debug == 6) {  // profiling aid: step 1 only
        if (nlist == 12345) A.count[0] = colcnt[0] + colcnt[1] + colcnt[2] + colcnt[3];
        return false;
      }
      if (lane == 0) {
        wcount[w] = min(max(nlist - win, 0), CAPL);
        if (nlist > win + CAPL) sflag[0] = 1;  // another window follows
      }
      if (hits && !diag) {  // |r| > tau, columns: summed over the 4 row groups, one LDS add per column
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          int c = colcnt[j] + __shfl_xor(colcnt[j], 16, 64);
          c += __shfl_xor(c, 32, 64);
          if (g4 == 0 && c) atomicAdd(&sccnt[wc * 64 + j * 16 + r16], c);
        }
      }
      __syncthreads();
      // the waves' lists as one sequence: entry q of wave u is at lists[u * CAPL + q - off(u)]
      int woff[G::NW + 1];
      woff[0] = 0;
#pragma unroll
      for (int u = 0; u < G::NW; ++u) woff[u + 1] = woff[u] + wcount[u];
      const int ntot = woff[G::NW];
      auto entry_at = [&](int q) -> int2* {
        int u = 0;
#pragma unroll
        for (int k = 1; k < G::NW; ++k) u += q >= woff[k] ? 1 : 0;
        return lists + u * CAPL + (q - woff[u]);
      };
      const bool more = sflag[0] != 0;
      // ---- 2. classification -----------------------------------------------------------------
      for (int q = tid; q < ntot; q += G::NTH) {
        int2* ep = entry_at(q);
        const int2 ent = *ep;
        const int row = ent.x & 255, col = (ent.x >> 8) & 255;
        const float v = __int_as_float(ent.y);
        int tag = classify(row, col, v);
        if (SETTLE && (tag & 8)) {
          atomicAdd(&srcnt[row], 1);
          if (!diag) atomicAdd(&sccnt[col], 1);
        }
        int rank = 0;
        const uint64_t mam = __ballot((tag & 4) != 0);
        if (mam) {
          const int leader = __builtin_ctzll(mam);
          int base = 0;
          if (lane == leader) base = atomicAdd(&sflag[1], __builtin_popcountll(mam));
          base = __shfl(base, leader, 64);
          rank = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mam >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mam, 0u));
        }
        *ep = make_int2((int)(((uint32_t)ent.x & 0xffffu) | ((uint32_t)(tag & 3) << 16) |
                              ((tag & 4) ? (uint32_t)(rank + 1) << 18 : 0u)),
                        ent.y);
      }
      __syncthreads();
      // ---- 3. counts, the window's ambiguous range, entries out --------------------------------
      if (SETTLE) {  // one global add per row / column of the tile
        if (rq < TB && srcnt[rq]) atomicAdd(&A.count[rowA + rq], srcnt[rq]);
        if (!diag && cq >= 0 && cq < TC && sccnt[cq]) atomicAdd(&A.count[rowB + cq], sccnt[cq]);
      }
      // the ambiguous range's reservation, the candidates' slot reservations and the count adds are
      // all in flight together (the range first, then the candidates: 0.5 % slower main pass)
      long long abase_t = -1;
      const int atot = RECT ? 0 : sflag[1];
      if (!RECT && tid == 0 && atot) abase_t = (long long)atomicAdd(A.amb_n, (unsigned long long)atot);
      if (debug == 5) return false;
      for (int q = tid; q < ntot; q += G::NTH) {
        const int2 ent = *entry_at(q);
        const int row = ent.x & 255, col = (ent.x >> 8) & 255, tag = (ent.x >> 16) & 3;
        const int gr = RECT ? spod[row] : (int)(rowA + row);
        const int gc = (int)(rowB + col);
        const int64_t lr = RECT ? gr - sh.lo : gr;  // rect: local buffers
        const int s1 = (tag & 1) ? atomicAdd(&A.cnt[lr], 1) : CAPC;
        const int s2 = (!RECT && (tag & 2)) ? atomicAdd(&A.cnt[gc], 1) : CAPC;
        if (s1 < A.capc) A.buf[lr * CAPC + s1] = make_int2(ent.y, gc);
        if (s2 < A.capc) A.buf[(int64_t)gc * CAPC + s2] = make_int2(ent.y, gr);
      }
      if (!RECT && atot) {  // block-uniform
        if (tid == 0) *sbase = abase_t;
        __syncthreads();
        // the list slots [abase, abase + atot) were reserved; those below amb_cap are written (the
        // re-score kernel reads min(fill, amb_cap) entries, so every one of them must be), the rest
        // -- a tile straddling the cap, or past it -- are decided here
        const long long room = A.amb_cap - *sbase;  // entries of this tile that fit (may be <= 0)
        if (room > 0) {
          for (int q = tid; q < ntot; q += G::NTH) {
            const int2 ent = *entry_at(q);
            const uint32_t rk = (uint32_t)ent.x >> 18;
            if (rk && (long long)rk <= room) {
              const long long slot = *sbase + rk - 1;
              A.amb[slot] = make_int2((int)(rowA + (ent.x & 255)), (int)(rowB + ((ent.x >> 8) & 255)) | (diag ? 0 : AMB_BOTH));
              A.ambv[slot] = __int_as_float(ent.y);
            }
          }
        }
        if (room < atot) {
          // the batch's list is full (a tau inside the bulk of |r|): this tile's ambiguous pairs past
          // it are decided here, 16 lanes per pair, float64 from the two fp32 rows
          // (corr_amb_rescore's arithmetic)
          const int sub = tid & 15;
          for (int q0 = 0; q0 < ntot; q0 += G::NTH / 16) {
            const int q = q0 + (tid >> 4);
            const int2 ent = q < ntot ? *entry_at(q) : make_int2(0, 0);
            const uint32_t rk = (uint32_t)ent.x >> 18;
            if (q < ntot && rk != 0 && (long long)rk > room) {  // uniform over the 16-lane group
              const int64_t a = rowA + (ent.x & 255), b = rowB + ((ent.x >> 8) & 255);
              const double acc = dot16_f64(A.z32 + a * A.T, A.z32 + b * A.T, A.T, sub);
              if (sub == 0 && fabs(acc) > (double)A.tau) {
                atomicAdd(&A.count[a], 1);
                if (!diag) atomicAdd(&A.count[b], 1);
              }
            }
          }
        }
      }
      return more;
    }
    };
    return epi(win);
  } else {
    // ---- sample pass: park each 128-row half in LDS, two lanes per (row, 128-column half) -------
    float* tile = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if (wr == half) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int row = i * 16 + 4 * g4 + e;
              const int col = wc * 64 + j * 16 + r16;
              tile[row * EPI_LD + col] = acc[i][j][e];
            }
      }
      __syncthreads();
      // row scan: pod rowA + half*128 + r against the 128 columns of block 2J + ch, two threads per
      // row and block (part 0: columns 0-63, part 1: 64-127; the lanes of a wave scan different
      // rows, so the insert network runs at every column where any lane inserts: halving the
      // columns per thread halves that).  Part 1 leaves its sorted list in its own (scanned) columns
      // of the parked row; part 0 inserts it after its own: part 1's columns are all higher, so the
      // index tie rule of the ascending scan still holds and the list equals a single scan's.
      const int r = tid & 127, ch = (tid >> 7) & 1, part = tid >> 8;
      const int64_t g = rowA + half * BM + r;
      const int jb = 2 * (int)(J - sh.j0) + ch;  // list slot of this chunk
      const int64_t c0 = rowB + ch * BM;
      const bool active = g < P && (own || jb < A.nsb);
      float* rowp = tile + r * EPI_LD + ch * BM;
      Cand<KC> cd;
      cd.init();
      // the self product, also from a 128-block the sample does not scan: with an odd sample size
      // the last sampled 256-block's second half is not scanned and, being a sample block, it is
      // nobody's own block either, so its pods' self products were never recorded (and a stale
      // value below 0.25 made a live pod "flat": its top-k the lowest indices)
      const int self = (g < P && g >= c0 && g < c0 + BM) ? (int)(g - c0) : -1;
      if (self >= 0 && (self >= BM / 2) == (part == 1)) A.selfd[g] = rowp[self];  // before part 1's list lands
      // a later chunk of the sample: only values above the running k-th best of the chunks before
      // can change the k-th best of the whole sample (corr_theta keeps the running values), so the
      // lists start at that floor and the scan skips everything below it with one compare
      const float floor_ = (active && A.samp_run) ? A.samp_run[g * KMAX + A.k - 1] : -1.f;
      if (active) {
        const int cend = (int)std::min<int64_t>(BM, P - c0);
        float lim = floor_;
        const int cb = part * (BM / 2), ce = std::min(cend, cb + BM / 2);
        for (int c4 = cb; c4 < ce; c4 += 4) {
          const float4 q4 = *reinterpret_cast<const float4*>(rowp + c4);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int c = c4 + u;
            const float vu = u == 0 ? q4.x : u == 1 ? q4.y : u == 2 ? q4.z : q4.w;
            if (c < ce && c != self && fabsf(vu) > lim) {
              cd.insert(vu, (int32_t)(c0 + c));
              lim = fmaxf(cd.thr, floor_);
            }
          }
        }
        if (part == 1) {
#pragma unroll
          for (int q = 0; q < KC; ++q) {
            rowp[BM / 2 + 2 * q] = cd.value(q);
            rowp[BM / 2 + 2 * q + 1] = __int_as_float(cd.partner(q));
          }
        }
      }
      static_assert(2 * KC <= BM / 2, "part 1's list fits in its columns");
      __syncthreads();
      if (active && part == 0) {
        float lim = fmaxf(cd.thr, floor_);
#pragma unroll
        for (int q = 0; q < KC; ++q) {
          const float vu = rowp[BM / 2 + 2 * q];
          const int32_t iq = __float_as_int(rowp[BM / 2 + 2 * q + 1]);
          if (iq >= 0 && fabsf(vu) > lim) {
            cd.insert(vu, iq);
            lim = fmaxf(cd.thr, floor_);
          }
        }
        const int64_t slot = g * NSL + (own ? NSB + ch : jb);
        // 16-byte stores (a list is KC * 4 bytes at a multiple of 16): a lane's dword stores to its
        // own list went to 64 lines per wave instruction, KC of them per array
        static_assert(KC % 4 == 0, "lists are whole 16-byte pieces");
        float4* ov = reinterpret_cast<float4*>(A.samp_v + slot * KC);
        int4* oi = reinterpret_cast<int4*>(A.samp_i + slot * KC);
#pragma unroll
        for (int q = 0; q < KC / 4; ++q) {
          ov[q] = make_float4(cd.value(4 * q), cd.value(4 * q + 1), cd.value(4 * q + 2), cd.value(4 * q + 3));
          oi[q] = make_int4(cd.partner(4 * q), cd.partner(4 * q + 1), cd.partner(4 * q + 2), cd.partner(4 * q + 3));
        }
      }
      __syncthreads();  // the next half overwrites the tile
    }
    return false;
  }
}

// TC: the main pass's column-tile width (256 for the other modes).  Two workgroups
// per CU for TC = 128 (<= 256 registers per lane).
template <int KC, int MODE, int TC>
__global__ __launch_bounds__(Geo<TC>::NTH) __attribute__((amdgpu_waves_per_eu(2))) void corr_tiles(TileArgs A) {
  // RECT / SAMPLE: XCD-aware slots as in the main pass (L = (b % 8) * per_xcd + b / 8, each XCD a
  // contiguous run), ordered so that the tiles sharing the operand fetched from beyond L2 run on one
  // XCD together: rect, column-block-major (the gathered row blocks are few and stay cached); sample,
  // row-block-major (the sample column blocks are shared by every tile).  Row-major over blockIdx
  // spread each such panel over all 8 XCDs' L2s.
  const int64_t L = (int64_t)(blockIdx.x & 7) * A.per_xcd + (blockIdx.x >> 3);
  if constexpr (MODE == MODE_RECT) {
    if (L >= A.n_tiles) return;
    const int64_t nri = A.n_tiles / A.nb2;  // gathered row blocks of this launch
    const int64_t I = L % nri, J = L / nri;
    if (tile_body<KC, MODE_RECT, TC>(A, I, J, false, 0)) {  // window 0 outside the loop (as MODE_MAIN)
      for (int win = Geo<TC>::CAPL;; win += Geo<TC>::CAPL) {
        __syncthreads();  // the next window reuses the LDS
        if (!tile_body<KC, MODE_RECT, TC>(A, I, J, false, win)) break;
      }
    }
  } else if constexpr (MODE == MODE_SAMPLE) {
    if (L >= A.n_tiles) return;
    const int nsb2 = (A.nsb + 1) / 2;  // this chunk's 256-blocks
    const int64_t I = A.sh.I0 + L / (nsb2 + 1);
    int64_t J = L % (nsb2 + 1);
    bool own = false;
    if (J == nsb2) {  // the row block's own 256-block, unless it is already a sample block
      if (!A.sh.own || I < A.sh.nsb2_all) return;
      J = I;
      own = true;
    } else {
      J += A.sh.j0;
    }
    tile_body<KC, MODE_SAMPLE, TC>(A, I, J, own, 0);
  } else {  // MODE_MAIN
    // XCD-aware order: workgroups are dispatched round-robin over the 8 XCDs, so slot
    // L = (b % 8) * per_xcd + b / 8 gives each XCD a contiguous run of slots; SPLIT consecutive
    // slots are the column tiles of one 256 x 256 block pair, and the pairs walk the upper triangle
    // in SUPER x SUPER super-tiles, so the tiles an XCD has in flight share 2*SUPER row blocks
    // through its L2.  Slots below the diagonal or past nb2 exit at once.
    constexpr int SPLIT = TB / TC;
    const int64_t b = blockIdx.x;
    const int64_t L2 = (b & 7) * A.per_xcd + (b >> 3);
    const int64_t L = L2 / SPLIT;
    const int part = (int)(L2 % SPLIT);
    int64_t I, J;
    if (!main_slot(A, L, I, J)) return;
    if (A.debug == 4) I = J = (blockIdx.x & 7);  // profiling aid: product only, operands L2-resident
    // window 0 outside the loop: the loop's copy may hold more registers (values kept across its
    // iterations); it runs only for a tile whose lists pass CAPL entries in some wave
    if (tile_body<KC, MODE_MAIN, TC>(A, I, J * SPLIT + part, false, 0)) {
      for (int win = Geo<TC>::CAPL;; win += Geo<TC>::CAPL) {
        __syncthreads();  // the next window reuses the LDS
        if (!tile_body<KC, MODE_MAIN, TC>(A, I, J * SPLIT + part, false, win)) break;
      }
    }
  }
}

// The main pass as persistent workgroups (KRCA_CORR_PERSIST=1; A/B only, R7a: 2-5 % slower than a
// workgroup per tile, so the per-tile prologue and launch were not what the main pass waits on): one 160 KiB workgroup
// per CU takes the tiles of its XCD's run by ticket (so a workgroup that starts late, its CU busy
// with a re-score, takes fewer), and each tile's last K step loads the next tile's first stage: no
// tile waits on a prologue load or a workgroup launch.  Same tiles, same per-tile arithmetic and
// epilogue as corr_tiles<MODE_MAIN>, so the same bits.
template <int KC>
__global__ __launch_bounds__(Geo<256>::NTH) __attribute__((amdgpu_waves_per_eu(2))) void corr_main_persist(TileArgs A) {
  using G = Geo<256>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* tk = reinterpret_cast<int*>(smem + G::LDS_STAGE + TK_OFF);  // two slots {I, J}: this tile's, the next
  const int x = blockIdx.x & 7;
  if (threadIdx.x == 0) take_tile(A, x, atomicAdd(&A.tick[x], 1u), tk);
  __syncthreads();
  const int nk = A.Tp / G::BKS;
  PState ps;
  ps.b0 = 0;
  ps.staged = false;
  ps.redo = false;
  ps.x = x;
  for (int cur = 0;; cur ^= 1) {
    const int I = tk[2 * cur], J = tk[2 * cur + 1];
    if (I < 0) break;  // uniform: every wave read the slot after the same barriers
    ps.tk_next = tk + 2 * (cur ^ 1);
    const bool more = tile_body<KC, MODE_MAIN, 256, true>(A, I, J, false, 0, &ps);
    ps.b0 ^= nk & 1;  // the last K step loaded the next tile's first stage into the other buffer
    ps.staged = true;
    if (more) {
      // rare: some wave listed more than CAPL_P values; each later window runs the product again
      // (its own stage loads: the next tile's prefetched stage is overwritten and loaded again)
      PState pr = ps;
      pr.redo = true;
      pr.staged = false;
      for (int win = Geo<256>::CAPL_P;; win += Geo<256>::CAPL_P) {
        __syncthreads();  // the window reuses the LDS
        if (!tile_body<KC, MODE_MAIN, 256, true>(A, I, J, false, win, &pr)) break;
      }
      ps.staged = false;
    }
  }
}

// The threshold sample runs in chunks of NSB 128-pod column blocks (its size grows with P, the
// lists of one chunk are [P][NSL][KC]).  After each chunk, one wave per pod merges the chunk's lists
// into the pod's running top-k |r| VALUES (chunks hold disjoint partners, so the k-th best of the
// whole sample is the k-th best of the running values and the chunk's); after the last chunk,
// phi[g] = (k-th best sampled |r|) - 2 eps (-1 if fewer than k): every member of g's exact top-k
// has a screening |r| above it (exact k-th >= sampled k-th - eps).  A flat pod (self product 0:
// z = 0) gets phi = 3 (never a candidate owner; handled exactly).
template <int KC>
__global__ __launch_bounds__(TPB) void corr_theta(const float* __restrict__ sv, const int32_t* __restrict__ si,
                                                  const float* __restrict__ selfd, int64_t g0, int64_t g1, int nsb,
                                                  int k, float eps, float* __restrict__ run, int first, int last,
                                                  float* __restrict__ phi) {
  const int64_t g = g0 + (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (g >= g1) return;
  constexpr int PER = (NSL * KC + 63) / 64 + 1;  // + the running values (lanes < k of the last slot)
  float a[PER];
#pragma unroll
  for (int u = 0; u < PER - 1; ++u) {
    const int q = lane + 64 * u;
    const int lst = q / KC;
    const int64_t e = g * NSL * KC + q;
    const bool used = q < NSL * KC && (lst < nsb || lst >= NSB);
    a[u] = (used && si[e] >= 0) ? fabsf(sv[e]) : -1.f;
  }
  a[PER - 1] = (!first && lane < k) ? run[g * KMAX + lane] : -1.f;
  float kth = -1.f, keep = -1.f;
  for (int r = 0; r < k; ++r) {
    float m = a[0];
#pragma unroll
    for (int u = 1; u < PER; ++u) m = fmaxf(m, a[u]);
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    kth = m;
    if (lane == r) keep = m;
    if (m < 0.f) break;
    // remove one instance of m: the lowest lane holding it, its first slot
    bool has = false;
#pragma unroll
    for (int u = 0; u < PER; ++u) has = has || a[u] == m;
    const uint64_t bal = __ballot(has);
    if (lane == __ffsll((unsigned long long)bal) - 1) {
      bool done = false;
#pragma unroll
      for (int u = 0; u < PER; ++u)
        if (!done && a[u] == m) {
          a[u] = -1.f;
          done = true;
        }
    }
  }
  if (lane < k) run[g * KMAX + lane] = keep;
  if (last && lane == 0) phi[g] = selfd[g] < 0.25f ? 3.f : (kth < 0.f ? -1.f : kth - 2.f * eps - 1e-6f);
}

// ---- exact |r| > tau counts -------------------------------------------------------------------
// dn[p] = || z32[p] - fp16(z32[p]) ||, the fp16 rounding error of row p (float64, rounded up): the
// screening product of a pair then differs from the exact one by at most
//   |h_a.d_b| + |d_a.h_b| + |d_a.d_b| + acc <= dn_a + dn_b + 3 dn_a dn_b + acc
// (||h|| <= 1 + dn, unit-norm rows, acc = the fp32 accumulation terms of eps), typically ~60 % of the
// worst-case eps: most listed pairs are decided from their screening value without reading a row.
//
// With zq (KRCA_CORR_RS_Q16) the same pass writes the re-score's int16 partner rows: step
// qs[p] = max|z32[p]| / 32767, zq[p][t] = rint(z32[p][t] / qs[p]) (zero past T up to Tq, a multiple
// of 8), qn[p] = || z32[p] - qs[p] zq[p] || and nrm[p] = || z32[p] || (float64, rounded up).  A
// pair's za . (qs_b zq_b) then differs from za . zb by at most nrm_a qn_b (~4e-5 at T = 1440).
// VEC (T % 4 == 0): 16-byte loads of z32 and 8-byte loads of zh, 4 steps per lane and load (the
// scalar form was one 4-byte and one 2-byte load per step, 0.38 ms at C3).  zq rounds z / qs by a
// multiply with the reciprocal: any integer q is a valid copy, because qn is the norm of the residual
// z - qs q actually left.
template <bool VEC>
__global__ __launch_bounds__(TPB) void corr_dnorm(const float* __restrict__ z32, const uint16_t* __restrict__ zh,
                                                  int64_t P, int T, int Tp, float* __restrict__ dn,
                                                  int16_t* __restrict__ zq, int Tq, float* __restrict__ qs,
                                                  float* __restrict__ qn, float* __restrict__ nrm) {
  const int lane = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  if (p >= P) return;
  typedef float f4 __attribute__((ext_vector_type(4)));
  typedef unsigned short h4 __attribute__((ext_vector_type(4)));
  typedef short s4 __attribute__((ext_vector_type(4)));
  const float* zr = z32 + p * T;
  const uint16_t* hr = zh + p * Tp;
  double s2 = 0.0, n2 = 0.0;
  float mx = 0.f;
  auto acc = [&](float z, uint16_t h) {
    const double d = (double)z - (double)(float)__builtin_bit_cast(_Float16, h);
    s2 += d * d;
    n2 += (double)z * (double)z;
    mx = fmaxf(mx, fabsf(z));
  };
  if constexpr (VEC) {
    for (int t = 4 * lane; t < T; t += 256) {
      const f4 z = *reinterpret_cast<const f4*>(zr + t);
      const h4 h = *reinterpret_cast<const h4*>(hr + t);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc(z[q], h[q]);
    }
  } else {
    for (int t = lane; t < T; t += 64) acc(zr[t], hr[t]);
  }
  for (int off = 32; off > 0; off >>= 1) {
    s2 += __shfl_xor(s2, off, 64);
    n2 += __shfl_xor(n2, off, 64);
    mx = fmaxf(mx, __shfl_xor(mx, off, 64));
  }
  if (lane == 0) dn[p] = (float)(sqrt(s2) * (1.0 + 1e-6)) + 1e-12f;
  if (!zq) return;
  const float s = mx / 32767.f;  // 0 for a flat row: every q is 0 and so is the error
  const float inv = s > 0.f ? 1.f / s : 0.f;
  double e2 = 0.0;
  auto quant = [&](float z) -> int {
    int q = (int)rintf(z * inv);
    q = q > 32767 ? 32767 : q < -32767 ? -32767 : q;
    const double e = (double)z - (double)q * (double)s;
    e2 += e * e;
    return q;
  };
  int16_t* qr = zq + p * Tq;
  if constexpr (VEC) {
    for (int t = 4 * lane; t < Tq; t += 256) {  // (Tq is a multiple of 8, T of 4: a group is all in or all out)
      s4 o = {0, 0, 0, 0};
      if (t < T) {
        const f4 z = *reinterpret_cast<const f4*>(zr + t);
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (short)quant(z[q]);
      }
      *reinterpret_cast<s4*>(qr + t) = o;
    }
  } else {
    for (int t = lane; t < Tq; t += 64) qr[t] = (int16_t)(t < T ? quant(zr[t]) : 0);
  }
  for (int off = 32; off > 0; off >>= 1) e2 += __shfl_xor(e2, off, 64);
  if (lane == 0) {
    qs[p] = s;
    qn[p] = (float)(sqrt(e2) * (1.0 + 1e-6)) + 1e-12f;
    nrm[p] = (float)(sqrt(n2) * (1.0 + 1e-6)) + 1e-12f;
  }
}

// ---- projection bound of the exact-count re-score (round 6) ----------------------------------
// A listed pair (a, b) has screening value S (the fp16 product) and exact r = z_a . z_b.  With the fp16
// residuals e = z - fp16(z) (f64, exact), r = S_exact + z_a . e_b + e_a . z_b - e_a . e_b, and for an
// orthonormal basis B of KP rows (the first KP DCT-II vectors; the series are smooth -- random walks
// and daily sinusoids -- so most of each row lies in their span):
//   z_a . e_b = (B z_a) . (B e_b) + (Q z_a) . (Q e_b),   |(Q z_a) . (Q e_b)| <= |Q z_a| |Q e_b|,
// with |Q x|^2 = |x|^2 - |B x|^2.  So r lies within
//   |Q z_a| |Q e_b| + |Q e_a| |Q z_b| + |e_a| |e_b| + acc_err
// of S + c, c = (B z_a) . (B e_b) + (B e_a) . (B z_b): a KP-term dot product from the rows'
// projections (256 B per partner) instead of the 2.9 KB int16 partner row.  On the bench's series
// |Q z| is ~0.26 of |z| (tools: the band experiment in DESIGN.md §3.5), so 2.5x fewer pairs read a
// partner row.  Every quantity is float64 (rounded up where it bounds; +1e-9 covers the float64
// sums, as everywhere in the re-score), so the decision is the exact one.
constexpr int KP = 16;  // basis vectors: proj[p] = B z_p (KP floats) | B e_p (KP floats)
__global__ __launch_bounds__(TPB) void corr_dct_basis(double* __restrict__ B, int T) {
  const int64_t n = (int64_t)KP * T;
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    const int j = (int)(i / T), t = (int)(i % T);
    // (rows j >= T are zero: the DCT-II vectors are orthonormal for j < T only, aliases past it)
    B[i] = j >= T ? 0.0 : j == 0 ? sqrt(1.0 / T) : sqrt(2.0 / T) * cospi((2.0 * t + 1.0) * j / (2.0 * T));
  }
}

// 64 rows per workgroup: wave jg owns basis vectors [jg KP/4, (jg + 1) KP/4) and lane r row r, over
// every step, so a basis value is one broadcast LDS read per wave and a row value one conflict-free
// read per lane (a handful of float64 sums per lane).  (R6c/R6d: a lane per row quarter of the steps
// with all KP sums held 256 registers, 3.5 ms at C3; lanes of four basis groups per wave read four
// basis rows 512 B apart, a 4-way bank conflict per read, 1.08 ms.)
constexpr int PJ_ROWS = 64, PJ_TC = 64, PJ_J = KP / 4;
static_assert(TPB == 4 * PJ_ROWS, "four waves: one per basis group");
template <bool VEC>
__global__ __launch_bounds__(TPB) void corr_proj(const float* __restrict__ z32, const uint16_t* __restrict__ zh,
                                                 int64_t P, int T, int Tp, const double* __restrict__ B,
                                                 float* __restrict__ proj, float* __restrict__ pqz,
                                                 float* __restrict__ pqe) {
  __shared__ double sB[KP][PJ_TC];
  __shared__ float sz[PJ_ROWS][PJ_TC + 1];
  __shared__ float se[PJ_ROWS][PJ_TC + 1];
  __shared__ double sn[4][PJ_ROWS][4];  // per wave: |B z|^2, |B e|^2 of its vectors, its share of |z|^2, |e|^2
  const int tid = threadIdx.x, r = tid & 63;
  const int jg = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t p0 = (int64_t)blockIdx.x * PJ_ROWS;
  double bz[PJ_J], be[PJ_J];
#pragma unroll
  for (int j = 0; j < PJ_J; ++j) bz[j] = be[j] = 0.0;
  double nz = 0.0, ne = 0.0;  // this wave's steps [16 jg, 16 jg + 16) of every chunk
  constexpr int NB = KP * PJ_TC / TPB, NZ = PJ_ROWS * PJ_TC / TPB;  // values per lane and chunk
  // a chunk's loads all go out before any is used (a loop of dependent load -> store rounds paid one
  // memory latency per round: 0.96 ms at C3, R6e), and the next chunk's right after this one is in
  // LDS, so they are in flight during its sums (the registers are free by then).  VEC (T % 4 == 0):
  // 16-byte loads, 4 floats / halves or 2 basis values each, so 10 loads per lane and chunk instead
  // of 36 (the scalar form's addresses took the kernel to 212 VGPRs, 2 waves per SIMD)
  constexpr int NZV = VEC ? NZ / 4 : NZ, NBV = VEC ? NB / 2 : NB;
  typedef float f4 __attribute__((ext_vector_type(4)));
  typedef double d2 __attribute__((ext_vector_type(2)));
  typedef unsigned short h4 __attribute__((ext_vector_type(4)));
  d2 bv[NBV];
  f4 zv[NZV];
  h4 hv[NZV];
  auto load = [&](const int t0) {
    if constexpr (VEC) {
#pragma unroll
      for (int u = 0; u < NBV; ++u) {  // basis row j, steps t, t + 1
        const int i = tid + u * TPB, j = i >> 5, t = 2 * (i & 31);
        const bool in = t0 + t < T;
        const d2 v = *reinterpret_cast<const d2*>(B + (int64_t)j * T + (in ? t0 + t : 0));
        bv[u] = in ? v : d2{0.0, 0.0};
      }
#pragma unroll
      for (int u = 0; u < NZV; ++u) {  // row rr, steps t .. t + 3 (16 lanes per row: coalesced)
        const int i = tid + u * TPB, rr = i >> 4, t = 4 * (i & 15);
        const int64_t p = p0 + rr;
        const bool in = p < P && t0 + t < T;
        const int64_t pc = in ? p : 0, tc = in ? t0 + t : 0;
        const f4 zz = *reinterpret_cast<const f4*>(z32 + pc * T + tc);
        const h4 hh = *reinterpret_cast<const h4*>(zh + pc * Tp + tc);
        zv[u] = in ? zz : f4{0.f, 0.f, 0.f, 0.f};
        hv[u] = in ? hh : h4{0, 0, 0, 0};
      }
    } else {
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int i = tid + u * TPB, j = i / PJ_TC, t = i % PJ_TC;
        bv[u].x = t0 + t < T ? B[(int64_t)j * T + t0 + t] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < NZ; ++u) {  // coalesced along t
        const int i = tid + u * TPB, rr = i / PJ_TC, t = i % PJ_TC;
        const int64_t p = p0 + rr;
        const bool in = p < P && t0 + t < T;
        zv[u].x = in ? z32[p * T + t0 + t] : 0.f;
        hv[u].x = in ? zh[p * Tp + t0 + t] : (uint16_t)0;
      }
    }
  };
  auto err = [](float z, unsigned short h) {  // z - fp16(z), exact in float
    return (float)((double)z - (double)(float)__builtin_bit_cast(_Float16, h));
  };
  load(0);
  for (int t0 = 0; t0 < T; t0 += PJ_TC) {
    __syncthreads();  // the previous chunk's reads are done
    if constexpr (VEC) {
#pragma unroll
      for (int u = 0; u < NBV; ++u) {
        const int i = tid + u * TPB, j = i >> 5, t = 2 * (i & 31);
        sB[j][t] = bv[u].x;
        sB[j][t + 1] = bv[u].y;
      }
#pragma unroll
      for (int u = 0; u < NZV; ++u) {
        const int i = tid + u * TPB, rr = i >> 4, t = 4 * (i & 15);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          sz[rr][t + q] = zv[u][q];
          se[rr][t + q] = err(zv[u][q], hv[u][q]);
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int i = tid + u * TPB;
        sB[i / PJ_TC][i % PJ_TC] = bv[u].x;
      }
#pragma unroll
      for (int u = 0; u < NZ; ++u) {
        const int i = tid + u * TPB, rr = i / PJ_TC, t = i % PJ_TC;
        sz[rr][t] = zv[u].x;
        se[rr][t] = err(zv[u].x, hv[u].x);
      }
    }
    __syncthreads();
    if (t0 + PJ_TC < T) load(t0 + PJ_TC);
#pragma unroll 4
    for (int t = 0; t < PJ_TC; ++t) {
      const double z = (double)sz[r][t], e = (double)se[r][t];
      // explicit fused multiply-adds (the library builds with -ffp-contract=off: a * b + c is a
      // multiply and an add there, twice the instructions on this float64 loop)
#pragma unroll
      for (int j = 0; j < PJ_J; ++j) {
        const double b = sB[jg * PJ_J + j][t];  // wave-uniform: a broadcast
        bz[j] = fma(z, b, bz[j]);
        be[j] = fma(e, b, be[j]);
      }
    }
#pragma unroll 4
    for (int t = 16 * jg; t < 16 * jg + 16; ++t) {  // the norms: a quarter of the steps per wave
      const double z = (double)sz[r][t], e = (double)se[r][t];
      nz = fma(z, z, nz);
      ne = fma(e, e, ne);
    }
  }
  double nbz = 0.0, nbe = 0.0;
#pragma unroll
  for (int j = 0; j < PJ_J; ++j) {
    nbz = fma(bz[j], bz[j], nbz);
    nbe = fma(be[j], be[j], nbe);
  }
  sn[jg][r][0] = nbz;
  sn[jg][r][1] = nbe;
  sn[jg][r][2] = nz;
  sn[jg][r][3] = ne;
  const int64_t p = p0 + r;
  if (p < P) {
    float* out = proj + p * (2 * KP);
#pragma unroll
    for (int j = 0; j < PJ_J; ++j) {
      out[jg * PJ_J + j] = (float)bz[j];
      out[KP + jg * PJ_J + j] = (float)be[j];
    }
  }
  __syncthreads();
  if (jg == 0 && p < P) {  // |Q x| = sqrt(|x|^2 - |B x|^2), rounded up (+ the float64 sums' and B's rounding)
    const double bz2 = sn[0][r][0] + sn[1][r][0] + sn[2][r][0] + sn[3][r][0];
    const double be2 = sn[0][r][1] + sn[1][r][1] + sn[2][r][1] + sn[3][r][1];
    const double nz = sn[0][r][2] + sn[1][r][2] + sn[2][r][2] + sn[3][r][2];
    const double ne = sn[0][r][3] + sn[1][r][3] + sn[2][r][3] + sn[3][r][3];
    pqz[p] = (float)(sqrt(fmax(nz - bz2, 0.0) + 1e-12) * (1.0 + 1e-6));
    pqe[p] = (float)(sqrt(fmax(ne - be2, 0.0) + 1e-24) * (1.0 + 1e-6));
  }
}

// the ambiguous pairs in list order, 16 lanes each: decided from the screening value and the two
// rows' rounding-error norms when that suffices, else re-scored (float4 loads of the pair's rows of
// z32, float64 accumulation); persistent over the device-held list length
__global__ __launch_bounds__(TPB) void corr_amb_rescore(const int2* __restrict__ amb, const float* __restrict__ ambv,
                                                        const unsigned long long* __restrict__ amb_n, int64_t cap,
                                                        const float* __restrict__ z32, const float* __restrict__ dn,
                                                        int T, double tau, float acc_err, int32_t* __restrict__ count) {
  const int sub = threadIdx.x & 15;
  const int64_t n = (int64_t)min(*amb_n, (unsigned long long)cap);  // entries past cap were decided in their tiles
  // XCD-aware: workgroups are dispatched round-robin over the 8 XCDs; XCD x takes the contiguous
  // eighth [x n / 8, (x + 1) n / 8) of the list (which runs tile by tile), so the rows of a tile's
  // pairs are fetched into one L2
  const int xcd = blockIdx.x & 7, nb = gridDim.x >> 3;  // gridDim.x: a multiple of 8
  const int64_t q0 = n * xcd / 8, q1 = n * (xcd + 1) / 8;
  for (int64_t q = q0 + (int64_t)(blockIdx.x >> 3) * (TPB / 16) + (threadIdx.x >> 4); q < q1;
       q += (int64_t)nb * (TPB / 16)) {
    const int2 e = amb[q];
    const int64_t a = e.x, b = e.y & (AMB_BOTH - 1);
    const double sa = (double)dn[a], sb = (double)dn[b];
    const double band = sa + sb + 3.0 * sa * sb + (double)acc_err + 1e-9;
    const double v = fabs((double)ambv[q]);
    int hit;
    if (v > (double)tau + band) {
      hit = 1;
    } else if (v <= (double)tau - band) {
      hit = 0;
    } else {  // too close to call from the screening value: float64 from the rows
      hit = fabs(dot16_f64(z32 + a * T, z32 + b * T, T, sub)) > (double)tau;
    }
    if (sub == 0 && hit) {
      atomicAdd(&count[a], 1);
      if (e.y & AMB_BOTH) atomicAdd(&count[b], 1);
    }
  }
}

// ---- the re-score grouped by row pod (KRCA_CORR_RS_GROUP) -----------------------------------------
// corr_amb_rescore reads BOTH rows of every listed pair (11.5 KB at T = 1440; C3: 59.6 GB at the
// DRAM side for 6.5M pairs, 14 % L2 hits).  Grouped, a wave holds the row pod's z32 row in LDS and
// reads only the partner rows: a counting sort of the list by row pod (histogram, scan, scatter),
// then one wave per pod.  The dot products are dot16_f64's, same lanes and order: same bits.
constexpr int GSCAN = 4 * TPB;  // pods per scan block

__global__ __launch_bounds__(TPB) void corr_amb_hist(const int2* __restrict__ amb, const unsigned long long* __restrict__ amb_n,
                                                     int64_t cap, int32_t* __restrict__ gcnt) {
  const int64_t n = (int64_t)min(*amb_n, (unsigned long long)cap);
  for (int64_t q = (int64_t)blockIdx.x * TPB + threadIdx.x; q < n; q += (int64_t)gridDim.x * TPB)
    atomicAdd(&gcnt[amb[q].x], 1);
}

// exclusive scan of TPB x 4 values in LDS order (thread t holds v[4 t .. 4 t + 3]); returns the total
__device__ __forceinline__ int32_t block_scan4(int32_t (&v)[4], int32_t* sh) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int32_t s = v[0] + v[1] + v[2] + v[3];
  int32_t incl = s;
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) sh[wv] = incl;
  __syncthreads();
  int32_t base = 0, total = 0;
  for (int w = 0; w < TPB / 64; ++w) {
    base += w < wv ? sh[w] : 0;
    total += sh[w];
  }
  __syncthreads();
  int32_t run = base + incl - s;
  for (int j = 0; j < 4; ++j) {
    const int32_t x = v[j];
    v[j] = run;
    run += x;
  }
  return total;
}

__global__ __launch_bounds__(TPB) void corr_scan_blocks(const int32_t* __restrict__ gcnt, int64_t P, int32_t* __restrict__ gsum) {
  __shared__ int32_t sh[TPB / 64];
  int32_t v[4];
  const int64_t i0 = (int64_t)blockIdx.x * GSCAN + 4 * threadIdx.x;
  for (int j = 0; j < 4; ++j) v[j] = i0 + j < P ? gcnt[i0 + j] : 0;
  const int32_t tot = block_scan4(v, sh);
  if (threadIdx.x == 0) gsum[blockIdx.x] = tot;
}

// one workgroup: exclusive scan of the nb block totals, in place
__global__ __launch_bounds__(TPB) void corr_scan_top(int32_t* __restrict__ gsum, int64_t nb) {
  __shared__ int32_t sh[TPB / 64];
  int32_t carry = 0;
  for (int64_t c = 0; c < nb; c += GSCAN) {
    int32_t v[4];
    const int64_t i0 = c + 4 * threadIdx.x;
    for (int j = 0; j < 4; ++j) v[j] = i0 + j < nb ? gsum[i0 + j] : 0;
    const int32_t tot = block_scan4(v, sh);
    for (int j = 0; j < 4; ++j)
      if (i0 + j < nb) gsum[i0 + j] = v[j] + carry;
    carry += tot;
    __syncthreads();
  }
}

// goff[p] = exclusive prefix of gcnt (goff[P] = the list length), gcur = goff (scatter cursors)
__global__ __launch_bounds__(TPB) void corr_scan_apply(const int32_t* __restrict__ gcnt, int64_t P,
                                                       const int32_t* __restrict__ gsum, int32_t* __restrict__ goff,
                                                       int32_t* __restrict__ gcur) {
  __shared__ int32_t sh[TPB / 64];
  int32_t v[4], c[4];
  const int64_t i0 = (int64_t)blockIdx.x * GSCAN + 4 * threadIdx.x;
  for (int j = 0; j < 4; ++j) c[j] = v[j] = i0 + j < P ? gcnt[i0 + j] : 0;
  const int32_t tot = block_scan4(v, sh);
  const int32_t base = gsum[blockIdx.x];
  for (int j = 0; j < 4; ++j)
    if (i0 + j < P) {
      goff[i0 + j] = gcur[i0 + j] = base + v[j];
      if (i0 + j == P - 1) goff[P] = base + v[j] + c[j];
    }
  (void)tot;
}

// entries by row pod: {partner | AMB_BOTH, screening value bits} (order within a pod is free: the
// counts are integer sums)
__global__ __launch_bounds__(TPB) void corr_amb_scatter(const int2* __restrict__ amb, const float* __restrict__ ambv,
                                                        const unsigned long long* __restrict__ amb_n, int64_t cap,
                                                        int32_t* __restrict__ gcur, int2* __restrict__ gs) {
  const int64_t n = (int64_t)min(*amb_n, (unsigned long long)cap);
  for (int64_t q = (int64_t)blockIdx.x * TPB + threadIdx.x; q < n; q += (int64_t)gridDim.x * TPB) {
    const int2 e = amb[q];
    const int32_t pos = atomicAdd(&gcur[e.x], 1);
    gs[pos] = make_int2(e.y, __float_as_int(ambv[q]));
  }
}

// one wave per row pod with entries (persistent over the pods): its z32 row into the wave's LDS
// slot, then 4 groups of 16 lanes take its partners, corr_amb_rescore's decision for each
constexpr int RS_WAVES = TPB / 64;
constexpr int RS_QCAP = 64;  // pairs queued per wave for the row path
__global__ __launch_bounds__(TPB) void corr_amb_rescore_grouped(const int32_t* __restrict__ goff, const int2* __restrict__ gs,
                                                                int64_t P, const float* __restrict__ z32,
                                                                const float* __restrict__ dn, int T, double tau,
                                                                float acc_err, int32_t* __restrict__ count,
                                                                const int16_t* __restrict__ zq, int Tq,
                                                                const float* __restrict__ qs, const float* __restrict__ qn,
                                                                const float* __restrict__ nrm, const float* __restrict__ proj,
                                                                const float* __restrict__ pqz, const float* __restrict__ pqe) {
  extern __shared__ float4 rs_lds[];
  __shared__ int32_t rs_queue[RS_WAVES][RS_QCAP];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, sub = lane & 15, grp = lane >> 4;
  const int T4 = (T + 3) / 4;
  const int L4 = zq ? Tq / 4 : T4;  // floats per wave slot / 4 (the int16 dot reads zeros past T)
  float* ra = reinterpret_cast<float*>(rs_lds + (size_t)wv * L4);
  for (int64_t a = (int64_t)blockIdx.x * RS_WAVES + wv; a < P; a += (int64_t)gridDim.x * RS_WAVES) {
    const int32_t e0 = goff[a], e1 = goff[a + 1];
    if (e0 == e1) continue;  // wave-uniform
    const float* za = z32 + a * T;
    if ((T & 3) == 0) {
      for (int t = lane; t < T4; t += 64) rs_lds[(size_t)wv * L4 + t] = reinterpret_cast<const float4*>(za)[t];
    } else {
      for (int t = lane; t < T; t += 64) ra[t] = za[t];
    }
    for (int t = T + lane; t < 4 * L4; t += 64) ra[t] = 0.f;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const double sa = (double)dn[a];
    const double na = zq ? (double)nrm[a] : 0.0;
    // the row pod's projections for the projection bound: lane sub < 8 holds 2 floats of B e_a (they
    // pair with the partner's B z), sub >= 8 2 floats of B z_a (with the partner's B e)
    float2 pa = make_float2(0.f, 0.f);
    double qza = 0.0, qea = 0.0;
    if (proj) {
      static_assert(2 * KP == 32, "16 lanes x 2 floats hold a row's projections");
      pa = reinterpret_cast<const float2*>(proj + a * (2 * KP))[sub ^ 8];
      qza = (double)pqz[a];
      qea = (double)pqe[a];
    }
    int hits = 0;
    // the decision of one listed pair from the rows (int16 partner row, then the fp32 one within its
    // bound): uniform over the 16-lane group
    auto from_rows = [&](int64_t b) -> int {
      int dec = -1;
      if (zq) {  // |za . qs_b zq_b - za . zb| <= nrm_a qn_b (+ 1e-9 for the float64 sums)
        const double vq = fabs(dot16_q16(ra, zq + b * Tq, Tq, sub) * (double)qs[b]);
        const double bq = na * (double)qn[b] + 1e-9;
        dec = vq > (double)tau + bq ? 1 : vq <= (double)tau - bq ? 0 : -1;
      }
      return dec >= 0 ? dec : (fabs(dot16_f64_pf(ra, z32 + b * T, T, sub)) > (double)tau ? 1 : 0);
    };
    auto credit = [&](int hit, int2 e) {
      if (sub == 0 && hit) {
        ++hits;
        if (e.x & AMB_BOTH) atomicAdd(&count[(int64_t)(e.x & (AMB_BOTH - 1))], 1);
      }
    };
    // Pass 1: the pair's own bound, then the projection bound; the pairs neither settles go to the
    // wave's queue, which pass 2 drains with all four groups busy (a group waiting on a partner row
    // while the other three had settled theirs kept the wave for as long as the row path: R6c)
    int32_t* wq = rs_queue[wv];
    int nq = 0;  // wave-uniform
    auto drain = [&]() {
      for (int base = 0; base < nq; base += 4) {  // wave-uniform trip count
        const int i = base + grp;
        if (i < nq) {  // uniform over the group
          const int2 e = gs[wq[i]];
          credit(from_rows(e.x & (AMB_BOTH - 1)), e);
        }
      }
      nq = 0;
    };
    for (int32_t base = e0; base < e1; base += 4) {
      const int32_t q = base + grp;
      int need = 0;
      if (q < e1) {  // uniform over the group
        const int2 e = gs[q];
        const int64_t b = e.x & (AMB_BOTH - 1);
        const double sb = (double)dn[b];
        const double band = sa + sb + 3.0 * sa * sb + (double)acc_err + 1e-9;
        const double v = fabs((double)__int_as_float(e.y));
        int dec = v > (double)tau + band ? 1 : v <= (double)tau - band ? 0 : -1;
        if (dec < 0 && proj) {  // 128 B of the partner instead of its row
          const float2 pb = reinterpret_cast<const float2*>(proj + b * (2 * KP))[sub];
          double c = (double)pa.x * (double)pb.x + (double)pa.y * (double)pb.y;
          for (int off = 8; off > 0; off >>= 1) c += __shfl_xor(c, off, 16);
          const double est = fabs((double)__int_as_float(e.y) + c);
          const double bp = qza * (double)pqe[b] + qea * (double)pqz[b] + sa * sb + (double)acc_err + 1e-9;
          dec = est > (double)tau + bp ? 1 : est <= (double)tau - bp ? 0 : -1;
        }
        if (dec >= 0) credit(dec, e);
        else need = 1;
      }
      const uint64_t m = __ballot(need && sub == 0);  // one bit per group that queues its pair
      if (need && sub == 0)
        wq[nq + __builtin_popcountll(m & ((1ull << lane) - 1ull))] = q;
      nq += __builtin_popcountll(m);
      if (nq > RS_QCAP - 4) {  // wave-uniform
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        drain();
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    drain();
    if (sub == 0 && hits) atomicAdd(&count[a], hits);
    // every lane is past its partners before the next pod's row lands in the slot
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// ---- merge + exact re-scoring ------------------------------------------------------------------
__device__ __forceinline__ bool cbetter(float a, int32_t ia, float b, int32_t ib) {
  if (ib < 0) return ia >= 0;
  if (ia < 0) return false;
  const float fa = fabsf(a), fb = fabsf(b);
  return fa > fb || (fa == fb && ia < ib);
}

// rows of the overflowed pods, gathered for the second (rectangle) pass; padding rows are zero
__global__ __launch_bounds__(TPB) void corr_gather_rows(const uint16_t* __restrict__ zh, int Tp,
                                                        const int32_t* __restrict__ pods, int64_t n,
                                                        uint16_t* __restrict__ zs) {
  const int64_t r = blockIdx.x;
  const uint4* src = reinterpret_cast<const uint4*>(zh + (int64_t)(r < n ? pods[r] : 0) * Tp);
  uint4* dst = reinterpret_cast<uint4*>(zs + r * Tp);
  for (int c = threadIdx.x; c < Tp / 8; c += TPB) dst[c] = r < n ? src[c] : make_uint4(0, 0, 0, 0);
}

// compare-exchange of lane pairs (lane, lane ^ j) in (|r| desc, index asc, empties last) order:
// keep_better picks the better of the two, else the other one
__device__ __forceinline__ void cand_cx(float& v, int32_t& i, int j, bool keep_better) {
  const float pv = __shfl_xor(v, j, 64);
  const int32_t pi = __shfl_xor(i, j, 64);
  if (cbetter(pv, pi, v, i) == keep_better) {
    v = pv;
    i = pi;
  }
}

// lanes 0-31 hold a sorted list (best first); (cv, ci) a sorted 64-lane chunk: afterwards lanes
// 0-31 hold the best 32 of both (bitonic: the chunk's best 32 reversed into lanes 32-63, one merge)
__device__ __forceinline__ void cand_merge32(float& v, int32_t& i, float cv, int32_t ci, int lane) {
  const float rv = __shfl(cv, 63 - lane, 64);
  const int32_t ri = __shfl(ci, 63 - lane, 64);
  if (lane >= 32) {
    v = rv;
    i = ri;
  }
#pragma unroll
  for (int j = 32; j > 0; j >>= 1) cand_cx(v, i, j, (lane & j) == 0);
}

// one workgroup per pod (or per listed pod in the second pass): select the pod's best km + 1
// candidates, re-score the best km = k + 6 in float64, rank, certify.  Pass 0 turns an overflowed buffer into phi2 and
// queues the pod for the second main pass (over[0] = count, over[1..] = pods).
__global__ __launch_bounds__(TPB) void corr_merge(const int2* __restrict__ buf, int32_t* __restrict__ cnt,
                                                  const float* __restrict__ phi_used, const float* __restrict__ z32,
                                                  int64_t P, int T, int k, float eps, int pass,
                                                  const int32_t* __restrict__ pods, float* __restrict__ phi2,
                                                  int32_t* __restrict__ over, int32_t* __restrict__ out_i,
                                                  float* __restrict__ out_v, float* __restrict__ cert, int64_t lo,
                                                  int32_t* __restrict__ deep, int capc, int km_extra) {
  __shared__ float wl_v[TPB / 64][32];
  __shared__ int32_t wl_i[TPB / 64][32];
  __shared__ float top_v[KM + 1];
  __shared__ int32_t top_i[KM + 1];
  __shared__ double exact[KM];
  __shared__ int ord[KM];
  const int64_t g = pods ? pods[blockIdx.x] : lo + blockIdx.x;  // global pod id
  const int64_t gl = g - lo;  // index into this rank's buffers and outputs
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float ph = phi_used[g];
  const bool flat = ph > 2.f;
  const int n = cnt[gl];
  const bool overflow = n > capc;
  const int km = k + km_extra < KM ? k + km_extra : KM;
  if (flat) {  // r = 0 with every partner: the lowest other indices, in order
    if (tid <= KM) {
      const int64_t q = tid < g ? tid : tid + 1;
      top_i[tid] = q < P ? (int32_t)q : -1;
      top_v[tid] = 0.f;
    }
  } else {
    // selection instead of a sort: every wave keeps the best 32 of its 64-candidate chunks (a
    // bitonic sort of the chunk in registers, then one merge into the running list), wave 0 merges
    // the waves' lists; the order is total, so the best km + 1 are those of a full sort
    static_assert(KM + 1 <= 32, "the selection keeps 32 per wave");
    const int nn = overflow ? capc : n;
    float v = 0.f;
    int32_t iv = -1;
    for (int c0 = 64 * w; c0 < nn; c0 += TPB) {  // wave-uniform
      float cvv = 0.f;
      int32_t cii = -1;
      if (c0 + lane < nn) {
        const int2 c = buf[gl * CAPC + c0 + lane];
        cvv = __int_as_float(c.x);
        cii = c.y;
      }
#pragma unroll
      for (int kk = 2; kk <= 64; kk <<= 1)
#pragma unroll
        for (int j = kk >> 1; j > 0; j >>= 1) cand_cx(cvv, cii, j, ((lane & j) == 0) == ((lane & kk) == 0));
      if (c0 == 64 * w) {
        v = cvv;
        iv = cii;
      } else {
        cand_merge32(v, iv, cvv, cii, lane);
      }
    }
    if (lane < 32) {
      wl_v[w][lane] = v;
      wl_i[w][lane] = iv;
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int u = 1; u < TPB / 64; ++u)
        cand_merge32(v, iv, lane < 32 ? wl_v[u][lane] : 0.f, lane < 32 ? wl_i[u][lane] : -1, lane);
      if (lane <= KM) {
        top_v[lane] = v;
        top_i[lane] = iv;
      }
    }
    __syncthreads();
    if (overflow && pass == 0) {  // any stored subset bounds the exact k-th from below
      if (tid == 0) {
        phi2[g] = fabsf(top_v[k - 1]) - 2.f * eps - 1e-6f;
        cnt[gl] = 0;
        over[1 + atomicAdd(&over[0], 1)] = (int32_t)g;
      }
      return;
    }
  }
  __syncthreads();
  // exact float64 re-scoring of the best km (one wave per candidate, fixed reduction order)
  const float* zg = z32 + g * T;
  {  // wave w re-scores candidates w, w+4, ... together (independent loads in flight)
    constexpr int PER = (KM + TPB / 64 - 1) / (TPB / 64);
    const float* zj[PER];
    double acc2[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int q = w + u * (TPB / 64);
      zj[u] = (q < km && top_i[q] >= 0) ? z32 + (int64_t)top_i[q] * T : nullptr;
      acc2[u] = 0.0;
    }
    if ((T & 3) == 0) {  // rows are 16-B aligned: float4 loads (1 KiB per wave instruction)
      const float4* g4 = reinterpret_cast<const float4*>(zg);
      for (int t = lane; t < T / 4; t += 64) {
        const float4 a = g4[t];
#pragma unroll
        for (int u = 0; u < PER; ++u)
          if (zj[u]) {
            const float4 b = reinterpret_cast<const float4*>(zj[u])[t];
            acc2[u] += (double)a.x * (double)b.x + (double)a.y * (double)b.y + (double)a.z * (double)b.z +
                       (double)a.w * (double)b.w;
          }
      }
    } else {
      for (int t = lane; t < T; t += 64) {
        const double a = (double)zg[t];
#pragma unroll
        for (int u = 0; u < PER; ++u)
          if (zj[u]) acc2[u] += a * (double)zj[u][t];
      }
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      double s = acc2[u];
      for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
      const int q = w + u * (TPB / 64);
      if (lane == 0 && q < km) exact[q] = s;
    }
  }
  __syncthreads();
  if (tid < km) {  // rank of candidate tid: |exact| desc, index asc, empty last
    const double fk = fabs(exact[tid]);
    const int32_t ik = top_i[tid];
    int rank = 0;
    for (int o = 0; o < km; ++o) {
      const double fo = fabs(exact[o]);
      const int32_t io = top_i[o];
      rank += o != tid && io >= 0 && (ik < 0 || fo > fk || (fo == fk && io < ik));
    }
    ord[rank] = tid;
  }
  __syncthreads();
  for (int q = tid; q < k; q += TPB) {
    out_i[gl * k + q] = top_i[ord[q]];
    out_v[gl * k + q] = (float)exact[ord[q]];
  }
  if (tid == 0) {
    // everything not re-scored has a screening |r| <= max(phi, the first un-re-scored candidate)
    const float dropped = fmaxf(ph, top_i[km] >= 0 ? fabsf(top_v[km]) : 0.f);
    const float c = flat ? 1.f
                         : overflow ? -1.f : (float)(fabs(exact[ord[k - 1]]) - (double)dropped - (double)eps);
    cert[gl] = c;
    // near-ties around the k-th: re-score every candidate (corr_merge_deep)
    if (!(c > 0.f) && !flat && !overflow && n >= k) deep[1 + atomicAdd(&deep[0], 1)] = (int32_t)g;
  }
}

// one workgroup per listed pod (its merge left cert <= 0): buffered candidates re-scored in float64
// (one wave per candidate, the merge's fixed-order reduction), sorted by (|r| desc, index asc), top k
// written.  Pass 0 re-scores only the candidates whose screening |r| reaches the merge's k-th exact
// value - 2 eps (near-ties around the k-th: usually a handful, not the whole buffer); the rest have
// exact |r| <= their screening |r| + eps, so it certifies with that bound in place of phi when it
// can.  Pass 1 (only if not) re-scores every candidate: partners outside the buffer have a screening
// |r| <= phi, so the k-th exact |r| minus phi minus eps certifies the set (> 0 whenever the buffer
// holds the k sampled partners).
__global__ __launch_bounds__(TPB) void corr_merge_deep(const int2* __restrict__ buf, const int32_t* __restrict__ cnt,
                                                       const float* __restrict__ phi, const float* __restrict__ phi2,
                                                       const float* __restrict__ z32,
                                                       int T, int k, float eps, const int32_t* __restrict__ pods,
                                                       int32_t* __restrict__ out_i, float* __restrict__ out_v,
                                                       float* __restrict__ cert, int64_t lo, int capc) {
  __shared__ double ex[CAPC];
  __shared__ int32_t ci[CAPC];
  __shared__ int srest;  // pass 0: the largest screening |r| left out (float bits, >= 0), INT_MIN = none
  __shared__ int ssel;   // pass 0: candidates taken (packed at the front of ci)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nd = pods[0];  // list length first (device-held: no host round trip)
  for (int b = blockIdx.x; b < nd; b += gridDim.x) {
  const int64_t g = pods[1 + b];
  const int64_t gl = g - lo;
  const int n = min(cnt[gl], capc);
  int np = 32;
  while (np < n) np <<= 1;
  // the merge's k-th exact |r| (its output row, written before it listed the pod)
  const float thr = fabsf(out_v[gl * k + k - 1]) - 2.f * eps - 1e-6f;
  for (int pass = 0; pass < 2; ++pass) {
  __syncthreads();  // ex / ci / srest of the previous pod or pass
  if (tid == 0) {
    srest = INT_MIN;
    ssel = 0;
  }
  __syncthreads();
  int ns = np;  // slots re-scored and sorted
  if (pass == 0) {
    // the near-ties only, packed at the front (their order is free: the sort below is total), so
    // the re-score and the sort run over a power of two >= their count, not over the whole buffer
    for (int i = tid; i < n; i += TPB) {
      const int2 e = buf[gl * CAPC + i];
      const float a = fabsf(__int_as_float(e.x));
      if (a >= thr) ci[atomicAdd(&ssel, 1)] = e.y;
      else atomicMax(&srest, __float_as_int(a));
    }
    __syncthreads();
    const int m = ssel;
    ns = 32;
    while (ns < m) ns <<= 1;
    for (int i = m + tid; i < ns; i += TPB) ci[i] = -1;
  } else {
    for (int i = tid; i < np; i += TPB) ci[i] = i < n ? buf[gl * CAPC + i].y : -1;
  }
  __syncthreads();
  const float* zg = z32 + g * T;
  // wave w re-scores candidates 4w .. 4w + 3, then 4w + 16 .., together (independent loads in flight;
  // float4 loads when the rows are 16-B aligned)
  constexpr int PD = 4;
  for (int c0 = PD * w; c0 < ns; c0 += PD * (TPB / 64)) {
    const float* zj[PD];
    double acc[PD];
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      const int32_t j = c0 + u < ns ? ci[c0 + u] : -1;
      zj[u] = j >= 0 ? z32 + (int64_t)j * T : nullptr;
      acc[u] = 0.0;
    }
    if (!zj[0]) {  // (slots past the taken candidates: every one of the group is empty)
    } else if ((T & 3) == 0) {
      const float4* g4 = reinterpret_cast<const float4*>(zg);
      for (int t = lane; t < T / 4; t += 64) {
        const float4 a = g4[t];
#pragma unroll
        for (int u = 0; u < PD; ++u)
          if (zj[u]) {
            const float4 b = reinterpret_cast<const float4*>(zj[u])[t];
            acc[u] += (double)a.x * (double)b.x + (double)a.y * (double)b.y + (double)a.z * (double)b.z +
                      (double)a.w * (double)b.w;
          }
      }
    } else {
      for (int t = lane; t < T; t += 64) {
        const double a = (double)zg[t];
#pragma unroll
        for (int u = 0; u < PD; ++u)
          if (zj[u]) acc[u] += a * (double)zj[u][t];
      }
    }
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      double v = acc[u];
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
      if (lane == 0 && c0 + u < ns) ex[c0 + u] = zj[u] ? v : 0.0;
    }
  }
  __syncthreads();
  for (int kk = 2; kk <= ns; kk <<= 1) {  // bitonic: |r| desc, index asc, empties last
    for (int j = kk >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < ns; i += TPB) {
        const int l = i ^ j;
        if (l > i) {
          const bool desc = (i & kk) == 0;
          const double fa = fabs(ex[l]), fb = fabs(ex[i]);
          const int32_t ia = ci[l], ib = ci[i];
          const bool better = ib < 0 ? ia >= 0 : (ia >= 0 && (fa > fb || (fa == fb && ia < ib)));
          if (better == desc) {
            const double tv = ex[i];
            ex[i] = ex[l];
            ex[l] = tv;
            ci[i] = ia;
            ci[l] = ib;
          }
        }
      }
      __syncthreads();
    }
  }
  // the bound of the buffer: phi2 for a pod refilled by the rectangle pass (3 = not refilled); in
  // pass 0 also the screening |r| of the candidates left out
  const float ph = phi2[g] < 2.5f ? phi2[g] : phi[g];
  const float bound = srest == INT_MIN ? ph : fmaxf(ph, __int_as_float(srest));
  const float c = (float)(fabs(ex[k - 1]) - (double)bound - (double)eps);
  if (pass == 1 || (ci[k - 1] >= 0 && c > 0.f)) {  // block-uniform
    for (int q = tid; q < k; q += TPB) {
      out_i[gl * k + q] = ci[q];
      out_v[gl * k + q] = (float)ex[q];
    }
    if (tid == 0) cert[gl] = c;
    break;
  }
  }
  }
}

// profiling aid, KRCA_CORR_DEBUG (results are wrong when set): 1 = product only, 4 = product only
// with every tile reading the same few row blocks (operands L2-resident), 5 = no entries written out,
// 6 = the epilogue's first step only (counts and raw lists, nothing committed)
int debug_mode() { return krca::tuning().corr_debug; }

constexpr int RECT_ROWS = 4096;  // rows of the second (rectangle) pass per launch

// ---- exchange of the sharded run: candidates of pod p travel to its owner p / n_max ----------
// totals per destination (clipped at the cap: the owner's merge reads the all-reduced raw counts,
// so a pod past the cap on any rank overflows at its owner too)
__global__ __launch_bounds__(TPB) void corr_pack_count(const int32_t* __restrict__ cnt, int64_t P, int64_t n_max,
                                                       unsigned long long* __restrict__ tot, int capc) {
  const int64_t p = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (p >= P) return;
  const int c = min(cnt[p], capc);
  if (c) atomicAdd(&tot[p / n_max], (unsigned long long)c);
}

// one wave per pod: reserve its range in the destination's region, copy {pod, partner, r bits}
__global__ __launch_bounds__(TPB) void corr_pack(const int32_t* __restrict__ cnt, const int2* __restrict__ buf, int64_t P,
                                                 int64_t n_max, const unsigned long long* __restrict__ off,
                                                 unsigned long long* __restrict__ cursor, int4* __restrict__ send,
                                                 int capc) {
  const int64_t p = (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (p >= P) return;
  const int c = min(cnt[p], capc);
  if (c == 0) return;
  const int64_t h = p / n_max;
  unsigned long long base = 0;
  if (lane == 0) base = off[h] + atomicAdd(&cursor[h], (unsigned long long)c);
  base = __shfl(base, 0, 64);
  for (int i = lane; i < c; i += 64) {
    const int2 e = buf[p * CAPC + i];
    send[base + i] = make_int4((int)p, e.y, e.x, 0);
  }
}

// received entries -> this rank's per-pod buffers (any order: the merge sorts)
__global__ __launch_bounds__(TPB) void corr_unpack(const int4* __restrict__ recv, int64_t n, int64_t lo,
                                                   int32_t* __restrict__ fill, int2* __restrict__ lbuf, int capc) {
  const int64_t e = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (e >= n) return;
  const int4 v = recv[e];
  const int64_t q = v.x - lo;
  const int s = atomicAdd(&fill[q], 1);
  if (s < capc) lbuf[q * CAPC + s] = make_int2(v.z, v.y);
}

struct CorrWs {  // views into a caller's candidate workspace
  int2* buf;      // [P][CAPC] appends of the main pass (global pod index)
  int32_t* cnt;   // [P]
  float* samp_v;  // [P][NSL][KC]
  int32_t* samp_i;
  float *selfd, *phi2;  // [P]
  float* run;           // [P][KMAX] running top-k |r| of the threshold sample
  int32_t* over;        // [n_loc + 1]
  int32_t* deep;        // [n_loc + 1]: pods for corr_merge_deep (count first)
  int2* amb[2];         // [amb_cap] ambiguous pairs of a main-pass batch (contiguous per tile), two lists
  float* ambv[2];       // [amb_cap] their screening values
  int64_t amb_cap;
  int nlist;            // lists in use (2 when the main pass runs in more than one batch)
  float* dn;            // [P] fp16 rounding-error norm of each row
  int16_t* zq;          // [P][Tq] int16 partner rows of the grouped re-score (KRCA_CORR_RS_Q16), else null
  float *qs, *qn, *nrm; // [P] their step, error norm, the fp32 row's norm
  float* proj;          // [P][2 KP] B z | B e of each row (the projection bound), else unused
  float *pqz, *pqe;     // [P] |Q z|, |Q e|
  double* dct;          // [KP][T] the basis
  int Tq;               // T rounded up to 8
  unsigned long long* amb_n;  // [2]: the lists' fill
  unsigned* tick;             // [8 * batches]: the persistent main pass's ticket counters per XCD
  int32_t *gcnt, *goff, *gcur, *gsum;  // grouped re-score: entries per row pod, offsets [P + 1], cursors, scan blocks
  int2* gs;                            // [amb_cap] a list's entries grouped by row pod
  uint16_t* zs;         // [RECT_ROWS][Tp]
  int2* lbuf;           // sharded: [n_loc][CAPC] received candidates of the rank's pods
  int32_t* fill;        // sharded: [n_loc]
  unsigned long long* xc;  // sharded: tot[G] | off[G] | cursor[G]
};

// super-tiles of the upper triangle of nb2 256-blocks
inline int64_t n_supertiles(int64_t nb2) {
  const int64_t ns = (nb2 + SUPER - 1) / SUPER;
  return ns * (ns + 1) / 2;
}

// layout in 4-byte words; sharded adds the local buffers and the exchange counters
int64_t ws_layout(int64_t P, int T, int Tp, int KC, int64_t n_loc, int G, char* base, CorrWs* ws) {
  int64_t o = 0;
  auto take = [&](int64_t words) {
    char* ptr = base ? base + 4 * o : nullptr;
    o += krca::ceil_div(words, 4) * 4;  // 16-byte aligned pieces
    return ptr;
  };
  CorrWs w{};
  w.buf = reinterpret_cast<int2*>(take(2 * P * CAPC));
  w.cnt = reinterpret_cast<int32_t*>(take(P));
  w.samp_v = reinterpret_cast<float*>(take(P * NSL * KC));
  w.samp_i = reinterpret_cast<int32_t*>(take(P * NSL * KC));
  w.selfd = reinterpret_cast<float*>(take(P));
  w.run = reinterpret_cast<float*>(take(P * KMAX));
  w.phi2 = reinterpret_cast<float*>(take(P));
  w.over = reinterpret_cast<int32_t*>(take(n_loc + 1));
  w.deep = reinterpret_cast<int32_t*>(take(n_loc + 1));
  const int64_t n_st = n_supertiles(krca::ceil_div(P, TB));
  const int64_t SB = sb_batch();
  w.amb_cap = std::min(n_st, SB) * SUPER * SUPER * amb_per_tile();
  w.nlist = n_st > SB ? 2 : 1;  // (a sharded rank runs a subset: at most as many batches)
  for (int l = 0; l < 2; ++l) {
    w.amb[l] = l < w.nlist ? reinterpret_cast<int2*>(take(2 * w.amb_cap)) : nullptr;
    w.ambv[l] = l < w.nlist ? reinterpret_cast<float*>(take(w.amb_cap)) : nullptr;
  }
  w.dn = reinterpret_cast<float*>(take(P));
  w.Tq = (int)krca::ceil_div(T, 8) * 8;
  {  // reserved whatever the knobs say (a size query and the call must agree); used when both are on
    w.zq = reinterpret_cast<int16_t*>(take(P * w.Tq / 2));
    w.qs = reinterpret_cast<float*>(take(P));
    w.qn = reinterpret_cast<float*>(take(P));
    w.nrm = reinterpret_cast<float*>(take(P));
    w.proj = reinterpret_cast<float*>(take(P * 2 * KP));  // the projection bound's rows (corr_proj)
    w.pqz = reinterpret_cast<float*>(take(P));
    w.pqe = reinterpret_cast<float*>(take(P));
    w.dct = reinterpret_cast<double*>(take(2 * (int64_t)KP * T));
  }
  w.amb_n = reinterpret_cast<unsigned long long*>(take(4));
  w.tick = reinterpret_cast<unsigned*>(take(8 * krca::ceil_div(n_st, SB)));
  w.gcnt = reinterpret_cast<int32_t*>(take(P));
  w.goff = reinterpret_cast<int32_t*>(take(P + 1));
  w.gcur = reinterpret_cast<int32_t*>(take(P));
  w.gsum = reinterpret_cast<int32_t*>(take(krca::ceil_div(P, GSCAN) + 1));
  w.gs = reinterpret_cast<int2*>(take(2 * w.amb_cap));
  w.zs = reinterpret_cast<uint16_t*>(take((int64_t)RECT_ROWS * Tp / 2));
  if (G > 0) {
    w.lbuf = reinterpret_cast<int2*>(take(2 * n_loc * CAPC));
    w.fill = reinterpret_cast<int32_t*>(take(n_loc));
    w.xc = reinterpret_cast<unsigned long long*>(take(6 * (int64_t)G));
  }
  if (ws) *ws = w;
  return o;
}

template <int KC, int MODE, int TC>
int set_lds_attr1() {
  static bool done = false;  // > 64 KB of dynamic LDS needs the opt-in once per kernel
  if (!done) {
    KRCA_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_tiles<KC, MODE, TC>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, Geo<TC>::LDS_BYTES));
    done = true;
  }
  return KRCA_OK;
}
template <int KC>
int set_lds_attr() {
  int rc = set_lds_attr1<KC, MODE_MAIN, 256>();
  if (!rc) rc = set_lds_attr1<KC, MODE_SAMPLE, 256>();
  if (!rc) rc = set_lds_attr1<KC, MODE_RECT, 256>();
  static bool done_p = false;
  if (!rc && !done_p) {
    KRCA_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_main_persist<KC>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, Geo<256>::LDS_PERSIST));
    done_p = true;
  }
  return rc;
}

// compute units of the current device (the persistent main pass: one workgroup per CU)
inline int cu_count() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 256;
  return n > 0 ? n : 256;
}

struct Dims {
  int64_t P;
  int T, Tp, nb2, nsb, k;
  double tau;  // float64: the exact r of a pair is compared with it (a float tau = 0.6 is 0.60000002)
  float eps;
};

Dims dims_of(int64_t P, int T, int k, double tau) {
  Dims d;
  d.P = P;
  d.T = T;
  d.Tp = (int)krca::ceil_div(T, BK) * BK;
  d.nb2 = (int)krca::ceil_div(P, TB);
  // threshold sample: ~P*k/500 pods (>= NSB blocks of 128), so that about 500 partners per pod clear
  // phi at any P (2,048 at C3; a fixed 2,048 at 1M pods let ~0.4 % of a million partners through)
  d.nsb = (int)std::min<int64_t>(2 * d.nb2, std::max<int64_t>(NSB, krca::ceil_div(P * k, 500 * 128)));
  d.k = k;
  d.tau = tau;
  d.eps = (float)(std::ldexp(1.0, -10) * 1.001 + std::ldexp((double)T, -24) + std::ldexp(std::sqrt((double)T), -23));
  return d;
}

// 1. threshold sample of the row blocks holding pods [lo, lo + n): phi for those pods
template <int KC>
int stage_sample(const uint16_t* zh, const Dims& d, int64_t lo, int64_t n, const CorrWs& ws, float* phi,
                 hipStream_t st) {
  if (int rc = set_lds_attr<KC>()) return rc;
  const int64_t I0 = lo / TB, I1 = krca::ceil_div(lo + n, TB);
  const int nsb2_all = (d.nsb + 1) / 2;
  // self products default to 1 ("not flat"): every pod's is recorded by a sample tile, and a
  // missed one must never read as a stale value below the flat threshold
  KRCA_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(ws.selfd + lo), 0x3F800000 /* 1.0f */, (size_t)n, st));
  for (int c0 = 0; c0 < nsb2_all; c0 += NSB / 2) {  // chunks of NSB 128-blocks
    const int nsb_c = std::min(NSB, d.nsb - 2 * c0);
    const int nsb2 = (nsb_c + 1) / 2;
    KRCA_HIP(hipMemsetAsync(ws.samp_i + lo * NSL * KC, 0xff, (size_t)n * NSL * KC * sizeof(int32_t), st));
    Shard sh{0, 1, 0, I0};
    sh.j0 = c0;
    sh.own = c0 == 0;
    sh.nsb2_all = nsb2_all;
    TileArgs ta{};
    ta.zA = zh;
    ta.zh = zh;
    ta.P = d.P;
    ta.Tp = d.Tp;
    ta.nb2 = d.nb2;
    ta.nsb = nsb_c;
    ta.samp_v = ws.samp_v;
    ta.samp_i = ws.samp_i;
    ta.samp_run = c0 > 0 ? ws.run : nullptr;  // (written by corr_theta after the previous chunk)
    ta.k = d.k;
    ta.selfd = ws.selfd;
    ta.sh = sh;
    ta.debug = debug_mode();
    ta.n_tiles = (I1 - I0) * (nsb2 + 1);
    ta.per_xcd = (ta.n_tiles + 7) / 8;
    hipLaunchKernelGGL((corr_tiles<KC, MODE_SAMPLE, 256>), dim3((unsigned)(8 * ta.per_xcd)),
                       dim3(Geo<256>::NTH), Geo<256>::LDS_BYTES, st, ta);
    KRCA_LAUNCH_CHECK();
    hipLaunchKernelGGL(corr_theta<KC>, dim3((unsigned)krca::ceil_div(n, TPB / 64)), dim3(TPB), 0, st, ws.samp_v,
                       ws.samp_i, ws.selfd, lo, lo + n, nsb_c, d.k, d.eps, ws.run, (int)(c0 == 0),
                       (int)(c0 + NSB / 2 >= nsb2_all), phi);
    KRCA_LAUNCH_CHECK();
  }
  return KRCA_OK;
}

// candidates the merge re-scores past the k-th: KRCA_CORR_KM_EXTRA (1 .. KM - KMAX), default 6
inline int km_extra() {
  const int e = krca::tuning().corr_km_extra;
  return e >= 1 && e <= KM - KMAX ? e : 6;
}

// candidate slots used per pod: CAPC, or fewer under KRCA_CORR_CAPC (tests: overflows on purpose)
inline int cand_cap() {
  const int c = krca::tuning().corr_capc;
  return c >= 64 && c < CAPC ? c : CAPC;
}

// the grouped re-score reads int16 partner rows (written by corr_dnorm)
inline bool q16_rows() { return krca::tuning().corr_rs_q16 && krca::tuning().corr_rs_group; }
// ... and tries the projection bound before them (KRCA_CORR_PROJ: 2 = always, the default since R7d;
// 1 = when the main pass runs in more than one batch; 0 = never).  The projections cost ~1 ms at C3
// (100k pods, one batch): beside the main pass they slowed it by about as much as they saved on the
// re-score after it (R6e-g), so round 6 kept them for several batches only; krca_corr_topk now
// launches them on the side stream beside the threshold sample instead (launch_proj), where they
// slow nothing on the critical path: C3 21.85 -> ~21.3 ms, the re-score 5.8 -> 4.3 ms (R7d).
inline bool proj_bound(int64_t n_batches) {
  const int m = krca::tuning().corr_proj;
  return krca::tuning().corr_rs_group && (m == 2 || (m == 1 && n_batches > 1));
}

// exact |r| > tau counts of the ambiguous pairs in list l (float64 from z32), added to count
int launch_rescore(const float* z32, const Dims& d, const CorrWs& ws, int l, int32_t* count, hipStream_t st,
                   bool use_proj) {
  const float acc_err = (float)(std::ldexp((double)d.T, -24) + std::ldexp(std::sqrt((double)d.T), -23));
  const unsigned grid = (unsigned)std::max(8, krca::tuning().corr_rs_grid & ~7);
  const int16_t* zq = q16_rows() ? ws.zq : nullptr;
  const size_t lds = (size_t)RS_WAVES * (zq ? ws.Tq / 4 : (d.T + 3) / 4) * sizeof(float4);
  // grouped by row pod (above); its offsets are int32 (a list of up to 2^31 - 1 entries)
  if (krca::tuning().corr_rs_group && lds <= 64 * 1024 && d.P > 0 && ws.amb_cap < (int64_t(1) << 31)) {
    const int64_t nb = krca::ceil_div(d.P, GSCAN);
    KRCA_HIP(hipMemsetAsync(ws.gcnt, 0, (size_t)d.P * sizeof(int32_t), st));
    hipLaunchKernelGGL(corr_amb_hist, dim3(grid), dim3(TPB), 0, st, (const int2*)ws.amb[l],
                       (const unsigned long long*)(ws.amb_n + l), ws.amb_cap, ws.gcnt);
    KRCA_LAUNCH_CHECK();
    hipLaunchKernelGGL(corr_scan_blocks, dim3((unsigned)nb), dim3(TPB), 0, st, (const int32_t*)ws.gcnt, d.P, ws.gsum);
    KRCA_LAUNCH_CHECK();
    hipLaunchKernelGGL(corr_scan_top, dim3(1), dim3(TPB), 0, st, ws.gsum, nb);
    KRCA_LAUNCH_CHECK();
    hipLaunchKernelGGL(corr_scan_apply, dim3((unsigned)nb), dim3(TPB), 0, st, (const int32_t*)ws.gcnt, d.P,
                       (const int32_t*)ws.gsum, ws.goff, ws.gcur);
    KRCA_LAUNCH_CHECK();
    hipLaunchKernelGGL(corr_amb_scatter, dim3(grid), dim3(TPB), 0, st, (const int2*)ws.amb[l], (const float*)ws.ambv[l],
                       (const unsigned long long*)(ws.amb_n + l), ws.amb_cap, ws.gcur, ws.gs);
    KRCA_LAUNCH_CHECK();
    // KRCA_CORR_RSG_GRID caps the grouped kernel's workgroups (default 2048): a CU holding one of them
    // (23 KB of LDS at T = 1440) still fits a main-pass tile workgroup, more do not
    const int cap = krca::tuning().corr_rsg_grid > 0 ? krca::tuning().corr_rsg_grid : 2048;
    const unsigned gg = (unsigned)std::min<int64_t>(krca::ceil_div(d.P, RS_WAVES), cap);
    hipLaunchKernelGGL(corr_amb_rescore_grouped, dim3(gg), dim3(TPB), lds, st, (const int32_t*)ws.goff,
                       (const int2*)ws.gs, d.P, z32, (const float*)ws.dn, d.T, d.tau, acc_err, count,
                       zq, ws.Tq, (const float*)ws.qs, (const float*)ws.qn, (const float*)ws.nrm,
                       use_proj ? (const float*)ws.proj : nullptr, (const float*)ws.pqz, (const float*)ws.pqe);
    KRCA_LAUNCH_CHECK();
    return KRCA_OK;
  }
  hipLaunchKernelGGL(corr_amb_rescore, dim3(grid), dim3(TPB), 0, st,
                     (const int2*)ws.amb[l], (const float*)ws.ambv[l], (const unsigned long long*)(ws.amb_n + l),
                     ws.amb_cap, z32, (const float*)ws.dn, d.T, d.tau, acc_err, count);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

// Events of a fork from the caller's stream onto a side stream and the joins back; the destructor
// joins every fork that was made and frees the events on every return path.
struct SideWork {
  hipStream_t st, side;
  hipEvent_t ev[5] = {};  // 0, 1: batch b's list l filled (st); 2, 3: list l drained (side); 4: join
  bool forked = false;
  SideWork(hipStream_t s, hipStream_t sd) : st(s), side(sd) {}
  int init() {
    if (side == st) return KRCA_OK;
    for (hipEvent_t& e : ev) KRCA_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return KRCA_OK;
  }
  ~SideWork() {
    if (side != st) {
      if (forked && ev[4]) {
        (void)hipEventRecord(ev[4], side);
        (void)hipStreamWaitEvent(st, ev[4], 0);
      }
      for (hipEvent_t e : ev)
        if (e) (void)hipEventDestroy(e);
    }
  }
};

// the projection bound's rows (corr_dct_basis, corr_proj) on the side stream, ordered before every
// re-score there; only the re-score reads them
int launch_proj(const uint16_t* zh, const float* z32, const Dims& d, const CorrWs& ws, SideWork& sw) {
  hipStream_t ps = sw.st;
  if (sw.side != sw.st && krca::tuning().corr_side == 0) {  // (every re-score on the side stream)
    KRCA_HIP(hipEventRecord(sw.ev[4], sw.st));  // (ev[4] is re-recorded on the side stream at the join)
    KRCA_HIP(hipStreamWaitEvent(sw.side, sw.ev[4], 0));
    sw.forked = true;
    ps = sw.side;
  }
  hipLaunchKernelGGL(corr_dct_basis, dim3((unsigned)krca::ceil_div((int64_t)KP * d.T, TPB)), dim3(TPB), 0, ps, ws.dct,
                     d.T);
  KRCA_LAUNCH_CHECK();
  hipLaunchKernelGGL(d.T % 4 == 0 ? corr_proj<true> : corr_proj<false>, dim3((unsigned)krca::ceil_div(d.P, PJ_ROWS)),
                     dim3(TPB), 0, ps, z32, zh, d.P, d.T,
                     d.Tp, (const double*)ws.dct, ws.proj, ws.pqz, ws.pqe);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

// the rows' rounding-error norms and int16 copies (corr_dnorm): the main pass and the re-score read them
void launch_dnorm(const uint16_t* zh, const float* z32, const Dims& d, const CorrWs& ws, hipStream_t s) {
  hipLaunchKernelGGL(d.T % 4 == 0 ? corr_dnorm<true> : corr_dnorm<false>, dim3((unsigned)krca::ceil_div(d.P, TPB / 64)),
                     dim3(TPB), 0, s, z32, zh, d.P, d.T,
                     d.Tp, ws.dn, q16_rows() ? ws.zq : nullptr, ws.Tq, ws.qs, ws.qn, ws.nrm);
}


// whether rank g of G re-scores with the projection bound (its share of the super-tiles in batches)
inline bool proj_for(const Dims& d, int G, int g) {
  const int64_t n_st_all = n_supertiles(d.nb2);
  const int64_t n_mine0 = n_st_all > g ? (n_st_all - g + G - 1) / G : 0;
  return proj_bound((n_mine0 + sb_batch() - 1) / sb_batch());
}

// 2. upper-triangle tiles (every G-th super-tile from g): appends into ws.buf, tau counts.  The
//    main pass runs in batches of SB super-tiles; after batch b its ambiguous list (b & 1) is
//    re-scored on `sw.side` (the caller's stream itself when no side stream is wanted) while batch
//    b + 1 fills the other list.  count is final on sw.st once sw is destroyed (joined).
//    proj_launched: the caller already launched the projections (krca_corr_topk: beside the sample).
template <int KC>
int stage_tiles(const uint16_t* zh, const float* z32, const Dims& d, int G, int g, const float* phi, const CorrWs& ws,
                int32_t* count, int dbg, SideWork& sw, bool proj_launched = false) {
  hipStream_t st = sw.st;
  if (int rc = set_lds_attr<KC>()) return rc;
  KRCA_HIP(hipMemsetAsync(ws.cnt, 0, (size_t)d.P * sizeof(int32_t), st));
  KRCA_HIP(hipMemsetAsync(count, 0, (size_t)d.P * sizeof(int32_t), st));
  KRCA_HIP(hipMemsetAsync(ws.amb_n, 0, 2 * sizeof(unsigned long long), st));
  const int64_t n_st = n_supertiles(d.nb2);
  const bool persist = krca::tuning().corr_persist != 0;
  if (persist)  // the ticket counters of every batch (a rank runs at most as many as one device)
    KRCA_HIP(hipMemsetAsync(ws.tick, 0, (size_t)8 * krca::ceil_div(n_st, sb_batch()) * sizeof(unsigned), st));
  const int cu_per_xcd = std::max(1, cu_count() / 8);
  const int64_t n_mine = n_st > g ? (n_st - g + G - 1) / G : 0;
  if (n_mine == 0) return KRCA_OK;
  const Shard sh{0, G, g, 0};
  launch_dnorm(zh, z32, d, ws, st);
  KRCA_LAUNCH_CHECK();
  const bool use_proj = proj_for(d, G, g);
  if (use_proj && !proj_launched) {  // (the sharded path: beside the main pass)
    if (int rc = launch_proj(zh, z32, d, ws, sw)) return rc;
  }
  const float acc_err = (float)(std::ldexp((double)d.T, -24) + std::ldexp(std::sqrt((double)d.T), -23));
  // screening counts: certain above tau + eps, decided in the tile by the pair's own bound or
  // re-scored within it (exact counts)
  TileArgs ta{};
  ta.zA = zh;
  ta.zh = zh;
  ta.P = d.P;
  ta.Tp = d.Tp;
  ta.nb2 = d.nb2;
  ta.nsb = d.nsb;
  ta.tau_hi = (float)(d.tau + d.eps);  // (eps carries 1e-6 of slack over the float roundings)
  ta.tau_lo = (float)(d.tau - d.eps);
  ta.tau = d.tau;
  ta.acc_err = acc_err;
  ta.phi = phi;
  ta.buf = ws.buf;
  ta.capc = cand_cap();
  ta.cnt = ws.cnt;
  ta.count = count;
  ta.sh = sh;
  ta.debug = dbg;
  ta.amb_cap = ws.amb_cap;
  ta.dn = ws.dn;
  ta.z32 = z32;
  ta.T = d.T;
  const bool side_ok = sw.side != st;
  const int64_t SB = sb_batch();
  const int side_mode = krca::tuning().corr_side;
  for (int64_t b = 0, s0 = 0; s0 < n_mine; ++b, s0 += SB) {
    // KRCA_CORR_SIDE: 0 every batch's re-score on the side stream (beside the next batch's tiles), 1
    // each on st after its batch, 2 on st except the last batch's (beside the merge chain)
    const bool last = s0 + SB >= n_mine;
    const bool fork = side_ok && (side_mode == 0 || (side_mode == 2 && last));
    const int l = (int)(b & 1) % ws.nlist;
    if (b >= 2 || (b >= 1 && ws.nlist == 1)) {  // list l was drained by the re-score of batch b - nlist
      if (side_ok) KRCA_HIP(hipStreamWaitEvent(st, sw.ev[2 + l], 0));
      KRCA_HIP(hipMemsetAsync(ws.amb_n + l, 0, sizeof(unsigned long long), st));
    }
    ta.amb = ws.amb[l];
    ta.ambv = ws.ambv[l];
    ta.amb_n = ws.amb_n + l;
    ta.st0 = s0;
    ta.st_end = std::min(n_mine, s0 + SB);
    // 256 x 256 tiles, XCD-aware slots
    ta.per_xcd = ((ta.st_end - s0) * SUPER * SUPER + 7) / 8;
    if (persist) {
      ta.tick = ws.tick + 8 * b;
      const int64_t wg_x = std::min<int64_t>(cu_per_xcd, ta.per_xcd);  // workgroups per XCD
      hipLaunchKernelGGL(corr_main_persist<KC>, dim3((unsigned)(8 * wg_x)), dim3(Geo<256>::NTH),
                         Geo<256>::LDS_PERSIST, st, ta);
    } else {
      hipLaunchKernelGGL((corr_tiles<KC, MODE_MAIN, 256>), dim3((unsigned)(8 * ta.per_xcd)), dim3(Geo<256>::NTH),
                         Geo<256>::LDS_BYTES, st, ta);
    }
    KRCA_LAUNCH_CHECK();
    if (dbg != 0) continue;
    if (fork) {
      KRCA_HIP(hipEventRecord(sw.ev[l], st));
      KRCA_HIP(hipStreamWaitEvent(sw.side, sw.ev[l], 0));
      sw.forked = true;
    }
    if (int rc = launch_rescore(z32, d, ws, l, count, fork ? sw.side : st, use_proj)) return rc;
    if (side_ok) KRCA_HIP(hipEventRecord(sw.ev[2 + l], fork ? sw.side : st));
  }
  return KRCA_OK;
}

// 3. per pod of [lo, lo + n): sort, exact re-scoring, top-k, certificate; overflowed pods get the
//    rectangle pass (their rows x every column block against phi2) and a second merge.  Candidates
//    in lbuf [n][CAPC] / lcnt [n] (raw counts).  Synchronises the stream once.
template <int KC>
int stage_merge(const uint16_t* zh, const float* z32, const Dims& d, int64_t lo, int64_t n, const float* phi,
                int2* lbuf, int32_t* lcnt, const CorrWs& ws, int32_t* out_idx, float* out_val, float* cert,
                int dbg, hipStream_t st) {
  if (n == 0) return KRCA_OK;
  if (int rc = set_lds_attr<KC>()) return rc;
  KRCA_HIP(hipMemsetAsync(ws.over, 0, sizeof(int32_t), st));
  KRCA_HIP(hipMemsetAsync(ws.deep, 0, sizeof(int32_t), st));
  KRCA_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(ws.phi2), 0x40400000 /* 3.0f */, (size_t)d.P, st));
  hipLaunchKernelGGL(corr_merge, dim3((unsigned)n), dim3(TPB), 0, st, (const int2*)lbuf, lcnt, phi, z32, d.P, d.T,
                     d.k, d.eps, 0, (const int32_t*)nullptr, ws.phi2, ws.over, out_idx, out_val, cert, lo, ws.deep,
                     cand_cap(), km_extra());
  KRCA_LAUNCH_CHECK();
  int32_t n_over = 0;
  KRCA_HIP(hipMemcpyAsync(&n_over, ws.over, sizeof(int32_t), hipMemcpyDeviceToHost, st));
  KRCA_HIP(hipStreamSynchronize(st));
  auto deep_pass = [&]() -> int {  // pods whose merge left cert <= 0 (device-held list)
    hipLaunchKernelGGL(corr_merge_deep, dim3((unsigned)std::min<int64_t>(n, 2048)), dim3(TPB), 0, st,
                       (const int2*)lbuf, (const int32_t*)lcnt, phi, (const float*)ws.phi2, z32, d.T, d.k, d.eps,
                       (const int32_t*)ws.deep,
                       out_idx, out_val, cert, lo, cand_cap());
    KRCA_LAUNCH_CHECK();
    return KRCA_OK;
  };
  if (dbg != 0) return KRCA_OK;
  if (n_over == 0) return deep_pass();
  const Shard sh{lo, 1, 0, 0};
  for (int64_t r0 = 0; r0 < n_over; r0 += RECT_ROWS) {
    const int64_t nr = std::min<int64_t>(RECT_ROWS, n_over - r0);
    const int64_t npad = krca::ceil_div(nr, TB) * TB;
    hipLaunchKernelGGL(corr_gather_rows, dim3((unsigned)npad), dim3(TPB), 0, st, zh, d.Tp,
                       (const int32_t*)(ws.over + 1 + r0), nr, ws.zs);
    KRCA_LAUNCH_CHECK();
    TileArgs ta{};
    ta.zA = ws.zs;
    ta.zh = zh;
    ta.P = d.P;
    ta.Tp = d.Tp;
    ta.nb2 = d.nb2;
    ta.nsb = d.nsb;
    ta.phi = ws.phi2;
    ta.buf = lbuf;
    ta.capc = cand_cap();
    ta.cnt = lcnt;
    ta.rect_pods = ws.over + 1 + r0;
    ta.n_rect = nr;
    ta.sh = sh;
    ta.n_tiles = npad / TB * d.nb2;
    ta.per_xcd = (ta.n_tiles + 7) / 8;
    hipLaunchKernelGGL((corr_tiles<KC, MODE_RECT, 256>), dim3((unsigned)(8 * ta.per_xcd)), dim3(Geo<256>::NTH),
                       Geo<256>::LDS_BYTES, st, ta);
    KRCA_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(corr_merge, dim3((unsigned)n_over), dim3(TPB), 0, st, (const int2*)lbuf, lcnt,
                     (const float*)ws.phi2, z32, d.P, d.T, d.k, d.eps, 1, (const int32_t*)(ws.over + 1), ws.phi2,
                     ws.over, out_idx, out_val, cert, lo, ws.deep, cand_cap(), km_extra());
  KRCA_LAUNCH_CHECK();
  return deep_pass();
}

template <int KC>
int run_single(const uint16_t* zh, const float* z32, const Dims& d, char* cand, int32_t* count, int32_t* out_idx,
               float* out_val, float* cert, hipStream_t st) {
  CorrWs ws;
  const int64_t head = ws_layout(d.P, d.T, d.Tp, KC, d.P, 0, cand, &ws);
  float* phi = reinterpret_cast<float*>(cand + 4 * head);  // one more [P] after the layout
  const int dbg = debug_mode();
  // every launch below goes to st's device (the side stream is that device's)
  krca::DeviceGuard dg(st);
  if (int rc = dg.status()) return rc;
  // the exact-count re-scores (memory-bound, write count only) and the merge chain (sort, float64
  // top-k re-scoring, rectangle and deep passes: candidate buffers and outputs only) are
  // independent: the re-scores run on a side stream forked from st per main-pass batch (the last
  // one beside the merge chain) and joined back into st when sw goes out of scope.  The
  // projection bound's rows go first on the side stream, beside the threshold sample.
  SideWork sw(st, dbg ? st : krca::side_stream(st));
  if (int rc = sw.init()) return rc;
  const bool proj = dbg == 0 && proj_for(d, 1, 0);
  if (proj)
    if (int rc = launch_proj(zh, z32, d, ws, sw)) return rc;
  if (int rc = stage_sample<KC>(zh, d, 0, d.P, ws, phi, st)) return rc;
  if (int rc = stage_tiles<KC>(zh, z32, d, 1, 0, phi, ws, count, dbg, sw, proj)) return rc;
  return stage_merge<KC>(zh, z32, d, 0, d.P, phi, ws.buf, ws.cnt, ws, out_idx, out_val, cert, dbg, st);
}

int kc_for(int32_t k) { return k <= 8 ? 8 : k <= 12 ? 12 : 16; }  // the smallest list size >= k

}  // namespace

extern "C" {

int64_t krca_corr_pad_rows(int64_t P) { return krca::ceil_div(P, TB) * TB; }
int32_t krca_corr_pad_steps(int32_t T) { return (int32_t)krca::ceil_div(T, BK) * BK; }
// single-device candidate workspace (4-byte words): see ws_layout, then phi [P]
int64_t krca_corr_cand_size(int64_t P, int32_t T, int32_t k) {
  return ws_layout(P, T, krca_corr_pad_steps(T), kc_for(k), P, 0, nullptr, nullptr) + krca::ceil_div(P, 4) * 4;
}
int32_t krca_corr_max_k(void) { return KMAX; }
int32_t krca_corr_cand_cap(void) { return CAPC; }
float krca_corr_eps(int32_t T) {
  return (float)(std::ldexp(1.0, -10) * 1.001 + std::ldexp((double)T, -24) + std::ldexp(std::sqrt((double)T), -23));
}

int krca_corr_prepare(const float* x, int64_t P, int32_t M, int32_t T, int32_t channel, float* mean, float* scale,
                      float* z32, uint16_t* zh, void* stream) {
  KRCA_CHECK_ARG(P > 0 && M > 0 && T > 0 && channel >= 0 && channel < M, "krca_corr_prepare: bad sizes");
  KRCA_CHECK_ARG(x && mean && scale && z32 && zh, "krca_corr_prepare: null pointer");
  const int64_t Pp = krca_corr_pad_rows(P);
  const int Tp = krca_corr_pad_steps(T);
  hipStream_t st = krca::as_stream(stream);
  hipLaunchKernelGGL(corr_stats, dim3((unsigned)krca::ceil_div(P, TPB)), dim3(TPB), 0, st, x, P, M, T, channel, mean,
                     scale);
  KRCA_LAUNCH_CHECK();
  hipLaunchKernelGGL(corr_transpose, dim3((unsigned)(Pp / 64), (unsigned)(Tp / 64)), dim3(TPB), 0, st, x, P, M, T, Tp,
                     channel, mean, scale, z32, zh);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_corr_topk(const uint16_t* zh, const float* z32, int64_t P, int32_t T, int32_t k, double tau, void* cand,
                   int32_t* count, int32_t* out_idx, float* out_val, float* cert, void* stream) {
  KRCA_CHECK_ARG(P > 1 && P <= (int64_t(1) << 22) && T > 0, "krca_corr_topk: P must be in [2, 2^22]");
  KRCA_CHECK_ARG(k >= 1 && k <= KMAX && k < P, "krca_corr_topk: k must be in [1, %d] and < P", KMAX);
  KRCA_CHECK_ARG(tau >= 0.0, "krca_corr_topk: tau must be >= 0");
  KRCA_CHECK_ARG(zh && z32 && cand && count && out_idx && out_val && cert, "krca_corr_topk: null pointer");
  const Dims d = dims_of(P, T, k, tau);
  hipStream_t st = krca::as_stream(stream);
  char* c = reinterpret_cast<char*>(cand);
  switch (kc_for(k)) {
    case 8: return run_single<8>(zh, z32, d, c, count, out_idx, out_val, cert, st);
    case 12: return run_single<12>(zh, z32, d, c, count, out_idx, out_val, cert, st);
    default: return run_single<16>(zh, z32, d, c, count, out_idx, out_val, cert, st);
  }
}

// ---- pod-sharded correlation (orchestrated by krca/corr_dist.py) -------------
// Rank g owns pods [lo, lo + n_loc) (lo a multiple of 256).  Every rank holds the all-gathered
// zh / z32 and phi.  Per run: shard_sample (phi of own pods) -> all-gather phi -> shard_tiles
// (every G-th super-tile; candidates of ANY pod) -> all-reduce count and raw_cnt -> pack_sizes /
// pack -> all-to-all by owner -> unpack -> shard_merge (own pods; may run the rectangle pass).
int64_t krca_corr_shard_ws_size(int64_t P, int32_t T, int32_t k, int64_t n_loc, int32_t G) {
  return ws_layout(P, T, krca_corr_pad_steps(T), kc_for(k), n_loc, G, nullptr, nullptr);
}

#define KRCA_CORR_SHARD_ARGS(name)                                                                        \
  KRCA_CHECK_ARG(P > 1 && P <= (int64_t(1) << 22) && T > 0 && k >= 1 && k <= KMAX && k < P,               \
                 name ": bad sizes");                                                                      \
  KRCA_CHECK_ARG(n_loc >= 0 && G >= 1 && ws, name ": bad shard arguments");                                \
  CorrWs w;                                                                                                \
  ws_layout(P, T, krca_corr_pad_steps(T), kc_for(k), n_loc, G, reinterpret_cast<char*>(ws), &w);             \
  hipStream_t st = krca::as_stream(stream);

int krca_corr_shard_sample(const uint16_t* zh, int64_t P, int32_t T, int32_t k, int64_t lo, int64_t n_loc, int32_t G,
                           void* ws, float* phi, void* stream) {
  KRCA_CORR_SHARD_ARGS("krca_corr_shard_sample")
  if (n_loc == 0) return KRCA_OK;
  KRCA_CHECK_ARG(zh && phi && lo % TB == 0 && lo + n_loc <= P, "krca_corr_shard_sample: bad range");
  const Dims d = dims_of(P, T, k, 0.f);
  switch (kc_for(k)) {
    case 8: return stage_sample<8>(zh, d, lo, n_loc, w, phi, st);
    case 12: return stage_sample<12>(zh, d, lo, n_loc, w, phi, st);
    default: return stage_sample<16>(zh, d, lo, n_loc, w, phi, st);
  }
}

int krca_corr_shard_tiles(const uint16_t* zh, const float* z32, int64_t P, int32_t T, int32_t k, double tau, int32_t G,
                          int32_t g, const float* phi, int64_t n_loc, void* ws, int32_t* count, int32_t* raw_cnt,
                          void* stream) {
  KRCA_CORR_SHARD_ARGS("krca_corr_shard_tiles")
  KRCA_CHECK_ARG(zh && z32 && phi && count && raw_cnt && g >= 0 && g < G && tau >= 0.0,
                 "krca_corr_shard_tiles: bad args");
  const Dims d = dims_of(P, T, k, tau);
  int rc;
  {
    SideWork sw(st, st);  // the counts are all-reduced next: re-scores in order on st
    switch (kc_for(k)) {
      case 8: rc = stage_tiles<8>(zh, z32, d, G, g, phi, w, count, 0, sw); break;
      case 12: rc = stage_tiles<12>(zh, z32, d, G, g, phi, w, count, 0, sw); break;
      default: rc = stage_tiles<16>(zh, z32, d, G, g, phi, w, count, 0, sw);
    }
  }
  if (rc) return rc;
  KRCA_HIP(hipMemcpyAsync(raw_cnt, w.cnt, (size_t)P * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
  return KRCA_OK;
}

// entries (int4 {pod, partner, r bits, 0}) this rank sends to each owner; synchronises the stream
int krca_corr_shard_pack_sizes(int64_t P, int32_t T, int32_t k, int64_t n_loc, int32_t G, int64_t n_max, void* ws,
                               int64_t* tot_host, void* stream) {
  KRCA_CORR_SHARD_ARGS("krca_corr_shard_pack_sizes")
  KRCA_CHECK_ARG(tot_host && n_max > 0 && n_max * G >= P, "krca_corr_shard_pack_sizes: bad args");
  KRCA_HIP(hipMemsetAsync(w.xc, 0, 3 * (size_t)G * sizeof(unsigned long long), st));
  hipLaunchKernelGGL(corr_pack_count, dim3((unsigned)krca::ceil_div(P, TPB)), dim3(TPB), 0, st, (const int32_t*)w.cnt,
                     P, n_max, w.xc, cand_cap());
  KRCA_LAUNCH_CHECK();
  std::vector<unsigned long long> tot(G), off(G);
  KRCA_HIP(hipMemcpyAsync(tot.data(), w.xc, G * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
  KRCA_HIP(hipStreamSynchronize(st));
  unsigned long long acc = 0;
  for (int h = 0; h < G; ++h) {
    off[h] = acc;
    acc += tot[h];
    tot_host[h] = (int64_t)tot[h];
  }
  KRCA_HIP(hipMemcpyAsync(w.xc + G, off.data(), G * sizeof(unsigned long long), hipMemcpyHostToDevice, st));
  KRCA_HIP(hipStreamSynchronize(st));  // off[] is a stack copy
  return KRCA_OK;
}

int krca_corr_shard_pack(int64_t P, int32_t T, int32_t k, int64_t n_loc, int32_t G, int64_t n_max, void* ws,
                         void* send, void* stream) {
  KRCA_CORR_SHARD_ARGS("krca_corr_shard_pack")
  KRCA_CHECK_ARG(send && n_max > 0, "krca_corr_shard_pack: bad args");
  hipLaunchKernelGGL(corr_pack, dim3((unsigned)krca::ceil_div(P, TPB / 64)), dim3(TPB), 0, st, (const int32_t*)w.cnt,
                     (const int2*)w.buf, P, n_max, (const unsigned long long*)(w.xc + G), w.xc + 2 * G,
                     reinterpret_cast<int4*>(send), cand_cap());
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_corr_shard_unpack(int64_t P, int32_t T, int32_t k, int64_t n_loc, int32_t G, int64_t lo, void* ws,
                           const void* recv, int64_t n_recv, void* stream) {
  KRCA_CORR_SHARD_ARGS("krca_corr_shard_unpack")
  KRCA_CHECK_ARG(n_recv >= 0 && (recv || n_recv == 0), "krca_corr_shard_unpack: bad args");
  KRCA_HIP(hipMemsetAsync(w.fill, 0, (size_t)std::max<int64_t>(n_loc, 1) * sizeof(int32_t), st));
  if (n_recv == 0) return KRCA_OK;
  hipLaunchKernelGGL(corr_unpack, dim3((unsigned)krca::ceil_div(n_recv, TPB)), dim3(TPB), 0, st,
                     reinterpret_cast<const int4*>(recv), n_recv, lo, w.fill, w.lbuf, cand_cap());
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

// own pods: lcnt = this rank's slice of the all-reduced raw counts ([n_loc], may be reset here)
int krca_corr_shard_merge(const uint16_t* zh, const float* z32, int64_t P, int32_t T, int32_t k, double tau,
                          int64_t lo, int64_t n_loc, int32_t G, const float* phi, int32_t* lcnt, void* ws,
                          int32_t* out_idx, float* out_val, float* cert, void* stream) {
  KRCA_CORR_SHARD_ARGS("krca_corr_shard_merge")
  KRCA_CHECK_ARG(zh && z32 && phi && lcnt && out_idx && out_val && cert && lo + n_loc <= P,
                 "krca_corr_shard_merge: bad args");
  const Dims d = dims_of(P, T, k, tau);
  switch (kc_for(k)) {
    case 8: return stage_merge<8>(zh, z32, d, lo, n_loc, phi, w.lbuf, lcnt, w, out_idx, out_val, cert, 0, st);
    case 12: return stage_merge<12>(zh, z32, d, lo, n_loc, phi, w.lbuf, lcnt, w, out_idx, out_val, cert, 0, st);
    default: return stage_merge<16>(zh, z32, d, lo, n_loc, phi, w.lbuf, lcnt, w, out_idx, out_val, cert, 0, st);
  }
}
#undef KRCA_CORR_SHARD_ARGS

}  // extern "C"

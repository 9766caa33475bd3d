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
//                      128 rows / 64 steps).  |z| <= 1 (unit-norm rows), so fp16 keeps 11 bits.
//   krca_corr_tiles    MFMA (v_mfma_f32_32x32x16_f16, fp32 accumulation) over the UPPER triangle
//                      of 128x128 tiles only (P(P+1)/2 pairs, the algorithmic flop count), in an
//                      XCD-aware super-tile order, LDS double-buffered with register prefetch.
//                      Epilogue in LDS: each lane scans one row (-> candidates of that row from
//                      this column block) or one column (-> the symmetric candidates of that
//                      column's pod from this row block), keeping the KC best by |r|; |r| > tau
//                      counts go out as one int32 add per row/column and tile.
//   krca_corr_merge    one workgroup per pod: best KM of its nb*KC candidates, re-scored in
//                      float64 from z32 (fixed-order wave reduction), final top-k; cert[p] =
//                      (k-th re-scored |r|) - (best |r| the tiles could have dropped) - eps:
//                      cert > 0 proves the reported set equals the exact top-k.
//
// Error bound of the screening product (eps, host-computed): fp16 rounding of unit-norm rows
// moves a dot product by <= 2^-10 (+ 2^-24 sqrt(T) from subnormals), fp32 accumulation of T
// terms of a unit-norm product by <= T 2^-24.  It bounds the ranking pool and the |r| > tau
// counts (pairs within eps of tau may land on either side); reported r values are exact.
#include <cmath>
#include <cstdlib>

#include "krca_common.h"

namespace {

constexpr int TPB = 256;
constexpr int BM = 128;   // tile rows == cols
constexpr int BK = 64;    // K step (time samples)
constexpr int SUPER = 8;  // super-tile edge (tiles) of the XCD-aware order
constexpr int KM = 24;    // candidates re-scored per pod in the merge
constexpr int KMAX = 16;  // largest k served
// KC = candidates kept per (pod, block): a template parameter >= k (so every member of a pod's
// exact top-k survives its own block's cut), with headroom for the certificate: 8, 12 or 16

typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // (HIP's uint4 struct defeats SROA)

__device__ __forceinline__ uint16_t f16_bits(float f) {
  const _Float16 h = (_Float16)f;  // round to nearest even
  return __builtin_bit_cast(uint16_t, h);
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
  float v[KC];  // signed r
  int32_t i[KC];
  float thr;    // |v[KC-1]| (-1 while the list is not full)
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      v[j] = 0.f;
      i[j] = -1;
    }
    thr = -1.f;
  }
  __device__ __forceinline__ void insert(float nv, int32_t ni) {
    const float a = fabsf(nv);
#pragma unroll
    for (int j = KC - 1; j > 0; --j) {
      const bool up = a > fabsf(v[j - 1]) || i[j - 1] < 0;  // shift v[j-1] down
      const bool here = a > fabsf(v[j]) || i[j] < 0;
      const float pv = v[j - 1];
      const int32_t pi = i[j - 1];
      v[j] = up ? pv : (here ? nv : v[j]);
      i[j] = up ? pi : (here ? ni : i[j]);
    }
    if (a > fabsf(v[0]) || i[0] < 0) {
      v[0] = nv;
      i[0] = ni;
    }
    thr = i[KC - 1] < 0 ? -1.f : fabsf(v[KC - 1]);
  }
};

// Tile kernel: 256 x 256 pods per workgroup (8 waves = 2 row halves x 4 column quarters, a
// 128 x 64 wave tile = 4 x 2 MFMA 32x32 blocks), K steps of 64 through a double-buffered LDS
// stage (A and B 256 x 64 fp16 each) fed by a register prefetch.  Candidate lists keep the
// 128-pod block granularity: a row's list covers one 128-column half of the tile, a column's list
// one 128-row half.
constexpr int TB = 256;                                // tile edge (pods)
constexpr int NT = 512;                                // threads per tile workgroup
constexpr int STAGE_BYTES = 2 * TB * BK * 2;           // A and B, fp16
constexpr int LDS_STAGE = 2 * STAGE_BYTES;             // double buffered: 128 KB
constexpr int EPI_LD = TB + 4;  // padded row of the epilogue half tile (16-B rows; conflict-free b128 row reads)
constexpr int LDS_EPI = BM * EPI_LD * 4;               // 128 rows x 256 columns fp32
constexpr int LDS_MAIN = LDS_STAGE > LDS_EPI ? LDS_STAGE : LDS_EPI;
constexpr int LDS_JUNK = NT * 4;                       // landing slots of the L2 prefetch loads
constexpr int LDS_BYTES = LDS_MAIN + LDS_JUNK;

// 16-byte chunk c (0..7) of row r of a [rows][64] fp16 stage, XOR-swizzled against bank conflicts
// (the XOR key (r >> 1) & 7 makes every 16-lane ds_read_b128 phase of 16 rows hit 16 distinct
// 4-bank granules: row parity picks the 32-bank half, the key the granule inside it)
__device__ __forceinline__ int chunk_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

// SAMPLE = false: the upper triangle of 256-blocks (all pairs), lists filtered by phi, heads and
//                 |r| > tau counts out.
// SAMPLE = true:  rows x the first nsb 128-column blocks (the threshold sample), row lists only.
template <int KC, bool SAMPLE>
__global__ __launch_bounds__(NT) void corr_tiles(const uint16_t* __restrict__ zh, int64_t P, int Tp, int nb2,
                                                 int64_t per_xcd, int nsb, float tau, const float* __restrict__ phi,
                                                 float* __restrict__ cand_v, int32_t* __restrict__ cand_i,
                                                 float* __restrict__ cand_hd, int32_t* __restrict__ count,
                                                 int debug) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nb = 2 * nb2;  // 128-pod blocks
  int64_t I, J;
  if (SAMPLE) {
    const int nsb2 = (nsb + 1) / 2;
    I = blockIdx.x / nsb2;
    J = blockIdx.x % nsb2;
  } else {
    // XCD-aware order: workgroups are dispatched round-robin over the 8 XCDs, so slot
    // L = (b % 8) * per_xcd + b / 8 gives each XCD a contiguous run of slots; slots walk the
    // upper triangle in SUPER x SUPER super-tiles, so the tiles an XCD has in flight share 2*SUPER
    // row blocks through its L2.  Slots below the diagonal or past nb2 exit at once.
    const int64_t b = blockIdx.x;
    const int64_t L = (b & 7) * per_xcd + (b >> 3);
    const int64_t ns = (nb2 + SUPER - 1) / SUPER;
    const int64_t st = L / (SUPER * SUPER);
    if (st >= ns * (ns + 1) / 2) return;
    int64_t SJ = (int64_t)((sqrt(8.0 * (double)st + 1.0) - 1.0) * 0.5);
    while ((SJ + 1) * (SJ + 2) / 2 <= st) ++SJ;
    while (SJ * (SJ + 1) / 2 > st) --SJ;
    const int64_t SI = st - SJ * (SJ + 1) / 2;
    const int64_t in = L % (SUPER * SUPER);
    I = SI * SUPER + in / SUPER;
    J = SJ * SUPER + in % SUPER;
    if (I > J || J >= nb2) return;
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 2, wc = w & 3;
  const int64_t rowA = I * TB, rowB = J * TB;

  floatx16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // Staging: global -> LDS direct (global_load_lds_dwordx4, no VGPR round trip).  One wave
  // instruction writes a lane-linear 1 KiB piece = 8 rows of 128 B; lane l lands on row l/8,
  // slot l%8, so it fetches the global chunk (l%8) ^ key(row): the XOR swizzle is applied on the
  // SOURCE address.  64 pieces per K step (32 A + 32 B), 8 per wave.
  const uint16_t* gA = zh + rowA * Tp;
  const uint16_t* gB = zh + rowB * Tp;
  const int prow = lane >> 3, pslot = lane & 7;
#define CORR_GLDS(BUF, K0)                                                                             \
  _Pragma("unroll") for (int q = 0; q < 4; ++q) {                                                      \
    const int piece = w + 8 * q;      /* rows 8*piece .. +7 */                                         \
    const int row = 8 * piece + prow;                                                                  \
    const int64_t src = (int64_t)row * Tp + (K0) + ((pslot ^ ((row >> 1) & 7)) << 3);                 \
    char* dA = smem + (BUF) * STAGE_BYTES + piece * 1024;                                              \
    __builtin_amdgcn_global_load_lds(gA + src, (__attribute__((address_space(3))) void*)dA, 16, 0, 0); \
    __builtin_amdgcn_global_load_lds(gB + src, (__attribute__((address_space(3))) void*)(dA + TB * BK * 2), \
                                     16, 0, 0);                                                       \
  }
  const int r32 = lane & 31, h = lane >> 5;
#define CORR_COMPUTE(BUF)                                                                         \
  {                                                                                                \
    const char* sA = smem + (BUF) * STAGE_BYTES;                                                   \
    const char* sB = sA + TB * BK * 2;                                                             \
    _Pragma("unroll") for (int ks = 0; ks < BK / 16; ++ks) {                                       \
      const int c = ks * 2 + h;                                                                    \
      halfx8 fa[4], fb[2];                                                                         \
      _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                \
        fa[i] = *reinterpret_cast<const halfx8*>(sA + chunk_off(wr * 128 + i * 32 + r32, c));      \
      _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                \
        fb[j] = *reinterpret_cast<const halfx8*>(sB + chunk_off(wc * 64 + j * 32 + r32, c));       \
      _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                \
        _Pragma("unroll") for (int j = 0; j < 2; ++j)                                              \
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[i], fb[j], acc[i][j], 0, 0, 0);    \
    }                                                                                              \
  }
  // L2 prefetch of K step s+2 while step s+1 streams into LDS: one 4-byte LDS-DMA per 128-B line
  // (lane tid < 256: A row tid, else B row tid-256) into a junk LDS slot, so no VGPR is tied up;
  // step s+2's 16-byte loads then hit L2 instead of paying the HBM/MALL latency inside one
  // K step's compute.  The barrier waits vmcnt(1): the stage loads, issued before it, are done.
  const uint16_t* gP = (tid < TB ? gA + (int64_t)tid * Tp : gB + (int64_t)(tid - TB) * Tp);
  char* junk = smem + LDS_MAIN + w * 256;
#define CORR_L2PF(K0) \
  __builtin_amdgcn_global_load_lds(gP + (K0), (__attribute__((address_space(3))) void*)junk, 4, 0, 0);
  const int nk = Tp / BK;
  CORR_GLDS(0, 0)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int s = 0; s < nk; ++s) {
    // stage (s+1)&1 was last read in step s-1, which every wave finished before the barrier
    if (s + 1 < nk) {
      CORR_GLDS((s + 1) & 1, (s + 1) * BK)
    }
    if (s + 2 < nk) {
      CORR_L2PF((s + 2) * BK)
    } else {
      CORR_L2PF(0)  // keeps the count of outstanding loads uniform (re-touches a resident line)
    }
    __builtin_amdgcn_sched_barrier(0);  // issue the loads before the MFMAs, not after
    CORR_COMPUTE(s & 1)
    asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#undef CORR_GLDS
#undef CORR_COMPUTE
#undef CORR_L2PF
  // epilogue, one 128-row half at a time: the half's waves park their accumulators in LDS, then
  // 256 lanes scan rows (one 128-column half each) and 256 lanes scan columns (128 rows each)
  float* tile = reinterpret_cast<float*>(smem);
  const bool diag = I == J;
  if (debug == 1) {  // profiling aid (KRCA_CORR_DEBUG=1): product only, no epilogue
    if (tid == 0 && acc[0][0][0] == 12345.f) count[0] = 1;
    return;
  }
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    if (wr == half) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int row = i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
            const int col = wc * 64 + j * 32 + r32;
            tile[row * EPI_LD + col] = acc[i][j][e];
          }
    }
    __syncthreads();
    Cand<KC> cd;
    cd.init();
    int n_over = 0;
    int64_t g = -1, slot = 0;
    bool write = false;
    if (tid < 256) {  // row scan: pod rowA + half*128 + r against 128 columns of block 2J + ch
      const int r = tid & 127, ch = tid >> 7;
      g = rowA + half * BM + r;
      const int jb = 2 * (int)J + ch;
      const int64_t c0 = rowB + ch * BM;
      if (g < P && (!SAMPLE || jb < nsb)) {
        write = true;
        slot = SAMPLE ? g * 16 + jb : g * nb + jb;
        const float ph = SAMPLE ? -1.f : phi[g];
        float lim = ph;  // = max(list floor, phi), refreshed on insert
        const int cend = (int)std::min<int64_t>(BM, P - c0);
        const int self = (g >= c0 && g < c0 + BM) ? (int)(g - c0) : -1;
        const float* rowp = tile + r * EPI_LD + ch * BM;
        for (int c4 = 0; c4 < cend; c4 += 4) {
          const float4 q4 = *reinterpret_cast<const float4*>(rowp + c4);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int c = c4 + u;
            const float vu = u == 0 ? q4.x : u == 1 ? q4.y : u == 2 ? q4.z : q4.w;
            const float a = fabsf(vu);
            const bool ok = c < cend && c != self;
            n_over += (ok && a > tau) ? 1 : 0;
            if (ok && a > lim) {
              cd.insert(vu, (int32_t)(c0 + c));
              lim = fmaxf(cd.thr, ph);
            }
          }
        }
      }
    } else if (!SAMPLE && !diag) {  // column scan: pod rowB + c against the 128 rows of this half
      const int c = tid - 256;
      g = rowB + c;
      const int ib = 2 * (int)I + half;
      const int64_t r0 = rowA + half * BM;
      if (g < P) {
        write = true;
        slot = g * nb + ib;
        const float ph = phi[g];
        float lim = ph;
        const int rend = (int)std::min<int64_t>(BM, P - r0);
        for (int r = 0; r < rend; ++r) {
          const float v = tile[r * EPI_LD + c];
          const float a = fabsf(v);
          n_over += a > tau ? 1 : 0;
          if (a > lim) {
            cd.insert(v, (int32_t)(r0 + r));
            lim = fmaxf(cd.thr, ph);
          }
        }
      }
    }
    if (write) {
      if (SAMPLE || cd.i[0] >= 0) {  // empty main-pass lists are never read (head = -1)
        float* ov = cand_v + slot * KC;
        int32_t* oi = cand_i + slot * KC;
#pragma unroll
        for (int q = 0; q < KC; ++q) {
          ov[q] = cd.v[q];
          oi[q] = cd.i[q];
        }
      }
      if (!SAMPLE) {
        // list head (best |r|, -1 if empty) and floor (KC-th |r| if the list is full, else -1)
        cand_hd[slot * 2] = cd.i[0] < 0 ? -1.f : fabsf(cd.v[0]);
        cand_hd[slot * 2 + 1] = cd.thr;
        if (n_over) atomicAdd(&count[g], n_over);
      }
    }
    __syncthreads();  // the next half overwrites the tile
  }
}

// phi[g] = (k-th best |r| of g among the sampled partners) - 2 eps (-1 if fewer than k): every
// member of g's exact top-k has a screening |r| above it (exact k-th >= sampled k-th - eps).
template <int KC>
__global__ __launch_bounds__(TPB) void corr_theta(const float* __restrict__ sv, const int32_t* __restrict__ si,
                                                  int64_t P, int nsb, int k, float eps, float* __restrict__ phi) {
  const int64_t g = (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (g >= P) return;
  const int n = nsb * KC;  // <= 256; sample lists are [P][16][KC]
  float a[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int q = lane + 64 * u;
    const int64_t e = g * 16 * KC + q;
    a[u] = (q < n && si[e] >= 0) ? fabsf(sv[e]) : -1.f;
  }
  float kth = -1.f;
  for (int r = 0; r < k; ++r) {
    float m = fmaxf(fmaxf(a[0], a[1]), fmaxf(a[2], a[3]));
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    kth = m;
    if (m < 0.f) break;
    // remove one instance of m: the lowest lane holding it, its first slot
    const bool has = a[0] == m || a[1] == m || a[2] == m || a[3] == m;
    const uint64_t bal = __ballot(has);
    if (lane == __ffsll((unsigned long long)bal) - 1) {
      if (a[0] == m) a[0] = -1.f;
      else if (a[1] == m) a[1] = -1.f;
      else if (a[2] == m) a[2] = -1.f;
      else a[3] = -1.f;
    }
  }
  if (lane == 0) phi[g] = kth < 0.f ? -1.f : kth - 2.f * eps - 1e-6f;
}

// ---- merge + exact re-scoring ------------------------------------------------------------------
__device__ __forceinline__ bool cbetter(float a, int32_t ia, float b, int32_t ib) {
  if (ib < 0) return ia >= 0;
  if (ia < 0) return false;
  const float fa = fabsf(a), fb = fabsf(b);
  return fa > fb || (fa == fb && ia < ib);
}

struct Pool {  // sorted (|r| desc, index asc) list of KM + 1
  float v[KM + 1];
  int32_t i[KM + 1];
  __device__ __forceinline__ void insert(float nv, int32_t ni) {
    if (!cbetter(nv, ni, v[KM], i[KM])) return;
#pragma unroll
    for (int j = KM; j > 0; --j) {
      const bool up = cbetter(nv, ni, v[j - 1], i[j - 1]);
      const bool here = cbetter(nv, ni, v[j], i[j]);
      const float pv = v[j - 1];
      const int32_t pi = i[j - 1];
      v[j] = up ? pv : (here ? nv : v[j]);
      i[j] = up ? pi : (here ? ni : i[j]);
    }
    if (cbetter(nv, ni, v[0], i[0])) {
      v[0] = nv;
      i[0] = ni;
    }
  }
};

constexpr int CAP = 2048;  // merge: candidates collected above the head threshold (else fallback)

// theta = the (KM+1)-th largest list head (bitonic sort of the nb <= 4096 heads in LDS), or 0
// when fewer than KM+1 lists are non-empty: at least KM+1 candidates are >= theta, so the best
// KM+1 candidates all are.
__device__ float head_threshold(const float* __restrict__ hd, int nb, float* key) {
  const int tid = threadIdx.x;
  int np = 64;
  while (np < nb) np <<= 1;
  for (int i = tid; i < np; i += TPB) key[i] = i < nb ? hd[2 * i] : -1.f;  // empty lists: -1
  __syncthreads();
  for (int kk = 2; kk <= np; kk <<= 1) {
    for (int j = kk >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < np; i += TPB) {
        const int l = i ^ j;
        if (l > i) {
          const float a = key[i], c = key[l];
          if ((a < c) == ((i & kk) == 0)) {  // descending runs first
            key[i] = c;
            key[l] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  const float t = key[KM];
  __syncthreads();
  return t < 0.f ? 0.f : t;
}

template <int KC>
__global__ __launch_bounds__(TPB) void corr_merge(const float* __restrict__ cand_v, const int32_t* __restrict__ cand_i,
                                                  const float* __restrict__ cand_hd, const float* __restrict__ phi,
                                                  const float* __restrict__ z32, int64_t P, int T, int nb, int k,
                                                  float eps,
                                                  int32_t* __restrict__ out_i, float* __restrict__ out_v,
                                                  float* __restrict__ cert) {
  __shared__ int hist[4096];  // the sorted list heads, then the collected candidates (v, i)
  __shared__ int lid[4096];   // lists whose head is >= theta
  __shared__ int n_lists;
  __shared__ int ord[KM];
  __shared__ float sv[TPB / 64];
  __shared__ int32_t si[TPB / 64];
  __shared__ float top_v[KM + 1];
  __shared__ int32_t top_i[KM + 1];
  __shared__ double exact[KM];
  __shared__ int n_col;
  const int64_t g = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t base = g * nb * KC;
  const float* hd = cand_hd + g * nb * 2;
  // largest |r| any full per-block list could have cut off
  float floor_ = 0.f;
  for (int b = tid; b < nb; b += TPB) floor_ = fmaxf(floor_, hd[2 * b + 1]);
  for (int off = 32; off > 0; off >>= 1) floor_ = fmaxf(floor_, __shfl_xor(floor_, off, 64));
  if (lane == 0) sv[w] = floor_;
  __syncthreads();
  floor_ = fmaxf(fmaxf(sv[0], sv[1]), fmaxf(sv[2], sv[3]));
  const float theta = head_threshold(hd, nb, reinterpret_cast<float*>(hist));
  // collect every candidate >= theta (lists are sorted, so a list is read only while >= theta)
  float* cv = reinterpret_cast<float*>(hist);
  int32_t* ci = hist + CAP;
  if (tid == 0) {
    n_col = 0;
    n_lists = 0;
  }
  __syncthreads();
  for (int b = tid; b < nb; b += TPB)
    if (hd[2 * b] >= theta && hd[2 * b] >= 0.f) lid[atomicAdd(&n_lists, 1)] = b;
  __syncthreads();
  const int nl = n_lists;
  for (int item = tid; item < nl * KC; item += TPB) {  // every (list, entry): independent loads
    const int64_t e = base + (int64_t)lid[item / KC] * KC + item % KC;
    const int32_t id = cand_i[e];
    const float v = cand_v[e];
    if (id >= 0 && fabsf(v) >= theta) {
      const int slot = atomicAdd(&n_col, 1);
      if (slot < CAP) {
        cv[slot] = v;
        ci[slot] = id;
      }
    }
  }
  __syncthreads();
  const int n = n_col;
  if (n <= CAP) {
    // bitonic sort of the collected candidates (|r| desc, index asc; padding last)
    int np = 32;
    while (np < n) np <<= 1;
    for (int i = n + tid; i < np; i += TPB) {
      cv[i] = 0.f;
      ci[i] = -1;
    }
    __syncthreads();
    for (int kk = 2; kk <= np; kk <<= 1) {
      for (int j = kk >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < np; i += TPB) {
          const int l = i ^ j;
          if (l > i) {
            const bool desc = (i & kk) == 0;
            const bool lbetter = cbetter(cv[l], ci[l], cv[i], ci[i]);
            if (lbetter == desc) {
              const float tv = cv[i];
              const int32_t ti = ci[i];
              cv[i] = cv[l];
              ci[i] = ci[l];
              cv[l] = tv;
              ci[l] = ti;
            }
          }
        }
        __syncthreads();
      }
    }
    if (tid <= KM) {
      top_v[tid] = tid < np ? cv[tid] : 0.f;
      top_i[tid] = tid < np ? ci[tid] : -1;
    }
  } else {
    // fallback (ties at the threshold, e.g. a flat series): per-lane pools over every candidate
    Pool c;
#pragma unroll
    for (int j = 0; j <= KM; ++j) {
      c.v[j] = 0.f;
      c.i[j] = -1;
    }
    for (int64_t q = tid; q < (int64_t)nb * KC; q += TPB) {
      const int32_t id = cand_i[base + q];
      if (id >= 0) c.insert(cand_v[base + q], id);
    }
    for (int r = 0; r <= KM; ++r) {  // block-wide extraction, one winner per round
      float bv = c.v[0];
      int32_t bi = c.i[0];
      for (int off = 32; off > 0; off >>= 1) {
        const float ov = __shfl_xor(bv, off, 64);
        const int32_t oi = __shfl_xor(bi, off, 64);
        if (cbetter(ov, oi, bv, bi)) {
          bv = ov;
          bi = oi;
        }
      }
      if (lane == 0) {
        sv[w] = bv;
        si[w] = bi;
      }
      __syncthreads();
      float wv = sv[0];
      int32_t wi = si[0];
      for (int q = 1; q < TPB / 64; ++q)
        if (cbetter(sv[q], si[q], wv, wi)) {
          wv = sv[q];
          wi = si[q];
        }
      __syncthreads();
      if (tid == 0) {
        top_v[r] = wv;
        top_i[r] = wi;
      }
      if (wi >= 0 && c.i[0] == wi) {  // each partner sits in exactly one lane's pool
#pragma unroll
        for (int j = 0; j < KM; ++j) {
          c.v[j] = c.v[j + 1];
          c.i[j] = c.i[j + 1];
        }
        c.v[KM] = 0.f;
        c.i[KM] = -1;
      }
    }
  }
  __syncthreads();
  // exact float64 re-scoring of the best km = min(KM, k + 6) (one wave per candidate, fixed
  // reduction order); the certificate bounds everything outside them by the (km+1)-th
  const int km = k + 6 < KM ? k + 6 : KM;
  const float dropped = fmaxf(fmaxf(floor_, phi[g]), top_i[km] >= 0 ? fabsf(top_v[km]) : 0.f);
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
    for (int t = lane; t < T; t += 64) {
      const double a = (double)zg[t];
#pragma unroll
      for (int u = 0; u < PER; ++u)
        if (zj[u]) acc2[u] += a * (double)zj[u][t];
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
    out_i[g * k + q] = top_i[ord[q]];
    out_v[g * k + q] = (float)exact[ord[q]];
  }
  if (tid == 0) cert[g] = (float)(fabs(exact[ord[k - 1]]) - (double)dropped - (double)eps);
}

int debug_mode() {
  static int m = -1;
  if (m < 0) {
    const char* e = getenv("KRCA_CORR_DEBUG");
    m = e ? atoi(e) : 0;
  }
  return m;
}

template <int KC>
int launch_corr(const uint16_t* zh, const float* z32, int64_t P, int T, int Tp, int nb, int nsb, int k, float tau,
                float eps, float* cand_v, int32_t* cand_i, float* cand_hd, float* samp_v, int32_t* samp_i, float* phi,
                int32_t* count, int32_t* out_idx, float* out_val, float* cert, hipStream_t st) {
  static bool lds_attr = false;  // > 64 KB of dynamic LDS needs the opt-in once per kernel
  if (!lds_attr) {
    KRCA_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_tiles<KC, false>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
    KRCA_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_tiles<KC, true>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
    lds_attr = true;
  }
  // 1. threshold sample: every pod against the first nsb column blocks
  const int nb2 = nb / 2;
  hipLaunchKernelGGL((corr_tiles<KC, true>), dim3((unsigned)(nb2 * ((nsb + 1) / 2))), dim3(NT), LDS_BYTES, st, zh, P,
                     Tp, nb2, (int64_t)0, nsb, tau, (const float*)nullptr, samp_v, samp_i, (float*)nullptr,
                     (int32_t*)nullptr, 0);
  KRCA_LAUNCH_CHECK();
  hipLaunchKernelGGL(corr_theta<KC>, dim3((unsigned)krca::ceil_div(P, TPB / 64)), dim3(TPB), 0, st, samp_v, samp_i, P,
                     nsb, k, eps, phi);
  KRCA_LAUNCH_CHECK();
  // 2. all pairs (upper triangle), filtered by phi
  const int64_t ns = (nb2 + SUPER - 1) / SUPER;
  const int64_t slots = ns * (ns + 1) / 2 * SUPER * SUPER;
  const int64_t per_xcd = (slots + 7) / 8;
  hipLaunchKernelGGL((corr_tiles<KC, false>), dim3((unsigned)(8 * per_xcd)), dim3(NT), LDS_BYTES, st, zh, P, Tp, nb2,
                     per_xcd, nsb, tau, (const float*)phi, cand_v, cand_i, cand_hd, count, debug_mode());
  KRCA_LAUNCH_CHECK();
  // 3. per pod: pool, exact re-scoring, top-k, certificate
  hipLaunchKernelGGL(corr_merge<KC>, dim3((unsigned)P), dim3(TPB), 0, st, cand_v, cand_i, cand_hd, phi, z32, P, T, nb,
                     k, eps, out_idx, out_val, cert);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int kc_for(int32_t k) { return k <= 4 ? 8 : k <= 8 ? 12 : 16; }

}  // namespace

extern "C" {

int64_t krca_corr_pad_rows(int64_t P) { return krca::ceil_div(P, TB) * TB; }
int32_t krca_corr_pad_steps(int32_t T) { return (int32_t)krca::ceil_div(T, BK) * BK; }
constexpr int NSB = 16;  // column blocks in the threshold sample (2048 pods)
// candidate workspace (4-byte words): values and indices [P][nb][KC] each, heads [P][nb][2],
// sample lists [P][nsb][KC] x 2, phi [P]
int64_t krca_corr_cand_size(int64_t P, int32_t k) {
  const int64_t nb = krca_corr_pad_rows(P) / BM;
  return P * nb * (2 * kc_for(k) + 2) + P * NSB * 2 * kc_for(k) + P;
}
int32_t krca_corr_max_k(void) { return KMAX; }
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

int krca_corr_topk(const uint16_t* zh, const float* z32, int64_t P, int32_t T, int32_t k, float tau, void* cand,
                   int32_t* count, int32_t* out_idx, float* out_val, float* cert, void* stream) {
  KRCA_CHECK_ARG(P > 1 && krca_corr_pad_rows(P) <= 4096 * BM && T > 0,
                 "krca_corr_topk: P must be in [2, %d]", 4096 * BM);
  KRCA_CHECK_ARG(k >= 1 && k <= KMAX && k < P, "krca_corr_topk: k must be in [1, %d] and < P", KMAX);
  KRCA_CHECK_ARG(zh && z32 && cand && count && out_idx && out_val && cert, "krca_corr_topk: null pointer");
  const int64_t Pp = krca_corr_pad_rows(P);
  const int Tp = krca_corr_pad_steps(T);
  const int nb = (int)(Pp / BM);
  const float eps = krca_corr_eps(T);
  const int nsb = nb < NSB ? nb : NSB;
  const int KCr = kc_for(k);
  const int64_t lists = P * nb;
  float* cand_v = reinterpret_cast<float*>(cand);
  int32_t* cand_i = reinterpret_cast<int32_t*>(cand_v + lists * KCr);
  float* cand_hd = reinterpret_cast<float*>(cand_i + lists * KCr);
  float* samp_v = cand_hd + lists * 2;
  int32_t* samp_i = reinterpret_cast<int32_t*>(samp_v + P * NSB * KCr);
  float* phi = reinterpret_cast<float*>(samp_i + P * NSB * KCr);
  hipStream_t st = krca::as_stream(stream);
  KRCA_HIP(hipMemsetAsync(count, 0, P * sizeof(int32_t), st));
  switch (kc_for(k)) {
    case 8: return launch_corr<8>(zh, z32, P, T, Tp, nb, nsb, k, tau, eps, cand_v, cand_i, cand_hd, samp_v, samp_i, phi, count, out_idx, out_val, cert, st);
    case 12:
      return launch_corr<12>(zh, z32, P, T, Tp, nb, nsb, k, tau, eps, cand_v, cand_i, cand_hd, samp_v, samp_i, phi, count, out_idx, out_val, cert, st);
    default:
      return launch_corr<16>(zh, z32, P, T, Tp, nb, nsb, k, tau, eps, cand_v, cand_i, cand_hd, samp_v, samp_i, phi, count, out_idx, out_val, cert, st);
  }
}

}  // extern "C"

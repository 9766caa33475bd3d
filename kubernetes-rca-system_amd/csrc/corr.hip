// Cross-pod Pearson correlation with per-row top-k (configs C3/C4).
//
// R = Z·Zᵀ where z[p,t] = (x[p,t] - mean_p) / (std_p * sqrt(T)) (population std over the T
// samples of one metric channel; a flat series gives z = 0).  Per pod: the k partners with the
// largest |R| (self excluded; ties -> lower index) and the number of partners with |R| > tau.
// The full P x P matrix is never materialised.
//
//   krca_corr_prepare  time-major x[T][P][M] -> per-pod mean/scale (one float64 pass, shifted
//                      sums), then an LDS-tiled transpose to pod-major rows: z32[P][T] (fp32,
//                      used for the exact re-scoring) and the bf16 split z = hi + lo
//                      (zhi/zlo[Pp][Tp], zero padded to 128 rows / 64 steps).
//   krca_corr_tiles    MFMA (v_mfma_f32_32x32x16_bf16) over the UPPER triangle of 128x128
//                      tiles only (P(P+1)/2 pairs, the algorithmic flop count): three bf16
//                      products hi·hi + hi·lo + lo·hi per tile, fp32 accumulation (~fp32
//                      accuracy at the bf16 rate).  Epilogue in LDS: each lane scans one row
//                      (-> candidates of that row from this column block) or one column (-> the
//                      symmetric candidates of that column's pod from this row block), keeping
//                      the KC best (|r| desc, index asc); |r| > tau counts go out as int32 adds.
//   krca_corr_merge    one workgroup per pod: best 16 of its nb*KC candidates, re-scored in
//                      float64 from z32 (fixed-order wave reduction), final top-k; cert[p] =
//                      (k-th re-scored |r|) - (best |r| the tiles could have dropped) - eps:
//                      cert > 0 proves the reported set equals the exact top-k.
#include "krca_common.h"

namespace {

constexpr int TPB = 256;
constexpr int BM = 128;  // tile rows == cols
constexpr int BK = 64;   // K step (time samples)
constexpr int KC = 12;   // candidates kept per (pod, block)
constexpr int KM = 16;   // candidates re-scored per pod in the merge
constexpr float kEps = 1e-4f;  // bound on |r_approx - r| used by the certificate (bf16x3, fp32 acc)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint16_t bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf16_to_f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

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

// 64 pods x 64 steps per block: coalesced-ish reads of the channel, LDS transpose, row writes
__global__ __launch_bounds__(TPB) void corr_transpose(const float* __restrict__ x, int64_t P, int M, int T, int Tp,
                                                      int ch, const float* __restrict__ mean,
                                                      const float* __restrict__ scale, float* __restrict__ z32,
                                                      uint16_t* __restrict__ zhi, uint16_t* __restrict__ zlo) {
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
    if (t < Tp) {
      const uint16_t h = bf16_rne(z);
      const uint16_t l = bf16_rne(z - bf16_to_f(h));
      zhi[pp * Tp + t] = h;  // rows up to Pp (padding rows are zero: pp >= P -> z = 0)
      zlo[pp * Tp + t] = l;
      if (pp < P && t < T) z32[pp * T + t] = z;
    }
  }
}

// ---- tiles -----------------------------------------------------------------------------------
struct Cand {
  float v[KC];  // signed r
  int32_t i[KC];
};

__device__ __forceinline__ bool cbetter(float a, int32_t ia, float b, int32_t ib) {
  const float fa = fabsf(a), fb = fabsf(b);
  return fa > fb || (fa == fb && (uint32_t)ia < (uint32_t)ib);
}

__device__ __forceinline__ void cinit(Cand& c) {
#pragma unroll
  for (int j = 0; j < KC; ++j) {
    c.v[j] = 0.f;
    c.i[j] = -1;
  }
}

__device__ __forceinline__ void cinsert(Cand& c, float nv, int32_t ni) {
  if (!cbetter(nv, ni, c.v[KC - 1], c.i[KC - 1])) return;
#pragma unroll
  for (int j = KC - 1; j > 0; --j) {
    const bool up = cbetter(nv, ni, c.v[j - 1], c.i[j - 1]);
    const bool here = cbetter(nv, ni, c.v[j], c.i[j]);
    const float pv = c.v[j - 1];
    const int32_t pi = c.i[j - 1];
    c.v[j] = up ? pv : (here ? nv : c.v[j]);
    c.i[j] = up ? pi : (here ? ni : c.i[j]);
  }
  if (cbetter(nv, ni, c.v[0], c.i[0])) {
    c.v[0] = nv;
    c.i[0] = ni;
  }
}

constexpr int LDS_STAGE = 4 * BM * BK * 2;        // A_hi, A_lo, B_hi, B_lo (bf16)
constexpr int LDS_EPI = BM * (BM + 1) * 4;        // fp32 tile, padded rows
constexpr int LDS_BYTES = LDS_STAGE > LDS_EPI ? LDS_STAGE : LDS_EPI;

// 16-byte chunk c (0..7) of row r of a [128][64] bf16 tile, XOR-swizzled against bank conflicts
__device__ __forceinline__ int chunk_off(int r, int c) { return r * 128 + ((c ^ (r & 7)) << 4); }

__global__ __launch_bounds__(TPB) void corr_tiles(const uint16_t* __restrict__ zhi, const uint16_t* __restrict__ zlo,
                                                  int64_t P, int Tp, int nb, float tau, float* __restrict__ cand_v,
                                                  int32_t* __restrict__ cand_i, int32_t* __restrict__ count) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // triangular tile index -> (I, J), I <= J
  const int64_t b = blockIdx.x;
  int64_t J = (int64_t)((sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
  while ((J + 1) * (J + 2) / 2 <= b) ++J;
  while (J * (J + 1) / 2 > b) --J;
  const int64_t I = b - J * (J + 1) / 2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;
  const int64_t rowA = I * BM, rowB = J * BM;
  char* sAh = smem;
  char* sAl = smem + BM * BK * 2;
  char* sBh = smem + 2 * BM * BK * 2;
  char* sBl = smem + 3 * BM * BK * 2;

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int r32 = lane & 31, h = lane >> 5;
  for (int k0 = 0; k0 < Tp; k0 += BK) {
    // stage: 4 operands x 128 rows x 8 chunks = 4096 16-byte chunks, 16 per lane
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int id = tid + q * TPB;  // 0..1023
      const int r = id >> 3, c = id & 7;
      const int64_t ga = (rowA + r) * Tp + k0 + c * 8;
      const int64_t gb = (rowB + r) * Tp + k0 + c * 8;
      const uint4 ah = *reinterpret_cast<const uint4*>(zhi + ga);
      const uint4 al = *reinterpret_cast<const uint4*>(zlo + ga);
      const uint4 bh = *reinterpret_cast<const uint4*>(zhi + gb);
      const uint4 bl = *reinterpret_cast<const uint4*>(zlo + gb);
      const int o = chunk_off(r, c);
      *reinterpret_cast<uint4*>(sAh + o) = ah;
      *reinterpret_cast<uint4*>(sAl + o) = al;
      *reinterpret_cast<uint4*>(sBh + o) = bh;
      *reinterpret_cast<uint4*>(sBl + o) = bl;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int c = ks * 2 + h;
      bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int ra = wr * 64 + i * 32 + r32;
        const int rb = wc * 64 + i * 32 + r32;
        ah[i] = *reinterpret_cast<const bf16x8*>(sAh + chunk_off(ra, c));
        al[i] = *reinterpret_cast<const bf16x8*>(sAl + chunk_off(ra, c));
        bh[i] = *reinterpret_cast<const bf16x8*>(sBh + chunk_off(rb, c));
        bl[i] = *reinterpret_cast<const bf16x8*>(sBl + chunk_off(rb, c));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
    __syncthreads();
  }
  // epilogue: tile -> LDS [row][col] (padded), then row / column scans
  float* tile = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = wr * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        const int col = wc * 64 + j * 32 + r32;
        tile[row * (BM + 1) + col] = acc[i][j][e];
      }
  __syncthreads();
  Cand cd;
  cinit(cd);
  int n_over = 0;
  if (tid < BM) {  // row scan: pod rowA+tid against the columns of block J
    const int64_t g = rowA + tid;
    if (g < P) {
      for (int c = 0; c < BM; ++c) {
        const int64_t gc = rowB + c;
        if (gc >= P || gc == g) continue;
        const float v = tile[tid * (BM + 1) + c];
        n_over += fabsf(v) > tau;
        cinsert(cd, v, (int32_t)gc);
      }
      float* ov = cand_v + (g * nb + J) * KC;
      int32_t* oi = cand_i + (g * nb + J) * KC;
#pragma unroll
      for (int q = 0; q < KC; ++q) {
        ov[q] = cd.v[q];
        oi[q] = cd.i[q];
      }
      if (n_over) atomicAdd(&count[g], n_over);
    }
  } else if (I != J) {  // column scan: pod rowB+c against the rows of block I (symmetric half)
    const int c = tid - BM;
    const int64_t g = rowB + c;
    if (g < P) {
      for (int r = 0; r < BM; ++r) {
        const int64_t gr = rowA + r;
        if (gr >= P) continue;
        const float v = tile[r * (BM + 1) + c];
        n_over += fabsf(v) > tau;
        cinsert(cd, v, (int32_t)gr);
      }
      float* ov = cand_v + (g * nb + I) * KC;
      int32_t* oi = cand_i + (g * nb + I) * KC;
#pragma unroll
      for (int q = 0; q < KC; ++q) {
        ov[q] = cd.v[q];
        oi[q] = cd.i[q];
      }
      if (n_over) atomicAdd(&count[g], n_over);
    }
  }
}

// ---- merge + exact re-scoring ------------------------------------------------------------------
struct Cand16 {
  float v[KM + 1];
  int32_t i[KM + 1];
};

__device__ __forceinline__ void minsert(Cand16& c, float nv, int32_t ni) {
  if (!cbetter(nv, ni, c.v[KM], c.i[KM])) return;
#pragma unroll
  for (int j = KM; j > 0; --j) {
    const bool up = cbetter(nv, ni, c.v[j - 1], c.i[j - 1]);
    const bool here = cbetter(nv, ni, c.v[j], c.i[j]);
    const float pv = c.v[j - 1];
    const int32_t pi = c.i[j - 1];
    c.v[j] = up ? pv : (here ? nv : c.v[j]);
    c.i[j] = up ? pi : (here ? ni : c.i[j]);
  }
  if (cbetter(nv, ni, c.v[0], c.i[0])) {
    c.v[0] = nv;
    c.i[0] = ni;
  }
}

__global__ __launch_bounds__(TPB) void corr_merge(const float* __restrict__ cand_v, const int32_t* __restrict__ cand_i,
                                                  const float* __restrict__ z32, int64_t P, int T, int nb, int k,
                                                  int32_t* __restrict__ out_i, float* __restrict__ out_v,
                                                  float* __restrict__ cert) {
  __shared__ float sv[TPB / 64];
  __shared__ int32_t si[TPB / 64];
  __shared__ float top_v[KM + 1];
  __shared__ int32_t top_i[KM + 1];
  __shared__ double exact[KM];
  __shared__ float dropped;
  const int64_t g = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  Cand16 c;
#pragma unroll
  for (int j = 0; j <= KM; ++j) {
    c.v[j] = 0.f;
    c.i[j] = -1;
  }
  float tile_floor = 0.f;  // largest |r| a full tile list could have cut off
  const int64_t base = g * nb * KC;
  for (int64_t q = tid; q < (int64_t)nb * KC; q += TPB) {
    const int32_t id = cand_i[base + q];
    if (id < 0) continue;
    const float v = cand_v[base + q];
    minsert(c, v, id);
    if ((q % KC) == KC - 1) tile_floor = fmaxf(tile_floor, fabsf(v));
  }
  // block-wide extraction of the best KM+1 (k rounds of arg-max over the lane heads)
  for (int r = 0; r <= KM; ++r) {
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
    if (wi != -1 && c.i[0] == wi && c.v[0] == wv) {
#pragma unroll
      for (int j = 0; j < KM; ++j) {
        c.v[j] = c.v[j + 1];
        c.i[j] = c.i[j + 1];
      }
      c.v[KM] = 0.f;
      c.i[KM] = -1;
    }
  }
  // tile_floor: max over lanes
  for (int off = 32; off > 0; off >>= 1) tile_floor = fmaxf(tile_floor, __shfl_xor(tile_floor, off, 64));
  if (lane == 0) sv[w] = tile_floor;
  __syncthreads();
  if (tid == 0) dropped = fmaxf(fmaxf(fmaxf(sv[0], sv[1]), fmaxf(sv[2], sv[3])), fabsf(top_v[KM]));
  __syncthreads();
  // exact float64 re-scoring of the best KM (one wave per candidate, fixed reduction order)
  const float* zg = z32 + g * T;
  for (int q = w; q < KM; q += TPB / 64) {
    const int32_t j = top_i[q];
    double s = 0.0;
    if (j >= 0) {
      const float* zj = z32 + (int64_t)j * T;
      for (int t = lane; t < T; t += 64) s += (double)zg[t] * (double)zj[t];
    }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) exact[q] = s;
  }
  __syncthreads();
  if (tid == 0) {
    // order the re-scored candidates (|r| desc, index asc), keep k
    int ord[KM];
    for (int q = 0; q < KM; ++q) ord[q] = q;
    for (int a = 1; a < KM; ++a) {
      const int key = ord[a];
      int bpos = a - 1;
      while (bpos >= 0) {
        const int o = ord[bpos];
        const double fo = fabs(exact[o]), fk = fabs(exact[key]);
        const bool kb = top_i[key] >= 0 && (top_i[o] < 0 || fk > fo ||
                                            (fk == fo && (uint32_t)top_i[key] < (uint32_t)top_i[o]));
        if (!kb) break;
        ord[bpos + 1] = o;
        --bpos;
      }
      ord[bpos + 1] = key;
    }
    for (int q = 0; q < k; ++q) {
      out_i[g * k + q] = top_i[ord[q]];
      out_v[g * k + q] = (float)exact[ord[q]];
    }
    cert[g] = (float)(fabs(exact[ord[k - 1]]) - (double)dropped - (double)kEps);
  }
}

}  // namespace

extern "C" {

int64_t krca_corr_pad_rows(int64_t P) { return krca::ceil_div(P, BM) * BM; }
int32_t krca_corr_pad_steps(int32_t T) { return (int32_t)krca::ceil_div(T, BK) * BK; }
int64_t krca_corr_cand_size(int64_t P) { return P * (krca_corr_pad_rows(P) / BM) * KC; }
int32_t krca_corr_max_k(void) { return KM; }

int krca_corr_prepare(const float* x, int64_t P, int32_t M, int32_t T, int32_t channel, float* mean, float* scale,
                      float* z32, uint16_t* zhi, uint16_t* zlo, void* stream) {
  KRCA_CHECK_ARG(P > 0 && M > 0 && T > 0 && channel >= 0 && channel < M, "krca_corr_prepare: bad sizes");
  KRCA_CHECK_ARG(x && mean && scale && z32 && zhi && zlo, "krca_corr_prepare: null pointer");
  const int64_t Pp = krca_corr_pad_rows(P);
  const int Tp = krca_corr_pad_steps(T);
  hipStream_t st = krca::as_stream(stream);
  hipLaunchKernelGGL(corr_stats, dim3((unsigned)krca::ceil_div(P, TPB)), dim3(TPB), 0, st, x, P, M, T, channel, mean,
                     scale);
  KRCA_LAUNCH_CHECK();
  hipLaunchKernelGGL(corr_transpose, dim3((unsigned)(Pp / 64), (unsigned)(Tp / 64)), dim3(TPB), 0, st, x, P, M, T, Tp,
                     channel, mean, scale, z32, zhi, zlo);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_corr_topk(const uint16_t* zhi, const uint16_t* zlo, const float* z32, int64_t P, int32_t T, int32_t k,
                   float tau, float* cand_v, int32_t* cand_i, int32_t* count, int32_t* out_idx, float* out_val,
                   float* cert, void* stream) {
  KRCA_CHECK_ARG(P > 1 && P < INT32_MAX && T > 0, "krca_corr_topk: bad sizes");
  KRCA_CHECK_ARG(k >= 1 && k <= KM && k < P, "krca_corr_topk: k must be in [1, %d] and < P", KM);
  KRCA_CHECK_ARG(zhi && zlo && z32 && cand_v && cand_i && count && out_idx && out_val && cert,
                 "krca_corr_topk: null pointer");
  const int64_t Pp = krca_corr_pad_rows(P);
  const int Tp = krca_corr_pad_steps(T);
  const int nb = (int)(Pp / BM);
  const int64_t ntiles = (int64_t)nb * (nb + 1) / 2;
  hipStream_t st = krca::as_stream(stream);
  static bool lds_attr = false;
  if (!lds_attr) {
    KRCA_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_tiles),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
    lds_attr = true;
  }
  KRCA_HIP(hipMemsetAsync(count, 0, P * sizeof(int32_t), st));
  hipLaunchKernelGGL(corr_tiles, dim3((unsigned)ntiles), dim3(TPB), LDS_BYTES, st, zhi, zlo, P, Tp, nb, tau, cand_v,
                     cand_i, count);
  KRCA_LAUNCH_CHECK();
  hipLaunchKernelGGL(corr_merge, dim3((unsigned)P), dim3(TPB), 0, st, cand_v, cand_i, z32, P, T, nb, k, out_idx,
                     out_val, cert);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

}  // extern "C"

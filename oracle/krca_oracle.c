/*
 * krca_oracle.c — CPU restatement of the krca numeric core.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library;
 * the product path (krca.native -> libkrca.so) never does.  It restates, with the same
 * arithmetic in the same order, the device algorithms of include/krca.h, so that integer
 * outputs can be compared bit-for-bit:
 *
 *   krco_usage_flags    ref:agents/metrics_agent.py:88-114, 135-161 (x > 80, high if > 90)
 *   krco_rolling_score  rolling z-score (new primitive, no reference code):
 *                       float64 sliding sums in a fixed order, |z| > thr <=> A^2 > thr^2*B
 *   krco_ppr            networkx 3.4.2 pagerank semantics (_pagerank_scipy) in 2^-60 fixed point
 *   krco_rca_key        root-cause ordering key r x q (PageRank mass x own anomaly; Config key "rq")
 *   krco_rca_explain    the explanation pass of krca_rca_explain: anomalous callers per pod and, per
 *                       pod, the largest anomaly of a dependency that explains it
 *   krco_rca_key_explained  the default root-cause key: received mass x unexplained anomaly
 *   krco_corr_z32       the standardized fp32 rows krca_corr_prepare writes (float64 shifted sums
 *                       for mean / scale, then (x - mean) * scale in float32): bit-exact twin
 *   krco_corr_counts    |r| > tau counts over those rows with float64 dot products, and the pairs
 *                       within a band of tau (where another float64 summation order may differ)
 *
 * The floating-point reference for a5/a10 (float64, independent formulation) is the NumPy
 * oracle in oracle/oracle.py; this file pins the exact bits.  Build: oracle/Makefile
 * (gcc -O2 -fopenmp -ffp-contract=off).  OpenMP parallelises over independent series / nodes
 * only; every per-element computation is the sequential restatement.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define VAR_EPS 1e-12
static const double kFix = 1152921504606846976.0; /* 2^60 */

void krco_usage_flags(const float* usage, int64_t P, uint8_t* flags) {
  for (int64_t p = 0; p < P; ++p) {
    const float c = usage[2 * p], m = usage[2 * p + 1];
    flags[p] = (uint8_t)((c > 80.f ? 1 : 0) | (c > 90.f ? 2 : 0) | (m > 80.f ? 4 : 0) | (m > 90.f ? 8 : 0));
  }
}

/* x: time-major [T][P][M] float32.  Same outputs as krca_rolling_score, same operations in the
 * same order: A = fma(W, x_t, -s1), B = fma(W, s2, -s1*s1), exceed iff B > 1e-12*W*W and
 * fma(A, A, -thr^2*B) > 0; s1 = (s1 + x_t) - x_{t-W}; s2 = fma(-x_{t-W}, x_{t-W}, fma(x_t, x_t, s2)). */
void krco_rolling_score(const float* x, int64_t P, int32_t M, int32_t T, int32_t W, float z_thr, float* z_last,
                        float* score, int32_t* n_exceed, uint8_t* flags) {
  const int64_t S = P * (int64_t)M;
  const double Wd = (double)W, epsB = VAR_EPS * Wd * Wd;
  const double thr2 = (double)z_thr * (double)z_thr;
#pragma omp parallel for schedule(static)
  for (int64_t p = 0; p < P; ++p) {
    float best = 0.f;
    int32_t cnt = 0;
    unsigned f = 0;
    for (int32_t m = 0; m < M; ++m) {
      const int64_t s = p * M + m;
      double s1 = 0.0, s2 = 0.0, al = 0.0, bl = 0.0;
      for (int32_t j = 0; j < W && j < T; ++j) {
        const double vd = (double)x[(int64_t)j * S + s];
        s1 = s1 + vd;
        s2 = fma(vd, vd, s2);
      }
      for (int32_t t = W; t < T; ++t) {
        const double vd = (double)x[(int64_t)t * S + s];
        const double od = (double)x[(int64_t)(t - W) * S + s];
        const double A = fma(Wd, vd, -s1);
        const double B = fma(Wd, s2, -(s1 * s1));
        cnt += (B > epsB) && (fma(A, A, -(thr2 * B)) > 0.0);
        if (t == T - 1) {
          al = A;
          bl = B;
        }
        s1 = (s1 + vd) - od;
        s2 = fma(-od, od, fma(vd, vd, s2));
      }
      const float z = bl > epsB ? (float)(al / sqrt(bl)) : 0.f;
      z_last[s] = z;
      const float az = fabsf(z);
      if (az > best) best = az;
      if (T > 0) {
        const float v = x[(int64_t)(T - 1) * S + s];
        if (m == 0) f |= (v > 80.f ? 1u : 0u) | (v > 90.f ? 2u : 0u);
        if (m == 1) f |= (v > 80.f ? 4u : 0u) | (v > 90.f ? 8u : 0u);
      }
    }
    score[p] = best;
    n_exceed[p] = cnt;
    flags[p] = (uint8_t)f;
  }
}

static int64_t edge_weight(int64_t rj, int32_t deg, double alpha) {
  if (deg == 0) return 0;
  const double coef = alpha / (double)deg;
  return (int64_t)((double)rj * coef);
}

/* the 32-bit weight code the rows gather (csrc/ppr.hip wenc / wdec): w < 2^26 as is, above that
 * the top 26 bits and the shift in the top 6 bits (truncating) */
static uint32_t wenc(int64_t w) {
  if (w < ((int64_t)1 << 26)) return (uint32_t)w;
  const int sh = 63 - __builtin_clzll((unsigned long long)w) - 25;
  return ((uint32_t)sh << 26) | (uint32_t)(w >> sh);
}
static int64_t wdec(uint32_t c) { return (int64_t)(c & 0x3FFFFFFu) << (c >> 26); }

/* csrc/ppr.hip / explain.hip quantise: 2^32 per |z| unit above the floor, clamped at 256 units */
static int64_t quantise(float s, float seed_floor) {
  const double v = (double)s - (double)seed_floor;
  return v > 0.0 ? (int64_t)(fmin(v, 256.0) * 4294967296.0) : 0;
}

/* Pull-CSR personalized PageRank; returns iterations (negative if no convergence).
 * warm != 0: r holds the start vector on entry (krca_ppr_shard_init_warm), else r0 = 2^60/N.
 * recv (optional): the mass each node received from its callers in the last iteration that updated
 * the ranks (r = recv + teleport share; what krca_rca_key_explained recovers as r - t). */
int32_t krco_ppr_ex(const int64_t* row_ptr, const int32_t* col, const int32_t* outdeg, int64_t N, const float* seed,
                    float seed_floor, double alpha, int32_t max_iter, double tol, int64_t* r, float* r_out, int64_t* q,
                    int warm, int64_t* recv) {
  uint32_t* w = (uint32_t*)malloc(sizeof(uint32_t) * N);
  int64_t qtot = 0, dang = 0;
  const int64_t r0 = (int64_t)(kFix / (double)N);
  for (int64_t i = 0; i < N; ++i) {
    q[i] = quantise(seed[i], seed_floor);
    qtot += q[i];
    if (!warm) r[i] = r0;
    w[i] = wenc(edge_weight(r[i], outdeg[i], alpha));
    if (outdeg[i] == 0) dang += r[i];
  }
  const double err_limit = tol > 0.0 ? (double)N * tol * kFix : 0.0;
  double tele = (1.0 - alpha) * kFix + alpha * (double)dang;
  int32_t it = 0, conv = 0;
  int64_t* acc = (int64_t*)malloc(sizeof(int64_t) * N);
  while (it < max_iter) {
#pragma omp parallel for schedule(dynamic, 1024)
    for (int64_t i = 0; i < N; ++i) {
      int64_t s = 0;
      for (int64_t e = row_ptr[i]; e < row_ptr[i + 1]; ++e) s += wdec(w[col[e]]);
      acc[i] = s;
    }
    int64_t err = 0, dn = 0;
    /* teleport share t_i = q_i * (tele / qtot) (csrc/ppr.hip update_row: one scale per iteration,
       no per-row division); uniform 1/N when every seed is at the floor */
    const double tq = tele / (double)qtot;
    const int64_t tu = (int64_t)((1.0 / (double)N) * tele);
    for (int64_t i = 0; i < N; ++i) {
      const int64_t t = qtot > 0 ? (int64_t)((double)q[i] * tq) : tu;
      const int64_t rn = acc[i] + t;
      const int64_t ro = r[i];
      r[i] = rn;
      err += rn > ro ? rn - ro : ro - rn;
      if (outdeg[i] == 0) dn += rn;
      w[i] = wenc(edge_weight(rn, outdeg[i], alpha));
    }
    ++it;
    if (err_limit > 0.0 && (double)err < err_limit) {
      conv = 1;
      break;
    }
    tele = (1.0 - alpha) * kFix + alpha * (double)dn;
  }
  for (int64_t i = 0; i < N; ++i) r_out[i] = (float)((double)r[i] * (1.0 / kFix));
  if (recv) {
    /* no iteration: no teleport share was added either (the device's recorded share is 0) */
    memcpy(recv, it > 0 ? acc : r, sizeof(int64_t) * N);
  }
  free(w);
  free(acc);
  return (err_limit > 0.0 && !conv) ? -it : it;
}

int32_t krco_ppr_start(const int64_t* row_ptr, const int32_t* col, const int32_t* outdeg, int64_t N,
                       const float* seed, float seed_floor, double alpha, int32_t max_iter, double tol, int64_t* r,
                       float* r_out, int64_t* q, int warm) {
  return krco_ppr_ex(row_ptr, col, outdeg, N, seed, seed_floor, alpha, max_iter, tol, r, r_out, q, warm, NULL);
}

int32_t krco_ppr(const int64_t* row_ptr, const int32_t* col, const int32_t* outdeg, int64_t N, const float* seed,
                 float seed_floor, double alpha, int32_t max_iter, double tol, int64_t* r, float* r_out, int64_t* q) {
  return krco_ppr_start(row_ptr, col, outdeg, N, seed, seed_floor, alpha, max_iter, tol, r, r_out, q, 0);
}

/* root-cause key of krca_ppr_rca_key */
void krco_rca_key(const int64_t* r, const int64_t* q, int64_t n, int64_t* key) {
  for (int64_t i = 0; i < n; ++i) {
    const double v = (double)r[i] * (double)q[i];
    memcpy(&key[i], &v, sizeof(v));
  }
}


/* The explanation pass of krca_rca_explain (csrc/explain.hip), over the whole pull-CSR (row k = the
 * callers j of k, edges j -> k).  q_j = the quantised seed of krca_ppr_shard_init.  For every
 * anomalous pod k (q_k > 0): A_k = its edges from anomalous callers and S_k = the sum of their q.  An
 * anomalous dependency k of an anomalous pod j (edge j -> k, j != k) EXPLAINS j when
 *   (A_k - 1 >= A_j  or  q_k >= 2 q_j)   -- the symptoms converge on k (at least as many anomalous
 *                                           callers besides j), or k is at least twice as anomalous --
 *   and A_k q_j <= 3 S_k                 -- j looks like k's other symptoms (its anomaly at most 3x
 *                                           the mean over k's anomalous callers; a pod far above
 *                                           them is a fault of its own that happens to call k).
 * d[j - lo] = the largest q_k over the dependencies that explain j (0: none), for pods [lo, hi).
 * Integer arithmetic throughout: q <= 2^40 (quantise), S_k summed and A_k q_j <= 3 S_k compared in
 * 128 bits (exact for any row length; ADVICE r5: the int64 form wrapped for large seeds). */
void krco_rca_explain(const float* score, int64_t N, float seed_floor, const int64_t* row_ptr, const int32_t* col,
                      int64_t lo, int64_t hi, int64_t* d) {
  int64_t* q = (int64_t*)malloc(sizeof(int64_t) * (N > 0 ? N : 1));
  __int128* S = (__int128*)calloc(N > 0 ? N : 1, sizeof(__int128));
  int32_t* A = (int32_t*)calloc(N > 0 ? N : 1, sizeof(int32_t));
  for (int64_t i = 0; i < N; ++i) q[i] = quantise(score[i], seed_floor);
#pragma omp parallel for schedule(dynamic, 1024)
  for (int64_t k = 0; k < N; ++k) {
    if (q[k] <= 0) continue;
    int32_t a = 0;
    __int128 sum = 0;
    for (int64_t e = row_ptr[k]; e < row_ptr[k + 1]; ++e) {
      const int64_t qc = q[col[e]];
      if (qc > 0) {
        a += 1;
        sum += qc;
      }
    }
    A[k] = a;
    S[k] = sum;
  }
  memset(d, 0, sizeof(int64_t) * (hi > lo ? hi - lo : 0));
  for (int64_t k = 0; k < N; ++k) {
    const int64_t qk = q[k];
    if (qk <= 0) continue;
    for (int64_t e = row_ptr[k]; e < row_ptr[k + 1]; ++e) {
      const int64_t j = col[e];
      if (j < lo || j >= hi || j == k) continue;
      const int64_t qj = q[j];
      if (qj <= 0) continue;
      if ((A[k] - 1 >= A[j] || qk >= 2 * qj) && (__int128)A[k] * qj <= 3 * S[k] && qk > d[j - lo]) d[j - lo] = qk;
    }
  }
  free(q);
  free(S);
  free(A);
}

/* root-cause key of krca_rca_key_explained: u_i = max(q_i - d_i, 0) (the anomaly no explaining
 * dependency accounts for), t_i = r_i - recv_i (the row's own teleport share in the last step),
 * key = bits(((double)recv_i + (double)t_i / 32) * (double)u_i), 0 when u_i = 0 */
void krco_rca_key_explained(const int64_t* r, const int64_t* recv, const int64_t* q, const int64_t* d, int64_t n,
                            int64_t* key) {
  for (int64_t i = 0; i < n; ++i) {
    const int64_t u = q[i] - d[i];
    const double v = u > 0 ? ((double)recv[i] + (double)(r[i] - recv[i]) * 0.03125) * (double)u : 0.0;
    memcpy(&key[i], &v, sizeof(v));
  }
}

/* corr_stats + corr_transpose of csrc/corr.hip (a9, new primitive): x time-major [T][P][M] */
void krco_corr_z32(const float* x, int64_t P, int32_t M, int32_t T, int32_t ch, float* mean, float* scale,
                   float* z32) {
  const int64_t S = P * (int64_t)M;
#pragma omp parallel for schedule(static)
  for (int64_t p = 0; p < P; ++p) {
    const float* xs = x + p * M + ch;
    const double x0 = (double)xs[0];
    double s1 = 0.0, s2 = 0.0;
    for (int32_t t = 0; t < T; ++t) {
      const double d = (double)xs[(int64_t)t * S] - x0;
      s1 += d;
      s2 += d * d;
    }
    const double mu = s1 / T;
    const double var = s2 / T - mu * mu;
    const float mf = (float)(x0 + mu);
    const float sc = var > 1e-20 ? (float)(1.0 / sqrt(var * (double)T)) : 0.f;
    mean[p] = mf;
    scale[p] = sc;
    for (int32_t t = 0; t < T; ++t) {
      const float v = xs[(int64_t)t * S] - mf;
      z32[p * T + t] = v * sc;
    }
  }
}

/* for each row p of rows[]: count[i] = #{q != p : |sum_t z32[p,t] z32[q,t]| > tau} in float64
 * (every product is exact in float64; the sum's rounding is <= T 2^-53 sum |products|), and
 * band[i] = #{q != p : | |r| - tau | <= band_eps} (pairs a different summation order could flip) */
void krco_corr_counts(const float* z32, int64_t P, int32_t T, const int64_t* rows, int64_t n_rows, double tau,
                      double band_eps, int32_t* count, int32_t* band) {
#pragma omp parallel for schedule(dynamic, 4)
  for (int64_t i = 0; i < n_rows; ++i) {
    const int64_t p = rows[i];
    const float* za = z32 + p * T;
    int32_t c = 0, b = 0;
    for (int64_t q = 0; q < P; ++q) {
      if (q == p) continue;
      const float* zb = z32 + q * T;
      double acc = 0.0;
      for (int32_t t = 0; t < T; ++t) acc += (double)za[t] * (double)zb[t];
      const double a = fabs(acc);
      c += a > tau;
      b += fabs(a - tau) <= band_eps;
    }
    count[i] = c;
    band[i] = b;
  }
}

// Error-template hashing and per-container template histograms.
//
// New primitive (no reference code; semantics defined here and restated in oracle/oracle.py):
//   template(line) = the line's bytes with every maximal run of [A-Za-z0-9_] that contains an
//                    ASCII digit, or that is >= 8 characters of [0-9a-fA-F], replaced by "<*>"
//                    (masks counters, ids, addresses, timestamps, hashes and UUID groups;
//                    bytes >= 0x80 are never word characters and pass through unchanged);
//   h(line)        = FNV-1a-64 over the template bytes (offset 0xcbf29ce484222325,
//                    prime 0x100000001b3);
//   per container  = the distinct h of its lines in ascending order with their line counts.
//
// krca_template_hash: one lane per line (lines from krca_log_match), bytes through the same
//   16-byte register window as the log scanner; word bytes are hashed once the word's fate is
//   known (the word is re-read from L1/L2, never from HBM twice in practice).
// krca_template_hist: sort-based, atomics-free.  Containers with <= 64 lines: one wave, bitonic
//   sort of 64-bit keys across lanes (shuffles), run heads by ballot, counts by ballot distance.
//   <= 4096 lines: one workgroup, bitonic sort in LDS, run compaction by a block scan.
#include "krca_common.h"

#include <algorithm>
#include <climits>

namespace {

constexpr int TPB = 256;
constexpr int BIG = 4096;  // max lines per container handled by the LDS path
constexpr uint64_t kFnvOff = 0xcbf29ce484222325ull;
constexpr uint64_t kFnvPrime = 0x100000001b3ull;

struct Bytes16 {  // 16-byte register window over the text (as in logscan.hip)
  const uint8_t* t;
  int64_t n, base;
  uint32_t w0, w1, w2, w3;
  __device__ void init(const uint8_t* text, int64_t nbytes) {
    t = text;
    n = nbytes;
    base = -1;
  }
  __device__ __forceinline__ uint32_t at(int64_t p) {
    const int64_t b = p & ~(int64_t)15;
    if (b != base) {
      base = b;
      if (b + 16 <= n) {
        const uint4 v = *reinterpret_cast<const uint4*>(t + b);
        w0 = v.x;
        w1 = v.y;
        w2 = v.z;
        w3 = v.w;
      } else {
        uint32_t ww[4] = {0, 0, 0, 0};
        for (int k = 0; k < 16; ++k)
          if (b + k < n) ww[k >> 2] |= (uint32_t)t[b + k] << (8 * (k & 3));
        w0 = ww[0];
        w1 = ww[1];
        w2 = ww[2];
        w3 = ww[3];
      }
    }
    const int q = (int)((p >> 2) & 3);
    const uint32_t w = q == 0 ? w0 : (q == 1 ? w1 : (q == 2 ? w2 : w3));
    return (w >> (8 * (int)(p & 3))) & 0xFFu;
  }
};

__device__ __forceinline__ uint64_t fnv(uint64_t h, uint32_t b) { return (h ^ b) * kFnvPrime; }
__device__ __forceinline__ bool is_word(uint32_t b) {
  return (b >= '0' && b <= '9') || (b >= 'A' && b <= 'Z') || (b >= 'a' && b <= 'z') || b == '_';
}
__device__ __forceinline__ bool is_hex(uint32_t b) {
  return (b >= '0' && b <= '9') || (b >= 'A' && b <= 'F') || (b >= 'a' && b <= 'f');
}

__global__ __launch_bounds__(TPB) void tmpl_hash_kernel(const uint8_t* __restrict__ text, int64_t nbytes,
                                                        const int64_t* __restrict__ ls, const int64_t* __restrict__ le,
                                                        int64_t L, uint64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= L) return;
  Bytes16 B;
  B.init(text, nbytes);
  const int64_t s = ls[i], e = le[i];
  uint64_t h = kFnvOff;
  int64_t w0 = -1;  // start of the current word
  bool digit = false, hex = true;
  for (int64_t p = s; p <= e; ++p) {
    const uint32_t b = p < e ? B.at(p) : 0u;  // sentinel closes a trailing word
    if (p < e && is_word(b)) {
      if (w0 < 0) {
        w0 = p;
        digit = false;
        hex = true;
      }
      digit |= (b >= '0' && b <= '9');
      hex &= is_hex(b);
      continue;
    }
    if (w0 >= 0) {  // the word [w0, p) ends here
      if (digit || (hex && p - w0 >= 8)) {
        h = fnv(fnv(fnv(h, '<'), '*'), '>');
      } else {
        for (int64_t q = w0; q < p; ++q) h = fnv(h, B.at(q));
      }
      w0 = -1;
    }
    if (p < e) h = fnv(h, b);
  }
  out[i] = h;
}

// ---- per-container histograms ----------------------------------------------------------------
__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  return (uint64_t)__shfl_xor((long long)v, m, 64);
}

// wave per container with <= 64 lines
__global__ __launch_bounds__(TPB) void tmpl_hist_small(const uint64_t* __restrict__ hash,
                                                       const int32_t* __restrict__ doc_lines,
                                                       const int64_t* __restrict__ doc_line0, int64_t D,
                                                       uint64_t* __restrict__ out_hash, int32_t* __restrict__ out_cnt,
                                                       int32_t* __restrict__ n_tmpl) {
  const int64_t d = (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (d >= D) return;
  const int n = doc_lines[d];
  if (n > 64) return;  // handled by tmpl_hist_big
  const int64_t lo = doc_line0[d];
  uint64_t v = lane < n ? hash[lo + lane] : ~0ull;
  // bitonic sort ascending across the 64 lanes
  for (int k = 2; k <= 64; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      const uint64_t o = shfl_xor_u64(v, j);
      const bool up = ((lane & k) == 0);
      const bool lower = (lane & j) == 0;
      const bool take_min = (up == lower);
      v = take_min ? (o < v ? o : v) : (o > v ? o : v);
    }
  }
  const uint64_t prev = (uint64_t)__shfl_up((long long)v, 1, 64);
  const bool valid = lane < n;
  const bool head = valid && (lane == 0 || prev != v);
  const uint64_t heads = __ballot(head);
  if (head) {
    const uint64_t after = lane == 63 ? 0ull : (heads >> (lane + 1));
    const int next = after ? lane + 1 + (__ffsll((unsigned long long)after) - 1) : n;
    const int idx = __popcll(heads & ((1ull << lane) - 1ull));
    out_hash[lo + idx] = v;
    out_cnt[lo + idx] = next - lane;
  }
  if (lane == 0) n_tmpl[d] = __popcll(heads);
}

// workgroup per container with 64 < lines <= 4096
__global__ __launch_bounds__(TPB) void tmpl_hist_big(const uint64_t* __restrict__ hash,
                                                     const int32_t* __restrict__ doc_lines,
                                                     const int64_t* __restrict__ doc_line0,
                                                     const int32_t* __restrict__ big_docs, int32_t n_big,
                                                     uint64_t* __restrict__ out_hash, int32_t* __restrict__ out_cnt,
                                                     int32_t* __restrict__ n_tmpl) {
  __shared__ uint64_t key[BIG];
  __shared__ int32_t pos[BIG];
  __shared__ int32_t wsum[TPB / 64];
  const int b = blockIdx.x;
  if (b >= n_big) return;
  const int64_t d = big_docs[b];
  const int n = doc_lines[d];
  const int64_t lo = doc_line0[d];
  int np = 64;
  while (np < n) np <<= 1;
  for (int i = threadIdx.x; i < np; i += TPB) key[i] = i < n ? hash[lo + i] : ~0ull;
  __syncthreads();
  for (int k = 2; k <= np; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < np; i += TPB) {
        const int l = i ^ j;
        if (l > i) {
          const uint64_t a = key[i], c = key[l];
          const bool up = (i & k) == 0;
          if ((a > c) == up) {
            key[i] = c;
            key[l] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  // run heads -> exclusive scan -> compaction
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int carry = 0;
  for (int base = 0; base < n; base += TPB) {
    const int i = base + threadIdx.x;
    const bool head = i < n && (i == 0 || key[i] != key[i - 1]);
    const uint64_t bal = __ballot(head);
    const int in_wave = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wid] = __popcll(bal);
    __syncthreads();
    int before = carry;
    for (int w = 0; w < wid; ++w) before += wsum[w];
    if (head) pos[before + in_wave] = i;
    int tot = 0;
    for (int w = 0; w < TPB / 64; ++w) tot += wsum[w];
    __syncthreads();
    carry += tot;
  }
  __syncthreads();
  for (int r = threadIdx.x; r < carry; r += TPB) {
    const int i = pos[r];
    const int next = r + 1 < carry ? pos[r + 1] : n;
    out_hash[lo + r] = key[i];
    out_cnt[lo + r] = next - i;
  }
  if (threadIdx.x == 0) n_tmpl[d] = carry;
}

// ---- containers with more than BIG lines -----------------------------------------------------
// Exact and sort-based on the DISTINCT templates: (1) an open-addressing table in the workspace
// counts each distinct hash (CAS insert, count atomics — a chatty container repeats a few
// templates millions of times, so deduplicating first keeps every later step small); (2) the
// distinct (hash, count) pairs are bucketed by their top hash bits, buckets sized for <= 2048
// expected entries (the hashes are FNV-1a-64 outputs, so the top bits spread them); (3) one
// workgroup per bucket sorts its pairs in LDS; buckets are in hash order and placed at their
// exclusive-scan offsets, so the output is globally ascending with no gaps.  A bucket above
// BIG entries (practically impossible for distinct 64-bit hashes) sets the error flag.
constexpr uint64_t kEmpty = ~0ull;

struct HugeLayout {  // workspace of one huge container of n lines (byte offsets)
  int64_t cap, nb, shift;
  int64_t keys, cnts, bcnt, bfill, boff, tk, tc, misc, total;
  __host__ __device__ explicit HugeLayout(int64_t n) {
    cap = 1;
    while (cap < 2 * n) cap <<= 1;
    nb = 1;
    int lg = 0;
    while (nb * 2048 < n) {
      nb <<= 1;
      ++lg;
    }
    shift = 64 - lg;
    keys = 0;
    cnts = keys + cap * 8;
    bcnt = cnts + cap * 4;
    bfill = bcnt + nb * 4;
    boff = bfill + nb * 4;
    tk = ((boff + (nb + 1) * 4 + 15) / 16) * 16;
    tc = tk + n * 8;
    misc = ((tc + n * 4 + 15) / 16) * 16;  // [0] special count, [1] flag
    total = misc + 16;
  }
};

__device__ __forceinline__ int64_t bucket_of(uint64_t h, int64_t shift) { return shift >= 64 ? 0 : (int64_t)(h >> shift); }

__global__ __launch_bounds__(TPB) void huge_init(char* ws, int64_t n) {
  const HugeLayout L(n);
  uint64_t* keys = reinterpret_cast<uint64_t*>(ws + L.keys);
  int32_t* cnts = reinterpret_cast<int32_t*>(ws + L.cnts);
  const int64_t stride = (int64_t)gridDim.x * TPB;
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < L.cap; i += stride) {
    keys[i] = kEmpty;
    cnts[i] = 0;
  }
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < L.nb; i += stride) {
    reinterpret_cast<int32_t*>(ws + L.bcnt)[i] = 0;
    reinterpret_cast<int32_t*>(ws + L.bfill)[i] = 0;
  }
  if (blockIdx.x == 0 && threadIdx.x < 2) reinterpret_cast<int32_t*>(ws + L.misc)[threadIdx.x] = 0;
}

__global__ __launch_bounds__(TPB) void huge_insert(const uint64_t* __restrict__ hash, int64_t n, char* ws) {
  const HugeLayout L(n);
  uint64_t* keys = reinterpret_cast<uint64_t*>(ws + L.keys);
  int32_t* cnts = reinterpret_cast<int32_t*>(ws + L.cnts);
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = hash[i];
  if (h == kEmpty) {  // the sentinel value itself: counted aside, emitted last (largest key)
    atomicAdd(reinterpret_cast<int32_t*>(ws + L.misc), 1);
    return;
  }
  int64_t s = (int64_t)(h & (uint64_t)(L.cap - 1));
  for (;;) {  // the table has >= 2n slots: a free or matching slot is always found
    const uint64_t prev = atomicCAS((unsigned long long*)(keys + s), (unsigned long long)kEmpty, (unsigned long long)h);
    if (prev == kEmpty || prev == h) {
      atomicAdd(cnts + s, 1);
      return;
    }
    s = (s + 1) & (L.cap - 1);
  }
}

__global__ __launch_bounds__(TPB) void huge_bucket(int64_t n, char* ws, bool scatter) {
  const HugeLayout L(n);
  const uint64_t* keys = reinterpret_cast<const uint64_t*>(ws + L.keys);
  const int32_t* cnts = reinterpret_cast<const int32_t*>(ws + L.cnts);
  int32_t* bcnt = reinterpret_cast<int32_t*>(ws + L.bcnt);
  int32_t* bfill = reinterpret_cast<int32_t*>(ws + L.bfill);
  const int32_t* boff = reinterpret_cast<const int32_t*>(ws + L.boff);
  const int64_t stride = (int64_t)gridDim.x * TPB;
  for (int64_t s = (int64_t)blockIdx.x * TPB + threadIdx.x; s < L.cap; s += stride) {
    const int32_t c = cnts[s];
    if (c == 0) continue;
    const uint64_t k = keys[s];
    const int64_t b = bucket_of(k, L.shift);
    if (!scatter) {
      atomicAdd(bcnt + b, 1);
    } else {
      const int64_t pos = boff[b] + atomicAdd(bfill + b, 1);
      reinterpret_cast<uint64_t*>(ws + L.tk)[pos] = k;
      reinterpret_cast<int32_t*>(ws + L.tc)[pos] = c;
    }
  }
}

// one workgroup: exclusive scan of the bucket sizes, the template count, the sentinel entry
__global__ __launch_bounds__(1024) void huge_scan(int64_t n, char* ws, uint64_t* __restrict__ out_hash,
                                                  int32_t* __restrict__ out_cnt, int32_t* __restrict__ n_tmpl) {
  const HugeLayout L(n);
  const int32_t* bcnt = reinterpret_cast<const int32_t*>(ws + L.bcnt);
  int32_t* boff = reinterpret_cast<int32_t*>(ws + L.boff);
  int32_t* misc = reinterpret_cast<int32_t*>(ws + L.misc);
  __shared__ int32_t wsum[16];
  __shared__ int32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int64_t base = 0; base < L.nb; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const int32_t v = i < L.nb ? bcnt[i] : 0;
    if (v > BIG) misc[1] = 1;
    int32_t x = v;
    for (int off = 1; off < 64; off <<= 1) {
      const int32_t y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    int32_t before = carry;
    for (int w = 0; w < wid; ++w) before += wsum[w];
    if (i < L.nb) boff[i] = before + x - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = before + x;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const int32_t u = carry;
    boff[L.nb] = u;
    const int32_t sp = misc[0];
    if (sp > 0) {
      out_hash[u] = kEmpty;
      out_cnt[u] = sp;
    }
    *n_tmpl = u + (sp > 0 ? 1 : 0);
  }
}

// workgroup per bucket: LDS bitonic sort of its (hash, count) pairs, written at the bucket offset
__global__ __launch_bounds__(TPB) void huge_sort(int64_t n, const char* __restrict__ ws, uint64_t* __restrict__ out_hash,
                                                 int32_t* __restrict__ out_cnt) {
  const HugeLayout L(n);
  __shared__ uint64_t key[BIG];
  __shared__ int32_t val[BIG];
  const int64_t b = blockIdx.x;
  if (b >= L.nb) return;
  const int32_t m = reinterpret_cast<const int32_t*>(ws + L.bcnt)[b];
  const int32_t o = reinterpret_cast<const int32_t*>(ws + L.boff)[b];
  if (m == 0 || m > BIG) return;  // m > BIG: flagged by huge_scan
  const uint64_t* tk = reinterpret_cast<const uint64_t*>(ws + L.tk) + o;
  const int32_t* tc = reinterpret_cast<const int32_t*>(ws + L.tc) + o;
  int np = 64;
  while (np < m) np <<= 1;
  for (int i = threadIdx.x; i < np; i += TPB) {
    key[i] = i < m ? tk[i] : kEmpty;
    val[i] = i < m ? tc[i] : 0;
  }
  __syncthreads();
  for (int k = 2; k <= np; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < np; i += TPB) {
        const int l = i ^ j;
        if (l > i) {
          const uint64_t a = key[i], c = key[l];
          const bool up = (i & k) == 0;
          if ((a > c) == up) {
            key[i] = c;
            key[l] = a;
            const int32_t t = val[i];
            val[i] = val[l];
            val[l] = t;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < m; i += TPB) {
    out_hash[o + i] = key[i];
    out_cnt[o + i] = val[i];
  }
}

}  // namespace

extern "C" {

int krca_template_hash(const uint8_t* text, int64_t nbytes, const int64_t* line_start, const int64_t* line_end,
                       int64_t n_lines, uint64_t* hash, void* stream) {
  KRCA_CHECK_ARG(nbytes >= 0 && n_lines >= 0, "krca_template_hash: bad sizes");
  if (n_lines == 0) return KRCA_OK;
  KRCA_CHECK_ARG(text && line_start && line_end && hash, "krca_template_hash: null pointer");
  KRCA_CHECK_ARG(((uintptr_t)text & 15) == 0, "krca_template_hash: text must be 16-byte aligned");
  hipLaunchKernelGGL(tmpl_hash_kernel, dim3((unsigned)krca::ceil_div(n_lines, TPB)), dim3(TPB), 0,
                     krca::as_stream(stream), text, nbytes, line_start, line_end, n_lines, hash);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_template_hist(const uint64_t* hash, const int32_t* doc_lines, const int64_t* doc_line0, int64_t ndocs,
                       const int32_t* big_docs_host, int32_t n_big, int32_t* big_docs_dev, uint64_t* out_hash,
                       int32_t* out_count, int32_t* n_templates, void* stream) {
  KRCA_CHECK_ARG(ndocs >= 0 && n_big >= 0, "krca_template_hist: bad sizes");
  if (ndocs == 0) return KRCA_OK;
  KRCA_CHECK_ARG(doc_lines && doc_line0 && n_templates && out_hash && out_count, "krca_template_hist: null pointer");
  hipStream_t st = krca::as_stream(stream);
  hipLaunchKernelGGL(tmpl_hist_small, dim3((unsigned)krca::ceil_div(ndocs, TPB / 64)), dim3(TPB), 0, st, hash,
                     doc_lines, doc_line0, ndocs, out_hash, out_count, n_templates);
  KRCA_LAUNCH_CHECK();
  if (n_big > 0) {
    KRCA_CHECK_ARG(big_docs_host && big_docs_dev, "krca_template_hist: null big-doc list");
    KRCA_HIP(hipMemcpyAsync(big_docs_dev, big_docs_host, n_big * sizeof(int32_t), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(tmpl_hist_big, dim3((unsigned)n_big), dim3(TPB), 0, st, hash, doc_lines, doc_line0, big_docs_dev,
                       n_big, out_hash, out_count, n_templates);
    KRCA_LAUNCH_CHECK();
  }
  return KRCA_OK;
}

int32_t krca_template_max_lines(void) { return BIG; }

int64_t krca_template_huge_ws_size(int64_t n_lines) { return HugeLayout(n_lines).total; }

int krca_template_hist_huge(const uint64_t* hash, int64_t n_lines, void* workspace, uint64_t* out_hash,
                            int32_t* out_count, int32_t* n_templates, int32_t* flag, void* stream) {
  KRCA_CHECK_ARG(n_lines > 0 && n_lines < INT32_MAX, "krca_template_hist_huge: n_lines out of range");
  KRCA_CHECK_ARG(hash && workspace && out_hash && out_count && n_templates && flag,
                 "krca_template_hist_huge: null pointer");
  KRCA_CHECK_ARG(((uintptr_t)workspace & 15) == 0, "krca_template_hist_huge: workspace must be 16-byte aligned");
  const HugeLayout L(n_lines);
  char* ws = static_cast<char*>(workspace);
  hipStream_t st = krca::as_stream(stream);
  const unsigned g_cap = (unsigned)std::min<int64_t>(krca::ceil_div(L.cap, TPB), 8192);
  hipLaunchKernelGGL(huge_init, dim3(g_cap), dim3(TPB), 0, st, ws, n_lines);
  KRCA_LAUNCH_CHECK();
  hipLaunchKernelGGL(huge_insert, dim3((unsigned)krca::ceil_div(n_lines, TPB)), dim3(TPB), 0, st, hash, n_lines, ws);
  KRCA_LAUNCH_CHECK();
  hipLaunchKernelGGL(huge_bucket, dim3(g_cap), dim3(TPB), 0, st, n_lines, ws, false);
  KRCA_LAUNCH_CHECK();
  hipLaunchKernelGGL(huge_scan, dim3(1), dim3(1024), 0, st, n_lines, ws, out_hash, out_count, n_templates);
  KRCA_LAUNCH_CHECK();
  hipLaunchKernelGGL(huge_bucket, dim3(g_cap), dim3(TPB), 0, st, n_lines, ws, true);
  KRCA_LAUNCH_CHECK();
  hipLaunchKernelGGL(huge_sort, dim3((unsigned)L.nb), dim3(TPB), 0, st, n_lines, (const char*)ws, out_hash, out_count);
  KRCA_LAUNCH_CHECK();
  KRCA_HIP(hipMemcpyAsync(flag, ws + L.misc + 4, sizeof(int32_t), hipMemcpyDeviceToDevice, st));
  return KRCA_OK;
}

}  // extern "C"

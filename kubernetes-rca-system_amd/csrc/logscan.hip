// 13-category log line histograms.
//
// Exactly reproduces, for every container log text, ref:agents/logs_agent.py:140-151:
//   lines = text.splitlines();  bin c = number of lines with re.search(pattern_c, line, re.I)
// plus the first three matching lines per bin (the evidence of :159-163) and len(lines).
//
// Input: one UTF-8 blob holding D container logs back to back (doc_off[D+1] byte offsets).
// Pipeline (HBM-bound; the blob is read twice, the 2nd time mostly from L2):
//   log_count   lane = 256-byte chunk: count line starts (str.splitlines separators: \n \r \r\n
//               \v \f \x1c \x1d \x1e U+0085 U+2028 U+2029; container starts).
//   log_scan    one workgroup: exclusive scan of the per-tile totals -> tile_base, n_lines.
//   log_match   lane = chunk again, persistent workgroups with the DFA in LDS: line ids from
//               the tile scan, UTF-8 decode, DFA step per code point (csrc/log_dfa_tables.h,
//               compiled from the 13 regexes with Python's IGNORECASE folds and \d digit set),
//               per-line OR of the state outputs.  A chunk starting mid-line warms the DFA up
//               over the preceding <= 23 code points (the longest pattern is 23 long, so the DFA
//               state depends on no more).  Line pieces that straddle chunks are combined in LDS
//               by the owning lane; only lines straddling a 64 KiB tile use an atomic OR
//               (deterministic: OR is order-free).
//   log_hist    lane per container: one binary search for its first line (the next lane's is its
//               end), a private loop over <= 32 line masks, or the whole wave (13 ballots per 64
//               lines) for a larger container — counts and first three line ids per bin, no atomics.
#include <stdint.h>

#include "krca_common.h"
#define KRCA_DFA_QUAL static __device__ __constant__ const
#include "log_dfa_tables.h"

namespace {

constexpr int TPB = 256;
constexpr int CH = 256;               // bytes per lane-chunk
constexpr int64_t TILE = (int64_t)TPB * CH;  // bytes per workgroup tile
constexpr int WARM = 23;              // code points of DFA warm-up (longest pattern length)

// ---- byte access with a 16-byte register window ------------------------------------------
struct Bytes {
  const uint8_t* t;
  int64_t n;
  int64_t base;
  uint32_t w0, w1, w2, w3;
  __device__ void init(const uint8_t* text, int64_t nbytes) {
    t = text;
    n = nbytes;
    base = -1;
  }
  __device__ __forceinline__ void fill(int64_t b) {
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
  __device__ __forceinline__ uint32_t at(int64_t p) {
    const int64_t b = p & ~(int64_t)15;
    if (b != base) fill(b);
    const int q = (int)((p >> 2) & 3);
    const uint32_t w = q == 0 ? w0 : (q == 1 ? w1 : (q == 2 ? w2 : w3));
    return (w >> (8 * (int)(p & 3))) & 0xFFu;
  }
};

__device__ __forceinline__ bool is_ascii_sep(uint32_t b) {
  return b == 0x0A || b == 0x0B || b == 0x0C || b == 0x0D || b == 0x1C || b == 0x1D || b == 0x1E;
}

// a separator ends at p-1, given bytes b3 b2 b1 = text[p-3..p-1] (0 outside the container)
// and b0 = text[p] (0 at the container end): position p starts a line (if inside the container)
__device__ __forceinline__ bool sep_before(uint32_t b3, uint32_t b2, uint32_t b1, uint32_t b0) {
  if (b1 == 0x0D) return b0 != 0x0A;
  if (b1 == 0x0A || b1 == 0x0B || b1 == 0x0C || b1 == 0x1C || b1 == 0x1D || b1 == 0x1E) return true;
  if (b2 == 0xC2 && b1 == 0x85) return true;
  return b3 == 0xE2 && b2 == 0x80 && (b1 == 0xA8 || b1 == 0xA9);
}

// The container window of a lane: the current container d and the next boundaries off[d .. d+4]
// held in registers, refilled one load ahead, so crossing a container boundary (a ~184-byte
// container per 256-byte chunk at C5) does not wait on a dependent global load.
struct DocWin {
  const int64_t* off;
  int64_t D, d;
  int64_t b[5];
  __device__ __forceinline__ void load(const int64_t* o, int64_t nd, int64_t d0) {
    off = o;
    D = nd;
    d = d0;
#pragma unroll
    for (int i = 0; i < 5; ++i) b[i] = d0 + i <= nd ? o[d0 + i] : INT64_MAX;
  }
  // move to the container holding byte p (skipping empty containers sitting at p)
  __device__ __forceinline__ void advance(int64_t p) {
    while (d + 1 < D && b[1] <= p) {
      ++d;
#pragma unroll
      for (int i = 0; i < 4; ++i) b[i] = b[i + 1];
      b[4] = d + 4 <= D ? off[d + 4] : INT64_MAX;
    }
  }
};

// chunk -> container holding its first byte: one thread per container writes the chunks that start
// inside it (every chunk start lies in exactly one non-empty container), so no chunk searches
__global__ __launch_bounds__(TPB) void log_chunk_doc(const int64_t* __restrict__ doc_off, int64_t D,
                                                     int32_t* __restrict__ chunk_doc) {
  const int64_t d = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (d >= D) return;
  const int64_t s = doc_off[d], e = doc_off[d + 1];
  for (int64_t c = (s + CH - 1) / CH; c * CH < e; ++c) chunk_doc[c] = (int32_t)d;
}

// ---- phase 1: line starts per chunk ---------------------------------------------------------
__global__ __launch_bounds__(TPB) void log_count(const uint8_t* __restrict__ text, int64_t nbytes,
                                                 const int64_t* __restrict__ doc_off, int64_t D,
                                                 const int32_t* __restrict__ chunk_doc,
                                                 int32_t* __restrict__ chunk_cnt, int64_t* __restrict__ tile_tot) {
  __shared__ int32_t red[TPB / 64];
  const int64_t g = (int64_t)blockIdx.x * TPB + threadIdx.x;
  const int64_t c0 = g * CH;
  int32_t cnt = 0;
  if (c0 < nbytes) {
    const int64_t c1 = min(c0 + CH, nbytes);
    Bytes B;
    B.init(text, nbytes);
    DocWin dw;
    dw.load(doc_off, D, chunk_doc[g]);
    int64_t dstart = dw.b[0], dend = dw.b[1];
    uint32_t b1 = c0 - 1 >= dstart ? B.at(c0 - 1) : 0;
    uint32_t b2 = c0 - 2 >= dstart ? B.at(c0 - 2) : 0;
    uint32_t b3 = c0 - 3 >= dstart ? B.at(c0 - 3) : 0;
    for (int64_t p = c0; p < c1; ++p) {
      if (p >= dend) {  // next container(s)
        dw.advance(p);
        dstart = dw.b[0];
        dend = dw.b[1];
        b1 = b2 = b3 = 0;
      }
      const uint32_t b0 = B.at(p);
      cnt += (p == dstart) || sep_before(b3, b2, b1, b0);
      b3 = b2;
      b2 = b1;
      b1 = b0;
    }
  }
  chunk_cnt[g] = cnt;
  int32_t s = cnt;
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) tile_tot[blockIdx.x] = (int64_t)red[0] + red[1] + red[2] + red[3];
}

// ---- phase 2: exclusive scan of tile totals (one workgroup) --------------------------------
__global__ __launch_bounds__(1024) void log_scan(int64_t* __restrict__ tile, int64_t ntiles, int64_t* __restrict__ n_lines) {
  __shared__ int64_t wsum[16];
  __shared__ int64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int64_t b = 0; b < ntiles; b += 1024) {
    const int64_t i = b + threadIdx.x;
    const int64_t v = i < ntiles ? tile[i] : 0;
    int64_t x = v;  // inclusive wave scan
    for (int off = 1; off < 64; off <<= 1) {
      const int64_t y = (int64_t)__shfl_up((long long)x, off, 64);
      if (lane >= off) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    int64_t before = carry;
    for (int w = 0; w < wid; ++w) before += wsum[w];
    if (i < ntiles) tile[i] = before + x - v;  // exclusive
    __syncthreads();
    if (threadIdx.x == 1023) carry = before + x;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    tile[ntiles] = carry;
    *n_lines = carry;
  }
}

// ---- phase 3: DFA per chunk ----------------------------------------------------------------
struct DfaLds {
  uint16_t trans[KRCA_DFA_NSTATE * KRCA_DFA_NSYM];
  uint16_t out[KRCA_DFA_NSTATE];
  uint8_t ascii[128];
};

__device__ __forceinline__ uint32_t cp_symbol(const DfaLds& dfa, uint32_t cp) {
  if (cp < 128) return dfa.ascii[cp];
  int lo = 0, hi = KRCA_DFA_NRANGE - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    if (cp < krca_dfa_ranges[mid][0]) hi = mid - 1;
    else if (cp > krca_dfa_ranges[mid][1]) lo = mid + 1;
    else return krca_dfa_ranges[mid][2];
  }
  return KRCA_DFA_OTHER;
}

// decode the code point starting at p (valid UTF-8 or surrogatepass); returns its byte length
__device__ __forceinline__ int decode(Bytes& B, int64_t p, uint32_t& cp) {
  const uint32_t b = B.at(p);
  if (b < 0x80) {
    cp = b;
    return 1;
  }
  if (b < 0xE0) {
    cp = ((b & 0x1F) << 6) | (B.at(p + 1) & 0x3F);
    return 2;
  }
  if (b < 0xF0) {
    cp = ((b & 0x0F) << 12) | ((B.at(p + 1) & 0x3F) << 6) | (B.at(p + 2) & 0x3F);
    return 3;
  }
  cp = ((b & 0x07) << 18) | ((B.at(p + 1) & 0x3F) << 12) | ((B.at(p + 2) & 0x3F) << 6) | (B.at(p + 3) & 0x3F);
  return 4;
}

__device__ __forceinline__ int64_t cp_align(Bytes& B, int64_t p, int64_t lim) {
  while (p < lim && (B.at(p) & 0xC0) == 0x80) ++p;
  return p;
}

__global__ __launch_bounds__(TPB) void log_match(const uint8_t* __restrict__ text, int64_t nbytes,
                                                 const int64_t* __restrict__ doc_off, int64_t D,
                                                 const int32_t* __restrict__ chunk_doc,
                                                 const int32_t* __restrict__ chunk_cnt,
                                                 const int64_t* __restrict__ tile_base, int64_t ntiles, int64_t L,
                                                 int64_t* __restrict__ line_start, int64_t* __restrict__ line_end,
                                                 uint32_t* __restrict__ line_mask) {
  __shared__ DfaLds dfa;
  __shared__ int64_t s_scan[TPB];
  __shared__ int64_t s_first_id[TPB];
  __shared__ uint32_t s_first_mask[TPB];
  __shared__ int32_t s_first_closed[TPB];
  for (int i = threadIdx.x; i < KRCA_DFA_NSTATE * KRCA_DFA_NSYM; i += TPB) dfa.trans[i] = krca_dfa_trans[i];
  for (int i = threadIdx.x; i < KRCA_DFA_NSTATE; i += TPB) dfa.out[i] = krca_dfa_out[i];
  for (int i = threadIdx.x; i < 128; i += TPB) dfa.ascii[i] = krca_dfa_ascii_sym[i];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;

  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    // exclusive scan of the tile's chunk counts -> first line id of this lane's chunk
    const int64_t g = tile * TPB + threadIdx.x;
    const int64_t v = chunk_cnt[g];
    int64_t x = v;
    for (int off = 1; off < 64; off <<= 1) {
      const int64_t y = (int64_t)__shfl_up((long long)x, off, 64);
      if (lane >= off) x += y;
    }
    __syncthreads();  // protects s_scan / s_first_* of the previous tile and the DFA fill
    if (lane == 63) s_scan[wid] = x;
    __syncthreads();
    int64_t base = tile_base[tile];
    for (int w = 0; w < wid; ++w) base += s_scan[w];
    base += x - v;

    const int64_t c0 = g * CH;
    int64_t first_id = -1;
    uint32_t first_mask = 0;
    int32_t first_closed = 0;
    int64_t tail_id = -1;  // a line this lane opened and did not close
    uint32_t tail_mask = 0;
    if (c0 < nbytes) {
      const int64_t c1 = min(c0 + CH, nbytes);
      Bytes B;
      B.init(text, nbytes);
      DocWin dw;
      dw.load(doc_off, D, chunk_doc[g]);
      int64_t dstart = dw.b[0], dend = dw.b[1];
      const int64_t p0 = cp_align(B, c0, dend);  // first code point starting in this chunk
      int64_t cur = base - 1;  // id of the open line (lines before this chunk: base)
      bool open = false, own = false, after_sep = false, prev_cr = false;
      uint32_t st = 0, mask = 0;
      if (p0 < dend && p0 > dstart) {
        const uint32_t b1 = B.at(p0 - 1);
        const uint32_t b2 = p0 - 2 >= dstart ? B.at(p0 - 2) : 0;
        const uint32_t b3 = p0 - 3 >= dstart ? B.at(p0 - 3) : 0;
        const uint32_t b0 = B.at(p0);
        if (b1 == 0x0D) {
          after_sep = true;
          prev_cr = true;
        } else if (sep_before(b3, b2, b1, b0)) {
          after_sep = true;
        } else {
          open = true;  // continuation of line `cur` opened by an earlier chunk
          // DFA warm-up over the preceding <= WARM code points of this line
          int64_t k = p0;
          int seen = 0;
          while (k > dstart && seen < WARM) {
            const uint32_t b = B.at(k - 1);
            if (is_ascii_sep(b)) break;
            --k;
            if ((b & 0xC0) != 0x80) ++seen;
          }
          while (k < p0) {
            uint32_t cp;
            const int len = decode(B, k, cp);
            const uint32_t sym = cp_symbol(dfa, cp);
            st = sym == KRCA_DFA_SEP ? 0u : dfa.trans[st * KRCA_DFA_NSYM + sym];
            k += len;
          }
          // pieces before p0 belong to earlier chunks; only the state is carried over
        }
      }
      int64_t p = p0;
      // process code points starting in [p0, c1) (the last one may extend past c1)
      while (p < c1) {
        if (p >= dend) {  // container end: close its open last line, enter the next container
          if (open) {
            if (cur < L) line_end[cur] = dend;
            if (own && cur < L) line_mask[cur] = mask;
            else {
              first_id = cur;
              first_mask = mask;
              first_closed = 1;
            }
            open = false;
          }
          dw.advance(p);
          dstart = dw.b[0];
          dend = dw.b[1];
          after_sep = false;
          prev_cr = false;
        }
        uint32_t cp;
        const int len = decode(B, p, cp);
        if (p == dstart || after_sep) {
          if (after_sep && prev_cr && cp == 0x0A) {  // second byte of "\r\n"
            prev_cr = false;
            p += len;
            continue;
          }
          ++cur;  // a new line starts here
          if (cur < L) line_start[cur] = p;
          open = true;
          own = true;
          after_sep = false;
          prev_cr = false;
          st = 0;
          mask = 0;
        }
        const uint32_t sym = cp_symbol(dfa, cp);
        if (sym == KRCA_DFA_SEP) {
          if (open) {
            if (cur < L) line_end[cur] = p;
            if (own && cur < L) line_mask[cur] = mask;
            else {
              first_id = cur;
              first_mask = mask;
              first_closed = 1;
            }
          }
          open = false;
          after_sep = true;
          prev_cr = cp == 0x0D;
          st = 0;
        } else {
          st = dfa.trans[st * KRCA_DFA_NSYM + sym];
          mask |= dfa.out[st];
        }
        p += len;
      }
      if (open && p >= dend) {  // the container ends exactly at the chunk end
        if (cur < L) line_end[cur] = dend;
        if (own && cur < L) line_mask[cur] = mask;
        else {
          first_id = cur;
          first_mask = mask;
          first_closed = 1;
        }
        open = false;
      }
      if (open) {
        if (own) {
          tail_id = cur;
          tail_mask = mask;
        } else {  // the line crosses this whole chunk
          first_id = cur;
          first_mask = mask;
          first_closed = 0;
        }
      }
    }
    s_first_id[threadIdx.x] = first_id;
    s_first_mask[threadIdx.x] = first_mask;
    s_first_closed[threadIdx.x] = first_closed;
    __syncthreads();
    // owners of open lines collect the continuation pieces of the following lanes
    if (tail_id >= 0 && tail_id < L) {
      uint32_t m = tail_mask;
      bool closed = false;
      for (int j = threadIdx.x + 1; j < TPB && s_first_id[j] == tail_id; ++j) {
        m |= s_first_mask[j];
        if (s_first_closed[j]) {
          closed = true;
          break;
        }
      }
      if (closed) line_mask[tail_id] = m;
      else atomicOr(&line_mask[tail_id], m);  // continues into the next tile
    }
    // lane 0 finishes a line opened in an earlier tile
    if (threadIdx.x == 0 && s_first_id[0] >= 0 && s_first_id[0] < L) {
      const int64_t id = s_first_id[0];
      uint32_t m = 0;
      for (int j = 0; j < TPB && s_first_id[j] == id; ++j) {
        m |= s_first_mask[j];
        if (s_first_closed[j]) break;
      }
      atomicOr(&line_mask[id], m);
    }
  }
}

// ---- phase 4: per-container histogram + first three examples (wave per container) ----------
__device__ __forceinline__ int64_t lower_bound_i64(const int64_t* __restrict__ a, int64_t n, int64_t key) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// One lane per container: its first line by one binary search over line_start (the next lane's
// result is its end), then, for a container of <= 32 lines, a private loop over the line masks;
// larger containers are taken by the whole wave one at a time (13 ballots per 64 lines give the
// counts and the first three line ids per bin).  No atomics; ~1M containers of ~2.5 lines are
// one pass of short lane loops instead of a wave (and two dependent searches) each.
constexpr int HIST_SMALL = 32;

__global__ __launch_bounds__(TPB) void log_hist(const int64_t* __restrict__ doc_off, int64_t D,
                                                const int64_t* __restrict__ line_start,
                                                const uint32_t* __restrict__ line_mask, int64_t L,
                                                int32_t* __restrict__ doc_lines, int32_t* __restrict__ hist,
                                                int32_t* __restrict__ examples, int64_t* __restrict__ doc_line0) {
  const int64_t d = (int64_t)blockIdx.x * TPB + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const bool valid = d < D;
  const int64_t lo = valid ? lower_bound_i64(line_start, L, doc_off[d]) : L;
  int64_t hi = __shfl_down(lo, 1, 64);
  if (valid && (lane == 63 || d + 1 == D)) hi = lower_bound_i64(line_start, L, doc_off[d + 1]);
  const bool small = valid && hi - lo <= HIST_SMALL;
  if (small) {
    int32_t cnt[KRCA_NCAT], ex[KRCA_NCAT][3];
#pragma unroll
    for (int c = 0; c < KRCA_NCAT; ++c) {
      cnt[c] = 0;
      ex[c][0] = ex[c][1] = ex[c][2] = -1;
    }
    for (int64_t l = lo; l < hi; ++l) {
      const uint32_t m = line_mask[l];
#pragma unroll
      for (int c = 0; c < KRCA_NCAT; ++c) {
        if ((m >> c) & 1u) {
          const int f = cnt[c];
          if (f == 0) ex[c][0] = (int32_t)l;
          if (f == 1) ex[c][1] = (int32_t)l;
          if (f == 2) ex[c][2] = (int32_t)l;
          cnt[c] = f + 1;
        }
      }
    }
    doc_lines[d] = (int32_t)(hi - lo);
    if (doc_line0) doc_line0[d] = lo;
    int32_t* hd = hist + d * KRCA_NCAT;
    int32_t* ed = examples + d * KRCA_NCAT * 3;
#pragma unroll
    for (int c = 0; c < KRCA_NCAT; ++c) {
      hd[c] = cnt[c];
      ed[c * 3] = ex[c][0];
      ed[c * 3 + 1] = ex[c][1];
      ed[c * 3 + 2] = ex[c][2];
    }
  }
  uint64_t big = __ballot(valid && !small);
  while (big) {  // wave-uniform: the wave takes the large containers one at a time
    const int j = __ffsll((unsigned long long)big) - 1;
    big &= big - 1;
    const int64_t dj = d - lane + j;
    const int64_t blo = __shfl(lo, j, 64), bhi = __shfl(hi, j, 64);
    int32_t cnt[KRCA_NCAT];
    int32_t found[KRCA_NCAT];
#pragma unroll
    for (int c = 0; c < KRCA_NCAT; ++c) {
      cnt[c] = 0;
      found[c] = 0;
    }
    int32_t* ex = examples + dj * KRCA_NCAT * 3;
    for (int64_t b = blo; b < bhi; b += 64) {
      const uint32_t m = (b + lane < bhi) ? line_mask[b + lane] : 0u;
#pragma unroll
      for (int c = 0; c < KRCA_NCAT; ++c) {
        uint64_t bal = __ballot((m >> c) & 1u);
        cnt[c] += __popcll(bal);
        while (found[c] < 3 && bal) {
          const int q = __ffsll((unsigned long long)bal) - 1;
          if (lane == 0) ex[c * 3 + found[c]] = (int32_t)(b + q);
          ++found[c];
          bal &= bal - 1;
        }
      }
    }
    if (lane == 0) {
      doc_lines[dj] = (int32_t)(bhi - blo);
      if (doc_line0) doc_line0[dj] = blo;
#pragma unroll
      for (int c = 0; c < KRCA_NCAT; ++c) {
        hist[dj * KRCA_NCAT + c] = cnt[c];
        for (int k = found[c]; k < 3; ++k) ex[c * 3 + k] = -1;
      }
    }
  }
}

int64_t num_tiles(int64_t nbytes) { return std::max<int64_t>(1, krca::ceil_div(nbytes, TILE)); }

}  // namespace

extern "C" {

// workspace (int64 units): [ntiles+1] tile base | [ntiles*TPB] int32 chunk counts |
// [ntiles*TPB] int32 chunk -> container
int64_t krca_log_index_size(int64_t nbytes) {
  const int64_t nt = num_tiles(nbytes);
  return (nt + 1) + 2 * krca::ceil_div(nt * TPB, 2) + 2;
}

int krca_log_index(const uint8_t* text, int64_t nbytes, const int64_t* doc_off, int64_t ndocs, int64_t* ws,
                   int64_t* n_lines, void* stream) {
  KRCA_CHECK_ARG(nbytes >= 0 && ndocs >= 1, "krca_log_index: need nbytes >= 0 and ndocs >= 1");
  KRCA_CHECK_ARG(doc_off && ws && n_lines, "krca_log_index: null pointer");
  KRCA_CHECK_ARG(nbytes == 0 || text, "krca_log_index: null text");
  KRCA_CHECK_ARG(((uintptr_t)text & 15) == 0, "krca_log_index: text must be 16-byte aligned");
  const int64_t nt = num_tiles(nbytes);
  KRCA_CHECK_ARG(ndocs < INT32_MAX, "krca_log_index: too many containers");
  int64_t* tile = ws;
  int32_t* chunk = reinterpret_cast<int32_t*>(ws + nt + 1);
  int32_t* cdoc = chunk + 2 * krca::ceil_div(nt * TPB, 2);
  hipStream_t st = krca::as_stream(stream);
  hipLaunchKernelGGL(log_chunk_doc, dim3((unsigned)krca::ceil_div(ndocs, TPB)), dim3(TPB), 0, st, doc_off, ndocs, cdoc);
  KRCA_LAUNCH_CHECK();
  hipLaunchKernelGGL(log_count, dim3((unsigned)nt), dim3(TPB), 0, st, text, nbytes, doc_off, ndocs,
                     (const int32_t*)cdoc, chunk, tile);
  KRCA_LAUNCH_CHECK();
  hipLaunchKernelGGL(log_scan, dim3(1), dim3(1024), 0, st, tile, nt, n_lines);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_log_match(const uint8_t* text, int64_t nbytes, const int64_t* doc_off, int64_t ndocs, const int64_t* ws,
                   int64_t n_lines, int64_t* line_start, int64_t* line_end, uint32_t* line_mask, int32_t* doc_lines,
                   int32_t* hist, int32_t* examples, int64_t* doc_line0, void* stream) {
  KRCA_CHECK_ARG(nbytes >= 0 && ndocs >= 1 && n_lines >= 0, "krca_log_match: bad sizes");
  KRCA_CHECK_ARG(doc_off && ws && doc_lines && hist && examples, "krca_log_match: null pointer");
  KRCA_CHECK_ARG(((uintptr_t)text & 15) == 0, "krca_log_match: text must be 16-byte aligned");
  KRCA_CHECK_ARG(n_lines == 0 || (line_start && line_end && line_mask), "krca_log_match: null line arrays");
  const int64_t nt = num_tiles(nbytes);
  const int64_t* tile = ws;
  const int32_t* chunk = reinterpret_cast<const int32_t*>(ws + nt + 1);
  const int32_t* cdoc = chunk + 2 * krca::ceil_div(nt * TPB, 2);
  hipStream_t st = krca::as_stream(stream);
  if (n_lines > 0) {
    KRCA_HIP(hipMemsetAsync(line_mask, 0, n_lines * sizeof(uint32_t), st));
    const int64_t grid = std::min<int64_t>(nt, 256 * 4);
    hipLaunchKernelGGL(log_match, dim3((unsigned)grid), dim3(TPB), 0, st, text, nbytes, doc_off, ndocs, cdoc, chunk,
                       tile, nt, n_lines, line_start, line_end, line_mask);
    KRCA_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(log_hist, dim3((unsigned)krca::ceil_div(ndocs, TPB)), dim3(TPB), 0, st, doc_off, ndocs,
                     line_start, line_mask, n_lines, doc_lines, hist, examples, doc_line0);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

}  // extern "C"

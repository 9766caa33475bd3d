// 13-category log line histograms.
//
// Exactly reproduces, for every container log text, ref:agents/logs_agent.py:140-151:
//   lines = text.splitlines();  bin c = number of lines with re.search(pattern_c, line, re.I)
// plus the first three matching lines per bin (the evidence of :159-163) and len(lines).
//
// Input: one UTF-8 blob holding D container logs back to back (doc_off[D+1] byte offsets).
// krca_log_scan (one call, one stream synchronisation for the line count):
//   log_chunk_doc     thread per container: the 256-byte chunk -> container map; zeroes the
//                     look-back status words, the tile ticket and the queue counts.
//   log_index_lines   persistent workgroups take 64 KiB tiles in ticket order: line-start bits and
//                     separator lengths per 16-byte piece (str.splitlines separators: \n \r \r\n \v
//                     \f \x1c \x1d \x1e U+0085 U+2028 U+2029; container starts from a per-tile LDS
//                     bitmap), chunk counts, the tile's first line id by a decoupled look-back,
//                     line_start / line_end written.  Containers are valid UTF-8 each, so no
//                     multi-byte separator straddles two of them.
//   log_dfa           lane per line, lockstep 16-byte blocks, the 13-pattern DFA
//                     (csrc/log_dfa_tables.h: the 13 regexes with Python's IGNORECASE folds and \d)
//                     from an LDS table; lines over 1 KiB queue for log_dfa_long (a wave per line,
//                     64 segments each warmed up over the <= 23 code points before it).
//   log_hist          lane per container (or a wave for a large one): 13 counts, the first three
//                     example lines per bin marked in the line masks, no atomics.
// A/B paths (tests require identical outputs): KRCA_LOG_FUSED = 1 / 2, log_index_match walking the
// DFA inside the index pass from the LDS-resident tile (+ the LOOK bytes after it, for its last line);
// KRCA_LOG_IMPL = 1, the chunk-lane log_match; = 2, the round-1 walk log_dfa_window.  When the
// caller's line arrays are too small, krca_log_match finishes from the index in the workspace.
#include <stdint.h>
#include <cstdlib>

#include <algorithm>
#include <type_traits>

#include "krca_common.h"
#define KRCA_DFA_QUAL static __device__ __constant__ const
#include "log_dfa_tables.h"

#ifndef LOG_IDX_BATCH
#define LOG_IDX_BATCH 4  // pieces per lane whose loads log_index_lines' first phase issues together
#endif
#ifndef LOG_IDX_PERSIST
#define LOG_IDX_PERSIST 1  // log_index_lines: resident workgroups loop over the tiles (0: one tile each)
#endif

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
  // b is 16-byte aligned and (callers read only p < n) holds at least one byte of the text: the
  // aligned 16-byte block lies inside the text's last page, so the full load never faults; bytes
  // past n are never returned by at()
  __device__ __forceinline__ void fill(int64_t b) {
    base = b;
    const uint4 v = *reinterpret_cast<const uint4*>(t + b);
    w0 = v.x;
    w1 = v.y;
    w2 = v.z;
    w3 = v.w;
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

// byte k (0..3) of a little-endian word
__device__ __forceinline__ uint32_t byte_of(uint32_t w, int k) { return (w >> (8 * k)) & 0xFFu; }

// chunk -> container holding its first byte: one thread per container writes the chunks that start
// inside it (every chunk start lies in exactly one non-empty container), so no chunk searches.
// (Line starts at container first bytes are counted by log_count from its tile bitmap: every
// container is valid UTF-8 on its own, so away from those bytes the raw separator test is exact.)
// doc_off outside the contract (include/krca.h) is clamped to [0, nbytes] so no write leaves the map.
// (krca_log_scan: also zeroes the look-back status words + ticket and the long-line count, so the
// scan needs no memset launches of its own)
__global__ __launch_bounds__(TPB) void log_chunk_doc(const int64_t* __restrict__ doc_off, int64_t D, int64_t nbytes,
                                                     int32_t* __restrict__ chunk_doc,
                                                     unsigned long long* __restrict__ zero64, int64_t n_zero64,
                                                     int32_t* __restrict__ zero32) {
  const int64_t d = (int64_t)blockIdx.x * TPB + threadIdx.x;
  for (int64_t i = d; i < n_zero64; i += (int64_t)gridDim.x * TPB) zero64[i] = 0ull;
  if (d == 0 && zero32) *zero32 = 0;
  if (d >= D) return;
  const int64_t s = min(max(doc_off[d], (int64_t)0), nbytes);
  const int64_t e = min(max(doc_off[d + 1], s), nbytes);
  for (int64_t c = (s + CH - 1) / CH; c * CH < e; ++c) chunk_doc[c] = (int32_t)d;
}

// ---- phase 1: line starts per chunk (streaming) -------------------------------------------
// A workgroup takes one 64 KiB tile in 16 passes of 4 KiB; a lane reads 16 consecutive bytes
// (one coalesced dwordx4 per lane: a wave reads 1 KiB contiguous), the 3 bytes before them come
// from the previous lane by a shuffle (lane 0: one extra 4-byte load).  16 lanes = one 256-byte
// chunk: count = line starts = raw separator tests OR non-empty container first bytes.
constexpr int PIECE = 16;
constexpr int LANES_PER_CHUNK = CH / PIECE;  // 16

// SWAR byte tests on 4 bytes at once: the high bit of each byte of the result is the test
__device__ __forceinline__ uint32_t swar_eq(uint32_t x, uint32_t c) {  // byte == c
  const uint32_t v = x ^ (c * 0x01010101u);
  return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v) & 0x80808080u;
}
__device__ __forceinline__ uint32_t swar_range(uint32_t x, uint32_t lo, uint32_t hi) {  // lo <= byte <= hi < 0x80
  const uint32_t y = x & 0x7F7F7F7Fu;
  const uint32_t ge = y + (0x80u - lo) * 0x01010101u;
  const uint32_t gt = y + (0x7Fu - hi) * 0x01010101u;
  return ge & ~gt & ~x & 0x80808080u;
}

// line starts at the 4 byte positions of word w (sep_before of each, raw bytes), given the word
// before it; high bit per byte
__device__ __forceinline__ uint32_t sep_flags(uint32_t wprev, uint32_t w) {
  const uint32_t B1 = __builtin_amdgcn_alignbit(w, wprev, 24);  // text[p-1] at byte k
  uint32_t f = (swar_range(B1, 0x0A, 0x0D) | swar_range(B1, 0x1C, 0x1E)) & ~(swar_eq(B1, 0x0D) & swar_eq(w, 0x0A));
  if ((w | wprev) & 0x80808080u) {  // U+0085 (C2 85), U+2028 / U+2029 (E2 80 A8/A9)
    const uint32_t B2 = __builtin_amdgcn_alignbit(w, wprev, 16);
    const uint32_t B3 = __builtin_amdgcn_alignbit(w, wprev, 8);
    f |= swar_eq(B2, 0xC2) & swar_eq(B1, 0x85);
    f |= swar_eq(B3, 0xE2) & swar_eq(B2, 0x80) & (swar_eq(B1, 0xA8) | swar_eq(B1, 0xA9));
  }
  return f;
}

// The tile's non-empty container starts in [tile0-1, tile0+TILE) as bits of s_cs (bit j = byte
// tile0-32+j): one coalesced pass over doc_off from the container holding byte tile0-1 (chunk_doc),
// instead of a dependent doc_off walk per 16-byte piece.  Used by log_count and log_lines.
constexpr int NBW = (int)(TILE / 32) + 2;  // bytes tile0-32 .. tile0+TILE+31
// ZEROED: the caller cleared s_cs after its last read of the previous tile's bitmap (behind a
// barrier), so no clearing pass and barrier here; the chunk_doc load goes out before either.
template <int64_t TL, bool ZEROED = false>
__device__ __forceinline__ void tile_container_starts_t(uint32_t* s_cs, int64_t tile0, int64_t nbytes,
                                                        const int64_t* __restrict__ doc_off, int64_t D,
                                                        const int32_t* __restrict__ chunk_doc) {
  constexpr int NB = (int)(TL / 32) + 2;
  int64_t k0 = tile0 < nbytes ? chunk_doc[(tile0 > 0 ? tile0 - 1 : 0) / CH] : D;
  if (!ZEROED) {
    for (int i = threadIdx.x; i < NB; i += blockDim.x) s_cs[i] = 0u;
    __syncthreads();
  }
  const int64_t tend = tile0 + TL;
  k0 = k0 < 0 ? 0 : (k0 > D ? D : k0);  // memory safety only: the map is exact under the doc_off contract
  for (int64_t kb = k0;; kb += blockDim.x) {
    const int64_t k = kb + threadIdx.x;
    const int64_t st = k < D ? doc_off[k] : INT64_MAX;
    if (st >= tile0 - 1 && st < tend && doc_off[k + 1] > st) {
      const int64_t j = st - (tile0 - 32);
      atomicOr(&s_cs[j >> 5], 1u << (int)(j & 31));
    }
    if (__syncthreads_or(st >= tend)) break;  // doc_off is sorted: no later container starts inside
  }
}
__device__ __forceinline__ void tile_container_starts(uint32_t* s_cs, int64_t tile0, int64_t nbytes,
                                                      const int64_t* __restrict__ doc_off, int64_t D,
                                                      const int32_t* __restrict__ chunk_doc) {
  tile_container_starts_t<TILE>(s_cs, tile0, nbytes, doc_off, D, chunk_doc);
}

// container first bytes at q-1+j, j = 0..16, from the tile bitmap
__device__ __forceinline__ uint32_t piece_container_starts(const uint32_t* s_cs, int64_t tile0, int64_t q) {
  const int j = (int)(q - 1 - (tile0 - 32));
  const uint64_t two = ((uint64_t)s_cs[(j >> 5) + 1] << 32) | s_cs[j >> 5];
  return (uint32_t)(two >> (j & 31)) & 0x1FFFFu;
}

__device__ __forceinline__ uint32_t high_bits4(uint32_t f) {  // byte high bits -> 4-bit mask
  return ((f >> 7) & 1u) | ((f >> 14) & 2u) | ((f >> 21) & 4u) | ((f >> 28) & 8u);
}

__global__ __launch_bounds__(TPB) void log_count(const uint8_t* __restrict__ text, int64_t nbytes,
                                                 const int64_t* __restrict__ doc_off, int64_t D,
                                                 const int32_t* __restrict__ chunk_doc,
                                                 int32_t* __restrict__ chunk_cnt, int64_t* __restrict__ tile_tot) {
  constexpr int NIT = TILE / (TPB * PIECE);  // 16 passes of 4 KiB
  __shared__ int32_t s_cnt[TPB];             // the tile's 256 chunk counts
  __shared__ int64_t red[TPB / 64];
  __shared__ uint32_t s_cs[NBW];
  const int lane = threadIdx.x & 63;
  const int64_t tile0 = (int64_t)blockIdx.x * TILE;
  s_cnt[threadIdx.x] = 0;
  tile_container_starts(s_cs, tile0, nbytes, doc_off, D, chunk_doc);  // (its barriers cover s_cnt)
#pragma unroll 4
  for (int it = 0; it < NIT; ++it) {
    const int64_t q = tile0 + (int64_t)it * TPB * PIECE + (int64_t)threadIdx.x * PIECE;
    uint32_t w[4] = {0, 0, 0, 0};
    if (q + PIECE <= nbytes) {
      const uint4 v = *reinterpret_cast<const uint4*>(text + q);
      w[0] = v.x;
      w[1] = v.y;
      w[2] = v.z;
      w[3] = v.w;
    } else if (q < nbytes) {
      for (int k = 0; k < PIECE; ++k)
        if (q + k < nbytes) w[k >> 2] |= (uint32_t)text[q + k] << (8 * (k & 3));
    }
    uint32_t wp = __shfl_up(w[3], 1, 64);  // bytes q-4 .. q-1
    if (lane == 0) wp = q >= 4 && q <= nbytes ? *reinterpret_cast<const uint32_t*>(text + q - 4) : 0u;
    uint32_t f0 = sep_flags(wp, w[0]), f1 = sep_flags(w[0], w[1]), f2 = sep_flags(w[1], w[2]),
             f3 = sep_flags(w[2], w[3]);
    if (q + PIECE > nbytes) {  // positions past the text are no line starts
      const int64_t n = nbytes - q;  // < 16
      f0 &= n >= 4 ? ~0u : (n <= 0 ? 0u : (0x80808080u >> (8 * (4 - n))));
      f1 &= n >= 8 ? ~0u : (n <= 4 ? 0u : (0x80808080u >> (8 * (8 - n))));
      f2 &= n >= 12 ? ~0u : (n <= 8 ? 0u : (0x80808080u >> (8 * (12 - n))));
      f3 &= n <= 12 ? 0u : (0x80808080u >> (8 * (16 - n)));
    }
    // a non-empty container's first byte starts a line whatever precedes it
    uint32_t S = high_bits4(f0) | (high_bits4(f1) << 4) | (high_bits4(f2) << 8) | (high_bits4(f3) << 12);
    if (q < nbytes) {
      S |= piece_container_starts(s_cs, tile0, q) >> 1;
      if (q + PIECE > nbytes) S &= (1u << (int)(nbytes - q)) - 1u;
    }
    uint32_t c = __popc(S);
#pragma unroll
    for (int o = LANES_PER_CHUNK / 2; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);  // 16 lanes = one chunk
    if ((threadIdx.x & (LANES_PER_CHUNK - 1)) == 0)
      s_cnt[it * (TPB / LANES_PER_CHUNK) + threadIdx.x / LANES_PER_CHUNK] += (int32_t)c;
  }
  __syncthreads();
  const int32_t mine = s_cnt[threadIdx.x];
  chunk_cnt[(int64_t)blockIdx.x * TPB + threadIdx.x] = mine;
  int64_t tot = mine;
  for (int off = 32; off > 0; off >>= 1) tot += __shfl_xor(tot, off, 64);
  if (lane == 0) red[threadIdx.x >> 6] = tot;
  __syncthreads();
  if (threadIdx.x == 0) tile_tot[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
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
template <class SRC>
__device__ __forceinline__ int decode(SRC& B, int64_t p, uint32_t& cp) {
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
                                                 uint32_t* __restrict__ line_mask, int64_t* __restrict__ chunk_line0) {
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
    chunk_line0[g] = base;  // first line id of the chunk (narrows log_hist's search)

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
      dw.load(doc_off, D, min(max((int64_t)chunk_doc[g], (int64_t)0), D - 1));
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

// ---- phase 3 (default, KRCA_LOG_IMPL != 1): line index, then a DFA lane per line ---------------
// log_lines  re-streams the text like log_count (coalesced 16-byte pieces, SWAR separator tests)
//            plus the container starts of each piece, numbers every line start from the chunk
//            bases and writes line_start[id] and line_end[id-1] (the previous line ends at the
//            separator that precedes the start, or at its container's end).
// log_dfa    one lane per line: the line holds no separator and lies inside one container, so the
//            per-byte loop is just UTF-8 decode + DFA step + mask OR; lines longer than LONG_LINE
//            are queued for
// log_dfa_long  one wave per long line: 64 segments, each warmed up over the <= 23 code points
//            before it (as log_match's chunks), OR-reduced across the wave.
constexpr int LONG_LINE = 1024;

// bytes of the separator that ends right before p (0: none), from the raw bytes before p; p1_cs:
// p-1 is a container's first byte (then a "\r" before it belongs to the previous container)
__device__ __forceinline__ int sep_len(uint32_t b3, uint32_t b2, uint32_t b1, bool p1_cs) {
  if (b1 == 0x0A) return (b2 == 0x0D && !p1_cs) ? 2 : 1;
  if (b1 == 0x0B || b1 == 0x0C || b1 == 0x0D || b1 == 0x1C || b1 == 0x1D || b1 == 0x1E) return 1;
  if (b2 == 0xC2 && b1 == 0x85) return 2;
  if (b3 == 0xE2 && b2 == 0x80 && (b1 == 0xA8 || b1 == 0xA9)) return 3;
  return 0;
}

__global__ __launch_bounds__(TPB) void log_lines(const uint8_t* __restrict__ text, int64_t nbytes,
                                                 const int64_t* __restrict__ doc_off, int64_t D,
                                                 const int32_t* __restrict__ chunk_doc,
                                                 const int32_t* __restrict__ chunk_cnt,
                                                 const int64_t* __restrict__ tile_base, int64_t L,
                                                 int64_t* __restrict__ line_start, int64_t* __restrict__ line_end,
                                                 int64_t* __restrict__ chunk_line0) {
  constexpr int NIT = TILE / (TPB * PIECE);
  __shared__ int64_t s_base[TPB];
  __shared__ int64_t s_wsum[TPB / 64];
  __shared__ uint32_t s_cs[NBW];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t tile = blockIdx.x;
  const int64_t tile0 = tile * TILE;
  tile_container_starts(s_cs, tile0, nbytes, doc_off, D, chunk_doc);
  {  // first line id of each of the tile's 256 chunks
    const int64_t v = chunk_cnt[tile * TPB + threadIdx.x];
    int64_t x = v;
    for (int off = 1; off < 64; off <<= 1) {
      const int64_t y = (int64_t)__shfl_up((long long)x, off, 64);
      if (lane >= off) x += y;
    }
    if (lane == 63) s_wsum[wid] = x;
    __syncthreads();
    int64_t base = tile_base[tile] + x - v;
    for (int w = 0; w < wid; ++w) base += s_wsum[w];
    s_base[threadIdx.x] = base;
    chunk_line0[tile * TPB + threadIdx.x] = base;
    __syncthreads();
  }
  for (int it = 0; it < NIT; ++it) {
    const int64_t q = tile0 + (int64_t)it * TPB * PIECE + (int64_t)threadIdx.x * PIECE;
    uint32_t w[4] = {0, 0, 0, 0};
    if (q < nbytes) {  // an aligned 16-byte block holding a text byte never crosses the last page
      const uint4 v = *reinterpret_cast<const uint4*>(text + q);
      w[0] = v.x;
      w[1] = v.y;
      w[2] = v.z;
      w[3] = v.w;
    }
    uint32_t wp = __shfl_up(w[3], 1, 64);  // bytes q-4 .. q-1
    if (lane == 0) wp = q >= 4 && q <= nbytes ? *reinterpret_cast<const uint32_t*>(text + q - 4) : 0u;
    uint32_t S = high_bits4(sep_flags(wp, w[0])) | (high_bits4(sep_flags(w[0], w[1])) << 4) |
                 (high_bits4(sep_flags(w[1], w[2])) << 8) | (high_bits4(sep_flags(w[2], w[3])) << 12);
    uint32_t C = 0;  // container first bytes at q-1+j, j = 0..16 (non-empty containers only)
    if (q < nbytes) {
      C = piece_container_starts(s_cs, tile0, q);
      S |= C >> 1;
      if (q + PIECE > nbytes) S &= (1u << (int)(nbytes - q)) - 1u;
    } else {
      S = 0;
    }
    // line ids: the chunk's base + the starts of the lanes before this one in the chunk (16 lanes)
    const uint32_t n = __popc(S);
    uint32_t x = n;
#pragma unroll
    for (int off = 1; off < LANES_PER_CHUNK; off <<= 1) {
      const uint32_t y = __shfl_up(x, off, 64);
      if ((lane & (LANES_PER_CHUNK - 1)) >= off) x += y;
    }
    int64_t id = s_base[it * (TPB / LANES_PER_CHUNK) + threadIdx.x / LANES_PER_CHUNK] + (x - n);
    uint32_t rem = S;
    while (rem) {
      const int k = __ffs(rem) - 1;
      rem &= rem - 1;
      const int64_t pos = q + k;
      // bytes pos-1, pos-2, pos-3 from the piece (or the 4 bytes before it)
      const uint64_t lo64 = ((uint64_t)w[0] << 32) | wp;  // bytes q-4 .. q+3
      uint32_t b1, b2, b3;
      if (k < 4) {
        b1 = (uint32_t)(lo64 >> (8 * (k + 3))) & 0xFFu;
        b2 = (uint32_t)(lo64 >> (8 * (k + 2))) & 0xFFu;
        b3 = (uint32_t)(lo64 >> (8 * (k + 1))) & 0xFFu;
      } else {
        const uint32_t ww[4] = {w[0], w[1], w[2], w[3]};
        auto at = [&](int j) { return (ww[j >> 2] >> (8 * (j & 3))) & 0xFFu; };
        b1 = at(k - 1);
        b2 = at(k - 2);
        b3 = k >= 3 ? at(k - 3) : 0u;
      }
      if (id < L) line_start[id] = pos;
      if (id >= 1 && id - 1 < L) line_end[id - 1] = pos - sep_len(b3, b2, b1, (C >> k) & 1u);
      ++id;
    }
  }
}

// the line count a kernel works on: the host's L, or (fused scan, Ld != null) the device count when
// it fits the caller's arrays (0 otherwise: the caller re-runs with larger arrays)
__device__ __forceinline__ int64_t lines_of(int64_t L, const int64_t* Ld, int64_t cap) {
  if (!Ld) return L;
  const int64_t n = *Ld;
  return n <= cap ? n : 0;
}

// the end of the last line: the text's end, minus a trailing separator (L >= 1, nbytes >= 1)
__device__ __forceinline__ int64_t last_line_end(const uint8_t* __restrict__ text, int64_t nbytes,
                                                 const int64_t* __restrict__ doc_off, int64_t D) {
  int64_t k = D - 1;
  while (k > 0 && doc_off[k] >= nbytes) --k;  // the last non-empty container
  const uint32_t b1 = text[nbytes - 1], b2 = nbytes >= 2 ? text[nbytes - 2] : 0u, b3 = nbytes >= 3 ? text[nbytes - 3] : 0u;
  return nbytes - sep_len(b3, b2, b1, doc_off[k] == nbytes - 1);
}

__global__ void log_last_end(const uint8_t* __restrict__ text, int64_t nbytes, const int64_t* __restrict__ doc_off,
                             int64_t D, int64_t L, const int64_t* __restrict__ Ld, int64_t cap,
                             int64_t* __restrict__ line_end) {
  L = lines_of(L, Ld, cap);
  if (L == 0 || nbytes == 0) return;
  line_end[L - 1] = last_line_end(text, nbytes, doc_off, D);
}

// per-phase cycle counters of the tile kernels (a -DLOG_TIMING build, tools/log_timing.py)
#ifdef LOG_TIMING
// per workgroup: phase cycles (log_index_match: ticket, A, scan, look-back, list, walk, write, [7] tiles, then
// A's parts: loads issued, container starts, pieces; log_index_lines: ticket + container starts, loads + flags,
// scan, look-back, writes), 16 slots
__device__ unsigned long long g_log_timing[1024 * 16];
#define LT_INIT() uint64_t lt_acc[16] = {}; uint64_t lt_p = clock64()
#define LT(i) do { const uint64_t tn = clock64(); lt_acc[i] += tn - lt_p; lt_p = tn; } while (0)
#define LT_FLUSH() do { if (threadIdx.x == 0 && blockIdx.x < 1024) for (int i_ = 0; i_ < 16; ++i_) g_log_timing[blockIdx.x * 16 + i_] += lt_acc[i_]; } while (0)
#else
#define LT_INIT() do {} while (0)
#define LT(i) do {} while (0)
#define LT_FLUSH() do {} while (0)
#endif
// ---- log_index_lines: log_count + log_scan + log_lines in ONE pass over the text -------------
// The text is read once: a workgroup keeps its tile's per-piece line-start masks and separator
// lengths in registers while it finds the tile's first line id by a decoupled look-back over the
// tiles before it (status word per tile: flag AGG = the tile's own total, INC = inclusive prefix;
// tiles take their index from a ticket counter in start order, so every tile waited on has started
// and never waits on a later one), then writes line_start / line_end from the registers.
// Separator lengths as bit planes over the 16 positions of a piece (sep_len's cases): L0 = odd
// lengths (1, 3), L1 = lengths 2 and 3.  Also writes chunk_cnt / tile bases / chunk_line0, so
// krca_log_match can take over when the caller's line arrays are too small.
constexpr uint64_t LB_AGG = 1ull << 62, LB_INC = 2ull << 62, LB_VAL = (1ull << 62) - 1;

__device__ __forceinline__ uint64_t lb_load(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// high bits of sep_len's length-1 / length-2 / length-3 cases at the 4 positions of word w (given
// the word before it), as 4-bit masks; cs4 = container first byte at p-1 for each position
__device__ __forceinline__ void sep_planes(uint32_t wprev, uint32_t w, uint32_t cs4, uint32_t& l0, uint32_t& l1) {
  const uint32_t B1 = __builtin_amdgcn_alignbit(w, wprev, 24);  // text[p-1] at byte k
  const uint32_t B2 = __builtin_amdgcn_alignbit(w, wprev, 16);
  const uint32_t nl = high_bits4(swar_eq(B1, 0x0A));
  const uint32_t crlf = nl & high_bits4(swar_eq(B2, 0x0D)) & ~cs4;
  uint32_t one = (nl & ~crlf) | high_bits4(swar_range(B1, 0x0B, 0x0D) | swar_range(B1, 0x1C, 0x1E));
  uint32_t two = crlf;
  if ((w | wprev) & 0x80808080u) {  // U+0085 (2 bytes), U+2028 / U+2029 (3 bytes)
    const uint32_t B3 = __builtin_amdgcn_alignbit(w, wprev, 8);
    two |= high_bits4(swar_eq(B2, 0xC2) & swar_eq(B1, 0x85));
    const uint32_t three = high_bits4(swar_eq(B3, 0xE2) & swar_eq(B2, 0x80) & (swar_eq(B1, 0xA8) | swar_eq(B1, 0xA9)));
    one |= three;
    two |= three;
  }
  l0 = one;
  l1 = two;
}

// high bits of the 4 bytes of f -> bits 0..3 (one multiply: the four partial products land on
// distinct bits, no carries)
__device__ __forceinline__ uint32_t gather4(uint32_t f) { return ((f & 0x80808080u) * 0x00204081u) >> 28; }

// Line starts S and the separator-length planes L0 (lengths 1, 3) / L1 (lengths 2, 3) at the 16
// positions q..q+15 of a piece, sep_before / sep_len restated on 16-bit masks: the byte tests run
// once per byte of the piece (T(k) = test of byte q+k; bit -1 = byte q-1 from wp) and the "byte
// before p" forms are those masks shifted by one -- instead of re-testing the shifted words
// (sep_flags + sep_planes: ~390 vector instructions per piece and wave).  cs = container first
// bytes at q-1+k (bit k): a "\r" there belongs to the previous container, so "\r\n" is not one
// separator across it.
// Common case first (round 6): a piece whose bytes, and the two before it, hold no separator but
// "\n" and no byte >= 0x80 has S = L0 = the positions after its "\n"s, L1 = 0 -- the other tests'
// gathers and the "\r\n" logic are skipped (a wave takes the full path only when one of its lanes
// needs it).
__device__ __forceinline__ void piece_flags(uint32_t wp, const uint32_t (&w)[4], uint32_t cs, uint32_t& S,
                                            uint32_t& L0, uint32_t& L1) {
  uint32_t nl = 0, r[4];  // bit k of nl: byte q+k is "\n"; r: the other one-byte separators, per byte
  uint32_t odd = (wp | w[0] | w[1] | w[2] | w[3]) & 0x80808080u;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    nl |= gather4(swar_eq(w[j], 0x0A)) << (4 * j);
    r[j] = swar_range(w[j], 0x0B, 0x0D) | swar_range(w[j], 0x1C, 0x1E);
    odd |= r[j];
  }
  // bytes q-1, q-2 (bit 0, 1 of the "before" masks)
  const uint32_t b1 = wp >> 24, b2 = (wp >> 16) & 0xFFu;
  if (!odd && !((b1 >= 0x0B && b1 <= 0x0D) || (b1 >= 0x1C && b1 <= 0x1E) || b2 == 0x0D)) {
    S = ((nl << 1) | (uint32_t)(b1 == 0x0A)) & 0xFFFFu;
    L0 = S;
    L1 = 0;
    return;
  }
  uint32_t cr = 0, sep = nl;  // bit k: byte q+k is "\r" / a one-byte separator
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    cr |= gather4(swar_eq(w[j], 0x0D)) << (4 * j);
    sep |= gather4(r[j]) << (4 * j);
  }
  const uint32_t sep1 = (sep << 1) | (uint32_t)((b1 >= 0x0A && b1 <= 0x0D) || (b1 >= 0x1C && b1 <= 0x1E));  // byte p-1
  const uint32_t cr1 = (cr << 1) | (uint32_t)(b1 == 0x0D);
  const uint32_t nl1 = (nl << 1) | (uint32_t)(b1 == 0x0A);
  const uint32_t cr2 = (cr << 2) | ((uint32_t)(b1 == 0x0D) << 1) | (uint32_t)(b2 == 0x0D);
  S = (sep1 & ~(cr1 & nl)) & 0xFFFFu;
  const uint32_t crlf = nl1 & cr2 & ~cs;  // "\r\n" ends at p-1 (length 2)
  L0 = sep1 & ~crlf;
  L1 = crlf;
  if ((wp | w[0] | w[1] | w[2] | w[3]) & 0x80808080u) {  // U+0085 (C2 85), U+2028 / U+2029 (E2 80 A8/A9)
    uint32_t c2 = 0, x85 = 0, e2 = 0, x80 = 0, a8 = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      c2 |= gather4(swar_eq(w[j], 0xC2)) << (4 * j);
      x85 |= gather4(swar_eq(w[j], 0x85)) << (4 * j);
      e2 |= gather4(swar_eq(w[j], 0xE2)) << (4 * j);
      x80 |= gather4(swar_eq(w[j], 0x80)) << (4 * j);
      a8 |= gather4(swar_eq(w[j], 0xA8) | swar_eq(w[j], 0xA9)) << (4 * j);
    }
    const uint32_t b3 = (wp >> 8) & 0xFFu;
    const uint32_t two = ((x85 << 1) | (uint32_t)(b1 == 0x85)) & ((c2 << 2) | ((uint32_t)(b1 == 0xC2) << 1) | (uint32_t)(b2 == 0xC2));
    const uint32_t three = ((a8 << 1) | (uint32_t)(b1 == 0xA8 || b1 == 0xA9)) &
                           ((x80 << 2) | ((uint32_t)(b1 == 0x80) << 1) | (uint32_t)(b2 == 0x80)) &
                           ((e2 << 3) | ((uint32_t)(b1 == 0xE2) << 2) | ((uint32_t)(b2 == 0xE2) << 1) | (uint32_t)(b3 == 0xE2));
    S |= (two | three) & 0xFFFFu;
    L0 |= three;
    L1 |= two | three;
  }
  L0 &= 0xFFFFu;
  L1 &= 0xFFFFu;
}

__global__ __launch_bounds__(TPB) void log_index_lines(const uint8_t* __restrict__ text, int64_t nbytes,
                                                       const int64_t* __restrict__ doc_off, int64_t D,
                                                       const int32_t* __restrict__ chunk_doc,
                                                       int32_t* __restrict__ chunk_cnt, int64_t* __restrict__ tile_base,
                                                       unsigned long long* __restrict__ status,
                                                       unsigned int* __restrict__ ticket, int64_t ntiles, int64_t cap,
                                                       int64_t* __restrict__ line_start, int64_t* __restrict__ line_end,
                                                       int64_t* __restrict__ chunk_line0, int64_t* __restrict__ n_lines) {
  constexpr int NIT = TILE / (TPB * PIECE);  // 16 passes of 4 KiB
  __shared__ int32_t s_cnt[TPB];
  __shared__ int64_t s_base[TPB];
  __shared__ int64_t s_wsum[TPB / 64];
  __shared__ uint32_t s_cs[NBW];
  __shared__ int64_t s_tile, s_excl;
  // per piece: line starts (low half) | odd separator lengths (high half), and the lengths 2 / 3;
  // in LDS rather than registers (16 pieces x 2 words per lane took the kernel to 215 VGPRs)
  __shared__ uint32_t s_sl[NIT * TPB];
  __shared__ uint16_t s_l1[NIT * TPB];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  LT_INIT();
  // tiles in ticket order, each workgroup taking the next until none is left: every tile a
  // look-back waits on has been taken by a running workgroup, so the wait always ends.  (Taking
  // the next tile's ticket while still on this one, to build its container bitmap during the
  // look-back, measured slower: 113.6 -> 135.8 us, r4r -- a claimed tile publishes its aggregate
  // only after its holder finishes the current one, and later tiles' look-backs wait for it.)
  // (round 6: the container bitmap is cleared once the flags are done, not in a pass and barrier of
  // its own at the tile's start.  Taking the next ticket at the start of the writes, as
  // log_index_match does, was slower here: 109 -> 113 us, the look-back 11k -> 16k cycles per tile,
  // r6r -- with four workgroups per CU the claimed tile's aggregate waits for the whole writes phase.)
  for (int i = threadIdx.x; i < NBW; i += TPB) s_cs[i] = 0u;
  for (;;) {
  if (threadIdx.x == 0) s_tile = (int64_t)atomicAdd(ticket, 1u);
  s_cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t tile = (int64_t)__builtin_amdgcn_readfirstlane((int)s_tile);  // < 2^31 tiles
  if (tile >= ntiles) {  // uniform
    LT_FLUSH();
    return;
  }
  const int64_t tile0 = tile * TILE;
  tile_container_starts_t<TILE, true>(s_cs, tile0, nbytes, doc_off, D, chunk_doc);  // (its barriers cover s_cnt)
  LT(0);
  // the pieces' loads go out LOG_IDX_BATCH at a time, unconditionally (a piece past the text
  // reloads the last aligned block, an aligned 16-byte block holding a text byte never crosses the
  // text's last page; its bytes are zeroed below): a load under `if (q < nbytes)` made each piece
  // wait for its own load, one piece in flight per lane
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const int64_t qlast = nbytes > 0 ? (nbytes - 1) & ~(int64_t)(PIECE - 1) : 0;  // (krca_log_scan returns before any kernel when nbytes == 0)
  const int64_t wave0 = tile0 + (int64_t)__builtin_amdgcn_readfirstlane(wid) * 64 * PIECE;
  for (int it0 = 0; it0 < NIT; it0 += LOG_IDX_BATCH) {
    u32x4 raw[LOG_IDX_BATCH];
    uint32_t pw[LOG_IDX_BATCH];  // bytes q0-4 .. q0-1 of the wave's first piece (wave-uniform)
#pragma unroll
    for (int j = 0; j < LOG_IDX_BATCH; ++j) {
      const int64_t q = tile0 + (int64_t)(it0 + j) * TPB * PIECE + (int64_t)threadIdx.x * PIECE;
      raw[j] = *reinterpret_cast<const u32x4*>(text + (q < nbytes ? q : qlast));
      const int64_t q0 = wave0 + (int64_t)(it0 + j) * TPB * PIECE;
      pw[j] = q0 >= 4 && q0 <= nbytes ? *reinterpret_cast<const uint32_t*>(text + q0 - 4) : 0u;
    }
#pragma unroll
  for (int jj = 0; jj < LOG_IDX_BATCH; ++jj) {
    const int it = it0 + jj;
    const int64_t q = tile0 + (int64_t)it * TPB * PIECE + (int64_t)threadIdx.x * PIECE;
    const bool in = q < nbytes;
    uint32_t w[4] = {in ? raw[jj].x : 0u, in ? raw[jj].y : 0u, in ? raw[jj].z : 0u, in ? raw[jj].w : 0u};
    uint32_t wp = __shfl_up(w[3], 1, 64);  // bytes q-4 .. q-1
    if (lane == 0) wp = pw[jj];
    uint32_t C = 0;  // container first bytes at q-1+j, j = 0..16 (non-empty containers only)
    if (q < nbytes) C = piece_container_starts(s_cs, tile0, q);
    uint32_t S, l0, l1;
    piece_flags(wp, w, C & 0xFFFFu, S, l0, l1);
    if (q < nbytes) {
      S |= C >> 1;
      if (q + PIECE > nbytes) S &= (1u << (int)(nbytes - q)) - 1u;
    } else {
      S = 0;
    }
    s_sl[it * TPB + threadIdx.x] = S | ((l0 & S) << 16);
    s_l1[it * TPB + threadIdx.x] = (uint16_t)(l1 & S);
    uint32_t c = __popc(S);
#pragma unroll
    for (int o = LANES_PER_CHUNK / 2; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);  // 16 lanes = one chunk
    if ((threadIdx.x & (LANES_PER_CHUNK - 1)) == 0)
      s_cnt[it * (TPB / LANES_PER_CHUNK) + threadIdx.x / LANES_PER_CHUNK] = (int32_t)c;
  }
  }
  __syncthreads();
  LT(1);
  for (int i = threadIdx.x; i < NBW; i += TPB) s_cs[i] = 0u;  // the next tile's bitmap (its reads are done)
  // chunk counts, their scan inside the tile, the tile total
  const int64_t v = s_cnt[threadIdx.x];
  chunk_cnt[tile * TPB + threadIdx.x] = (int32_t)v;
  int64_t x = v;
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = (int64_t)__shfl_up((long long)x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) s_wsum[wid] = x;
  __syncthreads();
  int64_t before = x - v;
  for (int u = 0; u < wid; ++u) before += s_wsum[u];
  const int64_t total = s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
  LT(2);
  // decoupled look-back (wave 0): the tile's first line id
  if (wid == 0) {
    int64_t excl = 0;
    if (tile == 0) {
      if (lane == 0) __hip_atomic_store(&status[0], LB_INC | (uint64_t)total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0) __hip_atomic_store(&status[tile], LB_AGG | (uint64_t)total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int64_t top = tile - 1;; top -= 64) {
        const int64_t t = top - lane;  // lane 0 = the nearest predecessor of the window
        uint64_t s = t >= 0 ? lb_load(&status[t]) : LB_INC;
        while (__any((s >> 62) == 0)) {  // some predecessor has not published yet
          __builtin_amdgcn_s_sleep(1);
          if ((s >> 62) == 0) s = lb_load(&status[t]);
        }
        const uint64_t inc = __ballot((s >> 62) == 2);
        const int first = inc ? __builtin_ctzll(inc) : 64;  // nearest inclusive prefix (lowest lane)
        int64_t val = (lane <= first && t >= 0) ? (int64_t)(s & LB_VAL) : 0;
        for (int off = 32; off > 0; off >>= 1) val += (int64_t)__shfl_xor((long long)val, off, 64);
        excl += val;
        if (inc) break;
      }
      if (lane == 0) __hip_atomic_store(&status[tile], LB_INC | (uint64_t)(excl + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) s_excl = excl;
  }
  __syncthreads();
  const int64_t excl = s_excl;
  if (threadIdx.x == 0) {
    tile_base[tile] = excl;
    if (tile == ntiles - 1) {
      const int64_t n = excl + total;
      tile_base[ntiles] = n;
      *n_lines = n;
      // the last line's end (no later line start writes it; log_last_end's work)
      if (n >= 1 && n <= cap && nbytes > 0) line_end[n - 1] = last_line_end(text, nbytes, doc_off, D);
    }
  }
  s_base[threadIdx.x] = excl + before;
  chunk_line0[tile * TPB + threadIdx.x] = excl + before;
  __syncthreads();
  LT(3);
  // line starts and the previous line's end, from the registers
#pragma unroll 2
  for (int it = 0; it < NIT; ++it) {
    const int64_t q = tile0 + (int64_t)it * TPB * PIECE + (int64_t)threadIdx.x * PIECE;
    const uint32_t sl_ = s_sl[it * TPB + threadIdx.x];
    const uint32_t S = sl_ & 0xFFFFu;
    const uint32_t n = __popc(S);
    uint32_t xs = n;
#pragma unroll
    for (int off = 1; off < LANES_PER_CHUNK; off <<= 1) {
      const uint32_t y = __shfl_up(xs, off, 64);
      if ((lane & (LANES_PER_CHUNK - 1)) >= off) xs += y;
    }
    int64_t id = s_base[it * (TPB / LANES_PER_CHUNK) + threadIdx.x / LANES_PER_CHUNK] + (xs - n);
    uint32_t rem = S;
    const uint32_t l0 = sl_ >> 16, l1 = s_l1[it * TPB + threadIdx.x];
    while (rem) {
      const int k = __ffs(rem) - 1;
      rem &= rem - 1;
      const int64_t pos = q + k;
      const int sl = (int)((l0 >> k) & 1u) | (int)(((l1 >> k) & 1u) << 1);
      if (id < cap) line_start[id] = pos;
      if (id >= 1 && id - 1 < cap) line_end[id - 1] = pos - sl;
      ++id;
    }
  }
  __syncthreads();  // the LDS planes and bases are rewritten by the next tile
  LT(4);
#ifdef LOG_TIMING
  lt_acc[7] += 1;
#endif
  }
}

// LDS form of the transition table for log_dfa / log_dfa_long: an entry holds the target state's
// row offset (target * NSYM, so the next lookup is one add, no multiply on the dependent chain) and
// kAcc when the target state reports a category.  The walk reads out[] only on those rare entries:
// two LDS loads per byte instead of three, same masks (or-ing a zero out[] entry is a no-op).
constexpr uint32_t kAcc = 0x8000u;
static_assert(KRCA_DFA_NSTATE * KRCA_DFA_NSYM <= (int)kAcc, "row offsets must fit below kAcc");

// Table fills.  Every entry needs the target's category mask, a load that depends on the
// transition load: a plain loop paid two dependent global-memory round trips per iteration (48 of
// them for a 256-lane workgroup: ~40 us, the whole time of log_dfa_strad, and ~20 us at the front
// of log_dfa and the fused scan, r4j).  Now the masks go to LDS first (one round), then U
// independent transition loads per lane are in flight at once.
template <int U, class LD, class ST>
__device__ __forceinline__ void fill_table(int n, LD load, ST store) {
  for (int i0 = threadIdx.x; i0 < n; i0 += U * (int)blockDim.x) {
    uint32_t t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * (int)blockDim.x;
      t[u] = i < n ? load(i) : 0u;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * (int)blockDim.x;
      if (i < n) store(i, t[u]);
    }
  }
}
__device__ __forceinline__ void fill_out(uint16_t* out) {
  for (int i = threadIdx.x; i < KRCA_DFA_NSTATE; i += blockDim.x) out[i] = krca_dfa_out[i];
  __syncthreads();
}

__device__ __forceinline__ uint32_t dfa_row_entry(int i) {
  const uint32_t t = krca_dfa_trans[i];
  return t * KRCA_DFA_NSYM | (krca_dfa_out[t] ? kAcc : 0u);
}

__device__ __forceinline__ void dfa_load(DfaLds& dfa) {
  for (int i = threadIdx.x; i < 128; i += blockDim.x) dfa.ascii[i] = krca_dfa_ascii_sym[i];
  fill_out(dfa.out);
  fill_table<16>(
      KRCA_DFA_NSTATE * KRCA_DFA_NSYM, [](int i) -> uint32_t { return krca_dfa_trans[i]; },
      [&](int i, uint32_t t) { dfa.trans[i] = (uint16_t)(t * KRCA_DFA_NSYM | (dfa.out[t] ? kAcc : 0u)); });
  __syncthreads();
}

// 512-lane workgroups: the 32 KB LDS table allows 4 workgroups per CU, so 512 lanes give 8 waves per
// SIMD to hide the walk's dependent LDS round trips (256-lane groups left it at 4).
constexpr int DFA_TPB = 512;

__global__ __launch_bounds__(DFA_TPB) void log_dfa_window(const uint8_t* __restrict__ text, int64_t nbytes, int64_t L,
                                                   const int64_t* __restrict__ line_start,
                                                   const int64_t* __restrict__ line_end, uint32_t* __restrict__ line_mask,
                                                   int32_t* __restrict__ long_q, int32_t* __restrict__ n_long) {
  __shared__ DfaLds dfa;
  dfa_load(dfa);
  Bytes B;
  B.init(text, nbytes);
  for (int64_t l = (int64_t)blockIdx.x * DFA_TPB + threadIdx.x; l < L; l += (int64_t)gridDim.x * DFA_TPB) {
    const int64_t s = line_start[l], e = line_end[l];
    if (e - s > LONG_LINE) {
      long_q[atomicAdd(n_long, 1)] = (int32_t)l;  // a wave per long line (log_dfa_long)
      continue;
    }
    uint32_t row = 0, mask = 0;
    if (s < e) {
      // software-pipelined walk: the symbol of the next code point is looked up while the
      // transition of the current one is in flight (one LDS round trip per byte, not two)
      uint32_t cp;
      int len = decode(B, s, cp);
      uint32_t sym = cp_symbol(dfa, cp);
      for (int64_t p = s;;) {
        const uint32_t t = dfa.trans[row + sym];
        p += len;
        const bool more = p < e;
        if (more) {
          len = decode(B, p, cp);
          sym = cp_symbol(dfa, cp);
        }
        row = t & (kAcc - 1);
        if (__builtin_expect((t & kAcc) != 0, 0)) mask |= dfa.out[row / KRCA_DFA_NSYM];
        if (!more) break;
      }
    }
    line_mask[l] = mask;
  }
}

// ---- log_dfa: the walk, four bytes per word and sixteen per block --------------------------
// The round-1 walk (log_dfa_window, kept for A/B) spent ~20 instructions per byte on the 16-byte
// window bookkeeping, the UTF-8 decode branches and the accept test, with a dependent global
// refill every 16 bytes at a different iteration in each lane (the memory counter being per
// wave, nearly every step of a wave waited on one).  This walk:
//  * moves every lane of a wave through its line in lockstep blocks of 16 bytes (starting at the
//    line's 4-byte-aligned start): one buffer load per block per lane, issued a block ahead into
//    the other half of a register ping-pong, so a wave's loads are issued together and each
//    wait covers a load issued 16 transitions earlier;
//  * maps bytes to symbols with one LDS byte table (bytes outside the line map to NOP, an
//    identity column), no decode, when the block's line bytes are all ASCII; blocks holding a
//    non-ASCII byte (or a code point continuing from the previous block) take the exact
//    code-point path of the reference (decode, range table);
//  * keeps a 32-bit entry per (state, symbol): the target's row offset (low half) and its
//    category mask (high half), so the accept test is one OR per byte.
// Per byte: a byte-table read, a 16-bit add, a table read and an OR.
constexpr int DFA_RS = 32;  // u32 entries per state row: the symbols, then NOP
constexpr uint32_t NOP_SYM = DFA_RS - 1;
// Row stride in the LDS table, in entries.  (A stride of 33 instead of 32 -- entry (state, symbol)
// in bank (state + symbol) mod 32 instead of bank `symbol` for every state -- measured the same:
// log_dfa 73.5 vs 73.4 us, r4t; the walk is not bound by these reads' bank conflicts.)
constexpr int DFA_STRIDE = DFA_RS;
static_assert(KRCA_DFA_NSYM <= (int)NOP_SYM, "no room for the NOP column");
static_assert(KRCA_DFA_NSTATE * DFA_STRIDE * 4 <= 65536, "row byte offsets must fit 16 bits");
static_assert(KRCA_NCAT <= 16, "category masks must fit 16 bits");

struct DfaLds4 {
  uint32_t trans[KRCA_DFA_NSTATE * DFA_STRIDE];  // (out[target] << 16) | target * DFA_STRIDE * 4
  uint16_t out[KRCA_DFA_NSTATE];             // (staging for the fill)
  uint8_t sym[256];                          // byte -> symbol * 4 (bytes >= 0x80 -> NOP)
};

// the DFA row entry at table index i (DFA_RS columns per state: the symbols, then NOP = itself)
__device__ __forceinline__ uint32_t dfa_target(int i, int rs) {
  const int st = i / rs, c = i % rs;
  return c < KRCA_DFA_NSYM ? (uint32_t)krca_dfa_trans[st * KRCA_DFA_NSYM + c] : (uint32_t)st;
}

__device__ __forceinline__ void dfa4_load(DfaLds4& d) {
  fill_out(d.out);
  fill_table<8>(
      KRCA_DFA_NSTATE * DFA_RS, [](int i) { return dfa_target(i, DFA_RS); },
      [&](int i, uint32_t t) {
        d.trans[(i / DFA_RS) * DFA_STRIDE + i % DFA_RS] = ((uint32_t)d.out[t] << 16) | (t * DFA_STRIDE * 4);
      });
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    const uint32_t sy = i < 128 ? krca_dfa_ascii_sym[i] : NOP_SYM;
    d.sym[i] = (uint8_t)((sy == KRCA_DFA_SEP ? NOP_SYM : sy) * 4);  // no separator inside a line
  }
  __syncthreads();
}

// the entry at byte offset (row + symoff) mod 2^16 of the table: the row offset sits in the low
// half of the previous entry, a 16-bit add drops the category bits above it
__device__ __forceinline__ uint32_t dfa4_step(const DfaLds4& d, uint32_t row, uint32_t symoff) {
  uint32_t a;  // (row + symoff) & 0xFFFF in one VALU op (SDWA: low word, upper bits zeroed)
  asm("v_add_u32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:DWORD"
      : "=v"(a)
      : "v"(row), "v"(symoff));
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(d.trans) + a);
}

// the DFA symbol of code point cp >= 0x80 (the reference's case folds and \d classes), by a binary
// search of the range table copied to LDS (rng: KRCA_DFA_NRANGE x {lo, hi, symbol}; from constant
// memory each probe was a dependent global load, ~7 per code point, and one line with a non-ASCII
// character held its wave: +5k cycles per 64 KiB tile of log_index_match, r6n)
__device__ __forceinline__ uint32_t cp_sym_lds(const uint32_t* rng, uint32_t cp) {
  uint32_t sy = KRCA_DFA_OTHER;
  int a = 0, z = KRCA_DFA_NRANGE - 1;
  while (a <= z) {
    const int mid = (a + z) >> 1;
    if (cp < rng[3 * mid]) z = mid - 1;
    else if (cp > rng[3 * mid + 1]) a = mid + 1;
    else {
      sy = rng[3 * mid + 2];
      break;
    }
  }
  return sy;
}
__device__ __forceinline__ void load_ranges(uint32_t* rng) {
  for (int i = threadIdx.x; i < 3 * KRCA_DFA_NRANGE; i += blockDim.x) rng[i] = krca_dfa_ranges[i / 3][i % 3];
}
// the code point starting with lead byte b (>= 0xC0) whose continuation bytes at(1..3) returns
template <class AT>
__device__ __forceinline__ uint32_t utf8_cp(uint32_t b, AT at) {
  if (b < 0xE0) return ((b & 0x1F) << 6) | (at(1) & 0x3F);
  if (b < 0xF0) return ((b & 0x0F) << 12) | ((at(1) & 0x3F) << 6) | (at(2) & 0x3F);
  return ((b & 0x07) << 18) | ((at(1) & 0x3F) << 12) | ((at(2) & 0x3F) << 6) | (at(3) & 0x3F);
}

// hi4x for word_in_line: the bytes 0x80 + hi - 1 (0x7F for hi = 0), so that hi4x - i has bit 7 set
// iff i < hi.  (Until round 4 the bytes were 0x80 + hi, which admitted i = hi: the byte at the
// line's end -- the separator, a NOP, or at a container without a trailing separator the NEXT
// container's first byte, which could complete a pattern: "Erro" | "r".  Found by
// test_log_scan_no_match_across_container_end.)
__device__ __forceinline__ uint32_t line_hi4x(int hi) {
  return (((uint32_t)hi * 0x01010101u) | 0x80808080u) - 0x01010101u;
}
// Line bytes of a block, four at a time: byte k of word j (block index i = 4j + k) is in the line
// iff lo <= i < hi (lo = s - P clamped to [0, 16], hi = e - P clamped to [0, 16], broadcast to
// the four bytes as lo4 / line_hi4x(hi)).  SWAR on bytes < 0x80, no borrows: bit 7 of each
// byte of the result is set iff the byte is in the line.
__device__ __forceinline__ uint32_t word_in_line(int j, uint32_t lo4, uint32_t hi4x) {
  const uint32_t idx = 0x03020100u + 0x04040404u * (uint32_t)j;
  return ((idx | 0x80808080u) - lo4) & (hi4x - idx) & 0x80808080u;
}

__global__ __launch_bounds__(DFA_TPB) void log_dfa(const uint8_t* __restrict__ text, int64_t nbytes, int64_t L,
                                                   const int64_t* __restrict__ Ld, int64_t cap,
                                                   const int64_t* __restrict__ line_start,
                                                   const int64_t* __restrict__ line_end, uint32_t* __restrict__ line_mask,
                                                   int32_t* __restrict__ long_q, int32_t* __restrict__ n_long) {
  __shared__ DfaLds4 d;
  __shared__ uint32_t d_rng[3 * KRCA_DFA_NRANGE];
  load_ranges(d_rng);
  dfa4_load(d);  // (its barrier covers d_rng)
  L = lines_of(L, Ld, cap);
  for (int64_t l0 = (int64_t)blockIdx.x * DFA_TPB; l0 < L; l0 += (int64_t)gridDim.x * DFA_TPB) {
    // buffer resource at the group's first line: offsets stay 32-bit (the group's short lines
    // span < 1 MiB), reads past the text return 0 and never fault
    const int64_t base = line_start[l0] & ~(int64_t)15;
    const int64_t rem = nbytes - base;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(text + base), 0, (int)(rem < (int64_t)INT32_MAX ? rem : (int64_t)INT32_MAX), 0x00020000);
    const int64_t l = l0 + threadIdx.x;
    if (l >= L) continue;
    const int64_t s = line_start[l], e = line_end[l];
    if (e - s > LONG_LINE) {
      long_q[atomicAdd(n_long, 1)] = (int32_t)l;  // a wave per long line (log_dfa_long)
      continue;
    }
    uint32_t row = 0, acc = 0;
    int off = (int)((s & ~(int64_t)3) - base);  // this block's first byte, from base
    int rs_ = (int)(s & 3);                      // s - P: 0..3 at the first block, then negative
    int re_ = (int)(e - (s & ~(int64_t)3));      // e - P
    const int end_off = (int)min(rem, (int64_t)INT32_MAX);
    auto load = [&](int q) -> uint4 {
      return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, q, 0, 0));
    };
    // one block: cur holds bytes off .. off+15; the block after the next is loaded into far first
    // (every lane, every block: a ring of three, so the wait on cur covers a load issued two
    // blocks -- 32 dependent steps -- earlier).  Each byte steps on its symbol: an in-line ASCII
    // byte's from the byte table; NOP (the identity column) for a byte outside the line and for a
    // UTF-8 continuation byte (the table maps bytes >= 0x80 to NOP); a lead byte's entry is then
    // replaced by the symbol of the code point it starts, decoded as the reference reads the text
    // -- a multi-byte code point is one transition (round 6: no code-point loop of its own).
    auto block = [&](uint4& cur, uint4& far) -> bool {
      far = load(off + 32);
      uint32_t w[4] = {cur.x, cur.y, cur.z, cur.w};
      if (off + 16 > end_off) {  // the text's last bytes (a buffer load straddling the end reads 0)
#pragma unroll 1
        for (int k = 0; k < 16; ++k) {
          const uint32_t b = off + k < end_off ? (uint32_t)text[base + off + k] : 0u;
          w[k >> 2] = (w[k >> 2] & ~(0xFFu << (8 * (k & 3)))) | (b << (8 * (k & 3)));
        }
      }
      const int lo = max(rs_, 0), hi = min(re_, 16);
      const uint32_t lo4 = (uint32_t)lo * 0x01010101u, hi4x = line_hi4x(hi);
      uint32_t so[16], hib = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t in = word_in_line(j, lo4, hi4x);
        hib |= w[j] & in;
        const uint32_t x = w[j] | (in ^ 0x80808080u);  // outside the line: >= 0x80, NOP
#pragma unroll
        for (int k = 0; k < 4; ++k) so[4 * j + k] = d.sym[(x >> (8 * k)) & 0xFFu];
      }
      if (hib) {  // in-line bytes >= 0x80 (rare): the lead bytes' code points
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const uint32_t b = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
          if (b >= 0xC0 && k >= lo && k < hi) {
            const uint32_t cp = utf8_cp(b, [&](int r) -> uint32_t {
              const int q = k + r;
              if (q < 16) return (w[q >> 2] >> (8 * (q & 3))) & 0xFFu;
              return off + q < end_off ? (uint32_t)text[base + off + q] : 0u;
            });
            so[k] = cp_sym_lds(d_rng, cp) * 4;
          }
        }
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const uint32_t t = dfa4_step(d, row, so[k]);
        row = t;
        acc |= t;
      }
      const bool more = re_ > 16;
      off += 16;
      rs_ -= 16;
      re_ -= 16;
      return more;
    };
    if (s < e) {
      uint4 R0 = load(off), R1 = load(off + 16), R2;
      while (block(R0, R2) && block(R1, R0) && block(R2, R1)) {
      }
    }
    line_mask[l] = acc >> 16;
  }
}

__global__ __launch_bounds__(TPB) void log_dfa_long(const uint8_t* __restrict__ text, int64_t nbytes,
                                                    const int64_t* __restrict__ line_start,
                                                    const int64_t* __restrict__ line_end,
                                                    uint32_t* __restrict__ line_mask, const int32_t* __restrict__ long_q,
                                                    const int32_t* __restrict__ n_long) {
  __shared__ DfaLds dfa;
  const int nq = *n_long;
  if ((int64_t)blockIdx.x * (TPB / 64) >= nq) return;  // no long line for this block: skip the table fill
  dfa_load(dfa);
  const int lane = threadIdx.x & 63;
  Bytes B;
  B.init(text, nbytes);
  for (int j = (int)(blockIdx.x * (TPB / 64) + (threadIdx.x >> 6)); j < nq; j += (int)(gridDim.x * (TPB / 64))) {
    const int64_t l = long_q[j];
    const int64_t s = line_start[l], e = line_end[l];
    const int64_t seg = (e - s + 63) / 64;
    const int64_t a = min(e, s + lane * seg), b = min(e, a + seg);
    uint32_t row = 0, mask = 0;
    const int64_t p0 = a > s ? cp_align(B, a, e) : s;  // first code point starting in [a, b)
    if (p0 > s && p0 < b) {  // warm-up over the <= WARM code points of the line before p0
      int64_t k = p0;
      int seen = 0;
      while (k > s && seen < WARM) {
        const uint32_t c = B.at(k - 1);
        --k;
        if ((c & 0xC0) != 0x80) ++seen;
      }
      while (k < p0) {
        uint32_t cp;
        const int len = decode(B, k, cp);
        row = dfa.trans[row + cp_symbol(dfa, cp)] & (kAcc - 1);
        k += len;
      }
    }
    for (int64_t p = p0; p < b;) {
      uint32_t cp;
      const int len = decode(B, p, cp);
      const uint32_t t = dfa.trans[row + cp_symbol(dfa, cp)];
      row = t & (kAcc - 1);
      if (__builtin_expect((t & kAcc) != 0, 0)) mask |= dfa.out[row / KRCA_DFA_NSYM];
      p += len;
    }
    for (int off = 32; off > 0; off >>= 1) mask |= __shfl_xor(mask, off, 64);
    if (lane == 0) line_mask[l] = mask;
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

// first line starting at or after byte s: only the lines of s's 256-byte chunk can be below it
__device__ __forceinline__ int64_t first_line_at(const int64_t* __restrict__ line_start, int64_t L,
                                                 const int64_t* __restrict__ chunk_line0, int64_t nchunks,
                                                 int64_t s) {
  const int64_t c = s / CH;
  if (L == 0 || c >= nchunks) return L;
  int64_t lo = chunk_line0[c], hi = c + 1 < nchunks ? chunk_line0[c + 1] : L;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (line_start[mid] < s) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Example lines as bits: bit 16 + c of line_mask[l] is set when line l is one of the first three
// lines of its container in category c (the reference's evidence, ref:agents/logs_agent.py:159-163),
// so the examples cost no more than the masks they sit beside (a dense [D][13][3] id table is 156 B
// per container: 2/3 of the scan's writes at C5).  DENSE also writes that table (A/B, compat).
constexpr uint32_t CAT_BITS = (1u << KRCA_NCAT) - 1u;
constexpr int EX_SHIFT = 16;
static_assert(EX_SHIFT + KRCA_NCAT <= 32, "example bits must fit the line mask");

template <bool DENSE>
__global__ __launch_bounds__(TPB) void log_hist(const int64_t* __restrict__ doc_off, int64_t D,
                                                const int64_t* __restrict__ chunk_line0, int64_t nchunks,
                                                const int64_t* __restrict__ line_start,
                                                uint32_t* __restrict__ line_mask, int64_t L,
                                                const int64_t* __restrict__ Ld, int64_t cap,
                                                int32_t* __restrict__ doc_lines, int32_t* __restrict__ hist,
                                                int32_t* __restrict__ examples, int64_t* __restrict__ doc_line0) {
  // the block's histograms (and dense examples) are assembled in LDS and leave in coalesced rows (a
  // lane writing its own 52 ints at a 208-byte stride touched ~26 lines per store instruction)
  __shared__ int32_t s_ex[TPB * KRCA_NCAT * (DENSE ? 3 : 1)];
  L = lines_of(L, Ld, cap);
  int32_t mycnt[KRCA_NCAT];  // this lane's container histogram (small or big path)
#pragma unroll
  for (int c = 0; c < KRCA_NCAT; ++c) mycnt[c] = 0;
  const int64_t d0 = (int64_t)blockIdx.x * TPB;
  const int64_t d = d0 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const bool valid = d < D;
  const int64_t lo = valid ? first_line_at(line_start, L, chunk_line0, nchunks, doc_off[d]) : L;
  int64_t hi = __shfl_down(lo, 1, 64);
  if (valid && (lane == 63 || d + 1 == D)) hi = first_line_at(line_start, L, chunk_line0, nchunks, doc_off[d + 1]);
  const bool small = valid && hi - lo <= HIST_SMALL;
  if (small) {
    int32_t cnt[KRCA_NCAT], ex[KRCA_NCAT][3];
#pragma unroll
    for (int c = 0; c < KRCA_NCAT; ++c) {
      cnt[c] = 0;
      ex[c][0] = ex[c][1] = ex[c][2] = -1;
    }
    uint32_t full = 0;  // bins holding three examples already
    for (int64_t l = lo; l < hi; ++l) {
      const uint32_t m = line_mask[l] & CAT_BITS;
      const uint32_t exb = m & ~full;
      if (exb) line_mask[l] = m | (exb << EX_SHIFT);
#pragma unroll
      for (int c = 0; c < KRCA_NCAT; ++c) {
        if ((m >> c) & 1u) {
          const int f = cnt[c];
          if (DENSE) {
            if (f == 0) ex[c][0] = (int32_t)l;
            if (f == 1) ex[c][1] = (int32_t)l;
            if (f == 2) ex[c][2] = (int32_t)l;
          }
          if (f == 2) full |= 1u << c;
          cnt[c] = f + 1;
        }
      }
    }
    doc_lines[d] = (int32_t)(hi - lo);
    if (doc_line0) doc_line0[d] = lo;
#pragma unroll
    for (int c = 0; c < KRCA_NCAT; ++c) mycnt[c] = cnt[c];
    if (DENSE) {
      int32_t* ed = s_ex + threadIdx.x * KRCA_NCAT * 3;
#pragma unroll
      for (int c = 0; c < KRCA_NCAT; ++c) {
        ed[c * 3] = ex[c][0];
        ed[c * 3 + 1] = ex[c][1];
        ed[c * 3 + 2] = ex[c][2];
      }
    }
  }
  uint64_t big = __ballot(valid && !small);
  const uint64_t below = (1ull << lane) - 1ull;  // lanes before this one
  while (big) {  // wave-uniform: the wave takes the large containers one at a time
    const int j = __ffsll((unsigned long long)big) - 1;
    big &= big - 1;
    const int64_t dj = d - lane + j;
    const int64_t blo = __shfl(lo, j, 64), bhi = __shfl(hi, j, 64);
    int32_t cnt[KRCA_NCAT];
#pragma unroll
    for (int c = 0; c < KRCA_NCAT; ++c) cnt[c] = 0;
    int32_t* ex = s_ex + (threadIdx.x - lane + j) * KRCA_NCAT * 3;
    for (int64_t b = blo; b < bhi; b += 64) {
      const bool in = b + lane < bhi;
      const uint32_t m = in ? (line_mask[b + lane] & CAT_BITS) : 0u;
      uint32_t exb = 0;
#pragma unroll
      for (int c = 0; c < KRCA_NCAT; ++c) {
        const uint64_t bal = __ballot((m >> c) & 1u);
        const int f = cnt[c];  // wave-uniform
        // this line is an example of bin c when fewer than three came before it in the container
        if (((m >> c) & 1u) && f + __popcll(bal & below) < 3) exb |= 1u << c;
        if (DENSE && f < 3) {
          uint64_t bb = bal;
          for (int k = f; k < 3 && bb; ++k) {
            const int q = __ffsll((unsigned long long)bb) - 1;
            if (lane == 0) ex[c * 3 + k] = (int32_t)(b + q);
            bb &= bb - 1;
          }
        }
        cnt[c] = f + __popcll(bal);
      }
      if (exb) line_mask[b + lane] = m | (exb << EX_SHIFT);
    }
    if (lane == j) {  // counts are wave-uniform (ballots): the container's own lane keeps them
#pragma unroll
      for (int c = 0; c < KRCA_NCAT; ++c) mycnt[c] = cnt[c];
    }
    if (lane == 0) {
      doc_lines[dj] = (int32_t)(bhi - blo);
      if (doc_line0) doc_line0[dj] = blo;
      if (DENSE) {
#pragma unroll
        for (int c = 0; c < KRCA_NCAT; ++c)
          for (int k = cnt[c] < 3 ? cnt[c] : 3; k < 3; ++k) ex[c * 3 + k] = -1;
      }
    }
  }
  const int nv = (int)(D - d0 < TPB ? D - d0 : TPB);
  if (DENSE) {
    __syncthreads();
    for (int i = threadIdx.x; i < nv * KRCA_NCAT * 3; i += TPB) examples[d0 * KRCA_NCAT * 3 + i] = s_ex[i];
  }
  __syncthreads();  // the buffer now takes the histograms
#pragma unroll
  for (int c = 0; c < KRCA_NCAT; ++c) s_ex[threadIdx.x * KRCA_NCAT + c] = mycnt[c];
  __syncthreads();
  for (int i = threadIdx.x; i < nv * KRCA_NCAT; i += TPB) hist[d0 * KRCA_NCAT + i] = s_ex[i];
}

// ---- log_index_match: line index AND DFA walk in ONE pass over the text (round 4) ------------
// log_index_lines + log_dfa re-read the text: the DFA pass fetched it a second time (290 MB at the
// DRAM-side counters for 184 MB of text, the scan 2.3x its algorithmic bytes).  Here a workgroup
// keeps its 32 KiB tile in LDS after the line-start pass and walks the tile's lines there.  Two
// workgroups per CU (75 KB of LDS each: the tile, a 16-bit transition table, the line list), so one
// can stream its tile in while the other walks (the walk is bound by LDS throughput, the load by
// memory latency; one 1024-thread workgroup per CU with a 64 KiB tile ran the phases one after the
// other: 262 us against 113 + 83 us for the two-kernel path, r4e):
//   A  each lane loads 4 pieces of 16 bytes, stores their symbol offsets to LDS (sym_word) and
//      computes their line-start / separator-length bits (piece_flags); per 256-byte chunk counts,
//      their scan inside the tile, the tile total published for the look-back (aggregate).  Wave 0
//      also takes the LOOK bytes after the tile: the first line start there ends the tile's last line;
//   B  the tile's lines in windows of LMAX: a list of (start, end) tile offsets in LDS built from
//      the start bits, then a lane per line walks it with the DFA from LDS (16-byte lockstep blocks
//      as in log_dfa, no byte table for ASCII blocks); masks in LDS;
//   C  the look-back resolves the tile's first line id (its predecessors have long published their
//      aggregates by then), and the window's line_start / line_end / line_mask go out coalesced by
//      line id.
// Deferred to log_dfa_long (a wave per line): lines longer than LONG_LINE.
// Two shapes (KRCA_LOG_FUSED = 1 / 2): 32 KiB tiles, 512 threads, the 16-bit table -- two
// workgroups per CU; or 64 KiB tiles, 1024 threads, DfaLds4's 32-bit table (the category mask in
// every entry: no branch per byte) -- one workgroup per CU, 16 waves.
// Bytes after the tile that log_index_match loads with it: the tile's last line ends in them unless
// it is longer than LONG_LINE (then log_dfa_long walks it), so no line of a tile waits on the next
// tile's workgroup (round 5's log_dfa_strad: a lane per straddling line, 35-41 us per scan).
constexpr int LOOK = LONG_LINE;
// log_index_match's walk: lines longer than SPLIT_T bytes are walked by two lanes (at most SPLIT_MAX
// per window, and only while the window's lines and halves fit one pass of the workgroup)
constexpr int SPLIT_T = 88;
constexpr int SPLIT_MAX = 512;
// any byte >= 0x80 among tile offsets [a, m) of s_text (a >= 0)
__device__ __forceinline__ bool any_high(const uint32_t* tx, int a, int m) {
  uint32_t h = 0;
  for (int p = a & ~3; p < m; p += 4) {
    uint32_t msk = 0x80808080u;
    if (p < a) msk &= 0x80808080u << (8 * (a - p));
    if (p + 4 > m) msk &= 0x80808080u >> (8 * (p + 4 - m));
    h |= tx[p >> 2] & msk;
  }
  return h != 0;
}
template <int64_t TILE_B, int NT, bool U32>
struct FCfg {
  static constexpr int64_t FTILE = TILE_B;                    // bytes per tile
  static constexpr int FTPB = NT;                             // threads
  static constexpr int FNIT = (int)(TILE_B / (NT * PIECE));   // 4 pieces of 16 bytes per lane
  static constexpr int FCH = (int)(TILE_B / CH);              // 256-byte chunks per tile
  static constexpr int FNBW = (int)((TILE_B + LOOK) / 32) + 2;  // container-start bitmap words (tile + LOOK)
  static constexpr int LMAX = (int)(TILE_B / 16);             // lines of a tile listed and walked per window
  static constexpr bool W32 = U32;
};
using FSmall = FCfg<32768, 512, false>;
using FBig = FCfg<65536, 1024, true>;

int64_t num_ftiles(int64_t nbytes, int64_t tile_b) { return std::max<int64_t>(1, krca::ceil_div(nbytes, tile_b)); }

// 16-bit transition table (25 KB instead of DfaLds4's 50 KB): entry = the target state's row as a
// byte offset (target * 64) | 0x8000 when the target reports a category; the category mask is read
// from out[] only on those (rare) entries.  Row 31 of every state is the NOP column (identity) for
// bytes outside the line, as in DfaLds4.
constexpr int D2_RS = 32;
struct DfaLds2 {
  uint16_t trans[KRCA_DFA_NSTATE * D2_RS];
  uint16_t out[KRCA_DFA_NSTATE];
  uint8_t sym[256];  // byte -> symbol * 2 (bytes >= 0x80 and separators -> NOP)
};
static_assert(KRCA_DFA_NSTATE * D2_RS * 2 <= 0x8000, "row byte offsets must fit 15 bits");

__device__ __forceinline__ void dfa2_load(DfaLds2& d) {
  fill_out(d.out);
  fill_table<8>(
      KRCA_DFA_NSTATE * D2_RS, [](int i) { return dfa_target(i, D2_RS); },
      [&](int i, uint32_t t) { d.trans[i] = (uint16_t)((t * D2_RS * 2) | (d.out[t] ? 0x8000u : 0u)); });
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    const uint32_t sy = i < 128 ? krca_dfa_ascii_sym[i] : NOP_SYM;
    d.sym[i] = (uint8_t)((sy == KRCA_DFA_SEP ? NOP_SYM : sy) * 2);  // no separator inside a line
  }
  __syncthreads();
}

__device__ __forceinline__ uint32_t dfa2_step(const DfaLds2& d, uint32_t row, uint32_t so, uint32_t& acc) {
  const uint32_t t =
      *reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(d.trans) + ((row & 0x7FFFu) + so));
  if (t & 0x8000u) acc |= d.out[(t & 0x7FFFu) >> 6];
  return t;
}

// one byte step of either table: the 32-bit one ORs its entry (mask in the high half), the 16-bit
// one reads out[] on a reporting entry
__device__ __forceinline__ uint32_t dstep(const DfaLds4& d, uint32_t row, uint32_t so, uint32_t& acc) {
  const uint32_t t = dfa4_step(d, row, so);
  acc |= t;
  return t;
}
__device__ __forceinline__ uint32_t dstep(const DfaLds2& d, uint32_t row, uint32_t so, uint32_t& acc) {
  return dfa2_step(d, row, so, acc);
}
__device__ __forceinline__ uint32_t dmask(const DfaLds4&, uint32_t acc) { return acc >> 16; }
__device__ __forceinline__ uint32_t dmask(const DfaLds2&, uint32_t acc) { return acc; }
__device__ __forceinline__ uint32_t dsym_scale(const DfaLds4&) { return 4; }
__device__ __forceinline__ uint32_t dsym_scale(const DfaLds2&) { return 2; }
__device__ __forceinline__ void dload(DfaLds4& d) { dfa4_load(d); }
__device__ __forceinline__ void dload(DfaLds2& d) { dfa2_load(d); }

// the step on symbol byte K of a word of symbol offsets: the 32-bit table takes the byte straight
// into the 16-bit add (SDWA source select), so a step is one add, one LDS read and one OR
#define KRCA_DSTEP_BYTE(K)                                                                                    \
  __device__ __forceinline__ uint32_t dstep_b##K(const DfaLds4& d, uint32_t row, uint32_t sw, uint32_t& acc) { \
    uint32_t a;                                                                                               \
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:BYTE_" #K     \
        : "=v"(a)                                                                                             \
        : "v"(row), "v"(sw));                                                                                 \
    const uint32_t t = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(d.trans) + a);     \
    acc |= t;                                                                                                 \
    return t;                                                                                                 \
  }                                                                                                           \
  __device__ __forceinline__ uint32_t dstep_b##K(const DfaLds2& d, uint32_t row, uint32_t sw, uint32_t& acc) { \
    return dfa2_step(d, row, (sw >> (8 * K)) & 0xFFu, acc);                                                  \
  }
KRCA_DSTEP_BYTE(0)
KRCA_DSTEP_BYTE(1)
KRCA_DSTEP_BYTE(2)
KRCA_DSTEP_BYTE(3)
#undef KRCA_DSTEP_BYTE

// s_text of log_index_match holds symbol offsets for ASCII bytes: phase A maps every byte below
// 0x80 through conv[] to its column's offset in a TAB row (separators -> NOP) and keeps the bytes
// >= 0x80 (the UTF-8 lead and continuation bytes) as they are, so an all-ASCII block reads no byte
// table and a block holding a multi-byte code point still decodes it.
static_assert(NOP_SYM * 4 < 0x80, "symbol offsets must stay below 0x80");
__device__ __forceinline__ uint32_t sym_word(const uint8_t* conv, uint32_t w) {
  return (uint32_t)conv[w & 0xFFu] | ((uint32_t)conv[(w >> 8) & 0xFFu] << 8) | ((uint32_t)conv[(w >> 16) & 0xFFu] << 16) |
         ((uint32_t)conv[w >> 24] << 24);
}

// the symbol offset of code point cp >= 0x80 in TAB's rows
template <class TAB>
__device__ __forceinline__ uint32_t cp_symoff(const TAB& d, const uint32_t* rng, uint32_t cp) {
  return cp_sym_lds(rng, cp) * dsym_scale(d);
}

// The DFA mask of the line at tile offsets [s, e) from s_text (e <= FTILE + LOOK; the array is
// padded so a block may read up to 20 bytes past e): lockstep 16-byte blocks from the line's first
// byte (funnel-shifted words), the next block's words read before this block's 16 dependent
// steps, each byte stepping on its symbol offset: an ASCII byte's stored offset; NOP (the identity
// column) for a byte outside the line and for a UTF-8 continuation byte; for a lead byte, the
// symbol of the code point it starts (decoded from the raw bytes after it, as the reference reads
// the text) -- so a multi-byte code point is one transition, and only blocks holding a byte >= 0x80
// do any decoding.
template <class TAB>
__device__ __forceinline__ uint32_t dfa_walk_sym(const uint32_t* __restrict__ tx, const TAB& d, const uint32_t* rng,
                                                 int s, int e) {
  // Blocks start at s itself (round 7; until then at s & ~3, with the bytes before s masked in every
  // block): each block's words are funnel-shifted out of five LDS words (one alignbyte per word, the
  // shift s & 3 fixed for the walk), so only the line's END is masked, one compare per word (~20 of
  // ~87 vector instructions per block fewer).
  uint32_t row = 0, acc = 0;
  int p = s;       // this block's first byte
  int re_ = e - s;  // e - p
  const uint32_t sh = (uint32_t)(s & 3);
  int q = s >> 2;  // the word holding byte p
  constexpr uint32_t nop = NOP_SYM * sizeof(d.trans[0]);
  uint32_t x[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) x[j] = tx[q + j];
  for (;;) {
    const uint32_t hi4x = line_hi4x(min(re_, 16));
    uint32_t so[4], hib = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t w = __builtin_amdgcn_alignbyte(x[j + 1], x[j], sh);  // bytes p + 4j .. p + 4j + 3
      const uint32_t in = (hi4x - (0x03020100u + 0x04040404u * (uint32_t)j)) & 0x80808080u;  // byte < hi
      const uint32_t fm = (in >> 7) * 0xFFu;
      so[j] = (w & fm) | (nop * 0x01010101u & ~fm);
      hib |= so[j];
    }
    const bool more = re_ > 16;
    if (hib & 0x80808080u) {  // bytes >= 0x80 in the line (rare): continuation bytes -> NOP, lead bytes -> their code point
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const uint32_t b = (so[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        if (b >= 0x80) {
          uint32_t sy = nop;
          if (b >= 0xC0) {
            const uint32_t cp = utf8_cp(b, [&](int r) -> uint32_t {
              const int pp = p + k + r;
              return (tx[pp >> 2] >> (8 * (pp & 3))) & 0xFFu;
            });
            sy = cp_symoff(d, rng, cp);
          }
          so[k >> 2] = (so[k >> 2] & ~(0xFFu << (8 * (k & 3)))) | (sy << (8 * (k & 3)));
        }
      }
    }
    if (more) {
      x[0] = x[4];
#pragma unroll
      for (int j = 1; j < 5; ++j) x[j] = tx[q + 4 + j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      row = dstep_b0(d, row, so[j], acc);
      row = dstep_b1(d, row, so[j], acc);
      row = dstep_b2(d, row, so[j], acc);
      row = dstep_b3(d, row, so[j], acc);
    }
    if (!more) break;
    p += 16;
    q += 4;
    re_ -= 16;
  }
  return dmask(d, acc);
}

// ntiles: FTILE tiles; tile_base / n_lines keep the TILE (64 KiB) tiles' bases that krca_log_match
// reads (tile_base[T] = the first line of 32 KiB tile 2T), chunk counts / bases are per 256-byte
// chunk as before
template <class CF>
__global__ __launch_bounds__(CF::FTPB, 4) void log_index_match(
    const uint8_t* __restrict__ text, int64_t nbytes, const int64_t* __restrict__ doc_off, int64_t D,
    const int32_t* __restrict__ chunk_doc, int32_t* __restrict__ chunk_cnt, int64_t* __restrict__ tile_base,
    int64_t nt64, unsigned long long* __restrict__ status, unsigned int* __restrict__ ticket, int64_t ntiles,
    int64_t cap, int64_t* __restrict__ line_start, int64_t* __restrict__ line_end, uint32_t* __restrict__ line_mask,
    int64_t* __restrict__ chunk_line0, int64_t* __restrict__ n_lines, int32_t* __restrict__ long_q,
    int32_t* __restrict__ n_long) {
  constexpr int64_t FTILE = CF::FTILE;
  constexpr int FTPB = CF::FTPB, FNIT = CF::FNIT, FCH = CF::FCH, FNBW = CF::FNBW, LMAX = CF::LMAX;
  using TAB = typename std::conditional<CF::W32, DfaLds4, DfaLds2>::type;
  // the symbol offsets (sym_word) of the tile and the LOOK bytes after it, + 32 zero bytes
  __shared__ __attribute__((aligned(16))) uint32_t s_text[(FTILE + LOOK) / 4 + 8];
  __shared__ TAB d;
  __shared__ uint8_t s_conv[256];  // byte -> symbol offset (bytes >= 0x80: themselves)
  __shared__ uint32_t s_rng[3 * KRCA_DFA_NRANGE];  // the code point ranges' symbols (cp_symoff)
  __shared__ uint32_t s_cs[FNBW];
  __shared__ uint16_t s_ls[LMAX], s_le[LMAX];
  __shared__ uint32_t s_lm[LMAX / 2];  // the window's masks, two per word (atomicOr: a split line's halves)
  __shared__ int16_t s_sj[SPLIT_MAX];  // the window's split lines
  __shared__ int32_t s_nsplit;
  __shared__ int32_t s_cnt[FCH], s_cb[FCH];  // per 256-byte chunk: line starts, exclusive base in the tile
  __shared__ int32_t s_wsum[FCH / 64];
  __shared__ int32_t s_prev_end;  // tile offset where the previous tile's last line ends (from line 0)
  __shared__ int32_t s_last_end;  // tile offset where this tile's last line ends (-1: past the LOOK bytes)
  __shared__ int64_t s_tile, s_excl;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  dload(d);  // once per workgroup (persistent)
  for (int i = tid; i < 256; i += FTPB) s_conv[i] = (uint8_t)(i < 128 ? d.sym[i] : i);  // (read after the ticket's barrier)
  load_ranges(s_rng);
  if (tid < 8) s_text[(FTILE + LOOK) / 4 + tid] = 0u;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  LT_INIT();
  // the next tile's ticket is taken at the start of this tile's writes (its atomic's round trip
  // under them), after this tile has published its inclusive prefix: a later tile's look-back never
  // waits on a claimed tile whose holder is still walking
  if (tid == 0) s_tile = (int64_t)atomicAdd(ticket, 1u);
  for (int i = tid; i < FNBW; i += FTPB) s_cs[i] = 0u;
  for (;;) {
    __syncthreads();
    const int64_t tile = (int64_t)__builtin_amdgcn_readfirstlane((int)s_tile);  // < 2^31 tiles
    if (tile >= ntiles) {  // uniform
      LT_FLUSH();
      return;
    }
    LT(0);
    const int64_t tile0 = tile * FTILE;
    // ---- A: text -> LDS, line-start bits, chunk counts -----------------------------------------
    const int64_t qlast = nbytes > 0 ? (nbytes - 1) & ~(int64_t)(PIECE - 1) : 0;  // (krca_log_scan returns before any kernel when nbytes == 0)
    u32x4 raw[FNIT];
    uint32_t pw[FNIT];
#pragma unroll
    for (int it = 0; it < FNIT; ++it) {  // every piece's load out before any is used
      const int64_t q = tile0 + ((int64_t)it * FTPB + tid) * PIECE;
      raw[it] = *reinterpret_cast<const u32x4*>(text + (q < nbytes ? q : qlast));
      const int64_t q0 = tile0 + ((int64_t)it * FTPB + (int64_t)__builtin_amdgcn_readfirstlane(wid) * 64) * PIECE;
      pw[it] = q0 >= 4 && q0 <= nbytes ? *reinterpret_cast<const uint32_t*>(text + q0 - 4) : 0u;
    }
    u32x4 rawx = {0u, 0u, 0u, 0u};  // the last wave: the LOOK bytes after the tile, a piece per lane
    uint32_t pwx = 0;
    if (wid == FTPB / 64 - 1) {
      const int64_t q = tile0 + FTILE + (int64_t)lane * PIECE;
      rawx = *reinterpret_cast<const u32x4*>(text + (q < nbytes ? q : qlast));
      pwx = tile0 + FTILE <= nbytes ? *reinterpret_cast<const uint32_t*>(text + tile0 + FTILE - 4) : 0u;
    }
    LT(8);
    tile_container_starts_t<FTILE + LOOK, true>(s_cs, tile0, nbytes, doc_off, D, chunk_doc);  // (its barriers order LDS reuse)
    LT(9);
    uint32_t regS[FNIT], regL1[FNIT];  // per piece: starts | odd lengths << 16; lengths 2/3
#pragma unroll
    for (int it = 0; it < FNIT; ++it) {
      const int pc = it * FTPB + tid;  // piece index in the tile
      const int64_t q = tile0 + (int64_t)pc * PIECE;
      const bool in = q < nbytes;
      uint32_t w[4] = {in ? raw[it].x : 0u, in ? raw[it].y : 0u, in ? raw[it].z : 0u, in ? raw[it].w : 0u};
      *reinterpret_cast<u32x4*>(s_text + pc * 4) =
          u32x4{sym_word(s_conv, w[0]), sym_word(s_conv, w[1]), sym_word(s_conv, w[2]), sym_word(s_conv, w[3])};
      uint32_t wp = __shfl_up(w[3], 1, 64);  // bytes q-4 .. q-1
      if (lane == 0) wp = pw[it];
      const uint32_t C = in ? piece_container_starts(s_cs, tile0, q) : 0u;
      uint32_t S, l0, l1;
      piece_flags(wp, w, C & 0xFFFFu, S, l0, l1);
      if (in) {
        S |= C >> 1;
        if (q + PIECE > nbytes) S &= (1u << (int)(nbytes - q)) - 1u;
      } else {
        S = 0;
      }
      regS[it] = S | ((l0 & S) << 16);
      regL1[it] = l1 & S;
      uint32_t c = __popc(S);
#pragma unroll
      for (int o = LANES_PER_CHUNK / 2; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);  // 16 lanes = one chunk
      if ((tid & (LANES_PER_CHUNK - 1)) == 0) s_cnt[pc / LANES_PER_CHUNK] = (int32_t)c;
    }
    LT(10);
    __syncthreads();
    LT(1);
    if (tid < FCH) {  // chunk counts -> exclusive bases inside the tile
      const int32_t v = s_cnt[tid];
      chunk_cnt[tile * FCH + tid] = v;
      int32_t x = v;
      for (int off = 1; off < 64; off <<= 1) {
        const int32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
      }
      if (lane == 63) s_wsum[wid] = x;
      s_cb[tid] = x - v;
    }
    __syncthreads();
    int total = 0;
#pragma unroll
    for (int u = 0; u < FCH / 64; ++u) total += s_wsum[u];
    if (tid < FCH) {
      int32_t before = 0;
      for (int u = 0; u < wid; ++u) before += s_wsum[u];
      s_cb[tid] += before;
    }
    if (tid == 0)  // publish the aggregate early: later tiles' look-backs need no more from this one
      __hip_atomic_store(&status[tile], (tile == 0 ? LB_INC : LB_AGG) | (uint64_t)total, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    LT(2);
    if (wid == FTPB / 64 - 1) {  // the LOOK bytes (the last wave, beside wave 0's look-back): their symbols,
                                 // and the first line start in them ends the tile's last line
      const int64_t q = tile0 + FTILE + (int64_t)lane * PIECE;
      const bool in = q < nbytes;
      uint32_t w[4] = {in ? rawx.x : 0u, in ? rawx.y : 0u, in ? rawx.z : 0u, in ? rawx.w : 0u};
      *reinterpret_cast<u32x4*>(s_text + FTILE / 4 + lane * 4) =
          u32x4{sym_word(s_conv, w[0]), sym_word(s_conv, w[1]), sym_word(s_conv, w[2]), sym_word(s_conv, w[3])};
      uint32_t wp = __shfl_up(w[3], 1, 64);
      if (lane == 0) wp = pwx;
      const uint32_t C = in ? piece_container_starts(s_cs, tile0, q) : 0u;
      uint32_t S, l0, l1;
      piece_flags(wp, w, C & 0xFFFFu, S, l0, l1);
      if (in) {
        S |= C >> 1;
        if (q + PIECE > nbytes) S &= (1u << (int)(nbytes - q)) - 1u;
      } else {
        S = 0;
      }
      const uint64_t any = __ballot(S != 0);
      if (any) {
        if (lane == __builtin_ctzll(any)) {
          const int k = __ffs(S) - 1;
          s_last_end = FTILE + lane * PIECE + k - ((int)((l0 >> k) & 1u) | (int)(((l1 >> k) & 1u) << 1));
        }
      } else if (lane == 0) {  // no line starts there: the text's last line, or one longer than LOOK
        s_last_end = tile0 + FTILE + LOOK >= nbytes ? (int32_t)(last_line_end(text, nbytes, doc_off, D) - tile0) : -1;
      }
    }
    // the look-back right away (wave 0): its inclusive prefix goes out before this tile's walk, so
    // later tiles find it within a round or two instead of summing aggregates back over every tile
    // still walking (published after the walk, the look-backs scanned ~2 x 512 tiles: 443 us, r4g)
    if (wid == 0) {
      int64_t excl = 0;
      if (tile > 0) {
        for (int64_t top = tile - 1;; top -= 64) {
          const int64_t t = top - lane;  // lane 0 = the nearest predecessor of the window
          uint64_t sv = t >= 0 ? lb_load(&status[t]) : LB_INC;
          while (__any((sv >> 62) == 0)) {  // some predecessor has not published yet
            __builtin_amdgcn_s_sleep(1);
            if ((sv >> 62) == 0) sv = lb_load(&status[t]);
          }
          const uint64_t inc = __ballot((sv >> 62) == 2);
          const int first = inc ? __builtin_ctzll(inc) : 64;  // nearest inclusive prefix (lowest lane)
          int64_t val = (lane <= first && t >= 0) ? (int64_t)(sv & LB_VAL) : 0;
          for (int off = 32; off > 0; off >>= 1) val += (int64_t)__shfl_xor((long long)val, off, 64);
          excl += val;
          if (inc) break;
        }
        if (lane == 0)
          __hip_atomic_store(&status[tile], LB_INC | (uint64_t)(excl + total), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
      if (lane == 0) {
        s_excl = excl;
        if (FTILE == TILE) tile_base[tile] = excl;  // the 64 KiB tiles' bases (krca_log_match)
        else if ((tile & 1) == 0) tile_base[tile >> 1] = excl;
        if (tile == ntiles - 1) {
          const int64_t nl = excl + total;
          tile_base[nt64] = nl;
          *n_lines = nl;
          if (nl >= 1 && nl <= cap && nbytes > 0) line_end[nl - 1] = last_line_end(text, nbytes, doc_off, D);
        }
      }
    }
    LT(3);  // (thread 0 is in wave 0: the look-back)
    // ---- B + C, one window of LMAX lines at a time (one window unless lines average < 16 B) ----
    const int nwin = total > 0 ? (total + LMAX - 1) / LMAX : 1;
    for (int win = 0; win < nwin; ++win) {
      const int lo = win * LMAX, hi = min(total, lo + LMAX);
      // the window's list: starts of lines [lo, hi), ends of lines [lo, hi) (from the next start)
#pragma unroll
      for (int it = 0; it < FNIT; ++it) {
        const int pc = it * FTPB + tid;
        const uint32_t S = regS[it] & 0xFFFFu;
        const uint32_t n = __popc(S);
        uint32_t xs = n;
#pragma unroll
        for (int off = 1; off < LANES_PER_CHUNK; off <<= 1) {
          const uint32_t y = __shfl_up(xs, off, 64);
          if ((lane & (LANES_PER_CHUNK - 1)) >= off) xs += y;
        }
        int id = s_cb[pc / LANES_PER_CHUNK] + (int)(xs - n);
        if (id > hi || id + (int)n <= lo) continue;  // none of this piece's starts touches the window
        uint32_t rem = S;
        const uint32_t l0 = regS[it] >> 16, l1 = regL1[it];
        while (rem) {
          const int k = __ffs(rem) - 1;
          rem &= rem - 1;
          const int pos = pc * PIECE + k;  // tile offset
          const int sl = (int)((l0 >> k) & 1u) | (int)(((l1 >> k) & 1u) << 1);
          if (id >= lo && id < hi) s_ls[id - lo] = (uint16_t)pos;
          if (id - 1 >= lo && id - 1 < hi) s_le[id - 1 - lo] = (uint16_t)(pos - sl);
          if (id == 0) s_prev_end = pos - sl;
          ++id;
        }
      }
      for (int i = tid; i < LMAX / 2; i += FTPB) s_lm[i] = 0u;
      if (tid == 0) s_nsplit = 0;
      __syncthreads();
      LT(4);
      // The DFA walk: a lane per line, from LDS (long lines: log_dfa_long).  The walk phase lasts as
      // long as the tile's longest line (a lane's steps are one dependent chain of LDS reads), so
      // lines over SPLIT_T bytes take two lanes when the window has the spare lanes: [s, m) and
      // [m', e), m' = m - WARM (warm-up: from the start state, every match starting at or after m'
      // is found, and no match is 24 code points or longer; further back when a byte >= 0x80 there).
      const int n = hi - lo;
      for (int j = tid; j < n; j += FTPB) {
        const int ls = s_ls[j], le = lo + j == total - 1 ? s_last_end : (int)s_le[j];
        if (le >= 0 && le - ls > SPLIT_T && le - ls <= LONG_LINE) {
          const int k = atomicAdd(&s_nsplit, 1);
          if (k < SPLIT_MAX) s_sj[k] = (int16_t)j;
        }
      }
      __syncthreads();
      const int ns = s_nsplit;
      const bool split = ns <= SPLIT_MAX && n + ns <= FTPB;
      for (int t = tid; t < n + (split ? ns : 0); t += FTPB) {
        const int j = t < n ? t : s_sj[t - n];
        const int ls = s_ls[j], le = lo + j == total - 1 ? s_last_end : (int)s_le[j];
        if (le < 0 || le - ls > LONG_LINE) continue;
        int a = ls, b = le;
        if (split && le - ls > SPLIT_T) {
          const int m = ls + (le - ls + WARM) / 2;
          if (t < n) b = m;
          else a = max(ls, any_high(s_text, m - WARM, m) ? m - 4 * WARM - 3 : m - WARM);
        }
        const uint32_t mk = a < b ? dfa_walk_sym(s_text, d, s_rng, a, b) : 0u;
        if (mk) atomicOr(&s_lm[j >> 1], mk << (16 * (j & 1)));
      }
      __syncthreads();
      LT(5);
      unsigned int next = 0;
      if (tid == 0 && win == nwin - 1) next = atomicAdd(ticket, 1u);
      if (win == nwin - 1)  // the next tile's container bitmap (A and the LOOK pass are done with it)
        for (int i = tid; i < FNBW; i += FTPB) s_cs[i] = 0u;
      const int64_t excl = s_excl;
      if (win == 0 && tid < FCH) chunk_line0[tile * FCH + tid] = excl + s_cb[tid];
      if (win == 0 && tid == 0 && total > 0 && excl >= 1 && excl - 1 < cap)
        line_end[excl - 1] = tile0 + s_prev_end;  // the previous tile's last line ends before line 0 here
      if (win == 0 && tile == ntiles - 1)  // an odd tile count: the last 64 KiB tile's missing half has no
        for (int64_t c = ntiles * FCH + tid; c < nt64 * TPB; c += FTPB) {  // line starts (log_hist and
          chunk_cnt[c] = 0;                                                 // log_lines read its chunks)
          chunk_line0[c] = excl + total;
        }
      for (int j = tid; j < hi - lo; j += FTPB) {  // coalesced by line id
        const int64_t id = excl + lo + j;
        if (id >= cap) continue;
        const int ls = s_ls[j], le = lo + j == total - 1 ? s_last_end : (int)s_le[j];
        line_start[id] = tile0 + ls;
        if (le >= 0) line_end[id] = tile0 + le;  // (a last line's end also comes from the next tile)
        if (le < 0 || le - ls > LONG_LINE) long_q[atomicAdd(n_long, 1)] = (int32_t)id;
        else line_mask[id] = (s_lm[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
      }
      if (tid == 0 && win == nwin - 1) s_tile = (int64_t)next;  // (read after the barrier below)
      __syncthreads();  // the window's lists (and, after the last, the tile's LDS) are rewritten next
      LT(6);
    }
#ifdef LOG_TIMING
    lt_acc[7] += 1;
#endif
  }
}

int64_t num_tiles(int64_t nbytes) { return std::max<int64_t>(1, krca::ceil_div(nbytes, TILE)); }
// int64 words of the int32 long-line queue (lines longer than LONG_LINE: at most nbytes / LONG_LINE,
// + one per tile whose last line runs past its LOOK bytes)
int64_t long_q_words(int64_t nbytes) { return krca::ceil_div(nbytes / LONG_LINE + 2 * num_tiles(nbytes) + 2, 2); }
// krca_log_scan's tail of the workspace (int64 words): look-back status words for the 2 x num_tiles
// 32 KiB tiles of log_index_match (num_tiles of log_index_lines use the first half), the tile ticket
int64_t scan_tail_words(int64_t nbytes) { return 2 * num_tiles(nbytes) + 1; }

}  // namespace

extern "C" {

// workspace (int64 units): [ntiles+1] tile base | [ntiles*TPB] int32 chunk counts |
// [ntiles*TPB] int32 chunk -> container | [ntiles*TPB] int64 first line id per chunk |
// [1] long-line count | int32 long-line queue [long_q_words] | [ntiles] look-back status |
// [1] tile ticket (the last two: krca_log_scan)
const char* krca_log_dfa_unicode(void) { return KRCA_DFA_UNIDATA; }
uint64_t krca_log_dfa_digest(void) { return KRCA_DFA_DIGEST; }

int64_t krca_log_index_size(int64_t nbytes) {
  const int64_t nt = num_tiles(nbytes);
  return (nt + 1) + 2 * krca::ceil_div(nt * TPB, 2) + 2 + nt * TPB + 1 + long_q_words(nbytes) +
         scan_tail_words(nbytes);  // + krca_log_scan's look-back status words, ticket, deferred-line queue
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
  KRCA_HIP(hipMemsetAsync(cdoc, 0, nt * TPB * sizeof(int32_t), st));  // defined map even off-contract
  hipLaunchKernelGGL(log_chunk_doc, dim3((unsigned)krca::ceil_div(ndocs, TPB)), dim3(TPB), 0, st, doc_off, ndocs,
                     nbytes, cdoc, (unsigned long long*)nullptr, (int64_t)0, (int32_t*)nullptr);
  KRCA_LAUNCH_CHECK();
  hipLaunchKernelGGL(log_count, dim3((unsigned)nt), dim3(TPB), 0, st, text, nbytes, doc_off, ndocs,
                     (const int32_t*)cdoc, chunk, tile);
  KRCA_LAUNCH_CHECK();
  hipLaunchKernelGGL(log_scan, dim3(1), dim3(1024), 0, st, tile, nt, n_lines);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_log_match(const uint8_t* text, int64_t nbytes, const int64_t* doc_off, int64_t ndocs, int64_t* ws,
                   int64_t n_lines, int64_t* line_start, int64_t* line_end, uint32_t* line_mask, int32_t* doc_lines,
                   int32_t* hist, int32_t* examples, int64_t* doc_line0, void* stream) {
  KRCA_CHECK_ARG(nbytes >= 0 && ndocs >= 1 && n_lines >= 0, "krca_log_match: bad sizes");
  KRCA_CHECK_ARG(doc_off && ws && doc_lines && hist, "krca_log_match: null pointer");
  KRCA_CHECK_ARG(((uintptr_t)text & 15) == 0, "krca_log_match: text must be 16-byte aligned");
  KRCA_CHECK_ARG(n_lines == 0 || (line_start && line_end && line_mask), "krca_log_match: null line arrays");
  const int64_t nt = num_tiles(nbytes);
  const int64_t* tile = ws;
  const int32_t* chunk = reinterpret_cast<const int32_t*>(ws + nt + 1);
  const int32_t* cdoc = chunk + 2 * krca::ceil_div(nt * TPB, 2);
  int64_t* chunk_line0 = ws + (nt + 1) + 2 * krca::ceil_div(nt * TPB, 2) + 2;
  int32_t* n_long = reinterpret_cast<int32_t*>(chunk_line0 + nt * TPB);
  int32_t* long_q = reinterpret_cast<int32_t*>(chunk_line0 + nt * TPB + 1);
  hipStream_t st = krca::as_stream(stream);
  const int impl = krca::tuning().log_impl;  // A/B: tests switch it with krca_tune_set
  if (n_lines > 0 && impl == 1) {  // A/B: lane per 256-byte chunk, DFA and line logic in one pass
    KRCA_HIP(hipMemsetAsync(line_mask, 0, n_lines * sizeof(uint32_t), st));
    const int64_t grid = std::min<int64_t>(nt, 256 * 4);
    hipLaunchKernelGGL(log_match, dim3((unsigned)grid), dim3(TPB), 0, st, text, nbytes, doc_off, ndocs, cdoc, chunk,
                       tile, nt, n_lines, line_start, line_end, line_mask, chunk_line0);
    KRCA_LAUNCH_CHECK();
  } else if (n_lines > 0) {  // line index, then a DFA lane per line (long lines: a wave each)
    KRCA_HIP(hipMemsetAsync(n_long, 0, sizeof(int32_t), st));
    hipLaunchKernelGGL(log_lines, dim3((unsigned)nt), dim3(TPB), 0, st, text, nbytes, doc_off, ndocs, cdoc, chunk, tile,
                       n_lines, line_start, line_end, chunk_line0);
    KRCA_LAUNCH_CHECK();
    hipLaunchKernelGGL(log_last_end, dim3(1), dim3(1), 0, st, text, nbytes, doc_off, ndocs, n_lines,
                       (const int64_t*)nullptr, (int64_t)0, line_end);
    KRCA_LAUNCH_CHECK();
    if (impl == 2) {  // A/B: the round-1 walk (16-byte window, code point per step)
      const int64_t grid = std::min<int64_t>(krca::ceil_div(n_lines, DFA_TPB), 256 * 4);
      hipLaunchKernelGGL(log_dfa_window, dim3((unsigned)grid), dim3(DFA_TPB), 0, st, text, nbytes, n_lines,
                         (const int64_t*)line_start, (const int64_t*)line_end, line_mask, long_q, n_long);
    } else {  // persistent: the 50 KB table is filled once per workgroup, 3 workgroups per CU
      const int64_t grid = std::min<int64_t>(krca::ceil_div(n_lines, DFA_TPB), 256 * 3);
      hipLaunchKernelGGL(log_dfa, dim3((unsigned)grid), dim3(DFA_TPB), 0, st, text, nbytes, n_lines,
                         (const int64_t*)nullptr, (int64_t)0, (const int64_t*)line_start, (const int64_t*)line_end, line_mask, long_q, n_long);
    }
    KRCA_LAUNCH_CHECK();
    hipLaunchKernelGGL(log_dfa_long, dim3(256), dim3(TPB), 0, st, text, nbytes, (const int64_t*)line_start,
                       (const int64_t*)line_end, line_mask, (const int32_t*)long_q, (const int32_t*)n_long);
    KRCA_LAUNCH_CHECK();
  } else {  // no lines: chunk_line0 = 0 for log_hist
    KRCA_HIP(hipMemsetAsync(chunk_line0, 0, nt * TPB * sizeof(int64_t), st));
  }
  hipLaunchKernelGGL(examples ? log_hist<true> : log_hist<false>, dim3((unsigned)krca::ceil_div(ndocs, TPB)), dim3(TPB),
                     0, st, doc_off, ndocs, (const int64_t*)chunk_line0, nt * TPB, line_start, line_mask, n_lines,
                     (const int64_t*)nullptr, (int64_t)0, doc_lines, hist, examples, doc_line0);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int krca_log_scan(const uint8_t* text, int64_t nbytes, const int64_t* doc_off, int64_t ndocs, int64_t* ws,
                  int64_t line_cap, int64_t* line_start, int64_t* line_end, uint32_t* line_mask, int32_t* doc_lines,
                  int32_t* hist, int32_t* examples, int64_t* doc_line0, int64_t* n_lines_host, void* stream) {
  KRCA_CHECK_ARG(nbytes >= 0 && ndocs >= 1 && ndocs < INT32_MAX && line_cap >= 0, "krca_log_scan: bad sizes");
  KRCA_CHECK_ARG(doc_off && ws && doc_lines && hist && n_lines_host, "krca_log_scan: null pointer");
  KRCA_CHECK_ARG(nbytes == 0 || text, "krca_log_scan: null text");
  KRCA_CHECK_ARG(((uintptr_t)text & 15) == 0, "krca_log_scan: text must be 16-byte aligned");
  KRCA_CHECK_ARG(line_cap == 0 || (line_start && line_end && line_mask), "krca_log_scan: null line arrays");
  const int64_t nt = num_tiles(nbytes);
  int64_t* tile = ws;  // tile[nt] = the line count, on the device
  int32_t* chunk = reinterpret_cast<int32_t*>(ws + nt + 1);
  int32_t* cdoc = chunk + 2 * krca::ceil_div(nt * TPB, 2);
  int64_t* chunk_line0 = ws + (nt + 1) + 2 * krca::ceil_div(nt * TPB, 2) + 2;
  int32_t* n_long = reinterpret_cast<int32_t*>(chunk_line0 + nt * TPB);
  int32_t* long_q = reinterpret_cast<int32_t*>(chunk_line0 + nt * TPB + 1);
  unsigned long long* status =
      reinterpret_cast<unsigned long long*>(chunk_line0 + nt * TPB + 1 + long_q_words(nbytes));
  unsigned int* ticket = reinterpret_cast<unsigned int*>(status + 2 * nt);
  hipStream_t st = krca::as_stream(stream);
  if (nbytes == 0) {
    // no text (the pointer may be null): every container is empty and no kernel may read text --
    // the index pass's unconditional piece loads clamp to the last 16-byte block that holds a
    // byte, and there is none (an empty window faulted there: test_log_scan_degenerate_texts)
    KRCA_HIP(hipMemsetAsync(tile, 0, (nt + 1) * sizeof(int64_t), st));  // tile bases, the line count
    KRCA_HIP(hipMemsetAsync(chunk_line0, 0, nt * TPB * sizeof(int64_t), st));
    KRCA_HIP(hipMemsetAsync(doc_lines, 0, ndocs * sizeof(int32_t), st));
    KRCA_HIP(hipMemsetAsync(hist, 0, ndocs * KRCA_NCAT * sizeof(int32_t), st));
    if (examples) KRCA_HIP(hipMemsetAsync(examples, 0xFF, ndocs * KRCA_NCAT * 3 * sizeof(int32_t), st));  // -1
    if (doc_line0) KRCA_HIP(hipMemsetAsync(doc_line0, 0, ndocs * sizeof(int64_t), st));
    *n_lines_host = 0;
    return KRCA_OK;
  }
  // one launch before the index: the chunk -> container map (every chunk of the text is written
  // under the doc_off contract; off it, tile_container_starts clamps what it reads), and the zeroed
  // look-back status words + ticket and long-line count (no memset launches: each dependent
  // launch costs ~10 us at the front of the scan)
  hipLaunchKernelGGL(log_chunk_doc, dim3((unsigned)krca::ceil_div(ndocs, TPB)), dim3(TPB), 0, st, doc_off, ndocs,
                     nbytes, cdoc, status, 2 * nt + 1, n_long);  // status words, ticket
  KRCA_LAUNCH_CHECK();
  const int64_t* Ld = tile + nt;  // the line count, on the device (written by the index's last tile)
  if (krca::tuning().log_fused) {
    // A/B: the line index and the DFA walk in one pass over the text (KRCA_LOG_FUSED = 1: 32 KiB
    // tiles, two 512-thread workgroups per CU; 2: 64 KiB tiles, one 1024-thread workgroup per CU);
    // long lines go to log_dfa_long.  It reads the text once but runs its phases one after the
    // other per tile
    auto launch = [&](auto cfg) -> int64_t {
      using CF = decltype(cfg);
      const int64_t ntf = num_ftiles(nbytes, CF::FTILE);
      const int64_t resident =
          krca::resident_workgroups(reinterpret_cast<const void*>(&log_index_match<CF>), CF::FTPB, st, 1);
      hipLaunchKernelGGL(log_index_match<CF>, dim3((unsigned)std::min<int64_t>(ntf, resident)), dim3(CF::FTPB), 0, st,
                         text, nbytes, doc_off, ndocs, (const int32_t*)cdoc, chunk, tile, nt, status, ticket, ntf,
                         line_cap, line_start, line_end, line_mask, chunk_line0, tile + nt, long_q, n_long);
      return ntf;
    };
    if (krca::tuning().log_fused == 2) launch(FBig{});
    else launch(FSmall{});
    KRCA_LAUNCH_CHECK();
  } else {  // default (KRCA_LOG_FUSED=0): the line index, then a DFA lane per line re-reading the text
    // workgroups the stream's device keeps resident (occupancy API, cached per device)
    const int64_t resident = krca::resident_workgroups(reinterpret_cast<const void*>(&log_index_lines), TPB, st, 4);
    const int64_t grid_ix = LOG_IDX_PERSIST ? std::min<int64_t>(nt, resident) : nt;
    hipLaunchKernelGGL(log_index_lines, dim3((unsigned)grid_ix), dim3(TPB), 0, st, text, nbytes, doc_off, ndocs,
                       (const int32_t*)cdoc, chunk, tile, status, ticket, nt, line_cap, line_start, line_end, chunk_line0,
                       tile + nt);
    KRCA_LAUNCH_CHECK();
    const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(krca::ceil_div(line_cap, DFA_TPB), 256 * 3));
    hipLaunchKernelGGL(log_dfa, dim3((unsigned)grid), dim3(DFA_TPB), 0, st, text, nbytes, (int64_t)0, Ld, line_cap,
                       (const int64_t*)line_start, (const int64_t*)line_end, line_mask, long_q, n_long);
    KRCA_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(log_dfa_long, dim3(256), dim3(TPB), 0, st, text, nbytes, (const int64_t*)line_start,
                     (const int64_t*)line_end, line_mask, (const int32_t*)long_q, (const int32_t*)n_long);
  KRCA_LAUNCH_CHECK();
  hipLaunchKernelGGL(examples ? log_hist<true> : log_hist<false>, dim3((unsigned)krca::ceil_div(ndocs, TPB)), dim3(TPB),
                     0, st, doc_off, ndocs, (const int64_t*)chunk_line0, nt * TPB, line_start, line_mask, (int64_t)0, Ld,
                     line_cap, doc_lines, hist, examples, doc_line0);
  KRCA_LAUNCH_CHECK();
  KRCA_HIP(hipMemcpyAsync(n_lines_host, Ld, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  KRCA_HIP(hipStreamSynchronize(st));
  return KRCA_OK;
}

#ifdef LOG_TIMING
int krca_log_debug_timing(unsigned long long* host, int reset) {  // timing variant builds only
  KRCA_HIP(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_log_timing), sizeof(g_log_timing)));
  if (reset) {
    static unsigned long long zero[1024 * 16];
    KRCA_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_log_timing), zero, sizeof(zero)));
  }
  return KRCA_OK;
}
#endif

}  // extern "C"

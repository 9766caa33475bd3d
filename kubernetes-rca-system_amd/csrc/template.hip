// Error-template hashing and per-container template histograms.
//
// New primitive (no reference code; semantics defined here and restated in oracle/oracle.py):
//   template(line) = the line's bytes with every UUID (five words of 8, 4, 4, 4 and 12 hex
//                    characters joined by single '-') and every other maximal run of [A-Za-z0-9_]
//                    that contains an ASCII digit, or that is >= 8 characters of [0-9a-fA-F],
//                    replaced by the one byte 0xFF (shown as "<*>"; 0xFF never occurs in UTF-8
//                    text, so a masked word can not collide with literal text as the 3-byte "<*>" of
//                    rounds 1-4 could) (masks counters, ids, addresses, timestamps, hashes and UUIDs;
//                    bytes >= 0x80 are never word characters and pass through unchanged);
//   h(line)        = FNV-1a-64 over the template bytes (offset 0xcbf29ce484222325,
//                    prime 0x100000001b3);
//   per container  = the distinct h of its lines in ascending order with their line counts.
//   The word machine is csrc/tmpl_dfa.h (a byte-indexed table built at compile time; round 6 added
//   the UUID rule: rounds 1-5 masked only the groups holding a digit or 8+ hex characters).
//
// krca_template_hash: one lane per line (lines from krca_log_match), each lane reading its line
//   straight from the text; FNV-1a runs through word bytes as if they stayed, and a word (or UUID)
//   that turns out masked is replaced by the mask byte from the hash saved at its start.
// krca_template_hist: sort-based, atomics-free.  Containers with <= 64 lines: one wave, bitonic
//   sort of 64-bit keys across lanes (shuffles), run heads by ballot, counts by ballot distance.
//   <= 4096 lines: one workgroup, bitonic sort in LDS, run compaction by a block scan.
#include "krca_common.h"
#include "tmpl_dfa.h"

#include <algorithm>
#include <climits>

namespace {

constexpr int TPB = 256;
constexpr int BIG = 4096;  // max lines per container handled by the LDS path
constexpr uint64_t kFnvOff = 0xcbf29ce484222325ull;
constexpr uint64_t kFnvPrime = 0x100000001b3ull;

// (the 64-bit multiply is ~10 % of tmpl_hash_kernel: a build with a multiply-free stand-in ran
// 140.9 against 156.2 us, r4w; the per-byte state-table read, a dependent LDS chain, is the rest)
__device__ __forceinline__ uint64_t fnv_mul(uint64_t x) { return x * kFnvPrime; }
__device__ __forceinline__ uint64_t fnv(uint64_t h, uint32_t b) { return fnv_mul(h ^ b); }

// A masked word (or UUID) becomes ONE mask byte: one FNV step from the hash saved at its start
// (with 64 lanes on 64 lines some lane ends a masked word at nearly every byte step, so this branch
// runs at nearly every step for the whole wave; R5v: three steps there, for "<*>", were the largest
// part of the kernel's vector instructions).
constexpr uint32_t kMaskByte = 0xFFu;
__device__ __forceinline__ uint64_t fnv_mask(uint64_t h) { return fnv(h, kMaskByte); }

// The table image (tmpl_dfa.h: kRows x 256 one-byte entries = the next row's index, flags encoded
// in the row ranges), built at compile time; a workgroup copies it into LDS with 16-byte loads
// (filling it entry by entry from class tests cost each wave ~550 instructions, R5zt).
#ifdef KRCA_TMPL_CLS  // A/B build (make tcls): the machine over byte classes (1.1 KB table)
constexpr bool kCls = true;
__device__ constexpr tdfa::ClsTable kClsTable = tdfa::make_cls_table();
constexpr int kTableBytes = (int)sizeof(tdfa::ClsTable);
#else
constexpr bool kCls = false;
constexpr int kTableBytes = tdfa::kRows * 256;
#endif
__device__ constexpr tdfa::Table kTable = tdfa::make_table();
static_assert(kTableBytes % 16 == 0, "16-byte copy");
template <int NT>
__device__ __forceinline__ void load_table(uint8_t* __restrict__ tstate) {  // (the caller syncs)
#ifdef KRCA_TMPL_CLS
  const uint4* src = reinterpret_cast<const uint4*>(&kClsTable);
#else
  const uint4* src = reinterpret_cast<const uint4*>(kTable.v);
#endif
  for (int i = threadIdx.x; i < kTableBytes / 16; i += NT) reinterpret_cast<uint4*>(tstate)[i] = src[i];
}

// h ^ byte k of w in one instruction (the byte read in place as a sub-dword operand; the compiler
// otherwise shifts bytes 1 and 2 down first)
__device__ __forceinline__ uint64_t xor_byte(uint64_t h, uint32_t w, int k) {
  uint32_t lo = (uint32_t)h;
  switch (k) {
    case 0: asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(lo) : "v"(lo), "v"(w)); break;
    case 1: asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(lo) : "v"(lo), "v"(w)); break;
    case 2: asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(lo) : "v"(lo), "v"(w)); break;
    default: asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(lo) : "v"(lo), "v"(w)); break;
  }
  return (h & 0xFFFFFFFF00000000ull) | lo;
}

// the flags of entering row t (tmpl_dfa.h): MEND rows end a masked word (the common case); the U
// rows (a UUID's first group ended / a whole UUID ended) sit past them behind a second, rarely taken
// test; then START (and every flagged row: harmless, a word's start saves it again) keeps the hash
__device__ __forceinline__ void tflags(uint32_t t, uint64_t& h, uint64_t& hb, uint64_t& hu) {
  if (t >= (uint32_t)tdfa::kM0) {
    if (t >= (uint32_t)tdfa::kU0) {
      const uint64_t src = t == (uint32_t)tdfa::kU0 ? hb : hu;
      if (t == (uint32_t)tdfa::kU0) hu = hb;
      h = fnv_mask(src);
    } else {
      h = fnv_mask(hb);
    }
  }
  if (t >= (uint32_t)tdfa::kS0) hb = h;
}

// byte k of dword w; st = the current row index
__device__ __forceinline__ void tstep_rows(const uint8_t* __restrict__ T, uint32_t w, int k, uint32_t& st,
                                           uint64_t& h, uint64_t& hb, uint64_t& hu) {
  uint32_t t;
  if constexpr (kCls) {  // class map (independent of the state), then (st << 3) | class
    const uint32_t c = T[__builtin_amdgcn_perm(0u, w, 0x0c0c0c00u | (uint32_t)k)];
    t = T[256 + ((st << 3) | c)];
  } else {
    t = T[__builtin_amdgcn_perm(st, w, 0x0c0c0400u | (uint32_t)k)];  // (st << 8) | byte k
  }
  tflags(t, h, hb, hu);
  h = fnv_mul(xor_byte(h, w, k));
  st = t;
}
// the end of a line: the flags of the transition on a non-word byte, without hashing it
__device__ __forceinline__ void tstep_end(const uint8_t* __restrict__ T, uint32_t st, uint64_t& h, uint64_t& hb,
                                          uint64_t& hu) {
  tflags(T[kCls ? 256 + ((st << 3) | tdfa::C_OTHER) : (st << 8) | tdfa::kEndByte], h, hb, hu);
}

// the template hash of line [s, e) read byte by byte from the text, the table from global memory
// (a line outside its workgroup's 2 GiB buffer window, or before it: lines not in text order)
__device__ __forceinline__ uint64_t line_hash_global(const uint8_t* __restrict__ text, int64_t nbytes, int64_t s,
                                                     int64_t e) {
  uint64_t h = kFnvOff, hb = 0, hu = 0;
  uint32_t st = 0;
  e = e < nbytes ? e : nbytes;
  for (int64_t q = s; q < e; ++q) {
    const uint32_t b = text[q];
    const uint32_t t = kTable.v[(st << 8) | b];
    tflags(t, h, hb, hu);
    h = fnv(h, b);
    st = t;
  }
  tflags(kTable.v[(st << 8) | tdfa::kEndByte], h, hb, hu);
  return h;
}

// A workgroup's lines ordered by length: a wave takes as long as its longest line, so the lanes of
// wave w take the w-th run of the lines sorted by length / 4 (a counting sort in LDS; lines past L
// land in bucket 0 and are skipped by the caller).  On the C5 corpus the mean of the waves'
// longest lines falls from 1.43x to 1.11x the mean line length at 256 lines per workgroup.
constexpr int NLB = 128;  // length buckets of 4 bytes (the last one takes every longer line)
template <int NT>
__device__ __forceinline__ int sort_by_length(int64_t len, bool valid, uint32_t* __restrict__ bcnt,
                                              uint16_t* __restrict__ perm) {
  const uint32_t bk = valid && len > 0 ? (uint32_t)min<int64_t>(len >> 2, NLB - 1) : 0u;
  for (int i = threadIdx.x; i < NLB; i += NT) bcnt[i] = 0u;
  __syncthreads();
  const uint32_t rank = atomicAdd(&bcnt[bk], 1u);  // (LDS) order inside a bucket: arrival
  __syncthreads();
  if (threadIdx.x < 64) {  // exclusive scan of the NLB counts, two per lane
    const int lane = threadIdx.x;
    const uint32_t c0 = bcnt[2 * lane], c1 = bcnt[2 * lane + 1];
    uint32_t x = c0 + c1;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    const uint32_t ex = x - c0 - c1;
    bcnt[2 * lane] = ex;
    bcnt[2 * lane + 1] = ex + c0;
  }
  __syncthreads();
  perm[bcnt[bk] + rank] = (uint16_t)threadIdx.x;
  __syncthreads();
  return perm[threadIdx.x];
}

// The hash kernel: a workgroup per NT consecutive lines, lane per line in length order, each lane
// reading its line straight from the text in 16-byte buffer loads at the line's dword-aligned start,
// one load ahead.  The workgroup holds the table (25.5 KB) and the sort in LDS; at 512 lanes per
// workgroup the wave cap (4 workgroups, 8 waves per SIMD) binds before the LDS does, so the CU keeps
// 8 waves per SIMD: the walk is bound by each wave's dependent per-byte chain (table read, flag
// tests, the hash's multiply), and the waves hide one another's.  (Round 4 staged each
// workgroup's text span in 24 KB of LDS at 256 lanes, which held the CU to 5 waves per SIMD: 159
// against 106 us for the same 2.5M lines, R5zu; two lines per lane in lockstep, bank-spread and
// flag-row tables at that occupancy were slower or equal, R5zj-R5zm.)
template <int NT>
__global__ __launch_bounds__(NT) void tmpl_hash_kernel(const uint8_t* __restrict__ text, int64_t nbytes,
                                                       const int64_t* __restrict__ ls, const int64_t* __restrict__ le,
                                                       int64_t L, uint64_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t tstate[kTableBytes];
  __shared__ uint32_t bcnt[NLB];
  __shared__ __attribute__((aligned(8))) uint16_t perm[4 * NT];  // (then the hashes, NT x 8 B)
  load_table<NT>(tstate);
  const int64_t l0 = (int64_t)blockIdx.x * NT;
  const int64_t i = l0 + threadIdx.x;
  const int j = sort_by_length<NT>(i < L ? le[i] - ls[i] : 0, i < L, bcnt, perm);  // (syncs: table ready)
  const int64_t li = l0 + j;
  const int64_t s = li < L ? ls[li] : 0, e = li < L ? le[li] : 0;
  const int64_t base = ls[l0] & ~(int64_t)15;  // the workgroup's buffer window starts at its first line
  // lines in the window are walked here; a line beyond a 2 GiB window, or before the window (lines
  // not in text order), is read directly after the walk (every lane reaches the barriers below)
  const bool in_window = s >= base && e - base <= (int64_t)INT32_MAX - 64;
  const int64_t rem = nbytes - base;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(text + base), 0, (int)(rem < (int64_t)INT32_MAX ? rem : (int64_t)INT32_MAX), 0x00020000);
  auto load = [&](int q) -> uint4 {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, q, 0, 0));
  };
  // (reads past the text return 0 and are never hashed; a load straddling the text's end reads 0
  // for all 16 bytes, so that piece is rebuilt byte by byte)
  auto fix = [&](uint4& v, int q) {
    if (q + 16 > rem && q < rem) {
      uint32_t ww[4] = {0, 0, 0, 0};
      for (int k = 0; k < 16; ++k)
        if (q + k < rem) ww[k >> 2] |= (uint32_t)text[base + q + k] << (8 * (k & 3));
      v = make_uint4(ww[0], ww[1], ww[2], ww[3]);
    }
  };
  // the line's next 16 bytes as dwords, realigned to its start
  auto words = [](const uint4& c, const uint4& nx, uint32_t sh, uint32_t* w) {
    w[0] = __builtin_amdgcn_alignbyte(c.y, c.x, sh);
    w[1] = __builtin_amdgcn_alignbyte(c.z, c.y, sh);
    w[2] = __builtin_amdgcn_alignbyte(c.w, c.z, sh);
    w[3] = __builtin_amdgcn_alignbyte(nx.x, c.w, sh);
  };
  const uint32_t sh = (uint32_t)(s & 3);
  int q = in_window ? (int)((s & ~(int64_t)3) - base) : 0;
  int n = in_window ? (int)(e - s) : 0;
  uint64_t h = kFnvOff, hb = 0, hu = 0;
  uint32_t st = 0;
  uint4 cur = load(q), nxt = load(q + 16);
  fix(cur, q);
  for (; n >= 16; n -= 16) {
    const uint4 nn = load(q + 32);
    fix(nxt, q + 16);
    uint32_t w[4];
    words(cur, nxt, sh, w);
#pragma unroll
    for (int k = 0; k < 16; ++k) tstep_rows(tstate, w[k >> 2], k & 3, st, h, hb, hu);
    cur = nxt;
    nxt = nn;
    q += 16;
  }
  if (n > 0) {  // the last 1..15 bytes: whole dwords with static byte positions, then 1..3 bytes
    fix(nxt, q + 16);
    uint32_t w[4];
    words(cur, nxt, sh, w);
    for (; n >= 4; n -= 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) tstep_rows(tstate, w[0], k, st, h, hb, hu);
      w[0] = w[1];
      w[1] = w[2];
      w[2] = w[3];
    }
    for (int k = 0; k < n; ++k) tstep_rows(tstate, w[0], k, st, h, hb, hu);
  }
  tstep_end(tstate, st, h, hb, hu);  // a trailing masked word or UUID
  if (!in_window) h = line_hash_global(text, nbytes, s, e);
  // the hashes leave through LDS in line order (full-line stores; one 8-byte store per lane at its
  // sorted line's slot wrote 41 MB at the DRAM side for 20 MB, R5zzi: 103.0 -> 100.9 us, R5zzj)
  uint64_t* sh_out = reinterpret_cast<uint64_t*>(perm);  // (perm is dead once every lane has read j)
  __syncthreads();
  if (li < L) sh_out[j] = h;
  __syncthreads();
  if (l0 + threadIdx.x < L) out[l0 + threadIdx.x] = sh_out[threadIdx.x];
}

// ---- per-container histograms ----------------------------------------------------------------
__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  return (uint64_t)__shfl_xor((long long)v, m, 64);
}

// Containers by size, one lane each (a C5 container holds ~2.5 lines): up to LANE_MAX lines are
// sorted in the lane's registers (odd-even transposition network, static indices) and emitted
// here; larger ones are appended to the mid (<= 64), big (<= BIG) or huge lists of the workspace,
// one atomic per wave and list.  (Round 1 gave every container a whole wave: 1M mostly idle waves,
// 0.5 ms per C5 window.)
constexpr int LANE_MAX = 8;
constexpr int MID_MAX = 64;
__device__ __forceinline__ void wave_append(bool take, int32_t d, int32_t* cnt, int32_t* list) {
  const uint64_t m = __ballot(take);
  if (!m) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((unsigned long long)m) - 1;
  int32_t base = 0;
  if (lane == leader) base = atomicAdd(cnt, __popcll(m));
  base = __shfl(base, leader, 64);
  if (take) list[base + __popcll(m & ((1ull << lane) - 1ull))] = d;
}

// A workgroup's 256 containers hold consecutive line ranges (the log scan's layout): their hashes
// are staged in LDS with coalesced loads and the results leave the same way (per-lane 8-byte loads
// and stores at each container's own slots otherwise: a wave's 16 store instructions each touched
// ~10 cache lines).  Slots of the larger containers in the span are written here too (their raw
// hashes) and rewritten by the kernels that take them.  A workgroup whose ranges are not
// consecutive, or whose span exceeds HCAP lines, takes the per-lane path.
constexpr int HCAP = 1024;
__global__ __launch_bounds__(TPB) void tmpl_hist_lane(const uint64_t* __restrict__ hash,
                                                      const int32_t* __restrict__ doc_lines,
                                                      const int64_t* __restrict__ doc_line0, int64_t D,
                                                      uint64_t* __restrict__ out_hash, int32_t* __restrict__ out_cnt,
                                                      int32_t* __restrict__ n_tmpl, int32_t* __restrict__ ws) {
  __shared__ uint64_t s_key[HCAP];
  __shared__ int32_t s_cn[HCAP];
  __shared__ int64_t s_lo[TPB + 1];
  const int64_t d0 = (int64_t)blockIdx.x * TPB;
  const int64_t d = d0 + threadIdx.x;
  const int nv = (int)(D - d0 < TPB ? D - d0 : TPB);
  const int n = d < D ? doc_lines[d] : 0;
  int32_t* cnt = ws;
  int32_t* lists = ws + 4;
  wave_append(d < D && n > LANE_MAX && n <= MID_MAX, (int32_t)d, cnt + 0, lists);
  wave_append(d < D && n > MID_MAX && n <= BIG, (int32_t)d, cnt + 1, lists + D);
  wave_append(d < D && n > BIG, (int32_t)d, cnt + 2, lists + 2 * D);
  const int64_t lo = d < D ? doc_line0[d] : 0;
  s_lo[threadIdx.x] = lo;
  if ((int)threadIdx.x == nv - 1) s_lo[TPB] = lo + n;  // the span's end
  __syncthreads();
  const int64_t s0 = s_lo[0], s1 = s_lo[TPB];
  const bool next_ok = d >= D || n < 0 || lo + n == ((int)threadIdx.x + 1 < nv ? s_lo[threadIdx.x + 1] : s1);
  const bool staged = __syncthreads_and(next_ok && (d >= D || n >= 0)) && s1 >= s0 && s1 - s0 <= HCAP;
  const int span = staged ? (int)(s1 - s0) : 0;
  uint64_t v[LANE_MAX];
  const bool mine = d < D && n <= LANE_MAX;
  if (staged) {
    for (int i = threadIdx.x; i < span; i += TPB) {
      s_key[i] = hash[s0 + i];
      s_cn[i] = 0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < LANE_MAX; ++j) v[j] = mine && j < n ? s_key[lo - s0 + j] : ~0ull;
  } else {
#pragma unroll
    for (int j = 0; j < LANE_MAX; ++j) v[j] = mine && j < n ? hash[lo + j] : ~0ull;
  }
#pragma unroll
  for (int r = 0; r < LANE_MAX; ++r)
#pragma unroll
    for (int j = r & 1; j + 1 < LANE_MAX; j += 2) {
      const uint64_t a = v[j], b = v[j + 1];
      v[j] = a < b ? a : b;
      v[j + 1] = a < b ? b : a;
    }
  uint64_t* oh = staged ? s_key + (lo - s0) : out_hash + lo;  // (this lane's own slots)
  int32_t* oc = staged ? s_cn + (lo - s0) : out_cnt + lo;
  if (mine) {
    int k = 0, run = 0;
#pragma unroll
    for (int j = 0; j < LANE_MAX; ++j) {  // runs of equal keys among the first n
      if (j < n) {
        ++run;
        if (j + 1 == n || v[j + 1] != v[j]) {
          oh[k] = v[j];
          oc[k] = run;
          ++k;
          run = 0;
        }
      }
    }
#pragma unroll
    for (int j = 1; j < LANE_MAX; ++j)  // the slots past the templates (every slot is written: no fill)
      if (j >= k && j < n) {
        oh[j] = 0ull;
        oc[j] = 0;
      }
    n_tmpl[d] = k;
  }
  if (staged) {
    __syncthreads();
    for (int i = threadIdx.x; i < span; i += TPB) {
      out_hash[s0 + i] = s_key[i];
      out_cnt[s0 + i] = s_cn[i];
    }
  }
}

// persistent waves over the mid list (LANE_MAX < lines <= 64): a wave per container, bitonic sort
// of 64-bit keys across lanes (shuffles), run heads by ballot, counts by ballot distance
__global__ __launch_bounds__(TPB) void tmpl_hist_small(const uint64_t* __restrict__ hash,
                                                       const int32_t* __restrict__ doc_lines,
                                                       const int64_t* __restrict__ doc_line0, int64_t D,
                                                       const int32_t* __restrict__ ws,
                                                       uint64_t* __restrict__ out_hash, int32_t* __restrict__ out_cnt,
                                                       int32_t* __restrict__ n_tmpl) {
  const int lane = threadIdx.x & 63;
  const int32_t nmid = ws[0];
  for (int64_t wv = (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6); wv < nmid;
       wv += (int64_t)gridDim.x * (TPB / 64)) {
  const int64_t d = ws[4 + wv];
  const int n = doc_lines[d];
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
  if (lane >= __popcll(heads) && lane < n) {  // the slots past the templates
    out_hash[lo + lane] = 0ull;
    out_cnt[lo + lane] = 0;
  }
  if (lane == 0) n_tmpl[d] = __popcll(heads);
  }
}

// workgroup per container with 64 < lines <= 4096
__global__ __launch_bounds__(TPB) void tmpl_hist_big(const uint64_t* __restrict__ hash,
                                                     const int32_t* __restrict__ doc_lines,
                                                     const int64_t* __restrict__ doc_line0, int64_t D,
                                                     const int32_t* __restrict__ ws,
                                                     uint64_t* __restrict__ out_hash, int32_t* __restrict__ out_cnt,
                                                     int32_t* __restrict__ n_tmpl) {
  __shared__ uint64_t key[BIG];
  __shared__ int32_t pos[BIG];
  __shared__ int32_t wsum[TPB / 64];
  const int32_t n_big = ws[1];
  for (int64_t b = blockIdx.x; b < n_big; b += gridDim.x) {
  __syncthreads();  // key / pos / wsum of the previous container
  const int64_t d = ws[4 + D + b];
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
  for (int r = carry + threadIdx.x; r < n; r += TPB) {  // the slots past the templates
    out_hash[lo + r] = 0ull;
    out_cnt[lo + r] = 0;
  }
  if (threadIdx.x == 0) n_tmpl[d] = carry;
  }
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
  const hipStream_t st = krca::as_stream(stream);
  hipLaunchKernelGGL(tmpl_hash_kernel<512>, dim3((unsigned)krca::ceil_div(n_lines, 512)), dim3(512), 0, st, text,
                     nbytes, line_start, line_end, n_lines, hash);
  KRCA_LAUNCH_CHECK();
  return KRCA_OK;
}

int64_t krca_template_hist_ws_size(int64_t ndocs) { return 16 + 12 * std::max<int64_t>(ndocs, 1); }

int krca_template_hist(const uint64_t* hash, const int32_t* doc_lines, const int64_t* doc_line0, int64_t ndocs,
                       void* workspace, uint64_t* out_hash, int32_t* out_count, int32_t* n_templates, void* stream) {
  KRCA_CHECK_ARG(ndocs >= 0 && ndocs < INT32_MAX, "krca_template_hist: bad sizes");
  if (ndocs == 0) return KRCA_OK;
  KRCA_CHECK_ARG(doc_lines && doc_line0 && n_templates && out_hash && out_count && workspace,
                 "krca_template_hist: null pointer");
  hipStream_t st = krca::as_stream(stream);
  int32_t* ws = static_cast<int32_t*>(workspace);
  KRCA_HIP(hipMemsetAsync(ws, 0, 16, st));
  hipLaunchKernelGGL(tmpl_hist_lane, dim3((unsigned)krca::ceil_div(ndocs, TPB)), dim3(TPB), 0, st, hash, doc_lines,
                     doc_line0, ndocs, out_hash, out_count, n_templates, ws);
  KRCA_LAUNCH_CHECK();
  hipLaunchKernelGGL(tmpl_hist_small, dim3(1024), dim3(TPB), 0, st, hash, doc_lines, doc_line0, ndocs,
                     (const int32_t*)ws, out_hash, out_count, n_templates);
  KRCA_LAUNCH_CHECK();
  hipLaunchKernelGGL(tmpl_hist_big, dim3(512), dim3(TPB), 0, st, hash, doc_lines, doc_line0, ndocs,
                     (const int32_t*)ws, out_hash, out_count, n_templates);
  KRCA_LAUNCH_CHECK();
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
  // the container's slots zeroed first; the distinct templates then fill the front (every slot of
  // the line range is written, as by krca_template_hist)
  KRCA_HIP(hipMemsetAsync(out_hash, 0, (size_t)n_lines * sizeof(uint64_t), st));
  KRCA_HIP(hipMemsetAsync(out_count, 0, (size_t)n_lines * sizeof(int32_t), st));
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

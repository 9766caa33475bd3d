// PageRank block / exchange layout shared by the device kernels (ppr.hip) and the host-side
// packing (ppr_pack.cpp, a plain C++ translation unit so it can be built with the host sanitizer).
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define KRCA_HD __host__ __device__ __forceinline__
#else
#define KRCA_HD inline
#endif

namespace pprl {

constexpr int TPB = 256;
constexpr int EDGE_BUDGET = 2048;       // edges per short block == LDS slots
constexpr int ROW_BUDGET = TPB;         // rows per short block (one updating lane per row)
constexpr int SEG = EDGE_BUDGET / TPB;  // edges per lane: gathered lane-strided, summed contiguous
constexpr int NSPREAD = 32;             // partial-sum slots per quantity (spreads the atomics)
constexpr int SET_WORDS = 3 * NSPREAD;  // one slot set: residual[32] | dangling[32] | seed total[32]
constexpr int NSET = 3;                 // folded iterations rotate over 3 sets (read, write, zero)
constexpr int NSLOT = NSET * SET_WORDS; // send tail
constexpr int CTL_BYTES = 256;  // ctl buffer header (the device Ctl block)

// 32-bit weight code: w < 2^26 as is; above, the top 26 bits (bit 25 set) and the shift in the top
// 6 bits (w < 2^61, so the shift is <= 35).  Decoding is one mask and one 64-bit shift.
KRCA_HD uint32_t wenc(int64_t w) {
  if (w < ((int64_t)1 << 26)) return (uint32_t)w;
  const int sh = 63 - __builtin_clzll((unsigned long long)w) - 25;
  return ((uint32_t)sh << 26) | (uint32_t)(w >> sh);
}
KRCA_HD int64_t wdec(uint32_t c) { return (int64_t)(c & 0x3FFFFFFu) << (c >> 26); }

// one rank's exchange slice in int64 words: the n_max codes (uint32, padded to 8 bytes), then the
// NSLOT partial-sum slots at int64 offset wslots(n_max)
KRCA_HD int64_t wslots(int64_t n_max) { return (n_max + 1) / 2; }
KRCA_HD int64_t slice_words(int64_t n_max) { return wslots(n_max) + NSLOT; }
// uint32 index of node j's code in w_all
KRCA_HD int64_t remap_col(int64_t j, int64_t n_max) {
  return j + (j / n_max) * (2 * slice_words(n_max) - n_max);
}

// host: CSR-adaptive row blocks (ppr_pack.cpp)
int64_t build_plan(const int64_t* rp, int64_t N, int64_t* out);
int64_t pack_blocks(const int64_t* rp, const int32_t* col, int64_t N, int64_t n_max, int64_t* plan, int64_t plan_len,
                    int32_t* pk, uint16_t* lane);

}  // namespace pprl

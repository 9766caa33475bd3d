// Host-side PageRank block planning and column packing (include/krca.h krca_ppr_plan /
// krca_ppr_pack): plain C++ (no device code), so the same source also builds into the
// host-sanitizer library (Makefile `asan`, tests/test_host_asan_cpu.py).
#include <stdarg.h>

#include <algorithm>
#include <vector>

#include "../../include/krca.h"
#include "ppr_layout.h"

namespace krca {
void set_error(const char* fmt, ...);
struct Tuning;
const Tuning& tuning();
int tuning_ppr_dict();
}  // namespace krca

#define KRCA_CHECK_ARG(cond, ...)     \
  do {                                \
    if (!(cond)) {                    \
      ::krca::set_error(__VA_ARGS__); \
      return KRCA_EINVAL;             \
    }                                 \
  } while (0)

namespace pprl {
namespace {
inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
}  // namespace

// host: CSR-adaptive row blocks {rb, code, e0, e1} (code > 0: short rows [rb, code); code <= 0:
// chunk -code of long row rb); returns the number of int64 entries (4 per block)
int64_t build_plan(const int64_t* rp, int64_t N, int64_t* out) {
  int64_t n = 0;
  int64_t r = 0;
  auto put = [&](int64_t rb, int64_t code, int64_t e0, int64_t e1) {
    if (out) {
      out[n] = rb;
      out[n + 1] = code;
      out[n + 2] = e0;
      out[n + 3] = e1;
    }
    n += 4;
  };
  while (r < N) {
    const int64_t deg = rp[r + 1] - rp[r];
    if (deg > EDGE_BUDGET) {
      const int64_t chunks = ceil_div(deg, EDGE_BUDGET);
      for (int64_t c = 0; c < chunks; ++c) {
        const int64_t e0 = rp[r] + c * EDGE_BUDGET;
        put(r, -c, e0, std::min<int64_t>(rp[r + 1], e0 + EDGE_BUDGET));  // chunk 0 encodes as 0
      }
      r += 1;
      continue;
    }
    int64_t re = r + 1;
    while (re < N && re - r < ROW_BUDGET && rp[re + 1] - rp[r] <= EDGE_BUDGET) ++re;
    put(r, re, rp[r], rp[re]);
    r = re;
  }
  return n;
}

// host: the plan of build_plan plus the packed column array pk[E] (include/krca.h krca_ppr_pack):
// columns remapped to the [G][slice] exchange layout (uint32 units); a short-row block whose distinct
// columns fit becomes a dictionary block (sorted distinct columns, then uint16 slots per edge),
// every other block stays direct.  Returns the number of dictionary blocks.
int64_t pack_blocks(const int64_t* rp, const int32_t* col, int64_t N, int64_t n_max, int64_t* plan, int64_t plan_len,
                    int32_t* pk, uint16_t* lane) {
  auto remap = [n_max](int64_t j) { return (int32_t)remap_col(j, n_max); };
  std::vector<int32_t> uniq;
  std::vector<uint16_t> slot;
  int64_t ndict = 0;
  for (int64_t p = 0; p < plan_len; p += 4) {
    const int64_t rb = plan[p], code = plan[p + 1], e0 = plan[p + 2], e1 = plan[p + 3];
    const int64_t ne = e1 - e0;
    uint16_t* li = lane + (p / 4) * 2 * TPB;  // [TPB] lane words, then [TPB] row slots
    uint16_t* rs = li + TPB;
    for (int t = 0; t < TPB; ++t) {
      li[t] = 0;
      rs[t] = (uint16_t)ROW_BUDGET;  // no edges: the block's always-zero sum slot
    }
    if (code > 0) {
      // the block's non-empty rows get consecutive sum slots, so a lane's next segment is the next
      // slot: lane t = (slot of the row holding edge 8t) << 8 | bits of its edges that start a row
      int slot = -1;
      for (int64_t rr = rb; rr < code; ++rr) {
        if (rp[rr + 1] == rp[rr]) continue;
        rs[rr - rb] = (uint16_t)++slot;
        const int64_t f = rp[rr] - e0;  // the row's first edge
        if (f % SEG) li[f / SEG] |= (uint16_t)(1u << (f % SEG));
        for (int64_t e = (f + SEG - 1) / SEG * SEG; e < rp[rr + 1] - e0; e += SEG)  // lanes starting inside the row
          li[e / SEG] = (uint16_t)((li[e / SEG] & 0xFFu) | (slot << 8));
        if (f % SEG == 0) li[f / SEG] = (uint16_t)((li[f / SEG] & 0xFFu) | (slot << 8));
      }
    }
    bool dict = false;
    if (code > 0 && ne >= 32 && ::krca::tuning_ppr_dict()) {
      uniq.assign(col + e0, col + e1);
      std::sort(uniq.begin(), uniq.end());
      uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
      const int64_t nu = (int64_t)uniq.size();
      const int64_t dw = ((e0 + nu + 3) & ~int64_t(3)) - e0;  // slot words start 16-byte aligned
      dict = dw + 4 * ceil_div(ne, SEG) <= ne;          // the lanes' 16-byte slot loads stay inside
      if (dict) {
        for (int64_t u = 0; u < nu; ++u) pk[e0 + u] = remap(uniq[u]);
        for (int64_t u = nu; u < dw; ++u) pk[e0 + u] = 0;
        slot.assign(ceil_div(ne, SEG) * SEG, 0);
        for (int64_t e = 0; e < ne; ++e)
          slot[e] = (uint16_t)(std::lower_bound(uniq.begin(), uniq.end(), col[e0 + e]) - uniq.begin());
        uint32_t* words = reinterpret_cast<uint32_t*>(pk + e0 + dw);
        for (int64_t i = 0; i < (int64_t)slot.size() / 2; ++i)
          words[i] = (uint32_t)slot[2 * i] | ((uint32_t)slot[2 * i + 1] << 16);
        for (int64_t e = dw + (int64_t)slot.size() / 2; e < ne; ++e) pk[e0 + e] = 0;
        plan[p] = rb | (nu << 32);
        ++ndict;
      }
    }
    if (!dict)
      for (int64_t e = e0; e < e1; ++e) pk[e] = remap(col[e]);
  }
  return ndict;
}

}  // namespace pprl

using namespace pprl;

extern "C" {

int32_t krca_ppr_nslot(void) { return NSLOT; }
int64_t krca_ppr_slice_words(int64_t n_max) { return n_max > 0 ? slice_words(n_max) : 0; }

int64_t krca_ppr_plan_size(const int64_t* row_ptr_host, int64_t N) {
  if (!row_ptr_host || N <= 0) return 0;
  return build_plan(row_ptr_host, N, nullptr);
}

int krca_ppr_plan(const int64_t* row_ptr_host, int64_t N, int64_t* plan_host, int64_t plan_len) {
  KRCA_CHECK_ARG(row_ptr_host && plan_host && N > 0 && N < INT32_MAX, "krca_ppr_plan: bad arguments");
  for (int64_t i = 0; i < N; ++i)
    KRCA_CHECK_ARG(row_ptr_host[i + 1] >= row_ptr_host[i], "krca_ppr_plan: row_ptr not monotone at %lld", (long long)i);
  const int64_t need = build_plan(row_ptr_host, N, nullptr);
  KRCA_CHECK_ARG(plan_len == need, "krca_ppr_plan: plan_len %lld != %lld", (long long)plan_len, (long long)need);
  build_plan(row_ptr_host, N, plan_host);
  return KRCA_OK;
}

int64_t krca_ppr_lane_size(int64_t plan_len) { return plan_len / 4 * 2 * TPB; }

int64_t krca_ppr_pack(const int64_t* row_ptr_host, const int32_t* col_host, int64_t N, int64_t n_max,
                      int64_t* plan_host, int64_t plan_len, int32_t* pk_host, uint16_t* lane_host) {
  KRCA_CHECK_ARG(row_ptr_host && plan_host && pk_host && lane_host && N > 0 && N < INT32_MAX && n_max > 0,
                 "krca_ppr_pack: bad arguments");
  const int64_t E = row_ptr_host[N];
  KRCA_CHECK_ARG(E == 0 || col_host, "krca_ppr_pack: null col");
  int rc = krca_ppr_plan(row_ptr_host, N, plan_host, plan_len);
  if (rc) return rc;
  for (int64_t e = 0; e < E; ++e) {
    KRCA_CHECK_ARG(col_host[e] >= 0, "krca_ppr_pack: negative column at edge %lld", (long long)e);
    // the step gathers at 32-bit byte offsets of the exchange table
    KRCA_CHECK_ARG(remap_col(col_host[e], n_max) < (int64_t(1) << 30), "krca_ppr_pack: column %lld past the 2^30-word table",
                   (long long)col_host[e]);
  }
  return pack_blocks(row_ptr_host, col_host, N, n_max, plan_host, plan_len, pk_host, lane_host);
}

}  // extern "C"

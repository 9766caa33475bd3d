// Host walk of csrc/tmpl_dfa.h's table (tests/test_template_dfa_cpu.py): the device kernel's per-byte
// step (table read, flag ranges, FNV-1a) on the CPU, so the table is checked against
// oracle.template_of without a GPU.  Built by the test with hipcc (host code only).
#include <hip/hip_runtime.h>

#include "tmpl_dfa.h"

namespace {
constexpr tdfa::Table kT = tdfa::make_table();
constexpr tdfa::ClsTable kC = tdfa::make_cls_table();
constexpr uint64_t kOff = 0xcbf29ce484222325ull, kPrime = 0x100000001b3ull;
inline uint64_t fnv(uint64_t h, uint32_t b) { return (h ^ b) * kPrime; }
}  // namespace

extern "C" {
int tdfa_rows(void) { return tdfa::kRows; }
uint64_t tdfa_line_hash(const uint8_t* s, int64_t n) {
  uint64_t h = kOff, hb = 0, hu = 0;
  uint32_t st = 0;
  auto mask = [](uint64_t x) { return fnv(x, 0xFFu); };
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t t = kT.v[st * 256 + s[i]];
    tdfa::apply_flags(t, h, hb, hu, mask);
    h = fnv(h, s[i]);
    st = t;
  }
  tdfa::apply_flags(kT.v[st * 256 + tdfa::kEndByte], h, hb, hu, mask);
  return h;
}

// the same walk over the byte-class table (template.hip's KRCA_TMPL_CLS build)
uint64_t tdfa_line_hash_cls(const uint8_t* s, int64_t n) {
  uint64_t h = kOff, hb = 0, hu = 0;
  uint32_t st = 0;
  auto mask = [](uint64_t x) { return fnv(x, 0xFFu); };
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t t = kC.v[(st << 3) | kC.cls[s[i]]];
    tdfa::apply_flags(t, h, hb, hu, mask);
    h = fnv(h, s[i]);
    st = t;
  }
  tdfa::apply_flags(kC.v[(st << 3) | tdfa::C_OTHER], h, hb, hu, mask);
  return h;
}
}

// The word machine of the error-template hash, as a byte-indexed table
// built at compile time.  Shared by csrc/template.hip (device walk) and the host test library of
// tests/test_template_dfa_cpu.py (the same table walked on the CPU against oracle.template_of).
//
// Template semantics (restated in oracle/oracle.py template_of):
//   word    = a maximal run of [A-Za-z0-9_];
//   masked  = a word holding an ASCII digit, or of >= 8 characters all in [0-9a-fA-F];
//   UUID    = five words of exactly 8, 4, 4, 4 and 12 hex characters joined by single '-'
//             (regex (?<![A-Za-z0-9_])[0-9a-fA-F]{8}(-[0-9a-fA-F]{4}){3}-[0-9a-fA-F]{12}(?![A-Za-z0-9_]),
//             leftmost matches first);
//   a UUID becomes ONE mask byte, every other masked word one mask byte, the rest stays.
//
// The machine tracks, inside a word that has held only hex characters, its length, whether it
// held a digit and which UUID group it could be (g = 0 .. 4: every such word may also start a new
// UUID as group 0, so a candidate that fails on an 8-character word restarts there — UUID groups
// after the first are 4 or 12 long, so two candidates never overlap otherwise).  Outside a word:
// plain, or "after group g and its '-'" (D1..D3; D0 only entered with its flags).
//
// Flags are encoded in the DESTINATION row (rows are duplicated per flag), so the walk decodes them
// with range compares on the next row index:
//   rows [kS0, kM0)  START  the byte starts a word: hb = h (the hash before the word)
//   rows [kM0, kU0)  MEND   the byte ends a masked word: h = mask(hb)
//   row  kU0         USAVE + MEND: a UUID's first group ended ("-" follows): hu = hb, h = mask(hb)
//   row  kUE         UEND   a UUID ended: h = mask(hu) (the whole UUID becomes one mask byte)
// where mask(x) = FNV step of x with the mask byte 0xFF; then the byte itself is hashed.  At the
// end of a line the transition on a space (a non-word byte) is taken for its flags only.
#pragma once
#include <cstdint>

namespace tdfa {

enum Cls : int { C_DIG = 0, C_HEX = 1, C_WORD = 2, C_DASH = 3, C_OTHER = 4 };
__host__ __device__ constexpr int cls_of(uint32_t b) {
  if (b >= '0' && b <= '9') return C_DIG;
  if ((b >= 'a' && b <= 'f') || (b >= 'A' && b <= 'F')) return C_HEX;
  if ((b >= 'g' && b <= 'z') || (b >= 'G' && b <= 'Z') || b == '_') return C_WORD;
  if (b == '-') return C_DASH;
  return C_OTHER;
}

__host__ __device__ constexpr int lmax(int g) { return g == 4 ? 12 : 8; }  // lengths tracked per group

// row layout
constexpr int kO0 = 0;               // outside a word
constexpr int kD1 = 1;               // D1, D2, D3: rows 1..3 (after group g and its '-')
constexpr int kA2 = 4;               // A(g, len >= 2, d): all-hex word, groups 0..3 (len 2..8), 4 (len 2..12)
constexpr int kNA2 = 4 * 7 * 2 + 11 * 2;
constexpr int kH9 = kA2 + kNA2;      // all hex, no digit, >= 8 long, no UUID role (masked unless a letter g-z follows)
constexpr int kM = kH9 + 1;          // holds a digit: masked whatever follows
constexpr int kW = kM + 1;           // any other word (unmasked unless a digit follows)
constexpr int kS0 = kW + 1;          // START rows: A(g, 1, d) for g 0..4, d 0..1, then W_S
constexpr int kWS = kS0 + 10;
constexpr int kM0 = kWS + 1;         // MEND rows: O0_M, D1_M, D2_M, D3_M
constexpr int kU0 = kM0 + 4;         // D0 with USAVE + MEND
constexpr int kUE = kU0 + 1;         // O0 with UEND
constexpr int kRows = kUE + 1;
static_assert(kRows <= 255, "row index in one byte");

__host__ __device__ constexpr int row_a(int g, int len, int d) {
  if (len == 1) return kS0 + 2 * g + d;
  const int base = g < 4 ? kA2 + g * 14 : kA2 + 56;
  return base + 2 * (len - 2) + d;
}

struct Abs {
  int kind;  // 0 outside (g = the group just completed, -1 none), 1 all-hex word, 2 H9, 3 M, 4 W
  int g, len, d;
};
__host__ __device__ constexpr Abs decode(int r) {
  if (r == kO0 || r == kUE || r == kM0) return {0, -1, 0, 0};
  if (r >= kD1 && r <= kD1 + 2) return {0, r - kD1 + 1, 0, 0};
  if (r >= kM0 + 1 && r <= kM0 + 3) return {0, r - kM0, 0, 0};
  if (r == kU0) return {0, 0, 0, 0};
  if (r == kH9) return {2, 0, 0, 0};
  if (r == kM) return {3, 0, 0, 0};
  if (r == kW || r == kWS) return {4, 0, 0, 0};
  if (r >= kS0 && r < kWS) return {1, (r - kS0) / 2, 1, (r - kS0) % 2};
  const int q = r - kA2;  // A(g, len >= 2, d)
  if (q < 56) return {1, q / 14, 2 + (q % 14) / 2, q % 2};
  return {1, 4, 2 + (q - 56) / 2, (q - 56) % 2};
}

__host__ __device__ constexpr int next_row(int r, uint32_t b) {
  const Abs a = decode(r);
  const int c = cls_of(b);
  const bool word = c <= C_WORD;
  if (a.kind == 0) {  // outside: a word starts (START rows), or stays outside
    if (!word) return kO0;
    const int gn = a.g < 0 ? 0 : a.g + 1;
    if (c == C_WORD) return kWS;
    return row_a(gn, 1, c == C_DIG ? 1 : 0);
  }
  if (a.kind == 1) {
    if (c == C_DIG || c == C_HEX) {
      const int d = c == C_DIG ? 1 : a.d;
      if (a.len + 1 <= lmax(a.g)) return row_a(a.g, a.len + 1, d);
      return d ? kM : kH9;
    }
    if (c == C_WORD) return a.d ? kM : kW;
    // the word ends here (c is '-' or a non-word byte)
    const bool masked = a.d || a.len >= 8;
    if (a.g == 4 && a.len == 12) return kUE;                    // a whole UUID
    if (a.len == 8) return c == C_DASH ? kU0 : kM0;              // group 0 (or a restart there); 8 hex: masked
    if (a.g >= 1 && a.g <= 3 && a.len == 4 && c == C_DASH)       // group g of a candidate
      return masked ? kM0 + a.g : kD1 + a.g - 1;
    return masked ? kM0 : kO0;
  }
  if (a.kind == 2) {  // H9
    if (c == C_DIG) return kM;
    if (c == C_HEX) return kH9;
    if (c == C_WORD) return kW;
    return kM0;
  }
  if (a.kind == 3) return word ? kM : kM0;  // M
  // W
  if (c == C_DIG) return kM;
  if (word) return kW;
  return kO0;
}

// rows of a word that ends masked at the end of a line are found through the space transition
constexpr uint32_t kEndByte = ' ';

struct Table {
  alignas(16) uint8_t v[kRows * 256];
};
__host__ __device__ constexpr Table make_table() {
  Table t{};
  for (int r = 0; r < kRows; ++r)
    for (uint32_t b = 0; b < 256; ++b) t.v[r * 256 + b] = (uint8_t)next_row(r, b);
  return t;
}
// The same machine over byte CLASSES (next_row depends on a byte only through cls_of): a 256-byte
// class map, then kRows x 8 entries (1.1 KB instead of 25.5 KB; the A/B build of template.hip)
struct ClsTable {
  alignas(16) uint8_t cls[256];
  uint8_t v[kRows * 8];
  uint8_t pad[(16 - (kRows * 8) % 16) % 16];
};
__host__ __device__ constexpr ClsTable make_cls_table() {
  ClsTable t{};
  constexpr uint32_t rep[5] = {'0', 'a', 'g', '-', ' '};  // one byte of each class
  for (uint32_t b = 0; b < 256; ++b) t.cls[b] = (uint8_t)cls_of(b);
  for (int r = 0; r < kRows; ++r)
    for (int c = 0; c < 8; ++c) t.v[r * 8 + c] = (uint8_t)next_row(r, rep[c < 5 ? c : 4]);
  return t;
}

// one byte of the walk (the kernel's form, written out in template.hip with its register tricks)
template <class Mask>
__host__ __device__ inline void apply_flags(uint32_t t, uint64_t& h, uint64_t& hb, uint64_t& hu, Mask&& mask) {
  if (t >= (uint32_t)kM0) {
    if (t >= (uint32_t)kU0) {
      if (t == (uint32_t)kU0) {
        hu = hb;
        h = mask(hb);
      } else {
        h = mask(hu);
      }
    } else {
      h = mask(hb);
    }
  }
  if (t >= (uint32_t)kS0) hb = h;
}

}  // namespace tdfa

// GF(2^8) arithmetic core shared by host C++ and gfx950 device code.
//
// Field: primitive polynomial 0x11D = x^8+x^4+x^3+x^2+1, generator 2 — bit-compatible with the
// reference (/root/reference/src/matrix.cu:49, src/cpu-rs.c:37, src/cpu-decode.c:34).
//
// Two table layouts are generated at compile time (no hard-coded literals):
//   * `exp[1021]` / `log[256]` with log(0) = 510 and a zero band exp[510..1020] = 0, so
//     mul(a,b) = exp[log a + log b] is branch-free. This is the layout the reference keeps in
//     __constant__/__shared__ memory (src/matrix.cu:34-39, src/cpu-rs-log-exp-3.c:51-52,89-96).
//   * per-coefficient "perm tables": a GF(2)-linear byte map L (multiplication by a constant c is
//     one) is split over the byte's bit-chunks [2:0], [5:3], [7:6]:
//         L(x) = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6]
//     T0/T1 are 8-entry byte tables (two dwords each) and T2 a 4-entry table (one dword), so each
//     lookup is ONE v_perm_b32 on gfx950 (byte-select from an 8-byte pool). This replaces the
//     reference's per-byte log/exp lookups (src/matrix.cu:105-110, :304-314).
#pragma once

#include <cstdint>
#include <cstddef>

#if defined(__HIPCC__)
#define GFRS_HD __host__ __device__
#else
#define GFRS_HD
#endif

namespace gfrs {

constexpr unsigned kPoly = 0x11D;  // 0435 octal
constexpr int kLogZero = 510;      // log(0) sentinel: exp[510 + x] == 0 for every x in [0, 510]
constexpr int kExpLen = 1021;      // two periods [0,510) + zero band [510,1021)

struct Tables {
  uint8_t exp[kExpLen];
  uint16_t log[256];
  uint8_t inv[256];
};

constexpr Tables make_tables() {
  Tables t{};
  unsigned x = 1;
  for (int i = 0; i < 255; ++i) {
    t.exp[i] = static_cast<uint8_t>(x);
    t.exp[i + 255] = static_cast<uint8_t>(x);
    t.log[x] = static_cast<uint16_t>(i);
    x <<= 1;
    if (x & 0x100) x ^= kPoly;
  }
  for (int i = 510; i < kExpLen; ++i) t.exp[i] = 0;
  t.log[0] = kLogZero;
  t.inv[0] = 0;
  for (int a = 1; a < 256; ++a) t.inv[a] = t.exp[255 - t.log[a]];
  return t;
}

inline constexpr Tables kTables = make_tables();

// ---- scalar host arithmetic (the device kernels keep their own LDS/perm copies) -------------
constexpr uint8_t mul(uint8_t a, uint8_t b) { return kTables.exp[kTables.log[a] + kTables.log[b]]; }
constexpr uint8_t inv(uint8_t a) { return kTables.inv[a]; }
constexpr uint8_t div(uint8_t a, uint8_t b) {
  // b == 0 is a caller bug; returns 0 like the reference's a==0 short-circuit (src/matrix.cu:152-170)
  return (a == 0 || b == 0) ? 0 : kTables.exp[kTables.log[a] + 255 - kTables.log[b]];
}
// Reference-compatible power: gf_pow(a, e) = exp[(log a * e) % 255] (src/matrix.cu:204-208),
// including its quirk pow(0, e) == 1 (log(0)=510, 510*e mod 255 == 0).
constexpr uint8_t pow_ref(uint8_t a, unsigned e) {
  return kTables.exp[(static_cast<unsigned>(kTables.log[a]) * e) % 255u];
}
// Mathematically correct power (0^0 = 1, 0^e = 0 for e > 0).
constexpr uint8_t pow(uint8_t a, unsigned e) {
  if (e == 0) return 1;
  if (a == 0) return 0;
  return kTables.exp[(static_cast<unsigned>(kTables.log[a]) * e) % 255u];
}
// Bitwise shift-and-xor multiply (the cpu-rs-loop.c strategy, with the accumulator initialised).
constexpr uint8_t mul_loop(uint8_t a, uint8_t b) {
  unsigned r = 0, x = a;
  for (int i = 0; i < 8; ++i) {
    if (b & (1u << i)) r ^= x;
    x <<= 1;
    if (x & 0x100) x ^= kPoly;
  }
  return static_cast<uint8_t>(r);
}

// ---- perm tables ------------------------------------------------------------------------------
// Packed layout of one GF(2)-linear byte map, 5 dwords (padded to kPermStride):
//   w[0] = T0[0..3], w[1] = T0[4..7], w[2] = T1[0..3], w[3] = T1[4..7], w[4] = T2[0..3]
constexpr int kPermWords = 5;
constexpr int kPermStride = 8;  // 32-byte aligned records -> s_load_dwordx8 friendly

struct PermTable {
  uint32_t w[kPermStride];
};

// Perm table for the map x -> L(x) given L's images of the 8 basis bits.
constexpr PermTable perm_from_basis(const uint8_t basis[8]) {
  PermTable t{};
  uint8_t t0[8]{}, t1[8]{}, t2[4]{};
  for (unsigned v = 0; v < 8; ++v) {
    uint8_t a = 0, b = 0;
    for (int bit = 0; bit < 3; ++bit) {
      if (v & (1u << bit)) {
        a ^= basis[bit];
        b ^= basis[bit + 3];
      }
    }
    t0[v] = a;
    t1[v] = b;
  }
  for (unsigned v = 0; v < 4; ++v) {
    uint8_t c = 0;
    for (int bit = 0; bit < 2; ++bit)
      if (v & (1u << bit)) c ^= basis[bit + 6];
    t2[v] = c;
  }
  auto pack = [](const uint8_t* b) -> uint32_t {
    return uint32_t(b[0]) | (uint32_t(b[1]) << 8) | (uint32_t(b[2]) << 16) | (uint32_t(b[3]) << 24);
  };
  t.w[0] = pack(t0);
  t.w[1] = pack(t0 + 4);
  t.w[2] = pack(t1);
  t.w[3] = pack(t1 + 4);
  t.w[4] = pack(t2);
  return t;
}

// Perm table of "multiply by c" in GF(2^8).
constexpr PermTable perm_for_coeff(uint8_t c) {
  uint8_t basis[8]{};
  for (int b = 0; b < 8; ++b) basis[b] = mul(c, static_cast<uint8_t>(1u << b));
  return perm_from_basis(basis);
}

// GF(16) (poly x^4 + x + 1 = 0x13, src/gf16.h / src/galoisfield.cu:22) multiply.
constexpr uint8_t gf16_mul(uint8_t a, uint8_t b) {
  unsigned r = 0, x = a & 15u;
  for (int i = 0; i < 4; ++i) {
    if (b & (1u << i)) r ^= x;
    x <<= 1;
    if (x & 0x10u) x ^= 0x13u;
  }
  return static_cast<uint8_t>(r & 15u);
}

// Perm table of the design doc's "GF(16) method" (doc/design.tex:190-209): each byte is two
// independent GF(16) symbols, both multiplied by c (c < 16) — a GF(2)-linear byte map like any other,
// so the GF(256) kernels run it unchanged.
constexpr PermTable perm_for_coeff_gf16(uint8_t c) {
  uint8_t basis[8]{};
  for (int b = 0; b < 4; ++b) {
    basis[b] = gf16_mul(c, static_cast<uint8_t>(1u << b));
    basis[b + 4] = static_cast<uint8_t>(gf16_mul(c, static_cast<uint8_t>(1u << b)) << 4);
  }
  return perm_from_basis(basis);
}

// Evaluate a perm table on the host (byte-exact emulation of the device v_perm path).
constexpr uint8_t perm_apply(const PermTable& t, uint8_t x) {
  const unsigned s0 = x & 7u, s1 = (x >> 3) & 7u, s2 = x >> 6;
  const uint8_t a = static_cast<uint8_t>((s0 < 4 ? t.w[0] >> (8 * s0) : t.w[1] >> (8 * (s0 - 4))) & 0xFF);
  const uint8_t b = static_cast<uint8_t>((s1 < 4 ? t.w[2] >> (8 * s1) : t.w[3] >> (8 * (s1 - 4))) & 0xFF);
  const uint8_t c = static_cast<uint8_t>((t.w[4] >> (8 * s2)) & 0xFF);
  return static_cast<uint8_t>(a ^ b ^ c);
}

}  // namespace gfrs

// GF(2^16) host arithmetic and linear algebra (the w = 16 member of the reference's field family).
//
// Field: primitive polynomial 0210013 octal = 0x1100B = x^16 + x^12 + x^3 + x + 1, generator 2 —
// the reference's `prim_poly_16` (/root/reference/src/galoisfield.cu:22-32; that file was never
// built, so no reference binary ever produced a w = 16 stripe: the on-disk layout is defined here,
// see gfrs/format.h). Symbols are little-endian uint16 pairs of bytes in a chunk.
//
// The device never multiplies in GF(2^16) directly. Multiplication by a constant c is GF(2)-linear
// on 16 bits, so it splits into four byte maps over the symbol's low byte l and high byte h:
//     c * (l | h << 8) = [L_ll(l) ^ L_hl(h)]  |  [L_lh(l) ^ L_hh(h)] << 8
// where L_ab is the map "source byte a -> destination byte b" of multiplying by c. Each of the four
// is an ordinary v_perm byte-map record (gfrs/gf256.h perm_from_basis), which is what the w = 16
// kernel (csrc/kernels/gf_gemm16.hip) applies to de-interleaved byte planes.
#pragma once

#include <algorithm>
#include <array>
#include <cstdint>
#include <stdexcept>
#include <vector>

#include "gfrs/gf256.h"

namespace gfrs {
namespace gf16w {

constexpr unsigned kPoly = 0x1100B;  // 0210013 octal
constexpr unsigned kOrder = 65536;
constexpr unsigned kMax = 65535;  // multiplicative group order

struct Tables {
  std::vector<uint16_t> exp;  // 2 * kMax entries (no modulo in mul)
  std::vector<uint32_t> log;  // log[0] unused
  Tables() : exp(2 * kMax), log(kOrder, 0) {
    unsigned x = 1;
    for (unsigned i = 0; i < kMax; ++i) {
      exp[i] = exp[i + kMax] = static_cast<uint16_t>(x);
      log[x] = i;
      x <<= 1;
      if (x & kOrder) x ^= kPoly;
    }
  }
};

inline const Tables& tables() {
  static const Tables t;
  return t;
}

inline uint16_t mul(uint16_t a, uint16_t b) {
  if (!a || !b) return 0;
  const Tables& t = tables();
  return t.exp[t.log[a] + t.log[b]];
}
inline uint16_t inv(uint16_t a) {
  if (!a) throw std::domain_error("gf2^16: inverse of 0");
  const Tables& t = tables();
  return t.exp[(kMax - t.log[a]) % kMax];
}
// Mathematically correct power (0^0 = 1).
inline uint16_t pow(uint16_t a, unsigned e) {
  if (e == 0) return 1;
  if (a == 0) return 0;
  const Tables& t = tables();
  return t.exp[(uint64_t(t.log[a]) * e) % kMax];
}

using Mat = std::vector<uint16_t>;  // row-major

// Reference Vandermonde block E[i][j] = (j+1)^i (the construction of src/matrix.cu:752-759 in this
// field; k < 65535 so (j+1) never wraps to 0).
inline Mat vandermonde_ref(int k, int p) {
  if (k < 1 || p < 0 || k + p > int(kMax)) throw std::invalid_argument("gf2^16 vandermonde: 1 <= k, k + p <= 65535");
  Mat e(size_t(p) * k);
  for (int i = 0; i < p; ++i)
    for (int j = 0; j < k; ++j) e[size_t(i) * k + j] = pow(static_cast<uint16_t>(j + 1), unsigned(i));
  return e;
}

// Cauchy block C[i][j] = 1 / (x_i + y_j), x_i = k + i, y_j = j (MDS, k + p <= 65536).
inline Mat cauchy(int k, int p) {
  if (k + p > int(kOrder)) throw std::invalid_argument("gf2^16 cauchy: k + p must be <= 65536");
  Mat e(size_t(p) * k);
  for (int i = 0; i < p; ++i)
    for (int j = 0; j < k; ++j) e[size_t(i) * k + j] = inv(static_cast<uint16_t>((k + i) ^ j));
  return e;
}

inline Mat identity(int n) {
  Mat m(size_t(n) * n, 0);
  for (int i = 0; i < n; ++i) m[size_t(i) * n + i] = 1;
  return m;
}

inline Mat matmul(const Mat& a, const Mat& b, int n, int m, int p) {  // (n x m) . (m x p)
  Mat c(size_t(n) * p, 0);
  for (int i = 0; i < n; ++i)
    for (int t = 0; t < m; ++t) {
      const uint16_t av = a[size_t(i) * m + t];
      if (!av) continue;
      for (int j = 0; j < p; ++j) c[size_t(i) * p + j] ^= mul(av, b[size_t(t) * p + j]);
    }
  return c;
}

// Gauss-Jordan with row pivoting (as gfrs::invert). Returns false when `a` is singular. Rows are
// scaled and eliminated through log-domain row multipliers: one log lookup per element instead
// of two per product.
inline bool invert(const Mat& a, int n, Mat& out) {
  const Tables& t = tables();
  Mat w = a;
  out = identity(n);
  auto axpy = [&](uint16_t* dst, const uint16_t* src, uint16_t f) {  // dst ^= f * src
    const uint32_t lf = t.log[f];
    for (int j = 0; j < n; ++j)
      if (src[j]) dst[j] ^= t.exp[lf + t.log[src[j]]];
  };
  for (int c = 0; c < n; ++c) {
    int piv = -1;
    for (int r = c; r < n; ++r)
      if (w[size_t(r) * n + c]) { piv = r; break; }
    if (piv < 0) return false;
    if (piv != c)
      for (int j = 0; j < n; ++j) {
        std::swap(w[size_t(piv) * n + j], w[size_t(c) * n + j]);
        std::swap(out[size_t(piv) * n + j], out[size_t(c) * n + j]);
      }
    const uint16_t ip = inv(w[size_t(c) * n + c]);
    for (int j = 0; j < n; ++j) {
      w[size_t(c) * n + j] = mul(w[size_t(c) * n + j], ip);
      out[size_t(c) * n + j] = mul(out[size_t(c) * n + j], ip);
    }
    for (int r = 0; r < n; ++r) {
      if (r == c) continue;
      const uint16_t f = w[size_t(r) * n + c];
      if (!f) continue;
      axpy(&w[size_t(r) * n], &w[size_t(c) * n], f);
      axpy(&out[size_t(r) * n], &out[size_t(c) * n], f);
    }
  }
  return true;
}

inline Mat generator(const Mat& e, int k, int p) {
  Mat g = identity(k);
  g.insert(g.end(), e.begin(), e.begin() + size_t(p) * k);
  return g;
}

inline bool decode_matrix(const Mat& g, int k, const std::vector<int>& rows, Mat& out) {
  if (int(rows.size()) != k) throw std::invalid_argument("gf2^16 decode_matrix: need exactly k rows");
  Mat a(size_t(k) * k);
  for (int i = 0; i < k; ++i)
    for (int j = 0; j < k; ++j) a[size_t(i) * k + j] = g[size_t(rows[i]) * k + j];
  return invert(a, k, out);
}

// Rows `want` of inv(G[rows]) (e.g. the erased natives), as want.size() x k coefficients over the
// survivors in `rows` order. For a systematic G (top k rows = identity) only the e x e block
// M = E[parity survivors][erased natives] is inverted: an erased native is
//   x_t = sum_p invM[t][p] * (y_p + sum_{surviving native s} E[p][s] * x_s)     (characteristic 2)
// O(e^2 k) instead of the full k x k inverse (k = 300, e = 40: ~0.5 M products against 27 M).
// Any other G, or a wanted row that survived, falls back to / is answered from the full inverse.
// Returns false when G[rows] is singular.
inline bool decode_rows(const Mat& g, int k, const std::vector<int>& rows, const std::vector<int>& want, Mat& out) {
  if (int(rows.size()) != k) throw std::invalid_argument("gf2^16 decode_rows: need exactly k rows");
  if (k <= 0 || g.size() % size_t(k)) throw std::invalid_argument("gf2^16 decode_rows: G is not n x k");
  const int n = int(g.size() / size_t(k));
  for (int r : rows)
    if (r < 0 || r >= n) throw std::invalid_argument("gf2^16 decode_rows: bad chunk id");
  for (int i : want)  // checked before either path (the full-inverse fallback indexes with it)
    if (i < 0 || i >= k) throw std::invalid_argument("gf2^16 decode_rows: wanted row is not a native");
  bool systematic = true;
  for (int i = 0; i < k && systematic; ++i)
    for (int j = 0; j < k; ++j)
      if (g[size_t(i) * k + j] != (i == j ? 1 : 0)) {
        systematic = false;
        break;
      }
  std::vector<int> pos(size_t(k), -1);  // native -> position in rows (-1: erased)
  std::vector<int> par;                 // positions of parity survivors
  for (int j = 0; j < k; ++j) {
    if (rows[size_t(j)] < 0) throw std::invalid_argument("gf2^16 decode_rows: bad chunk id");
    if (rows[size_t(j)] < k)
      pos[size_t(rows[size_t(j)])] = j;
    else
      par.push_back(j);
  }
  std::vector<int> erased;
  for (int i = 0; i < k; ++i)
    if (pos[size_t(i)] < 0) erased.push_back(i);
  const int e = int(erased.size());
  if (!systematic || e != int(par.size())) {
    Mat full;
    if (!decode_matrix(g, k, rows, full)) return false;
    out.assign(want.size() * size_t(k), 0);
    for (size_t w = 0; w < want.size(); ++w)
      std::copy(full.begin() + size_t(want[w]) * k, full.begin() + size_t(want[w] + 1) * k, out.begin() + w * k);
    return true;
  }
  Mat m(size_t(e) * e), im;
  for (int p = 0; p < e; ++p)
    for (int t = 0; t < e; ++t) m[size_t(p) * e + t] = g[size_t(rows[size_t(par[size_t(p)])]) * k + erased[size_t(t)]];
  if (e > 0 && !invert(m, e, im)) return false;
  std::vector<int> slot(size_t(k), -1);  // erased native -> index t
  for (int t = 0; t < e; ++t) slot[size_t(erased[size_t(t)])] = t;
  out.assign(want.size() * size_t(k), 0);
  for (size_t w = 0; w < want.size(); ++w) {
    uint16_t* o = &out[w * k];
    const int i = want[w];
    if (i < 0 || i >= k) throw std::invalid_argument("gf2^16 decode_rows: wanted row is not a native");
    if (pos[size_t(i)] >= 0) {  // survived: itself
      o[pos[size_t(i)]] = 1;
      continue;
    }
    const int t = slot[size_t(i)];
    for (int p = 0; p < e; ++p) {
      const uint16_t c = im[size_t(t) * e + p];
      if (!c) continue;
      const int pr = rows[size_t(par[size_t(p)])];
      o[par[size_t(p)]] ^= c;
      for (int s = 0; s < k; ++s)
        if (pos[size_t(s)] >= 0) o[pos[size_t(s)]] ^= mul(c, g[size_t(pr) * k + s]);
    }
  }
  return true;
}

// The four byte-map records of "multiply by c", order q = 2 * src + dst (src/dst: 0 = low byte,
// 1 = high byte): {L_ll, L_lh, L_hl, L_hh}.
inline std::array<PermTable, 4> perm_quad(uint16_t c) {
  std::array<PermTable, 4> q{};
  for (int src = 0; src < 2; ++src) {
    uint8_t lo[8]{}, hi[8]{};
    for (int b = 0; b < 8; ++b) {
      const uint16_t img = mul(c, static_cast<uint16_t>(1u << (b + 8 * src)));
      lo[b] = static_cast<uint8_t>(img & 0xFF);
      hi[b] = static_cast<uint8_t>(img >> 8);
    }
    q[2 * src + 0] = perm_from_basis(lo);
    q[2 * src + 1] = perm_from_basis(hi);
  }
  return q;
}

// Host emulation of the device path for one symbol (tests): out = XOR of the four maps.
inline uint16_t quad_apply(const std::array<PermTable, 4>& q, uint16_t x) {
  const uint8_t l = static_cast<uint8_t>(x & 0xFF), h = static_cast<uint8_t>(x >> 8);
  const uint8_t ol = perm_apply(q[0], l) ^ perm_apply(q[2], h);
  const uint8_t oh = perm_apply(q[1], l) ^ perm_apply(q[3], h);
  return static_cast<uint16_t>(ol | (oh << 8));
}

}  // namespace gf16w
}  // namespace gfrs

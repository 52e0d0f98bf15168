// Host-side GF(2^8) linear algebra: coding-matrix construction, Gauss-Jordan inversion,
// perm-table packing. Header-only so the CPU codec, the HIP runtime and the CLIs share it.
//
// Parity with the reference:
//   * vandermonde_ref(): E[i][j] = (j+1)^i with the reference's pow quirk
//     (src/matrix.cu:752-759, src/cpu-rs.c:446-457). G = [I_k; E] (src/cpu-rs.c:459-463).
//   * invert(): Gauss-Jordan on [A|I] like src/cpu-decode.c:251-298, but with ROW pivoting (the
//     reference's column swap of the result is a no-op, src/cpu-decode.c:133-135, which permutes
//     decoded chunks — SURVEY §3.2) and explicit singularity detection (the reference indexes
//     column -1, src/cpu-decode.c:237-247,274-278).
//   * cauchy() / sys_vandermonde(): opt-in MDS generators (the reference's [I;V] is not MDS,
//     SURVEY §2.2).
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "gfrs/gf256.h"

namespace gfrs {

using Mat = std::vector<uint8_t>;  // row-major

enum class MatrixKind : int { kVandermondeRef = 0, kCauchy = 1, kSysVandermonde = 2 };

inline MatrixKind parse_matrix_kind(const std::string& s) {
  if (s == "vandermonde" || s == "vand" || s == "ref") return MatrixKind::kVandermondeRef;
  if (s == "cauchy") return MatrixKind::kCauchy;
  if (s == "sys_vandermonde" || s == "sysvand") return MatrixKind::kSysVandermonde;
  throw std::invalid_argument("unknown matrix kind: " + s);
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
      const uint8_t av = a[size_t(i) * m + t];
      if (!av) continue;
      for (int j = 0; j < p; ++j) c[size_t(i) * p + j] ^= mul(av, b[size_t(t) * p + j]);
    }
  return c;
}

// Returns false (and leaves `out` unspecified) when `a` is singular.
inline bool invert(const Mat& a, int n, Mat& out) {
  Mat w = a;
  out = identity(n);
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
    const uint8_t ip = inv(w[size_t(c) * n + c]);
    for (int j = 0; j < n; ++j) {
      w[size_t(c) * n + j] = mul(w[size_t(c) * n + j], ip);
      out[size_t(c) * n + j] = mul(out[size_t(c) * n + j], ip);
    }
    for (int r = 0; r < n; ++r) {
      if (r == c) continue;
      const uint8_t f = w[size_t(r) * n + c];
      if (!f) continue;
      for (int j = 0; j < n; ++j) {
        w[size_t(r) * n + j] ^= mul(f, w[size_t(c) * n + j]);
        out[size_t(r) * n + j] ^= mul(f, out[size_t(c) * n + j]);
      }
    }
  }
  return true;
}

// p x k reference Vandermonde block E[i][j] = (j+1)^i.
inline Mat vandermonde_ref(int k, int p) {
  Mat e(size_t(p) * k);
  for (int i = 0; i < p; ++i)
    for (int j = 0; j < k; ++j) e[size_t(i) * k + j] = pow_ref(static_cast<uint8_t>((j + 1) % 256), i);
  return e;
}

// p x k Cauchy block C[i][j] = 1 / (x_i + y_j), x_i = k + i, y_j = j (all distinct, k + p <= 256).
inline Mat cauchy(int k, int p) {
  if (k + p > 256) throw std::invalid_argument("cauchy: k + p must be <= 256");
  Mat e(size_t(p) * k);
  for (int i = 0; i < p; ++i)
    for (int j = 0; j < k; ++j) e[size_t(i) * k + j] = inv(static_cast<uint8_t>((k + i) ^ j));
  return e;
}

// Systematic Vandermonde: V (n x k, V[r][j] = r^j over distinct points r = 0..n-1) times
// inv(V_top) gives [I; E] with every k x k submatrix invertible (MDS).
inline Mat sys_vandermonde(int k, int p) {
  const int n = k + p;
  if (n > 256) throw std::invalid_argument("sys_vandermonde: n must be <= 256");
  Mat v(size_t(n) * k);
  for (int r = 0; r < n; ++r)
    for (int j = 0; j < k; ++j) v[size_t(r) * k + j] = pow(static_cast<uint8_t>(r), j);
  Mat top(v.begin(), v.begin() + size_t(k) * k), top_inv;
  if (!invert(top, k, top_inv)) throw std::runtime_error("sys_vandermonde: singular top block");
  Mat bottom(v.begin() + size_t(k) * k, v.end());
  return matmul(bottom, top_inv, p, k, k);
}

inline Mat encoding_matrix(MatrixKind kind, int k, int p) {
  switch (kind) {
    case MatrixKind::kVandermondeRef: return vandermonde_ref(k, p);
    case MatrixKind::kCauchy: return cauchy(k, p);
    case MatrixKind::kSysVandermonde: return sys_vandermonde(k, p);
  }
  throw std::invalid_argument("bad matrix kind");
}

// Generator G = [I_k ; E]  ((k+p) x k).
inline Mat generator(const Mat& e, int k, int p) {
  Mat g = identity(k);
  g.insert(g.end(), e.begin(), e.begin() + size_t(p) * k);
  return g;
}

// Decode matrix for surviving rows `rows` (k indices into G): inv(G[rows]). Returns false when
// the sub-matrix is singular (the erasure pattern is unrecoverable with this generator).
inline bool decode_matrix(const Mat& g, int k, const std::vector<int>& rows, Mat& out) {
  if (int(rows.size()) != k) throw std::invalid_argument("decode_matrix: need exactly k rows");
  Mat a(size_t(k) * k);
  for (int i = 0; i < k; ++i)
    for (int j = 0; j < k; ++j) a[size_t(i) * k + j] = g[size_t(rows[i]) * k + j];
  return invert(a, k, out);
}

// Perm tables for an m x k coefficient matrix, laid out [k][m] (row j of the input stream
// first) so a kernel walking the k inputs reads one contiguous m-record slab per input row.
// field_w = 8: GF(2^8) multiply by each coefficient; 4: the GF(16) nibble method (coefficients < 16).
inline std::vector<PermTable> perm_tables_kmajor(const Mat& coeff, int m, int k, int field_w = 8) {
  std::vector<PermTable> t(size_t(k) * m);
  for (int j = 0; j < k; ++j)
    for (int i = 0; i < m; ++i) {
      const uint8_t c = coeff[size_t(i) * k + j];
      t[size_t(j) * m + i] = field_w == 4 ? perm_for_coeff_gf16(c) : perm_for_coeff(c);
    }
  return t;
}

}  // namespace gfrs

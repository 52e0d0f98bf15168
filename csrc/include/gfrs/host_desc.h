// Host-side construction of GF-GEMM descriptors (layout in gfrs/desc.h).
#pragma once

#include <cstring>
#include <stdexcept>
#include <vector>

#include "gfrs/desc.h"
#include "gfrs/gf65536.h"
#include "gfrs/matrix.h"

namespace gfrs {

// Coefficients of a GF(2^16) matrix carried in a byte Mat: little-endian pairs, 2 * m * k bytes
// (so GF(2^16) jobs travel through the same GemmFn / pipeline interfaces as GF(2^8) ones, tagged by
// field_w = 16).
inline Mat pack16(const gf16w::Mat& c) {
  Mat b(2 * c.size());
  for (size_t i = 0; i < c.size(); ++i) {
    b[2 * i] = static_cast<uint8_t>(c[i] & 0xFF);
    b[2 * i + 1] = static_cast<uint8_t>(c[i] >> 8);
  }
  return b;
}
inline gf16w::Mat unpack16(const Mat& b) {
  gf16w::Mat c(b.size() / 2);
  for (size_t i = 0; i < c.size(); ++i) c[i] = static_cast<uint16_t>(b[2 * i] | (b[2 * i + 1] << 8));
  return c;
}
// Bytes of an m x k coefficient matrix of field width w (8, 4: one byte each; 16: two).
inline size_t coeff_bytes(int m, int k, int field_w) { return size_t(m) * k * (field_w == 16 ? 2 : 1); }
// Largest k and m a descriptor of field width w takes (GF(2^16): n <= 65535 chunks).
inline int max_rows(int field_w) { return field_w == 16 ? 65535 : 256; }

// coeff: m x k row-major (GF(2^8), GF(16) nibble-method coefficients with field_w = 4, or packed
// GF(2^16) with field_w = 16 — layout desc_layout16, four records per coefficient), or empty to
// leave the table block zeroed (filled later on device by launch_perm_tables / launch_gf_invert).
// copy may be empty (no fused copies).
inline std::vector<uint8_t> build_desc(int k, int m, const std::vector<uint64_t>& in,
                                       const std::vector<uint64_t>& copy, const std::vector<uint64_t>& out,
                                       const Mat& coeff, int field_w = 8) {
  if (field_w != 8 && field_w != 4 && field_w != 16) throw std::invalid_argument("build_desc: field_w must be 8, 4 or 16");
  if (k <= 0 || m <= 0 || k > max_rows(field_w) || m > max_rows(field_w))
    throw std::invalid_argument("build_desc: 1 <= k,m <= 256 (65535 for GF(2^16))");
  if (int(in.size()) != k) throw std::invalid_argument("build_desc: need k input pointers");
  if (int(out.size()) != m) throw std::invalid_argument("build_desc: need m output pointers");
  if (!copy.empty() && int(copy.size()) != k) throw std::invalid_argument("build_desc: copy must be empty or k long");
  if (!coeff.empty() && coeff.size() != coeff_bytes(m, k, field_w))
    throw std::invalid_argument("build_desc: coeff must be m*k (2*m*k bytes for GF(2^16))");
  const int m_pad = pad_m(m);
  const DescLayout l = field_w == 16 ? desc_layout16(k, m_pad) : desc_layout(k, m_pad);
  std::vector<uint8_t> d(l.bytes, 0);
  DescHeader h{k, m, m_pad, 1};
  std::memcpy(d.data(), &h, sizeof(h));
  std::memcpy(d.data() + l.in_off, in.data(), 8 * size_t(k));
  if (!copy.empty()) std::memcpy(d.data() + l.copy_off, copy.data(), 8 * size_t(k));
  std::memcpy(d.data() + l.out_off, out.data(), 8 * size_t(m));
  if (!coeff.empty() && field_w == 16) {
    const gf16w::Mat c = unpack16(coeff);
    auto* tab = reinterpret_cast<PermTable*>(d.data() + l.tab_off);  // [k][m_pad][4]
    for (int j = 0; j < k; ++j)
      for (int i = 0; i < m; ++i) {
        const auto q = gf16w::perm_quad(c[size_t(i) * k + j]);
        std::memcpy(tab + (size_t(j) * m_pad + i) * 4, q.data(), sizeof(q));
      }
  } else if (!coeff.empty()) {
    const std::vector<PermTable> t = perm_tables_kmajor(coeff, m, k, field_w);
    for (int j = 0; j < k; ++j)
      std::memcpy(d.data() + l.tab_off + (size_t(j) * m_pad) * sizeof(PermTable), &t[size_t(j) * m],
                  sizeof(PermTable) * size_t(m));
  }
  return d;
}

}  // namespace gfrs

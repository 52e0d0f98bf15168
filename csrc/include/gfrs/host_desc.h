// Host-side construction of GF-GEMM descriptors (layout in gfrs/desc.h).
#pragma once

#include <cstring>
#include <stdexcept>
#include <vector>

#include "gfrs/desc.h"
#include "gfrs/matrix.h"

namespace gfrs {

// coeff: m x k row-major (GF(2^8), or GF(16) nibble-method coefficients with field_w = 4), or empty
// to leave the table block zeroed (filled later on device by
// launch_perm_tables / launch_gf_invert). copy may be empty (no fused copies).
inline std::vector<uint8_t> build_desc(int k, int m, const std::vector<uint64_t>& in,
                                       const std::vector<uint64_t>& copy, const std::vector<uint64_t>& out,
                                       const Mat& coeff, int field_w = 8) {
  if (k <= 0 || m <= 0 || k > 256 || m > 256) throw std::invalid_argument("build_desc: 1 <= k,m <= 256");
  if (int(in.size()) != k) throw std::invalid_argument("build_desc: need k input pointers");
  if (int(out.size()) != m) throw std::invalid_argument("build_desc: need m output pointers");
  if (!copy.empty() && int(copy.size()) != k) throw std::invalid_argument("build_desc: copy must be empty or k long");
  if (!coeff.empty() && coeff.size() != size_t(m) * k) throw std::invalid_argument("build_desc: coeff must be m*k");
  const int m_pad = pad_m(m);
  const DescLayout l = desc_layout(k, m_pad);
  std::vector<uint8_t> d(l.bytes, 0);
  DescHeader h{k, m, m_pad, 1};
  std::memcpy(d.data(), &h, sizeof(h));
  std::memcpy(d.data() + l.in_off, in.data(), 8 * size_t(k));
  if (!copy.empty()) std::memcpy(d.data() + l.copy_off, copy.data(), 8 * size_t(k));
  std::memcpy(d.data() + l.out_off, out.data(), 8 * size_t(m));
  if (!coeff.empty()) {
    if (field_w != 8 && field_w != 4) throw std::invalid_argument("build_desc: field_w must be 8 or 4");
    const std::vector<PermTable> t = perm_tables_kmajor(coeff, m, k, field_w);
    for (int j = 0; j < k; ++j)
      std::memcpy(d.data() + l.tab_off + (size_t(j) * m_pad) * sizeof(PermTable), &t[size_t(j) * m],
                  sizeof(PermTable) * size_t(m));
  }
  return d;
}

}  // namespace gfrs

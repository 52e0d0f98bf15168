// Device-resident GF-GEMM descriptor shared by the host runtime and the HIP kernels.
//
// A "GF-GEMM" computes, over a byte-column range [c0, c0+ncols):
//     out[i][c] = XOR_j  coeff[i][j] * in[j][c]        i in [0,m), j in [0,k)
// and optionally copies in[j][c] -> copy[j][c] while streaming (fused survivor copy of decode).
// Rows are addressed through pointer arrays so native chunks, parity chunks and decode survivors
// may live in separate allocations (the reference instead copies every row into one staging
// buffer, src/encode.cu:389-398, src/decode.cu:149-170).
//
// Layout (all offsets from the descriptor base, 32-byte aligned records):
//   [0,  16)              header {k, m, m_pad, batch}
//   [16, 16+8k)           in_ptr[k]      (uint64 device addresses)
//   [.., +8k)             copy_ptr[k]    (0 = no copy)
//   [.., +8*m_pad)        out_ptr[m_pad] (0 = padding row, never stored)
//   align 32, [.., +32*k*m_pad)   PermTable tab[k][m_pad]
#pragma once

#include <cstdint>
#include <cstddef>

#include "gfrs/gf256.h"

namespace gfrs {

struct DescHeader {
  int32_t k;
  int32_t m;
  int32_t m_pad;
  int32_t batch;
};

struct DescLayout {
  size_t in_off, copy_off, out_off, tab_off, bytes;
};

constexpr size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// `batch` stripes share one table block; stripe b's pointers are in[b*k + j], copy[b*k + j],
// out[b*m_pad + i] (batched small-object encode/decode in one launch).
constexpr DescLayout desc_layout(int k, int m_pad, int batch = 1) {
  DescLayout l{};
  l.in_off = sizeof(DescHeader);
  l.copy_off = l.in_off + 8 * size_t(k) * size_t(batch);
  l.out_off = l.copy_off + 8 * size_t(k) * size_t(batch);
  l.tab_off = align_up(l.out_off + 8 * size_t(m_pad) * size_t(batch), 32);
  l.bytes = l.tab_off + sizeof(PermTable) * size_t(k) * size_t(m_pad);
  return l;
}

// GF(2^16) descriptor (csrc/kernels/gf_gemm16.hip): the same header and pointer arrays (rows are
// byte rows holding little-endian 16-bit symbols), and FOUR records per coefficient, tab[j][i][q]
// with q = 2 * src_byte + dst_byte (gfrs/gf65536.h perm_quad).
constexpr DescLayout desc_layout16(int k, int m_pad, int batch = 1) {
  DescLayout l = desc_layout(k, m_pad, batch);
  l.bytes = l.tab_off + 4 * sizeof(PermTable) * size_t(k) * size_t(m_pad);
  return l;
}

// Output tile (outputs computed per thread). Tiles are powers of two; m is padded to a multiple.
constexpr int kMaxTile = 16;
constexpr int tile_for(int m) {
  int t = 1;
  while (t < m && t < kMaxTile) t <<= 1;
  return t;
}
constexpr int pad_m(int m) {
  const int t = tile_for(m);
  return (m + t - 1) / t * t;
}

}  // namespace gfrs

// GF(2^16) GEMM on gfx950 VALU: out[i][s] = XOR_j c[i][j] * in[j][s] over 16-bit symbols.
//
// Completes the reference's field family on the device: its generic field code names w = 4, 8 and
// 16 (/root/reference/src/galoisfield.cu:22-32, poly 0210013 for w = 16) but only GF(2^8) was ever
// built. A 16-bit field also lifts the n <= 256 chunk limit of GF(2^8) (n <= 65535 here).
//
// How it maps to the v_perm engine (gfrs/gf65536.h): multiplying by c is GF(2)-linear on 16 bits,
// so with a symbol's low byte l and high byte h
//     c * s = [L_ll(l) ^ L_hl(h)] | [L_lh(l) ^ L_hh(h)] << 8,
// four ordinary byte maps. A lane loads 16 bytes (8 little-endian symbols) of a row and
// de-interleaves them with two v_perm_b32 per 8 bytes into a low-byte plane LO and a high-byte
// plane HI (4 symbols per dword). Accumulators stay de-interleaved for the whole k loop:
//     acc_lo ^= L_ll(LO) ^ L_hl(HI)      acc_hi ^= L_lh(LO) ^ L_hh(HI)
// each one mac_pair (6 v_perm + 3 v_bitop3), with the selectors of LO and HI computed once per row
// and shared by every output of the tile. The planes are re-interleaved (2 v_perm per 8 bytes) only
// at the final store. Per byte and coefficient that is twice the GF(2^8) kernel's VALU work — the
// field's 16x16 bit map has four times the terms of the 8x8 one, spread over twice the bytes.
//
// Same streaming structure as gf_gemm.hip: 16-byte non-temporal loads, rows kept in flight by a
// register ring, XCD-aware block mapping, fused survivor copies on output tile 0 (decode), ragged
// tail symbols on extra lanes of the same launch, and a symbol kernel for rows that are not 16-byte
// aligned. Rows must be 2-byte aligned and column ranges whole symbols (even byte offsets/counts).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "gfrs/desc.h"
#include "gfrs/kernels.h"
#include "gfrs/tune.h"
#include "gfrs/perm_device.h"

namespace gfrs {
namespace {

using namespace permdev;

constexpr int kQuad = 4 * kPermStride;  // words per coefficient: {L_ll, L_lh, L_hl, L_hh}

// byte-plane shuffles (v_perm pool: bytes 0..3 = second operand, 4..7 = first operand)
constexpr uint32_t kSelLo = 0x06040200u;  // [l0 l1 l2 l3] from [l0 h0 l1 h1][l2 h2 l3 h3]
constexpr uint32_t kSelHi = 0x07050301u;  // [h0 h1 h2 h3]
constexpr uint32_t kSelW0 = 0x05010400u;  // [l0 h0 l1 h1] from lo=[l0..l3], hi=[h0..h3]
constexpr uint32_t kSelW1 = 0x07030602u;  // [l2 h2 l3 h3]

inline DescView view16(const void* desc, int k, int m_pad, int batch = 1) {
  const DescLayout l = desc_layout16(k, m_pad, batch);
  const char* b = static_cast<const char*>(desc);
  return {(cptr<uint64_t>)(b + l.in_off), (cptr<uint64_t>)(b + l.copy_off), (cptr<uint64_t>)(b + l.out_off),
          (cptr<uint32_t>)(b + l.tab_off)};
}

// Stripe b of a batched descriptor (blockIdx.y): its own row pointers, the shared table block.
__device__ __forceinline__ DescView stripe16(DescView d, int k, int m_pad) {
  const int b = blockIdx.y;
  d.in += size_t(b) * k;
  d.copy += size_t(b) * k;
  d.out += size_t(b) * m_pad;
  return d;
}

// One symbol column (2 bytes at `off`), one lane: k symbols loaded 8 at a time before use (see
// gf_gemm.hip tail_byte: a load-use-store loop would serialise every load behind the copy store).
template <int MT>
__device__ void tail_sym(const DescView& d, int k, int m_pad, int i0, bool do_copy, int64_t off) {
  constexpr int kB = 8;
  uint32_t lo[MT], hi[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) lo[i] = hi[i] = 0;
  for (int j0 = 0; j0 < k; j0 += kB) {
    uint16_t x[kB];
#pragma unroll
    for (int u = 0; u < kB; ++u)
      x[u] = j0 + u < k ? *(gptr<const uint16_t>)(d.in[j0 + u] + uint64_t(off)) : uint16_t(0);
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      const int j = j0 + u;
      if (j < k) {
        if (do_copy && d.copy[j]) *(gptr<uint16_t>)(d.copy[j] + uint64_t(off)) = x[u];
        const Sel sl = make_sel(x[u] & 0xFFu), sh = make_sel(uint32_t(x[u]) >> 8);
        const auto t = d.tab + (size_t(j) * m_pad + i0) * kQuad;
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const auto q = t + i * kQuad;
          lo[i] = mac_pair(lo[i], q, sl, q + 2 * kPermStride, sh);
          hi[i] = mac_pair(hi[i], q + kPermStride, sl, q + 3 * kPermStride, sh);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MT; ++i)
    if (d.out[i0 + i])
      *(gptr<uint16_t>)(d.out[i0 + i] + uint64_t(off)) = static_cast<uint16_t>((lo[i] & 0xFFu) | ((hi[i] & 0xFFu) << 8));
}

// Vector kernel: each lane owns G 16-byte groups (8 symbols each, kBlock groups apart so every load
// stays coalesced) of every row, PF rows in flight. The perm tables of a (row, output) pair are
// scalar loads, and a v_perm can read only one SGPR (the gfx9 constant-bus limit), so each table
// pair is first copied to a VGPR: with G = 2 that copy, the row's pointer and loop bookkeeping
// serve twice the symbols (profiles/gf65536/r08_k10: the w = 16 kernel is VALU-bound). A group
// past the row end reads group 0's bytes and stores nothing; lanes past the groups take one ragged
// tail symbol each.
template <int MT, int PF, int G>
__global__ __launch_bounds__(kBlock) void gf_gemm16_vec_kernel(DescView d, int k, int m_pad, int ntiles, int64_t col0,
                                                               int64_t ngroups, int64_t nblk, int64_t ncb,
                                                               int tail_syms) {
  d = stripe16(d, k, m_pad);
  const TileMap tm = map_block(ntiles);
  const int i0 = sgpr_int(tm.tile * MT);  // (first, with every lane active)
  if (tm.cb0 >= ncb) return;
  const bool do_copy = (tm.tile == 0);

  for (int64_t cb = tm.cb0; cb < nblk; cb += ncb) {
    const int64_t g0 = cb * (G * kBlock) + threadIdx.x;
    bool live[G];
    int64_t off[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      live[u] = g0 + u * kBlock < ngroups;
      off[u] = col0 + (live[u] ? g0 + u * kBlock : g0) * 16;
    }
    if (live[0]) {
      uint32_t lo[G][MT][2], hi[G][MT][2];
#pragma unroll
      for (int v = 0; v < G; ++v)
#pragma unroll
        for (int i = 0; i < MT; ++i) lo[v][i][0] = lo[v][i][1] = hi[v][i][0] = hi[v][i][1] = 0;

      u32x4 ring[PF][G];
#pragma unroll
      for (int u = 0; u < PF; ++u)
        if (u < k)
#pragma unroll
          for (int v = 0; v < G; ++v) ring[u][v] = ld16<true>(row_vec(d.in[u], off[v]));

      for (int j0 = 0; j0 < k; j0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
          const int j = j0 + u;
          if (j >= k) break;
          u32x4 x[G];
#pragma unroll
          for (int v = 0; v < G; ++v) {
            x[v] = ring[u][v];
            if (j + PF < k) ring[u][v] = ld16<true>(row_vec(d.in[j + PF], off[v]));
          }
          if (do_copy) {
            const uint64_t cp = d.copy[j];
            if (cp)
#pragma unroll
              for (int v = 0; v < G; ++v)
                if (live[v]) st16<true>(row_vec_w(cp, off[v]), x[v]);
          }
          const auto t = d.tab + (size_t(j) * m_pad + i0) * kQuad;
          MapV mv[MT][4];  // this row's tables, shared by the G groups and both plane words
#pragma unroll
          for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) mv[i][e] = map_v(t + i * kQuad + e * kPermStride);
#pragma unroll
          for (int v = 0; v < G; ++v) {
            const uint32_t L0 = __builtin_amdgcn_perm(x[v][1], x[v][0], kSelLo);
            const uint32_t H0 = __builtin_amdgcn_perm(x[v][1], x[v][0], kSelHi);
            const uint32_t L1 = __builtin_amdgcn_perm(x[v][3], x[v][2], kSelLo);
            const uint32_t H1 = __builtin_amdgcn_perm(x[v][3], x[v][2], kSelHi);
            const Sel sl0 = make_sel(L0), sh0 = make_sel(H0), sl1 = make_sel(L1), sh1 = make_sel(H1);
#pragma unroll
            for (int i = 0; i < MT; ++i) {
              const MapV& ll = mv[i][0];
              const MapV& lh = mv[i][1];
              const MapV& hl = mv[i][2];
              const MapV& hh = mv[i][3];
              lo[v][i][0] = mac_pair_v(lo[v][i][0], ll, sl0, hl, sh0);
              hi[v][i][0] = mac_pair_v(hi[v][i][0], lh, sl0, hh, sh0);
              lo[v][i][1] = mac_pair_v(lo[v][i][1], ll, sl1, hl, sh1);
              hi[v][i][1] = mac_pair_v(hi[v][i][1], lh, sl1, hh, sh1);
            }
          }
        }
      }

#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const uint64_t op = d.out[i0 + i];
        if (!op) continue;
#pragma unroll
        for (int v = 0; v < G; ++v) {
          if (!live[v]) continue;
          const u32x4 w{__builtin_amdgcn_perm(hi[v][i][0], lo[v][i][0], kSelW0),
                        __builtin_amdgcn_perm(hi[v][i][0], lo[v][i][0], kSelW1),
                        __builtin_amdgcn_perm(hi[v][i][1], lo[v][i][1], kSelW0),
                        __builtin_amdgcn_perm(hi[v][i][1], lo[v][i][1], kSelW1)};
          st16<true>(row_vec_w(op, off[v]), w);
        }
      }
    }
    // ragged tail symbols: virtual groups ngroups .. ngroups + tail_syms - 1, one symbol each
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int64_t t = g0 + u * kBlock - ngroups;
      if (t >= 0 && t < tail_syms) tail_sym<MT>(d, k, m_pad, i0, do_copy, col0 + ngroups * 16 + 2 * t);
    }
  }
}

// Symbol kernel: one lane per symbol, any 2-byte alignment (rows or column start off 16 bytes).
template <int MT>
__global__ __launch_bounds__(kBlock) void gf_gemm16_sym_kernel(DescView d, int k, int m_pad, int ntiles, int64_t col0,
                                                               int64_t nsyms, int64_t nblk, int64_t ncb) {
  d = stripe16(d, k, m_pad);
  const TileMap tm = map_block(ntiles);
  const int i0 = sgpr_int(tm.tile * MT);  // (first, with every lane active)
  if (tm.cb0 >= ncb) return;
  const bool do_copy = (tm.tile == 0);
  for (int64_t cb = tm.cb0; cb < nblk; cb += ncb) {
    const int64_t s = cb * kBlock + threadIdx.x;
    if (s < nsyms) tail_sym<MT>(d, k, m_pad, i0, do_copy, col0 + 2 * s);
  }
}

constexpr int64_t kMaxGridBlocks = int64_t(UINT32_MAX) / kBlock;

struct Grid {
  int64_t nblk, ncb;
  unsigned blocks;
};

inline Grid make_grid(int64_t items, int ntiles, int max_blocks) {
  Grid g{};
  g.nblk = (items + kBlock - 1) / kBlock;
  g.ncb = g.nblk;
  if (max_blocks > 0 && g.ncb > max_blocks) g.ncb = max_blocks;
  const int64_t cap = kMaxGridBlocks / ntiles / 8 * 8;
  if (g.ncb > cap) g.ncb = cap;
  g.blocks = static_cast<unsigned>((g.ncb < 8 ? g.ncb : (g.ncb + 7) / 8 * 8) * ntiles);  // see map_block
  return g;
}

// 16-byte groups per lane of the vector kernel where it may take two (GFRS_TUNE=gf16_vec_g=1: always
// one, for A/B measurements)
int vec_groups() {
  static const int v = tune_int("gf16_vec_g", 2) == 1 ? 1 : 2;
  return v;
}

// Output tile of the w = 16 kernel: the GF(2^8) tile (gfrs/desc.h tile_for) capped at 8, since
// each output holds four accumulator dwords per 16-byte group here (two planes x two dwords).
template <typename F>
hipError_t dispatch16(int m_pad, int mt_cap, F&& f) {
  switch (std::min(tile_for(m_pad), mt_cap)) {
    case 1: return f(std::integral_constant<int, 1>{});
    case 2: return f(std::integral_constant<int, 2>{});
    case 4: return f(std::integral_constant<int, 4>{});
    default: return f(std::integral_constant<int, 8>{});
  }
}

}  // namespace

hipError_t launch_gf_gemm16(const void* desc, int k, int m_pad, int64_t col0, int64_t ncols, bool symwise,
                            int max_blocks, hipStream_t stream, bool one_tile) {
  return launch_gf_gemm16_batched(desc, k, m_pad, 1, col0, ncols, symwise, max_blocks, stream, one_tile);
}

hipError_t launch_gf_gemm16_batched(const void* desc, int k, int m_pad, int batch, int64_t col0, int64_t ncols,
                                    bool symwise, int max_blocks, hipStream_t stream, bool one_tile) {
  if (k <= 0 || m_pad <= 0 || ncols <= 0) return ncols < 0 ? hipErrorInvalidValue : hipSuccess;
  if ((col0 | ncols) & 1) return hipErrorInvalidValue;  // whole 16-bit symbols only
  if (m_pad % tile_for(m_pad) != 0 || batch < 1 || batch > 65535) return hipErrorInvalidValue;
  const DescView d = view16(desc, k, m_pad, batch);
  // Short rows: one output per tile. The kernel parallelises over columns and output tiles only,
  // so a row of a few KiB is a handful of blocks each walking all k rows for 8 outputs (k = 300,
  // m = 40, 3.4 KiB: 5 blocks). One output per tile puts m times as many blocks on the chip; the
  // inputs they re-read are small enough to stay in L2. GFRS_TUNE=gf16_short_groups=N sets the cut
  // (16-byte groups per row, default 32768 = 512 KiB; 0 = never). Measured (profiles/gf65536/
  // r07_short): k = 300 m = 40, 3.4 KiB rows 1.05 -> 0.24 ms, 218 KiB rows 1.11 -> 0.64 ms;
  // k = 64 m = 16, 256 KiB rows 0.145 -> 0.055 ms; at 1 MiB rows one output per tile loses.
  static const int64_t short_groups = std::max<int64_t>(0, tune_int("gf16_short_groups", 32768));
  // (a batch fills the chip with its own grid rows: the cut counts the groups of every stripe)
  const int mt_cap = (ncols / 16 * batch < short_groups && !one_tile) ? 1 : 8;
  return dispatch16(m_pad, mt_cap, [&](auto mt) -> hipError_t {
    constexpr int MT = decltype(mt)::value;
    const int ntiles = m_pad / MT;
    if (symwise || (col0 & 15)) {
      const Grid g = make_grid(ncols / 2, ntiles, max_blocks);
      gf_gemm16_sym_kernel<MT>
          <<<dim3(g.blocks, batch), kBlock, 0, stream>>>(d, k, m_pad, ntiles, col0, ncols / 2, g.nblk, g.ncb);
      return hipGetLastError();
    }
    const int64_t ngroups = ncols / 16;
    const int tail_syms = int((ncols - ngroups * 16) / 2);
    // (a Grid item is one lane's G groups) Two groups per lane where the tile is small enough to
    // keep the registers low (MT <= 4: 111 VGPRs, against 177 at MT = 8) and the rows are long
    // (the short-row regime wants as many blocks as it can get). k = 10, m = 4, 1 GiB: 208 M VALU
    // instructions against 232 M, kernel 401 vs 431 us (profiles/gf65536/r08_k10).
    if (MT <= 4 && mt_cap > 1 && vec_groups() == 2) {
      const Grid g = make_grid((ngroups + tail_syms + 1) / 2, ntiles, max_blocks);
      gf_gemm16_vec_kernel<MT, 2, 2>
          <<<dim3(g.blocks, batch), kBlock, 0, stream>>>(d, k, m_pad, ntiles, col0, ngroups, g.nblk, g.ncb, tail_syms);
    } else {
      const Grid g = make_grid(ngroups + tail_syms, ntiles, max_blocks);
      gf_gemm16_vec_kernel<MT, 2, 1>
          <<<dim3(g.blocks, batch), kBlock, 0, stream>>>(d, k, m_pad, ntiles, col0, ngroups, g.nblk, g.ncb, tail_syms);
    }
    return hipGetLastError();
  });
}

}  // namespace gfrs

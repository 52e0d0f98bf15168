// GF(2^8) GEMM on gfx950 VALU: out[i][c] = XOR_j coeff[i][j] * in[j][c].
//
// Replaces the reference's K1/K2 `matrix_mul` kernels (src/matrix.cu:232-407). What changes and why
// (SURVEY §2.3, §3.3):
//   * GF multiply: the reference does 3 dependent LDS lookups per byte product
//     (gflog[a], gflog[b], gfexp[sum]; src/matrix.cu:105-110). Here every coefficient is a
//     GF(2)-linear byte map split over bit-chunks [2:0],[5:3],[7:6]; each chunk is ONE
//     v_perm_b32 byte-select from an 8-byte pool, applied to 4 bytes per instruction. Per 4
//     byte-products: 3 v_perm + 1.5 v_xor3 — no LDS, no branches. The selectors depend only on
//     the input bytes and are shared by all outputs of the tile.
//   * Tables are wave-uniform and live in a device descriptor read with scalar loads; nothing is
//     copied into LDS per block (the reference re-copies 1.5 KB of LUTs per block and every thread
//     redundantly re-stores the coefficient and data tiles, src/matrix.cu:250-292).
//   * 16-byte vector loads/stores per lane (global_load_dwordx4), one-row software prefetch,
//     no barriers at all (the reference has divergent __syncthreads on ragged tails,
//     src/matrix.cu:269-322). Ragged byte tails take one extra lane per byte in the same launch
//     instead of the reference's all-or-nothing `C % 8` switch to its slow byte path
//     (src/matrix.cu:796).
//   * XCD-aware block mapping: output tiles of the same column block are dealt to one XCD so the
//     re-read of the input rows by tile > 0 hits that XCD's L2 (cdna_hip_programming.md §5.5 T1).
//   * Fused survivor copy: decode streams every survivor row once and, when asked, writes it to
//     its destination row in the same pass (saves a full re-read of the survivors).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include <cstdint>

#include "gfrs/desc.h"
#include "gfrs/kernels.h"
#include "gfrs/tune.h"
#include "gfrs/perm_device.h"

namespace gfrs {
namespace {

using namespace permdev;  // Sel, mac_pair, DescView, map_block, ... (gfrs/perm_device.h)

// One byte column of the ragged tail (< 16 V bytes past the last full group), one lane per byte.
// The row bytes are loaded 8 at a time before any of them is used: a copy store may alias the
// next row's input as far as the compiler knows, so a plain load-use-store loop serialises every
// load behind the previous store. One lane walking the whole tail that way cost ~20 us per launch
// (k=10, 10-byte tail: 100 dependent HBM loads), the whole kernel time of a 1 MiB object
// (scripts/tail_probe.py, profiles/headline/r04_tail).
template <int MT>
__device__ void tail_byte(const DescView& d, int k, int m_pad, int i0, bool do_copy, int64_t off) {
  constexpr int kB = 8;
  uint32_t acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = 0;
  for (int j0 = 0; j0 < k; j0 += kB) {
    uint8_t x[kB];
#pragma unroll
    for (int u = 0; u < kB; ++u) x[u] = j0 + u < k ? ((gptr<const uint8_t>)d.in[j0 + u])[off] : uint8_t(0);
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      const int j = j0 + u;
      if (j < k) {
        if (do_copy && d.copy[j]) ((gptr<uint8_t>)d.copy[j])[off] = x[u];
        const Sel s = make_sel(x[u]);
        const auto t = d.tab + (size_t(j) * m_pad + i0) * kPermStride;
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[i] = mac_map(acc[i], t + i * kPermStride, s);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MT; ++i)
    if (d.out[i0 + i]) ((gptr<uint8_t>)d.out[i0 + i])[off] = uint8_t(acc[i]);
}

// Vector kernel: each lane owns V consecutive 16-byte groups of every row and keeps PF input rows
// in flight (a static register ring: the ring slot of row j is j % PF, resolved at compile time by
// unrolling the row loop PF-fold). Lanes ngroups .. ngroups + tail - 1 (past the last full group)
// take one ragged tail byte each, so no second launch is needed for odd chunk sizes.
// Stripe b of a batched descriptor (blockIdx.y): its own row pointers, the shared table block.
__device__ __forceinline__ DescView stripe(DescView d, int k, int m_pad) {
  const int b = blockIdx.y;
  d.in += size_t(b) * k;
  d.copy += size_t(b) * k;
  d.out += size_t(b) * m_pad;
  return d;
}

template <int MT, int V, int PF, bool NT>
__global__ __launch_bounds__(kBlock) void gf_gemm_vec_kernel(DescView d, int k, int m_pad, int ntiles,
                                                             int64_t col0, int64_t ngroups, int64_t nblk,
                                                             int64_t ncb, int tail) {
  d = stripe(d, k, m_pad);
  const TileMap tm = map_block(ntiles);
  if (tm.cb0 >= ncb) return;
  const int i0 = tm.tile * MT;
  const bool do_copy = (tm.tile == 0);

  for (int64_t cb = tm.cb0; cb < nblk; cb += ncb) {
    const int64_t g = cb * kBlock + threadIdx.x;
    if (g >= ngroups) {
      if (g - ngroups < tail) tail_byte<MT>(d, k, m_pad, i0, do_copy, col0 + ngroups * (16 * V) + (g - ngroups));
      continue;
    }
    const int64_t off = col0 + g * (16 * V);

    uint32_t acc[MT][4 * V];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int w = 0; w < 4 * V; ++w) acc[i][w] = 0;

    u32x4 ring[PF][V];
#pragma unroll
    for (int u = 0; u < PF; ++u)
      if (u < k) {
        const auto src = row_vec(d.in[u], off);
#pragma unroll
        for (int v = 0; v < V; ++v) ring[u][v] = ld16<NT>(src + v);
      }

    // Rows are consumed in pairs when PF is even: the six lookups of a pair fold into three
    // v_bitop3 XORs (1.5 per coefficient instead of 2). Pairs only for MT <= 8: at MT = 16 the
    // second row's live selectors/tables cost a wave per SIMD and the VALU-bound wide tile got
    // slower (profiles/r01_kbench3).
    constexpr bool kPairs = (PF % 2 == 0) && MT <= 8;
    for (int j0 = 0; j0 < k; j0 += PF) {
#pragma unroll
      for (int u = 0; u < PF; u += (kPairs ? 2 : 1)) {
        const int j = j0 + u;
        if (kPairs && j + 1 < k) {
          u32x4 x0[V], x1[V];
#pragma unroll
          for (int v = 0; v < V; ++v) {
            x0[v] = ring[u][v];
            x1[v] = ring[u + 1][v];
          }
          if (j + PF < k) {
            const auto src = row_vec(d.in[j + PF], off);
#pragma unroll
            for (int v = 0; v < V; ++v) ring[u][v] = ld16<NT>(src + v);
          }
          if (j + 1 + PF < k) {
            const auto src = row_vec(d.in[j + 1 + PF], off);
#pragma unroll
            for (int v = 0; v < V; ++v) ring[u + 1][v] = ld16<NT>(src + v);
          }
          if (do_copy) {
            const uint64_t cp0 = d.copy[j], cp1 = d.copy[j + 1];
            if (cp0) {
              const auto dst = row_vec_w(cp0, off);
#pragma unroll
              for (int v = 0; v < V; ++v) st16<NT>(dst + v, x0[v]);
            }
            if (cp1) {
              const auto dst = row_vec_w(cp1, off);
#pragma unroll
              for (int v = 0; v < V; ++v) st16<NT>(dst + v, x1[v]);
            }
          }
          const auto t0 = d.tab + (size_t(j) * m_pad + i0) * kPermStride;
          const auto t1 = t0 + size_t(m_pad) * kPermStride;
#pragma unroll
          for (int v = 0; v < V; ++v) {
#pragma unroll
            for (int w = 0; w < 4; ++w) {
              const Sel s0 = make_sel(x0[v][w]);
              const Sel s1 = make_sel(x1[v][w]);
#pragma unroll
              for (int i = 0; i < MT; ++i)
                acc[i][v * 4 + w] = mac_pair(acc[i][v * 4 + w], t0 + i * kPermStride, s0, t1 + i * kPermStride, s1);
            }
          }
        } else if (j < k) {
          u32x4 x[V];
#pragma unroll
          for (int v = 0; v < V; ++v) x[v] = ring[u][v];
          if (j + PF < k) {
            const auto src = row_vec(d.in[j + PF], off);
#pragma unroll
            for (int v = 0; v < V; ++v) ring[u][v] = ld16<NT>(src + v);
          }
          if (do_copy) {
            const uint64_t cp = d.copy[j];
            if (cp) {
              const auto dst = row_vec_w(cp, off);
#pragma unroll
              for (int v = 0; v < V; ++v) st16<NT>(dst + v, x[v]);
            }
          }
          const auto t = d.tab + (size_t(j) * m_pad + i0) * kPermStride;
#pragma unroll
          for (int v = 0; v < V; ++v) {
#pragma unroll
            for (int w = 0; w < 4; ++w) {
              const Sel s = make_sel(x[v][w]);
#pragma unroll
              for (int i = 0; i < MT; ++i) acc[i][v * 4 + w] = mac_map(acc[i][v * 4 + w], t + i * kPermStride, s);
            }
          }
        }
      }
    }

#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const uint64_t op = d.out[i0 + i];
      if (!op) continue;
      const auto dst = row_vec_w(op, off);
#pragma unroll
      for (int v = 0; v < V; ++v)
        st16<NT>(dst + v, u32x4{acc[i][v * 4 + 0], acc[i][v * 4 + 1], acc[i][v * 4 + 2], acc[i][v * 4 + 3]});
    }
  }
}

// Rows-in-flight kernel (narrow codes, compile-time K): each lane issues the loads of all K rows of
// its 16-byte group before the first multiply, so a wave keeps K KiB in flight instead of the vec
// kernel's PF KiB, and each row is consumed as it lands (the compiler counts vmcnt exactly: the
// loop is fully unrolled and every load unconditional). This is the access form that reaches the
// pattern ceiling with no math at all (scripts/membench.hip: 252 us for 10 rows in and 4 out,
// against 292 us for the PF = 2 vec kernel on the same box, profiles/headline/r05_rows). Fused copies (tile
// 0 of a decode) are stored as their row lands.
template <int MT, int K>
__global__ __launch_bounds__(kBlock) void gf_gemm_rows_kernel(DescView d, int k_tail, int m_pad, int ntiles,
                                                              int64_t col0, int64_t ngroups, int tail) {
  // One group per lane and no grid-stride loop: around a loop, every table word (K x MT x 5, all
  // loop-invariant) would be hoisted into SGPRs ahead of it and spilled (162 VGPRs at K = 10,
  // MT = 4); straight-line code keeps only one row pair's tables live (80-ish VGPRs).
  d = stripe(d, K, m_pad);
  const TileMap tm = map_block(ntiles);
  const int i0 = tm.tile * MT;
  const bool do_copy = (tm.tile == 0);
  const int64_t g = tm.cb0 * kBlock + threadIdx.x;
  if (g >= ngroups) {
    // (k_tail == K, passed at run time: a compile-time K would unroll the tail's row loop too)
    if (g - ngroups < tail) tail_byte<MT>(d, k_tail, m_pad, i0, do_copy, col0 + ngroups * 16 + (g - ngroups));
    return;
  }
  const int64_t off = col0 + g * 16;
  u32x4 x[K];
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = ld16<true>(row_vec(d.in[j], off));
  uint32_t acc[MT][4];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int w = 0; w < 4; ++w) acc[i][w] = 0;
#pragma unroll
  for (int j = 0; j < K; j += 2) {
    if (do_copy) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
        if (j + u < K) {
          const uint64_t cp = d.copy[j + u];
          if (cp) st16<true>(row_vec_w(cp, off), x[j + u]);
        }
    }
    const auto t0 = d.tab + (size_t(j) * m_pad + i0) * kPermStride;
    if (j + 1 < K) {
      const auto t1 = t0 + size_t(m_pad) * kPermStride;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const Sel s0 = make_sel(x[j][w]);
        const Sel s1 = make_sel(x[j + 1][w]);
#pragma unroll
        for (int i = 0; i < MT; ++i)
          acc[i][w] = mac_pair(acc[i][w], t0 + i * kPermStride, s0, t1 + i * kPermStride, s1);
      }
    } else {
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const Sel s = make_sel(x[j][w]);
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[i][w] = mac_map(acc[i][w], t0 + i * kPermStride, s);
      }
    }
    // one row pair at a time: the scheduler would otherwise compute every row's selectors (and
    // load every pair's tables) as soon as the rows land, 12 VGPRs + 2 MT x 5 SGPRs per row
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const uint64_t op = d.out[i0 + i];
    if (op) st16<true>(row_vec_w(op, off), u32x4{acc[i][0], acc[i][1], acc[i][2], acc[i][3]});
  }
}

// The rows kernel's latency form, for copy-free launches up to rows_lat_groups() (serving batches,
// single objects). In the kernel above the compiler issues every row pair's table loads up front,
// each behind its own lgkmcnt(0), and spills them to VGPR lanes (102 SGPRs, 140-151 VGPRs at
// K = 10, MT = 4): a serial chain of scalar-load latencies that a lone wave cannot hide. Here the
// table pointer is re-issued by an empty asm after each pair's math (its input), so each pair's
// loads wait only for the previous pair, and the tile index sits in an SGPR: no spills, 74 VGPRs.
// Alone it is also faster on big launches (245.7 vs 250.7 us per GiB), but in the two-lane
// bench step it competes with the other lane's decode instead of trickling beside it and the step
// runs 6 % slower (profiles/headline/r07_rows), so big launches keep the kernel above.
// COPY: fused survivor copies (tile 0 of a decode), stored as each row pair is consumed.
template <int MT, int K, bool COPY>
__global__ __launch_bounds__(kBlock) void gf_gemm_rows_lat_kernel(DescView d, int k_tail, int m_pad, int ntiles,
                                                                  int64_t col0, int64_t ngroups, int tail) {
  d = stripe(d, K, m_pad);
  const TileMap tm = map_block(ntiles);
  const int i0 = sgpr_int(tm.tile * MT);
  const bool do_copy = COPY && (tm.tile == 0);
  const int64_t g = tm.cb0 * kBlock + threadIdx.x;
  if (g >= ngroups) {
    if (g - ngroups < tail) tail_byte<MT>(d, k_tail, m_pad, i0, do_copy, col0 + ngroups * 16 + (g - ngroups));
    return;
  }
  const int64_t off = col0 + g * 16;
  u32x4 x[K];
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = ld16<true>(row_vec(d.in[j], off));
  u32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = u32x4{0u, 0u, 0u, 0u};
  uint64_t tb = (uint64_t)d.tab;
#pragma unroll
  for (int j = 0; j < K; j += 2) {
    if (j > 0) {
#pragma unroll
      for (int i = 0; i < MT; ++i) asm volatile("" ::"v"(acc[i]));
    }
    asm volatile("" : "+s"(tb));
    asm volatile("" : "+v"(x[j]));
    if (j + 1 < K) asm volatile("" : "+v"(x[j + 1]));
    if (COPY && do_copy) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
        if (j + u < K) {
          const uint64_t cp = d.copy[j + u];
          if (cp) st16<true>(row_vec_w(cp, off), x[j + u]);
        }
    }
    const auto t0 = (cptr<uint32_t>)tb + (size_t(j) * m_pad + i0) * kPermStride;
    if (j + 1 < K) {
      const auto t1 = t0 + size_t(m_pad) * kPermStride;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const Sel s0 = make_sel(x[j][w]);
        const Sel s1 = make_sel(x[j + 1][w]);
#pragma unroll
        for (int i = 0; i < MT; ++i)
          acc[i][w] = mac_pair(acc[i][w], t0 + i * kPermStride, s0, t1 + i * kPermStride, s1);
      }
    } else {
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const Sel s = make_sel(x[j][w]);
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[i][w] = mac_map(acc[i][w], t0 + i * kPermStride, s);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const uint64_t op = d.out[i0 + i];
    if (op) st16<true>(row_vec_w(op, off), acc[i]);
  }
}

// K-split kernel (short rows of wide codes, e.g. batched RS(128,160) serving objects): the vec
// kernel parallelises over 16-byte column groups and output tiles only, so a 512-byte row gives
// 32 lanes per tile and each of them walks all k rows with PF in flight — at k = 128 a 64-deep
// chain of load latencies per launch (~70 us whatever the batch, profiles/serving/r07_wide).
// Here the k rows are split over the KS waves of a block (wave s owns rows [s R, s R + R), R =
// ceil(k / KS), 8 in flight per lane), each wave covers the same 64 column groups, and the KS
// partial products are XOR-reduced through LDS; every thread of the block then stores part of
// the MT x 64 result groups. Fused copies: tile 0 stores each row it loads. Column tails
// (ncols % 16) go to the byte kernel.
template <int MT, int KS>
__global__ __launch_bounds__(64 * KS) void gf_gemm_ksplit_kernel(DescView d, int k, int m_pad, int ntiles,
                                                                 int64_t col0, int64_t ngroups, int copies) {
  constexpr int kRB = 8;
  // one LDS area, used twice: first the tile's perm records of all k rows (k x MT x 32 bytes, at
  // most 256 x MT x 32 = KS x MT KiB), then the KS partial products for the reduction
  __shared__ u32x4 smem[KS * MT * 64];
  d = stripe(d, k, m_pad);
  const int tile = int(blockIdx.x % unsigned(ntiles));
  const int64_t cb = int64_t(blockIdx.x / unsigned(ntiles));
  const int i0 = tile * MT;
  const int lane = int(threadIdx.x & 63u);
  const int s = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int64_t g = cb * 64 + lane;
  const bool live = g < ngroups;
  const int64_t off = col0 + (live ? g : cb * 64) * 16;  // dead lanes re-read the block's first group
  const bool do_copy = copies && tile == 0;
  const int R = (k + KS - 1) / KS;
  const int jb = s * R, je = min(k, jb + R);

  // stage the tables: one L2 round trip per block instead of a chain of scalar loads per row (the
  // scalar cache cannot hold a wide code's tables, 32 KiB per tile at k = 128)
  for (int c = int(threadIdx.x); c < k * MT * 2; c += 64 * KS) {
    const int row = c / (MT * 2), part = c % (MT * 2);
    smem[c] = ((gptr<const u32x4>)(uint64_t)(d.tab + (size_t(row) * m_pad + i0) * kPermStride))[part];
  }
  __syncthreads();
  const uint32_t* tl = reinterpret_cast<const uint32_t*>(smem);

  u32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = u32x4{0u, 0u, 0u, 0u};
  for (int j0 = jb; j0 < je; j0 += kRB) {
    u32x4 x[kRB];
#pragma unroll
    for (int u = 0; u < kRB; ++u) x[u] = j0 + u < je ? ld16<false>(row_vec(d.in[j0 + u], off)) : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int u = 0; u < kRB; u += 2) {
      const int j = j0 + u;
      if (j >= je) break;
      if (do_copy && live) {
        const uint64_t cp0 = d.copy[j];
        if (cp0) st16<false>(row_vec_w(cp0, off), x[u]);
        if (j + 1 < je) {
          const uint64_t cp1 = d.copy[j + 1];
          if (cp1) st16<false>(row_vec_w(cp1, off), x[u + 1]);
        }
      }
      const uint32_t* t0 = tl + size_t(j) * MT * kPermStride;
      if (j + 1 < je) {
        const uint32_t* t1 = t0 + MT * kPermStride;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const Sel s0 = make_sel(x[u][w]);
          const Sel s1 = make_sel(x[u + 1][w]);
#pragma unroll
          for (int i = 0; i < MT; ++i)
            acc[i][w] = mac_pair(acc[i][w], t0 + i * kPermStride, s0, t1 + i * kPermStride, s1);
        }
      } else {
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const Sel s0 = make_sel(x[u][w]);
#pragma unroll
          for (int i = 0; i < MT; ++i) acc[i][w] = mac_map(acc[i][w], t0 + i * kPermStride, s0);
        }
      }
    }
  }
  __syncthreads();  // every wave is done with the tables
#pragma unroll
  for (int i = 0; i < MT; ++i) smem[(s * MT + i) * 64 + lane] = acc[i];
  __syncthreads();
  for (int r = int(threadIdx.x); r < MT * 64; r += 64 * KS) {
    const int i = r >> 6, l = r & 63;
    u32x4 v = smem[i * 64 + l];
#pragma unroll
    for (int q = 1; q < KS; ++q) v ^= smem[(q * MT + i) * 64 + l];
    const int64_t gg = cb * 64 + l;
    const uint64_t op = d.out[i0 + i];
    if (gg < ngroups && op) st16<false>(row_vec_w(op, col0 + gg * 16), v);
  }
}

// Byte kernel: one lane per byte column; any alignment (unaligned rows, column starts off a 16-byte
// boundary). Each lane runs tail_byte: its k row bytes are loaded 8 at a time before use. SERIAL =
// the round-3 form (load, copy-store, use, one row at a time: every load waits for the previous
// store), kept as an ablation (gemm_variant vec = -1).
template <int MT, bool SERIAL>
__global__ __launch_bounds__(kBlock) void gf_gemm_byte_kernel(DescView d, int k, int m_pad, int ntiles,
                                                              int64_t col0, int64_t ncols, int64_t nblk,
                                                              int64_t ncb) {
  d = stripe(d, k, m_pad);
  const TileMap tm = map_block(ntiles);
  if (tm.cb0 >= ncb) return;
  const int i0 = tm.tile * MT;
  const bool do_copy = (tm.tile == 0);
  for (int64_t cb = tm.cb0; cb < nblk; cb += ncb) {
    const int64_t c = cb * kBlock + threadIdx.x;
    if (c >= ncols) continue;
    const int64_t off = col0 + c;
    if constexpr (!SERIAL) {
      tail_byte<MT>(d, k, m_pad, i0, do_copy, off);
      continue;
    }
    uint32_t acc[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) acc[i] = 0;
    for (int j = 0; j < k; ++j) {
      const uint8_t x = ((gptr<const uint8_t>)d.in[j])[off];
      if (do_copy) {
        const uint64_t cp = d.copy[j];
        if (cp) ((gptr<uint8_t>)cp)[off] = x;
      }
      const Sel s = make_sel(x);
      const auto t = d.tab + (size_t(j) * m_pad + i0) * kPermStride;
#pragma unroll
      for (int i = 0; i < MT; ++i) acc[i] = mac_map(acc[i], t + i * kPermStride, s);
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const uint64_t op = d.out[i0 + i];
      if (op) ((gptr<uint8_t>)op)[off] = static_cast<uint8_t>(acc[i] & 0xFF);
    }
  }
}

struct Grid {
  int64_t nblk, ncb;
  unsigned blocks;
};

// A launch holds at most 2^32 - 1 work-items along x: past that the column blocks are capped (the
// vec and byte kernels stride over the rest; the rows kernel has no stride loop and is not used).
constexpr int64_t kMaxGridBlocks = int64_t(UINT32_MAX) / kBlock;
inline int64_t grid_cap(int ntiles) { return kMaxGridBlocks / ntiles / 8 * 8; }

inline Grid make_grid(int64_t items, int ntiles, int max_blocks) {
  Grid g{};
  g.nblk = (items + kBlock - 1) / kBlock;
  g.ncb = g.nblk;
  if (max_blocks > 0 && g.ncb > max_blocks) g.ncb = max_blocks;
  if (g.ncb > grid_cap(ntiles)) g.ncb = grid_cap(ntiles);
  const int64_t ncb8 = g.ncb < 8 ? g.ncb : (g.ncb + 7) / 8 * 8;  // short: unpadded (map_block)
  g.blocks = static_cast<unsigned>(ncb8 * ntiles);
  return g;
}

template <int MT, int V, int PF, bool NT>
hipError_t launch_vec_cfg(const DescView& d, int k, int m_pad, int batch, int64_t col0, int64_t ngroups, int tail,
                          int max_blocks, hipStream_t stream) {
  const int ntiles = m_pad / MT;
  // one extra lane per ragged tail byte past the last group
  const Grid g = make_grid(ngroups + tail, ntiles, max_blocks);
  if (g.nblk == 0) return hipSuccess;
  gf_gemm_vec_kernel<MT, V, PF, NT>
      <<<dim3(g.blocks, batch), kBlock, 0, stream>>>(d, k, m_pad, ntiles, col0, ngroups, g.nblk, g.ncb, tail);
  return hipGetLastError();
}

template <int MT>
hipError_t launch_byte(const DescView& d, int k, int m_pad, int batch, int64_t col0, int64_t ncols, int max_blocks,
                       hipStream_t stream, bool serial = false) {
  if (ncols <= 0) return hipSuccess;
  const int ntiles = m_pad / MT;
  const Grid g = make_grid(ncols, ntiles, max_blocks);
  if (serial)
    gf_gemm_byte_kernel<MT, true>
        <<<dim3(g.blocks, batch), kBlock, 0, stream>>>(d, k, m_pad, ntiles, col0, ncols, g.nblk, g.ncb);
  else
    gf_gemm_byte_kernel<MT, false>
        <<<dim3(g.blocks, batch), kBlock, 0, stream>>>(d, k, m_pad, ntiles, col0, ncols, g.nblk, g.ncb);
  return hipGetLastError();
}

template <typename F>
hipError_t dispatch_tile(int t, F&& f) {
  switch (t) {
    case 1: return f(std::integral_constant<int, 1>{});
    case 2: return f(std::integral_constant<int, 2>{});
    case 4: return f(std::integral_constant<int, 4>{});
    case 8: return f(std::integral_constant<int, 8>{});
    default: return f(std::integral_constant<int, 16>{});
  }
}

// Kernel configuration (V = 16-byte groups per lane, PF = rows in flight, NT = non-temporal).
struct Cfg {
  int vec = 1, pf = 2;
  bool nt = false;
};

// Launches of at most this many 16-byte groups (all stripes of a batch) take the latency form of
// the rows kernel: 2^22 groups = 64 MiB of every row. Measured (profiles/serving/r07_serve):
// every serving batch up to 256 x 1 MiB objects encodes 15-30 % faster with it (256 x 64 KiB
// 20.6 vs 28.0 us, 256 x 1 MiB 67 vs 96 us); the 1 GiB headline stripe (6.7 M groups) keeps the
// throughput form for its two-lane overlap. GFRS_TUNE=rows_lat_groups=N overrides (0 = never).
int64_t rows_lat_groups() {
  static const int64_t v = std::max<int64_t>(0, tune_int("rows_lat_groups", int64_t(1) << 22));
  return v;
}

// Lane target of a wide-code launch (output tile of 8+ rows) that the k-split kernel does not
// take, before its tile is narrowed; GFRS_TUNE=short_lanes=N sets it (default 0 = never narrow:
// the k-split kernel beat every narrowed tile on the short-row points, profiles/serving/r07_wide).
int64_t short_lanes() {
  static const int64_t v = std::max<int64_t>(0, tune_int("short_lanes", 0));
  return v;
}

// Launches whose lanes (16-byte groups x stripes x output tiles at the widest tile) number fewer
// than this take the k-split kernel when 32 <= k <= 256 (its LDS holds 256 rows of tables);
// GFRS_TUNE=ksplit_lanes=N overrides (0 = never).
// Measured with scripts/serve_bench.py --code (profiles/serving/r07_wide/xcd): the k-split kernel
// wins every point up to 65 K lanes (RS(128,160) 16 x 64 KiB encode 294 -> 23 us, 16 x 1 MiB
// 263 -> 51 us; RS(64,80) 16 x 4 MiB 141 -> 88 us; RS(32,40) 16 x 1 MiB 33 -> 18 us) and the vec
// kernel every point from 131 K (RS(128,160) 256 x 1 MiB 432 vs 738 us; RS(32,40) 256 x 256 KiB
// 41 vs 51 us).
int64_t ksplit_lanes() {
  static const int64_t v = std::max<int64_t>(0, tune_int("ksplit_lanes", int64_t(1) << 17));
  return v;
}

constexpr int kSplit = 8;  // waves per k-split block

template <int MT>
hipError_t launch_ksplit(const DescView& d, int k, int m_pad, int batch, int64_t col0, int64_t ncols, bool copies,
                         hipStream_t stream) {
  if constexpr (MT > 8) {
    return hipErrorInvalidValue;  // LDS: KS x MT x 1 KiB
  } else {
    const int ntiles = m_pad / MT;
    const int64_t ngroups = ncols / 16;
    const int64_t ncb = (ngroups + 63) / 64;
    if (ncb * ntiles > int64_t(UINT32_MAX)) return hipErrorInvalidValue;
    if (ncb > 0)
      gf_gemm_ksplit_kernel<MT, kSplit><<<dim3(unsigned(ncb * ntiles), batch), 64 * kSplit, 0, stream>>>(
          d, k, m_pad, ntiles, col0, ngroups, copies ? 1 : 0);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess || ncols % 16 == 0) return e;
    return launch_byte<MT>(d, k, m_pad, batch, col0 + ngroups * 16, ncols % 16, 0, stream);
  }
}

template <int MT, int K>
hipError_t launch_rows_k(const DescView& d, int m_pad, int batch, int64_t col0, int64_t ngroups, int tail,
                         bool copies, hipStream_t stream) {
  const int ntiles = m_pad / MT;
  const Grid g = make_grid(ngroups + tail, ntiles, 0);  // one group per lane: the whole grid
  if (g.nblk == 0) return hipSuccess;
  if (g.ncb < g.nblk) return hipErrorInvalidValue;  // beyond one launch's work-items
  if ((ngroups + tail) * batch <= rows_lat_groups()) {
    if (copies)
      gf_gemm_rows_lat_kernel<MT, K, true>
          <<<dim3(g.blocks, batch), kBlock, 0, stream>>>(d, K, m_pad, ntiles, col0, ngroups, tail);
    else
      gf_gemm_rows_lat_kernel<MT, K, false>
          <<<dim3(g.blocks, batch), kBlock, 0, stream>>>(d, K, m_pad, ntiles, col0, ngroups, tail);
  } else
    gf_gemm_rows_kernel<MT, K><<<dim3(g.blocks, batch), kBlock, 0, stream>>>(d, K, m_pad, ntiles, col0, ngroups, tail);
  return hipGetLastError();
}

// the rows-in-flight kernel exists for the BASELINE codes' k (4, 10, 16) and k = 8, with tiles of at
// most 4 outputs (its K x 4 VGPRs of loads plus 4 MT accumulators stay near the vec kernel's count)
bool rows_supported(int k, int mt) { return mt <= 4 && (k == 4 || k == 8 || k == 10 || k == 16); }

template <int MT>
hipError_t launch_rows(const DescView& d, int k, int m_pad, int batch, int64_t col0, int64_t ngroups, int tail,
                       bool copies, hipStream_t stream) {
  if constexpr (MT <= 4) {
    switch (k) {
      case 4: return launch_rows_k<MT, 4>(d, m_pad, batch, col0, ngroups, tail, copies, stream);
      case 8: return launch_rows_k<MT, 8>(d, m_pad, batch, col0, ngroups, tail, copies, stream);
      case 10: return launch_rows_k<MT, 10>(d, m_pad, batch, col0, ngroups, tail, copies, stream);
      case 16: return launch_rows_k<MT, 16>(d, m_pad, batch, col0, ngroups, tail, copies, stream);
      default: break;
    }
  }
  return hipErrorInvalidValue;
}

template <int MT>
hipError_t launch_vec(const DescView& d, int k, int m_pad, int batch, int64_t col0, int64_t ncols, Cfg c,
                      int max_blocks, hipStream_t stream) {
  const int gbytes = 16 * c.vec;
  const int64_t ngroups = ncols / gbytes;
  const int tail = int(ncols - ngroups * gbytes);
  if (c.pf <= 0) {  // all rows in flight (vec = 1 only); pf = -t: output tiles of t rows instead of MT
    const int mt = c.pf == 0 ? MT : -c.pf;
    if (c.vec != 1 || max_blocks > 0 || m_pad % mt != 0 || !rows_supported(k, mt)) return hipErrorInvalidValue;
    switch (mt) {
      case 1: return launch_rows<1>(d, k, m_pad, batch, col0, ngroups, tail, true, stream);
      case 2: return launch_rows<2>(d, k, m_pad, batch, col0, ngroups, tail, true, stream);
      case 4: return launch_rows<4>(d, k, m_pad, batch, col0, ngroups, tail, true, stream);
      default: return hipErrorInvalidValue;
    }
  }
#define GFRS_CFG(V, PF, NT)                                                                             \
  if (c.vec == V && c.pf == PF && c.nt == NT)                                                           \
    return launch_vec_cfg<MT, V, PF, NT>(d, k, m_pad, batch, col0, ngroups, tail, max_blocks, stream);
  GFRS_CFG(1, 1, false)
  GFRS_CFG(1, 2, false)
  GFRS_CFG(1, 4, false)
  GFRS_CFG(1, 2, true)
  GFRS_CFG(1, 4, true)
  GFRS_CFG(2, 1, false)
  GFRS_CFG(2, 2, false)
  GFRS_CFG(2, 2, true)
  GFRS_CFG(1, 8, true)
  GFRS_CFG(1, 16, true)
  GFRS_CFG(2, 4, true)
  GFRS_CFG(2, 8, true)
#undef GFRS_CFG
  return hipErrorInvalidValue;
}

// Default configuration per output tile, chosen by scripts/kbench.py on MI355X
// (profiles/r01_kbench/kbench.json): non-temporal streaming with two rows in flight wins on every
// HBM-bound shape (k=10 encode 5.6 TB/s, 4-erasure decode 5.8 TB/s); the VALU-bound wide tile
// (MT = 16) prefers two 16-byte groups per lane to amortise the per-row table moves.
// GFRS_TUNE=vec_cfg=V:PF:NT (e.g. 1:4:1) replaces the default for every vector-kernel launch
// without an explicit variant (in the k=10 step: the decode; A/B measurements)
Cfg default_cfg(int mt) {
  static const int env[3] = {[] {
    const std::string v = tune_str("vec_cfg");
    return v.empty() ? 0 : std::atoi(v.c_str());
  }(), [] {
    const std::string v = tune_str("vec_cfg");
    const size_t c = v.find(':');
    return c == std::string::npos ? 0 : std::atoi(v.c_str() + c + 1);
  }(), [] {
    const std::string v = tune_str("vec_cfg");
    const size_t c = v.find(':');
    const size_t d = c == std::string::npos ? c : v.find(':', c + 1);
    return d == std::string::npos ? 1 : std::atoi(v.c_str() + d + 1);
  }()};
  Cfg c;
  c.vec = mt >= 16 ? 2 : 1;
  c.pf = 2;
  c.nt = true;
  if (env[0] > 0 && env[1] > 0) {
    c.vec = env[0];
    c.pf = env[1];
    c.nt = env[2] != 0;
  }
  return c;
}

// Where the rows-in-flight kernel is the default (copy-free descriptors, uncapped grid): measured
// on the encode shapes (scripts/kbench.py, profiles/headline/r05_rows) it wins only at k = 10 with 4-row
// tiles (262.6 vs 278.5 us per GiB); at k = 4 and 16 and in the decode (fused copies) the vec kernel
// is faster.
bool rows_default(int k, int mt) { return k == 10 && mt == 4; }

hipError_t run(const void* desc, int k, int m_pad, int batch, int64_t col0, int64_t ncols, bool bytewise,
               const Cfg* cfg, int max_blocks, hipStream_t stream, bool copies = true) {
  if (k <= 0 || m_pad <= 0 || ncols <= 0 || batch <= 0) return batch < 0 ? hipErrorInvalidValue : hipSuccess;
  if (m_pad % tile_for(m_pad) != 0 || batch > 65535) return hipErrorInvalidValue;
  const DescView d = view(desc, k, m_pad, batch);
  int tile = tile_for(m_pad);
  const bool auto_cfg = !cfg && max_blocks == 0 && !bytewise && !(col0 & 15);
  const bool ksplit = auto_cfg && k >= 32 && k <= 256 && (ncols / 16 + ncols % 16) * batch * (m_pad / tile) < ksplit_lanes();
  if (ksplit) tile = std::min(tile, 8);
  if (auto_cfg && !ksplit && tile >= 8) {
    // short rows of a wide code: the column groups alone leave lanes idle, so trade output-tile
    // width for more tiles until the launch has short_lanes() lanes
    int64_t lanes = (ncols / 16 + ncols % 16) * batch * (m_pad / tile);
    while (tile > 1 && lanes < short_lanes()) {
      tile /= 2;
      lanes *= 2;
    }
  }
  return dispatch_tile(tile, [&](auto mt) -> hipError_t {
    constexpr int MT = decltype(mt)::value;
    if (ksplit) return launch_ksplit<MT>(d, k, m_pad, batch, col0, ncols, copies, stream);
    if (bytewise || (col0 & 15) || (cfg && cfg->vec < 0))
      return launch_byte<MT>(d, k, m_pad, batch, col0, ncols, max_blocks, stream, cfg && cfg->vec < 0);
    const bool fits = (ncols / 16 + kBlock) / kBlock <= grid_cap(m_pad / MT);
    // small launches (serving): the latency form of the rows kernel for every shape it has, with
    // or without fused copies (launch_rows_k picks it by size)
    if (!cfg && max_blocks == 0 && fits && rows_supported(k, MT) &&
        (ncols / 16 + ncols % 16) * batch <= rows_lat_groups())
      return launch_rows<MT>(d, k, m_pad, batch, col0, ncols / 16, int(ncols % 16), copies, stream);
    if (!cfg && !copies && max_blocks == 0 && rows_default(k, MT) && fits)
      return launch_rows<MT>(d, k, m_pad, batch, col0, ncols / 16, int(ncols % 16), false, stream);
    return launch_vec<MT>(d, k, m_pad, batch, col0, ncols, cfg ? *cfg : default_cfg(MT), max_blocks, stream);
  });
}

}  // namespace

hipError_t launch_gf_gemm(const void* desc, int k, int m_pad, int64_t col0, int64_t ncols, bool force_bytewise,
                          int max_blocks, hipStream_t stream, bool copies) {
  return run(desc, k, m_pad, 1, col0, ncols, force_bytewise, nullptr, max_blocks, stream, copies);
}

hipError_t launch_gf_gemm_batched(const void* desc, int k, int m_pad, int batch, int64_t col0, int64_t ncols,
                                  bool force_bytewise, hipStream_t stream, bool copies) {
  return run(desc, k, m_pad, batch, col0, ncols, force_bytewise, nullptr, 0, stream, copies);
}

hipError_t launch_gf_gemm_variant(const void* desc, int k, int m_pad, int64_t col0, int64_t ncols, int vec, int pf,
                                  bool nt, int max_blocks, hipStream_t stream) {
  if (vec == 0) return run(desc, k, m_pad, 1, col0, ncols, true, nullptr, max_blocks, stream);
  Cfg c;
  c.vec = vec;  // vec < 0: the serial byte kernel (ablation)
  if (vec < 0) return run(desc, k, m_pad, 1, col0, ncols, true, &c, max_blocks, stream);
  c.pf = pf;
  c.nt = nt;
  return run(desc, k, m_pad, 1, col0, ncols, false, &c, max_blocks, stream);
}

}  // namespace gfrs

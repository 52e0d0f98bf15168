// GF(2^8) GEMM on gfx950 matrix cores, FP4 bit-matrix form — TILE-MAJOR variant ("tm").
//
// Same algebra, bit-matrix layout, B expansion and biased-float parity as gf_mfma_fp4.hip (read its
// header first); what changes is the loop order. The LDS kernels there walk a chunk K-step by
// K-step with every M-tile's accumulator live (224 AGPRs at 7 tiles), so a chunk ends with all
// tiles finishing at once: 224 accumulator reads and 196 bit inserts that the matrix pipe waits out,
// plus one bias MFMA per tile (56 % MFMA pipe on the k = 128 decode, profiles/wide_stripe/r07_pmc).
//
// Here a wave keeps its chunk's B operand resident instead — all 16 K-steps x 2 N-tiles, 128
// registers, in the AGPRs (this file is compiled with -amdgpu-mfma-vgpr-form, so the scaled MFMA
// reads B from AGPRs and keeps its accumulators in arch VGPRs) — and runs the M-tiles in pairs,
// 16 K-steps per pair (a pair is four independent accumulator chains; one tile alone is two, and
// the matrix pipe then waits on every other MFMA: profiles/wide_stripe/r08_tm):
//   * only two groups' accumulators are live: the pair accumulating and the previous one, whose
//     epilogue (bit inserts straight from VGPRs, 4 stores) runs under this pair's MFMAs;
//   * the bias is the C operand of a tile's first MFMA (a constant VGPR block), no extra MFMA;
//   * the next chunk's 8 ring slots are DMA'd during the first tile pair and expanded into the B
//     registers during the last group, step by step right after the last MFMA that reads each step's
//     old value; the fused survivor copies are stored in the same group, block-wide: each store
//     instruction writes 4 rows x 256 B out of the four waves' rings (two barriers per chunk), which
//     the memory system takes at 1.7x the rate of one wave's 16 rows x 64 B.
// With an odd tile count the last group is one tile: the next chunk's B expansion fills its stalls.
// Per 256-column chunk at 7 tiles: 224 MFMAs and ~680 VALU (v1: 238 MFMAs, ~840 VALU).
// At 8 tiles the A slice (128 KiB) plus the rings (32 KiB) and pointer tables would not fit the
// 160 KiB LDS, so tile 7's 16 A fragments stay in registers (64 AGPRs beside the 128 of B) and
// only tiles 0..6 are staged in LDS (112 KiB).
//
// Accumulator sets alternate by global group number; with an odd group count the chunk loop is
// unrolled by two so the set a group writes is never the one still waiting to be packed. An odd
// chunk count ends with a phantom chunk (its loads are dummies, its stores go to the sink) whose
// first group packs the last real chunk's last group.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <utility>

#include "gfrs/desc.h"
#include "gfrs/device_cache.h"
#include "gfrs/kernels.h"

namespace gfrs {
namespace {

using i32x8 = int __attribute__((ext_vector_type(8)));
using i32x4 = int __attribute__((ext_vector_type(4)));
using u32x4 = unsigned __attribute__((ext_vector_type(4)));
using f32x16 = float __attribute__((ext_vector_type(16)));
template <typename T>
using cptr = const __attribute__((address_space(4))) T*;
template <typename T>
using gptr = __attribute__((address_space(1))) T*;
using lds_u8 = __attribute__((address_space(3))) uint8_t;

constexpr int kSlotBytes = 1024;  // one ring slot: 16 input rows x the wave's 64 columns
constexpr int kCW = 64;           // columns per wave (two 32-column N-tiles, interleaved 2c + t)
constexpr int kNS = 16;           // K-steps per chunk (k in (112, 128]: 128 rows = 1024 bits)
constexpr int kKS = 8;            // ring slots per chunk (2 K-steps each) = the ring depth
constexpr int kRS = 16;           // input rows per ring slot
constexpr int kQ = 2;             // K-steps per super-step (LDS reads one super-step ahead)
constexpr int kBlockCols = 256;   // 4 waves x 64 columns
constexpr int kPtrBytes = 8 * (256 + 32 + 256);  // LDS: row, output-row and copy pointer tables

__device__ __forceinline__ void lgkm_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
template <typename T>
__device__ __forceinline__ void tie(T& v) {
  asm volatile("" : "+v"(v));
}
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}
// mask ? a : b per bit, one v_bitop3 (a builtin, so the compiler sees the accumulator reads and
// inserts the MFMA -> VALU wait states itself)
__device__ __forceinline__ uint32_t bfi(uint32_t mask, uint32_t a, uint32_t b) {
  return __builtin_amdgcn_bitop3_b32(mask, a, b, 0xCA);
}

// accumulator set of tile group g in chunk parity P (alternating over the global group sequence)
template <int NG>
__host__ __device__ constexpr int acc_set(int P, int g) {
  return (P * NG + g) & 1;
}

template <int MG, bool UNI, bool COPY>
__global__ __launch_bounds__(256, 1) void gf_gemm_fp4tm_kernel(cptr<uint64_t> in, cptr<uint64_t> out,
                                                               cptr<uint64_t> copy, const i32x4* __restrict__ bitmat,
                                                               int k, int m, int64_t col0, int64_t nchunks,
                                                               int64_t chunk_slots, int64_t in_stride) {
  static_assert(MG >= 5 && MG <= 8, "three tile groups at least: DMAs in group 0, the wait in group NG-2");
  constexpr int kLT = MG < 8 ? MG : 7;             // tiles whose A is staged in LDS (tile 7: registers)
  constexpr size_t kA = size_t(kLT) * kNS * 1024;  // LDS A slice [kstep][tile < kLT][lane] x 16 B
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  i32x4* afrag = reinterpret_cast<i32x4*>(smem);
  uint64_t* rowptr = reinterpret_cast<uint64_t*>(smem + kA);
  uint64_t* outptr = rowptr + 256;
  uint64_t* copyptr = outptr + 32;
  const int bid = blockIdx.x;
  const int64_t slot0 = int64_t(bid >> 3) * 8 + (bid & 7);  // slot -> one XCD (blocks round-robin)
  if (slot0 >= chunk_slots) return;
  const int my_chunks = int((nchunks - slot0 + chunk_slots - 1) / chunk_slots);
  if (my_chunks <= 0) return;

  for (int i = threadIdx.x; i < kLT * kNS * 64; i += 256)  // bitmat: [kstep][tile < MG][lane]
    afrag[i] = bitmat[(i / (kLT * 64)) * (MG * 64) + i % (kLT * 64)];
  if (!UNI)
    for (int i = threadIdx.x; i < k; i += 256) rowptr[i] = in[i];
  for (int i = threadIdx.x; i < 32; i += 256) outptr[i] = i < m ? out[i] : 0;
  if (COPY)
    for (int i = threadIdx.x; i < k; i += 256) copyptr[i] = copy[i];
  __syncthreads();

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>((lds_u8*)smem));
  lds_u8* ring = (lds_u8*)(smem + kA + kPtrBytes) + size_t(wave) * kKS * kSlotBytes;
  const uint32_t ring_base = uint32_t(reinterpret_cast<uintptr_t>(ring));
  const uint32_t ring_x = ring_base + uint32_t(4 * h * kCW + 2 * c);  // rows 4h.., column pair (2c, 2c+1)
  // block-wide fused copy: this lane stores row 4 * wave + lane / 16 of a slot, the block's columns
  // 16 * (lane % 16) .. + 15, which wave (lane % 16) / 4 DMA'd into its ring (4 rows x 256 B per
  // store instruction: 1.7x the copy bandwidth of 16 rows x 64 B, scripts/fp4_pattern_probe.hip)
  const int wrow = 4 * wave + (lane >> 4), wcol = 16 * (lane & 15);
  const uint32_t wring = uint32_t(reinterpret_cast<uintptr_t>((lds_u8*)(smem + kA + kPtrBytes))) +
                         uint32_t(((lane & 15) >> 2) * kKS * kSlotBytes + wrow * kCW + 16 * (lane & 3));
  const uint32_t a_lo = lds0 + 16u * lane, a_hi = a_lo + 65536u;
  const uint32_t optr_addr = lds0 + uint32_t(kA) + 2048u + 16u * h;  // outptr[4t + 2h + u]: + 32t + 8u
  const unsigned sslot = (blockIdx.x * 4u + unsigned(wave)) % unsigned(kFp4SinkSlots);
  const uint64_t sink = uint64_t(bitmat + size_t(MG) * kNS * 64) + uint64_t(sslot) * 1024u + 16 * lane;
  const int scale = 0x7F7F7F7F;  // E8M0 1.0 for every block of 32
  const uint64_t in0 = UNI ? in[0] : 0;
  const int drow = lane >> 2;                      // this lane's row within a DMA'd slot
  const int dcol = wave * kCW + 16 * (lane & 3);   // and its 16 columns (block-relative)
  const uint32_t rowptr_addr = lds0 + uint32_t(kA);
  const uint32_t cptr_addr = rowptr_addr + 8u * (256u + 32u);
  // (row indices pass through an empty asm at each use: hoisted out of the chunk loop, the 8 + 8
  // per-slot LDS addresses they feed were spilled to scratch at MG = 6 with copies, and every
  // reload made the compiler wait for the LDS-DMAs in flight)
  auto opaque = [](int v) __attribute__((always_inline)) {
    asm volatile("" : "+v"(v));
    return v;
  };
  auto slot_row = [&](int p) __attribute__((always_inline)) {
    const int r = kRS * p + opaque(drow);
    return r < k ? r : k - 1;
  };
  auto cbase = [&](int ci) __attribute__((always_inline)) {
    return col0 + (slot0 + int64_t(ci) * chunk_slots) * kBlockCols;
  };
  // DMA of ring slot p for chunk cn (past my chunks: chunk 0's bytes, never used); rowp: the slot
  // row's input pointer (scattered rows) read from LDS beforehand
  auto dma = [&](int cn, int p, uint64_t rowp) __attribute__((always_inline)) {
    const int64_t col = cbase(cn < my_chunks ? cn : 0) + dcol;
    const uint64_t base = UNI ? in0 + uint64_t(int64_t(slot_row(p)) * in_stride) : rowp;
    __builtin_amdgcn_global_load_lds((gptr<const void>)(base + uint64_t(col)), ring + p * kSlotBytes, 16, 0, 0);
  };
  // fused copy of ring slot p (chunk cn's bytes), block-wide (wrow, wcol); cp: the row's copy pointer
  auto copy_store = [&](int cn, int p, uint64_t cp, u32x4 v) __attribute__((always_inline)) {
    // (the address is a select, not a branch: as a divergent branch it split the last tile group into
    // basic blocks, and the compiler then moved that group's MFMAs away from the B expansion they
    // were scheduled to hide — 4x less VALU/MFMA co-execution; k128n160 1.472-1.480 -> 1.443-1.445
    // ms/step on one box, profiles/wide_stripe/r09_select)
    const uint64_t live = uint64_t(cn < my_chunks) & uint64_t(kRS * p + wrow < k) & uint64_t(cp != 0);
    const uint64_t m = 0 - live;
    uint64_t addr = ((cp + uint64_t(cbase(cn) + wcol)) & m) | (sink & ~m);
    asm volatile("" : "+v"(addr));  // (kept a select: see above)
    __builtin_nontemporal_store(v, (gptr<u32x4>)addr);
  };
  auto copy_row = [&](int p) __attribute__((always_inline)) {
    const int r = kRS * p + opaque(wrow);
    return r < k ? r : k - 1;
  };
  auto read_ptr = [&](uint64_t& v, uint32_t addr) __attribute__((always_inline)) {
    uint64_t r;
    asm volatile("ds_read_b64 %0, %1" : "=&v"(r) : "v"(addr) : "memory");
    v = r;
  };
  // rows 4h+i of K-step S (slot S / 2, half S % 2), this lane's column pair
  auto read_x = [&](uint32_t (&x)[4], auto s_tag) __attribute__((always_inline)) {
    constexpr int S = decltype(s_tag)::value;
    constexpr int off = (S / 2) * kSlotBytes + (S % 2) * 8 * kCW;
    const uint32_t addr = ring_x;
    uint32_t x0, x1, x2, x3;
    asm volatile(
        "ds_read_u16 %0, %4 offset:%5\n\t"
        "ds_read_u16 %1, %4 offset:%6\n\t"
        "ds_read_u16 %2, %4 offset:%7\n\t"
        "ds_read_u16 %3, %4 offset:%8"
        : "=&v"(x0), "=&v"(x1), "=&v"(x2), "=&v"(x3)
        : "v"(addr), "n"(off), "n"(off + 64), "n"(off + 128), "n"(off + 192)
        : "memory");
    x[0] = x0;
    x[1] = x1;
    x[2] = x2;
    x[3] = x3;
  };
  // A fragment of (tile T < kLT, K-step S) from LDS
  auto read_a = [&](i32x4& a, auto t_tag, auto s_tag) __attribute__((always_inline)) {
    static_assert(decltype(t_tag)::value < kLT, "tile 7 of 8 is register-resident");
    constexpr int off = (decltype(s_tag)::value * kLT + decltype(t_tag)::value) * 1024;
    const uint32_t base = off >= 65536 ? a_hi : a_lo;
    i32x4 v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=&v"(v) : "v"(base), "n"(off % 65536) : "memory");
    a = v;
  };
  auto read_slot = [&](u32x4& v, auto p_tag) __attribute__((always_inline)) {
    constexpr int off = decltype(p_tag)::value * kSlotBytes;
    const uint32_t addr = wring;
    u32x4 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=&v"(r) : "v"(addr), "n"(off) : "memory");
    v = r;
  };
  // output row pointers of tile T: rows 4T + 2h + u
  auto read_op = [&](uint64_t (&o)[2], auto t_tag) __attribute__((always_inline)) {
    constexpr int T = decltype(t_tag)::value;
    const uint32_t addr = optr_addr;
    uint64_t o0, o1;
    asm volatile("ds_read_b64 %0, %2 offset:%3\n\tds_read_b64 %1, %2 offset:%4"
                 : "=&v"(o0), "=&v"(o1)
                 : "v"(addr), "n"(32 * T), "n"(32 * T + 8)
                 : "memory");
    o[0] = o0;
    o[1] = o1;
  };
  // B operands of a K-step from its 4 raw ring words (gf_mfma_fp4.hip expand, kAOne order)
  auto expand = [&](i32x4 (&bo)[2], const uint32_t (&x)[4]) __attribute__((always_inline)) {
    const uint32_t p01 = x[0] | (x[1] << 16), p23 = x[2] | (x[3] << 16);
    const uint32_t w[2] = {__builtin_amdgcn_perm(p23, p01, 0x06040200u), __builtin_amdgcn_perm(p23, p01, 0x07050301u)};
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      bo[t][0] = int(w[t] & 0x11111111u);
      bo[t][1] = int(w[t] & 0x22222222u);
      bo[t][2] = int(w[t] & 0x44444444u);
      bo[t][3] = int((w[t] >> 1) & 0x44444444u);
    }
  };
  // the two output words (byte rows 2h, 2h + 1 of the tile, both N-tiles) of one accumulator tile
  auto pack = [&](uint32_t (&w)[2], const f32x16 (&a)[2]) __attribute__((always_inline)) {
    uint32_t y[2][2];
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const uint32_t v = __float_as_uint(a[n][8 * u + b]);
          y[n][u] = b == 0 ? v : bfi(1u << b, v, y[n][u]);
        }
#pragma unroll
    for (int u = 0; u < 2; ++u) w[u] = __builtin_amdgcn_perm(y[1][u], y[0][u], 0x0c0c0400u);
  };

  i32x4 Bc[kNS][2];     // B of the chunk being multiplied, resident in AGPRs
  // tile 7's A at MG = 8 (every K-step), loaded once and kept in AGPRs: its group reads it in place
  [[maybe_unused]] i32x4 A7[kNS];
  if constexpr (MG == 8) {
#pragma unroll
    for (int q = 0; q < kNS; ++q) A7[q] = bitmat[(size_t(q) * MG + 7) * 64 + lane];
#pragma unroll
    for (int q = 0; q < kNS; ++q) asm volatile("" : "+a"(A7[q]));
  }
  // whether tile T's A is register-resident (read in place, never through Acur)
  constexpr auto kRegA = [](int T) { return MG == 8 && T == 7; };
  f32x16 acc[2][2][2];  // [set][tile of the group][N-tile]
  f32x16 bias;          // start value 2^(23 - b) on output bit b = accumulator register & 7
#pragma unroll
  for (int v = 0; v < 16; ++v) bias[v] = float(1u << (23 - (v & 7)));
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 2; ++e) acc[i][e][0] = acc[i][e][1] = bias;

  // prologue: chunk 0's slots, expanded into B and copied
#pragma unroll
  for (int p = 0; p < kKS; ++p) dma(0, p, UNI ? 0 : rowptr[slot_row(p)]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (COPY) {  // chunk 0's copies, block-wide: every wave's ring has landed
    __builtin_amdgcn_s_barrier();
    static_for<kKS>([&](auto p_tag) {
      constexpr int Pp = decltype(p_tag)::value;
      u32x4 v;
      uint64_t cp;
      read_slot(v, p_tag);
      read_ptr(cp, cptr_addr + 8u * uint32_t(copy_row(Pp)));
      lgkm_wait();
      tie(v);
      tie(cp);
      copy_store(0, Pp, cp, v);
    });
    __builtin_amdgcn_s_barrier();  // (no wave refills its ring before every copy has read it)
  }
  static_for<kNS>([&](auto s_tag) {
    constexpr int S = decltype(s_tag)::value;
    uint32_t x[4];
    read_x(x, s_tag);
    lgkm_wait();
#pragma unroll
    for (int i = 0; i < 4; ++i) tie(x[i]);
    expand(Bc[S], x);
#pragma unroll
    for (int n = 0; n < 2; ++n) asm volatile("" : "+a"(Bc[S][n]));
  });
  // tile groups: pairs (2g, 2g + 1), the last one single when MG is odd
  constexpr int NG = (MG + 1) / 2;
  using I0 = std::integral_constant<int, 0>;
  i32x4 Acur[2][kQ];  // A of the current super-step: [tile of the group][K-step]
  static_for<kQ>([&](auto j) {
    read_a(Acur[0][decltype(j)::value], I0{}, j);
    read_a(Acur[1][decltype(j)::value], std::integral_constant<int, 1>{}, j);
  });
  uint64_t opc[2][2];  // output row pointers of the group packed next (the last of "chunk -1": discarded)
  read_op(opc[0], std::integral_constant<int, 2 * (NG - 1)>{});
  if constexpr (MG % 2 == 0) read_op(opc[1], std::integral_constant<int, MG - 1>{});
  lgkm_wait();
#pragma unroll
  for (int j = 0; j < kQ; ++j) {
    tie(Acur[0][j]);
    tie(Acur[1][j]);
  }
  tie(opc[0][0]);
  tie(opc[0][1]);
  if constexpr (MG % 2 == 0) {
    tie(opc[1][0]);
    tie(opc[1][1]);
  }
  uint32_t xc[kQ][4] = {};  // raw bytes of the next chunk's K-steps of this super-step (last group)

  // One chunk ci with chunk parity P (ci == my_chunks: the phantom).
  auto chunk_body = [&](int ci, auto p_tag) __attribute__((always_inline)) {
    constexpr int P = decltype(p_tag)::value;
    const bool live = ci < my_chunks;
    const int64_t colw = cbase(ci) + wave * kCW + 2 * c;  // this chunk
    const int64_t pcolw = colw - chunk_slots * kBlockCols;  // previous chunk
    static_for<NG>([&](auto g_tag) {
      constexpr int G = decltype(g_tag)::value;
      constexpr int T0 = 2 * G;
      constexpr int GS = T0 + 1 < MG ? 2 : 1;  // tiles in this group
      constexpr int PG = G == 0 ? NG - 1 : G - 1;  // the group packed during this one
      constexpr int PGS = 2 * PG + 1 < MG ? 2 : 1;
      constexpr int kSet = acc_set<NG>(P, G);
      constexpr int kPSet = G == 0 ? acc_set<NG>(P ^ 1, NG - 1) : acc_set<NG>(P, G - 1);
      static_assert(kSet != kPSet, "a group must not write the set still waiting to be packed");
      constexpr int kSS = kNS / kQ;  // super-steps per group
      static_for<kSS>([&](auto q_tag) {
        constexpr int Q = decltype(q_tag)::value;
        // ---- LDS reads for the next super-step (retired by this one's closing lgkmcnt(0))
        constexpr int NGi = Q + 1 < kSS ? G : (G + 1 < NG ? G + 1 : 0);
        constexpr int NQ = Q + 1 < kSS ? Q + 1 : 0;
        constexpr int NT0 = 2 * NGi;
        constexpr int NGS = NT0 + 1 < MG ? 2 : 1;
        i32x4 An[2][kQ];
        static_for<kQ>([&](auto j) {
          constexpr int J = decltype(j)::value;
          read_a(An[0][J], std::integral_constant<int, NT0>{}, std::integral_constant<int, kQ * NQ + J>{});
          if constexpr (NGS == 2 && !kRegA(NT0 + 1))
            read_a(An[1][J], std::integral_constant<int, NT0 + 1>{}, std::integral_constant<int, kQ * NQ + J>{});
        });
        constexpr bool kLastG = G == NG - 1;
        // the next chunk's raw bytes for the expansion in the last group, one super-step ahead
        constexpr bool kXn = (kLastG && Q + 1 < kSS) || (G == NG - 2 && Q + 1 == kSS);
        if constexpr (G == NG - 2 && Q + 1 == kSS) {
          // the next chunk's 8 DMAs (group 0) have landed: younger are the 4 epilogue stores of each
          // of groups 1 .. NG-2 (pairs; vmcnt retires in issue order)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (NG - 2)) : "memory");
        }
        uint32_t xn[kQ][4];
        if constexpr (kXn) {
          static_for<kQ>([&](auto j) {
            read_x(xn[decltype(j)::value], std::integral_constant<int, kQ * NQ + decltype(j)::value>{});
          });
        }
        // fused copy of the next chunk's slot Q (last group, block-wide: the first super-step waits
        // at a barrier until every wave's DMAs have landed), and group 0's DMA row pointer
        [[maybe_unused]] u32x4 cd;
        [[maybe_unused]] uint64_t cpp = 0, rpp = 0;
        if constexpr (COPY && kLastG) {
          if constexpr (Q == 0) __builtin_amdgcn_s_barrier();
          read_slot(cd, q_tag);
          read_ptr(cpp, cptr_addr + 8u * uint32_t(copy_row(Q)));
        }
        if constexpr (!UNI && G == 0) read_ptr(rpp, rowptr_addr + 8u * uint32_t(slot_row(Q)));
        uint64_t opn[2][2];
        if constexpr (Q + 1 == kSS) {  // this group's output pointers: it is packed during the next
          read_op(opn[0], std::integral_constant<int, T0>{});
          if constexpr (GS == 2) read_op(opn[1], std::integral_constant<int, T0 + 1>{});
        }
        __builtin_amdgcn_sched_barrier(0);

        // ---- kQ K-steps x GS tiles x 2 N-tiles from the resident B (GS x 2 independent chains)
        static_for<kQ>([&](auto j_tag) {
          constexpr int J = decltype(j_tag)::value;
          constexpr int S = kQ * Q + J;
#pragma unroll
          for (int e = 0; e < GS; ++e) {
            const i32x4& af = kRegA(T0 + e) ? A7[S] : Acur[e][J];
            const i32x8 a = {af[0], af[1], af[2], af[3], 0, 0, 0, 0};
#pragma unroll
            for (int n = 0; n < 2; ++n) {
              const i32x8 bb = {Bc[S][n][0], Bc[S][n][1], Bc[S][n][2], Bc[S][n][3], 0, 0, 0, 0};
              acc[kSet][e][n] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
                  a, bb, S == 0 ? bias : acc[kSet][e][n], 4, 4, 0, scale, 0, scale);
            }
          }
        });
        // ---- VALU under the MFMAs: the next chunk's B (last group), the previous group's epilogue
        if constexpr (kLastG) {
          static_for<kQ>([&](auto j_tag) {
            constexpr int J = decltype(j_tag)::value;
            expand(Bc[kQ * Q + J], xc[J]);
#pragma unroll
            for (int n = 0; n < 2; ++n) asm volatile("" : "+a"(Bc[kQ * Q + J][n]));
          });
        }
        [[maybe_unused]] uint32_t w[2][2];
        if constexpr (Q == 0) {
          pack(w[0], acc[kPSet][0]);
          if constexpr (PGS == 2) pack(w[1], acc[kPSet][1]);
        }
        constexpr int kMfma = kQ * GS * 2;
        constexpr int kValu = (kLastG ? kQ * 22 : 0) + (Q == 0 ? 30 * PGS : 0);  // (22: 14 + 8 AGPR writes)
        constexpr int kPer = (kValu + kMfma - 1) / kMfma;
#pragma unroll
        for (int i = 0; i < kMfma; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);     // MFMA
          __builtin_amdgcn_sched_group_barrier(0x002, kPer, 0);  // VALU
        }
        __builtin_amdgcn_sched_barrier(0);

        // ---- stores
        if constexpr (Q == 0) {
          // (group 0 packs the previous chunk's last group; the phantom's own groups go to the sink)
          const bool plive = G == 0 ? ci > 0 : live;
          const int64_t pc = G == 0 ? pcolw : colw;
#pragma unroll
          for (int e = 0; e < PGS; ++e)
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              const uint64_t o = opc[e][u];
              *(gptr<uint16_t>)(plive && o ? o + uint64_t(pc) : sink) = uint16_t(w[e][u]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        lgkm_wait();
#pragma unroll
        for (int j = 0; j < kQ; ++j) {
          tie(An[0][j]);
          Acur[0][j] = An[0][j];
          if constexpr (NGS == 2 && !kRegA(NT0 + 1)) {
            tie(An[1][j]);
            Acur[1][j] = An[1][j];
          }
        }
        if constexpr (kXn) {
#pragma unroll
          for (int j = 0; j < kQ; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              tie(xn[j][i]);
              xc[j][i] = xn[j][i];
            }
        }
        if constexpr (Q + 1 == kSS) {
#pragma unroll
          for (int e = 0; e < GS; ++e) {
            tie(opn[e][0]);
            tie(opn[e][1]);
            opc[e][0] = opn[e][0];
            opc[e][1] = opn[e][1];
          }
        }
        if constexpr (COPY && kLastG) {
          tie(cd);
          tie(cpp);
          copy_store(ci + 1, Q, cpp, cd);
          // every wave has read its copies out of the rings before any refills them (group 0)
          if constexpr (Q + 1 == kSS) __builtin_amdgcn_s_barrier();
        }
        // group 0: the next chunk's DMA of slot Q (its bytes were expanded and copied in the
        // previous chunk's last group)
        if constexpr (G == 0) {
          if constexpr (!UNI) tie(rpp);
          dma(ci + 1, Q, rpp);
        }
      });
    });
  };

  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  // chunk pairs; with an odd count the last pair's second chunk is the phantom, whose first group
  // packs the last real chunk's last group
  int ci = 0;
  for (; ci < my_chunks; ci += 2) {
    chunk_body(ci, P0{});
    chunk_body(ci + 1, P1{});
  }
  if (ci == my_chunks) {
    // an even count: pack the last real chunk's last group here (parity 1)
    constexpr int kLast = acc_set<NG>(1, NG - 1);
    const int64_t pcolw = cbase(ci - 1) + wave * kCW + 2 * c;
    constexpr int LGS = 2 * (NG - 1) + 1 < MG ? 2 : 1;
#pragma unroll
    for (int e = 0; e < LGS; ++e) {
      uint32_t w[2];
      pack(w, acc[kLast][e]);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint64_t o = opc[e][u];
        *(gptr<uint16_t>)(o ? o + uint64_t(pcolw) : sink) = uint16_t(w[u]);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA (dummy or not) outlives the wave
}

template <int MG, bool UNI, bool COPY>
hipError_t launch_tm(const Fp4ArLaunch& a, int64_t* done, hipStream_t stream) {
  const void* f = reinterpret_cast<const void*>(&gf_gemm_fp4tm_kernel<MG, UNI, COPY>);
  const size_t lds = size_t(MG < 8 ? MG : 7) * kNS * 1024 + kPtrBytes + size_t(4) * kKS * kSlotBytes;
  if (lds > 160 * 1024) return hipErrorInvalidConfiguration;
  hipError_t e = ensure_lds_optin(f, int(lds));
  if (e != hipSuccess) return e;
  static DeviceMemo<int, int> occ_memo;
  const int occ = occ_memo.get_or(0, [&] {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, f, 256, lds) != hipSuccess) o = 0;
    return o;
  });
  if (occ <= 0) return hipErrorInvalidConfiguration;
  const int64_t nchunks = a.ncols / kBlockCols;
  *done = nchunks * kBlockCols;
  if (nchunks == 0) return hipSuccess;
  const int64_t slots = persistent_slots(occ, 1, nchunks);
  gf_gemm_fp4tm_kernel<MG, UNI, COPY><<<unsigned(slots), 256, lds, stream>>>(
      (cptr<uint64_t>)a.in, (cptr<uint64_t>)a.out, (cptr<uint64_t>)a.copy, static_cast<const i32x4*>(a.bitmat), a.k,
      a.m, a.col0, nchunks, slots, a.in_stride);
  return hipGetLastError();
}

template <int MG>
hipError_t launch_tm_var(const Fp4ArLaunch& a, int64_t* done, hipStream_t stream) {
  if (a.copy) return launch_tm<MG, false, true>(a, done, stream);
  return a.in_stride ? launch_tm<MG, true, false>(a, done, stream) : launch_tm<MG, false, false>(a, done, stream);
}

}  // namespace

bool fp4tm_supported(int k, int mg, bool copies) {
  (void)copies;
  return k > 112 && k <= 128 && mg >= 5 && mg <= 8;
}

hipError_t launch_gf_gemm_fp4tm(const Fp4ArLaunch& a, int64_t* done, hipStream_t stream) {
  *done = 0;
  if (!fp4tm_supported(a.k, a.mg, a.copy != nullptr) || a.m > 4 * a.mg || a.ncols < 0 || (a.col0 & 1) ||
      a.batch != 1)
    return hipErrorInvalidValue;
  switch (a.mg) {
    case 5: return launch_tm_var<5>(a, done, stream);
    case 6: return launch_tm_var<6>(a, done, stream);
    case 7: return launch_tm_var<7>(a, done, stream);
    default: return launch_tm_var<8>(a, done, stream);
  }
}

}  // namespace gfrs

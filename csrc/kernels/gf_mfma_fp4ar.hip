// GF(2^8) GEMM on gfx950 matrix cores, FP4 bit-matrix form — A-RESIDENT variant ("ar").
//
// Same algebra, bit-matrix layout, B expansion and biased-float parity epilogue as
// gf_mfma_fp4.hip (read its header first); what changes is where the operands live. The LDS
// kernels there keep the whole coefficient bit-matrix (128 KiB at k=128, p=32) in LDS and their
// 256 accumulators in AGPRs. Measured on the k=128, p=32 encode (profiles/wide_stripe/r02_fp4_ablate), that
// costs per MFMA: one v_accvgpr_read per accumulator in the epilogue, half an A-fragment
// ds_read_b128, and a bias MFMA per accumulator tile per chunk — 4.05 VALU per MFMA, the issue
// slots of the 32-cycle MFMA nearly full, and a power-capped clock (the kernel is clock-bound:
// dropping the epilogue VALU alone cut cycles 7 % and raised the clock 6 %).
//
// Here each wave holds its share of A in REGISTERS for the whole kernel: the block's 4 waves split
// the output rows into WPG halves (WPG = 2 for p = 32: 4 M-tiles of 32 bit-rows per wave) and
// the columns into 4 / WPG groups of 64. A wave's 4 tiles x 16 K-steps of A are 64 fragments of
// 16 B = 256 registers — exactly the AGPR file, which the scaled MFMA reads as its A operand. The
// accumulators move to ARCH VGPRs (this file is compiled with -amdgpu-mfma-vgpr-form), so:
//   * the parity epilogue's v_bfi reads the accumulators directly (no accvgpr reads);
//   * the bias (2^(23-b) start value, gf_mfma_fp4.hip bias_scale_of_lane) is the C operand of a
//     tile's first MFMA of each chunk — a constant 16-VGPR block, no extra MFMA;
//   * no A traffic through LDS at all; LDS holds only the per-wave input rings.
// Cost: B is expanded for 4 M-tiles instead of 8 (14 VALU per 8 MFMAs instead of per 16), and the
// two waves of a column group both DMA the same input bytes (the second is an L2 hit).
// Net per MFMA: ~2.7 VALU, no LDS A reads, 6 % fewer MFMAs.
//
// Schedule (as the sk kernel of gf_mfma_fp4.hip): tile t of a wave runs its K loop t K-steps
// behind tile 0, so tile j finishes its chunk at step j-1 and is packed, stored and restarted in
// step j, between the other tiles' MFMAs; B of K-step s is kept for the window of WN steps its
// tiles need. Every ring slot, DMA cursor, wait count and window index is a compile-time
// constant; a phantom chunk drains the last real one.
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
constexpr int kKS = 8;            // ring slots per chunk (2 K-steps each)
constexpr int kRS = 16;           // input rows per ring slot
constexpr int kPtrBytes = 8 * (256 + 32 + 256);  // LDS: row, output-row and copy pointer tables

__device__ __forceinline__ uint32_t bfi(uint32_t mask, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(mask), "v"(a), "v"(b));
  return r;
}
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

__host__ __device__ constexpr int ar_mod(int a, int n) { return ((a % n) + n) % n; }
// epilogue stores (2 ushort per packed tile) in chunk-relative steps [s0, s1)
__host__ __device__ constexpr int ar_stores_in(int s0, int s1, int mgw) {
  int n = 0;
  for (int s = s0; s < s1; ++s) n += ar_mod(s, kNS) < mgw ? 2 : 0;
  return n;
}
// vm ops younger than DMA(sp+1) at its wait (first step of slot sp): R-2 DMAs, the copy stores of
// slots sp+1-R .. sp-1, the epilogue stores of steps [2 (sp+1-R) + 1, 2 sp). The prologue issues
// the stores of the virtual slots of chunk -1 as dummies, so the count is exact from slot 0.
__host__ __device__ constexpr int ar_wait_count(int sp, int mgw, int r, bool copy) {
  const int n = (r - 2) + (copy ? r - 1 : 0) + ar_stores_in(2 * (sp + 1 - r) + 1, 2 * sp, mgw);
  return n < 63 ? n : 63;
}

// MGW: M-tiles (of 4 output rows = 32 bit-rows) per wave; WPG: waves per column group (the row
// split); UNI: input row j at in[0] + j * in_stride (else row pointers from LDS); COPY: fused
// survivor copy (input row j also written to copy[j], from the ring slot the DMA filled; with two
// row halves each wave of a column group stores half of every slot's rows — measured worse: one
// wave storing everything while its partner parked its stores on the shared sink lines (every CU
// serialised on them, 1100 vs 880 us at m = 24), or both storing everything (non-temporal: both
// reach HBM, 1320 us)); R: ring slots per wave (divides the 8-slot chunk).
// BATCH: nchunks counts the chunks of `batch` stripes laid out at fixed strides (cps chunks each):
// global chunk g is chunk g % cps of stripe g / cps, whose rows are stripe 0's (the pointer tables)
// plus (g / cps) * in_bstride (inputs) / out_bstride (outputs and copies) — one persistent grid,
// one A load per wave, for a whole batch of small objects (serving).
template <int MGW, int WPG, bool UNI, bool COPY, int R, bool BATCH = false>
__global__ __launch_bounds__(256, 1) void gf_gemm_fp4ar_kernel(cptr<uint64_t> in, cptr<uint64_t> out,
                                                               cptr<uint64_t> copy, const i32x4* __restrict__ bitmat,
                                                               int k, int m, int mg, int64_t col0, int64_t nchunks,
                                                               int64_t chunk_slots, int64_t in_stride,
                                                               int64_t cps, int64_t in_bstride,
                                                               int64_t out_bstride) {
  constexpr int CG = 4 / WPG;               // column groups per block
  constexpr int kBC = CG * kCW;             // block columns per chunk
  constexpr int WN = MGW == 3 ? 4 : MGW;    // B window (a power of two dividing kNS, >= MGW)
  static_assert(kKS % R == 0 && R >= 3, "ring depth must divide the chunk");
  static_assert(WPG == 1 || WPG == 2, "one or two row halves");
  static_assert(MGW >= 1 && MGW <= 4 && MGW * WPG <= 8, "at most 4 M-tiles per wave (the AGPR file)");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint64_t* rowptr = reinterpret_cast<uint64_t*>(smem);
  uint64_t* outptr = rowptr + 256;
  uint64_t* copyptr = outptr + 32;
  const int bid = blockIdx.x;
  const int64_t slot0 = int64_t(bid >> 3) * 8 + (bid & 7);  // slot -> one XCD (blocks round-robin)
  if (slot0 >= chunk_slots) return;
  const int my_chunks = int((nchunks - slot0 + chunk_slots - 1) / chunk_slots);
  if (my_chunks <= 0) return;

  if (!UNI)
    for (int i = threadIdx.x; i < k; i += 256) rowptr[i] = in[i];
  for (int i = threadIdx.x; i < 32; i += 256) outptr[i] = i < m ? out[i] : 0;
  if (COPY)
    for (int i = threadIdx.x; i < k; i += 256) copyptr[i] = copy[i];
  __syncthreads();

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  const int mh = wave % WPG, cg = wave / WPG;
  const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>((lds_u8*)smem));
  lds_u8* rings = (lds_u8*)(smem + kPtrBytes);
  lds_u8* ring = rings + size_t(wave) * R * kSlotBytes;
  lds_u8* spare = rings + size_t(4) * R * kSlotBytes;
  const uint32_t ring_x = uint32_t(reinterpret_cast<uintptr_t>(ring)) + uint32_t(4 * h * kCW + 2 * c);
  // fused copy: the WPG waves of a column group split each slot's rows (16 / WPG rows per wave,
  // 16 B per lane for one wave, 8 B for two), every byte stored once
  constexpr int kCB = 16 / WPG;                                   // copy bytes per lane
  const int crow0 = (16 / WPG) * mh + lane / (4 * WPG);           // copy row within a slot
  const int ccol = kCB * (lane % (4 * WPG));                      // copy column within the wave's 64
  const uint32_t ring_lane = uint32_t(reinterpret_cast<uintptr_t>(ring)) + uint32_t(crow0 * kCW + ccol);
  // outptr[4 (mh MGW + e) + 2h + u] at + 32e + 8u
  const uint32_t optr_addr = lds0 + 8u * 256u + uint32_t(32 * mh * MGW + 16 * h);
  const uint32_t rowptr_addr = lds0;
  const uint32_t cptr_addr = lds0 + 8u * (256u + 32u);
  // this wave's 1-KiB slot of the sink past the bit-matrix (kFp4SinkSlots, kernels.h)
  const unsigned sslot = (blockIdx.x * 4u + unsigned(wave)) % unsigned(kFp4SinkSlots);
  const uint64_t sink = uint64_t(bitmat + size_t(mg) * kNS * 64) + uint64_t(sslot) * 1024u + 16 * lane;
  const int scale = 0x7F7F7F7F;  // E8M0 1.0 for every block of 32
  const uint64_t in0 = UNI ? in[0] : 0;
  const int drow = lane >> 2;                      // this lane's row within a DMA'd slot
  const int dcol = cg * kCW + 16 * (lane & 3);    // and its 16 columns (block-relative)
  auto dma_row = [&](int p) __attribute__((always_inline)) { return kRS * p + drow < k ? kRS * p + drow : k - 1; };

  // A of this wave's tiles, resident in AGPRs for the whole kernel. All 64 loads are unconditional
  // and issued before the first register tie: a conditional load (tiles past mg read zero) tied
  // right after it made every load wait for the one before — 64 serialised L2 round trips per block
  // (batched RS(128,160) encode of 16 x 64 KiB 18.0 -> 12.5-13.1 us, profiles/wide_stripe/r09_select).
  // A padding tile (past mg) now reads the last real tile's A: its rows have no output pointer, so
  // whatever it accumulates goes to the sink.
  i32x4 A[MGW][kNS];
  static_for<MGW>([&](auto t_tag) {
    constexpr int T = decltype(t_tag)::value;
    const int mt = min(mh * MGW + T, mg - 1);
    static_for<kNS>([&](auto s_tag) {
      constexpr int S = decltype(s_tag)::value;
      A[T][S] = bitmat[(size_t(S) * mg + mt) * 64 + lane];
    });
  });
#pragma unroll
  for (int t = 0; t < MGW; ++t)
#pragma unroll
    for (int q = 0; q < kNS; ++q) asm volatile("" : "+a"(A[t][q]));
  // accumulator start value: 2^(23 - b) on output bit b = accumulator register & 7
  f32x16 bias;
#pragma unroll
  for (int v = 0; v < 16; ++v) bias[v] = float(1u << (23 - (v & 7)));

  uint64_t pn = UNI ? 0 : rowptr[dma_row(R % kKS)];
  // Byte offsets of this block's chunk ci from column col0 of stripe 0's rows, inputs and outputs
  // (plain: the global chunk's columns; BATCH: its stripe's offset plus its columns there). Rolled
  // once per chunk (prev / cur / next), so a batched launch divides once per chunk.
  struct Off {
    int64_t in, out;
  };
  auto chunk_off = [&](int ci) __attribute__((always_inline)) {
    const int64_t gc = slot0 + int64_t(ci) * chunk_slots;
    if constexpr (BATCH) {
      const int64_t b = int64_t(uint32_t(gc) / uint32_t(cps));  // (gc, cps < 2^31: host-checked)
      const int64_t lc = (gc - b * cps) * kBC;
      return Off{b * in_bstride + lc, b * out_bstride + lc};
    } else {
      return Off{gc * kBC, gc * kBC};
    }
  };
  const Off off_first = chunk_off(0);
  Off off_prev = off_first, off_cur = off_first, off_nxt = chunk_off(1);
  // DMA of slot T of chunk ci + T / kKS (T / kKS: 0 = cur, 1 = next; past my_chunks: chunk 0 into
  // the spare slot)
  auto dma_issue = [&](int ci, auto t_tag, uint64_t rowp) __attribute__((always_inline)) {
    constexpr int T = decltype(t_tag)::value;
    constexpr int p = T % kKS, ring_slot = T % R;
    static_assert(T / kKS <= 1, "a DMA runs at most one chunk ahead");
    const int chunk = ci + T / kKS;
    const bool live = chunk < my_chunks;
    const int64_t col = col0 + (live ? (T / kKS ? off_nxt.in : off_cur.in) : off_first.in) + dcol;
    uint64_t sa;
    if constexpr (UNI)
      sa = in0 + uint64_t(int64_t(dma_row(p)) * in_stride + col);
    else
      sa = rowp + uint64_t(col);
    __builtin_amdgcn_global_load_lds((gptr<const void>)sa, live ? ring + ring_slot * kSlotBytes : spare, 16, 0, 0);
  };
  auto read_x = [&](uint32_t (&x)[4], auto sl_tag, auto hs_tag) __attribute__((always_inline)) {
    constexpr int off = decltype(sl_tag)::value * kSlotBytes + decltype(hs_tag)::value * 8 * kCW;
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
  constexpr int kExpandValu = 14;
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

  f32x16 acc[MGW][2];
  i32x4 bw[WN][2];  // B of K-step s in bw[s % WN]
#pragma unroll
  for (int t = 0; t < MGW; ++t) acc[t][0] = acc[t][1] = bias;

  // prologue: R slots in flight, with the stores their steady-state position has as dummies
  static_for<R>([&](auto t) {
    constexpr int T = decltype(t)::value;
    dma_issue(0, t, UNI ? 0 : rowptr[dma_row(T % kKS)]);
    constexpr int v = kKS + T - R;  // the virtual slot of chunk -1 issuing it
    constexpr int n_epi = ar_stores_in(2 * v + 1, 2 * v + 2, MGW) + (T + 1 < R ? ar_stores_in(2 * v + 2, 2 * v + 3, MGW) : 0);
    const uint64_t sk = sink;
    if constexpr (COPY) {
      if constexpr (WPG == 1) {
        const u32x4 zero = {0u, 0u, 0u, 0u};
        asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(sk), "v"(zero) : "memory");
      } else {
        const uint64_t zero = 0;
        asm volatile("global_store_dwordx2 %0, %1, off nt" ::"v"(sk), "v"(zero) : "memory");
      }
    }
#pragma unroll
    for (int i = 0; i < n_epi; ++i) asm volatile("global_store_short %0, %1, off" ::"v"(sk), "v"(0) : "memory");
  });
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(R - 1) : "memory");
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  uint32_t x0[4], x1[4], x2[4];  // raw bytes: x1 = step s+1 (in registers), x2 = step s+2 (in flight)
  read_x(x0, I0{}, I0{});
  read_x(x1, I0{}, I1{});
  uint64_t opc[2] = {0, 0};  // output row pointers of the tile packed at the next step
  {
    const uint32_t addr = optr_addr;
    uint64_t o0, o1;
    asm volatile("ds_read_b64 %0, %2\n\tds_read_b64 %1, %2 offset:8" : "=&v"(o0), "=&v"(o1) : "v"(addr) : "memory");
    lgkm_wait();
    tie(o0);
    tie(o1);
    opc[0] = o0;
    opc[1] = o1;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    tie(x0[i]);
    tie(x1[i]);
  }
#pragma unroll
  for (int s = 1; s < WN; ++s) bw[s][0] = bw[s][1] = i32x4{0, 0, 0, 0};  // K-steps of chunk -1: discarded
  expand(bw[0], x0);

  auto chunk_body = [&](int ci) __attribute__((always_inline)) {
    const bool live = ci < my_chunks;
    const int64_t cbase = col0 + off_cur.out;  // this chunk's output columns (copies)
    const bool plive = ci > 0;  // packs of "chunk -1" go to the sink
    const int64_t pcolw = col0 + off_prev.out + cg * kCW + 2 * c;
    using cvec = std::conditional_t<WPG == 1, u32x4, unsigned __attribute__((ext_vector_type(2)))>;
    [[maybe_unused]] cvec cdat;
    [[maybe_unused]] uint64_t cp = 0;
    static_for<kKS>([&](auto sp_tag) {
      constexpr int SP = decltype(sp_tag)::value;
      constexpr int RS = SP % R, RS1 = (SP + 1) % R;
      [[maybe_unused]] const int crow = kRS * SP + crow0;
      static_for<2>([&](auto jj_tag) {
        constexpr int JJ = decltype(jj_tag)::value;
        constexpr int J = SP * 2 + JJ;                              // step of the chunk
        constexpr int EP = J < MGW ? J : -1;                        // tile packed and restarted now
        constexpr int EN = (J + 1) % kNS < MGW ? (J + 1) % kNS : -1;  // tile packed at the next step
        // tile T works on K-step (J - T) mod 16; its first (bias) MFMA of a chunk is at J == T
        auto mfma_tile = [&](auto t_tag) __attribute__((always_inline)) {
          constexpr int T = decltype(t_tag)::value;
          constexpr int S = ar_mod(J - T, kNS);
          const i32x8 a = {A[T][S][0], A[T][S][1], A[T][S][2], A[T][S][3], 0, 0, 0, 0};
#pragma unroll
          for (int n = 0; n < 2; ++n) {
            const i32x8 bb = {bw[S % WN][n][0], bw[S % WN][n][1], bw[S % WN][n][2], bw[S % WN][n][3], 0, 0, 0, 0};
            acc[T][n] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, bb, S == 0 ? bias : acc[T][n], 4, 4, 0,
                                                                         scale, 0, scale);
          }
        };
        // the tile finishing its chunk now goes first (complete when packed next step)
        constexpr int EE = EN;
        constexpr int kFirst = EE >= 0 && EE != EP ? EE : (EP == 0 ? (MGW > 1 ? 1 : -1) : 0);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (kFirst >= 0) mfma_tile(std::integral_constant<int, (kFirst >= 0 ? kFirst : 0)>{});
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (JJ == 0)  // slot SP+1 has landed: exact count of the younger vm ops
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ar_wait_count(SP, MGW, R, COPY)) : "memory");
        read_x(x2, std::integral_constant<int, RS1>{}, jj_tag);
        [[maybe_unused]] uint64_t opn[2];
        if constexpr (EN >= 0) {
          const uint32_t addr = optr_addr;
          uint64_t o0, o1;
          asm volatile("ds_read_b64 %0, %2 offset:%3\n\tds_read_b64 %1, %2 offset:%4"
                       : "=&v"(o0), "=&v"(o1)
                       : "v"(addr), "n"(32 * (EN >= 0 ? EN : 0)), "n"(32 * (EN >= 0 ? EN : 0) + 8)
                       : "memory");
          opn[0] = o0;
          opn[1] = o1;
        }
        if constexpr (JJ == 1) {  // this slot is consumed: refill its ring slot R ahead
          dma_issue(ci, std::integral_constant<int, SP + R>{}, pn);
          if constexpr (!UNI) {
            const uint32_t addr = rowptr_addr + 8u * uint32_t(dma_row((SP + 1 + R) % kKS));
            uint64_t v;
            asm volatile("ds_read_b64 %0, %1" : "=&v"(v) : "v"(addr) : "memory");
            pn = v;
          }
        }
        if constexpr (JJ == 0 && COPY) {  // this lane's 16 B of the current slot and its copy pointer
          const uint32_t addr = ring_lane + uint32_t(RS * kSlotBytes);
          const uint32_t caddr = cptr_addr + 8u * uint32_t(crow < k ? crow : k - 1);
          cvec v;
          uint64_t cv;
          if constexpr (WPG == 1)
            asm volatile("ds_read_b128 %0, %1" : "=&v"(v) : "v"(addr) : "memory");
          else
            asm volatile("ds_read_b64 %0, %1" : "=&v"(v) : "v"(addr) : "memory");
          asm volatile("ds_read_b64 %0, %1" : "=&v"(cv) : "v"(caddr) : "memory");
          cdat = v;
          cp = cv;
        }
        __builtin_amdgcn_sched_barrier(0);
        // the other tiles, descending (tile WN-1 reads the window slot the expansion refills)
        static_for<MGW>([&](auto t) {
          constexpr int T = MGW - 1 - decltype(t)::value;
          if constexpr (T != kFirst && T != EP) mfma_tile(std::integral_constant<int, T>{});
        });
        [[maybe_unused]] uint32_t w[2];
        if constexpr (EP >= 0) {
          constexpr int E = EP >= 0 ? EP : 0;
          // output bytes of tile E: 7 v_bfi per byte straight from the accumulator VGPRs
          uint32_t y[2][2];
#pragma unroll
          for (int b = 0; b < 8; ++b)
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
              for (int u = 0; u < 2; ++u) {
                const uint32_t v = __float_as_uint(acc[E][n][8 * u + b]);
                y[n][u] = b == 0 ? v : bfi(1u << b, v, y[n][u]);
              }
#pragma unroll
          for (int u = 0; u < 2; ++u) w[u] = __builtin_amdgcn_perm(y[1][u], y[0][u], 0x0c0c0400u);
          mfma_tile(std::integral_constant<int, E>{});  // K-step 0 of the new chunk, from the bias
        }
        expand(bw[(J + 1) % WN], x1);  // B of the next K-step
        constexpr int kMfma = 2 * MGW - (kFirst >= 0 ? 2 : 0);
        constexpr int kValu = kExpandValu + (EP >= 0 ? 2 * 2 * 7 + 2 : 0);
        if constexpr (kMfma > 0) {
#pragma unroll
          for (int i = 0; i < kMfma; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                            // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, (kValu + kMfma - 1) / kMfma, 0);  // VALU
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (EP >= 0) {
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const uint64_t o = opc[u];
            *(gptr<uint16_t>)(plive && o ? o + uint64_t(pcolw) : sink) = uint16_t(w[u]);
          }
        }
        if constexpr (COPY && JJ == 1) {
          __builtin_nontemporal_store(
              cdat, (gptr<cvec>)(live && crow < k && cp ? cp + uint64_t(cbase + cg * kCW + ccol) : sink));
        }
        __builtin_amdgcn_sched_barrier(0);
        lgkm_wait();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          tie(x2[i]);
          x1[i] = x2[i];
        }
        if constexpr (EN >= 0) {
          uint64_t o0 = opn[0], o1 = opn[1];
          tie(o0);
          tie(o1);
          opc[0] = o0;
          opc[1] = o1;
        }
        if constexpr (JJ == 1 && !UNI) {
          uint64_t v = pn;
          tie(v);
          pn = v;
        }
        if constexpr (JJ == 0 && COPY) {
          cvec d = cdat;
          uint64_t cv = cp;
          tie(d);
          tie(cv);
          cdat = d;
          cp = cv;
        }
      });
    });
  };

  for (int ci = 0; ci <= my_chunks; ++ci) {
    chunk_body(ci);
    off_prev = off_cur;
    off_cur = off_nxt;
    off_nxt = chunk_off(ci + 2);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA (dummy or not) outlives the wave
}

constexpr size_t ar_lds(int r) { return size_t(kPtrBytes) + (4 * size_t(r) + 1) * kSlotBytes; }

template <int MGW, int WPG, bool UNI, bool COPY, int R, bool BATCH>
hipError_t launch_ar(const Fp4ArLaunch& a, int64_t* done, hipStream_t stream) {
  constexpr int kBC = (4 / WPG) * kCW;
  const void* f = reinterpret_cast<const void*>(&gf_gemm_fp4ar_kernel<MGW, WPG, UNI, COPY, R, BATCH>);
  const size_t lds = ar_lds(R);
  hipError_t e = ensure_lds_optin(f, int(lds));
  if (e != hipSuccess) return e;
  static DeviceMemo<int, int> occ_memo;
  const int occ = occ_memo.get_or(0, [&] {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, f, 256, lds) != hipSuccess) o = 0;
    return o;
  });
  if (occ <= 0) return hipErrorInvalidConfiguration;
  const int64_t cps = a.ncols / kBC;  // chunks per stripe
  const int64_t nchunks = cps * std::max(1, a.batch);
  *done = cps * kBC;
  if (nchunks == 0) return hipSuccess;
  if (BATCH && nchunks >= (int64_t(1) << 31)) return hipErrorInvalidValue;
  const int64_t slots = persistent_slots(occ, 1, nchunks);
  gf_gemm_fp4ar_kernel<MGW, WPG, UNI, COPY, R, BATCH><<<unsigned(slots), 256, lds, stream>>>(
      (cptr<uint64_t>)a.in, (cptr<uint64_t>)a.out, (cptr<uint64_t>)a.copy, static_cast<const i32x4*>(a.bitmat), a.k,
      a.m, a.mg, a.col0, nchunks, slots, a.in_stride, cps, a.in_bstride, a.out_bstride);
  return hipGetLastError();
}

template <int MGW, int WPG, bool BATCH>
hipError_t launch_ar_var(const Fp4ArLaunch& a, int64_t* done, hipStream_t stream) {
  constexpr int R = 8;
  if (a.copy) return launch_ar<MGW, WPG, false, true, R, BATCH>(a, done, stream);
  return a.in_stride ? launch_ar<MGW, WPG, true, false, R, BATCH>(a, done, stream)
                     : launch_ar<MGW, WPG, false, false, R, BATCH>(a, done, stream);
}

template <int MGW, int WPG>
hipError_t launch_ar_b(const Fp4ArLaunch& a, int64_t* done, hipStream_t stream) {
  return a.batch > 1 ? launch_ar_var<MGW, WPG, true>(a, done, stream) : launch_ar_var<MGW, WPG, false>(a, done, stream);
}

}  // namespace

bool fp4ar_supported(int k, int mg) { return k > 112 && k <= 128 && mg >= 1 && mg <= 8; }

hipError_t launch_gf_gemm_fp4ar(const Fp4ArLaunch& a, int64_t* done, hipStream_t stream) {
  *done = 0;
  if (!fp4ar_supported(a.k, a.mg) || a.m > 4 * a.mg || a.ncols < 0 || (a.col0 & 1)) return hipErrorInvalidValue;
  // rows split in two halves of at most 4 tiles when more than 4 tiles (padding tiles reuse the last
  // tile's A and store to the sink), else one wave covers every tile and the block 4 column groups
  switch (a.mg) {
    case 1: return launch_ar_b<1, 1>(a, done, stream);
    case 2: return launch_ar_b<2, 1>(a, done, stream);
    case 3: return launch_ar_b<3, 1>(a, done, stream);
    case 4: return launch_ar_b<4, 1>(a, done, stream);
    case 5:
    case 6: return launch_ar_b<3, 2>(a, done, stream);
    default: return launch_ar_b<4, 2>(a, done, stream);
  }
}

}  // namespace gfrs

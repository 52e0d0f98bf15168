// GF(2^8) GEMM on gfx950 matrix cores, FP4 (e2m1) form of the GF(2) bit-matrix product.
//
// Same algebra as gf_mfma.hip (out_bits = A . in_bits mod 2 over the (8m x 8k) bit-matrix), but on
// `v_mfma_scale_f32_32x32x64_f8f6f4` with FP4 operands: {0, 1.0} are exact e2m1 codes (0x0, 0x2),
// the f32 accumulator holds the exact integer count (<= 8k <= 2048), and its parity is the GF(2)
// result. Why FP4 and not i8 (measured, profiles/r01_pmc):
//   * rate: the scaled FP4 MFMA does 64 K per 32 cycles — twice the i8 32x32x32 rate;
//   * size: an A fragment is 32 nibbles (16 B) per lane, so the k=128, p=32 coefficient bit-matrix
//     is 128 KiB and ALL of its M-tiles fit in one CU's LDS: each input byte is loaded and
//     bit-expanded once per block instead of once per M-group (the i8 kernel re-expanded every
//     byte 4x and was VALU-bound: 87 VALU per 8 MFMA, PMC in profiles/).
// Per wave and K-step (8 input rows = 64 K bits): 2 N-tiles (64 interleaved columns: tile t holds
// columns 2c + t, so one ushort load / store serves both), MG M-tiles (MG <= 8) from LDS,
// 2 x MG MFMAs. The order of the 64 K bits inside a step is free (the bit-matrix is built to
// match), so it is the one that is cheapest to expand: a lane's 4 rows of one column are gathered
// into one dword W (one shift-or + one v_perm per tile), and B dword q is bit plane q of W masked
// in place (kAOne below) — 1-2 VALU per B dword, 14 per K-step for 16 MFMAs (26 with one v_perm
// pool lookup per dword, ~56 with one expansion per input byte).
// Output bits are placed on MFMA rows exactly as in gf_mfma.hip so every lane owns whole bytes;
// each accumulator starts at a bias that puts the parity of its f32 count on its output bit (see
// bias_scale_of_lane).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <utility>

#include "gfrs/desc.h"
#include "gfrs/device_cache.h"
#include "gfrs/kernels.h"
#include "gfrs/tune.h"

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

constexpr int kNTW = 2;        // N-tiles per wave (64 columns)
constexpr int kBlockCols = 256;  // 4 waves x 64 columns
constexpr int kMaxLdsKiB = 137;  // A slice; + 2.25 KiB row/out pointers + 4 waves x 5 x 1 KiB rings <= 160 KiB

__constant__ Tables d_tab = make_tables();

__device__ __forceinline__ uint8_t dmul(uint8_t a, uint8_t b) { return d_tab.exp[d_tab.log[a] + d_tab.log[b]]; }
__host__ __device__ constexpr int out_row_of(int r) { return 2 * ((r >> 2) & 1) + (r >> 4); }
__host__ __device__ constexpr int out_bit_of(int r) { return ((r >> 3) & 1) * 4 + (r & 3); }

// B operand: dword q of a lane is bit plane {q, q + 4} of W (its 4 input bytes of the step, rows
// 4h..4h+3 of its column) masked in place, with no shift into a common nibble position:
// q = 0: W & 0x11111111 (FP4 0.5), q = 1: W & 0x22222222 (1.0), q = 2: W & 0x44444444 (2.0),
// q = 3: (W >> 1) & 0x44444444 (2.0). The A entry at such a K index is the reciprocal weight
// (2.0 / 1.0 / 0.5 / 0.5, all exact e2m1), so every product is exactly 0 or 1 and the f32 sum is
// still the integer count whose parity is the GF(2) result.
constexpr uint8_t kAOne[4] = {0x4, 0x2, 0x1, 0x1};

// bitmat layout: [group][kstep][mt < MG][lane][16 bytes]; element j = nibble j of the 16 bytes (one
// K-step's MG fragments are contiguous, so the kernel reads them with immediate LDS offsets).
// K order inside a step (lane half h): nibble j <-> input row 8s + 4h + ((j & 7) >> 1), bit
// (j >> 3) + 4 (j & 1) — the order the kernel's expansion produces (expand() below).
// coefficient (o, i) = coeff[row(o) * ld + i], row(o) = sel ? sel[o] : o (sel: rows of a device
// matrix, e.g. the erased-native rows of a device-computed inverse)
__global__ void fp4_bitmat_kernel(const uint8_t* __restrict__ coeff, int ld, const int* __restrict__ sel, int m, int k,
                                  int ksteps, int mg, int groups, uint8_t* __restrict__ bitmat) {
  const int64_t total = int64_t(groups) * mg * ksteps * 64 * 16;
  for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < total;
       idx += int64_t(gridDim.x) * blockDim.x) {
    const int q = int(idx & 15);
    const int lane = int((idx >> 4) & 63);
    int64_t rest = idx >> 10;
    const int mt = int(rest % mg);
    rest /= mg;
    const int s = int(rest % ksteps);
    const int g = int(rest / ksteps);
    const int r = lane & 31, h = lane >> 5;
    const int orow = 4 * (g * mg + mt) + out_row_of(r);
    const int obit = out_bit_of(r);
    uint8_t v = 0;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int j = 2 * q + half;       // nibble j: B dword j >> 3, nibble j & 7 of it
      const int dq = j >> 3, jj = j & 7;
      const int irow = 8 * s + 4 * h + (jj >> 1);
      const int ibit = dq + 4 * (jj & 1);
      if (orow < m && irow < k &&
          ((dmul(coeff[size_t(sel ? sel[orow] : orow) * ld + irow], uint8_t(1u << ibit)) >> obit) & 1))
        v |= uint8_t(kAOne[dq] << (4 * half));
    }
    bitmat[idx] = v;
  }
}

// (a & mask) | (b & ~mask) as ONE v_bfi_b32 (written as C the compiler splits it into and + or3)
__device__ __forceinline__ uint32_t bfi(uint32_t mask, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(mask), "v"(a), "v"(b));
  return r;
}

// Parity placement. Accumulator register j of a 32x32 tile holds output bit b = j & 7 (of output
// byte j >> 3) as an exact f32 integer count c (<= 8k <= 2048). Every chunk STARTS its
// accumulators at 2^(23-b) instead of 0 (one extra "bias" MFMA per accumulator, below), which pins
// the f32 exponent: the mantissa field of 2^(23-b) + c is c << b, so the parity of c sits on bit
// b with zeros below, and an output byte is 7 bit-field inserts (v_bfi) of 8 raw accumulator words
// — no convert / mask / shift per bit.
//
// Bias MFMA operands: A = B = 1.0 at K index 0 only (nibble 0 of the lanes holding K-block 0),
// unit B scale, and an A scale (E8M0, per lane = per A row r) of 2^(23 - out_bit_of(r)).
__device__ __forceinline__ int bias_scale_of_lane(int lane) { return 127 + 23 - out_bit_of(lane & 31); }

// Per-wave input ring in LDS filled by LDS-DMA: a slot holds one K-PAIR (16 input rows x the
// wave's 64 columns = 1 KiB, row r at byte 64r) and is written by ONE `global_load_lds_dwordx4`
// (lane l -> row l/4, columns 16*(l%4)..+15): an LDS-DMA costs ~60-180 issue cycles whatever its
// width (MI355X_MICROARCH.md, constants table), so the widest form and two K-steps per DMA. The
// loads of the next kRing-1 pairs (kRing = 6..32, as deep as the LDS left over by the A slice
// allows) stay in flight across chunk boundaries without costing VGPRs. Each wave owns its ring
// (no barriers); a slot's bytes are ordered for the wave's own ds_reads by its counted vmcnt.
//
// The K loop is software-pipelined by hand: while the 2 x MG MFMAs of step g run, the ring bytes
// and the MG A fragments of step g+1 (and, for scattered input rows, the row pointer of the next
// DMA) are already being read from LDS. Those reads are inline asm, retired by one explicit
// `s_waitcnt lgkmcnt(0)` at the end of the step, and "tied" to their destination registers by
// empty asm statements so no use can be scheduled above the wait; the compiler's own alias
// tracking would otherwise put a vmcnt(0)/lgkmcnt(0) in front of every read.
constexpr int kSlotBytes = 1024;
// The bit-matrix allocation ends with a sink: output rows past m (padding of the last M-tile group)
// and fused copies with no destination are stored there, so neither the epilogue nor the K loop
// branches — one basic block the scheduler can interleave (MFMAs and conditional stores in
// separate blocks serialise). Nothing reads the sink. One 1-KiB slot per wave, spread over
// kFp4SinkSlots (kernels.h): a single shared slot serialised every CU on its lines (1100 vs 880 us
// at m = 24, profiles/wide_stripe/r02_fp4_ablate).
constexpr int kSinkBytes = 1024 * kFp4SinkSlots;
__device__ __forceinline__ uint64_t sink_slot(uint64_t base) {
  const unsigned slot = (blockIdx.x * 4u + (threadIdx.x >> 6)) % unsigned(kFp4SinkSlots);
  return base + uint64_t(slot) * 1024u + 16u * (threadIdx.x & 63u);
}
// LDS the launcher tries to leave free next to a persistent block, so a side-stream kernel (the
// decode-system solve, gf_invert.hip: 8.4 KiB at k=128, e=32) can co-reside instead of waiting
// for the whole GEMM.
constexpr size_t kSideReserve = 9 * 1024;
using lds_u8 = __attribute__((address_space(3))) uint8_t;

__device__ __forceinline__ void lgkm_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
template <typename T>
__device__ __forceinline__ void tie(T& v) {
  asm volatile("" : "+v"(v));
}

// UNI: input row j lives at in[0] + j * in_stride (rows from one allocation, the usual case), so
// DMA addresses are pure VALU arithmetic; otherwise the row pointers come from an LDS table.
// ksteps is a multiple of the K-steps per ring slot (the bitmat pads zero K-steps).
// COPY: fused survivor copy (decode): input row j is also written to copy[j] (when nonzero) from
// the LDS ring slot the DMA already filled — one ds_read_b128 + one global_store_dwordx4 per lane
// and slot, no second read of the survivors from HBM.
//
// One wave per SIMD (4 waves, 64 columns each). Measured alternatives that lost (profiles/r01_s3):
// two waves per SIMD with 32 columns each (128 AGPRs of accumulators: the rest no longer fits
// the 256 registers, it spills; 1061 vs 848 us), and MG = 4 blocks two per CU (1051 us).
//
// vmcnt accounting. `s_waitcnt vmcnt(N)` retires everything but the wave's N youngest vector-memory
// ops, loads, stores and LDS-DMA alike, in issue order (MI355X_MICROARCH.md). The wait for the next
// slot therefore counts every op issued after that slot's DMA: the kRing-2 younger DMAs, the fused
// copy stores (COPY; the prologue issues dummy ones to the sink so the pattern holds from slot 0)
// and, in the first slots of a chunk, the previous chunk's 2*MG epilogue stores. A count that
// ignored the stores (as before) also waited for them: a store-latency bubble at every chunk start.
//
// KS > 0: the chunk's slot count is the compile-time KS (= ksteps / kSPS) and a multiple of kRing,
// so every chunk starts at ring slot 0: the slot loop unrolls and every ring position, DMA cursor
// and bit-matrix step is a constant (LDS immediates, no cursor bookkeeping per slot).
template <int MG, bool UNI, bool COPY, int kRing, int KS>
__global__ __launch_bounds__(256, 1) void gf_gemm_fp4_kernel(cptr<uint64_t> in, cptr<uint64_t> out, cptr<uint64_t> copy,
                                                             const i32x4* __restrict__ bitmat, int k, int m,
                                                             int ksteps, int groups, int64_t col0, int64_t nchunks,
                                                             int64_t chunk_slots, int64_t in_stride) {
  constexpr int NTW = kNTW;              // N-tiles (32 columns each) per wave
  constexpr int kWaves = 4, kThreads = 256;
  constexpr int kCW = 32 * NTW;          // columns per wave
  constexpr int kRS = kSlotBytes / kCW;  // input rows per ring slot (16)
  constexpr int kSPS = kRS / 8;          // K-steps per ring slot (2)
  constexpr int kLPR = kCW / 16;         // DMA lanes per row (4)
  constexpr bool kStatic = KS > 0;
  static_assert(!kStatic || KS % kRing == 0, "KS must be a multiple of the ring depth");
  constexpr int kCopyN = COPY ? kRing - 2 : 0;
  // younger ops than the awaited DMA in steady state, and with the previous chunk's epilogue
  // stores (clamped to the 6-bit counter: a smaller count only waits longer)
  constexpr int kWaitN = std::min(kRing - 2 + kCopyN, 63);
  constexpr int kWaitEpiN = std::min(kRing - 2 + kCopyN + 2 * MG, 63);
  // LDS: A [ksteps][MG][64] x 16 B | row pointers [256] | out pointers [32] | (COPY) copy pointers
  // [256] | rings [kWaves][kRing][1 KiB] | one spare slot shared by the waves' dummy DMAs
  extern __shared__ __attribute__((aligned(16))) i32x4 afrag[];
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int local = bid >> 3;
  const int g = local % groups;
  const int64_t slot0 = int64_t(local / groups) * 8 + xcd;
  if (slot0 >= chunk_slots) return;

  const size_t a_bytes = size_t(MG) * ksteps * 1024;
  uint64_t* rowptr = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(afrag) + a_bytes);
  uint64_t* outptr = rowptr + 256;  // this group's 4*MG output rows
  const i32x4* src = bitmat + size_t(g) * MG * ksteps * 64;
  // this lane's 16 bytes of the sink past the bit-matrix (kSinkBytes)
  const uint64_t sink = sink_slot(uint64_t(bitmat + size_t(groups) * MG * ksteps * 64));
  for (int i = threadIdx.x; i < MG * ksteps * 64; i += kThreads) afrag[i] = src[i];
  if (!UNI)
    for (int i = threadIdx.x; i < k; i += kThreads) rowptr[i] = in[i];
  for (int i = threadIdx.x; i < 4 * MG; i += kThreads) {
    const int row = 4 * g * MG + i;
    outptr[i] = row < m ? out[row] : 0;
  }
  uint64_t* copyptr = rowptr + 256 + 32;
  if (COPY)
    for (int i = threadIdx.x; i < k; i += kThreads) copyptr[i] = g == 0 ? copy[i] : 0;  // group 0 copies
  __syncthreads();

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>((lds_u8*)afrag));
  const uint32_t a_addr = lds0 + 16u * lane;
  const uint32_t rowptr_addr = lds0 + uint32_t(a_bytes);
  const uint32_t optr_addr = rowptr_addr + 2048u + 16u * h;  // outptr[2h + u] of M-tile 0
  const uint32_t cptr_addr = rowptr_addr + 2304u;
  lds_u8* rings = (lds_u8*)(reinterpret_cast<uint8_t*>(afrag) + a_bytes + 2304 + (COPY ? 2048 : 0));
  lds_u8* ring = rings + size_t(wave) * kRing * kSlotBytes;
  lds_u8* spare = rings + size_t(kWaves) * kRing * kSlotBytes;
  // this lane's bytes of K-step half hs, row i: ring + hs*8*kCW + (4h + i)*kCW + NTW*c
  const uint32_t ring_addr = uint32_t(reinterpret_cast<uintptr_t>(ring)) + uint32_t(4 * h * kCW + NTW * c);
  const uint32_t ring_lane = uint32_t(reinterpret_cast<uintptr_t>(ring)) + 16u * lane;  // this lane's DMA'd 16 B
  const int scale = 0x7F7F7F7F;  // E8M0 1.0 for every block of 32
  const int bias_scale = bias_scale_of_lane(lane);
  const i32x8 one_k0 = {h == 0 ? 0x2 : 0, 0, 0, 0, 0, 0, 0, 0};  // 1.0 at K index 0 (A and B)
  const int my_chunks = int((nchunks - slot0 + chunk_slots - 1) / chunk_slots);
  const int kslots = kStatic ? KS : ksteps / kSPS;
  if (my_chunks <= 0) return;
  const uint64_t in0 = UNI ? in[0] : 0;
  const int drow = lane / kLPR;  // this lane's row within a DMA'd slot
  const int dcol = wave * kCW + 16 * (lane % kLPR);

  // DMA cursor (odometer over my chunks x slots) and, off the UNI path, the row pointer of the
  // cursor's slot. Past the last slot the cursor keeps issuing "dummy" DMAs (a valid source, the
  // spare slot as destination) so the number in flight — and with it every counted vmcnt below —
  // stays the same and the K loop has no branches.
  int d_chunk = 0, d_p = 0, d_slot = 0;
  uint64_t pn = 0;
  auto row_of = [&]() __attribute__((always_inline)) {
    const int r = kRS * d_p + drow;
    return r < k ? r : k - 1;  // rows >= k meet zero bit-matrix columns
  };
  auto ptr_sync = [&]() __attribute__((always_inline)) { pn = rowptr[row_of()]; };
  auto ptr_async = [&]() __attribute__((always_inline)) {
    asm volatile("ds_read_b64 %0, %1" : "=&v"(pn) : "v"(rowptr_addr + 8u * row_of()) : "memory");
  };
  auto dma_issue = [&]() __attribute__((always_inline)) {
    const bool live = d_chunk < my_chunks;
    const int64_t col = col0 + (slot0 + int64_t(live ? d_chunk : 0) * chunk_slots) * kBlockCols + dcol;
    uint64_t sa;
    if constexpr (UNI)
      sa = in0 + uint64_t(int64_t(row_of()) * in_stride + col);
    else
      sa = pn + uint64_t(col);
    __builtin_amdgcn_global_load_lds((gptr<const void>)sa, live ? ring + d_slot * kSlotBytes : spare, 16, 0, 0);
    const bool wrap = d_p + 1 == kslots;
    d_p = live ? (wrap ? 0 : d_p + 1) : d_p;
    d_chunk += (live && wrap) ? 1 : 0;
    d_slot = live ? (d_slot + 1 == kRing ? 0 : d_slot + 1) : d_slot;
  };
  // rows 4h+i of K-step half `hs` of a slot, this lane's column pair (2c, 2c+1). (d16 reads cannot
  // pack two rows into one register here: with SRAM ECC on, a d16 load zeroes the other half.)
  auto read_x = [&](uint32_t (&x)[4], int slot, int hs) {
    asm volatile(
        "ds_read_u16 %0, %4\n\t"
        "ds_read_u16 %1, %4 offset:64\n\t"
        "ds_read_u16 %2, %4 offset:128\n\t"
        "ds_read_u16 %3, %4 offset:192"
        : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3])
        : "v"(ring_addr + uint32_t(slot * kSlotBytes + hs * 8 * kCW))
        : "memory");
  };
  auto read_a = [&](i32x4 (&a)[MG], int s) {
    const uint32_t base = a_addr + uint32_t(s) * (MG * 1024u);
#pragma unroll
    for (int mt = 0; mt < MG; ++mt)
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=&v"(a[mt]) : "v"(base), "n"(mt * 1024) : "memory");
  };

  // B operands of a K-step from its 4 ring words: W_t = the 4 rows' bytes of column 2c + t (two
  // shift-ors and two v_perm for both tiles), then the bit planes of W_t masked in place (kAOne).
  // Rows >= k hold finite garbage (the DMA clamps to row k-1) that meets zero bit-matrix columns.
  constexpr int kExpandValu = 14;
  auto expand = [&](i32x4 (&bo)[NTW], const uint32_t (&x)[4]) __attribute__((always_inline)) {
    const uint32_t p01 = x[0] | (x[1] << 16), p23 = x[2] | (x[3] << 16);
    const uint32_t w[2] = {__builtin_amdgcn_perm(p23, p01, 0x06040200u), __builtin_amdgcn_perm(p23, p01, 0x07050301u)};
#pragma unroll
    for (int t = 0; t < NTW; ++t) {
      bo[t][0] = int(w[t] & 0x11111111u);
      bo[t][1] = int(w[t] & 0x22222222u);
      bo[t][2] = int(w[t] & 0x44444444u);
      bo[t][3] = int((w[t] >> 1) & 0x44444444u);
    }
  };

  // prologue: kRing-1 slots in flight (each followed, on the copy path, by a dummy store to the
  // sink: the K loop's vmcnt count assumes one copy store after every DMA); B(0), A(0) and the
  // raw bytes of step 1 in registers
  for (int i = 0; i < kRing - 1; ++i) {
    if (!UNI) ptr_sync();
    dma_issue();
    if constexpr (COPY) {
      const u32x4 zero = {0u, 0u, 0u, 0u};
      asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(sink), "v"(zero) : "memory");
    }
  }
  if (!UNI) ptr_sync();
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kRing - 2) : "memory");
  uint32_t x0[4], x1[4], x2[4];  // raw bytes: x1 = step s+1 (in registers), x2 = step s+2 (in flight)
  i32x4 ac[MG], an[MG];
  i32x4 bc[NTW], bn[NTW];
  read_x(x0, 0, 0);
  read_x(x1, 0, 1);
  read_a(ac, 0);
  lgkm_wait();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    tie(x0[i]);
    tie(x1[i]);
  }
#pragma unroll
  for (int mt = 0; mt < MG; ++mt) tie(ac[mt]);
  expand(bc, x0);

  f32x16 acc[MG][NTW];
  // (re)start M-tile mt's accumulators at the parity bias (see bias_scale_of_lane)
  auto bias_init = [&](int mt) __attribute__((always_inline)) {
    // (an opaque copy of the scale per MFMA keeps these loop-invariant, identical MFMAs from being
    // hoisted out of the chunk loop or merged, either of which turns them into v_accvgpr_write
    // copies of one result)
#pragma unroll
    for (int t = 0; t < NTW; ++t) {
      int bs = bias_scale;
      asm volatile("" : "+v"(bs));
      acc[mt][t] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(one_k0, one_k0, (f32x16)(0.0f), 4, 4, 0, bs, 0,
                                                                    scale);
    }
  };
#pragma unroll
  for (int mt = 0; mt < MG; ++mt) bias_init(mt);
  // one K-step s: its NTW x MG MFMAs with the B operand of step s+1 expanded in between (VALU
  // co-issues under the MFMA pipe); then retire the LDS reads of A(s+1) and the raw bytes of step
  // s+2, issued by the caller before the step
  auto step = [&](int s) __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int mt = 0; mt < MG; ++mt) {
      const i32x8 a = {ac[mt][0], ac[mt][1], ac[mt][2], ac[mt][3], 0, 0, 0, 0};
#pragma unroll
      for (int t = 0; t < NTW; ++t) {
        const i32x8 bb = {bc[t][0], bc[t][1], bc[t][2], bc[t][3], 0, 0, 0, 0};
        acc[mt][t] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, bb, acc[mt][t], 4, 4, 0, scale, 0, scale);
      }
    }
    expand(bn, x1);
    // interleave: one MFMA, then a slice of the next step's expansion
#pragma unroll
    for (int i = 0; i < NTW * MG; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, (kExpandValu + NTW * MG - 1) / (NTW * MG), 0);  // VALU
    }
    __builtin_amdgcn_sched_barrier(0);
    lgkm_wait();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      tie(x2[i]);
      x1[i] = x2[i];
    }
#pragma unroll
    for (int mt = 0; mt < MG; ++mt) {
      tie(an[mt]);
      ac[mt] = an[mt];
    }
#pragma unroll
    for (int t = 0; t < NTW; ++t) bc[t] = bn[t];
  };
  using last_t = std::integral_constant<bool, true>;
  using rest_t = std::integral_constant<bool, false>;

  int r_slot = 0;
  // the chunk's output: NTW bytes per lane per (M-tile, byte row), one M-tile at a time, straight
  // from the last MFMAs' accumulators (inside the last slot, so acc never leaves the AGPRs
  // through a loop-exit copy); exactly 2*MG stores per wave (kWaitEpiN)
  auto store_chunk = [&](int ci) __attribute__((always_inline)) {
    // pin the last step's MFMAs here (before the epilogue had one basic block per store, machine
    // sinking moved each MFMA into its reader's block, which then waited out its full latency)
#pragma unroll
    for (int mt = 0; mt < MG; ++mt)
#pragma unroll
      for (int t = 0; t < NTW; ++t) asm volatile("" ::"a"(acc[mt][t]));
    const int64_t colw = col0 + (slot0 + int64_t(ci) * chunk_slots) * kBlockCols + wave * kCW + NTW * c;
    // output row pointers of M-tile mt: 32-bit LDS address + immediate (a C++ read of outptr[]
    // would be hoisted out of the chunk loop as 2*MG live 64-bit flat addresses), read one M-tile
    // ahead under the packing so only 4 pointer registers are live (all 2*MG at once made the
    // two-waves-per-SIMD form spill)
    auto read_op = [&](uint64_t (&o)[2], int mt) __attribute__((always_inline)) {
      asm volatile("ds_read_b64 %0, %2 offset:%3\n\tds_read_b64 %1, %2 offset:%4"
                   : "=&v"(o[0]), "=&v"(o[1])
                   : "v"(optr_addr), "n"(32 * mt), "n"(32 * mt + 8)
                   : "memory");
    };
    uint64_t opn[2];
    read_op(opn, 0);
    lgkm_wait();
    tie(opn[0]);
    tie(opn[1]);
#pragma unroll
    for (int mt = 0; mt < MG; ++mt) {
      const uint64_t op[2] = {opn[0], opn[1]};
      if (mt + 1 < MG) read_op(opn, mt + 1);
      // both byte rows of both N-tiles from one pass over the M-tile's 32 accumulators: 4
      // interleaved chains of 7 v_bfi (no back-to-back dependency)
      uint32_t y[NTW][2];
#pragma unroll
      for (int b = 0; b < 8; ++b)
#pragma unroll
        for (int t = 0; t < NTW; ++t)
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const uint32_t v = __float_as_uint(acc[mt][t][8 * u + b]);
            y[t][u] = b == 0 ? v : bfi(1u << b, v, y[t][u]);
          }
      uint32_t w[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) w[u] = __builtin_amdgcn_perm(y[1][u], y[0][u], 0x0c0c0400u);
      // the next chunk's bias goes into this tile now: its MFMA pipe time runs under the next
      // tile's packing (after the last chunk it is simply unused)
      bias_init(mt);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint64_t o = op[u];
        *(gptr<uint16_t>)(o ? o + colw : sink) = uint16_t(w[u]);
      }
      if (mt + 1 < MG) {
        lgkm_wait();
        tie(opn[0]);
        tie(opn[1]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // one ring slot (r_slot) = kSPS K-steps: (1) the DMA kRing-1 slots ahead; (2) under each step's
  // MFMAs, the raw bytes of the step after next (from this slot, or — after waiting for it — the
  // next one) and the A fragments of the next step. Reads past the last step hit valid LDS and are
  // discarded.
  auto slot_run = [&](int sp, int ci, auto last_tag) __attribute__((always_inline)) {
    if constexpr (kStatic) {  // the cursor of slot sp as constants (see the KS note above)
      constexpr int lead = kRing - 1;
      r_slot = sp % kRing;
      d_p = (sp + lead) % KS;
      d_slot = (sp + lead) % kRing;
      d_chunk = ci + (sp + lead) / KS;
    }
    dma_issue();
    if (!UNI) ptr_async();
    const int s0 = kSPS * sp;
    const int slot1 = r_slot + 1 == kRing ? 0 : r_slot + 1;
    [[maybe_unused]] u32x4 cdat;
    [[maybe_unused]] uint64_t cp = 0;
    [[maybe_unused]] const int crow = kRS * sp + drow;
    if constexpr (COPY) {  // this lane's 16 B of the current slot and its row's copy pointer
      asm volatile("ds_read_b128 %0, %1" : "=&v"(cdat) : "v"(ring_lane + uint32_t(r_slot * kSlotBytes)) : "memory");
      asm volatile("ds_read_b64 %0, %1"
                   : "=&v"(cp)
                   : "v"(cptr_addr + 8u * uint32_t(crow < k ? crow : k - 1))
                   : "memory");
    }
#pragma unroll
    for (int j = 0; j < kSPS; ++j) {
      if (j + 2 == kSPS) {  // the next slot has landed: count the younger ops (see the header)
        if (ci > 0 && sp + 3 <= kRing)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kWaitEpiN) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kWaitN) : "memory");
      }
      if (j + 2 < kSPS)
        read_x(x2, r_slot, j + 2);
      else
        read_x(x2, slot1, j + 2 - kSPS);
      read_a(an, s0 + j + 1 == kSPS * kslots ? 0 : s0 + j + 1);
      step(s0 + j);  // (the first step's closing lgkmcnt(0) also retires the copy / pointer reads)
      if (j == 0) {
        if (!UNI) tie(pn);
        if constexpr (COPY) {
          tie(cdat);
          tie(cp);
          const int64_t col = col0 + (slot0 + int64_t(ci) * chunk_slots) * kBlockCols + dcol;
          __builtin_nontemporal_store(cdat, (gptr<u32x4>)(crow < k && cp ? cp + uint64_t(col) : sink));
        }
      }
    }
    r_slot = slot1;
    if constexpr (decltype(last_tag)::value) store_chunk(ci);
  };

  for (int ci = 0; ci < my_chunks; ++ci) {
    if constexpr (kStatic) {
#pragma unroll
      for (int sp = 0; sp < KS - 1; ++sp) slot_run(sp, ci, rest_t{});
      slot_run(KS - 1, ci, last_t{});
    } else {
      for (int sp = 0; sp < kslots - 1; ++sp) slot_run(sp, ci, rest_t{});
      slot_run(kslots - 1, ci, last_t{});
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA (dummy or not) outlives the wave
}

struct Fp4Geometry {
  int ksteps, mtiles, mg, groups;
  size_t fixed;  // LDS bytes before the rings: A slice + row/out pointers
};

size_t bitmat_matrix_bytes(const Fp4Geometry& g) { return size_t(g.groups) * g.mg * g.ksteps * 64 * 16; }

// ring LDS of a block: R slots per wave plus the one spare slot the waves share
constexpr size_t ring_lds(int r) { return (4 * size_t(r) + 1) * kSlotBytes; }

Fp4Geometry geometry(int k, int m, int mg_cap, bool copy = false) {
  Fp4Geometry g{};
  g.ksteps = ((k + 15) / 16) * 2;  // ring slots: one 1-KiB DMA slot = 2 K-steps
  g.mtiles = (m + 3) / 4;
  // MG = M-tiles per block: next power of two >= mtiles (<= 8, the accumulator budget), halved
  // until the block's A slice fits the LDS
  g.mg = 1;
  while (g.mg < g.mtiles && g.mg < mg_cap) g.mg <<= 1;
  // (the copy-pointer block is always budgeted, so the bitmat layout does not depend on `copy`)
  while (g.mg > 1 && g.mg * g.ksteps > kMaxLdsKiB - 2) g.mg >>= 1;
  // the static wide-stripe chunk (k in (112, 128]): exactly mtiles M-tiles instead of a padded 8 or
  // 4 — a decode rebuilding 20..28 natives skips 1..3 tiles of MFMAs that would only compute padding
  // rows (12.5-37.5 % of the matrix-core work; profiles/wide_stripe/r02_exact_mg)
  if (g.ksteps == 16 && ((g.mg == 8 && g.mtiles > 4 && g.mtiles < 8) || (g.mg == 4 && g.mtiles == 3)))
    g.mg = g.mtiles;
  g.groups = (g.mtiles + g.mg - 1) / g.mg;
  g.fixed = size_t(g.mg) * g.ksteps * 64 * 16 + 2304 + (copy ? 2048 : 0);
  return g;
}

// the kernel's address, opted into the full 160 KiB of LDS on the current device (per device:
// one process may drive several GPUs, gfrs/device_cache.h)
template <int MG, bool UNI, bool COPY, int R, int KS>
const void* fp4_fn() {
  const void* f = reinterpret_cast<const void*>(&gf_gemm_fp4_kernel<MG, UNI, COPY, R, KS>);
  (void)ensure_lds_optin(f);
  return f;
}

// co-resident blocks per CU of the ring-depth-R kernel (LDS and VGPR bound); 0 if it does not fit
template <int MG, bool UNI, bool COPY, int R, int KS>
int fp4_occupancy(size_t fixed) {
  const size_t lds = fixed + ring_lds(R);
  if (lds > 160 * 1024) return 0;
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fp4_fn<MG, UNI, COPY, R, KS>(), 256, lds) != hipSuccess)
    return 0;
  return occ;
}

struct Fp4Args {
  cptr<uint64_t> in, out, copy;
  const void* bitmat;
  int k, m;
  int64_t col0, nchunks, in_stride;
};

template <int MG, bool UNI, bool COPY, int R, int KS>
hipError_t launch_fp4(const Fp4Geometry& geo, int occ, const Fp4Args& a, hipStream_t stream) {
  // a persistent grid: as many blocks as are co-resident, chunk slots a multiple of 8 so each
  // slot stays on one XCD
  const size_t lds = geo.fixed + ring_lds(R);
  (void)fp4_fn<MG, UNI, COPY, R, KS>();
  const int64_t slots = persistent_slots(occ, geo.groups, a.nchunks);
  const unsigned blocks = unsigned(slots * geo.groups);
  gf_gemm_fp4_kernel<MG, UNI, COPY, R, KS><<<blocks, 256, lds, stream>>>(
      a.in, a.out, a.copy, static_cast<const i32x4*>(a.bitmat), a.k, a.m, geo.ksteps, geo.groups, a.col0, a.nchunks,
      slots, a.in_stride);
  return hipGetLastError();
}

template <int MG, bool UNI, bool COPY, int KS, int... Rs>
hipError_t launch_fp4_ring(const Fp4Geometry& geo, const Fp4Args& a, hipStream_t stream) {
  // ring depth (candidates Rs, deepest first): the most blocks per CU first (up to 4), then — at
  // equal occupancy — a ring that leaves kSideReserve of the CU's LDS free (measured: DMA latency
  // costs ~2 % at ring 6, profiles/r01_s3; a full-LDS persistent grid instead locks the
  // side-stream decode solve out of every CU until the GEMM ends), then the deepest ring. Cached
  // per A size.
  constexpr int kN = sizeof...(Rs);
  constexpr int rings[kN] = {Rs...};
  // per (device, A size in KiB) -> {ring index + 1 (0 = nothing fits), occupancy}
  static DeviceMemo<size_t, std::pair<int, int>> choice;
  const std::pair<int, int> ch = choice.get_or(geo.fixed / 1024, [&] {
    const int occs[kN] = {fp4_occupancy<MG, UNI, COPY, Rs, KS>(geo.fixed)...};
    auto reserve_ok = [&](int i) { return geo.fixed + ring_lds(rings[i]) + kSideReserve <= 160 * 1024; };
    int best = -1;
    for (int i = 0; i < kN; ++i) {
      if (occs[i] <= 0) continue;
      if (best < 0 || std::min(occs[i], 4) > std::min(occs[best], 4) ||
          (std::min(occs[i], 4) == std::min(occs[best], 4) && reserve_ok(i) && !reserve_ok(best)))
        best = i;
    }
    return best < 0 ? std::pair<int, int>{0, 0} : std::pair<int, int>{best + 1, occs[best]};
  });
  if (ch.first == 0) return hipErrorInvalidConfiguration;
  hipError_t err = hipErrorInvalidConfiguration;
  int i = 0;
  ((i++ == ch.first - 1 ? (err = launch_fp4<MG, UNI, COPY, Rs, KS>(geo, ch.second, a, stream), 0) : 0), ...);
  return err;
}

// k in (112, 128] (8 ring slots per chunk, the BASELINE wide stripe): the unrolled static-cursor
// kernel with the rings that divide 8; any other k: the runtime-cursor kernel
template <int MG, bool UNI, bool COPY>
hipError_t launch_fp4_var(const Fp4Geometry& geo, const Fp4Args& a, hipStream_t stream) {
  // (fused-copy form: ring 4 only — the depth-8 form ran 0-6 % slower at m = 8..16,
  // profiles/wide_stripe/r02_exact_mg/session_k_*)
  if (geo.ksteps == 16)
    return COPY ? launch_fp4_ring<MG, UNI, COPY, 8, 4>(geo, a, stream) : launch_fp4_ring<MG, UNI, COPY, 8, 8, 4>(geo, a, stream);
  return launch_fp4_ring<MG, UNI, COPY, 0, 32, 16, 12, 8, 6, 4>(geo, a, stream);
}

// variants: uniform-stride inputs (encode), scattered inputs, scattered inputs + fused copy (decode)
template <int MG>
hipError_t launch_fp4_any(const Fp4Geometry& geo, const Fp4Args& a, hipStream_t stream) {
  if (a.copy) return launch_fp4_var<MG, false, true>(geo, a, stream);
  return a.in_stride ? launch_fp4_var<MG, true, false>(geo, a, stream)
                     : launch_fp4_var<MG, false, false>(geo, a, stream);
}

// MG = 3 and 6 exist for the static 8-slot chunk only (geometry() picks them there; fp4_route sends
// 5 to 7 tiles to the tile-major kernel, so MG = 6 runs here only under GFRS_TUNE=fp4=v1), ring depth 4: the depth-8 forms fit the LDS but need ~90
// more VGPRs (256 with spills into AGPRs) and ran 0-19 % slower at every shape
// (profiles/wide_stripe/r02_exact_mg: k=128, m=28 + 100 copies 885 vs 1050 us)
template <int MG>
hipError_t launch_fp4_static_any(const Fp4Geometry& geo, const Fp4Args& a, hipStream_t stream) {
  if (geo.ksteps != 16) return hipErrorInvalidConfiguration;
  if (a.copy) return launch_fp4_ring<MG, false, true, 8, 4>(geo, a, stream);
  return a.in_stride ? launch_fp4_ring<MG, true, false, 8, 4>(geo, a, stream)
                     : launch_fp4_ring<MG, false, false, 8, 4>(geo, a, stream);
}

// ---- the one routing decision of the GF(2^8) FP4 engine ------------------------------------------
// Forms: v1 (the LDS-ring kernel above: any k, any M-tile count, groups of M-tiles), ar (A-resident,
// gf_mfma_fp4ar.hip: bit-matrix in AGPRs, k in (112, 128], one group of <= 8 tiles, also the batched
// launch) and tm (tile-major, gf_mfma_fp4tm.hip: B in AGPRs, tiles in pairs, 5..8 tiles). Every
// branch is a measured win (k = 128, 1 GiB, medians, two interleaved rounds each):
//   * 1..3 tiles: v1 — memory-bound shapes; ar loses there (profiles/wide_stripe/r02_fp4_ablate);
//   * 4 tiles: ar, plain and with fused copies (m = 16: 490 vs 530 us plain, 659 vs 722 with 112
//     copies; r02_fp4_ablate);
//   * 5 tiles: tm, plain and copies (m = 20: 595-611 vs 625-631 us plain, 750-766 vs 776-784 with
//     108 copies; profiles/wide_stripe/r09_route);
//   * 6 tiles: tm, plain (m = 22/24: 644-673 vs 696-719 on v1, 668-677 on ar; r09_route, r08_tm)
//     and with copies (818-842 vs 833-842 us; k128n160 1.405-1.416 vs 1.414-1.420 ms/step,
//     profiles/wide_stripe/r09_tm6 — before its row indices were laundered, the tm copy build
//     spilled 16 VGPRs to scratch and ran 1300 us);
//   * 7 tiles: tm, plain and copies (m = 26: 729-767 vs 795-798 plain, 877-884 vs 935-940 with 102
//     copies; r09_route);
//   * 8 tiles: ar plain (the p = 32 encode: 809 vs 842 us on v1, r02_fp4_ablate; 798-827 vs 809-835
//     on tm, profiles/wide_stripe/r10_tm8), tm with copies (tile 7's A in registers: m = 29 / 30 / 32
//     + 99 / 98 / 96 copies 931-950 vs 979-1007 us on v1 and 997-1018 on ar; k128n160 1.418 vs
//     1.426 ms/step over 100 steps, r10_tm8);
//   * more than one group (m > 32) or k outside (112, 128]: v1.
// GFRS_TUNE=fp4=v1|ar|tm forces that form wherever it is built for the shape (A/B measurements).
enum class Fp4Form { kV1, kAResident, kTileMajor };

bool form_built(Fp4Form f, const Fp4Geometry& geo, int k, bool copies) {
  switch (f) {
    case Fp4Form::kAResident: return geo.groups == 1 && fp4ar_supported(k, geo.mg);
    case Fp4Form::kTileMajor: return geo.groups == 1 && fp4tm_supported(k, geo.mg, copies);
    default: return geo.ksteps != 16 || geo.mg == 1 || geo.mg == 2 || geo.mg == 3 || geo.mg == 4 || geo.mg == 6 ||
                    geo.mg == 8;
  }
}

Fp4Form fp4_route(const Fp4Geometry& geo, int k, bool copies) {
  // (read per call: the form does not change the bit-matrix layout, so an A/B run may switch it
  // between launches of one plan)
  const int forced = [] {
    const std::string e = tune_str("fp4");
    if (e == "v1") return int(Fp4Form::kV1);
    if (e == "ar") return int(Fp4Form::kAResident);
    if (e == "tm") return int(Fp4Form::kTileMajor);
    return -1;
  }();
  if (forced >= 0 && form_built(Fp4Form(forced), geo, k, copies)) return Fp4Form(forced);
  if (geo.groups != 1 || k <= 112 || k > 128) return Fp4Form::kV1;
  switch (geo.mg) {
    case 4: return Fp4Form::kAResident;
    case 5:
    case 7: return Fp4Form::kTileMajor;
    case 6: return Fp4Form::kTileMajor;
    case 8:  // (GFRS_TUNE=tm8=0: copies back on v1, for A/B runs)
      return copies ? (tune_int("tm8", 1) ? Fp4Form::kTileMajor : Fp4Form::kV1) : Fp4Form::kAResident;
    default: return Fp4Form::kV1;
  }
}

}  // namespace

size_t fp4_bitmat_bytes(int k, int m, int mg_cap) {
  const Fp4Geometry g = geometry(k, m, mg_cap);
  return bitmat_matrix_bytes(g) + kSinkBytes;
}

hipError_t launch_fp4_bitmat_sel(const uint8_t* coeff, int ld, const int* sel, int m, int k, void* bitmat, int mg_cap,
                                 hipStream_t stream) {
  if (m <= 0 || k <= 0 || m > 256 || k > 256 || mg_cap < 1 || ld < k) return hipErrorInvalidValue;
  const Fp4Geometry g = geometry(k, m, mg_cap);
  const int64_t total = int64_t(bitmat_matrix_bytes(g));
  const int blocks = int(std::min<int64_t>((total + 255) / 256, 4096));
  fp4_bitmat_kernel<<<blocks, 256, 0, stream>>>(coeff, ld, sel, m, k, g.ksteps, g.mg, g.groups,
                                                static_cast<uint8_t*>(bitmat));
  return hipGetLastError();
}

hipError_t launch_fp4_bitmat(const uint8_t* coeff, int m, int k, void* bitmat, int mg_cap, hipStream_t stream) {
  return launch_fp4_bitmat_sel(coeff, k, nullptr, m, k, bitmat, mg_cap, stream);
}

hipError_t launch_gf_gemm_fp4(const void* bitmat, const void* desc, int k, int m, int64_t col0, int64_t ncols,
                              int mg_cap, int64_t in_stride, bool copies, hipStream_t stream) {
  if (k <= 0 || m <= 0 || ncols < 0 || (col0 & 1) || mg_cap < 1) return hipErrorInvalidValue;
  const int m_pad = pad_m(m);
  const DescLayout l = desc_layout(k, m_pad);
  const char* b = static_cast<const char*>(desc);
  const Fp4Geometry geo = geometry(k, m, mg_cap, copies);
  const Fp4Form form = fp4_route(geo, k, copies);
  if (form != Fp4Form::kV1) {  // the AGPR-resident forms (launch record of gfrs/kernels.h)
    Fp4ArLaunch a{};
    a.in = reinterpret_cast<const uint64_t*>(b + l.in_off);
    a.out = reinterpret_cast<const uint64_t*>(b + l.out_off);
    a.copy = copies ? reinterpret_cast<const uint64_t*>(b + l.copy_off) : nullptr;
    a.bitmat = bitmat;
    a.k = k;
    a.m = m;
    a.mg = geo.mg;
    a.col0 = col0;
    a.ncols = ncols;
    a.in_stride = copies ? 0 : in_stride;
    int64_t done = 0;
    const hipError_t e = form == Fp4Form::kTileMajor ? launch_gf_gemm_fp4tm(a, &done, stream)
                                                     : launch_gf_gemm_fp4ar(a, &done, stream);
    if (e != hipSuccess) return e;
    if (done < ncols) return launch_gf_gemm(desc, k, m_pad, col0 + done, ncols - done, false, 0, stream);
    return hipSuccess;
  }
  const int64_t chunk_cols = kBlockCols;
  const int64_t nchunks = ncols / chunk_cols;
  if (nchunks > 0) {
    Fp4Args a{};
    a.in = (cptr<uint64_t>)(b + l.in_off);
    a.out = (cptr<uint64_t>)(b + l.out_off);
    a.copy = copies ? (cptr<uint64_t>)(b + l.copy_off) : nullptr;
    a.bitmat = bitmat;
    a.k = k;
    a.m = m;
    a.col0 = col0;
    a.nchunks = nchunks;
    a.in_stride = copies ? 0 : in_stride;  // the copy variant reads row pointers from the table
    hipError_t e;
    switch (geo.mg) {
      case 8: e = launch_fp4_any<8>(geo, a, stream); break;
      case 6: e = launch_fp4_static_any<6>(geo, a, stream); break;
      case 4: e = launch_fp4_any<4>(geo, a, stream); break;
      case 3: e = launch_fp4_static_any<3>(geo, a, stream); break;
      case 2: e = launch_fp4_any<2>(geo, a, stream); break;
      case 1: e = launch_fp4_any<1>(geo, a, stream); break;
      default: e = hipErrorInvalidConfiguration; break;  // (5, 7 tiles: tile-major only, fp4_route)
    }
    if (e != hipSuccess) return e;
  }
  const int64_t done = nchunks * chunk_cols;
  if (done < ncols) return launch_gf_gemm(desc, k, m_pad, col0 + done, ncols - done, false, 0, stream);
  return hipSuccess;
}

const char* fp4_route_name(int k, int m, bool copies, int mg_cap) {
  if (k <= 0 || m <= 0 || mg_cap < 1) return "invalid";
  switch (fp4_route(geometry(k, m, mg_cap, copies), k, copies)) {
    case Fp4Form::kAResident: return "ar";
    case Fp4Form::kTileMajor: return "tm";
    default: return "v1";
  }
}

hipError_t launch_gf_gemm_fp4_batched(const void* bitmat, const void* desc, int k, int m, int batch, int64_t col0,
                                      int64_t ncols, int mg_cap, int64_t in_stride, int64_t in_bstride,
                                      int64_t out_bstride, bool copies, hipStream_t stream) {
  if (k <= 0 || m <= 0 || ncols < 0 || (col0 & 1) || mg_cap < 1 || batch < 1 || batch > 65535)
    return hipErrorInvalidValue;
  const int m_pad = pad_m(m);
  const Fp4Geometry geo = geometry(k, m, mg_cap, copies);
  if (geo.groups != 1 || !fp4ar_supported(k, geo.mg)) return hipErrorNotSupported;
  const DescLayout l = desc_layout(k, m_pad, batch);
  const char* b = static_cast<const char*>(desc);
  Fp4ArLaunch a{};
  a.in = reinterpret_cast<const uint64_t*>(b + l.in_off);  // stripe 0's tables (the first k / m_pad entries)
  a.out = reinterpret_cast<const uint64_t*>(b + l.out_off);
  a.copy = copies ? reinterpret_cast<const uint64_t*>(b + l.copy_off) : nullptr;
  a.bitmat = bitmat;
  a.k = k;
  a.m = m;
  a.mg = geo.mg;
  a.col0 = col0;
  a.ncols = ncols;
  a.in_stride = copies ? 0 : in_stride;
  a.batch = batch;
  a.in_bstride = in_bstride;
  a.out_bstride = out_bstride;
  int64_t done = 0;
  const hipError_t e = launch_gf_gemm_fp4ar(a, &done, stream);
  if (e != hipSuccess) return e;
  // every stripe's ragged remainder (under one chunk) on the batched v_perm kernel
  if (done < ncols) return launch_gf_gemm_batched(desc, k, m_pad, batch, col0 + done, ncols - done, false, stream, copies);
  return hipSuccess;
}

}  // namespace gfrs

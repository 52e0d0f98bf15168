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
// 2 x MG MFMAs. Input bytes are expanded to 8 FP4 nibbles with one v_perm of a 4-entry pool
// {0x00,0x02,0x20,0x22} indexed by the byte's 2-bit chunks.
// Output bits are placed on MFMA rows exactly as in gf_mfma.hip so every lane owns whole bytes.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "gfrs/desc.h"
#include "gfrs/kernels.h"

namespace gfrs {
namespace {

using i32x8 = int __attribute__((ext_vector_type(8)));
using i32x4 = int __attribute__((ext_vector_type(4)));
using f32x16 = float __attribute__((ext_vector_type(16)));
template <typename T>
using cptr = const __attribute__((address_space(4))) T*;
template <typename T>
using gptr = __attribute__((address_space(1))) T*;

constexpr int kNTW = 2;        // N-tiles per wave (64 columns)
constexpr int kBlockCols = 256;  // 4 waves x 64 columns
constexpr int kMaxLdsKiB = 139;  // A slice; + 2.25 KiB row/out pointers + 4 waves x 9 x 512 B rings <= 160 KiB

__constant__ Tables d_tab = make_tables();

__device__ __forceinline__ uint8_t dmul(uint8_t a, uint8_t b) { return d_tab.exp[d_tab.log[a] + d_tab.log[b]]; }
__host__ __device__ constexpr int out_row_of(int r) { return 2 * ((r >> 2) & 1) + (r >> 4); }
__host__ __device__ constexpr int out_bit_of(int r) { return ((r >> 3) & 1) * 4 + (r & 3); }

// bitmat layout: [group][kstep][mt < MG][lane][16 bytes]; element j = nibble j of the 16 bytes (one
// K-step's MG fragments are contiguous, so the kernel reads them with immediate LDS offsets).
__global__ void fp4_bitmat_kernel(const uint8_t* __restrict__ coeff, int m, int k, int ksteps, int mg, int groups,
                                  uint8_t* __restrict__ bitmat) {
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
      const int j = 2 * q + half;
      const int irow = 8 * s + 4 * h + (j >> 3);
      const int ibit = j & 7;
      if (orow < m && irow < k && ((dmul(coeff[size_t(orow) * k + irow], uint8_t(1u << ibit)) >> obit) & 1))
        v |= uint8_t(0x2u << (4 * half));
    }
    bitmat[idx] = v;
  }
}

// 8 bits of x -> 8 FP4 nibbles (bit b -> nibble b = 0x2 if set).
__device__ __forceinline__ int expand_fp4(uint32_t x) {
  const uint32_t sel = (((x & 0x33u) * 0x1001u) | ((x & 0xCCu) * 0x40040u)) & 0x03030303u;
  return int(__builtin_amdgcn_perm(0u, 0x22200200u, sel));
}

__device__ __forceinline__ uint32_t parity(float v) { return uint32_t(v) & 1u; }

// Output byte u (0/1) of one accumulator tile (regs 8u .. 8u+7).
__device__ __forceinline__ uint32_t pack_byte(const f32x16& acc, int u) {
  uint32_t v = 0;
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int low = 0; low < 4; ++low) v |= parity(acc[4 * (2 * u + q) + low]) << (q * 4 + low);
  return v;
}

// Per-wave input ring in LDS filled by LDS-DMA (global_load_lds, 4 B per lane): the loads of the
// next kRing-1 K-steps stay in flight across chunk boundaries without costing VGPRs, which the
// one-wave-per-SIMD MFMA loop needs to cover HBM latency. Each wave owns its ring (no barriers):
// a slot = 8 input rows x the wave's 64 columns = 512 B, written by two 256-B DMA instructions
// (lane l -> row 4*half + l/16, columns 4*(l%16)..+3).
//
// The K loop is software-pipelined by hand: while the 2 x MG MFMAs of step g run, the ring bytes
// and the MG A fragments of step g+1 (and, for scattered input rows, the row pointers of the next
// DMA) are already being read from LDS. Those reads are inline asm, retired by one explicit
// `s_waitcnt lgkmcnt(0)` at the end of the step, and "tied" to their destination registers by
// empty asm statements so no use can be scheduled above the wait; the compiler's own alias
// tracking would otherwise put a vmcnt(0)/lgkmcnt(0) in front of every read.
constexpr int kRing = 8;
constexpr int kSlotBytes = 512;
using lds_u8 = __attribute__((address_space(3))) uint8_t;

__device__ __forceinline__ void lgkm_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
template <typename T>
__device__ __forceinline__ void tie(T& v) {
  asm volatile("" : "+v"(v));
}

// UNI: input row j lives at in[0] + j * in_stride (rows from one allocation, the usual case), so
// DMA addresses are pure VALU arithmetic; otherwise the row pointers come from an LDS table.
template <int MG, bool UNI>
__global__ __launch_bounds__(256, 1) void gf_gemm_fp4_kernel(cptr<uint64_t> in, cptr<uint64_t> out,
                                                             const i32x4* __restrict__ bitmat, int k, int m,
                                                             int ksteps, int groups, int64_t col0, int64_t nchunks,
                                                             int64_t chunk_slots, int64_t in_stride) {
  // LDS: A [ksteps][MG][64] x 16 B | row pointers [256] | out pointers [32] | rings [4][kRing+1][512]
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
  for (int i = threadIdx.x; i < MG * ksteps * 64; i += 256) afrag[i] = src[i];
  if (!UNI)
    for (int i = threadIdx.x; i < k; i += 256) rowptr[i] = in[i];
  for (int i = threadIdx.x; i < 4 * MG; i += 256) {
    const int row = 4 * g * MG + i;
    outptr[i] = row < m ? out[row] : 0;
  }
  __syncthreads();

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>((lds_u8*)afrag));
  const uint32_t a_addr = lds0 + 16u * lane;
  const uint32_t rowptr_addr = lds0 + uint32_t(a_bytes);
  lds_u8* ring =
      (lds_u8*)(reinterpret_cast<uint8_t*>(afrag) + a_bytes + 2304 + size_t(wave) * (kRing + 1) * kSlotBytes);
  const uint32_t ring_addr = uint32_t(reinterpret_cast<uintptr_t>(ring)) + uint32_t(256 * h + 2 * c);
  const int scale = 0x7F7F7F7F;  // E8M0 1.0 for every block of 32
  const int my_chunks = int((nchunks - slot0 + chunk_slots - 1) / chunk_slots);
  const int total = my_chunks * ksteps;
  if (total <= 0) return;
  const uint64_t in0 = UNI ? in[0] : 0;

  // DMA cursor (odometer over my chunks x K-steps) and, off the UNI path, the row pointers of the
  // cursor's step. Past the last step the cursor keeps issuing "dummy" DMAs (a valid source, the
  // wave's spare slot kRing as destination) so the number in flight — and with it every counted
  // vmcnt below — stays the same and the K loop has no branches.
  int d_chunk = 0, d_s = 0, d_slot = 0;
  uint64_t pn0 = 0, pn1 = 0;
  auto row_of = [&](int half) {
    const int r = 8 * d_s + 4 * half + (lane >> 4);
    return r < k ? r : k - 1;  // rows >= k are masked to zero at expansion time
  };
  auto ptr_sync = [&]() {
    pn0 = rowptr[row_of(0)];
    pn1 = rowptr[row_of(1)];
  };
  auto ptr_async = [&]() {
    asm volatile("ds_read_b64 %0, %2\n\tds_read_b64 %1, %3"
                 : "=&v"(pn0), "=&v"(pn1)
                 : "v"(rowptr_addr + 8u * row_of(0)), "v"(rowptr_addr + 8u * row_of(1))
                 : "memory");
  };
  auto dma_issue = [&]() {
    const bool live = d_chunk < my_chunks;
    const int64_t col = col0 + (slot0 + int64_t(live ? d_chunk : 0) * chunk_slots) * kBlockCols + wave * 64 +
                        4 * (lane & 15);
    uint64_t s0, s1;
    if constexpr (UNI) {
      s0 = in0 + uint64_t(int64_t(row_of(0)) * in_stride + col);
      s1 = in0 + uint64_t(int64_t(row_of(1)) * in_stride + col);
    } else {
      s0 = pn0 + uint64_t(col);
      s1 = pn1 + uint64_t(col);
    }
    lds_u8* dst = ring + (live ? d_slot : kRing) * kSlotBytes;
    __builtin_amdgcn_global_load_lds((gptr<const void>)s0, dst, 4, 0, 0);
    __builtin_amdgcn_global_load_lds((gptr<const void>)s1, dst + 256, 4, 0, 0);
    const bool wrap = d_s + 1 == ksteps;
    d_s = live ? (wrap ? 0 : d_s + 1) : d_s;
    d_chunk += (live && wrap) ? 1 : 0;
    d_slot = live ? (d_slot + 1 == kRing ? 0 : d_slot + 1) : d_slot;
  };
  auto read_x = [&](uint32_t (&x)[4], int slot) {
    asm volatile(
        "ds_read_u16 %0, %4\n\t"
        "ds_read_u16 %1, %4 offset:64\n\t"
        "ds_read_u16 %2, %4 offset:128\n\t"
        "ds_read_u16 %3, %4 offset:192"
        : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3])
        : "v"(ring_addr + uint32_t(slot * kSlotBytes))
        : "memory");
  };
  auto read_a = [&](i32x4 (&a)[MG], int s) {
    const uint32_t base = a_addr + uint32_t(s) * (MG * 1024u);
#pragma unroll
    for (int mt = 0; mt < MG; ++mt)
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=&v"(a[mt]) : "v"(base), "n"(mt * 1024) : "memory");
  };

  // prologue: kRing-1 steps in flight, step 0's operands in registers
  for (int i = 0; i < kRing - 1; ++i) {
    if (!UNI) ptr_sync();
    dma_issue();
  }
  if (!UNI) ptr_sync();
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (kRing - 2)) : "memory");
  uint32_t xc[4], xn[4];
  i32x4 ac[MG], an[MG];
  read_x(xc, 0);
  read_a(ac, 0);
  lgkm_wait();
#pragma unroll
  for (int i = 0; i < 4; ++i) tie(xc[i]);
#pragma unroll
  for (int mt = 0; mt < MG; ++mt) tie(ac[mt]);

  int r_slot = 0;
  for (int ci = 0; ci < my_chunks; ++ci) {
    f32x16 acc[MG][kNTW];
#pragma unroll
    for (int mt = 0; mt < MG; ++mt)
#pragma unroll
      for (int t = 0; t < kNTW; ++t) acc[mt][t] = (f32x16)(0.0f);
    for (int s = 0; s < ksteps; ++s) {
      // (1) the DMA kRing-1 steps ahead; (2) step s+1's ring bytes and A fragments (its slot is
      // the oldest of the kRing-1 pairs in flight); (3) this step's expansion + MFMAs; (4) retire
      // the reads of (2). Reads past the last step hit valid LDS and are discarded.
      dma_issue();
      if (!UNI) ptr_async();
      const int slot1 = r_slot + 1 == kRing ? 0 : r_slot + 1;
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (kRing - 2)) : "memory");
      read_x(xn, slot1);
      read_a(an, s + 1 == ksteps ? 0 : s + 1);
      __builtin_amdgcn_sched_barrier(0);

      const int rbase = 8 * s + 4 * h;
      const uint32_t xs[4] = {rbase < k ? xc[0] : 0u, rbase + 1 < k ? xc[1] : 0u, rbase + 2 < k ? xc[2] : 0u,
                              rbase + 3 < k ? xc[3] : 0u};
      i32x8 b[kNTW];
#pragma unroll
      for (int t = 0; t < kNTW; ++t) {
#pragma unroll
        for (int i = 0; i < 4; ++i) b[t][i] = expand_fp4((xs[i] >> (8 * t)) & 0xFFu);
#pragma unroll
        for (int i = 4; i < 8; ++i) b[t][i] = 0;
      }
#pragma unroll
      for (int mt = 0; mt < MG; ++mt) {
        const i32x8 a = {ac[mt][0], ac[mt][1], ac[mt][2], ac[mt][3], 0, 0, 0, 0};
#pragma unroll
        for (int t = 0; t < kNTW; ++t)
          acc[mt][t] =
              __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b[t], acc[mt][t], 4, 4, 0, scale, 0, scale);
      }
      r_slot = slot1;
      __builtin_amdgcn_sched_barrier(0);
      lgkm_wait();
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        tie(xn[i]);
        xc[i] = xn[i];
      }
#pragma unroll
      for (int mt = 0; mt < MG; ++mt) {
        tie(an[mt]);
        ac[mt] = an[mt];
      }
      if (!UNI) {
        tie(pn0);
        tie(pn1);
      }
    }
    const int64_t colw = col0 + (slot0 + int64_t(ci) * chunk_slots) * kBlockCols + wave * 64 + 2 * c;
#pragma unroll
    for (int mt = 0; mt < MG; ++mt)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint64_t op = outptr[4 * mt + 2 * h + u];
        if (!op) continue;
        const uint32_t w = pack_byte(acc[mt][0], u) | (pack_byte(acc[mt][1], u) << 8);
        *(gptr<uint16_t>)(op + colw) = uint16_t(w);
      }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA (dummy or not) outlives the wave
}

struct Fp4Geometry {
  int ksteps, mtiles, mg, groups;
  size_t lds;
};

Fp4Geometry geometry(int k, int m, int mg_cap) {
  Fp4Geometry g{};
  g.ksteps = (k + 7) / 8;
  g.mtiles = (m + 3) / 4;
  // MG = M-tiles per block: next power of two >= mtiles (<= 8, the accumulator budget), halved
  // until the block's A slice fits the LDS
  g.mg = 1;
  while (g.mg < g.mtiles && g.mg < mg_cap) g.mg <<= 1;
  while (g.mg > 1 && g.mg * g.ksteps > kMaxLdsKiB) g.mg >>= 1;
  g.groups = (g.mtiles + g.mg - 1) / g.mg;
  g.lds = size_t(g.mg) * g.ksteps * 64 * 16 + 2304 + 4 * (kRing + 1) * kSlotBytes;
  return g;
}

template <int MG, bool UNI>
hipError_t launch_fp4(const Fp4Geometry& geo, cptr<uint64_t> in, cptr<uint64_t> out, const void* bitmat, int k, int m,
                      int64_t col0, int64_t nchunks, int64_t in_stride, hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gf_gemm_fp4_kernel<MG, UNI>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  // one block per CU in total (the LDS holds the whole A slice), chunk slots a multiple of 8
  int64_t slots = std::max<int64_t>(8, (256 / geo.groups) / 8 * 8);
  slots = std::min<int64_t>(slots, (nchunks + 7) / 8 * 8);
  const unsigned blocks = unsigned(slots * geo.groups);
  gf_gemm_fp4_kernel<MG, UNI><<<blocks, 256, geo.lds, stream>>>(in, out, static_cast<const i32x4*>(bitmat), k, m,
                                                                geo.ksteps, geo.groups, col0, nchunks, slots,
                                                                in_stride);
  return hipGetLastError();
}

template <int MG>
hipError_t launch_fp4_any(const Fp4Geometry& geo, cptr<uint64_t> in, cptr<uint64_t> out, const void* bitmat, int k,
                          int m, int64_t col0, int64_t nchunks, int64_t in_stride, hipStream_t stream) {
  return in_stride ? launch_fp4<MG, true>(geo, in, out, bitmat, k, m, col0, nchunks, in_stride, stream)
                   : launch_fp4<MG, false>(geo, in, out, bitmat, k, m, col0, nchunks, 0, stream);
}

}  // namespace

size_t fp4_bitmat_bytes(int k, int m, int mg_cap) {
  const Fp4Geometry g = geometry(k, m, mg_cap);
  return size_t(g.groups) * g.mg * g.ksteps * 64 * 16;
}

hipError_t launch_fp4_bitmat(const uint8_t* coeff, int m, int k, void* bitmat, int mg_cap, hipStream_t stream) {
  if (m <= 0 || k <= 0 || m > 256 || k > 256 || mg_cap < 1) return hipErrorInvalidValue;
  const Fp4Geometry g = geometry(k, m, mg_cap);
  const int64_t total = int64_t(fp4_bitmat_bytes(k, m, mg_cap));
  const int blocks = int(std::min<int64_t>((total + 255) / 256, 4096));
  fp4_bitmat_kernel<<<blocks, 256, 0, stream>>>(coeff, m, k, g.ksteps, g.mg, g.groups, static_cast<uint8_t*>(bitmat));
  return hipGetLastError();
}

hipError_t launch_gf_gemm_fp4(const void* bitmat, const void* desc, int k, int m, int64_t col0, int64_t ncols,
                              int mg_cap, int64_t in_stride, hipStream_t stream) {
  if (k <= 0 || m <= 0 || ncols < 0 || (col0 & 1) || mg_cap < 1) return hipErrorInvalidValue;
  const int m_pad = pad_m(m);
  const DescLayout l = desc_layout(k, m_pad);
  const char* b = static_cast<const char*>(desc);
  const Fp4Geometry geo = geometry(k, m, mg_cap);
  const int64_t nchunks = ncols / kBlockCols;
  if (nchunks > 0) {
    const auto in = (cptr<uint64_t>)(b + l.in_off);
    const auto out = (cptr<uint64_t>)(b + l.out_off);
    hipError_t e;
    switch (geo.mg) {
      case 8: e = launch_fp4_any<8>(geo, in, out, bitmat, k, m, col0, nchunks, in_stride, stream); break;
      case 4: e = launch_fp4_any<4>(geo, in, out, bitmat, k, m, col0, nchunks, in_stride, stream); break;
      case 2: e = launch_fp4_any<2>(geo, in, out, bitmat, k, m, col0, nchunks, in_stride, stream); break;
      default: e = launch_fp4_any<1>(geo, in, out, bitmat, k, m, col0, nchunks, in_stride, stream); break;
    }
    if (e != hipSuccess) return e;
  }
  const int64_t done = nchunks * kBlockCols;
  if (done < ncols) return launch_gf_gemm(desc, k, m_pad, col0 + done, ncols - done, false, 0, stream);
  return hipSuccess;
}

}  // namespace gfrs

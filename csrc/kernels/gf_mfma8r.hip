// GF(2^8) on the FP4 matrix cores, register-streamed: the gf_mfma16.hip design (eight waves per
// block sharing an LDS A slice, input rows through registers with one buffer resource per K-step,
// a branch-free load pipeline, per-step LDS pointer tables, copies spread over the M-tile groups)
// carried back to bytes. Read gf_mfma_fp4.hip's header first for the engine itself (e2m1 operands,
// biased-float parity epilogue); gf_mfma16.hip's for the register pipeline.
//
// The LDS-ring kernels of gf_mfma_fp4.hip stream input through LDS-DMA slots with one wave per
// SIMD, hand-scheduled; their wide decode with fused copies sat at 56 % MFMA pipe (k = 128, 26
// rebuilt + 102 copied, profiles/wide_stripe/r03_final). Here two waves per SIMD hide each other's
// bookkeeping, as they did for GF(2^16) (36 -> 66 %, profiles/gf65536/r08_mfma16).
//
// Operands. A lane reads one 16-bit word of each of 4 input rows per K-step: bytes 2c and 2c+1 of
// its wave's 64-byte column span, rows 8s + 4h + i. Its B operands are the bit planes of the two
// byte columns (sub-block j = byte 2c + j; gf_mfma16.hip's expand16<0> gathers both at once). One A
// fragment per M-tile and K-step (the 8 x 8 maps of 4 output rows x 8 input rows), shared by both
// sub-blocks: 2 MFMAs per (M-tile, K-step), MG M-tiles per block (acc = MG x 2 x 16 VGPRs).
//
// Reference: the GF-GEMM of /root/reference/src/matrix.cu:232-323 (encode_chunk / decode_chunk's
// kernel, one byte column per thread, LDS log/exp tables); the decode's survivor copy is the host
// memcpy of /root/reference/src/decode.cu:335-408, fused here into the GEMM pass.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "gfrs/desc.h"
#include "gfrs/device_cache.h"
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

constexpr int kWaveBytes = 64;  // byte columns per wave (2 per lane)
constexpr int kWaves = 8;       // per block: two per SIMD, sharing the LDS A slice
constexpr int kThreads = 64 * kWaves;
constexpr int kChunkBytes = kWaves * kWaveBytes;  // per block and chunk
constexpr int kDepth = 6;                         // K-steps of input in flight per lane
constexpr int kSinkBytes = 64 * 1024;             // write-only sink after the bit-matrix
constexpr int kRsrcWord3 = 0x00020000;            // raw buffer resource, dword 3 on gfx9
constexpr int kLoadNT = 2;                        // streamed input: non-temporal

__host__ __device__ constexpr int out_row_of(int r) { return 2 * ((r >> 2) & 1) + (r >> 4); }
__host__ __device__ constexpr int out_bit_of(int r) { return ((r >> 3) & 1) * 4 + (r & 3); }
constexpr uint8_t kAOne[4] = {0x4, 0x2, 0x1, 0x1};  // reciprocal weights of the B planes

__device__ __forceinline__ uint32_t mul_pow2(uint32_t c, int e) {  // c * 2^e in GF(2^8), poly 0x11D
  for (int i = 0; i < e; ++i) c = (c & 0x80u) ? ((c << 1) ^ 0x11Du) : (c << 1);
  return c;
}

// Bit-matrix layout: [pass][group][step < S][mt < MG][lane < 64][16 B]; nibble j of a lane's 16 bytes
// <-> input row 8 (pass S + s) + 4 h + ((j & 7) >> 1), bit (j >> 3) + 4 (j & 1); output row
// 4 (g MG + mt) + out_row_of(r), bit out_bit_of(r). Coefficient (o, i) = coeff[row(o) * ld + i],
// row(o) = sel ? sel[o] : o.
__global__ void fp8r_bitmat_kernel(const uint8_t* __restrict__ coeff, int ld, const int* __restrict__ sel, int m,
                                   int k, int S, int mg, int groups, int passes, uint8_t* __restrict__ bitmat) {
  const int64_t total = int64_t(passes) * groups * S * mg * 64 * 16;
  for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < total;
       idx += int64_t(gridDim.x) * blockDim.x) {
    const int q = int(idx & 15);
    const int lane = int((idx >> 4) & 63);
    int64_t rest = idx >> 10;
    const int mt = int(rest % mg);
    rest /= mg;
    const int s = int(rest % S);
    rest /= S;
    const int g = int(rest % groups);
    const int pass = int(rest / groups);
    const int r = lane & 31, h = lane >> 5;
    const int orow = 4 * (g * mg + mt) + out_row_of(r);
    const int obit = out_bit_of(r);
    uint8_t v = 0;
    for (int half = 0; half < 2; ++half) {
      const int j = 2 * q + half;
      const int dq = j >> 3, jj = j & 7;
      const int irow = 8 * (pass * S + s) + 4 * h + (jj >> 1);
      const int ibit = dq + 4 * (jj & 1);
      if (orow < m && irow < k) {
        const uint32_t c = coeff[size_t(sel ? sel[orow] : orow) * ld + irow];
        if ((mul_pow2(c, ibit) >> obit) & 1u) v |= uint8_t(kAOne[dq] << (4 * half));
      }
    }
    bitmat[idx] = v;
  }
}

__device__ __forceinline__ uint32_t bfi(uint32_t mask, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(mask), "v"(a), "v"(b));
  return r;
}
// (see gf_mfma16.hip: the inline-asm epilogue reads accumulator VGPRs, which the compiler's hazard
// recognizer does not track; scripts/mfma_hazard_check.py lints the emitted code)
__device__ __forceinline__ void mfma_result_fence() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7");
  __builtin_amdgcn_sched_barrier(0);
}

// B operands of the lane's two byte columns from the 4 rows' 16-bit words (low halves of x):
// bo[j] = bit planes of (x0.bj, x1.bj, x2.bj, x3.bj)
__device__ __forceinline__ void expand8(i32x4 (&bo)[2], const uint32_t (&x)[4]) {
  const uint32_t p01 = __builtin_amdgcn_perm(x[1], x[0], 0x05040100u);
  const uint32_t p23 = __builtin_amdgcn_perm(x[3], x[2], 0x05040100u);
  const uint32_t w[2] = {__builtin_amdgcn_perm(p23, p01, 0x06040200u), __builtin_amdgcn_perm(p23, p01, 0x07050301u)};
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    bo[t][0] = int(w[t] & 0x11111111u);
    bo[t][1] = int(w[t] & 0x22222222u);
    bo[t][2] = int(w[t] & 0x44444444u);
    bo[t][3] = int((w[t] >> 1) & 0x44444444u);
  }
}

// MG: M-tiles per block; UNI: input row r at in[0] + r * in_stride (8 in_stride <= 2^31); COPY:
// fused survivor copies; ACC: XOR into the outputs (K passes after the first; k <= 255 fits one pass
// at MG <= 4, kept for generality). nchunks counts whole chunks plus, when tail_bytes > 0, one last
// partial chunk of that many bytes.
template <int MG, bool UNI, bool COPY, bool ACC>
__global__ __launch_bounds__(kThreads, 1) void gf_gemm_fp4r_kernel(cptr<uint64_t> in, cptr<uint64_t> out,
                                                                   cptr<uint64_t> copy,
                                                                   const i32x4* __restrict__ bitmat, int k, int m,
                                                                   int row0, int S, int groups, int64_t col0,
                                                                   int64_t nchunks, int64_t chunk_slots,
                                                                   int64_t in_stride, uint64_t sink, int tail_bytes) {
  extern __shared__ __attribute__((aligned(16))) i32x4 afrag[];  // [S][MG][64]
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int local = bid >> 3;
  const int g = local % groups;
  const int64_t slot0 = int64_t(local / groups) * 8 + xcd;
  if (slot0 >= chunk_slots) return;
  const int my_chunks = int((nchunks - slot0 + chunk_slots - 1) / chunk_slots);
  if (my_chunks <= 0) return;
  const size_t a_frags = size_t(S) * MG * 64;
  const i32x4* src = bitmat + size_t(g) * a_frags;
  for (size_t i = threadIdx.x; i < a_frags; i += kThreads) afrag[i] = src[i];
  // pointer inputs / copies: per-step row tables after the A slice (itab[s][j] = in[min(row, k-1)],
  // ctab[s][j] = copy[row] or 0, row = row0 + 8 s + j)
  uint64_t* itab = reinterpret_cast<uint64_t*>(afrag + a_frags);
  uint64_t* ctab = itab + (UNI ? 0 : 8 * S);
  if constexpr (!UNI || COPY) {
    for (int i = threadIdx.x; i < 8 * S; i += kThreads) {
      const int row = row0 + i;
      if constexpr (!UNI) itab[i] = in[min(row, k - 1)];
      if constexpr (COPY) ctab[i] = row < k ? copy[row] : 0;
    }
  }
  __syncthreads();

  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63, h = lane >> 5, c = lane & 31;
  const int scale = 0x7F7F7F7F;  // E8M0 1.0
  const int bias_scale = 127 + 23 - out_bit_of(lane & 31);
  const i32x8 one_k0 = {h == 0 ? 0x2 : 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t optr[MG][2];  // output rows 4 (g MG + mt) + 2h + u (padding rows: the sink)
#pragma unroll
  for (int mt = 0; mt < MG; ++mt)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int row = 4 * (g * MG + mt) + 2 * h + u;
      optr[mt][u] = row < m ? out[row] : 0;
    }
  const uint64_t my_sink = sink + uint64_t(((bid * kWaves + wave) % 256) * 256 + 2 * c);
  const uint64_t in0 = UNI ? in[0] : 0;
  const int lane_off = wave * kWaveBytes + 2 * c;
  const int tail_valid = min(2, max(0, tail_bytes - lane_off));  // the lane's bytes of the partial chunk
  const int part_rel =
      (tail_bytes > 0 && (nchunks - 1 - slot0) % chunk_slots == 0) ? int((nchunks - 1 - slot0) / chunk_slots) : -1;
  const int my_full = my_chunks - (part_rel >= 0 ? 1 : 0);
  const int64_t chunk_step = chunk_slots * kChunkBytes;
  const int64_t wave_col0 = col0 + slot0 * kChunkBytes + int64_t(wave) * kWaveBytes;
  uint32_t voff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) voff[i] = uint32_t((4 * h + i) * in_stride) + uint32_t(2 * c);
  auto load_masked = [&](uint64_t addr, int nv) __attribute__((always_inline)) -> uint32_t {
    if (nv == 2) return uint32_t(__builtin_nontemporal_load((gptr<const uint16_t>)addr));
    if (nv == 1) return uint32_t(*(gptr<const uint8_t>)addr);
    return 0u;
  };
  auto store_masked = [&](uint64_t addr, uint32_t v, int nv) __attribute__((always_inline)) {
    if (nv == 2)
      *(gptr<uint16_t>)addr = uint16_t(v);
    else if (nv == 1)
      *(gptr<uint8_t>)addr = uint8_t(v);
  };

  f32x16 acc[MG][2];  // [tile][byte column]
  auto bias_init = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int mt = 0; mt < MG; ++mt)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        int bs = bias_scale;  // (opaque: identical MFMAs must not be merged or hoisted)
        asm volatile("" : "+v"(bs));
        acc[mt][j] =
            __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(one_k0, one_k0, (f32x16)(0.0f), 4, 4, 0, bs, 0, scale);
      }
  };

  // load cursor (uniform): chunk lc, step ls; past the whole chunks loads read zeros / the sink
  int lc = 0, ls = 0;
  int64_t lcol = wave_col0;
  uint64_t lbase = UNI ? in0 + uint64_t(int64_t(row0) * in_stride + lcol) : 0;
  const uint64_t step_bytes = UNI ? uint64_t(8 * in_stride) : 0;
  [[maybe_unused]] uint64_t loff = uint64_t(lcol) + 2 * c;
  auto load_step = [&](uint32_t (&x)[4]) __attribute__((always_inline)) {
    const int rbase = row0 + 8 * ls;
    const bool live = lc < my_full;
    if constexpr (UNI) {
      const int rem = live ? k - rbase : 0;
      const int nrec = __builtin_amdgcn_readfirstlane(
          rem >= 8 ? int(uint32_t(8) * uint32_t(in_stride)) : rem > 0 ? int(uint32_t(rem) * uint32_t(in_stride)) : 0);
      const uint64_t b = (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int(lbase >> 32)))) << 32) |
                         uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(lbase))));
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(b), 0, nrec, kRsrcWord3);
#pragma unroll
      for (int i = 0; i < 4; ++i) x[i] = __builtin_amdgcn_raw_buffer_load_b16(rs, int(voff[i]), 0, kLoadNT);
      lbase += step_bytes;
    } else {
      const i32x4* tp = reinterpret_cast<const i32x4*>(itab + 8 * ls + 4 * h);
      const i32x4 q0 = tp[0], q1 = tp[1];
      const uint64_t p[4] = {uint64_t(uint32_t(q0[0])) | (uint64_t(uint32_t(q0[1])) << 32),
                             uint64_t(uint32_t(q0[2])) | (uint64_t(uint32_t(q0[3])) << 32),
                             uint64_t(uint32_t(q1[0])) | (uint64_t(uint32_t(q1[1])) << 32),
                             uint64_t(uint32_t(q1[2])) | (uint64_t(uint32_t(q1[3])) << 32)};
#pragma unroll
      for (int i = 0; i < 4; ++i)
        x[i] = __builtin_nontemporal_load((gptr<const uint16_t>)(live ? p[i] + loff : my_sink));
    }
    if (++ls == S) {
      ls = 0;
      ++lc;
      lcol += chunk_step;
      if constexpr (UNI) lbase = in0 + uint64_t(int64_t(row0) * in_stride + lcol);
      if constexpr (!UNI) loff = uint64_t(lcol) + 2 * c;
    }
  };

  int cc = 0, cs = 0;  // compute cursor
  int64_t ccol = wave_col0;
  [[maybe_unused]] int cturn = 0;  // COPY: this group stores step cs's copies when cturn == g
  [[maybe_unused]] uint32_t old[MG][2] = {};
  auto chunk_start = [&]() __attribute__((always_inline)) {
    if constexpr (ACC) {
      const bool live = cc < my_full;
#pragma unroll
      for (int mt = 0; mt < MG; ++mt)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const uint64_t o = optr[mt][u];
          old[mt][u] = __builtin_nontemporal_load((gptr<const uint16_t>)(live && o ? o + uint64_t(ccol) + 2 * c : my_sink));
        }
    }
    if constexpr (COPY) cturn = 0;
  };
  auto consume = [&](const uint32_t (&x)[4], int nv) __attribute__((always_inline)) {
    i32x4 af[MG];
#pragma unroll
    for (int mt = 0; mt < MG; ++mt) af[mt] = afrag[(cs * MG + mt) * 64 + lane];
    if constexpr (COPY) {  // the steps' survivor copies, round-robin over the groups
      if (cturn == g) {
        const i32x4* tp = reinterpret_cast<const i32x4*>(ctab + 8 * cs + 4 * h);
        const i32x4 q0 = tp[0], q1 = tp[1];
        const uint64_t cp[4] = {uint64_t(uint32_t(q0[0])) | (uint64_t(uint32_t(q0[1])) << 32),
                                uint64_t(uint32_t(q0[2])) | (uint64_t(uint32_t(q0[3])) << 32),
                                uint64_t(uint32_t(q1[0])) | (uint64_t(uint32_t(q1[1])) << 32),
                                uint64_t(uint32_t(q1[2])) | (uint64_t(uint32_t(q1[3])) << 32)};
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (cp[i]) store_masked(cp[i] + uint64_t(ccol) + 2 * c, x[i], nv);
      }
      cturn = cturn + 1 == groups ? 0 : cturn + 1;
    }
    i32x4 e[2];
    expand8(e, x);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int mt = 0; mt < MG; ++mt) {
        const i32x8 a = {af[mt][0], af[mt][1], af[mt][2], af[mt][3], 0, 0, 0, 0};
        const i32x8 b = {e[j][0], e[j][1], e[j][2], e[j][3], 0, 0, 0, 0};
        acc[mt][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc[mt][j], 4, 4, 0, scale, 0, scale);
      }
    if (++cs == S) {  // chunk done: pack, store, restart the accumulators
      mfma_result_fence();
#pragma unroll
      for (int mt = 0; mt < MG; ++mt) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          uint32_t y[2];
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            uint32_t v = __float_as_uint(acc[mt][j][8 * u]);
#pragma unroll
            for (int b = 1; b < 8; ++b) v = bfi(1u << b, __float_as_uint(acc[mt][j][8 * u + b]), v);
            y[j] = v;
          }
          uint32_t w = __builtin_amdgcn_perm(y[1], y[0], 0x0c0c0400u);  // (byte 2c, byte 2c + 1)
          if constexpr (ACC) w ^= old[mt][u];
          const uint64_t o = optr[mt][u];
          store_masked(o ? o + uint64_t(ccol) + 2 * c : my_sink, w, o ? nv : 2);
        }
      }
      bias_init();
      cs = 0;
      ++cc;
      ccol += chunk_step;
      chunk_start();
    }
  };

  bias_init();
  chunk_start();
  const int total_steps = my_full * S;
  uint32_t ring[kDepth][4];
#pragma unroll
  for (int d = 0; d < kDepth; ++d) load_step(ring[d]);
  for (int t0 = 0; t0 < total_steps; t0 += kDepth) {
#pragma unroll
    for (int d = 0; d < kDepth; ++d) {
      if (t0 + d >= total_steps) break;  // (uniform)
      uint32_t x[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) x[i] = ring[d][i];
      load_step(ring[d]);
      consume(x, 2);
    }
  }
  if (part_rel >= 0) {  // the partial chunk: per-lane masked loads
    if constexpr (ACC) {
#pragma unroll
      for (int mt = 0; mt < MG; ++mt)
#pragma unroll
        for (int u = 0; u < 2; ++u)
          old[mt][u] = optr[mt][u] ? load_masked(optr[mt][u] + uint64_t(ccol) + 2 * c, tail_valid) : 0u;
    }
    for (int s = 0; s < S; ++s) {
      uint32_t x[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = min(row0 + 8 * s + 4 * h + i, k - 1);
        const uint64_t base = UNI ? in0 + uint64_t(int64_t(r) * in_stride) : itab[r - row0];
        x[i] = load_masked(base + uint64_t(ccol) + 2 * c, tail_valid);
      }
      consume(x, tail_valid);
    }
  }
}

struct GeoR {
  int ksteps, mtiles, mg, groups, passes, S;
  size_t lds;
};

// M-tiles per block (mg in 1..4; the plan fixes it, since the bit-matrix layout depends on it)
GeoR geometry_r(int k, int m, int mg) {
  GeoR g{};
  g.ksteps = (k + 7) / 8;
  g.mtiles = (m + 3) / 4;
  g.mg = std::max(1, std::min({mg, 4, g.mtiles}));
  constexpr size_t kLds = 160 * 1024;
  const int smax = std::max(1, int(kLds / (size_t(g.mg) * 1024 + 128)));
  g.passes = (g.ksteps + smax - 1) / smax;
  g.S = (g.ksteps + g.passes - 1) / g.passes;
  g.groups = (g.mtiles + g.mg - 1) / g.mg;
  g.lds = size_t(g.S) * g.mg * 1024 + 2 * 64 * size_t(g.S);
  return g;
}

size_t bitmat_r_bytes(const GeoR& g) { return size_t(g.passes) * g.groups * g.S * g.mg * 64 * 16; }

template <int MG, bool UNI, bool COPY, bool ACC>
hipError_t launch_r_pass(const GeoR& geo, cptr<uint64_t> in, cptr<uint64_t> out, cptr<uint64_t> copy,
                         const uint8_t* bitmat, int k, int m, int pass, int64_t col0, int64_t nchunks,
                         int64_t in_stride, uint64_t sink, int tail, hipStream_t stream) {
  const void* f = reinterpret_cast<const void*>(&gf_gemm_fp4r_kernel<MG, UNI, COPY, ACC>);
  hipError_t e = ensure_lds_optin(f);
  if (e != hipSuccess) return e;
  static DeviceMemo<size_t, int> occ_memo;
  const int occ = occ_memo.get_or(geo.lds, [&] {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, f, kThreads, geo.lds) != hipSuccess) o = 0;
    return o;
  });
  if (occ <= 0) return hipErrorInvalidConfiguration;
  const int64_t slots = persistent_slots(std::min(occ, 4), geo.groups, nchunks);
  const unsigned blocks = unsigned(slots * geo.groups);
  const i32x4* bm = reinterpret_cast<const i32x4*>(bitmat) + size_t(pass) * geo.groups * geo.S * MG * 64;
  gf_gemm_fp4r_kernel<MG, UNI, COPY, ACC><<<blocks, kThreads, geo.lds, stream>>>(
      in, out, copy, bm, k, m, pass * 8 * geo.S, geo.S, geo.groups, col0, nchunks, slots, in_stride, sink, tail);
  return hipGetLastError();
}

template <int MG>
hipError_t launch_r_mg(const GeoR& geo, cptr<uint64_t> in, cptr<uint64_t> out, cptr<uint64_t> copy,
                       const uint8_t* bitmat, int k, int m, int64_t col0, int64_t nchunks, int64_t in_stride,
                       uint64_t sink, int tail, hipStream_t stream) {
  for (int p = 0; p < geo.passes; ++p) {
    const bool acc = p > 0;
    hipError_t e;
    if (copy) {
      e = acc ? launch_r_pass<MG, false, true, true>(geo, in, out, copy, bitmat, k, m, p, col0, nchunks, 0, sink, tail, stream)
              : launch_r_pass<MG, false, true, false>(geo, in, out, copy, bitmat, k, m, p, col0, nchunks, 0, sink, tail, stream);
    } else if (in_stride) {
      e = acc ? launch_r_pass<MG, true, false, true>(geo, in, out, copy, bitmat, k, m, p, col0, nchunks, in_stride, sink,
                                                     tail, stream)
              : launch_r_pass<MG, true, false, false>(geo, in, out, copy, bitmat, k, m, p, col0, nchunks, in_stride, sink,
                                                      tail, stream);
    } else {
      e = acc ? launch_r_pass<MG, false, false, true>(geo, in, out, copy, bitmat, k, m, p, col0, nchunks, 0, sink, tail, stream)
              : launch_r_pass<MG, false, false, false>(geo, in, out, copy, bitmat, k, m, p, col0, nchunks, 0, sink, tail,
                                                       stream);
    }
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace

int fp4r_choose_mg(int k, int m) {
  (void)k;
  const char* e = std::getenv("GFRS_FP4R_MG");  // (read per plan, not per launch)
  const int forced = e ? std::atoi(e) : 0;
  if (forced >= 1 && forced <= 4) return forced;
  // the widest grouping with no padded M-tile, else one tile per block
  const int tiles = (m + 3) / 4;
  for (int cand : {4, 3, 2})
    if (tiles % cand == 0) return cand;
  return 1;
}

size_t fp4r_bitmat_bytes(int k, int m, int mg) { return bitmat_r_bytes(geometry_r(k, m, mg)) + kSinkBytes; }

hipError_t launch_fp4r_bitmat(const uint8_t* coeff, int ld, const int* sel, int m, int k, void* bitmat, int mg,
                              hipStream_t stream) {
  if (m <= 0 || k <= 0 || m > 256 || k > 256 || ld < k || mg < 1) return hipErrorInvalidValue;
  const GeoR g = geometry_r(k, m, mg);
  const int64_t total = int64_t(bitmat_r_bytes(g));
  const int blocks = int(std::min<int64_t>((total + 255) / 256, 8192));
  fp8r_bitmat_kernel<<<blocks, 256, 0, stream>>>(coeff, ld, sel, m, k, g.S, g.mg, g.groups, g.passes,
                                                 static_cast<uint8_t*>(bitmat));
  return hipGetLastError();
}

hipError_t launch_gf_gemm_fp4r(const void* bitmat, const void* desc, int k, int m, int64_t col0, int64_t ncols,
                               int mg, int64_t in_stride, bool copies, hipStream_t stream) {
  if (k <= 0 || m <= 0 || ncols < 0 || (col0 & 1) || mg < 1) return hipErrorInvalidValue;
  const int m_pad = pad_m(m);
  const DescLayout l = desc_layout(k, m_pad);
  const char* b = static_cast<const char*>(desc);
  const GeoR geo = geometry_r(k, m, mg);
  const int64_t full = ncols / kChunkBytes;
  const int tail = int(ncols % kChunkBytes);
  const int64_t nchunks = full + (tail ? 1 : 0);
  if (nchunks == 0) return hipSuccess;
  const int64_t stride = (copies || in_stride <= 0 || in_stride > (int64_t(1) << 28)) ? 0 : in_stride;
  if (!stride && col0 + ncols + kChunkBytes > (int64_t(1) << 32))
    return launch_gf_gemm(desc, k, m_pad, col0, ncols, false, 0, stream, copies);
  cptr<uint64_t> in = (cptr<uint64_t>)(b + l.in_off);
  cptr<uint64_t> out = (cptr<uint64_t>)(b + l.out_off);
  cptr<uint64_t> copy = copies ? (cptr<uint64_t>)(b + l.copy_off) : nullptr;
  const uint64_t sink = reinterpret_cast<uint64_t>(bitmat) + bitmat_r_bytes(geo);
  const auto* bm = static_cast<const uint8_t*>(bitmat);
  switch (geo.mg) {
    case 4: return launch_r_mg<4>(geo, in, out, copy, bm, k, m, col0, nchunks, stride, sink, tail, stream);
    case 3: return launch_r_mg<3>(geo, in, out, copy, bm, k, m, col0, nchunks, stride, sink, tail, stream);
    case 2: return launch_r_mg<2>(geo, in, out, copy, bm, k, m, col0, nchunks, stride, sink, tail, stream);
    default: return launch_r_mg<1>(geo, in, out, copy, bm, k, m, col0, nchunks, stride, sink, tail, stream);
  }
}

}  // namespace gfrs

// GF(2^16) GEMM on gfx950 matrix cores: the FP4 (e2m1) GF(2) bit-matrix engine of gf_mfma_fp4.hip
// (read its header first: operand encoding, K order of the B expansion, biased-float parity
// epilogue) carried to 16-bit symbols.
//
// The reference's generic field code names w = 16 (/root/reference/src/galoisfield.cu:22-32, poly
// 0210013) but never built it; the v_perm kernel (gf_gemm16.hip) runs it on the VALU at ~0.23 TB/s
// for wide codes (k=300, m=40: 4.5 ms per GiB). Multiplication by c is a 16 x 16 GF(2) matrix, so
// a code's whole map is a (16m x 16k) bit-matrix and the GEMM is the same bit-matrix product as in
// GF(2^8), with twice the bit-MACs per byte.
//
// How 16-bit symbols meet the byte engine. A lane reads one dword of each of 4 input rows per
// K-step: symbols 2c and 2c+1 of its 64-symbol column group, little-endian (lo0 hi0 lo1 hi1). Its
// B operands are the gf_mfma_fp4.hip bit planes of 4 byte streams: sub-block j (symbol 2c+j) x
// byte plane t (lo, hi). With A split into the four byte-to-byte blocks of the 16 x 16 maps
// (f = 2 * src + dst: ll, lh, hl, hh — gfrs/gf65536.h perm_quad's order),
//     acc[j][lo] += A_ll . B[j][lo] + A_hl . B[j][hi]
//     acc[j][hi] += A_lh . B[j][lo] + A_hh . B[j][hi]
// — 4 MFMAs per (M-tile, sub-block, K-step), every A fragment shared by the two sub-blocks. An
// output dword (lo0 hi0 lo1 hi1 of one row) is packed from the four accumulators of (tile, u).
//
// K passes. A whole column of the bit-matrix does not fit the LDS for wide codes (one M-tile of 4
// output symbols x k=300 is 150 KiB of FP4 nibbles), so the K rows are split into passes of S
// K-steps (8 input rows each), one launch per pass: pass 0 stores its partial outputs, every later
// pass XORs into them (launch boundaries order the passes). Within a pass a persistent block holds
// its M-tile group's A slice (S x MG x 4 KiB) in LDS for all of its chunks; the group's blocks of
// one chunk share an XCD (the input re-read per group is an L2 hit).
//
// Input rows stream through registers (4 dword loads per lane and K-step, kDepth steps in flight
// across chunk boundaries); rows past k read zeros (buffer bounds) or are clamped to row k-1, and
// meet zero bit-matrix columns either way. Eight waves per block (two per SIMD) share the A slice:
// one wave's bookkeeping and load waits issue under the other's MFMAs. Fused survivor copies
// (decode): the store of K-step s's raw dwords goes to group s mod groups, so no group's blocks
// carry all of them.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "gfrs/desc.h"
#include "gfrs/device_cache.h"
#include "gfrs/kernels.h"
#include "gfrs/tune.h"

namespace gfrs {
namespace {

using i32x8 = int __attribute__((ext_vector_type(8)));
using i32x4 = int __attribute__((ext_vector_type(4)));
using f32x16 = float __attribute__((ext_vector_type(16)));
template <typename T>
using cptr = const __attribute__((address_space(4))) T*;
template <typename T>
using gptr = __attribute__((address_space(1))) T*;

constexpr int kWaveBytes = 128;  // byte columns per wave: 64 symbols (2 per lane)
constexpr int kWaves = 8;        // per block: two per SIMD, sharing the LDS A slice
constexpr int kThreads = 64 * kWaves;
constexpr int kChunkBytes = kWaves * kWaveBytes;  // per block and chunk
constexpr int kDepth = 4;                  // K-steps of input in flight per lane
constexpr int kSinkBytes16 = 64 * 1024;    // write-only sink after the bit-matrix (padding outputs)
constexpr uint32_t kPoly16 = 0x1100Bu;
constexpr int kRsrcWord3 = 0x00020000;  // raw buffer resource, dword 3 on gfx9 (32-bit data format)
constexpr int kLoadNT = 2;              // cache policy of the streamed input: slc (non-temporal)

__host__ __device__ constexpr int out_row_of(int r) { return 2 * ((r >> 2) & 1) + (r >> 4); }
__host__ __device__ constexpr int out_bit_of(int r) { return ((r >> 3) & 1) * 4 + (r & 3); }
constexpr uint8_t kAOne[4] = {0x4, 0x2, 0x1, 0x1};  // reciprocal weights of the B planes (gf_mfma_fp4.hip)

__device__ __forceinline__ uint32_t xtime16(uint32_t x) {
  x <<= 1;
  return (x & 0x10000u) ? (x ^ kPoly16) : x;
}
// c * 2^e in GF(2^16)
__device__ __forceinline__ uint32_t mul_pow2(uint32_t c, int e) {
  for (int i = 0; i < e; ++i) c = xtime16(c);
  return c;
}

// Bit-matrix layout: [pass][group][step < S][mt < MG][f < 4][lane < 64][16 B]; nibble j of a lane's
// 16 bytes <-> input symbol row row0 + 8 s + 4 h + ((j & 7) >> 1), bit (j >> 3) + 4 (j & 1) of byte
// plane src; output row 4 (g MG + mt) + out_row_of(r), bit out_bit_of(r) of byte plane dst
// (f = 2 src + dst). Coefficient (o, i) = coeff[row(o) * ld + i], row(o) = sel ? sel[o] : o.
__global__ void fp16_bitmat_kernel(const uint16_t* __restrict__ coeff, int ld, const int* __restrict__ sel, int m,
                                   int k, int S, int mg, int groups, int passes, uint8_t* __restrict__ bitmat) {
  const int64_t total = int64_t(passes) * groups * S * mg * 4 * 64 * 16;
  for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < total;
       idx += int64_t(gridDim.x) * blockDim.x) {
    const int q = int(idx & 15);
    const int lane = int((idx >> 4) & 63);
    int64_t rest = idx >> 10;
    const int f = int(rest & 3);
    rest >>= 2;
    const int mt = int(rest % mg);
    rest /= mg;
    const int s = int(rest % S);
    rest /= S;
    const int g = int(rest % groups);
    const int pass = int(rest / groups);
    const int src = f >> 1, dst = f & 1;
    const int r = lane & 31, h = lane >> 5;
    const int orow = 4 * (g * mg + mt) + out_row_of(r);
    const int obit = out_bit_of(r) + 8 * dst;
    uint8_t v = 0;
    for (int half = 0; half < 2; ++half) {
      const int j = 2 * q + half;
      const int dq = j >> 3, jj = j & 7;
      const int irow = 8 * (pass * S + s) + 4 * h + (jj >> 1);
      const int ibit = dq + 4 * (jj & 1) + 8 * src;
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
// The epilogue's v_bfi (inline asm) reads accumulator VGPRs, and the compiler's hazard recognizer
// does not look into inline asm: nothing crosses this point, and the last 16-pass MFMA gets its
// wait states before the first read (scripts/mfma_hazard_check.py lints the emitted code).
__device__ __forceinline__ void mfma_result_fence() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ int bias_scale_of_lane(int lane) { return 127 + 23 - out_bit_of(lane & 31); }

// B operands of sub-block j (symbol 2c + j) from the 4 rows' dwords: bytes 2j (lo) and 2j + 1 (hi)
// of x0..x3 gathered per plane (3 v_perm), then the bit planes masked in place (gf_mfma_fp4.hip).
template <int J>
__device__ __forceinline__ void expand16(i32x4 (&bo)[2], const uint32_t (&x)[4]) {
  constexpr uint32_t sel = J == 0 ? 0x05040100u : 0x07060302u;  // (x_a.b2j, x_a.b2j+1, x_b.b2j, x_b.b2j+1)
  const uint32_t p01 = __builtin_amdgcn_perm(x[1], x[0], sel);
  const uint32_t p23 = __builtin_amdgcn_perm(x[3], x[2], sel);
  const uint32_t w[2] = {__builtin_amdgcn_perm(p23, p01, 0x06040200u), __builtin_amdgcn_perm(p23, p01, 0x07050301u)};
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    bo[t][0] = int(w[t] & 0x11111111u);
    bo[t][1] = int(w[t] & 0x22222222u);
    bo[t][2] = int(w[t] & 0x44444444u);
    bo[t][3] = int((w[t] >> 1) & 0x44444444u);
  }
}

// MG: M-tiles (4 output symbol rows each) per block; UNI: input row r at in[0] + r * in_stride (8 *
// in_stride <= 2^31: a lane's rows sit at 32-bit offsets from the step's first row), else row
// pointers from the descriptor (columns below 2^32); COPY: fused survivor copies; ACC: XOR into the
// outputs (passes after the first). nchunks counts whole chunks plus, when tail_bytes > 0, one last
// partial chunk of that many bytes (lanes past it load zeros and store nothing).
//
// Issue budget. A wave's step is 8 MG MFMAs (32 cycles each); with two waves per SIMD every
// instruction the step issues besides them costs issue slots, so the per-step bookkeeping is a few
// scalar adds on uniform cursors (no 64-bit multiplies, one buffer resource per step), the
// bounds of the pass's last rows come from the resource's num_records (rows past k read zeros),
// and only the partial chunk takes the per-lane masked path.
template <int MG, bool UNI, bool COPY, bool ACC>
__global__ __launch_bounds__(kThreads, 1) void gf_gemm16_fp4_kernel(cptr<uint64_t> in, cptr<uint64_t> out,
                                                                    cptr<uint64_t> copy,
                                                                    const i32x4* __restrict__ bitmat, int k, int m,
                                                                    int row0, int S, int groups, int64_t col0,
                                                                    int64_t nchunks, int64_t chunk_slots,
                                                                    int64_t in_stride, uint64_t sink, int tail_bytes,
                                                                    int64_t fps, int64_t in_bstride,
                                                                    int64_t out_bstride) {
  extern __shared__ __attribute__((aligned(16))) i32x4 afrag[];  // [S][MG][4][64]
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int local = bid >> 3;
  const int g = local % groups;
  const int64_t slot0 = int64_t(local / groups) * 8 + xcd;
  if (slot0 >= chunk_slots) return;
  const int my_chunks = int((nchunks - slot0 + chunk_slots - 1) / chunk_slots);
  if (my_chunks <= 0) return;
  const size_t a_frags = size_t(S) * MG * 4 * 64;
  const i32x4* src = bitmat + size_t(g) * a_frags;
  for (size_t i = threadIdx.x; i < a_frags; i += kThreads) afrag[i] = src[i];
  // pointer inputs / copies: the pass's row pointers as per-step tables after the A slice (a lane
  // reads its row half's 4 pointers with two LDS loads instead of 8 scalar loads whose latency
  // every step would wait out): itab[s][j] = in[min(row, k - 1)], ctab[s][j] = copy[row] or 0
  // for row = row0 + 8 s + j
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
  const int bias_scale = bias_scale_of_lane(lane);
  const i32x8 one_k0 = {h == 0 ? 0x2 : 0, 0, 0, 0, 0, 0, 0, 0};
  // output rows of this lane: 4 (g MG + mt) + 2h + u (padding rows -> the sink, never read)
  uint64_t optr[MG][2];
#pragma unroll
  for (int mt = 0; mt < MG; ++mt)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int row = 4 * (g * MG + mt) + 2 * h + u;
      optr[mt][u] = row < m ? out[row] : 0;
    }
  const uint64_t my_sink = sink + uint64_t(((bid * kWaves + wave) % 256) * 256 + 4 * c);
  const uint64_t in0 = UNI ? in[0] : 0;
  const int lane_off = wave * kWaveBytes + 4 * c;  // byte offset inside a chunk
  // this lane's valid bytes (4, 2 or 0) in a partial chunk (the last of each stripe when the
  // columns end tail_bytes into a chunk)
  const int tail_valid = min(4, max(0, tail_bytes - lane_off));
  // chunk q of the launch is chunk q % fps of stripe q / fps (batched launches: fps chunks per
  // stripe, rows at fixed strides from stripe 0's). A cursor keeps (stripe, chunk) and steps by
  // chunk_slots without dividing (one division, here).
  const int64_t db = chunk_slots / fps, dch = chunk_slots - db * fps;
  const int64_t b_first = slot0 / fps, ch_first = slot0 - b_first * fps;
  // a cursor: chunk ch of stripe b, its wave column col and stripe byte offset soff (at stride
  // bstride); one step adds chunk_slots chunks with adds and one compare
  const int64_t dcol = dch * kChunkBytes, fcol = fps * kChunkBytes;
  auto advance = [&](int64_t& ch, int64_t& col, int64_t& soff, int64_t bstride) __attribute__((always_inline)) {
    ch += dch;
    col += dcol;
    soff += db * bstride;
    if (ch >= fps) {
      ch -= fps;
      col -= fcol;
      soff += bstride;
    }
  };
  auto col_of = [&](int64_t ch) __attribute__((always_inline)) {  // the wave's first byte column
    return col0 + ch * kChunkBytes + int64_t(wave) * kWaveBytes;
  };
  // the lane's valid bytes of chunk ch of a stripe: 4, or tail_valid in the partial chunk
  auto valid_of = [&](int64_t ch) __attribute__((always_inline)) {
    return (tail_bytes > 0 && ch == fps - 1) ? tail_valid : 4;
  };
  // UNI: the lane's 4 rows as 32-bit offsets from the step's first row (a lane past the columns of
  // a partial chunk: an offset past num_records, so it reads zeros)
  uint32_t voff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) voff[i] = uint32_t((4 * h + i) * in_stride) + uint32_t(4 * c);
  auto store_masked = [&](uint64_t addr, uint32_t v, int nv) __attribute__((always_inline)) {
    if (nv == 4)
      *(gptr<uint32_t>)addr = v;
    else if (nv == 2)
      *(gptr<uint16_t>)addr = uint16_t(v);
  };

  f32x16 acc[MG][2][2];  // [tile][sub-block][plane]
  auto bias_init = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int mt = 0; mt < MG; ++mt)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          int bs = bias_scale;  // (opaque: identical MFMAs must not be merged or hoisted)
          asm volatile("" : "+v"(bs));
          acc[mt][j][t] =
              __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(one_k0, one_k0, (f32x16)(0.0f), 4, 4, 0, bs, 0, scale);
        }
  };

  // Every chunk runs through one software pipeline whose loads never sit in a branch (a
  // conditional load makes the ring slots merge values, and every merge copy waits for all loads
  // in flight): loads past the block's last chunk read zeros (UNI: num_records 0) or the sink, and
  // a partial chunk's lanes past the columns read zeros / the sink through per-lane state set once
  // per chunk (a dword holding 2 valid bytes is read whole: its other 2 lie in the same word).
  // load cursor (uniform): chunk lc, step ls; rows row0 + 8 ls + 4h + i; UNI: lbase = the step's
  // first row at the wave's column
  int lc = 0, ls = 0;
  int64_t lch = ch_first, lcol = col_of(lch), lsoff = b_first * in_bstride;
  const uint64_t lrow0 = UNI ? in0 + uint64_t(int64_t(row0) * in_stride) : 0;
  uint64_t lbase = UNI ? lrow0 + uint64_t(lsoff + lcol) : 0;
  const uint64_t step_bytes = UNI ? uint64_t(8 * in_stride) : 0;
  // pointer inputs: the lane's byte in stripe 0's row pointers
  [[maybe_unused]] uint64_t loff = uint64_t(lsoff + lcol) + 4 * c;
  bool lok = valid_of(lch) > 0;  // this lane reads the load cursor's chunk
  uint32_t voffc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) voffc[i] = lok ? voff[i] : 0x80000000u;
  auto load_step = [&](uint32_t (&x)[4]) __attribute__((always_inline)) {
    const int rbase = row0 + 8 * ls;
    const bool live = lc < my_chunks;
    if constexpr (UNI) {  // one raw buffer resource; rows past k fall outside num_records and read 0
      // (readfirstlane: the resource is provably uniform, no waterfall)
      const int rem = live ? k - rbase : 0;
      const int nrec = __builtin_amdgcn_readfirstlane(
          rem >= 8 ? int(uint32_t(8) * uint32_t(in_stride)) : rem > 0 ? int(uint32_t(rem) * uint32_t(in_stride)) : 0);
      const uint64_t b = (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int(lbase >> 32)))) << 32) |
                         uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(lbase))));
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(b), 0, nrec, kRsrcWord3);
#pragma unroll
      for (int i = 0; i < 4; ++i) x[i] = __builtin_amdgcn_raw_buffer_load_b32(rs, int(voffc[i]), 0, kLoadNT);
      lbase += step_bytes;
    } else {  // the lane's 4 row pointers from the LDS table (two 16-byte reads)
      const i32x4* tp = reinterpret_cast<const i32x4*>(itab + 8 * ls + 4 * h);
      const i32x4 q0 = tp[0], q1 = tp[1];
      const uint64_t p[4] = {uint64_t(uint32_t(q0[0])) | (uint64_t(uint32_t(q0[1])) << 32),
                             uint64_t(uint32_t(q0[2])) | (uint64_t(uint32_t(q0[3])) << 32),
                             uint64_t(uint32_t(q1[0])) | (uint64_t(uint32_t(q1[1])) << 32),
                             uint64_t(uint32_t(q1[2])) | (uint64_t(uint32_t(q1[3])) << 32)};
#pragma unroll
      for (int i = 0; i < 4; ++i)
        x[i] = __builtin_nontemporal_load((gptr<const uint32_t>)(live && lok ? p[i] + loff : my_sink));
    }
    if (++ls == S) {
      ls = 0;
      ++lc;
      advance(lch, lcol, lsoff, in_bstride);
      if constexpr (UNI) lbase = lrow0 + uint64_t(lsoff + lcol);
      if constexpr (!UNI) loff = uint64_t(lsoff + lcol) + 4 * c;
      lok = valid_of(lch) > 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) voffc[i] = lok ? voff[i] : 0x80000000u;
    }
  };

  // compute cursor (uniform): chunk cc, step cs, wave column ccol, the lane's valid bytes cnv
  int cc = 0, cs = 0;
  int64_t cch = ch_first, ccol = col_of(cch);
  int64_t csoff = b_first * out_bstride;  // the chunk's stripe offset of outputs and copies
  uint64_t cout = uint64_t(csoff);
  int cnv = valid_of(cch);
  [[maybe_unused]] int cturn = 0;  // COPY: this group stores step cs's copies when cturn == g
  [[maybe_unused]] uint32_t old[MG][2] = {};
  auto chunk_start = [&]() __attribute__((always_inline)) {
    if constexpr (ACC) {  // the previous passes' outputs of the chunk, read S steps ahead of their use
      const bool live = cc < my_chunks && cnv > 0;
#pragma unroll
      for (int mt = 0; mt < MG; ++mt)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const uint64_t o = optr[mt][u];
          old[mt][u] =
              __builtin_nontemporal_load((gptr<const uint32_t>)(live && o ? o + cout + uint64_t(ccol) + 4 * c : my_sink));
        }
    }
    if constexpr (COPY) cturn = 0;
  };
  // one K-step on the 4 input dwords x
  auto consume = [&](const uint32_t (&x)[4]) __attribute__((always_inline)) {
    i32x4 af[MG][4];
#pragma unroll
    for (int mt = 0; mt < MG; ++mt)
#pragma unroll
      for (int f = 0; f < 4; ++f) af[mt][f] = afrag[((cs * MG + mt) * 4 + f) * 64 + lane];
    if constexpr (COPY) {  // the steps' survivor copies, spread round-robin over the groups
      if (cturn == g) {
        const i32x4* tp = reinterpret_cast<const i32x4*>(ctab + 8 * cs + 4 * h);
        const i32x4 q0 = tp[0], q1 = tp[1];
        const uint64_t cp[4] = {uint64_t(uint32_t(q0[0])) | (uint64_t(uint32_t(q0[1])) << 32),
                                uint64_t(uint32_t(q0[2])) | (uint64_t(uint32_t(q0[3])) << 32),
                                uint64_t(uint32_t(q1[0])) | (uint64_t(uint32_t(q1[1])) << 32),
                                uint64_t(uint32_t(q1[2])) | (uint64_t(uint32_t(q1[3])) << 32)};
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (cp[i]) store_masked(cp[i] + cout + uint64_t(ccol) + 4 * c, x[i], cnv);
      }
      cturn = cturn + 1 == groups ? 0 : cturn + 1;
    }
    i32x4 e[2][2];  // [sub-block][plane]
    expand16<0>(e[0], x);
    expand16<1>(e[1], x);
    // all lo-plane products, then all hi-plane ones: an accumulator's two MFMAs of the step are
    // 4 MG apart, never back to back
#pragma unroll
    for (int sp = 0; sp < 2; ++sp)
#pragma unroll
      for (int mt = 0; mt < MG; ++mt)
#pragma unroll
        for (int dst = 0; dst < 2; ++dst) {
          const i32x4 a4 = af[mt][2 * sp + dst];
          const i32x8 a = {a4[0], a4[1], a4[2], a4[3], 0, 0, 0, 0};
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const i32x8 b = {e[j][sp][0], e[j][sp][1], e[j][sp][2], e[j][sp][3], 0, 0, 0, 0};
            acc[mt][j][dst] =
                __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc[mt][j][dst], 4, 4, 0, scale, 0, scale);
          }
        }
    if (++cs == S) {  // chunk done: pack, store, restart the accumulators
      mfma_result_fence();
#pragma unroll
      for (int mt = 0; mt < MG; ++mt) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          uint32_t y[2][2];  // [sub-block][plane]: the byte in bits 0..7
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int t = 0; t < 2; ++t) {
              uint32_t v = __float_as_uint(acc[mt][j][t][8 * u]);
#pragma unroll
              for (int b = 1; b < 8; ++b) v = bfi(1u << b, __float_as_uint(acc[mt][j][t][8 * u + b]), v);
              y[j][t] = v;
            }
          // (lo0, hi0, lo1, hi1)
          uint32_t w = __builtin_amdgcn_perm(__builtin_amdgcn_perm(y[1][1], y[1][0], 0x0c0c0400u),
                                             __builtin_amdgcn_perm(y[0][1], y[0][0], 0x0c0c0400u), 0x05040100u);
          if constexpr (ACC) w ^= old[mt][u];
          const uint64_t o = optr[mt][u];
          store_masked(o ? o + cout + uint64_t(ccol) + 4 * c : my_sink, w, o ? cnv : 4);
        }
      }
      bias_init();
      cs = 0;
      ++cc;
      advance(cch, ccol, csoff, out_bstride);
      cout = uint64_t(csoff);
      cnv = valid_of(cch);
      chunk_start();
    }
  };

  bias_init();
  chunk_start();
  const int total_steps = my_chunks * S;
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
      load_step(ring[d]);  // kDepth steps ahead (past the block's chunks: zeros / the sink)
      consume(x);
    }
  }
}

struct Geo16 {
  int ksteps, mtiles, mg, groups, passes, S;
  size_t lds;
};

// M-tiles per block MG (<= mg_cap, power of two while it pays) and passes of S K-steps so one
// group's A slice plus its pointer tables fit the LDS.
Geo16 geometry16(int k, int m, int mg_cap, bool copy) {
  Geo16 g{};
  g.ksteps = (k + 7) / 8;
  g.mtiles = (m + 3) / 4;
  // MG in {2, 1} (<= mg_cap): the fewest padded M-tiles, then the wider (GFRS_TUNE=fp16_mg=N forces one).
  // (MG = 4 — 256 accumulator registers beside the unrolled input ring — spilled ~2 KiB per lane.)
  static const int forced = int(tune_int("fp16_mg", 0));
  g.mg = 1;
  for (int cand : {2, 1}) {
    if (cand > mg_cap || (forced && cand != forced)) continue;
    const int padded = (g.mtiles + cand - 1) / cand * cand;
    const int best = (g.mtiles + g.mg - 1) / g.mg * g.mg;
    if (g.mg == 1 || padded < best) g.mg = cand;
    if (forced) break;
  }
  constexpr size_t kLds = 160 * 1024;
  // per K-step: A (mg x 4 KiB) and 8 row + 8 copy pointers
  auto fit_steps = [&](int mg) { return int(kLds / (size_t(mg) * 4096 + 128)); };
  while (g.mg > 1 && fit_steps(g.mg) < 1) g.mg >>= 1;
  const int smax = std::max(1, fit_steps(g.mg));
  g.passes = (g.ksteps + smax - 1) / smax;
  g.S = (g.ksteps + g.passes - 1) / g.passes;
  g.groups = (g.mtiles + g.mg - 1) / g.mg;
  g.lds = size_t(g.S) * g.mg * 4096 + 2 * 64 * size_t(g.S);  // A slice + row / copy pointer tables
  (void)copy;
  return g;
}

size_t bitmat16_matrix_bytes(const Geo16& g) { return size_t(g.passes) * g.groups * g.S * g.mg * 4 * 64 * 16; }

struct Args16 {
  cptr<uint64_t> in, out, copy;
  const uint8_t* bitmat;
  int k, m;
  int64_t col0, nchunks, in_stride;
  uint64_t sink;
  int tail;
  int64_t fps, in_bstride, out_bstride;  // batched: whole chunks per stripe, stripe strides
};

template <int MG, bool UNI, bool COPY, bool ACC>
hipError_t launch16_pass(const Geo16& geo, const Args16& a, int pass, hipStream_t stream) {
  const void* f = reinterpret_cast<const void*>(&gf_gemm16_fp4_kernel<MG, UNI, COPY, ACC>);
  hipError_t e = ensure_lds_optin(f);
  if (e != hipSuccess) return e;
  static DeviceMemo<size_t, int> occ_memo;
  const int occ = occ_memo.get_or(geo.lds, [&] {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, f, kThreads, geo.lds) != hipSuccess) o = 0;
    return o;
  });
  if (occ <= 0) return hipErrorInvalidConfiguration;
  const int64_t slots = persistent_slots(std::min(occ, 4), geo.groups, a.nchunks);
  const unsigned blocks = unsigned(slots * geo.groups);
  const i32x4* bm = reinterpret_cast<const i32x4*>(a.bitmat) + size_t(pass) * geo.groups * geo.S * MG * 4 * 64;
  gf_gemm16_fp4_kernel<MG, UNI, COPY, ACC><<<blocks, kThreads, geo.lds, stream>>>(
      a.in, a.out, a.copy, bm, a.k, a.m, pass * 8 * geo.S, geo.S, geo.groups, a.col0, a.nchunks, slots,
      UNI ? a.in_stride : 0, a.sink, a.tail, a.fps, a.in_bstride, a.out_bstride);
  return hipGetLastError();
}

template <int MG>
hipError_t launch16_mg(const Geo16& geo, const Args16& a, hipStream_t stream) {
  for (int p = 0; p < geo.passes; ++p) {
    hipError_t e;
    const bool acc = p > 0;
    if (a.copy) {
      e = acc ? launch16_pass<MG, false, true, true>(geo, a, p, stream)
              : launch16_pass<MG, false, true, false>(geo, a, p, stream);
    } else if (a.in_stride) {
      e = acc ? launch16_pass<MG, true, false, true>(geo, a, p, stream)
              : launch16_pass<MG, true, false, false>(geo, a, p, stream);
    } else {
      e = acc ? launch16_pass<MG, false, false, true>(geo, a, p, stream)
              : launch16_pass<MG, false, false, false>(geo, a, p, stream);
    }
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// The matrix-core launch over `batch` stripes' chunks: each stripe's whole chunks plus its ragged
// rest as one partial chunk
hipError_t launch16(const void* bitmat, const void* desc, int k, int m, int batch, int64_t col0, int64_t full,
                    int tail, int mg_cap, int64_t in_stride, int64_t in_bstride, int64_t out_bstride, bool copies,
                    hipStream_t stream) {
  const int m_pad = pad_m(m);
  const DescLayout l = desc_layout16(k, m_pad, batch);
  const char* b = static_cast<const char*>(desc);
  const Geo16 geo = geometry16(k, m, mg_cap, true);
  Args16 a{};
  a.in = (cptr<uint64_t>)(b + l.in_off);
  a.out = (cptr<uint64_t>)(b + l.out_off);
  a.copy = copies ? (cptr<uint64_t>)(b + l.copy_off) : nullptr;
  a.bitmat = static_cast<const uint8_t*>(bitmat);
  a.k = k;
  a.m = m;
  a.col0 = col0;
  a.fps = full + (tail ? 1 : 0);
  a.nchunks = a.fps * batch;
  // uniform-stride inputs address rows as the step's first row + 32-bit lane offsets (8 rows)
  a.in_stride = (copies || in_stride <= 0 || in_stride > (int64_t(1) << 28)) ? 0 : in_stride;
  a.sink = reinterpret_cast<uint64_t>(bitmat) + bitmat16_matrix_bytes(geo);
  a.tail = tail;
  a.in_bstride = in_bstride;
  a.out_bstride = out_bstride;
  if (a.nchunks == 0) return hipSuccess;
  return geo.mg == 2 ? launch16_mg<2>(geo, a, stream) : launch16_mg<1>(geo, a, stream);
}

}  // namespace

size_t fp16_bitmat_bytes(int k, int m, int mg_cap) {
  return bitmat16_matrix_bytes(geometry16(k, m, mg_cap, true)) + kSinkBytes16;
}

hipError_t launch_fp16_bitmat(const uint16_t* coeff, int ld, const int* sel, int m, int k, void* bitmat, int mg_cap,
                              hipStream_t stream) {
  if (m <= 0 || k <= 0 || m > 65535 || k > 65535 || mg_cap < 1 || ld < k) return hipErrorInvalidValue;
  const Geo16 g = geometry16(k, m, mg_cap, true);
  const int64_t total = int64_t(bitmat16_matrix_bytes(g));
  const int blocks = int(std::min<int64_t>((total + 255) / 256, 8192));
  fp16_bitmat_kernel<<<blocks, 256, 0, stream>>>(coeff, ld, sel, m, k, g.S, g.mg, g.groups, g.passes,
                                                 static_cast<uint8_t*>(bitmat));
  return hipGetLastError();
}

hipError_t launch_gf_gemm16_fp4(const void* bitmat, const void* desc, int k, int m, int64_t col0, int64_t ncols,
                                int mg_cap, int64_t in_stride, bool copies, hipStream_t stream) {
  if (k <= 0 || m <= 0 || ncols < 0 || ((col0 | ncols) & 1) || mg_cap < 1) return hipErrorInvalidValue;
  if (col0 & 3)  // a start off a 4-byte boundary: the v_perm records
    return ncols > 0 ? launch_gf_gemm16(desc, k, pad_m(m), col0, ncols, false, 0, stream) : hipSuccess;
  // whole chunks plus the ragged rest as one partial chunk, all on the matrix cores
  return launch16(bitmat, desc, k, m, 1, col0, ncols / kChunkBytes, int(ncols % kChunkBytes), mg_cap, in_stride, 0, 0,
                  copies, stream);
}

hipError_t launch_gf_gemm16_fp4_batched(const void* bitmat, const void* desc, int k, int m, int batch, int64_t col0,
                                        int64_t ncols, int mg_cap, int64_t in_stride, int64_t in_bstride,
                                        int64_t out_bstride, bool copies, hipStream_t stream) {
  if (k <= 0 || m <= 0 || ncols < 0 || ((col0 | ncols) & 1) || mg_cap < 1 || batch < 1 || batch > 65535)
    return hipErrorInvalidValue;
  if (batch == 1) return launch_gf_gemm16_fp4(bitmat, desc, k, m, col0, ncols, mg_cap, in_stride, copies, stream);
  if (col0 & 3)  // a start off a 4-byte boundary: the batched v_perm kernel
    return launch_gf_gemm16_batched(desc, k, pad_m(m), batch, col0, ncols, false, 0, stream);
  // every stripe's whole chunks and its partial one, all in one launch per K pass
  return launch16(bitmat, desc, k, m, batch, col0, ncols / kChunkBytes, int(ncols % kChunkBytes), mg_cap, in_stride,
                  in_bstride, out_bstride, copies, stream);
}

}  // namespace gfrs

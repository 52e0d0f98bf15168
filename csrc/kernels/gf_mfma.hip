// GF(2^8) GEMM on gfx950 matrix cores: int8 MFMA over GF(2) bit-matrices (BASELINE config #5,
// the wide k=128, n=160 stripe).
//
// Multiplication by a constant c is GF(2)-linear on the 8 bits of a byte, i.e. an 8x8 bit-matrix,
// so an (m x k) GF(2^8) GEMM is an (8m x 8k) GF(2) GEMM: out_bits = A . in_bits (mod 2).
// `v_mfma_i32_32x32x32_i8` with {0,1} operands computes the integer sums; bit 0 of each i32
// accumulator is the GF(2) result (cdna_hip_programming.md §3). The reference has no counterpart
// (its only GEMM is the log/exp byte kernel, src/matrix.cu:232-407).
//
// Shapes per wave and K-step (4 input rows = 32 K bits):
//   * A fragments (16 x i8 per lane, 1 KiB per wave per M-tile) are precomputed once per coefficient
//     matrix (launch_mfma_bitmat) and staged into LDS per block: the block's 2 M-tiles x k/4 K-steps.
//   * B fragments: lane (c = l & 31, h = l >> 5) loads one dword (4 columns) from each of input rows
//     4s+2h and 4s+2h+1 and expands byte t of both into 16 {0,1} bytes for N-tile t (4 N-tiles =
//     128 columns per wave): 6 VALU ops per byte, shared by both M-tiles.
//   * The K order inside a fragment is a private choice: A and B use the same (h, j) -> (row, bit)
//     map, which is all the MFMA needs (it pairs A and B element j of the same lane half).
//   * Output-bit placement: MFMA row r holds output row 2*((r>>2)&1) + (r>>4), bit ((r>>3)&1)*4 +
//     (r&3). With the gfx950 C/D layout (row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)) every lane then
//     owns whole output bytes: 16 accumulators = 2 output rows x 8 bits, packed with no cross-lane
//     traffic and stored as one dword (4 N-tiles) per row.
// Blocks of the same column chunk and different M-groups are dealt to one XCD (T1) so the repeated
// input reads of the M-groups hit that XCD's L2.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "gfrs/desc.h"
#include "gfrs/device_cache.h"
#include "gfrs/kernels.h"

namespace gfrs {
namespace {

using i32x4 = int __attribute__((ext_vector_type(4)));
using i32x16 = int __attribute__((ext_vector_type(16)));
template <typename T>
using cptr = const __attribute__((address_space(4))) T*;
template <typename T>
using gptr = __attribute__((address_space(1))) T*;

constexpr int kMTW = 2;   // M-tiles (32 output bits = 4 output rows each) per wave
constexpr int kNT = 4;    // N-tiles (32 columns) per wave
constexpr int kCols = 512;  // columns per block iteration (4 waves x 128)

__constant__ Tables d_tab = make_tables();

__device__ __forceinline__ uint8_t dmul(uint8_t a, uint8_t b) { return d_tab.exp[d_tab.log[a] + d_tab.log[b]]; }

// Output (row-in-M-tile, bit) of MFMA row r; see file comment.
__host__ __device__ constexpr int out_row_of(int r) { return 2 * ((r >> 2) & 1) + (r >> 4); }
__host__ __device__ constexpr int out_bit_of(int r) { return ((r >> 3) & 1) * 4 + (r & 3); }

// bitmat layout: [group][mt][kstep][lane][16 bytes]
__global__ void mfma_bitmat_kernel(const uint8_t* __restrict__ coeff, int m, int k, int ksteps, int groups,
                                   uint8_t* __restrict__ bitmat) {
  const int64_t total = int64_t(groups) * kMTW * ksteps * 64 * 16;
  for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < total;
       idx += int64_t(gridDim.x) * blockDim.x) {
    const int j = int(idx & 15);
    const int lane = int((idx >> 4) & 63);
    int64_t rest = idx >> 10;
    const int s = int(rest % ksteps);
    rest /= ksteps;
    const int mt = int(rest % kMTW);
    const int g = int(rest / kMTW);
    const int r = lane & 31, h = lane >> 5;
    const int orow = 8 * g + 4 * mt + out_row_of(r);
    const int obit = out_bit_of(r);
    const int irow = 4 * s + 2 * h + (j >> 3);
    const int ibit = j & 7;
    uint8_t v = 0;
    if (orow < m && irow < k) v = (dmul(coeff[size_t(orow) * k + irow], uint8_t(1u << ibit)) >> obit) & 1;
    bitmat[idx] = v;
  }
}

__device__ __forceinline__ uint32_t spread4(uint32_t nib) { return (nib * 0x00204081u) & 0x01010101u; }

// B fragment for N-tile t: bits of byte t of x0 (elements 0..7) and of x1 (elements 8..15).
__device__ __forceinline__ i32x4 expand(uint32_t x0, uint32_t x1, int t) {
  i32x4 b;
  b[0] = int(spread4(__builtin_amdgcn_ubfe(x0, 8 * t, 4)));
  b[1] = int(spread4(__builtin_amdgcn_ubfe(x0, 8 * t + 4, 4)));
  b[2] = int(spread4(__builtin_amdgcn_ubfe(x1, 8 * t, 4)));
  b[3] = int(spread4(__builtin_amdgcn_ubfe(x1, 8 * t + 4, 4)));
  return b;
}

// Output byte u (0/1) of one accumulator tile: bits from regs 8u .. 8u+7.
__device__ __forceinline__ uint32_t pack_byte(const i32x16& acc, int u) {
  uint32_t v = 0;
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int low = 0; low < 4; ++low) v |= (uint32_t(acc[4 * (2 * u + q) + low]) & 1u) << (q * 4 + low);
  return v;
}

__global__ __launch_bounds__(256, 2) void gf_gemm_mfma_kernel(cptr<uint64_t> in, cptr<uint64_t> out,
                                                              const i32x4* __restrict__ bitmat, int k, int m,
                                                              int ksteps, int groups, int64_t col0,
                                                              int64_t nchunks, int64_t chunk_slots) {
  extern __shared__ __attribute__((aligned(16))) i32x4 afrag[];  // [kMTW][ksteps][64]
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int local = bid >> 3;
  const int g = local % groups;
  const int64_t slot = int64_t(local / groups) * 8 + xcd;
  if (slot >= chunk_slots) return;

  const i32x4* src = bitmat + size_t(g) * kMTW * ksteps * 64;
  for (int i = threadIdx.x; i < kMTW * ksteps * 64; i += 256) afrag[i] = src[i];
  __syncthreads();

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  for (int64_t chunk = slot; chunk < nchunks; chunk += chunk_slots) {
    const int64_t colw = col0 + chunk * kCols + wave * 128 + 4 * c;  // this lane's 4 columns
    i32x16 acc[kMTW][kNT];
#pragma unroll
    for (int mt = 0; mt < kMTW; ++mt)
#pragma unroll
      for (int t = 0; t < kNT; ++t) acc[mt][t] = (i32x16)(0);

    uint32_t n0 = 0, n1 = 0;
    {
      const int r0 = 2 * h;
      if (r0 < k) n0 = *(gptr<const uint32_t>)(in[r0] + colw);
      if (r0 + 1 < k) n1 = *(gptr<const uint32_t>)(in[r0 + 1] + colw);
    }
    for (int s = 0; s < ksteps; ++s) {
      const uint32_t x0 = n0, x1 = n1;
      if (s + 1 < ksteps) {  // prefetch the next K-step
        const int r0 = 4 * (s + 1) + 2 * h;
        n0 = r0 < k ? *(gptr<const uint32_t>)(in[r0] + colw) : 0u;
        n1 = r0 + 1 < k ? *(gptr<const uint32_t>)(in[r0 + 1] + colw) : 0u;
      }
      i32x4 a[kMTW];
#pragma unroll
      for (int mt = 0; mt < kMTW; ++mt) a[mt] = afrag[(mt * ksteps + s) * 64 + lane];
#pragma unroll
      for (int t = 0; t < kNT; ++t) {
        const i32x4 b = expand(x0, x1, t);
#pragma unroll
        for (int mt = 0; mt < kMTW; ++mt)
          acc[mt][t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[mt], b, acc[mt][t], 0, 0, 0);
      }
    }
#pragma unroll
    for (int mt = 0; mt < kMTW; ++mt)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int row = 8 * g + 4 * mt + 2 * h + u;
        if (row >= m) continue;
        const uint64_t op = out[row];
        if (!op) continue;
        uint32_t w = 0;
#pragma unroll
        for (int t = 0; t < kNT; ++t) w |= pack_byte(acc[mt][t], u) << (8 * t);
        __builtin_nontemporal_store(w, (gptr<uint32_t>)(op + colw));
      }
  }
}

}  // namespace

size_t mfma_bitmat_bytes(int k, int m) {
  const int groups = (m + 7) / 8, ksteps = (k + 3) / 4;
  return size_t(groups) * kMTW * ksteps * 64 * 16;
}

hipError_t launch_mfma_bitmat(const uint8_t* coeff, int m, int k, void* bitmat, hipStream_t stream) {
  if (m <= 0 || k <= 0 || m > 256 || k > 256) return hipErrorInvalidValue;
  const int groups = (m + 7) / 8, ksteps = (k + 3) / 4;
  const int64_t total = int64_t(mfma_bitmat_bytes(k, m));
  const int blocks = int(std::min<int64_t>((total + 255) / 256, 4096));
  mfma_bitmat_kernel<<<blocks, 256, 0, stream>>>(coeff, m, k, ksteps, groups, static_cast<uint8_t*>(bitmat));
  return hipGetLastError();
}

// Columns [col0, col0 + ncols): the MFMA kernel covers whole 512-column chunks (rows must be 4-byte
// aligned); the remainder goes through the v_perm kernel, whose tables must then be present in
// `desc` (launch_perm_tables) — the caller builds both from one coefficient matrix.
hipError_t launch_gf_gemm_mfma(const void* bitmat, const void* desc, int k, int m, int64_t col0, int64_t ncols,
                               hipStream_t stream) {
  if (k <= 0 || m <= 0 || ncols < 0 || (col0 & 3)) return hipErrorInvalidValue;
  const int m_pad = pad_m(m);
  const DescLayout l = desc_layout(k, m_pad);
  const char* b = static_cast<const char*>(desc);
  const int groups = (m + 7) / 8, ksteps = (k + 3) / 4;
  const int64_t nchunks = ncols / kCols;
  if (nchunks > 0) {
    // ~2 blocks per CU in total, chunk slots a multiple of 8 (one per XCD lane of the mapping)
    int64_t slots = std::max<int64_t>(8, (512 / groups) / 8 * 8);
    slots = std::min<int64_t>(slots, (nchunks + 7) / 8 * 8);
    const size_t lds = size_t(kMTW) * ksteps * 64 * 16;
    if (lds > 65536) {  // per device
      const hipError_t e = ensure_lds_optin(reinterpret_cast<const void*>(&gf_gemm_mfma_kernel));
      if (e != hipSuccess) return e;
    }
    const unsigned blocks = unsigned(slots * groups);
    gf_gemm_mfma_kernel<<<blocks, 256, lds, stream>>>(
        (cptr<uint64_t>)(b + l.in_off), (cptr<uint64_t>)(b + l.out_off), static_cast<const i32x4*>(bitmat), k, m,
        ksteps, groups, col0, nchunks, slots);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const int64_t done = nchunks * kCols;
  if (done < ncols) return launch_gf_gemm(desc, k, m_pad, col0 + done, ncols - done, false, 0, stream);
  return hipSuccess;
}

}  // namespace gfrs

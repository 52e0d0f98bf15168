// GF(2^8) GEMM with LDS lookup tables — the "LDS-LUT" path of BASELINE.json config #5, kept as an
// ablation next to the v_perm kernel (gf_gemm.hip) and the FP4 / int8 matrix-core kernels.
//
// The reference multiplies through log/exp tables copied into shared memory by every block
// (src/matrix.cu:38-39,250-262, three dependent lookups per byte product, src/matrix.cu:105-110).
// The north-star design names 4-bit nibble tables in LDS instead (cpu-rs-double.c's split,
// src/cpu-rs-double.c:52-55,164-222): for a coefficient c, lo[v] = c*v and hi[v] = c*(v << 4) for
// v < 16, so c*x = lo[x & 15] ^ hi[x >> 4] — two independent lookups per byte product.
//
// Layout: the block's output tile (MT rows) x all k inputs, 32 bytes per (input, output) pair
// ({lo[16], hi[16]}), built at block start from the descriptor's v_perm records (so every
// coefficient source — host matrix, device inverse, GF(16) maps — works unchanged). A lookup
// reads one byte of a 16-byte table: the 64 lanes of a ds_read_u8 touch at most 4 consecutive
// dwords (4 banks), which the LDS serves as broadcasts — conflict-free by construction.
// Per 16 input bytes and output row: 32 ds_read_u8 + 32 v_xor (v_perm: 12 v_perm + 6 v_bitop3).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "gfrs/desc.h"
#include "gfrs/device_cache.h"
#include "gfrs/kernels.h"

namespace gfrs {
namespace {

constexpr int kBlock = 256;
using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
template <typename T>
using cptr = const __attribute__((address_space(4))) T*;
template <typename T>
using gptr = __attribute__((address_space(1))) T*;

// Evaluate a v_perm record (gfrs::perm_apply) for one byte.
__device__ __forceinline__ uint32_t perm_eval(cptr<uint32_t> t, uint32_t x) {
  const uint32_t s0 = x & 7u, s1 = (x >> 3) & 7u, s2 = x >> 6;
  const uint32_t a = (s0 < 4 ? t[0] >> (8 * s0) : t[1] >> (8 * (s0 - 4))) & 0xFFu;
  const uint32_t b = (s1 < 4 ? t[2] >> (8 * s1) : t[3] >> (8 * (s1 - 4))) & 0xFFu;
  const uint32_t c = (t[4] >> (8 * s2)) & 0xFFu;
  return a ^ b ^ c;
}

template <int MT>
__global__ __launch_bounds__(kBlock) void gf_gemm_lut_kernel(const uint8_t* __restrict__ desc, int k, int m_pad,
                                                             int ntiles, int64_t col0, int64_t ngroups, int64_t nblk,
                                                             int64_t ncb) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lut[];  // [k][MT][32]
  const DescLayout l = desc_layout(k, m_pad);
  const cptr<uint64_t> in = (cptr<uint64_t>)(desc + l.in_off);
  const cptr<uint64_t> cpy = (cptr<uint64_t>)(desc + l.copy_off);
  const cptr<uint64_t> out = (cptr<uint64_t>)(desc + l.out_off);
  const cptr<uint32_t> tab = (cptr<uint32_t>)(desc + l.tab_off);
  const int bid = blockIdx.x;
  const int local = bid >> 3, xcd = bid & 7;  // output tiles of a column block on one XCD (gf_gemm.hip)
  const int tile = local % ntiles;
  const int64_t cb0 = int64_t(local / ntiles) * 8 + xcd;
  if (cb0 >= ncb) return;
  const int i0 = tile * MT;
  const bool do_copy = tile == 0;

  for (int e = threadIdx.x; e < k * MT * 32; e += kBlock) {
    const int v = e & 15, hi = (e >> 4) & 1, pair = e >> 5;  // pair = j * MT + i
    const int j = pair / MT, i = pair - j * MT;
    lut[e] = uint8_t(perm_eval(tab + (size_t(j) * m_pad + i0 + i) * kPermStride, hi ? uint32_t(v) << 4 : uint32_t(v)));
  }
  __syncthreads();

  for (int64_t cb = cb0; cb < nblk; cb += ncb) {
    const int64_t g = cb * kBlock + threadIdx.x;
    if (g >= ngroups) continue;
    const int64_t off = col0 + g * 16;
    uint32_t acc[MT][4];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int w = 0; w < 4; ++w) acc[i][w] = 0;
    u32x4 nxt = __builtin_nontemporal_load((gptr<const u32x4>)(in[0] + uint64_t(off)));
    for (int j = 0; j < k; ++j) {
      const u32x4 x = nxt;
      if (j + 1 < k) nxt = __builtin_nontemporal_load((gptr<const u32x4>)(in[j + 1] + uint64_t(off)));
      if (do_copy && cpy[j]) __builtin_nontemporal_store(x, (gptr<u32x4>)(cpy[j] + uint64_t(off)));
      const uint8_t* base = lut + size_t(j) * MT * 32;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const uint32_t byte = (x[w] >> (8 * b)) & 0xFFu;
          const uint32_t lo = byte & 15u, hi = 16u + (byte >> 4);
#pragma unroll
          for (int i = 0; i < MT; ++i)
            acc[i][w] ^= uint32_t(base[i * 32 + lo] ^ base[i * 32 + hi]) << (8 * b);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const uint64_t op = out[i0 + i];
      if (op) __builtin_nontemporal_store(u32x4{acc[i][0], acc[i][1], acc[i][2], acc[i][3]}, (gptr<u32x4>)(op + uint64_t(off)));
    }
  }
}

template <int MT>
hipError_t launch_lut(const void* desc, int k, int m_pad, int64_t col0, int64_t ncols, int64_t* done,
                      hipStream_t stream) {
  const int ntiles = m_pad / MT;
  const size_t lds = size_t(k) * MT * 32;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const void* f = reinterpret_cast<const void*>(&gf_gemm_lut_kernel<MT>);
  if (lds > 65536) {
    const hipError_t e = ensure_lds_optin(f, int(lds));
    if (e != hipSuccess) return e;
  }
  const int64_t ngroups = ncols / 16;
  *done = ngroups * 16;
  if (ngroups == 0) return hipSuccess;
  const int64_t nblk = (ngroups + kBlock - 1) / kBlock;
  // persistent-ish: enough blocks to fill every CU several times; each walks its column blocks
  int64_t ncb = std::min<int64_t>(nblk, 2048);
  ncb = (ncb + 7) / 8 * 8;
  gf_gemm_lut_kernel<MT><<<unsigned(ncb * ntiles), kBlock, lds, stream>>>(static_cast<const uint8_t*>(desc), k, m_pad,
                                                                          ntiles, col0, ngroups, nblk, ncb);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_gf_gemm_lut(const void* desc, int k, int m_pad, int64_t col0, int64_t ncols, hipStream_t stream) {
  if (k <= 0 || k > 256 || m_pad <= 0 || ncols < 0 || (col0 & 15) || m_pad % tile_for(m_pad)) return hipErrorInvalidValue;
  int64_t done = 0;
  hipError_t e;
  switch (tile_for(m_pad)) {
    case 1: e = launch_lut<1>(desc, k, m_pad, col0, ncols, &done, stream); break;
    case 2: e = launch_lut<2>(desc, k, m_pad, col0, ncols, &done, stream); break;
    case 4: e = launch_lut<4>(desc, k, m_pad, col0, ncols, &done, stream); break;
    case 8: e = launch_lut<8>(desc, k, m_pad, col0, ncols, &done, stream); break;
    default: e = launch_lut<16>(desc, k, m_pad, col0, ncols, &done, stream); break;
  }
  if (e != hipSuccess) return e;
  // the ragged tail (< 16 bytes) on the v_perm byte kernel
  if (done < ncols) return launch_gf_gemm(desc, k, m_pad, col0 + done, ncols - done, true, 0, stream);
  return hipSuccess;
}

}  // namespace gfrs

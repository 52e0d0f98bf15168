// Small device utilities around the GF-GEMM:
//   * gen_matrix   — coding-matrix generation on device (the reference's K3 `gen_encoding_matrix`,
//                    src/matrix.cu:752-759), one lane per element with bounds checks (K3 writes out of
//                    bounds when k or p > 16 and not a multiple of 16) and no per-thread
//                    table rebuild (K3 runs the serial setup_tables() in every thread).
//   * perm_tables  — coefficient matrix -> v_perm tables in a GEMM descriptor (device-side, so a
//                    matrix received by an RCCL broadcast never round-trips through the host).
//   * fill_random  — counter-based random bytes for synthetic benchmark input (16 B / lane stores).
//   * gather_rows  — decode-system assembly: rows of G selected by the surviving chunk ids
//                    (the reference's copy_matrix, src/decode.cu:75-81, done on the host).
#include <hip/hip_runtime.h>

#include "gfrs/desc.h"
#include "gfrs/kernels.h"

namespace gfrs {
namespace {

__constant__ Tables d_tab = make_tables();

__device__ __forceinline__ uint8_t dmul(uint8_t a, uint8_t b) { return d_tab.exp[d_tab.log[a] + d_tab.log[b]]; }

__global__ void gen_matrix_kernel(uint8_t* __restrict__ e, int k, int p, int kind) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= k * p) return;
  const int i = idx / k, j = idx % k;
  uint8_t v;
  if (kind == 1) {
    v = d_tab.inv[uint8_t((k + i) ^ j)];  // Cauchy 1/(x_i + y_j), x_i = k + i, y_j = j
  } else {
    // reference pow quirk: exp[(log a * e) % 255] with log(0) = 510 -> pow(0, e) = 1
    const unsigned a = unsigned((j + 1) % 256);
    v = d_tab.exp[(unsigned(d_tab.log[a]) * unsigned(i)) % 255u];
  }
  e[idx] = v;
}

__global__ void perm_tables_kernel(const uint8_t* __restrict__ coeff, int m, int k, uint32_t* __restrict__ tab,
                                   int m_pad) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= k * m_pad) return;
  const int j = idx / m_pad, i = idx % m_pad;
  uint32_t* rec = tab + size_t(idx) * kPermStride;
  if (i >= m) {
#pragma unroll
    for (int w = 0; w < kPermStride; ++w) rec[w] = 0;
    return;
  }
  const uint8_t c = coeff[size_t(i) * k + j];
  uint8_t basis[8];
#pragma unroll
  for (int b = 0; b < 8; ++b) basis[b] = dmul(c, uint8_t(1u << b));
  uint32_t w[5] = {0, 0, 0, 0, 0};
#pragma unroll
  for (int v = 0; v < 8; ++v) {
    uint8_t a = 0, bb = 0;
#pragma unroll
    for (int bit = 0; bit < 3; ++bit)
      if (v & (1 << bit)) {
        a ^= basis[bit];
        bb ^= basis[bit + 3];
      }
    w[v >> 2] |= uint32_t(a) << (8 * (v & 3));
    w[2 + (v >> 2)] |= uint32_t(bb) << (8 * (v & 3));
  }
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    uint8_t x = 0;
#pragma unroll
    for (int bit = 0; bit < 2; ++bit)
      if (v & (1 << bit)) x ^= basis[bit + 6];
    w[4] |= uint32_t(x) << (8 * v);
  }
#pragma unroll
  for (int q = 0; q < 5; ++q) rec[q] = w[q];
  rec[5] = rec[6] = rec[7] = 0;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void fill_random_kernel(uint8_t* __restrict__ dst, int64_t n16, int64_t tail,
                                                          uint64_t seed) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t g = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; g < n16; g += stride) {
    const uint64_t a = splitmix64(seed ^ (uint64_t(g) << 1));
    const uint64_t b = splitmix64(seed ^ ((uint64_t(g) << 1) | 1));
    reinterpret_cast<u32x4*>(dst)[g] = u32x4{uint32_t(a), uint32_t(a >> 32), uint32_t(b), uint32_t(b >> 32)};
  }
  if (blockIdx.x == 0 && threadIdx.x < tail) {
    const uint64_t a = splitmix64(seed ^ (uint64_t(n16) << 1) ^ 0xABCDull);
    dst[n16 * 16 + threadIdx.x] = uint8_t(a >> (8 * (threadIdx.x & 7)));
  }
}

__global__ void gather_rows_kernel(const uint8_t* __restrict__ g, const int* __restrict__ rows,
                                   uint8_t* __restrict__ out, int m, int k) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= m * k) return;
  const int i = idx / k, j = idx % k;
  out[idx] = g[size_t(rows[i]) * k + j];
}

}  // namespace

hipError_t launch_gen_matrix(uint8_t* e, int k, int p, int kind, hipStream_t stream) {
  if (k <= 0 || p <= 0) return hipErrorInvalidValue;
  const int n = k * p;
  gen_matrix_kernel<<<(n + 255) / 256, 256, 0, stream>>>(e, k, p, kind);
  return hipGetLastError();
}

hipError_t launch_perm_tables(const uint8_t* coeff, int m, int k, void* desc, int m_pad, hipStream_t stream) {
  if (m <= 0 || k <= 0 || m_pad < m) return hipErrorInvalidValue;
  uint32_t* tab = reinterpret_cast<uint32_t*>(static_cast<char*>(desc) + desc_layout(k, m_pad).tab_off);
  const int n = k * m_pad;
  perm_tables_kernel<<<(n + 255) / 256, 256, 0, stream>>>(coeff, m, k, tab, m_pad);
  return hipGetLastError();
}

hipError_t launch_fill_random(uint8_t* dst, int64_t bytes, uint64_t seed, hipStream_t stream) {
  if (bytes <= 0) return hipSuccess;
  if (reinterpret_cast<uintptr_t>(dst) & 15) return hipErrorInvalidValue;
  const int64_t n16 = bytes / 16;
  const int64_t tail = bytes % 16;
  int64_t blocks = (n16 + 255) / 256;
  if (blocks > 256 * 32) blocks = 256 * 32;
  if (blocks < 1) blocks = 1;
  fill_random_kernel<<<unsigned(blocks), 256, 0, stream>>>(dst, n16, tail, seed);
  return hipGetLastError();
}

hipError_t launch_gather_rows(const uint8_t* g, const int* rows, uint8_t* out, int m, int k, hipStream_t stream) {
  if (m <= 0 || k <= 0) return hipErrorInvalidValue;
  const int n = m * k;
  gather_rows_kernel<<<(n + 255) / 256, 256, 0, stream>>>(g, rows, out, m, k);
  return hipGetLastError();
}

}  // namespace gfrs

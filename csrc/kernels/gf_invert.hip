// Gauss-Jordan GF(2^8) matrix inverse on gfx950: one workgroup per matrix, [A|I] resident in LDS.
//
// Replaces the reference's GPU inversion family:
//   * `GPU_invert_matrix` (src/matrix.cu:666-744) launches 3-4 kernels per row and copies every
//     row back to the host to pick the pivot (src/matrix.cu:684); here the whole elimination is one
//     launch with the pivot search done by an LDS atomicMin — no host round trip, graph-capturable.
//   * `eliminate_by_row` (src/matrix.cu:525-556) has an inter-block race on the pivot column; here
//     the elimination factors are snapshotted into LDS (`flog`) behind a barrier before any row
//     is updated.
//   * Pivoting is by ROWS (the reference swaps columns and its result swap is a no-op,
//     src/matrix.cu:451-453 / src/cpu-decode.c:133-135, permuting decoded output — SURVEY §3.2),
//     and a column with no pivot reports `status = 1` instead of indexing column -1.
//   * The blocked 4x4 variant (src/decode-gj.cu:224-988, no pivoting, size % 4 == 0) is subsumed:
//     k <= 256 always fits one CU's LDS (2 * 256 * 256 B = 128 KiB of 160 KiB).
// Optionally the kernel also emits the v_perm tables of selected inverse rows straight into a
// GF-GEMM descriptor, so a decode is invert -> GEMM on one stream with zero host involvement.
#include <hip/hip_runtime.h>

#include "gfrs/desc.h"
#include "gfrs/kernels.h"

namespace gfrs {
namespace {

__constant__ Tables d_gf_tables = make_tables();


__device__ __forceinline__ uint8_t dmul_log(const uint8_t* exp_s, int la, int lb) { return exp_s[la + lb]; }

__device__ void perm_record(const uint8_t* exp_s, const uint16_t* log_s, uint8_t c, uint32_t* rec) {
  uint8_t basis[8];
#pragma unroll
  for (int b = 0; b < 8; ++b) basis[b] = exp_s[log_s[c] + log_s[1u << b]];
  uint8_t t0[8], t1[8], t2[4];
#pragma unroll
  for (int v = 0; v < 8; ++v) {
    uint8_t a = 0, bb = 0;
#pragma unroll
    for (int bit = 0; bit < 3; ++bit)
      if (v & (1 << bit)) {
        a ^= basis[bit];
        bb ^= basis[bit + 3];
      }
    t0[v] = a;
    t1[v] = bb;
  }
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    uint8_t x = 0;
#pragma unroll
    for (int bit = 0; bit < 2; ++bit)
      if (v & (1 << bit)) x ^= basis[bit + 6];
    t2[v] = x;
  }
  auto pack = [](const uint8_t* b) {
    return uint32_t(b[0]) | (uint32_t(b[1]) << 8) | (uint32_t(b[2]) << 16) | (uint32_t(b[3]) << 24);
  };
  rec[0] = pack(t0);
  rec[1] = pack(t0 + 4);
  rec[2] = pack(t1);
  rec[3] = pack(t1 + 4);
  rec[4] = pack(t2);
  rec[5] = rec[6] = rec[7] = 0;
}

// One wave (64 lanes) for n <= 64: the per-column barriers are then single-wave s_barriers and
// the k=10 decode system inverts in a few microseconds; 256 lanes for wide stripes.
template <int kInvBlock>
__global__ __launch_bounds__(kInvBlock) void gf_invert_kernel(const uint8_t* __restrict__ a,
                                                              uint8_t* __restrict__ a_inv, int n,
                                                              int* __restrict__ status, uint32_t* __restrict__ tab,
                                                              const int* __restrict__ sel_rows, int m, int m_pad) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  // carve: exp 1024 | log 512 | flog 512 | piv 16 | W n*n | R n*n
  uint8_t* exp_s = smem;
  uint16_t* log_s = reinterpret_cast<uint16_t*>(smem + 1024);
  uint16_t* flog = reinterpret_cast<uint16_t*>(smem + 1536);
  int* piv_s = reinterpret_cast<int*>(smem + 2048);
  uint8_t* W = smem + 2064;
  uint8_t* R = W + n * n;

  const int tid = threadIdx.x;
  const size_t base = size_t(blockIdx.x) * n * n;
  for (int i = tid; i < kExpLen; i += kInvBlock) exp_s[i] = d_gf_tables.exp[i];
  for (int i = kExpLen + tid; i < 1024; i += kInvBlock) exp_s[i] = 0;
  for (int i = tid; i < 256; i += kInvBlock) log_s[i] = d_gf_tables.log[i];
  for (int i = tid; i < n * n; i += kInvBlock) {
    W[i] = a[base + i];
    R[i] = (i / n == i % n) ? 1 : 0;
  }
  __syncthreads();

  int singular = 0;
  for (int c = 0; c < n; ++c) {
    if (tid == 0) *piv_s = n;
    __syncthreads();
    for (int r = c + tid; r < n; r += kInvBlock)
      if (W[r * n + c]) atomicMin(piv_s, r);
    __syncthreads();
    const int p = *piv_s;
    if (p == n) {  // uniform: every thread read the same LDS word after the barrier
      singular = 1;
      break;
    }
    if (p != c) {
      for (int e = tid; e < 2 * n; e += kInvBlock) {
        uint8_t* M = e < n ? W : R;
        const int col = e < n ? e : e - n;
        const uint8_t t = M[p * n + col];
        M[p * n + col] = M[c * n + col];
        M[c * n + col] = t;
      }
      __syncthreads();
    }
    const int inv_log = 255 - log_s[W[c * n + c]];
    __syncthreads();  // everyone has read the pivot before row c is rewritten
    for (int e = tid; e < 2 * n; e += kInvBlock) {
      uint8_t* M = e < n ? W : R;
      const int col = e < n ? e : e - n;
      M[c * n + col] = dmul_log(exp_s, log_s[M[c * n + col]], inv_log);
    }
    for (int r = tid; r < n; r += kInvBlock) flog[r] = (r == c) ? kLogZero : log_s[W[r * n + c]];
    __syncthreads();
    for (int idx = tid; idx < n * 2 * n; idx += kInvBlock) {
      const int r = idx / (2 * n);
      const int e = idx - r * 2 * n;
      if (r == c) continue;
      uint8_t* M = e < n ? W : R;
      const int col = e < n ? e : e - n;
      M[r * n + col] ^= dmul_log(exp_s, flog[r], log_s[M[c * n + col]]);
    }
    __syncthreads();
  }

  if (tid == 0 && status) status[blockIdx.x] = singular;
  if (a_inv)
    for (int i = tid; i < n * n; i += kInvBlock) a_inv[base + i] = singular ? 0 : R[i];
  if (tab && !singular) {
    // decode tables: tab[j][i] = perm(R[sel_rows[i]][j]) for i < m; padding rows stay zero.
    for (int idx = tid; idx < n * m; idx += kInvBlock) {
      const int j = idx / m;
      const int i = idx - j * m;
      uint32_t rec[8];
      perm_record(exp_s, log_s, R[sel_rows[i] * n + j], rec);
      uint32_t* dst = tab + (size_t(j) * m_pad + i) * kPermStride;
#pragma unroll
      for (int w = 0; w < 8; ++w) dst[w] = rec[w];
    }
  }
}

}  // namespace

hipError_t launch_gf_invert(const uint8_t* a, uint8_t* a_inv, int n, int batch, int* status, void* desc,
                            const int* sel_rows, int m, int m_pad, hipStream_t stream) {
  if (n <= 0 || n > 256 || batch <= 0) return hipErrorInvalidValue;
  if (desc && (batch != 1 || !sel_rows || m <= 0 || m > m_pad)) return hipErrorInvalidValue;
  const size_t lds = 2064 + 2 * size_t(n) * n;
  uint32_t* tab = nullptr;
  if (desc) tab = reinterpret_cast<uint32_t*>(static_cast<char*>(desc) + desc_layout(n, m_pad).tab_off);
  if (n <= 64) {
    gf_invert_kernel<64><<<batch, 64, lds, stream>>>(a, a_inv, n, status, tab, sel_rows, m, m_pad);
    return hipGetLastError();
  }
  static bool attr_set = false;  // >64 KiB of dynamic LDS must be opted into once per process
  if (lds > 65536 && !attr_set) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gf_invert_kernel<256>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  gf_invert_kernel<256><<<batch, 256, lds, stream>>>(a, a_inv, n, status, tab, sel_rows, m, m_pad);
  return hipGetLastError();
}

}  // namespace gfrs

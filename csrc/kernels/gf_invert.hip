// Gauss-Jordan GF(2^8) matrix inverse on gfx950: one workgroup per matrix, [A|I] resident in LDS.
//
// Replaces the reference's GPU inversion family:
//   * `GPU_invert_matrix` (src/matrix.cu:666-744) launches 3-4 kernels per row and copies every
//     row back to the host to pick the pivot (src/matrix.cu:684); here the whole elimination is one
//     launch with the pivot search done by an LDS atomicMin — no host round trip, graph-capturable.
//   * `eliminate_by_row` (src/matrix.cu:525-556) has an inter-block race on the pivot column; here
//     every row's elimination factor is snapshotted (as a v_perm table) behind a barrier before any
//     row is updated.
//   * Pivoting is by ROWS (the reference swaps columns and its result swap is a no-op,
//     src/matrix.cu:451-453 / src/cpu-decode.c:133-135, permuting decoded output — SURVEY §3.2),
//     and a column with no pivot reports `status = 1` instead of indexing column -1.
//   * The blocked 4x4 variant (src/decode-gj.cu:224-988, no pivoting, size % 4 == 0) is subsumed:
//     k <= 256 always fits one CU's LDS (256 rows x 516 B = 129 KiB of 160 KiB).
// Arithmetic is dword-packed: a row update `row_r ^= f_r * row_c` applies f_r's v_perm table
// (the GEMM kernel's 3-chunk scheme) to 4 bytes per lane-op, so the O(n^3) work runs at 4 bytes
// per ~6 VALU ops. Row pitch is an odd number of dwords so lanes walking different rows hit
// different LDS banks.
// Optionally the kernel also emits the v_perm tables of selected inverse rows straight into a
// GF-GEMM descriptor, so a decode is invert -> GEMM on one stream with zero host involvement.
#include <hip/hip_runtime.h>

#include "gfrs/desc.h"
#include "gfrs/device_cache.h"
#include "gfrs/kernels.h"

namespace gfrs {
namespace {

__constant__ Tables d_gf_tables = make_tables();

__device__ __forceinline__ uint32_t xtime(uint32_t x) { return ((x << 1) ^ ((x & 0x80u) ? 0x1Du : 0u)) & 0xFFu; }

// v_perm table of "multiply by f" (same layout as gfrs::perm_for_coeff).
__device__ __forceinline__ void perm_of(uint32_t f, uint32_t t[5]) {
  uint32_t b[8];
  b[0] = f & 0xFFu;
#pragma unroll
  for (int i = 1; i < 8; ++i) b[i] = xtime(b[i - 1]);
  auto tri = [](uint32_t x0, uint32_t x1, uint32_t x2, uint32_t& lo, uint32_t& hi) {
    // entries v = 0..7 : XOR of x_bit for the set bits of v
    lo = (x0 << 8) | (x1 << 16) | ((x0 ^ x1) << 24);
    hi = x2 | ((x2 ^ x0) << 8) | ((x2 ^ x1) << 16) | ((x2 ^ x1 ^ x0) << 24);
  };
  tri(b[0], b[1], b[2], t[0], t[1]);
  tri(b[3], b[4], b[5], t[2], t[3]);
  t[4] = (b[6] << 8) | (b[7] << 16) | ((b[6] ^ b[7]) << 24);
}

__device__ __forceinline__ uint32_t apply4(const uint32_t t[5], uint32_t w) {
  return __builtin_amdgcn_perm(t[1], t[0], w & 0x07070707u) ^
         __builtin_amdgcn_perm(t[3], t[2], (w >> 3) & 0x07070707u) ^
         __builtin_amdgcn_perm(0u, t[4], (w >> 6) & 0x03030303u);
}

template <int B>
__global__ __launch_bounds__(B) void gf_invert_kernel(const uint8_t* __restrict__ a, uint8_t* __restrict__ a_inv,
                                                      int n, int* __restrict__ status, uint32_t* __restrict__ tab,
                                                      const int* __restrict__ sel_rows, int m, int m_pad) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  // carve: exp 1024 | log 512 | misc 16 | Tinv 32 | T n*32 | M n*PW*4
  const int PW = (((2 * n + 3) / 4) | 1);  // row pitch in dwords, odd => conflict-free column walks
  uint8_t* exp_s = smem;
  uint16_t* log_s = reinterpret_cast<uint16_t*>(smem + 1024);
  int* piv_s = reinterpret_cast<int*>(smem + 1536);
  uint32_t* tinv_s = reinterpret_cast<uint32_t*>(smem + 1552);
  uint32_t* T = reinterpret_cast<uint32_t*>(smem + 1584);
  uint32_t* M = reinterpret_cast<uint32_t*>(smem + 1584 + 32 * n);
  uint8_t* Mb = reinterpret_cast<uint8_t*>(M);
  auto byte_at = [&](int r, int col) -> uint8_t& { return Mb[(r * PW) * 4 + col]; };

  const int tid = threadIdx.x;
  const size_t base = size_t(blockIdx.x) * n * n;
  for (int i = tid; i < kExpLen; i += B) exp_s[i] = d_gf_tables.exp[i];
  for (int i = kExpLen + tid; i < 1024; i += B) exp_s[i] = 0;
  for (int i = tid; i < 256; i += B) log_s[i] = d_gf_tables.log[i];
  for (int i = tid; i < n * PW; i += B) M[i] = 0;
  __syncthreads();
  for (int i0 = tid; i0 < n * n; i0 += 8 * B) {  // 8 independent global loads in flight per lane
    uint8_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (i0 + u * B < n * n) v[u] = a[base + i0 + u * B];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * B;
      if (i >= n * n) break;
      const int r = i / n, col = i - r * n;
      byte_at(r, col) = v[u];
      if (r == col) byte_at(r, n + col) = 1;
    }
  }
  __syncthreads();

  // work split for row-parallel phases: TPR lanes per row (power of two), rows strided
  int TPR = 1;
  while (TPR * 2 * n <= B && TPR < 64) TPR <<= 1;
  const int my_row0 = tid / TPR, sub = tid % TPR, row_step = B / TPR;

  int singular = 0;
  for (int c = 0; c < n; ++c) {
    if (tid == 0) *piv_s = n;
    __syncthreads();
    for (int r = c + tid; r < n; r += B)
      if (byte_at(r, c)) atomicMin(piv_s, r);
    __syncthreads();
    const int p = *piv_s;
    if (p == n) {  // uniform: every lane read the same LDS word after the barrier
      singular = 1;
      break;
    }
    if (p != c) {
      for (int w = tid; w < PW; w += B) {
        const uint32_t t = M[p * PW + w];
        M[p * PW + w] = M[c * PW + w];
        M[c * PW + w] = t;
      }
      __syncthreads();
    }
    if (tid == 0) {
      uint32_t t[5];
      perm_of(exp_s[255 - log_s[byte_at(c, c)]], t);
#pragma unroll
      for (int q = 0; q < 5; ++q) tinv_s[q] = t[q];
    }
    __syncthreads();
    {  // normalise the pivot row; snapshot every other row's factor as a perm table
      uint32_t ti[5];
#pragma unroll
      for (int q = 0; q < 5; ++q) ti[q] = tinv_s[q];
      for (int w = tid; w < PW; w += B) M[c * PW + w] = apply4(ti, M[c * PW + w]);
      for (int r = tid; r < n; r += B) {
        uint32_t t[5];
        perm_of(r == c ? 0u : byte_at(r, c), t);
#pragma unroll
        for (int q = 0; q < 5; ++q) T[r * 8 + q] = t[q];
      }
    }
    __syncthreads();
    for (int r = my_row0; r < n; r += row_step) {
      if (r == c) continue;
      uint32_t t[5];
#pragma unroll
      for (int q = 0; q < 5; ++q) t[q] = T[r * 8 + q];
      if ((t[0] | t[1] | t[2] | t[3] | t[4]) == 0) continue;  // factor 0: row already clear
      // batches of 8 dwords: all LDS reads issued before the writes (r != c, so no aliasing),
      // which the compiler cannot prove on its own and would otherwise serialise per dword
      int w = sub;
      for (; w + 7 * TPR < PW; w += 8 * TPR) {
        uint32_t pv[8], rv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          pv[u] = M[c * PW + w + u * TPR];
          rv[u] = M[r * PW + w + u * TPR];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) M[r * PW + w + u * TPR] = rv[u] ^ apply4(t, pv[u]);
      }
      for (; w < PW; w += TPR) M[r * PW + w] ^= apply4(t, M[c * PW + w]);
    }
    __syncthreads();
  }

  if (tid == 0 && status) status[blockIdx.x] = singular;
  if (a_inv)
    for (int i = tid; i < n * n; i += B) {
      const int r = i / n, col = i - r * n;
      a_inv[base + i] = singular ? 0 : byte_at(r, n + col);
    }
  if (tab && !singular) {
    // decode tables: tab[j][i] = perm(R[sel_rows[i]][j]) for i < m; padding rows stay zero.
    for (int idx = tid; idx < n * m; idx += B) {
      const int j = idx / m;
      const int i = idx - j * m;
      uint32_t t[5];
      perm_of(byte_at(sel_rows[i], n + j), t);
      uint32_t* dst = tab + (size_t(j) * m_pad + i) * kPermStride;
#pragma unroll
      for (int q = 0; q < 5; ++q) dst[q] = t[q];
      dst[5] = dst[6] = dst[7] = 0;
    }
  }
}


// Systematic decode system, solved directly (SURVEY §3.2 decode, done the erasure-code way): with
// G = [I; E] and survivors = (k-e) natives N + e parity rows P, the e erased natives x_E satisfy
// E[P,E] x_E = y_P + E[P,N] x_N (characteristic 2), so the decode rows are
// X = M^-1 B' with M = G[P, erased] (e x e) and B'[a][j] = G[P_a][rows_j] for a native survivor j,
// [rows_j == P_a] for a parity survivor j. Gauss-Jordan on [M | B'] (e x (e+k)) yields X directly:
// O(e^2 (e+k)) instead of inverting the whole k x k system (k=128, e=32: ~40x less work, and the
// wide decode no longer waits ~1 ms for a 128x128 inverse — profiles/r01_p128).
// LDS carve of the decode-system kernel before M: exp 1024 | log 512 | pivot-search slots, parity
// count, pattern-error flag 32 | pivot rows 256 | parity survivors 256 | rows 256 | erased 256 |
// pivot inverses 256 (ids are bytes). Kept small so the solve fits next to a full-LDS persistent
// GEMM block (k=128, e=32: 7.9 KiB; gf_mfma_fp4.hip kSideReserve).
constexpr size_t kDecSysFixed = 1568 + 5 * 256;

// Device-built decode plans (`ptrs` != null): the survivor list `rows` is the only input — e.g. an
// erasure pattern just RCCL-broadcast into device memory by a coordinator rank. The kernel checks
// it (k distinct chunk ids < n_chunks, exactly e natives missing; else status 2), derives the erased
// natives (written back to `erased`, ascending) and, besides the tables, writes the descriptor's
// row pointers from the stripe's pointer table ptrs = {chunk row 0..n_chunks-1, output row 0..k-1}:
// in[j] = chunk[rows[j]], copy[j] = out[rows[j]] for a native survivor, out[i] = out[erased[i]].
// A singular or invalid pattern leaves no output pointer (the GEMM then stores nothing).
template <int B>
__global__ __launch_bounds__(B) void gf_decode_system_kernel(const uint8_t* __restrict__ g, int k,
                                                             const int* __restrict__ rows,
                                                             int* __restrict__ erased, int e,
                                                             uint8_t* __restrict__ dm, int* __restrict__ status,
                                                             uint32_t* __restrict__ tab, int m_pad,
                                                             const uint64_t* __restrict__ ptrs, int n_chunks,
                                                             uint64_t* __restrict__ dptr) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int W = e + k;
  const int PW = (((W + 3) / 4) | 1);
  uint8_t* exp_s = smem;
  uint16_t* log_s = reinterpret_cast<uint16_t*>(smem + 1024);
  int* piv_s = reinterpret_cast<int*>(smem + 1536);  // [0..2] pivot-search slots, [3] parity count, [4] bad
  uint8_t* perm_s = smem + 1568;  // perm_s[c] = pivot row of column c
  uint8_t* prow = perm_s + 256;   // parity survivors (e of them), survivor order (ids < 256)
  uint8_t* rows_s = prow + 256;
  uint8_t* erased_s = rows_s + 256;
  uint8_t* pinv_s = erased_s + 256;  // 1 / M[perm_s[c]][c]
  uint32_t* M = reinterpret_cast<uint32_t*>(smem + kDecSysFixed);
  uint8_t* Mb = reinterpret_cast<uint8_t*>(M);
  auto byte_at = [&](int r, int col) -> uint8_t& { return Mb[(r * PW) * 4 + col]; };

  const int tid = threadIdx.x;
  for (int i = tid; i < kExpLen; i += B) exp_s[i] = d_gf_tables.exp[i];
  for (int i = kExpLen + tid; i < 1024; i += B) exp_s[i] = 0;
  for (int i = tid; i < 256; i += B) log_s[i] = d_gf_tables.log[i];
  for (int i = tid; i < e * PW; i += B) M[i] = 0;
  if (tid < 3) piv_s[tid] = e;
  if (tid == 4) piv_s[4] = 0;
  __syncthreads();
  if (ptrs) {
    for (int i = tid; i < k; i += B) {
      const int r = rows[i];
      const bool ok = r >= 0 && r < n_chunks;
      rows_s[i] = uint8_t(ok ? r : 0);
      if (!ok) piv_s[4] = 1;
    }
  } else {
    for (int i = tid; i < k; i += B) rows_s[i] = uint8_t(rows[i]);
    for (int i = tid; i < e; i += B) erased_s[i] = uint8_t(erased[i]);
  }
  __syncthreads();
  if (ptrs) {
    // chunk i (one lane each, n_chunks <= 256 = B) counts its occurrences among the survivors
    // (broadcast LDS reads); missing natives are flagged in perm_s, which the solve reuses later
    for (int i = tid; i < n_chunks; i += B) {
      int cnt = 0;
      for (int j = 0; j < k; ++j) cnt += rows_s[j] == i;
      if (cnt > 1) piv_s[4] = 1;
      if (i < k) perm_s[i] = uint8_t(cnt == 0);
    }
    __syncthreads();
    if (tid < 64) {  // erased natives in ascending order: ballot prefix sum in wave 0
      int base = 0;
      for (int i0 = 0; i0 < k; i0 += 64) {
        const int i = i0 + tid;
        const bool miss = i < k && perm_s[i];
        const unsigned long long bal = __ballot(miss);
        const int a = base + __popcll(bal & ((1ull << tid) - 1ull));
        if (miss && a < e) {
          erased_s[a] = uint8_t(i);
          erased[a] = i;
        }
        base += __popcll(bal);
      }
      if (tid == 0 && base != e) piv_s[4] = 1;
    }
    __syncthreads();
  }
  const int bad = piv_s[4];
  // parity survivors in survivor order: a ballot prefix sum in wave 0 (a one-lane scan of the
  // global ids was k dependent HBM round trips: ~130 us of the k=128 solve)
  if (tid < 64) {
    int base = 0;
    for (int j0 = 0; j0 < k; j0 += 64) {
      const int j = j0 + tid;
      const bool is_par = j < k && rows_s[j] >= k;
      const unsigned long long bal = __ballot(is_par);
      const int a = base + __popcll(bal & ((1ull << tid) - 1ull));
      if (is_par && a < e) prow[a] = rows_s[j];
      base += __popcll(bal);
    }
    if (tid == 0) piv_s[3] = base < e ? base : e;
  }
  __syncthreads();
  int singular = (bad || piv_s[3] != e) ? 1 : 0;  // not exactly e parity survivors: inconsistent pattern
  if (!singular) {
    // the e x (e+k) system, 8 independent global loads in flight per lane
    for (int i0 = tid; i0 < e * W; i0 += 8 * B) {
      uint8_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * B;
        if (i >= e * W) break;
        const int a = i / W, col = i - a * W;
        const size_t grow = size_t(prow[a]) * k;
        if (col < e) {
          v[u] = g[grow + erased_s[col]];
        } else {
          const int r = rows_s[col - e];
          v[u] = r < k ? g[grow + r] : uint8_t(r == prow[a]);
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * B;
        if (i >= e * W) break;
        const int a = i / W;
        byte_at(a, i - a * W) = v[u];
      }
    }
  }
  __syncthreads();

  // Gauss-Jordan with one barrier per column and no row swaps. Column c's pivot p — the lowest
  // unused row with a nonzero in column c, bid for with an LDS atomicMin while column c-1 was
  // eliminated — is recorded (perm_s[c]) and left unnormalised; every other row r adds
  // (M[r][c] / M[p][c]) * row p. The TPR lanes of row r (one wave: TPR divides 64) read that factor
  // before any of them writes the row; the lane owning column c+1 of the updated row then bids
  // for the next pivot. Three rotating bid slots: slot c%3 is read after the barrier, (c+1)%3 is
  // bid into, (c+2)%3 is reset. Rows are normalised once, in the output pass. (The former loop
  // had five barriers and a serial inverse per column: 75 us at e=32, k=128.)
  int TPR = 1;
  while (TPR * 2 * e <= B && TPR < 64) TPR <<= 1;
  const int r = tid / TPR, sub = tid % TPR;  // at most one row per lane group: B / TPR >= e
  bool used = false;
  if (!singular && sub == 0 && r < e && byte_at(r, 0)) atomicMin(&piv_s[0], r);
  __syncthreads();
  for (int c = 0; c < e && !singular; ++c) {
    const int p = piv_s[c % 3];
    if (p >= e) {  // uniform: every lane read the same LDS word after the barrier
      singular = 1;
      break;
    }
    if (tid == 0) {
      piv_s[(c + 2) % 3] = e;
      perm_s[c] = uint8_t(p);
    }
    if (r < e && r != p) {
      const uint32_t f = byte_at(r, c);
      if (f) {
        uint32_t t[5];
        perm_of(exp_s[log_s[f] + 255 - log_s[byte_at(p, c)]], t);
        // batches of 8 dwords: all LDS reads issued before the writes (r != p, so no aliasing)
        int w = sub;
        for (; w + 7 * TPR < PW; w += 8 * TPR) {
          uint32_t pv[8], rv[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            pv[u] = M[p * PW + w + u * TPR];
            rv[u] = M[r * PW + w + u * TPR];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) M[r * PW + w + u * TPR] = rv[u] ^ apply4(t, pv[u]);
        }
        for (; w < PW; w += TPR) M[r * PW + w] ^= apply4(t, M[p * PW + w]);
      }
      if (!used && c + 1 < e && sub == ((c + 1) >> 2) % TPR && byte_at(r, c + 1))
        atomicMin(&piv_s[(c + 1) % 3], r);
    }
    if (r == p) used = true;
    __syncthreads();
  }

  if (tid == 0 && status) *status = bad ? 2 : singular;
  if (!singular) {
    for (int b = tid; b < e; b += B) pinv_s[b] = exp_s[255 - log_s[byte_at(perm_s[b], b)]];
    __syncthreads();
  }
  if (dptr) {  // descriptor row pointers: in[k] | copy[k] | out[m_pad] (desc.h)
    const uint64_t* outp = ptrs + n_chunks;
    for (int j = tid; j < k; j += B) {
      const int r = rows_s[j];
      dptr[j] = ptrs[r];
      dptr[k + j] = (!singular && r < k) ? outp[r] : 0;
    }
    for (int i = tid; i < m_pad; i += B) dptr[2 * k + i] = (!singular && i < e) ? outp[erased_s[i]] : 0;
  }
  // X[b][j] = M[perm_s[b]][e + j] / M[perm_s[b]][b]
  auto x_at = [&](int b, int j) -> uint32_t {
    return exp_s[log_s[byte_at(perm_s[b], e + j)] + log_s[pinv_s[b]]];
  };
  if (dm)
    for (int i = tid; i < e * k; i += B) {
      const int b = i / k, j = i - b * k;
      dm[i] = singular ? 0 : uint8_t(x_at(b, j));
    }
  if (tab && !singular)
    for (int idx = tid; idx < k * e; idx += B) {  // tab[j][b] = perm(X[b][j])
      const int j = idx / e, b = idx - j * e;
      uint32_t t[5];
      perm_of(x_at(b, j), t);
      uint32_t* dst = tab + (size_t(j) * m_pad + b) * kPermStride;
#pragma unroll
      for (int q = 0; q < 5; ++q) dst[q] = t[q];
      dst[5] = dst[6] = dst[7] = 0;
    }
}

}  // namespace

hipError_t launch_gf_decode_system(const uint8_t* g, int k, const int* rows, int* erased, int e, uint8_t* dm,
                                   int* status, void* desc, int m_pad, hipStream_t stream, const uint64_t* ptrs,
                                   int n_chunks) {
  if (k <= 0 || k > 256 || e <= 0 || e > k || (desc && e > m_pad)) return hipErrorInvalidValue;
  if (ptrs && (!desc || !erased || n_chunks < k + e || n_chunks > 256)) return hipErrorInvalidValue;
  uint64_t* dptr = nullptr;
  if (ptrs) dptr = reinterpret_cast<uint64_t*>(static_cast<char*>(desc) + desc_layout(k, m_pad).in_off);
  const int W = e + k;
  const int PW = (((W + 3) / 4) | 1);
  const size_t lds = kDecSysFixed + 4 * size_t(e) * PW;
  uint32_t* tab = nullptr;
  if (desc) tab = reinterpret_cast<uint32_t*>(static_cast<char*>(desc) + desc_layout(k, m_pad).tab_off);
  // (256 lanes for every e: the system gather and the decode-table emission are O(e k) loads /
  // stores that one wave serialised — 135 us at k=128, e=32)
  if (lds > 65536) {  // per device (one process may drive several GPUs from several threads)
    const hipError_t err = ensure_lds_optin(reinterpret_cast<const void*>(&gf_decode_system_kernel<256>));
    if (err != hipSuccess) return err;
  }
  gf_decode_system_kernel<256><<<1, 256, lds, stream>>>(g, k, rows, erased, e, dm, status, tab, m_pad, ptrs,
                                                        n_chunks, dptr);
  return hipGetLastError();
}

hipError_t launch_gf_invert(const uint8_t* a, uint8_t* a_inv, int n, int batch, int* status, void* desc,
                            const int* sel_rows, int m, int m_pad, hipStream_t stream) {
  if (n <= 0 || n > 256 || batch <= 0) return hipErrorInvalidValue;
  if (desc && (batch != 1 || !sel_rows || m <= 0 || m > m_pad)) return hipErrorInvalidValue;
  const int PW = (((2 * n + 3) / 4) | 1);
  const size_t lds = 1584 + 32 * size_t(n) + 4 * size_t(n) * PW;
  uint32_t* tab = nullptr;
  if (desc) tab = reinterpret_cast<uint32_t*>(static_cast<char*>(desc) + desc_layout(n, m_pad).tab_off);
  if (n <= 32) {
    gf_invert_kernel<64><<<batch, 64, lds, stream>>>(a, a_inv, n, status, tab, sel_rows, m, m_pad);
    return hipGetLastError();
  }
  if (lds > 65536) {  // >64 KiB of dynamic LDS is opted into once per device
    const hipError_t e = ensure_lds_optin(reinterpret_cast<const void*>(&gf_invert_kernel<256>));
    if (e != hipSuccess) return e;
  }
  gf_invert_kernel<256><<<batch, 256, lds, stream>>>(a, a_inv, n, status, tab, sel_rows, m, m_pad);
  return hipGetLastError();
}

}  // namespace gfrs

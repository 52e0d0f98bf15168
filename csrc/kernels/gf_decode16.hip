// GF(2^16) systematic decode system on the device: the w = 16 form of gf_invert.hip's
// gf_decode_system_kernel, so a GF(2^16) decode plan is built with no host round trip.
//
// The reference never built its w = 16 field (/root/reference/src/galoisfield.cu:22-32, poly
// 0210013) and inverts every decode system on the host (src/decode.cu:333 -> src/cpu-decode.c:
// 251-298). Here, with G = [I; E] (n x k, 16-bit symbols) and k survivors = (k - e) natives N plus
// e parity rows P, the erased natives x_E solve E[P,E] x_E = y_P + E[P,N] x_N (characteristic 2):
// Gauss-Jordan on [M | B'] with M = G[P, erased] (e x e) and B'[a][j] = G[P_a][rows_j] for a native
// survivor j, [rows_j == P_a] for a parity one, leaves X = M^-1 B' — the decode rows over the
// survivors — in O(e^2 (e + k)) work instead of a k x k inverse.
//
// Field arithmetic without tables. GF(2^16) log/exp tables (384 KiB) fit neither constant memory
// nor LDS, so the kernel never looks a product up:
//   * row updates multiply by a constant c through c's four byte maps (gfrs/gf65536.h perm_quad:
//     c * (l | h << 8) = [L_ll(l) ^ L_hl(h)] | [L_lh(l) ^ L_hh(h)] << 8), built on the fly from
//     c * 2^i (15 shift-and-reduce steps) and applied with v_perm to 4 de-interleaved symbols at a
//     time — the GEMM kernel's engine (gf_gemm16.hip);
//   * elimination is fraction-free: row r <- a * row r + f * row p with a = M[p][c], f = M[r][c], so
//     no division happens inside the column loop (a row update costs two maps instead of one, far
//     less than a per-column inverse by exponentiation);
//   * the e pivots are inverted once at the end (a^(2^16 - 2), 30 shift-and-add products), one
//     lane each, and the output rows are scaled by them while the plan's tables are written.
// Pattern check and derivation as in the w = 8 kernel (status 2 = invalid survivor list), and the
// plan's tables (desc_layout16: four records per coefficient) and, with `ptrs`, its row pointers
// are written in place.
#include <hip/hip_runtime.h>

#include "gfrs/desc.h"
#include "gfrs/device_cache.h"
#include "gfrs/kernels.h"
#include "gfrs/perm_device.h"

namespace gfrs {
namespace {

using namespace permdev;

constexpr uint32_t kPoly16 = 0x1100Bu;
constexpr int kThreads = 256;

// plane shuffles of 4 little-endian symbols held in two dwords (as gf_gemm16.hip)
constexpr uint32_t kSelLo = 0x06040200u;
constexpr uint32_t kSelHi = 0x07050301u;
constexpr uint32_t kSelW0 = 0x05010400u;
constexpr uint32_t kSelW1 = 0x07030602u;

__device__ __forceinline__ uint32_t xtime16(uint32_t x) {
  x <<= 1;
  return (x & 0x10000u) ? (x ^ kPoly16) : x;
}

__device__ uint32_t mul16(uint32_t a, uint32_t b) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    r ^= ((b >> i) & 1u) ? a : 0u;
    a = xtime16(a);
  }
  return r;
}

// a^(2^16 - 2) = a^-1 for a != 0: r = prod_{i=1..15} a^(2^i)
__device__ uint32_t inv16(uint32_t a) {
  uint32_t r = 1, s = a;
  for (int i = 1; i < 16; ++i) {
    s = mul16(s, s);
    r = mul16(r, s);
  }
  return r;
}

// v_perm record of the byte map with basis images b[0..7] (layout of gfrs::perm_from_basis)
__device__ __forceinline__ void perm_rec(const uint32_t b[8], uint32_t t[5]) {
  auto tri = [](uint32_t x0, uint32_t x1, uint32_t x2, uint32_t& lo, uint32_t& hi) {
    lo = (x0 << 8) | (x1 << 16) | ((x0 ^ x1) << 24);
    hi = x2 | ((x2 ^ x0) << 8) | ((x2 ^ x1) << 16) | ((x2 ^ x1 ^ x0) << 24);
  };
  tri(b[0], b[1], b[2], t[0], t[1]);
  tri(b[3], b[4], b[5], t[2], t[3]);
  t[4] = (b[6] << 8) | (b[7] << 16) | ((b[6] ^ b[7]) << 24);
}

// The four byte maps of "multiply by c", q = 2 * src + dst (gfrs/gf65536.h perm_quad).
__device__ __forceinline__ void quad_of(uint32_t c, uint32_t q[4][5]) {
  uint32_t img[16];
  img[0] = c;
#pragma unroll
  for (int i = 1; i < 16; ++i) img[i] = xtime16(img[i - 1]);
#pragma unroll
  for (int src = 0; src < 2; ++src)
#pragma unroll
    for (int dst = 0; dst < 2; ++dst) {
      uint32_t b[8];
#pragma unroll
      for (int bit = 0; bit < 8; ++bit) b[bit] = (img[8 * src + bit] >> (8 * dst)) & 0xFFu;
      perm_rec(b, q[2 * src + dst]);
    }
}

// LDS carve of the kernel (bytes): misc int[8] | cnt int[n] | rows int[k] | erased int[e] |
// prow int[e] | perm int[e] | pinv int[e] | M (e rows x PU units of 4 symbols, 8 B each).
__host__ __device__ constexpr int units_of(int w) { return ((w + 3) / 4) | 1; }  // odd: rows on spread banks
__host__ __device__ constexpr size_t lds_fixed16(int n, int k, int e) { return 32 + 4 * (size_t(n) + k + 4 * size_t(e)); }
__host__ __device__ constexpr size_t lds16(int n, int k, int e) {
  return lds_fixed16(n, k, e) + 8 * size_t(e) * units_of(e + k);
}

__global__ __launch_bounds__(kThreads) void gf_decode_system16_kernel(
    const uint16_t* __restrict__ g, int n, int k, const int* __restrict__ rows, int* __restrict__ erased, int e,
    uint16_t* __restrict__ dm, int* __restrict__ status, uint32_t* __restrict__ tab, int m_pad,
    const uint64_t* __restrict__ ptrs, uint64_t* __restrict__ dptr) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int B = kThreads;
  const int W = e + k;
  const int PU = units_of(W);
  int* misc = reinterpret_cast<int*>(smem);  // [0..2] pivot bids, [3] parity count, [4] bad
  int* cnt = misc + 8;
  int* rows_s = cnt + n;
  int* erased_s = rows_s + k;
  int* prow = erased_s + e;
  int* perm_s = prow + e;
  int* pinv = perm_s + e;
  uint32_t* M = reinterpret_cast<uint32_t*>(smem + lds_fixed16(n, k, e));  // row a: 2 * PU dwords
  uint16_t* Ms = reinterpret_cast<uint16_t*>(M);
  auto sym = [&](int r, int col) -> uint16_t& { return Ms[size_t(r) * 4 * PU + col]; };

  const int tid = threadIdx.x;
  for (int i = tid; i < n; i += B) cnt[i] = 0;
  for (int i = tid; i < e * 2 * PU; i += B) M[i] = 0;
  if (tid < 3) misc[tid] = e;
  if (tid == 3) misc[3] = 0;
  if (tid == 4) misc[4] = 0;
  __syncthreads();
  for (int i = tid; i < k; i += B) {
    const int r = rows[i];
    const bool ok = r >= 0 && r < n;
    rows_s[i] = ok ? r : 0;
    if (ok) atomicAdd(&cnt[r], 1);
    else misc[4] = 1;
  }
  __syncthreads();
  for (int i = tid; i < n; i += B)
    if (cnt[i] > 1) misc[4] = 1;  // a chunk listed twice
  if (tid < 64) {  // erased natives (ascending) and parity survivors (survivor order): ballot prefix sums
    int base = 0;
    for (int i0 = 0; i0 < k; i0 += 64) {
      const int i = i0 + tid;
      const bool miss = i < k && cnt[i] == 0;
      const unsigned long long bal = __ballot(miss);
      const int a = base + __popcll(bal & ((1ull << tid) - 1ull));
      if (miss && a < e) erased_s[a] = i;
      base += __popcll(bal);
    }
    if (tid == 0 && base != e) misc[4] = 1;
    int pbase = 0;
    for (int j0 = 0; j0 < k; j0 += 64) {
      const int j = j0 + tid;
      const bool is_par = j < k && rows_s[j] >= k;
      const unsigned long long bal = __ballot(is_par);
      const int a = pbase + __popcll(bal & ((1ull << tid) - 1ull));
      if (is_par && a < e) prow[a] = rows_s[j];
      pbase += __popcll(bal);
    }
    if (tid == 0) misc[3] = pbase;
  }
  __syncthreads();
  const int bad = misc[4];
  int singular = (bad || misc[3] != e) ? 1 : 0;
  if (!bad)
    for (int i = tid; i < e; i += B) erased[i] = erased_s[i];
  if (!singular) {
    // the e x (e + k) system, 8 independent global loads in flight per lane
    for (int i0 = tid; i0 < e * W; i0 += 8 * B) {
      uint16_t v[8];
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
          v[u] = r < k ? g[grow + r] : uint16_t(r == prow[a]);
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * B;
        if (i >= e * W) break;
        const int a = i / W;
        sym(a, i - a * W) = v[u];
      }
    }
  }
  __syncthreads();

  // Fraction-free Gauss-Jordan, one barrier per column (the w = 8 kernel's bid scheme): column c's
  // pivot p is the lowest unused row with a nonzero in column c; every other row r with f = M[r][c]
  // != 0 becomes a * r + f * p (a = M[p][c]), which clears its column c. The TPR lanes of row r are
  // in one wave and read f before any of them writes the row; the lane owning column c + 1 of the
  // updated row then bids for the next pivot. Slots: c % 3 read, (c + 1) % 3 bid, (c + 2) % 3 reset.
  int TPR = 1;
  while (TPR * 2 * e <= B && TPR < 64) TPR <<= 1;
  const int r = tid / TPR, sub = tid % TPR;  // B / TPR >= e: one lane group per row
  bool used = false;
  if (!singular && sub == 0 && r < e && sym(r, 0)) atomicMin(&misc[0], r);
  __syncthreads();
  for (int c = 0; c < e && !singular; ++c) {
    const int p = misc[c % 3];
    if (p >= e) {  // uniform: every lane read the same LDS word after the barrier
      singular = 1;
      break;
    }
    if (tid == 0) {
      misc[(c + 2) % 3] = e;
      perm_s[c] = p;
    }
    if (r < e && r != p) {
      const uint32_t f = sym(r, c);
      if (f) {
        uint32_t qa[4][5], qf[4][5];
        quad_of(sym(p, c), qa);
        quad_of(f, qf);
        const uint32_t* rp = M + size_t(r) * 2 * PU;
        const uint32_t* pp = M + size_t(p) * 2 * PU;
        for (int u = sub; u < PU; u += TPR) {
          const uint32_t r0 = rp[2 * u], r1 = rp[2 * u + 1], p0 = pp[2 * u], p1 = pp[2 * u + 1];
          const Sel slr = make_sel(__builtin_amdgcn_perm(r1, r0, kSelLo));
          const Sel shr = make_sel(__builtin_amdgcn_perm(r1, r0, kSelHi));
          const Sel slp = make_sel(__builtin_amdgcn_perm(p1, p0, kSelLo));
          const Sel shp = make_sel(__builtin_amdgcn_perm(p1, p0, kSelHi));
          uint32_t lo = mac_pair(0u, qa[0], slr, qa[2], shr);
          lo = mac_pair(lo, qf[0], slp, qf[2], shp);
          uint32_t hi = mac_pair(0u, qa[1], slr, qa[3], shr);
          hi = mac_pair(hi, qf[1], slp, qf[3], shp);
          uint32_t* w = M + size_t(r) * 2 * PU + 2 * u;
          w[0] = __builtin_amdgcn_perm(hi, lo, kSelW0);
          w[1] = __builtin_amdgcn_perm(hi, lo, kSelW1);
        }
      }
      if (!used && c + 1 < e && sub == ((c + 1) >> 2) % TPR && sym(r, c + 1)) atomicMin(&misc[(c + 1) % 3], r);
    }
    if (r == p) used = true;
    __syncthreads();
  }

  if (tid == 0 && status) *status = bad ? 2 : singular;
  if (!singular) {
    for (int b = tid; b < e; b += B) pinv[b] = int(inv16(sym(perm_s[b], b)));
    __syncthreads();
  }
  if (dptr) {  // descriptor row pointers: in[k] | copy[k] | out[m_pad] (desc.h)
    const uint64_t* outp = ptrs + n;
    for (int j = tid; j < k; j += B) {
      const int rr = rows_s[j];
      dptr[j] = ptrs[rr];
      dptr[k + j] = (!singular && rr < k) ? outp[rr] : 0;
    }
    for (int i = tid; i < m_pad; i += B) dptr[2 * k + i] = (!singular && i < e) ? outp[erased_s[i]] : 0;
  }
  // X[b][j] = M[perm_s[b]][e + j] / M[perm_s[b]][b]
  auto x_at = [&](int b, int j) -> uint32_t { return mul16(sym(perm_s[b], e + j), uint32_t(pinv[b])); };
  if (dm)
    for (int i = tid; i < e * k; i += B) {
      const int b = i / k, j = i - b * k;
      dm[i] = singular ? uint16_t(0) : uint16_t(x_at(b, j));
    }
  if (tab && !singular)
    for (int idx = tid; idx < k * e; idx += B) {  // tab[j][b][q] = quad(X[b][j])[q]
      const int j = idx / e, b = idx - j * e;
      uint32_t q[4][5];
      quad_of(x_at(b, j), q);
      uint32_t* dst = tab + (size_t(j) * m_pad + b) * 4 * kPermStride;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
#pragma unroll
        for (int w = 0; w < 5; ++w) dst[qq * kPermStride + w] = q[qq][w];
        dst[qq * kPermStride + 5] = dst[qq * kPermStride + 6] = dst[qq * kPermStride + 7] = 0;
      }
    }
}

constexpr size_t kMaxLds16 = 160 * 1024;

}  // namespace

bool decode_system16_supported(int n, int k, int e) {
  return k >= 1 && e >= 1 && e <= k && e <= kThreads && n >= k + e && lds16(n, k, e) <= kMaxLds16;
}

hipError_t launch_gf_decode_system16(const uint16_t* g, int n, int k, const int* rows, int* erased, int e,
                                     uint16_t* dm, int* status, void* desc, int m_pad, hipStream_t stream,
                                     const uint64_t* ptrs) {
  if (!decode_system16_supported(n, k, e) || !erased || (desc && e > m_pad) || (ptrs && !desc))
    return hipErrorInvalidValue;
  const size_t lds = lds16(n, k, e);
  uint32_t* tab = nullptr;
  uint64_t* dptr = nullptr;
  if (desc) {
    const DescLayout l = desc_layout16(k, m_pad);
    tab = reinterpret_cast<uint32_t*>(static_cast<char*>(desc) + l.tab_off);
    if (ptrs) dptr = reinterpret_cast<uint64_t*>(static_cast<char*>(desc) + l.in_off);
  }
  if (lds > 65536) {
    const hipError_t err = ensure_lds_optin(reinterpret_cast<const void*>(&gf_decode_system16_kernel));
    if (err != hipSuccess) return err;
  }
  gf_decode_system16_kernel<<<1, kThreads, lds, stream>>>(g, n, k, rows, erased, e, dm, status, tab, m_pad, ptrs, dptr);
  return hipGetLastError();
}

}  // namespace gfrs

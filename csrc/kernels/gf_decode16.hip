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

#include <algorithm>

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

// a^2: squaring is GF(2)-linear — spread bit i to bit 2i, then reduce the 31-bit result with
// x^16 = x^12 + x^3 + x + 1 (four folds: each halves what is left above bit 15)
__device__ __forceinline__ uint32_t sq16(uint32_t a) {
  uint32_t x = a & 0xFFFFu;
  x = (x | (x << 8)) & 0x00FF00FFu;
  x = (x | (x << 4)) & 0x0F0F0F0Fu;
  x = (x | (x << 2)) & 0x33333333u;
  x = (x | (x << 1)) & 0x55555555u;
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const uint32_t hi = x >> 16;
    x = (x & 0xFFFFu) ^ (hi << 12) ^ (hi << 3) ^ (hi << 1) ^ hi;
  }
  return x;
}
__device__ __forceinline__ uint32_t sqn16(uint32_t a, int n) {
  for (int i = 0; i < n; ++i) a = sq16(a);
  return a;
}

// a^-1 = (a^(2^15 - 1))^2 for a != 0, by the Itoh-Tsujii chain b_k = a^(2^k - 1):
// b2 = b1^2 b1, b3 = b2^2 a, b6 = b3^(2^3) b3, b7 = b6^2 a, b14 = b7^(2^7) b7, b15 = b14^2 a —
// 15 squarings and 6 multiplies instead of 15 + 15 (the pivot inverses run on one lane)
__device__ uint32_t inv16(uint32_t a) {
  const uint32_t b2 = mul16(sq16(a), a);
  const uint32_t b3 = mul16(sq16(b2), a);
  const uint32_t b6 = mul16(sqn16(b3, 3), b3);
  const uint32_t b7 = mul16(sq16(b6), a);
  const uint32_t b14 = mul16(sqn16(b7, 7), b7);
  const uint32_t b15 = mul16(sq16(b14), a);
  return sq16(b15);
}

// nibble-product table of c: tab[q * 16 + v] (stride `stride` words) = c * (v << 4q)
template <typename T>
__device__ __forceinline__ void nib_table(uint32_t c, T* tab, int stride, int q) {
  uint32_t b0 = c;
  for (int s = 0; s < 4 * q; ++s) b0 = xtime16(b0);
  const uint32_t b1 = xtime16(b0), b2 = xtime16(b1), b3 = xtime16(b2);
#pragma unroll
  for (int v = 0; v < 16; ++v)
    tab[(q * 16 + v) * stride] = T(((v & 1) ? b0 : 0u) ^ ((v & 2) ? b1 : 0u) ^ ((v & 4) ? b2 : 0u) ^ ((v & 8) ? b3 : 0u));
}
// c * x from c's nibble table (stride words apart)
template <typename T>
__device__ __forceinline__ uint32_t nib_mul(const T* tab, int stride, uint32_t x) {
  return uint32_t(tab[(x & 15u) * stride]) ^ uint32_t(tab[(16 + ((x >> 4) & 15u)) * stride]) ^
         uint32_t(tab[(32 + ((x >> 8) & 15u)) * stride]) ^ uint32_t(tab[(48 + (x >> 12)) * stride]);
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

// (1024 threads: four times the lanes per row for the column loop, which is LDS-latency bound in
// one workgroup — as ds16_panel_kernel below)
constexpr int kSysThreads = 1024;
__global__ __launch_bounds__(kSysThreads) void gf_decode_system16_kernel(
    const uint16_t* __restrict__ g, int n, int k, const int* __restrict__ rows, int* __restrict__ erased, int e,
    uint16_t* __restrict__ dm, int* __restrict__ status, uint32_t* __restrict__ tab, int m_pad,
    const uint64_t* __restrict__ ptrs, uint64_t* __restrict__ dptr) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int B = kSysThreads;
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

// ---- blocked multi-workgroup solve (systems past one workgroup's LDS, or e > 256) --------------
//
// The reference's blocked Gauss-Jordan (decode-gj.cu, GPUGausSeidel :1059-1201 with its panel
// kernels :347-904) is a 4x4-block LU without pivoting on floats that never built; here the same
// e x (e + k) systematic system as above is reduced in HBM (L2-resident for the sizes that get here)
// panel by panel, with row pivoting and singular detection:
//   prep (1 WG)      pattern check and derivation (as above, counts in the workspace: n <= 65535)
//   gather (grid)    [M | B'] into the workspace, e rows of W = e + k symbols
//   for each panel of P pivot columns [c0, c0 + P):
//     panel (1 WG)   the e x P panel in LDS: Gauss-Jordan with row pivoting among the rows not yet
//                    pivots picks the P pivot rows pi (singular: status 1, every later kernel returns
//                    at once) and snapshots the panel A
//     ainv (1 WG)    A[pi]^-1 (P x P, Gauss-Jordan on [A[pi] | I] from the snapshot)
//     y (grid)       Y = A[pi]^-1 . M[pi] over columns [c0, W)
//     update (grid)  M[pi_j] = Y_j; every other row r: M_r += A_r . Y  (the rank-P update; columns
//                    before c0 are already reduced and Y is zero there)
//   finish (grid)    X[b] = M[piv(b)][e:] (pivot rows end normalised: no scaling), dm / tables /
//                    row pointers as the one-workgroup kernel writes them
// Work e^2 (e + k) GF(2^16) products over the panels (e = 500, k = 4000: ~1.1 G), spread over the
// chip instead of one CU; 4 launches per panel, all on `stream` (graph-capturable).
struct Ws16 {
  int* flags;     // [0] bad, [1] parity survivors, [2] singular
  int* cnt;       // [n]
  int* erased;    // [e]
  int* prow;      // [e]
  int* rows;      // [k]
  int* used;      // [e] pivot column + 1 of a row that is a pivot, 0 = not yet
  int* piv;       // [e] pivot row of column c
  uint16_t* ainv; // [P x P]
  uint16_t* asn;  // [e x P] panel snapshot
  uint16_t* y;    // [P x W]
  uint16_t* m;    // [e x ld]
  int ld;         // row stride of m (symbols)
};

constexpr int kPanelMax = 32;

__host__ __device__ constexpr size_t al256(size_t x) { return (x + 255) / 256 * 256; }

struct Ws16Layout {
  size_t off[11];
  size_t bytes;
  int ld;
};

__host__ __device__ inline Ws16Layout ws16_layout(int n, int k, int e, int P) {
  Ws16Layout L{};
  const int W = e + k;
  L.ld = (W + 7) / 8 * 8;
  const size_t sz[11] = {32, 4 * size_t(n), 4 * size_t(e), 4 * size_t(e), 4 * size_t(k), 4 * size_t(e),
                         4 * size_t(e), 2 * size_t(P) * P, 2 * size_t(e) * P, 2 * size_t(P) * W,
                         2 * size_t(e) * L.ld};
  size_t o = 0;
  for (int i = 0; i < 11; ++i) {
    L.off[i] = o;
    o += al256(sz[i]);
  }
  L.bytes = o;
  return L;
}

__host__ __device__ inline Ws16 ws16_of(void* base, int n, int k, int e, int P) {
  const Ws16Layout L = ws16_layout(n, k, e, P);
  char* b = static_cast<char*>(base);
  Ws16 w;
  w.flags = reinterpret_cast<int*>(b + L.off[0]);
  w.cnt = reinterpret_cast<int*>(b + L.off[1]);
  w.erased = reinterpret_cast<int*>(b + L.off[2]);
  w.prow = reinterpret_cast<int*>(b + L.off[3]);
  w.rows = reinterpret_cast<int*>(b + L.off[4]);
  w.used = reinterpret_cast<int*>(b + L.off[5]);
  w.piv = reinterpret_cast<int*>(b + L.off[6]);
  w.ainv = reinterpret_cast<uint16_t*>(b + L.off[7]);
  w.asn = reinterpret_cast<uint16_t*>(b + L.off[8]);
  w.y = reinterpret_cast<uint16_t*>(b + L.off[9]);
  w.m = reinterpret_cast<uint16_t*>(b + L.off[10]);
  w.ld = L.ld;
  return w;
}

// LDS of the panel kernel: product tables [4][16][P] u32 | panel [e][P] | used [e] | factors [e] |
// misc | pivots | pivot inverses
__host__ __device__ inline size_t panel_tab_bytes(int P) { return size_t(4) * 16 * P * 4; }
__host__ __device__ inline size_t panel_lds(int e, int P) {
  return panel_tab_bytes(P) + al256(size_t(e) * P * 2) + size_t(e) * 4 + size_t((e + 1) & ~1) * 2 + 16 +
         4 * kPanelMax + 2 * kPanelMax;
}

// panel width: the widest power of two <= 32 whose panel kernel fits the LDS
__host__ __device__ inline int panel_of(int e) {
  int P = kPanelMax;
  while (P > 4 && panel_lds(e, P) > kMaxLds16) P >>= 1;
  return P;
}

__device__ __forceinline__ bool ws_failed(const Ws16& w) {
  return *reinterpret_cast<volatile int*>(&w.flags[0]) || *reinterpret_cast<volatile int*>(&w.flags[2]);
}

__global__ __launch_bounds__(kThreads) void ds16_prep_kernel(const int* __restrict__ rows, int n, int k, int e,
                                                             Ws16 w, int* __restrict__ erased_out) {
  const int tid = threadIdx.x;
  constexpr int B = kThreads;
  __shared__ int bad_s, pcount_s;
  for (int i = tid; i < n; i += B) w.cnt[i] = 0;
  for (int i = tid; i < e; i += B) w.used[i] = 0;
  if (tid == 0) {
    bad_s = 0;
    pcount_s = 0;
  }
  __threadfence();  // (the zeroed counts reach L2 before any wave's atomics add to them)
  __syncthreads();
  for (int i = tid; i < k; i += B) {
    const int r = rows[i];
    const bool ok = r >= 0 && r < n;
    w.rows[i] = ok ? r : 0;
    if (ok) atomicAdd(&w.cnt[r], 1);
    else bad_s = 1;
  }
  __threadfence();  // (rows and counts visible past every wave's L1 before the ballots read them)
  __syncthreads();
  // (the counts were built by device-scope atomics in L2: read them past this CU's L1)
  auto count = [&](int i) { return __hip_atomic_load(&w.cnt[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  for (int i = tid; i < n; i += B)
    if (count(i) > 1) bad_s = 1;  // a chunk listed twice
  if (tid < 64) {  // erased natives (ascending) and parity survivors (survivor order)
    int base = 0;
    for (int i0 = 0; i0 < k; i0 += 64) {
      const int i = i0 + tid;
      const bool miss = i < k && count(i) == 0;
      const unsigned long long bal = __ballot(miss);
      const int a = base + __popcll(bal & ((1ull << tid) - 1ull));
      if (miss && a < e) w.erased[a] = i;
      base += __popcll(bal);
    }
    if (tid == 0 && base != e) bad_s = 1;
    int pbase = 0;
    for (int j0 = 0; j0 < k; j0 += 64) {
      const int j = j0 + tid;
      const bool is_par = j < k && __hip_atomic_load(&w.rows[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= k;
      const unsigned long long bal = __ballot(is_par);
      const int a = pbase + __popcll(bal & ((1ull << tid) - 1ull));
      if (is_par && a < e) w.prow[a] = __hip_atomic_load(&w.rows[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      pbase += __popcll(bal);
    }
    if (tid == 0) pcount_s = pbase;
  }
  __syncthreads();
  if (tid == 0) {
    w.flags[0] = bad_s;
    w.flags[1] = pcount_s;
    w.flags[2] = (bad_s || pcount_s != e) ? 1 : 0;
  }
  if (!bad_s)
    for (int i = tid; i < e; i += B) erased_out[i] = w.erased[i];
}

__global__ __launch_bounds__(kThreads) void ds16_gather_kernel(const uint16_t* __restrict__ g, int k, int e, Ws16 w) {
  if (ws_failed(w)) return;
  const int W = e + k;
  const int64_t total = int64_t(e) * W;
  for (int64_t i = int64_t(blockIdx.x) * kThreads + threadIdx.x; i < total; i += int64_t(gridDim.x) * kThreads) {
    const int a = int(i / W), col = int(i - int64_t(a) * W);
    const size_t grow = size_t(w.prow[a]) * k;
    uint16_t v;
    if (col < e) {
      v = g[grow + w.erased[col]];
    } else {
      const int r = w.rows[col - e];
      v = r < k ? g[grow + r] : uint16_t(r == w.prow[a]);
    }
    w.m[size_t(a) * w.ld + col] = v;
  }
}

// One panel [c0, c0 + P): pivot rows by Gauss-Jordan on the panel in LDS, and its snapshot.
// (1024 threads: one workgroup holds the whole panel, and its column loop is LDS-latency bound —
// 16 waves instead of 4 hide it: profiles/gf65536/r10_blocked_solve)
constexpr int kPanelThreads = 1024;
template <int P>
__global__ __launch_bounds__(kPanelThreads) void ds16_panel_kernel(int e, int c0, Ws16 w) {
  if (ws_failed(w)) return;
  static_assert(kPanelThreads % P == 0, "whole rows per pass");
  constexpr int kRP = kPanelThreads / P;  // rows per pass: lane tid works on column t = tid % P
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int B = kPanelThreads;
  const int tid = threadIdx.x;
  // ptab[(q * 16 + v) * P + t] = (pivot row value t) * (v << 4q): a product by a factor f is then
  // four nibble lookups (t fastest: the lanes of a row step hit spread banks)
  uint32_t* ptab = reinterpret_cast<uint32_t*>(smem);
  uint8_t* body = smem + panel_tab_bytes(P);
  uint16_t* pan = reinterpret_cast<uint16_t*>(body);                       // [e][P]
  int* used = reinterpret_cast<int*>(body + al256(size_t(e) * P * 2));     // [e]
  uint16_t* fcol = reinterpret_cast<uint16_t*>(used + e);                  // [e] (elimination factors)
  int* misc = reinterpret_cast<int*>(fcol + ((e + 1) & ~1));               // [0] bid, [1] fail, [2] inverse
  int* lpiv = misc + 4;                                                     // [P]
  uint16_t* linv = reinterpret_cast<uint16_t*>(lpiv + kPanelMax);        // [P] pivot inverses (ainv reuses)
  const int Pc = min(P, e - c0);
  const int tl = tid % P, rl = tid / P;
  for (int r0 = rl; r0 < e; r0 += 8 * kRP) {  // eight rows' loads in flight before their stores
    uint16_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = r0 + u * kRP;
      v[u] = (r < e && tl < Pc) ? w.m[size_t(r) * w.ld + c0 + tl] : uint16_t(0);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = r0 + u * kRP;
      if (r < e) {
        pan[r * P + tl] = v[u];
        w.asn[size_t(r) * P + tl] = v[u];
      }
    }
  }
  for (int i = tid; i < e; i += B) used[i] = w.used[i];
  if (tid == 0) misc[1] = 0;
  __syncthreads();
  for (int j = 0; j < Pc; ++j) {
    if (tid == 0) misc[0] = e;
    __syncthreads();
    {  // lowest unused row with a nonzero in column j: per lane, then per wave, one LDS atomic a wave
      int cand = e;
      for (int r = tid; r < e && cand == e; r += B)
        if (!used[r] && pan[r * P + j]) cand = r;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o));
      if ((tid & 63) == 0 && cand < e) atomicMin(&misc[0], cand);
    }
    __syncthreads();
    const int p = misc[0];
    if (p >= e) {  // no pivot in this column among the unused rows: singular (uniform)
      if (tid == 0) w.flags[2] = 1;
      return;
    }
    for (int r = tid; r < e; r += B) fcol[r] = pan[r * P + j];
    if (tid == 0) {
      used[p] = 1 + (c0 + j);
      lpiv[j] = p;
      misc[2] = int(inv16(pan[p * P + j]));
      linv[j] = uint16_t(misc[2]);
    }
    __syncthreads();
    const uint32_t iv = uint32_t(misc[2]);
    for (int t = tid; t < P; t += B) pan[p * P + t] = uint16_t(mul16(pan[p * P + t], iv));
    __syncthreads();
    // the scaled pivot row's nibble-product tables: one (t, q) pair per thread, 16 entries
    for (int tq = tid; tq < 4 * P; tq += B) nib_table(pan[p * P + tq % P], ptab + tq % P, P, tq / P);
    __syncthreads();
    // four rows per step, every LDS read of the step issued before its stores
    for (int r0 = rl; r0 < e; r0 += 4 * kRP) {
      uint32_t f[4], x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = r0 + u * kRP;
        f[u] = (r < e && r != p) ? uint32_t(fcol[r]) : 0u;
        x[u] = r < e ? uint32_t(pan[r * P + tl]) : 0u;
      }
      uint32_t d[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) d[u] = f[u] ? nib_mul(ptab + tl, P, f[u]) : 0u;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (f[u]) pan[(r0 + u * kRP) * P + tl] = uint16_t(x[u] ^ d[u]);
    }
    __syncthreads();
  }
  for (int j = tid; j < Pc; j += B) {
    w.piv[c0 + j] = lpiv[j];
    w.ainv[j] = linv[j];  // (read by ds16_ainv_kernel before it writes A[pi]^-1 there)
  }
  for (int r = tid; r < e; r += B) w.used[r] = used[r];
}

// A[pi]^-1 of the panel just factored: Gauss-Jordan on [A[pi] | I] (Pc x 2Pc) with the rows in the
// panel's pivot order. Restricted to the pivot rows, the panel kernel applied exactly these row
// operations, so step j's pivot is the one it found and its inverse is the one it computed (left in
// w.ainv[j]): no search, no swap, no inversion here. Its own launch: it reads the panel snapshot
// the panel kernel wrote, which another wave of that kernel's block could see stale in L1.
__global__ __launch_bounds__(kThreads) void ds16_ainv_kernel(int e, int c0, int P, Ws16 w) {
  if (ws_failed(w)) return;
  constexpr int B = kThreads;
  const int tid = threadIdx.x;
  __shared__ uint16_t aug[kPanelMax * 2 * kPanelMax];
  __shared__ uint16_t fcol[kPanelMax];
  __shared__ uint16_t pinv[kPanelMax];
  const int Pc = min(P, e - c0);
  const int P2 = 2 * Pc;
  for (int i = tid; i < Pc * P2; i += B) {
    const int a = i / P2, t = i - a * P2;
    aug[i] = t < Pc ? w.asn[size_t(w.piv[c0 + a]) * P + t] : uint16_t(t - Pc == a);
  }
  for (int j = tid; j < Pc; j += B) pinv[j] = w.ainv[j];
  __syncthreads();
  __shared__ uint16_t rtab[64 * 2 * kPanelMax];  // nibble tables of the scaled pivot row: [q * 16 + v][t]
  for (int j = 0; j < Pc; ++j) {
    const uint32_t iv = pinv[j];
    for (int t = tid; t < P2; t += B) aug[j * P2 + t] = uint16_t(mul16(aug[j * P2 + t], iv));
    for (int a = tid; a < Pc; a += B) fcol[a] = aug[a * P2 + j];
    __syncthreads();
    for (int tq = tid; tq < 4 * P2; tq += B) nib_table(aug[j * P2 + tq % P2], rtab + tq % P2, P2, tq / P2);
    __syncthreads();
    for (int i = tid; i < Pc * P2; i += B) {
      const int a = i / P2, t = i - a * P2;
      const uint32_t f = fcol[a];
      if (a != j && f) aug[i] = uint16_t(aug[i] ^ nib_mul(rtab + t, P2, f));
    }
    __syncthreads();
  }
  for (int i = tid; i < P * P; i += B) {
    const int a = i / P, t = i - a * P;
    w.ainv[i] = (a < Pc && t < Pc) ? aug[a * P2 + Pc + t] : uint16_t(0);
  }
}

// Y[j][col] = sum_i A[pi]^-1[j][i] M[pi_i][col], columns [c0, W); block (column block, j): the P
// coefficients of row j as nibble-product tables in LDS, so a product is four lookups
template <int P>
__global__ __launch_bounds__(kThreads) void ds16_y_kernel(int k, int e, int c0, Ws16 w) {
  if (ws_failed(w)) return;
  const int j = int(blockIdx.y);
  const int Pc = min(P, e - c0);
  if (j >= Pc) return;  // (uniform per block)
  constexpr int kS = P + 1;  // (odd row stride: lanes with different nibbles read different banks)
  __shared__ uint32_t tab[64 * kS];  // [q * 16 + v][i]
  __shared__ int pv[P];
  for (int iq = threadIdx.x; iq < 4 * P; iq += kThreads) nib_table(w.ainv[j * P + iq % P], tab + iq % P, kS, iq / P);
  for (int i = threadIdx.x; i < Pc; i += kThreads) pv[i] = w.piv[c0 + i];
  __syncthreads();
  const int W = e + k;
  const int col = c0 + int(blockIdx.x) * kThreads + int(threadIdx.x);
  if (col >= W) return;
  uint32_t acc = 0;
  for (int i = 0; i < Pc; ++i) {
    const uint32_t x = w.m[size_t(pv[i]) * w.ld + col];
    acc ^= nib_mul(tab + i, kS, x);
  }
  w.y[size_t(j) * W + col] = uint16_t(acc);
}

// rank-P update of rows [r0, r0 + kRowsPerBlock) over columns [c0, W): the block's rows' panel
// coefficients as nibble-product tables in LDS (kRowsPerBlock x P tables of 64 words)
constexpr int kRowsPerBlock = 8;
template <int P>
__global__ __launch_bounds__(kThreads) void ds16_update_kernel(int k, int e, int c0, Ws16 w) {
  if (ws_failed(w)) return;
  const int W = e + k;
  const int Pc = min(P, e - c0);
  const int r0 = int(blockIdx.y) * kRowsPerBlock;
  const int nr = min(e - r0, kRowsPerBlock);
  constexpr int kT = kRowsPerBlock * P;  // tables, interleaved: [q * 16 + v][row * P + j]
  // (row stride kT + 2 halfwords = an odd number of banks: lanes with different nibbles v read
  // different banks; at kT the 16 values of v all hit one bank)
  constexpr int kTs = kT + 2;
  __shared__ uint16_t tab[64 * kTs];      // (~32 KiB at P = 32)
  for (int iq = threadIdx.x; iq < 4 * kT; iq += kThreads) {
    const int t = iq % kT, rr = t / P, j = t - rr * P;
    nib_table(rr < nr && j < Pc ? uint32_t(w.asn[size_t(r0 + rr) * P + j]) : 0u, tab + t, kTs, iq / kT);
  }
  __syncthreads();
  const int col = c0 + int(blockIdx.x) * kThreads + int(threadIdx.x);
  if (col >= W) return;
  uint16_t y[P];
#pragma unroll
  for (int j = 0; j < P; ++j) y[j] = j < Pc ? w.y[size_t(j) * W + col] : uint16_t(0);
  for (int rr = 0; rr < nr; ++rr) {
    const int r = r0 + rr;
    const int u = w.used[r] - 1;  // pivot column of row r, if any
    uint16_t* dst = w.m + size_t(r) * w.ld + col;
    if (u >= c0 && u < c0 + Pc) {
      *dst = y[u - c0];
      continue;
    }
    uint32_t acc = *dst;
#pragma unroll
    for (int j = 0; j < P; ++j)
      if (j < Pc) acc ^= nib_mul(tab + rr * P + j, kTs, y[j]);
    *dst = uint16_t(acc);
  }
}

// X[b] = M[piv[b]][e:], then dm / tables / row pointers (as gf_decode_system16_kernel's epilogue)
__global__ __launch_bounds__(kThreads) void ds16_finish_kernel(int n, int k, int e, Ws16 w, uint16_t* __restrict__ dm,
                                                               int* __restrict__ status, uint32_t* __restrict__ tab,
                                                               int m_pad, const uint64_t* __restrict__ ptrs,
                                                               uint64_t* __restrict__ dptr) {
  const int bad = w.flags[0];
  const int singular = bad || w.flags[2];
  const int64_t tid = int64_t(blockIdx.x) * kThreads + threadIdx.x;
  const int64_t nthr = int64_t(gridDim.x) * kThreads;
  if (tid == 0 && status) *status = bad ? 2 : singular;
  if (dptr) {
    const uint64_t* outp = ptrs + n;
    for (int64_t j = tid; j < k; j += nthr) {
      const int rr = w.rows[j];
      dptr[j] = ptrs[rr];
      dptr[k + j] = (!singular && rr < k) ? outp[rr] : 0;
    }
    for (int64_t i = tid; i < m_pad; i += nthr) dptr[2 * k + i] = (!singular && i < e) ? outp[w.erased[i]] : 0;
  }
  auto x_at = [&](int b, int j) -> uint32_t { return w.m[size_t(w.piv[b]) * w.ld + e + j]; };
  if (dm)
    for (int64_t i = tid; i < int64_t(e) * k; i += nthr) {
      const int b = int(i / k), j = int(i - int64_t(b) * k);
      dm[i] = singular ? uint16_t(0) : uint16_t(x_at(b, j));
    }
  if (tab && !singular)
    for (int64_t idx = tid; idx < int64_t(k) * e; idx += nthr) {
      const int j = int(idx / e), b = int(idx - int64_t(j) * e);
      uint32_t q[4][5];
      quad_of(x_at(b, j), q);
      uint32_t* dst = tab + (size_t(j) * m_pad + b) * 4 * kPermStride;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
#pragma unroll
        for (int v = 0; v < 5; ++v) dst[qq * kPermStride + v] = q[qq][v];
        dst[qq * kPermStride + 5] = dst[qq * kPermStride + 6] = dst[qq * kPermStride + 7] = 0;
      }
    }
}

template <int P>
hipError_t launch_blocked16(const uint16_t* g, int n, int k, const int* rows, int* erased, int e, uint16_t* dm,
                            int* status, uint32_t* tab, int m_pad, const uint64_t* ptrs, uint64_t* dptr, void* ws,
                            hipStream_t stream) {
  const Ws16 w = ws16_of(ws, n, k, e, P);
  const int W = e + k;
  ds16_prep_kernel<<<1, kThreads, 0, stream>>>(rows, n, k, e, w, erased);
  const int64_t cells = int64_t(e) * W;
  const unsigned gblocks = unsigned(std::min<int64_t>((cells + kThreads - 1) / kThreads, 8 * 256));
  ds16_gather_kernel<<<gblocks, kThreads, 0, stream>>>(g, k, e, w);
  const size_t plds = panel_lds(e, P);
  if (plds > 65536) {
    const hipError_t err = ensure_lds_optin(reinterpret_cast<const void*>(&ds16_panel_kernel<P>));
    if (err != hipSuccess) return err;
  }
  for (int c0 = 0; c0 < e; c0 += P) {
    ds16_panel_kernel<P><<<1, kPanelThreads, plds, stream>>>(e, c0, w);
    ds16_ainv_kernel<<<1, kThreads, 0, stream>>>(e, c0, P, w);
    const unsigned cb = unsigned((W - c0 + kThreads - 1) / kThreads);
    ds16_y_kernel<P><<<dim3(cb, unsigned(P)), kThreads, 0, stream>>>(k, e, c0, w);
    ds16_update_kernel<P><<<dim3(cb, unsigned((e + kRowsPerBlock - 1) / kRowsPerBlock)), kThreads, 0, stream>>>(
        k, e, c0, w);
  }
  const int64_t fin = std::max<int64_t>(int64_t(k) * e, std::max(k, m_pad));
  const unsigned fblocks = unsigned(std::min<int64_t>((fin + kThreads - 1) / kThreads, 4 * 256));
  ds16_finish_kernel<<<fblocks, kThreads, 0, stream>>>(n, k, e, w, dm, status, tab, m_pad, ptrs, dptr);
  return hipGetLastError();
}

bool blocked16_fits(int n, int k, int e) {
  return k >= 1 && e >= 1 && e <= k && n >= k + e && n <= 65535 && panel_lds(e, panel_of(e)) <= kMaxLds16;
}

}  // namespace

bool decode_system16_supported(int n, int k, int e) {
  return k >= 1 && e >= 1 && e <= k && e <= kThreads && n >= k + e && lds16(n, k, e) <= kMaxLds16;
}

int64_t decode_system16_workspace(int n, int k, int e) {
  if (!blocked16_fits(n, k, e)) return -1;
  return int64_t(ws16_layout(n, k, e, panel_of(e)).bytes);
}

hipError_t launch_gf_decode_system16(const uint16_t* g, int n, int k, const int* rows, int* erased, int e,
                                     uint16_t* dm, int* status, void* desc, int m_pad, hipStream_t stream,
                                     const uint64_t* ptrs, void* workspace, bool force_blocked) {
  if (!erased || (desc && e > m_pad) || (ptrs && !desc)) return hipErrorInvalidValue;
  uint32_t* tab = nullptr;
  uint64_t* dptr = nullptr;
  if (desc) {
    const DescLayout l = desc_layout16(k, m_pad);
    tab = reinterpret_cast<uint32_t*>(static_cast<char*>(desc) + l.tab_off);
    if (ptrs) dptr = reinterpret_cast<uint64_t*>(static_cast<char*>(desc) + l.in_off);
  }
  if (force_blocked || !decode_system16_supported(n, k, e)) {  // the blocked multi-workgroup solve
    if (!workspace || !blocked16_fits(n, k, e)) return hipErrorInvalidValue;
    switch (panel_of(e)) {
      case 32: return launch_blocked16<32>(g, n, k, rows, erased, e, dm, status, tab, m_pad, ptrs, dptr, workspace, stream);
      case 16: return launch_blocked16<16>(g, n, k, rows, erased, e, dm, status, tab, m_pad, ptrs, dptr, workspace, stream);
      case 8: return launch_blocked16<8>(g, n, k, rows, erased, e, dm, status, tab, m_pad, ptrs, dptr, workspace, stream);
      default: return launch_blocked16<4>(g, n, k, rows, erased, e, dm, status, tab, m_pad, ptrs, dptr, workspace, stream);
    }
  }
  const size_t lds = lds16(n, k, e);
  if (lds > 65536) {
    const hipError_t err = ensure_lds_optin(reinterpret_cast<const void*>(&gf_decode_system16_kernel));
    if (err != hipSuccess) return err;
  }
  gf_decode_system16_kernel<<<1, kSysThreads, lds, stream>>>(g, n, k, rows, erased, e, dm, status, tab, m_pad, ptrs, dptr);
  return hipGetLastError();
}

}  // namespace gfrs

// CPU GF(2^8) GEMM with the reference's multiply strategies (see gfrs/cpu_codec.h).
#include "gfrs/cpu_codec.h"

#include <immintrin.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace gfrs {
namespace {

// ---- strategy tables, generated once -------------------------------------------------------
struct CpuTables {
  uint8_t exp255[256];   // exp[0..254], exp[255] = exp[0] (variant 1)
  uint8_t exp509[509];   // two periods (variant 2)
  uint8_t full[256][256];
  uint8_t nib_hi[16][256];  // (h << 4) * b
  uint8_t nib_lo[16][256];  // l * b
  CpuTables() {
    for (int i = 0; i < 255; ++i) exp255[i] = kTables.exp[i];
    exp255[255] = kTables.exp[0];
    for (int i = 0; i < 509; ++i) exp509[i] = kTables.exp[i % 255];
    for (int a = 0; a < 256; ++a)
      for (int b = 0; b < 256; ++b) full[a][b] = mul(uint8_t(a), uint8_t(b));
    for (int h = 0; h < 16; ++h)
      for (int b = 0; b < 256; ++b) {
        nib_hi[h][b] = full[h << 4][b];
        nib_lo[h][b] = full[h][b];
      }
  }
};

const CpuTables& tables() {
  static const CpuTables t;
  return t;
}

inline uint8_t m_logexp(uint8_t a, uint8_t b) {
  if (!a || !b) return 0;
  int s = kTables.log[a] + kTables.log[b];
  if (s >= 255) s -= 255;
  return kTables.exp[s];
}
inline uint8_t m_mod(uint8_t a, uint8_t b) {
  if (!a || !b) return 0;
  return kTables.exp[(kTables.log[a] + kTables.log[b]) % 255];
}
inline uint8_t m_fold(uint8_t a, uint8_t b) {
  if (!a || !b) return 0;
  const int s = kTables.log[a] + kTables.log[b];
  return tables().exp255[(s & 255) + (s >> 8)];
}
inline uint8_t m_double(uint8_t a, uint8_t b) {
  if (!a || !b) return 0;
  return tables().exp509[kTables.log[a] + kTables.log[b]];
}
inline uint8_t m_zeroband(uint8_t a, uint8_t b) { return kTables.exp[kTables.log[a] + kTables.log[b]]; }
inline uint8_t m_full(uint8_t a, uint8_t b) { return tables().full[a][b]; }
inline uint8_t m_nibble(uint8_t a, uint8_t b) { return tables().nib_hi[a >> 4][b] ^ tables().nib_lo[a & 15][b]; }

// out ^= c * in, 32 bytes per step: c * x = lo[x & 15] ^ hi[x >> 4] (GF multiply is linear over
// GF(2), so the two nibbles multiply separately), each 16-entry table one pshufb.
__attribute__((target("avx2"))) void axpy_avx2(uint8_t c, const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                               int64_t n) {
  const uint8_t* row = tables().full[c];
  alignas(16) uint8_t lo[16], hi[16];
  for (int x = 0; x < 16; ++x) {
    lo[x] = row[x];
    hi[x] = row[x << 4];
  }
  const __m256i tl = _mm256_broadcastsi128_si256(_mm_load_si128(reinterpret_cast<const __m128i*>(lo)));
  const __m256i th = _mm256_broadcastsi128_si256(_mm_load_si128(reinterpret_cast<const __m128i*>(hi)));
  const __m256i mask = _mm256_set1_epi8(0x0f);
  int64_t x = 0;
  for (; x + 32 <= n; x += 32) {
    const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(in + x));
    const __m256i l = _mm256_shuffle_epi8(tl, _mm256_and_si256(v, mask));
    const __m256i h = _mm256_shuffle_epi8(th, _mm256_and_si256(_mm256_srli_epi16(v, 4), mask));
    const __m256i o = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(out + x));
    _mm256_storeu_si256(reinterpret_cast<__m256i*>(out + x), _mm256_xor_si256(o, _mm256_xor_si256(l, h)));
  }
  for (; x < n; ++x) out[x] ^= row[in[x]];
}

// Register-blocked form for the whole GEMM over columns [a, b): groups of up to 4 output rows stay
// in ymm accumulators while every input row's 32 bytes are loaded once per group, split into
// nibbles once, and hit with each coefficient's two table shuffles (the tables sit in L1).
__attribute__((target("avx2"))) void gemm_avx2(const std::vector<const uint8_t*>& in, const std::vector<uint8_t*>& out,
                                               const Mat& coeff, int64_t a, int64_t b) {
  const int k = int(in.size()), m = int(out.size());
  struct alignas(32) Y {
    __m256i v;
  };
  std::vector<Y> tl(size_t(m) * k), th(size_t(m) * k);  // (C++17 aligned new: 32-byte elements)
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < k; ++j) {
      const uint8_t* row = tables().full[coeff[size_t(i) * k + j]];
      alignas(16) uint8_t lo[16], hi[16];
      for (int x = 0; x < 16; ++x) {
        lo[x] = row[x];
        hi[x] = row[x << 4];
      }
      tl[size_t(i) * k + j].v = _mm256_broadcastsi128_si256(_mm_load_si128(reinterpret_cast<const __m128i*>(lo)));
      th[size_t(i) * k + j].v = _mm256_broadcastsi128_si256(_mm_load_si128(reinterpret_cast<const __m128i*>(hi)));
    }
  const __m256i mask = _mm256_set1_epi8(0x0f);
  const int64_t vend = a + (b - a) / 32 * 32;
  constexpr int64_t kTile = 16 << 10;  // column tile: the k input slices stay in L2 across row groups
  for (int64_t t0 = a; t0 < vend; t0 += kTile) {
    const int64_t t1 = std::min(vend, t0 + kTile);
    for (int i0 = 0; i0 < m; i0 += 4) {
      const int g = std::min(4, m - i0);
      for (int64_t x = t0; x < t1; x += 32) {
        __m256i acc[4] = {_mm256_setzero_si256(), _mm256_setzero_si256(), _mm256_setzero_si256(),
                          _mm256_setzero_si256()};
        for (int j = 0; j < k; ++j) {
          const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(in[j] + x));
          const __m256i l = _mm256_and_si256(v, mask);
          const __m256i h = _mm256_and_si256(_mm256_srli_epi16(v, 4), mask);
          for (int t = 0; t < g; ++t) {
            const size_t c = size_t(i0 + t) * k + j;
            const __m256i prod = _mm256_xor_si256(_mm256_shuffle_epi8(tl[c].v, l), _mm256_shuffle_epi8(th[c].v, h));
            acc[t] = _mm256_xor_si256(acc[t], prod);
          }
        }
        for (int t = 0; t < g; ++t) _mm256_storeu_si256(reinterpret_cast<__m256i*>(out[i0 + t] + x), acc[t]);
      }
    }
  }
  for (int i = 0; i < m && vend < b; ++i) {  // ragged tail, scalar
    uint8_t* o = out[i];
    for (int64_t x = vend; x < b; ++x) {
      uint8_t r = 0;
      for (int j = 0; j < k; ++j) r ^= tables().full[coeff[size_t(i) * k + j]][in[j][x]];
      o[x] = r;
    }
  }
}

bool host_has_avx2() {
  static const bool has = __builtin_cpu_supports("avx2");
  return has;
}

// Per-row kernel for one coefficient c over bytes [0, n): out ^= c * in.
template <CpuMul S>
void axpy(uint8_t c, const uint8_t* __restrict__ in, uint8_t* __restrict__ out, int64_t n) {
  if (c == 0) return;
  if (c == 1) {
    for (int64_t x = 0; x < n; ++x) out[x] ^= in[x];
    return;
  }
  if constexpr (S == CpuMul::kSimd) {
    if (host_has_avx2()) return axpy_avx2(c, in, out, n);
    const uint8_t* row = tables().full[c];
    for (int64_t x = 0; x < n; ++x) out[x] ^= row[in[x]];
  } else if constexpr (S == CpuMul::kRow || S == CpuMul::kFull) {
    const uint8_t* row = tables().full[c];
    for (int64_t x = 0; x < n; ++x) out[x] ^= row[in[x]];
  } else if constexpr (S == CpuMul::kPerm) {
    const PermTable t = perm_for_coeff(c);
    for (int64_t x = 0; x < n; ++x) out[x] ^= perm_apply(t, in[x]);
  } else {
    for (int64_t x = 0; x < n; ++x) out[x] ^= cpu_mul(S, in[x], c);
  }
}

template <CpuMul S>
void gemm_range(const std::vector<const uint8_t*>& in, const std::vector<uint8_t*>& out, const Mat& coeff, int64_t a,
                int64_t b) {
  if constexpr (S == CpuMul::kSimd) {
    if (host_has_avx2()) return gemm_avx2(in, out, coeff, a, b);
  }
  const int k = int(in.size()), m = int(out.size());
  constexpr int64_t kTile = 32 << 10;  // keep the k input tiles + m outputs L2-resident
  for (int64_t t = a; t < b; t += kTile) {
    const int64_t n = std::min(kTile, b - t);
    for (int i = 0; i < m; ++i) {
      uint8_t* o = out[i] + t;
      std::memset(o, 0, size_t(n));
      for (int j = 0; j < k; ++j) axpy<S>(coeff[size_t(i) * k + j], in[j] + t, o, n);
    }
  }
}

template <CpuMul S>
void gemm_threads(const std::vector<const uint8_t*>& in, const std::vector<uint8_t*>& out, const Mat& coeff,
                  int64_t ncols, int threads) {
  if (threads <= 1 || ncols < (1 << 20)) {
    gemm_range<S>(in, out, coeff, 0, ncols);
    return;
  }
  std::vector<std::thread> th;
  const int64_t per = (ncols + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const int64_t a = int64_t(t) * per, b = std::min(ncols, a + per);
    if (a >= b) break;
    th.emplace_back([&, a, b] { gemm_range<S>(in, out, coeff, a, b); });
  }
  for (auto& x : th) x.join();
}

}  // namespace

CpuMul parse_cpu_mul(const std::string& s) {
  static const std::array<const char*, 11> names = {"logexp", "logexp0", "logexp1", "logexp2", "logexp3", "loop",
                                                    "full",   "double",  "perm",    "row",     "simd"};
  for (size_t i = 0; i < names.size(); ++i)
    if (s == names[i]) return CpuMul(i);
  throw std::invalid_argument("unknown CPU multiply strategy: " + s);
}

const char* cpu_mul_name(CpuMul m) {
  static const char* names[] = {"logexp", "logexp0", "logexp1", "logexp2", "logexp3", "loop",
                                "full",   "double",  "perm",    "row",     "simd"};
  return names[int(m)];
}

uint8_t cpu_mul(CpuMul s, uint8_t a, uint8_t b) {
  switch (s) {
    case CpuMul::kLogExp: return m_logexp(a, b);
    case CpuMul::kLogExpMod: return m_mod(a, b);
    case CpuMul::kLogExpFold: return m_fold(a, b);
    case CpuMul::kLogExpDouble: return m_double(a, b);
    case CpuMul::kZeroBand: return m_zeroband(a, b);
    case CpuMul::kLoop: return mul_loop(a, b);
    case CpuMul::kFull: return m_full(a, b);
    case CpuMul::kNibble: return m_nibble(a, b);
    case CpuMul::kPerm: return perm_apply(perm_for_coeff(b), a);
    case CpuMul::kRow: return m_full(a, b);
    case CpuMul::kSimd: return m_nibble(a, b);
  }
  return 0;
}

void cpu_gemm(const std::vector<const uint8_t*>& in, const std::vector<uint8_t*>& out, const Mat& coeff,
              int64_t ncols, CpuMul s, int threads) {
  const int k = int(in.size()), m = int(out.size());
  if (coeff.size() != size_t(m) * k) throw std::invalid_argument("cpu_gemm: coeff must be m x k");
  if (threads <= 0) threads = int(std::max(1u, std::thread::hardware_concurrency()));
  switch (s) {
    case CpuMul::kLogExp: return gemm_threads<CpuMul::kLogExp>(in, out, coeff, ncols, threads);
    case CpuMul::kLogExpMod: return gemm_threads<CpuMul::kLogExpMod>(in, out, coeff, ncols, threads);
    case CpuMul::kLogExpFold: return gemm_threads<CpuMul::kLogExpFold>(in, out, coeff, ncols, threads);
    case CpuMul::kLogExpDouble: return gemm_threads<CpuMul::kLogExpDouble>(in, out, coeff, ncols, threads);
    case CpuMul::kZeroBand: return gemm_threads<CpuMul::kZeroBand>(in, out, coeff, ncols, threads);
    case CpuMul::kLoop: return gemm_threads<CpuMul::kLoop>(in, out, coeff, ncols, threads);
    case CpuMul::kFull: return gemm_threads<CpuMul::kFull>(in, out, coeff, ncols, threads);
    case CpuMul::kNibble: return gemm_threads<CpuMul::kNibble>(in, out, coeff, ncols, threads);
    case CpuMul::kPerm: return gemm_threads<CpuMul::kPerm>(in, out, coeff, ncols, threads);
    case CpuMul::kRow: return gemm_threads<CpuMul::kRow>(in, out, coeff, ncols, threads);
    case CpuMul::kSimd: return gemm_threads<CpuMul::kSimd>(in, out, coeff, ncols, threads);
  }
}

}  // namespace gfrs

namespace gfrs {
namespace {

// Symbols [s0, s1) of every output: per coefficient two 256-entry product tables, c * l and
// c * (h << 8), built once per (i, j) and applied to the column range in one pass.
void gemm16_range(const std::vector<const uint8_t*>& in, const std::vector<uint8_t*>& out, const gf16w::Mat& coeff,
                  int64_t s0, int64_t s1) {
  const int k = int(in.size()), m = int(out.size());
  std::vector<uint16_t> acc(size_t(s1 - s0));
  uint16_t tlo[256], thi[256];
  for (int i = 0; i < m; ++i) {
    std::fill(acc.begin(), acc.end(), uint16_t(0));
    for (int j = 0; j < k; ++j) {
      const uint16_t c = coeff[size_t(i) * k + j];
      if (!c) continue;
      for (int x = 0; x < 256; ++x) {
        tlo[x] = gf16w::mul(c, static_cast<uint16_t>(x));
        thi[x] = gf16w::mul(c, static_cast<uint16_t>(x << 8));
      }
      const uint8_t* src = in[j] + 2 * s0;
      for (int64_t s = 0; s < s1 - s0; ++s) acc[size_t(s)] ^= tlo[src[2 * s]] ^ thi[src[2 * s + 1]];
    }
    uint8_t* dst = out[i] + 2 * s0;
    for (int64_t s = 0; s < s1 - s0; ++s) {
      dst[2 * s] = static_cast<uint8_t>(acc[size_t(s)] & 0xFF);
      dst[2 * s + 1] = static_cast<uint8_t>(acc[size_t(s)] >> 8);
    }
  }
}

}  // namespace

void cpu_gemm16(const std::vector<const uint8_t*>& in, const std::vector<uint8_t*>& out, const gf16w::Mat& coeff,
                int64_t ncols, int threads) {
  const int k = int(in.size()), m = int(out.size());
  if (coeff.size() != size_t(m) * k) throw std::invalid_argument("cpu_gemm16: coeff must be m x k");
  if (ncols % 2) throw std::invalid_argument("cpu_gemm16: ncols must be an even byte count (16-bit symbols)");
  if (threads <= 0) threads = int(std::max(1u, std::thread::hardware_concurrency()));
  const int64_t nsym = ncols / 2;
  // chunks of at most 1 Mi symbols keep each thread's accumulator row in cache-friendly size
  const int64_t per = std::max<int64_t>(1, std::min<int64_t>(1 << 20, (nsym + threads - 1) / threads));
  std::vector<std::thread> th;
  std::atomic<int64_t> next{0};
  for (int t = 0; t < threads; ++t)
    th.emplace_back([&] {
      for (int64_t a; (a = next.fetch_add(per)) < nsym;) gemm16_range(in, out, coeff, a, std::min(nsym, a + per));
    });
  for (auto& x : th) x.join();
}

}  // namespace gfrs

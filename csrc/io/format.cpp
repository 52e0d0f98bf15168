// File formats (see gfrs/format.h). 64-bit sizes throughout; tails zero-padded (the reference's GPU
// encoder leaves padding uninitialised, src/encode.cu:325).
#include "gfrs/format.h"
#include "gfrs/tune.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace gfrs {
namespace {

void split_path(const std::string& p, std::string& dir, std::string& base) {
  const size_t s = p.find_last_of('/');
  if (s == std::string::npos) {
    dir.clear();
    base = p;
  } else {
    dir = p.substr(0, s + 1);
    base = p.substr(s + 1);
  }
}

bool exists(const std::string& p) {
  struct stat sb;
  return ::stat(p.c_str(), &sb) == 0;
}

}  // namespace

std::string chunk_path(const std::string& file, int index) {
  std::string dir, base;
  split_path(file, dir, base);
  return dir + "_" + std::to_string(index) + "_" + base;
}

std::string metadata_path(const std::string& file) { return file + ".METADATA"; }

int chunk_index(const std::string& name) {
  std::string dir, base;
  split_path(name, dir, base);
  if (base.size() < 2 || base[0] != '_') return -1;
  char* end = nullptr;
  const long v = std::strtol(base.c_str() + 1, &end, 10);
  if (end == base.c_str() + 1 || v < 0) return -1;
  return int(v);
}

namespace {

// slicing-by-8 CRC-32 (IEEE 802.3, reflected 0xEDB88320) on the inverted register value
uint32_t crc32_slice8(const uint8_t* data, int64_t len, uint32_t state) {
  static uint32_t t[8][256];
  static bool init = [] {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int b = 0; b < 8; ++b) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
    return true;
  }();
  (void)init;
  uint32_t crc = state;
  int64_t i = 0;
  for (; i + 8 <= len; i += 8) {
    uint32_t lo, hi;
    std::memcpy(&lo, data + i, 4);
    std::memcpy(&hi, data + i + 4, 4);
    lo ^= crc;
    crc = t[7][lo & 0xFF] ^ t[6][(lo >> 8) & 0xFF] ^ t[5][(lo >> 16) & 0xFF] ^ t[4][lo >> 24] ^ t[3][hi & 0xFF] ^
          t[2][(hi >> 8) & 0xFF] ^ t[1][(hi >> 16) & 0xFF] ^ t[0][hi >> 24];
  }
  for (; i < len; ++i) crc = (crc >> 8) ^ t[0][(crc ^ data[i]) & 0xFF];
  return crc;
}

#if defined(__x86_64__)
// Carry-less-multiply folding (the method of Intel's "Fast CRC Computation for Generic Polynomials
// Using PCLMULQDQ"): four 128-bit lanes folded 64 bytes at a time, then into one lane, then 128 ->
// 64 -> 32 bits with a Barrett reduction. The constants are x^k mod P for the bit-reflected
// CRC-32 polynomial (k1/k2: the 512-bit fold, k3/k4: 128-bit, k5: 64-bit; P' and mu for Barrett).
// len >= 64 and a multiple of 16; works on the inverted register value like crc32_slice8. The
// survivor check of a decode reads and checks up to k whole chunks before any GPU work, so it is
// on the critical path of every file decode.
#define GFRS_CLMUL __attribute__((target("pclmul,sse4.1")))
GFRS_CLMUL inline __m128i ld128(const uint8_t* p) { return _mm_loadu_si128(reinterpret_cast<const __m128i*>(p)); }
// acc folded across 128 bits by the constant pair k (low x low, high x high) into next
GFRS_CLMUL inline __m128i fold128(__m128i acc, __m128i next, __m128i k) {
  const __m128i lo = _mm_clmulepi64_si128(acc, k, 0x00);
  return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(acc, k, 0x11), next), lo);
}
GFRS_CLMUL uint32_t crc32_clmul(const uint8_t* buf, int64_t len, uint32_t state) {
  alignas(16) static const uint64_t k1k2[2] = {0x0154442bd4ull, 0x01c6e41596ull};
  alignas(16) static const uint64_t k3k4[2] = {0x01751997d0ull, 0x00ccaa009eull};
  alignas(16) static const uint64_t k5k0[2] = {0x0163cd6124ull, 0x0000000000ull};
  alignas(16) static const uint64_t poly[2] = {0x01db710641ull, 0x01f7011641ull};
  __m128i x1 = ld128(buf), x2 = ld128(buf + 16), x3 = ld128(buf + 32), x4 = ld128(buf + 48);
  x1 = _mm_xor_si128(x1, _mm_cvtsi32_si128(int(state)));
  __m128i x0 = _mm_load_si128(reinterpret_cast<const __m128i*>(k1k2));
  buf += 64;
  len -= 64;
  while (len >= 64) {
    x1 = fold128(x1, ld128(buf), x0);
    x2 = fold128(x2, ld128(buf + 16), x0);
    x3 = fold128(x3, ld128(buf + 32), x0);
    x4 = fold128(x4, ld128(buf + 48), x0);
    buf += 64;
    len -= 64;
  }
  x0 = _mm_load_si128(reinterpret_cast<const __m128i*>(k3k4));
  x1 = fold128(x1, x2, x0);
  x1 = fold128(x1, x3, x0);
  x1 = fold128(x1, x4, x0);
  while (len >= 16) {
    x1 = fold128(x1, ld128(buf), x0);
    buf += 16;
    len -= 16;
  }
  // 128 -> 64 bits
  __m128i x2b = _mm_clmulepi64_si128(x1, x0, 0x10);
  const __m128i mask = _mm_setr_epi32(~0, 0, ~0, 0);
  x1 = _mm_xor_si128(_mm_srli_si128(x1, 8), x2b);
  x0 = _mm_loadl_epi64(reinterpret_cast<const __m128i*>(k5k0));
  x2b = _mm_srli_si128(x1, 4);
  x1 = _mm_xor_si128(_mm_clmulepi64_si128(_mm_and_si128(x1, mask), x0, 0x00), x2b);
  // Barrett reduction to 32 bits
  x0 = _mm_load_si128(reinterpret_cast<const __m128i*>(poly));
  x2b = _mm_clmulepi64_si128(_mm_and_si128(x1, mask), x0, 0x10);
  x2b = _mm_clmulepi64_si128(_mm_and_si128(x2b, mask), x0, 0x00);
  x1 = _mm_xor_si128(x1, x2b);
  return uint32_t(_mm_extract_epi32(x1, 1));
}

bool have_clmul() {
  static const bool v = [] {
    if (tune_str("crc") == "scalar") return false;  // (tests: the table path on the same machine)
    __builtin_cpu_init();
    return __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
  }();
  return v;
}
#endif

}  // namespace

int verify_threads() {
  static const int v = [] {
    const char* e = std::getenv("GFRS_VERIFY_THREADS");
    const int n = e ? std::atoi(e) : 16;
    return n < 1 ? 1 : n;
  }();
  return v;
}

uint32_t crc32(const uint8_t* data, int64_t len, uint32_t crc) {
  uint32_t state = ~crc;
#if defined(__x86_64__)
  if (len >= 64 && have_clmul()) {
    const int64_t n = len & ~int64_t(15);
    state = crc32_clmul(data, n, state);
    data += n;
    len -= n;
  }
#endif
  return ~crc32_slice8(data, len, state);
}

namespace {
// 32 x 32 GF(2) matrices as 32 column words: op[i] = image of register bit i
uint32_t gf2_apply(const uint32_t op[32], uint32_t v) {
  uint32_t r = 0;
  for (int i = 0; v; ++i, v >>= 1)
    if (v & 1u) r ^= op[i];
  return r;
}
void gf2_compose(uint32_t out[32], const uint32_t a[32], const uint32_t b[32]) {  // out = a . b
  for (int i = 0; i < 32; ++i) out[i] = gf2_apply(a, b[i]);
}
}  // namespace

uint32_t crc32_combine(uint32_t crc_a, uint32_t crc_b, int64_t len_b) {
  if (len_b <= 0) return crc_a ^ crc_b;  // (crc of nothing is 0)
  // one zero bit through the reflected register: bit 0 falls out through the polynomial, every
  // other bit moves down by one
  uint32_t step[32], tmp[32];
  step[0] = 0xEDB88320u;
  for (int i = 1; i < 32; ++i) step[i] = 1u << (i - 1);
  for (int s = 0; s < 3; ++s) {  // one zero byte: the bit operator squared three times (2^3 bits)
    gf2_compose(tmp, step, step);
    std::memcpy(step, tmp, sizeof(step));
  }
  uint32_t reg = crc_a;
  for (int64_t n = len_b; n; n >>= 1) {  // step = byte operator ^ (2^j) at bit j of len_b
    if (n & 1) reg = gf2_apply(step, reg);
    if (n > 1) {
      gf2_compose(tmp, step, step);
      std::memcpy(step, tmp, sizeof(step));
    }
  }
  return reg ^ crc_b;
}

namespace {

// the metadata text of either form, built in memory (one atomic commit below)
void matrix_lines(std::ostringstream& o, int p, int k, const std::vector<int>& e) {
  for (int i = 0; i < k; ++i) {
    for (int j = 0; j < k; ++j) o << (i == j ? "1 " : "0 ");
    o << '\n';
  }
  for (int i = 0; i < p; ++i) {
    for (int j = 0; j < k; ++j) o << e[size_t(i) * k + j] << ' ';
    o << '\n';
  }
}

void crc_line(std::ostringstream& o, const std::vector<uint32_t>& crc) {
  if (crc.empty()) return;
  o << "crc32";
  char hex[16];
  for (uint32_t c : crc) {
    std::snprintf(hex, sizeof(hex), " %08x", c);
    o << hex;
  }
  o << '\n';
}

[[noreturn]] void io_fail(const std::string& what, const std::string& path, int err) {
  throw std::runtime_error(what + " " + path + ": " + std::strerror(err));
}

void write_all_fd(int fd, const uint8_t* src, int64_t len, const std::string& path) {
  int64_t put = 0;
  while (put < len) {
    const ssize_t w = ::write(fd, src + put, size_t(std::min<int64_t>(len - put, int64_t(1) << 30)));
    if (w < 0) {
      if (errno == EINTR) continue;
      io_fail("write failed:", path, errno);
    }
    put += w;
  }
}

void fsync_dir_of(const std::string& path) {
  const size_t s = path.find_last_of('/');
  const std::string dir = s == std::string::npos ? "." : (s == 0 ? "/" : path.substr(0, s));
  const int fd = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
  if (fd < 0) return;  // (a directory we cannot open cannot be synced; the rename itself succeeded)
  ::fsync(fd);
  ::close(fd);
}

}  // namespace

void commit_file(const std::string& path, const std::vector<Piece>& pieces, bool durable) {
  const std::string tmp = path + ".gfrs-tmp";
  const int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) io_fail("cannot create", tmp, errno);
  try {
    for (const Piece& pc : pieces) write_all_fd(fd, pc.data, pc.len, tmp);
    if (durable && ::fsync(fd) != 0) io_fail("fsync failed:", tmp, errno);
  } catch (...) {
    ::close(fd);
    ::unlink(tmp.c_str());
    throw;
  }
  if (::close(fd) != 0) {
    const int err = errno;
    ::unlink(tmp.c_str());
    io_fail("close failed:", tmp, err);
  }
  if (std::rename(tmp.c_str(), path.c_str()) != 0) {
    const int err = errno;
    ::unlink(tmp.c_str());
    io_fail("cannot rename onto", path, err);
  }
  if (durable) fsync_dir_of(path);
}

void commit_file(const std::string& path, const uint8_t* data, int64_t len, bool durable) {
  commit_file(path, std::vector<Piece>{{data, len}}, durable);
}

void remove_file(const std::string& path, bool durable) {
  if (::unlink(path.c_str()) != 0) {
    if (errno == ENOENT) return;
    io_fail("cannot remove", path, errno);
  }
  if (durable) fsync_dir_of(path);
}

void write_metadata(const std::string& path, int64_t total_size, int p, int k, const Mat& e, bool with_matrix,
                    const std::vector<uint32_t>& crc) {
  std::ostringstream o;
  o << static_cast<long long>(total_size) << '\n' << p << ' ' << k << '\n';
  if (with_matrix) {
    matrix_lines(o, p, k, std::vector<int>(e.begin(), e.end()));
    crc_line(o, crc);
  }
  const std::string s = o.str();
  commit_file(path, reinterpret_cast<const uint8_t*>(s.data()), int64_t(s.size()));
}

void write_metadata16(const std::string& path, int64_t total_size, int p, int k, const gf16w::Mat& e,
                      const std::vector<uint32_t>& crc) {
  std::ostringstream o;
  o << "GFRS-METADATA " << kMetadataVersion << " 16\n" << static_cast<long long>(total_size) << '\n' << p << ' ' << k
    << '\n';
  matrix_lines(o, p, k, std::vector<int>(e.begin(), e.end()));
  crc_line(o, crc);
  const std::string s = o.str();
  commit_file(path, reinterpret_cast<const uint8_t*>(s.data()), int64_t(s.size()));
}

namespace {

// The optional crc32 line after the matrix rows.
void read_crc(std::istream& in, Metadata& md) {
  std::string tag;
  if (in >> tag && tag == "crc32") {
    std::string h;
    for (int i = 0; i < md.k + md.p && (in >> h); ++i) md.crc.push_back(uint32_t(std::stoul(h, nullptr, 16)));
    if (int(md.crc.size()) != md.k + md.p) md.crc.clear();
  }
}

Metadata read_metadata16(std::istream& in, const std::string& path) {
  Metadata md;
  md.w = 16;
  long long total = 0;
  if (!(in >> total >> md.p >> md.k)) throw std::runtime_error("malformed metadata " + path);
  if (md.k <= 0 || md.p < 0 || md.k + md.p > int(gf16w::kMax) || total < 0)
    throw std::runtime_error("metadata out of range in " + path);
  md.total_size = total;
  const size_t n = size_t(md.k + md.p) * md.k;
  md.g16.resize(n);
  long v;
  for (size_t got = 0; got < n; ++got) {
    if (!(in >> v)) throw std::runtime_error("truncated metadata matrix in " + path);
    if (v < 0 || v > 65535) throw std::runtime_error("metadata matrix entry out of range in " + path);
    md.g16[got] = uint16_t(v);
  }
  md.has_matrix = true;
  read_crc(in, md);
  return md;
}

}  // namespace

Metadata read_metadata(const std::string& path) {
  std::ifstream in(path);
  if (!in) throw std::runtime_error("cannot open metadata file " + path);
  std::string first;
  if (!(in >> first)) throw std::runtime_error("malformed metadata " + path);
  if (first == "GFRS-METADATA") {  // versioned form (GF(2^16))
    int version = 0, w = 0;
    if (!(in >> version >> w) || version != kMetadataVersion || w != 16)
      throw std::runtime_error("unsupported metadata version/field in " + path + " (this build reads version " +
                               std::to_string(kMetadataVersion) + ", field width 16)");
    return read_metadata16(in, path);
  }
  Metadata md;
  char* end = nullptr;
  const long long total = std::strtoll(first.c_str(), &end, 10);
  if (end == first.c_str() || *end || !(in >> md.p >> md.k)) throw std::runtime_error("malformed metadata " + path);
  if (md.k <= 0 || md.p < 0 || md.k + md.p > 256 || total < 0)
    throw std::runtime_error("metadata out of range in " + path);
  md.total_size = total;
  const size_t n = size_t(md.k + md.p) * md.k;
  md.g.resize(n);
  size_t got = 0;
  int v;
  while (got < n && (in >> v)) {
    if (v < 0 || v > 255) throw std::runtime_error("metadata matrix entry out of range in " + path);
    md.g[got++] = uint8_t(v);
  }
  if (got == n) {
    md.has_matrix = true;
    read_crc(in, md);
  } else if (got == 0) {
    md.g = generator(vandermonde_ref(md.k, md.p), md.k, md.p);  // CPU-format metadata
    md.has_matrix = false;
  } else {
    throw std::runtime_error("truncated metadata matrix in " + path);
  }
  return md;
}

std::vector<std::string> read_conf(const std::string& path) {
  std::ifstream in(path);
  if (!in) throw std::runtime_error("cannot open configuration file " + path);
  std::vector<std::string> names;
  std::string s;
  while (in >> s) names.push_back(s);
  return names;
}

void write_conf(const std::string& path, const std::vector<std::string>& names) {
  std::string s;
  for (const auto& n : names) s += n + "\n";
  commit_file(path, reinterpret_cast<const uint8_t*>(s.data()), int64_t(s.size()), false);
}

int64_t file_size(const std::string& path) {
  struct stat sb;
  if (::stat(path.c_str(), &sb) != 0) throw std::runtime_error("cannot stat " + path);
  return int64_t(sb.st_size);
}

void read_into(const std::string& path, int64_t offset, uint8_t* dst, int64_t len) {
  FILE* fp = std::fopen(path.c_str(), "rb");
  if (!fp) throw std::runtime_error("cannot open input file " + path);
  int64_t got = 0;
  if (fseeko(fp, offset, SEEK_SET) == 0) {
    while (got < len) {
      const size_t r = std::fread(dst + got, 1, size_t(len - got), fp);
      if (r == 0) break;
      got += int64_t(r);
    }
  }
  std::fclose(fp);
  if (got < len) std::memset(dst + got, 0, size_t(len - got));
}

void write_from(const std::string& path, const uint8_t* src, int64_t len, bool durable) {
  const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) io_fail("cannot open output file", path, errno);
  try {
    write_all_fd(fd, src, len, path);
    if (durable && ::fdatasync(fd) != 0) io_fail("fdatasync failed:", path, errno);
  } catch (...) {
    ::close(fd);
    throw;
  }
  // (a deferred write error, e.g. ENOSPC on an NFS flush, surfaces at close)
  if (::close(fd) != 0) io_fail("close failed:", path, errno);
}

std::string resolve_chunk(const std::string& name, const std::string& anchor) {
  if (exists(name) || name.empty() || name[0] == '/') return name;
  std::string dir, base;
  split_path(anchor, dir, base);
  const std::string alt = dir + name;
  return exists(alt) ? alt : name;
}

}  // namespace gfrs

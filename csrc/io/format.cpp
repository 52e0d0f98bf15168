// File formats (see gfrs/format.h). 64-bit sizes throughout; tails zero-padded (the reference's GPU
// encoder leaves padding uninitialised, src/encode.cu:325).
#include "gfrs/format.h"

#include <sys/stat.h>

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

uint32_t crc32(const uint8_t* data, int64_t len, uint32_t crc) {
  // slicing-by-8 CRC-32 (IEEE 802.3, reflected 0xEDB88320)
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
  crc = ~crc;
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
  return ~crc;
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

void write_metadata(const std::string& path, int64_t total_size, int p, int k, const Mat& e, bool with_matrix,
                    const std::vector<uint32_t>& crc) {
  FILE* fp = std::fopen(path.c_str(), "wb");
  if (!fp) throw std::runtime_error("cannot open metadata file " + path);
  std::fprintf(fp, "%lld\n%d %d\n", static_cast<long long>(total_size), p, k);
  if (with_matrix) {
    for (int i = 0; i < k; ++i) {
      for (int j = 0; j < k; ++j) std::fprintf(fp, "%d ", i == j ? 1 : 0);
      std::fprintf(fp, "\n");
    }
    for (int i = 0; i < p; ++i) {
      for (int j = 0; j < k; ++j) std::fprintf(fp, "%d ", int(e[size_t(i) * k + j]));
      std::fprintf(fp, "\n");
    }
    if (!crc.empty()) {
      std::fprintf(fp, "crc32");
      for (uint32_t c : crc) std::fprintf(fp, " %08x", c);
      std::fprintf(fp, "\n");
    }
  }
  std::fclose(fp);
}

void write_metadata16(const std::string& path, int64_t total_size, int p, int k, const gf16w::Mat& e,
                      const std::vector<uint32_t>& crc) {
  FILE* fp = std::fopen(path.c_str(), "wb");
  if (!fp) throw std::runtime_error("cannot open metadata file " + path);
  std::fprintf(fp, "GFRS-METADATA %d 16\n%lld\n%d %d\n", kMetadataVersion, static_cast<long long>(total_size), p, k);
  for (int i = 0; i < k; ++i) {
    for (int j = 0; j < k; ++j) std::fprintf(fp, "%d ", i == j ? 1 : 0);
    std::fprintf(fp, "\n");
  }
  for (int i = 0; i < p; ++i) {
    for (int j = 0; j < k; ++j) std::fprintf(fp, "%d ", int(e[size_t(i) * k + j]));
    std::fprintf(fp, "\n");
  }
  if (!crc.empty()) {
    std::fprintf(fp, "crc32");
    for (uint32_t c : crc) std::fprintf(fp, " %08x", c);
    std::fprintf(fp, "\n");
  }
  std::fclose(fp);
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
  std::ofstream out(path);
  if (!out) throw std::runtime_error("cannot write configuration file " + path);
  for (const auto& n : names) out << n << "\n";
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

void write_from(const std::string& path, const uint8_t* src, int64_t len) {
  FILE* fp = std::fopen(path.c_str(), "wb");
  if (!fp) throw std::runtime_error("cannot open output file " + path);
  int64_t put = 0;
  while (put < len) {
    const size_t w = std::fwrite(src + put, 1, size_t(len - put), fp);
    if (w == 0) break;
    put += int64_t(w);
  }
  std::fclose(fp);
  if (put < len) throw std::runtime_error("short write to " + path);
}

std::string resolve_chunk(const std::string& name, const std::string& anchor) {
  if (exists(name) || name.empty() || name[0] == '/') return name;
  std::string dir, base;
  split_path(anchor, dir, base);
  const std::string alt = dir + name;
  return exists(alt) ? alt : name;
}

}  // namespace gfrs

// On-disk formats shared with the reference:
//   * chunk files  "_<i>_<name>" next to the input file, natives 0..k-1 then parity k..n-1
//     (src/encode.cu:434-465). Unlike the reference, a path with directories works: the chunk
//     lands in the file's directory.
//   * "<file>.METADATA" text: totalSize \n p k \n then, in the GPU format, the k+p rows of
//     G = [I; E] as "%d " values (src/encode.cu:61-101). The CPU reference writes only the first
//     two lines (src/cpu-rs.c:465-476); read_metadata() accepts both and regenerates G from the
//     reference Vandermonde for the short form.
//   * decode config: whitespace-separated k chunk names; row index = atoi(basename + 1)
//     (src/decode.cu:302-318). Conf order defines the row order of the decode system.
//   * GF(2^16) stripes (an extension: the reference's w = 16 code, src/galoisfield.cu:22-32, was
//     never built, so it defined no file layout) carry an explicit format version as an extra first
//     line, "GFRS-METADATA 2 16" (format version, field width), then the same lines with 16-bit
//     matrix values. Chunks hold little-endian 16-bit symbols; C is rounded up to an even byte
//     count. GF(2^8) METADATA stays exactly the reference's (no version line), so every file the
//     reference can read is still written the reference's way.
#pragma once

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <string>
#include <thread>
#include <vector>

#include "gfrs/gf65536.h"
#include "gfrs/matrix.h"

namespace gfrs {

constexpr int kMetadataVersion = 2;  // the versioned (GF(2^16)) form; unversioned = the reference's

struct Metadata {
  int64_t total_size = 0;
  int p = 0, k = 0;
  int w = 8;                // field width: 8 (reference format) or 16 (versioned format)
  Mat g;                    // (k+p) x k generator (w = 8)
  gf16w::Mat g16;           // (k+p) x k generator (w = 16)
  bool has_matrix = false;  // false: 2-line CPU format, g regenerated (reference Vandermonde)
  std::vector<uint32_t> crc;  // optional per-chunk CRC-32 (n entries) — extension, see below
};

// Extension (failure detection): after the matrix rows the GPU-format METADATA may
// carry a line "crc32 <c_0> ... <c_{n-1}>" (hex). The reference's reader stops after the matrix
// (src/decode.cu:272-281) and ignores it, so files stay readable by the reference.
uint32_t crc32(const uint8_t* data, int64_t len, uint32_t crc = 0);
// CRC-32 of A || B from crc32(A), crc32(B) and len(B): advances crc(A) over len(B) zero bytes (a
// 32 x 32 GF(2) operator raised to 8 len(B) by repeated squaring). Column shards of a chunk, each
// CRC'd by its own rank, combine into the chunk's METADATA CRC this way (multi-GPU file codec).
uint32_t crc32_combine(uint32_t crc_a, uint32_t crc_b, int64_t len_b);

// fn(i) for every i in [0, n) on up to max_threads threads, each taking the next index in turn
// (the decode's survivor check: k chunk files read and CRC-checked at once). fn must not throw.
template <typename F>
void parallel_indices(int n, int max_threads, F&& fn) {
  const int nt = std::max(1, std::min(n, max_threads));
  if (nt <= 1) {
    for (int i = 0; i < n; ++i) fn(i);
    return;
  }
  std::atomic<int> next{0};
  std::vector<std::thread> th;
  th.reserve(size_t(nt));
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&] {
      for (int i = next.fetch_add(1); i < n; i = next.fetch_add(1)) fn(i);
    });
  for (auto& x : th) x.join();
}
// threads for the survivor check (GFRS_VERIFY_THREADS, default 16; 1 = serial)
int verify_threads();

std::string chunk_path(const std::string& file, int index);
std::string metadata_path(const std::string& file);
int chunk_index(const std::string& name);  // atoi(basename + 1); -1 if malformed

// Durable commit of a small file: written to "<path>.gfrs-tmp", checked at every write and at
// close, fsync'ed, renamed over `path`, and the directory fsync'ed (durable = true). A failure
// (ENOSPC, EFBIG, EIO) throws and leaves `path` as it was — never a partial file. METADATA is always
// written this way: a stripe whose METADATA exists was completely written before it
// (the reference fopen/fprintf's it in place, src/encode.cu:61-101).
void commit_file(const std::string& path, const uint8_t* data, int64_t len, bool durable = true);
// the same for a file made of consecutive pieces (a decoded file: k rows, the last one cut)
struct Piece {
  const uint8_t* data;
  int64_t len;
};
void commit_file(const std::string& path, const std::vector<Piece>& pieces, bool durable = true);
// unlink (missing is fine) and, durable, fsync the directory: an encode removes an older METADATA
// before its first chunk byte so a crash mid-way cannot leave a METADATA describing other chunks
void remove_file(const std::string& path, bool durable = true);

void write_metadata(const std::string& path, int64_t total_size, int p, int k, const Mat& e, bool with_matrix = true,
                    const std::vector<uint32_t>& crc = {});
// GF(2^16): the versioned form (always with the matrix).
void write_metadata16(const std::string& path, int64_t total_size, int p, int k, const gf16w::Mat& e,
                      const std::vector<uint32_t>& crc = {});
Metadata read_metadata(const std::string& path);
std::vector<std::string> read_conf(const std::string& path);
void write_conf(const std::string& path, const std::vector<std::string>& names);

// Chunk geometry: C = ceil(total / k) (src/encode.cu:317); GF(2^16) rounds up to whole symbols.
inline int64_t chunk_size(int64_t total, int k) { return (total + k - 1) / k; }
inline int64_t chunk_size(int64_t total, int k, int field_w) {
  const int64_t c = chunk_size(total, k);
  return field_w == 16 ? (c + 1) / 2 * 2 : c;
}

int64_t file_size(const std::string& path);
// Reads up to `len` bytes at `offset` into dst; zero-fills what the file does not cover.
void read_into(const std::string& path, int64_t offset, uint8_t* dst, int64_t len);
// Writes `len` bytes to `path` (created / truncated); every write and the close are checked and
// throw with errno's text (ENOSPC, EFBIG), durable: fdatasync'ed before the close.
void write_from(const std::string& path, const uint8_t* src, int64_t len, bool durable = false);
// Resolve a chunk name from a conf: as given (relative to the CWD, like the reference), else
// relative to the directory of `anchor`.
std::string resolve_chunk(const std::string& name, const std::string& anchor);

}  // namespace gfrs

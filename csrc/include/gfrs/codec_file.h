// File-level encode/decode shared by the GPU CLI (bin/RS), the CPU CLI (bin/CPU-RS) and the Python
// bindings. The arithmetic backend is a callback, so the same code drives the gfx950 streaming
// pipeline and the CPU reference codec. Mirrors encode_file/decode_file of the reference
// (src/encode.cu:301-473, src/decode.cu:236-434; call stacks in SURVEY §3.1-3.2) with its defects
// fixed: zero-padded tails, 64-bit sizes, singular-pattern detection, row-pivoted inversion,
// survivor rows passed through instead of re-multiplied by the identity.
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "gfrs/format.h"
#include "gfrs/matrix.h"

namespace gfrs {

// coeff: m x k coefficients of field width `field_w` — 8 (GF(2^8), one byte each) or 16 (GF(2^16),
// little-endian byte pairs, gfrs/host_desc.h pack16; ncols is then an even byte count).
using GemmFn = std::function<void(const std::vector<const uint8_t*>& in, const std::vector<uint8_t*>& out,
                                  const Mat& coeff, int64_t ncols, int field_w)>;

struct HostAlloc {
  std::function<uint8_t*(size_t)> alloc;  // e.g. pinned hipHostMalloc for the GPU path
  std::function<void(uint8_t*)> release;
};
HostAlloc default_host_alloc();

struct FileReport {
  int64_t total_size = 0, chunk_size = 0;
  int k = 0, p = 0, erased = 0;
  int rejected = 0;  // chunks skipped because their CRC-32 did not match METADATA
  double ms_alloc = 0;  // host buffer allocation (pinned hipHostMalloc on the GPU path), all buffers
  double ms_read = 0, ms_matrix = 0, ms_compute = 0, ms_write = 0;
};

// Writes _0_<file> .. _{n-1}_<file> and <file>.METADATA (full matrix format unless `cpu_meta`).
// field_w = 16: GF(2^16) symbols (n <= 65535, even chunk size, versioned METADATA — gfrs/format.h).
FileReport encode_file(const std::string& file, int k, int p, MatrixKind kind, const GemmFn& gemm,
                       const HostAlloc& alloc, bool cpu_meta = false, int field_w = 8);

// Reads <file>.METADATA and the k chunks named in `conf`, writes `out` (or overwrites `file` when
// `out` is empty, like the reference, src/decode.cu:410-425). Throws std::runtime_error for an
// unrecoverable (singular) erasure pattern. The field comes from the METADATA.
FileReport decode_file(const std::string& file, const std::string& conf, const std::string& out,
                       const GemmFn& gemm, const HostAlloc& alloc);

// GF(2^16) coding block of `kind` (reference Vandermonde, Cauchy, systematic Vandermonde).
gf16w::Mat encoding_matrix16(MatrixKind kind, int k, int p);

// Decode coefficients in the METADATA's field: rows `erased` of inv(G[rows]) packed as GemmFn
// coefficients (GF(2^16): the e x e systematic solve). With erased == nullptr only checks that the
// pattern is recoverable. False when G[rows] is singular.
bool decode_coefficients(const Metadata& md, const std::vector<int>& rows, const std::vector<int>* erased, Mat* coeff);

// The reference's src/unit-test.sh: conf keeping the LAST k chunks (erases natives 0..n-k-1).
std::vector<std::string> worst_case_conf(const std::string& file, int n, int k);

}  // namespace gfrs

// CPU reference codec: the test oracle and the BASELINE config #1 path (runs without a GPU).
//
// The reference ships nine single-threaded CPU programs that differ only in how they multiply in
// GF(2^8). They are one selectable strategy here, bit-identical by construction
// (the bugs that made some variants wrong — uninitialised accumulators in cpu-rs-loop.c:51-64 and
// cpu-rs-full.c:55-68, the bit-7 test in cpu-rs-double.c:139 — are not reproduced):
//   kLogExp        cpu-rs.c           log/exp, conditional subtract (src/cpu-rs.c:106-120)
//   kLogExpMod     cpu-rs-log-exp-0.c (log a + log b) % 255
//   kLogExpFold    cpu-rs-log-exp-1.c (s & 255) + (s >> 8), exp[255] = exp[0]
//   kLogExpDouble  cpu-rs-log-exp-2.c doubled 509-entry exp table, no modulo
//   kZeroBand      cpu-rs-log-exp-3.c 1021-entry table, log(0) = 510, branch-free (the GPU scheme
//                                     of src/matrix.cu:34-39)
//   kLoop          cpu-rs-loop.c      shift-and-xor
//   kFull          cpu-rs-full.c      64 KiB gfmul[256][256] table
//   kNibble        cpu-rs-double.c    L[a>>4][b] ^ R[a&15][b] nibble-split tables
//   kPerm          (new)              host emulation of the gfx950 v_perm 3-chunk tables
//   kRow           (new)              one 256-byte product row per coefficient, multi-threaded
//   kSimd          (new, default)     cpu-rs-double.c's nibble split, vectorised: the two 16-entry
//                                     tables of a coefficient in one register each, 32 bytes per
//                                     pshufb pair (AVX2; kRow where the host lacks it)
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "gfrs/gf65536.h"
#include "gfrs/matrix.h"

namespace gfrs {

enum class CpuMul : int {
  kLogExp = 0,
  kLogExpMod,
  kLogExpFold,
  kLogExpDouble,
  kZeroBand,
  kLoop,
  kFull,
  kNibble,
  kPerm,
  kRow,
  kSimd,
};

CpuMul parse_cpu_mul(const std::string& s);
const char* cpu_mul_name(CpuMul m);

// out_rows[i][c] = XOR_j coeff[i][j] * in_rows[j][c], c in [0, ncols). threads <= 0: hardware.
void cpu_gemm(const std::vector<const uint8_t*>& in_rows, const std::vector<uint8_t*>& out_rows, const Mat& coeff,
              int64_t ncols, CpuMul strategy = CpuMul::kSimd, int threads = 1);

// GF(2^16) (gfrs/gf65536.h): out_rows[i][s] = XOR_j coeff[i][j] * in_rows[j][s] over little-endian
// 16-bit symbols; ncols is a byte count (even). Two 256-entry product tables per coefficient (low
// and high source byte), columns split over `threads` (<= 0: hardware).
void cpu_gemm16(const std::vector<const uint8_t*>& in_rows, const std::vector<uint8_t*>& out_rows,
                const gf16w::Mat& coeff, int64_t ncols, int threads = 1);

// Scalar multiply through a given strategy (exposed for the per-strategy unit tests).
uint8_t cpu_mul(CpuMul strategy, uint8_t a, uint8_t b);

}  // namespace gfrs

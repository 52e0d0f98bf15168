// Launch entry points of the gfx950 HIP kernels (csrc/kernels/*.hip). Every launcher is
// asynchronous on `stream`, performs no allocation and no host synchronisation, so callers may
// capture it into a hipGraph (cdna_hip_programming.md Guideline 9).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace gfrs {

// ---- GF-GEMM (csrc/kernels/gf_gemm.hip) -------------------------------------------------------
// desc: device descriptor (gfrs/desc.h) for k inputs and m_pad outputs. Processes byte columns
// [col0, col0 + ncols). Uses the 16-byte v_perm kernel for the aligned body and a byte kernel for
// the ragged tail; `force_bytewise` routes everything through the byte kernel (unaligned rows).
// max_blocks caps grid.x (the reference's -p gridDim knob, src/main.c:74-77); 0 = uncapped.
// copies = false promises the descriptor has no fused-copy rows (an encode): k = 10 with 4-row
// output tiles then runs the rows-in-flight kernel (all k loads issued before the first multiply).
hipError_t launch_gf_gemm(const void* desc, int k, int m_pad, int64_t col0, int64_t ncols,
                          bool force_bytewise, int max_blocks, hipStream_t stream, bool copies = true);

// GF(2^16) form (csrc/kernels/gf_gemm16.hip): desc built with desc_layout16 (build_desc field_w =
// 16); rows hold little-endian 16-bit symbols, col0 and ncols are even byte counts. `symwise`
// routes every column through the one-symbol-per-lane kernel (rows not 16-byte aligned).
// one_tile: keep every output in one tile whatever the row length (the zero-copy pipeline, whose
// inputs cross PCIe once per tile; short rows otherwise run one output per tile).
hipError_t launch_gf_gemm16(const void* desc, int k, int m_pad, int64_t col0, int64_t ncols, bool symwise,
                            int max_blocks, hipStream_t stream, bool one_tile = false);
// batched: `batch` stripes (grid.y), desc built with desc_layout16(k, m_pad, batch)
hipError_t launch_gf_gemm16_batched(const void* desc, int k, int m_pad, int batch, int64_t col0, int64_t ncols,
                                    bool symwise, int max_blocks, hipStream_t stream, bool one_tile = false);

// Batched form: `batch` stripes of identical shape share the coefficient tables (small-object
// serving: one launch for many objects). desc built with desc_layout(k, m_pad, batch).
// copies = false promises no fused-copy rows (a batched encode: the rows-in-flight kernel may run).
hipError_t launch_gf_gemm_batched(const void* desc, int k, int m_pad, int batch, int64_t col0, int64_t ncols,
                                  bool force_bytewise, hipStream_t stream, bool copies = true);

// Variant selector for benchmarks/ablation: vec = 16-byte groups per lane (0 = byte kernel, -1 = the
// byte kernel's serial round-3 form),
// pf = input rows kept in flight per lane, nt = non-temporal loads/stores.
hipError_t launch_gf_gemm_variant(const void* desc, int k, int m_pad, int64_t col0, int64_t ncols,
                                  int vec, int pf, bool nt, int max_blocks, hipStream_t stream);

// LDS-LUT ablation (gf_gemm_lut.hip): the same GEMM with per-coefficient 4-bit nibble tables in LDS
// (two ds_read_u8 per byte product), built from the descriptor's tables; 16-byte aligned columns,
// the < 16-byte tail on the byte kernel.
hipError_t launch_gf_gemm_lut(const void* desc, int k, int m_pad, int64_t col0, int64_t ncols, hipStream_t stream);

// ---- Gauss-Jordan inverse (csrc/kernels/gf_invert.hip) ---------------------------------------
// Inverts `batch` n x n matrices (row-major, contiguous) with row pivoting, one workgroup each,
// [A|I] resident in LDS. status[b] = 0 ok, 1 singular. n <= 256.
// If `desc` is non-null, additionally writes the perm tables of rows `sel_rows[0..m)` of each
// inverse into desc's table block (k = n, m_pad given) — the decode GEMM then runs without a
// host round-trip. (batch must be 1 in that mode.)
// Systematic decode rows without the k x k inverse: g = G (n x k, [I; E]), rows = the k survivor
// ids, erased = the e erased native ids (device int32). Writes X (e x k, decode coefficients of the
// erased natives in survivor order) to dm (optional), status (1 = unrecoverable), and the v_perm
// tables tab[j][b] into desc (k inputs, m_pad >= e outputs) when given.
// Device-built plan (ptrs != null, desc required): `erased` becomes an OUTPUT (derived from rows on
// the device) and the descriptor's row pointers are written from ptrs = {chunk row 0..n_chunks-1,
// output row 0..k-1} (uint64 device addresses); status 2 = invalid pattern.
hipError_t launch_gf_decode_system(const uint8_t* g, int k, const int* rows, int* erased, int e, uint8_t* dm,
                                   int* status, void* desc, int m_pad, hipStream_t stream,
                                   const uint64_t* ptrs = nullptr, int n_chunks = 0);
hipError_t launch_gf_invert(const uint8_t* a, uint8_t* a_inv, int n, int batch, int* status,
                            void* desc, const int* sel_rows, int m, int m_pad, hipStream_t stream);

// GF(2^16) form (csrc/kernels/gf_decode16.hip): g = G (n x k little-endian uint16, [I; E]), rows =
// the k survivor ids (device int32). `erased` (device int32 [e]) is always an OUTPUT: the erased
// natives, ascending, derived from rows. Writes X (e x k uint16) to dm (optional), status (0 ok,
// 1 singular, 2 invalid survivor list) and, into a desc_layout16 descriptor (k inputs, m_pad >= e
// outputs), the four v_perm records per coefficient; with ptrs = {chunk row 0..n-1, output row
// 0..k-1} also the descriptor's row pointers. Systems that fit one workgroup's LDS
// (decode_system16_supported: e <= 256, ~ 8 e (e + k) + 4 n + 4 k bytes) are solved there in one
// launch; larger ones (e.g. k = 2000, e = 100, or any e > 256) by the blocked multi-workgroup solve
// (panels of pivot columns, row pivoting, rank-P updates over the chip), which needs a device
// `workspace` of decode_system16_workspace(n, k, e) bytes (-1: too large even for it: e past
// ~19 K). force_blocked takes the blocked solve for any size (tests).
bool decode_system16_supported(int n, int k, int e);
int64_t decode_system16_workspace(int n, int k, int e);
hipError_t launch_gf_decode_system16(const uint16_t* g, int n, int k, const int* rows, int* erased, int e,
                                     uint16_t* dm, int* status, void* desc, int m_pad, hipStream_t stream,
                                     const uint64_t* ptrs = nullptr, void* workspace = nullptr,
                                     bool force_blocked = false);

// ---- matrix utilities (csrc/kernels/gf_matrix.hip) -------------------------------------------
// kind: 0 = reference Vandermonde, 1 = Cauchy. Writes the p x k block.
hipError_t launch_gen_matrix(uint8_t* e, int k, int p, int kind, hipStream_t stream);
// Build perm tables [k][m_pad] for an m x k coefficient matrix into desc's table block.
hipError_t launch_perm_tables(const uint8_t* coeff, int m, int k, void* desc, int m_pad,
                              hipStream_t stream);
// Deterministic counter-based random bytes (synthetic benchmark input), 16 B per lane stores.
hipError_t launch_fill_random(uint8_t* dst, int64_t bytes, uint64_t seed, hipStream_t stream);
// Gather an m x k sub-matrix: out[i][:] = g[rows[i]][:]  (decode system assembly on device).
hipError_t launch_gather_rows(const uint8_t* g, const int* rows, uint8_t* out, int m, int k,
                              hipStream_t stream);

// ---- int8-MFMA bit-matrix GF-GEMM (csrc/kernels/gf_mfma.hip) ----------------------------------
// Same contract as launch_gf_gemm but on matrix cores; requires k % 4 == 0 (see kernel notes).
hipError_t launch_gf_gemm_mfma(const void* bitmat, const void* desc, int k, int m, int64_t col0,
                               int64_t ncols, hipStream_t stream);
size_t mfma_bitmat_bytes(int k, int m);

// ---- FP4 (e2m1) block-scaled MFMA bit-matrix GF-GEMM (csrc/kernels/gf_mfma_fp4.hip) ------------
// Rows must be 2-byte aligned; whole 256-column chunks run on the matrix cores, the remainder on
// the v_perm kernel (desc must carry the perm tables too).
// mg_cap bounds the M-tiles (4 output rows each) one block keeps in LDS/accumulators; the bitmat
// must be built with the same cap. in_stride != 0 promises input row j == input row 0 + j*in_stride
// (rows of one allocation): DMA addresses are then computed instead of read from a pointer table.
// copies: also write input row j to the descriptor's copy[j] (fused survivor copy of decode).
hipError_t launch_gf_gemm_fp4(const void* bitmat, const void* desc, int k, int m, int64_t col0,
                              int64_t ncols, int mg_cap, int64_t in_stride, bool copies, hipStream_t stream);
size_t fp4_bitmat_bytes(int k, int m, int mg_cap);
// the form launch_gf_gemm_fp4 runs for (k, m, copies): "v1", "ar" or "tm" (fp4_route,
// gf_mfma_fp4.hip, documents each choice with its measurement)
const char* fp4_route_name(int k, int m, bool copies, int mg_cap);
// Batched form (small-object serving): `batch` stripes of identical shape whose rows sit at fixed
// strides — stripe b's input rows are stripe 0's + b * in_bstride, its output and copy rows stripe
// 0's + b * out_bstride (desc built with desc_layout(k, m_pad, batch); the kernel reads stripe 0's
// tables). ncols per stripe; whole chunks of every stripe run in ONE persistent matrix-core launch
// (A loaded once per wave for the whole batch), the ragged remainders on the batched v_perm kernel.
// hipErrorNotSupported when the shape has no batched matrix-core form (currently the A-resident
// kernel: k in (112, 128], one M-tile group), so the caller keeps the v_perm path.
hipError_t launch_gf_gemm_fp4_batched(const void* bitmat, const void* desc, int k, int m, int batch, int64_t col0,
                                      int64_t ncols, int mg_cap, int64_t in_stride, int64_t in_bstride,
                                      int64_t out_bstride, bool copies, hipStream_t stream);
hipError_t launch_fp4_bitmat(const uint8_t* coeff, int m, int k, void* bitmat, int mg_cap, hipStream_t stream);
// row o of the coefficient matrix = coeff + sel[o] * ld (device pointers; e.g. erased rows of a
// device-computed inverse, so a decode needs no host round trip)
hipError_t launch_fp4_bitmat_sel(const uint8_t* coeff, int ld, const int* sel, int m, int k, void* bitmat, int mg_cap,
                                 hipStream_t stream);
hipError_t launch_mfma_bitmat(const uint8_t* coeff, int m, int k, void* bitmat,
                              hipStream_t stream);

// ---- GF(2^16) on the FP4 matrix cores (csrc/kernels/gf_mfma16.hip) -----------------------------
// desc: a desc_layout16 descriptor (its v_perm records run the columns past the last 512-byte chunk
// and any start not 4-byte aligned); bitmat from launch_fp16_bitmat with the same (k, m, mg_cap).
// Rows 4-byte aligned; col0 / ncols even. K is split into passes (one launch each, later passes XOR
// into the outputs); copies: fused survivor copy (decode), in_stride as launch_gf_gemm_fp4.
hipError_t launch_gf_gemm16_fp4(const void* bitmat, const void* desc, int k, int m, int64_t col0, int64_t ncols,
                                int mg_cap, int64_t in_stride, bool copies, hipStream_t stream);
// Batched: `batch` stripes whose rows are stripe 0's plus b * in_bstride (inputs) / b * out_bstride
// (outputs, copies), desc built with desc_layout16(k, m_pad, batch). Every stripe's whole chunks run
// in one persistent launch per K pass; the ragged remainders on the batched v_perm kernel.
hipError_t launch_gf_gemm16_fp4_batched(const void* bitmat, const void* desc, int k, int m, int batch, int64_t col0,
                                        int64_t ncols, int mg_cap, int64_t in_stride, int64_t in_bstride,
                                        int64_t out_bstride, bool copies, hipStream_t stream);
size_t fp16_bitmat_bytes(int k, int m, int mg_cap);
// coefficient (o, i) = coeff[row(o) * ld + i] (uint16, device), row(o) = sel ? sel[o] : o
hipError_t launch_fp16_bitmat(const uint16_t* coeff, int ld, const int* sel, int m, int k, void* bitmat, int mg_cap,
                              hipStream_t stream);

// FP4 kernels: the bit-matrix allocation ends with a write-only sink of kFp4SinkSlots 1-KiB slots;
// each wave stores its dummy / destination-less bytes into slot (4 * block + wave) % slots, so the
// sink writes of concurrent waves land on different L2 lines (one shared 1-KiB sink made every CU of
// an XCD queue on the same L2 channel). Nothing reads it.
constexpr int kFp4SinkSlots = 256;

// ---- FP4 A-resident form (csrc/kernels/gf_mfma_fp4ar.hip; called by launch_gf_gemm_fp4) ---------
// k in (112, 128], one bitmat group of mg <= 8 M-tiles (the layout launch_fp4_bitmat builds).
// Processes the leading whole chunks of [col0, col0 + ncols) and reports how many columns in
// *done (the caller finishes the rest).
struct Fp4ArLaunch {
  const uint64_t* in;    // descriptor in_ptr[k]
  const uint64_t* out;   // descriptor out_ptr[m_pad]
  const uint64_t* copy;  // descriptor copy_ptr[k] (nullptr: no fused copy)
  const void* bitmat;
  int k, m, mg;
  int64_t col0, ncols, in_stride;
  // batched launch: `batch` stripes whose rows are stripe 0's (the tables above) plus b * in_bstride
  // (inputs) / b * out_bstride (outputs and copies); ncols is per stripe, *done per stripe
  int batch = 1;
  int64_t in_bstride = 0, out_bstride = 0;
};
bool fp4ar_supported(int k, int mg);
hipError_t launch_gf_gemm_fp4ar(const Fp4ArLaunch& a, int64_t* done, hipStream_t stream);
// Tile-major form (csrc/kernels/gf_mfma_fp4tm.hip): same launch record (batch must be 1), k in
// (112, 128] with one group of 5..8 M-tiles; the chunk's B operand resident
// in AGPRs, tiles in pairs.
bool fp4tm_supported(int k, int mg, bool copies);
hipError_t launch_gf_gemm_fp4tm(const Fp4ArLaunch& a, int64_t* done, hipStream_t stream);

}  // namespace gfrs

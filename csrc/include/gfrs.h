/* gfrs.h — C API of the gfx950 Reed-Solomon codec (libgfrs.so).
 *
 * The reference exports its codec to C as `encode_file` / `decode_file` (src/encode.h:36,
 * src/decode.h:38) and nothing finer. This header keeps those two entry points and adds what an
 * embedding storage service needs: coding matrices, a reusable device GF-GEMM plan (the
 * encode or decode of a stripe already in HBM, one kernel launch per run), a decoder whose erasure
 * pattern lives in device memory, and the pinned-host streaming pipeline. Plain C99; no HIP header
 * needed (streams are passed as `void*` = hipStream_t, NULL = the null stream, and device buffers
 * can be allocated through gfrs_dev_alloc).
 *
 * Every function returning int returns GFRS_OK (0) or a negative GFRS_E* code; the message of the
 * last failure on the calling thread is gfrs_last_error(). Launch functions are asynchronous on
 * their stream, like the kernels under them. Build: `make -C csrc capi` -> lib/libgfrs.so;
 * example: csrc/capi/demo.c.
 */
#ifndef GFRS_H
#define GFRS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GFRS_API_VERSION 3

enum {
  GFRS_OK = 0,
  GFRS_EINVAL = -1,    /* bad argument */
  GFRS_ESINGULAR = -2, /* erasure pattern not recoverable */
  GFRS_EHIP = -3,      /* HIP runtime error */
  GFRS_EIO = -4,       /* file or format error */
  GFRS_EINTERNAL = -5
};

enum { GFRS_MATRIX_VANDERMONDE_REF = 0, GFRS_MATRIX_CAUCHY = 1, GFRS_MATRIX_SYS_VANDERMONDE = 2 };
enum { GFRS_ENGINE_AUTO = 0, GFRS_ENGINE_VALU = 1, GFRS_ENGINE_MFMA = 2 };

int gfrs_api_version(void);
const char* gfrs_last_error(void);
int gfrs_device_count(void);

/* ---- device memory helpers (for callers that do not link HIP themselves) ------------------- */
void* gfrs_dev_alloc(int device, size_t bytes); /* NULL on failure */
void gfrs_dev_free(void* p);
int gfrs_copy(void* dst, const void* src, size_t bytes); /* any direction, synchronous */
int gfrs_sync(int device);

/* ---- coding matrices (host, GF(2^8) poly 0x11D) --------------------------------------------- */
/* e: p x k row-major. kind: GFRS_MATRIX_* (VANDERMONDE_REF = the reference's (j+1)^i matrix). */
int gfrs_encoding_matrix(int kind, int k, int p, uint8_t* e);
/* dm: k x k decode matrix for survivors[0..k) of G = [I_k; E] (E p x k). GFRS_ESINGULAR if the
 * pattern is not recoverable. */
int gfrs_decode_matrix(const uint8_t* e, int k, int p, const int* survivors, uint8_t* dm);

/* ---- device GF-GEMM plan: out[i] = XOR_j coeff[i][j] * in[j] over ncols bytes ---------------- */
typedef struct gfrs_plan gfrs_plan;
/* in: k device rows, out: m device rows, copy: NULL or k device rows (input j is also copied to
 * copy[j] in the same pass when copy[j] != NULL: the fused survivor copy of a decode); coeff: m x k
 * host matrix. Engine AUTO picks the FP4 matrix-core kernel for wide stripes (k >= 64, m >= 16). */
int gfrs_plan_create(gfrs_plan** plan, int device, int k, int m, const uint8_t* coeff, const void* const* in,
                     void* const* out, void* const* copy, int64_t ncols, int engine);
int gfrs_plan_set_coeff(gfrs_plan* plan, const uint8_t* coeff); /* synchronous */
int gfrs_plan_run(gfrs_plan* plan, void* stream);
int gfrs_plan_engine(const gfrs_plan* plan); /* GFRS_ENGINE_VALU or GFRS_ENGINE_MFMA */
void gfrs_plan_destroy(gfrs_plan* plan);

/* ---- GF(2^16) (API version 3): 16-bit little-endian symbols, poly 0x1100B --------------------- */
/* e: p x k row-major uint16 (k + p <= 65535); kind as gfrs_encoding_matrix. */
int gfrs_encoding_matrix16(int kind, int k, int p, uint16_t* e);
/* rows_out: the erased natives' rows of the decode matrix (len(erased) x k) for survivors[0..k) of
 * G = [I_k; E] (the e x e systematic solve, not a k x k inverse). GFRS_ESINGULAR if not recoverable. */
int gfrs_decode_rows16(const uint16_t* e, int k, int p, const int* survivors, const int* erased, int n_erased,
                       uint16_t* rows_out);
/* The GF(2^16) device GEMM plan: out[i] = XOR_j coeff[i][j] * in[j] over ncols bytes (even; rows
 * 2-byte aligned). coeff: m x k host uint16. Engine AUTO picks the FP4 matrix-core kernel (each
 * coefficient's 16 x 16 GF(2) map) for codes from k = 16 and the v_perm kernel for narrower ones;
 * copy as gfrs_plan_create (fused survivor copy). */
typedef struct gfrs_plan16 gfrs_plan16;
int gfrs_plan16_create(gfrs_plan16** plan, int device, int k, int m, const uint16_t* coeff, const void* const* in,
                       void* const* out, void* const* copy, int64_t ncols, int engine);
int gfrs_plan16_run(gfrs_plan16* plan, void* stream);
int gfrs_plan16_engine(const gfrs_plan16* plan); /* GFRS_ENGINE_VALU or GFRS_ENGINE_MFMA */
void gfrs_plan16_destroy(gfrs_plan16* plan);

/* ---- decoder with a device-resident erasure pattern ------------------------------------------ */
/* chunks: the stripe's n = k + p device rows (natives, then parity), out: k device rows, all
 * 16-byte aligned; e: p x k host encoding matrix; erased: natives lost per pattern (1..min(k, p)).
 * gfrs_decoder_rows() is a device int32[k] buffer for the survivor ids (write it with a kernel, a
 * copy or an RCCL broadcast); solve checks the pattern and builds the plan on the device; run
 * rebuilds the erased natives into out and copies the surviving natives in the same pass. */
typedef struct gfrs_decoder gfrs_decoder;
int gfrs_decoder_create(gfrs_decoder** dec, int device, int k, int p, const uint8_t* e, void* const* chunks,
                        void* const* out, int64_t ncols, int erased, int engine);
int* gfrs_decoder_rows(gfrs_decoder* dec);
int gfrs_decoder_solve(gfrs_decoder* dec, const int* rows_dev, void* stream); /* rows_dev NULL: dec's own */
int gfrs_decoder_run(gfrs_decoder* dec, void* stream);
/* synchronises `stream`; returns 0 (plan built), 1 (singular) or 2 (invalid survivor list) */
int gfrs_decoder_status(gfrs_decoder* dec, void* stream);
int gfrs_decoder_engine(const gfrs_decoder* dec); /* GFRS_ENGINE_VALU or GFRS_ENGINE_MFMA */
void gfrs_decoder_destroy(gfrs_decoder* dec);

/* ---- host rows through the streaming pipeline (pinned rows give async DMA) ------------------- */
int gfrs_gemm_host(const int* devices, int ndev, int k, int m, const uint8_t* coeff, const uint8_t* const* in,
                   uint8_t* const* out, int64_t ncols, int streams, int64_t slice_bytes);

/* ---- files: the reference's encode_file / decode_file (same chunk names and METADATA) -------- */
typedef struct {
  int64_t total_size, chunk_size;
  int k, p, erased, rejected;
  double ms_alloc, ms_read, ms_matrix, ms_compute, ms_write;
} gfrs_file_report;
/* devices NULL / ndev 0: device 0. report may be NULL. */
int gfrs_encode_file(const char* file, int k, int p, int matrix_kind, const int* devices, int ndev, int streams,
                     gfrs_file_report* report);
/* out NULL or "": overwrite `file`, as the reference does */
int gfrs_decode_file(const char* file, const char* conf, const char* out, const int* devices, int ndev, int streams,
                     gfrs_file_report* report);

/* Extended forms (API version 2). field_w: 8 (GF(2^8), the reference's field) or 16 (GF(2^16),
 * poly 0x1100B: n <= 65535 chunks, even chunk size, versioned METADATA; decode reads the field from
 * the METADATA). flags: GFRS_FLAG_ZERO_COPY — the GEMM kernel reads and writes the pinned host rows
 * itself over PCIe (no device slice buffers, no copy engines). */
enum { GFRS_FLAG_ZERO_COPY = 1 };
int gfrs_encode_file_ex(const char* file, int k, int p, int matrix_kind, int field_w, unsigned flags,
                        const int* devices, int ndev, int streams, gfrs_file_report* report);
int gfrs_decode_file_ex(const char* file, const char* conf, const char* out, unsigned flags, const int* devices,
                        int ndev, int streams, gfrs_file_report* report);

/* frees the pipeline's persistent per-device workspaces */
int gfrs_release(void);

#ifdef __cplusplus
}
#endif

#endif /* GFRS_H */

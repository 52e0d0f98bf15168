/* The C API (csrc/include/gfrs.h, lib/libgfrs.so) end to end from plain C99, checked against a
 * host GF(2^8) multiply written here:
 *   1. RS(10,14) encode of a device-resident stripe through a plan (v_perm kernel);
 *   2. a decode whose survivor list is written into device memory: the decoder checks it, builds
 *      its plan on the GPU and rebuilds the lost natives while copying the surviving ones (3 of
 *      10 lost; 20 of 128 on the wide stripe, whose decoder then runs on the matrix cores);
 *   3. an invalid survivor list (status 2) and a singular one via gfrs_decode_matrix;
 *   4. a wide stripe, k=128 p=32, on the FP4 matrix-core engine;
 *   5. host rows through the streaming pipeline.
 * Build: make -C csrc capi   (bin/gfrs_capi_demo). Exit 0 = OK, 77 = no GPU visible.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gfrs.h"

static uint8_t gexp[512], glog[256];

static void gf_init(void) {
  int x = 1;
  for (int i = 0; i < 255; ++i) {
    gexp[i] = (uint8_t)x;
    glog[x] = (uint8_t)i;
    x <<= 1;
    if (x & 0x100) x ^= 0x11D;
  }
  for (int i = 255; i < 512; ++i) gexp[i] = gexp[i - 255];
}
static uint8_t gmul(uint8_t a, uint8_t b) { return (a && b) ? gexp[glog[a] + glog[b]] : 0; }

#define CHECK(x)                                                                      \
  do {                                                                                \
    int rc_ = (x);                                                                    \
    if (rc_ != GFRS_OK) {                                                             \
      fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_, gfrs_last_error()); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)
#define EXPECT(c, msg)                          \
  do {                                          \
    if (!(c)) {                                 \
      fprintf(stderr, "FAILED: %s\n", msg);     \
      exit(1);                                  \
    }                                           \
  } while (0)

/* host reference: out[i] = XOR_j coeff[i][j] * in[j] */
static void host_gemm(const uint8_t* coeff, int m, int k, uint8_t** in, uint8_t** out, int64_t C) {
  for (int i = 0; i < m; ++i) {
    memset(out[i], 0, (size_t)C);
    for (int j = 0; j < k; ++j) {
      const uint8_t c = coeff[i * k + j];
      for (int64_t x = 0; x < C; ++x) out[i][x] ^= gmul(c, in[j][x]);
    }
  }
}

static uint8_t** host_rows(int n, int64_t C) {
  uint8_t** r = malloc(sizeof(uint8_t*) * (size_t)n);
  for (int i = 0; i < n; ++i) r[i] = malloc((size_t)C);
  return r;
}
static void** dev_rows(int n, int64_t C) {
  void** r = malloc(sizeof(void*) * (size_t)n);
  for (int i = 0; i < n; ++i) {
    r[i] = gfrs_dev_alloc(0, (size_t)C);
    EXPECT(r[i] != NULL, "gfrs_dev_alloc");
  }
  return r;
}
static void free_rows(void** d, uint8_t** h, int n) {
  for (int i = 0; i < n; ++i) {
    if (d) gfrs_dev_free(d[i]);
    if (h) free(h[i]);
  }
  free(d);
  free(h);
}

static int rows_equal_device(void** dev, uint8_t** want, int n, int64_t C) {
  uint8_t* buf = malloc((size_t)C);
  int ok = 1;
  for (int i = 0; i < n && ok; ++i) {
    CHECK(gfrs_copy(buf, dev[i], (size_t)C));
    ok = memcmp(buf, want[i], (size_t)C) == 0;
  }
  free(buf);
  return ok;
}

static void stripe_round_trip(int k, int p, int64_t C, int expect_engine, int nlost) {
  const int n = k + p;
  uint8_t* e = malloc((size_t)(p * k));
  CHECK(gfrs_encoding_matrix(GFRS_MATRIX_VANDERMONDE_REF, k, p, e));
  uint8_t** data = host_rows(k, C);
  uint8_t** par = host_rows(p, C);
  srand(1234 + k);
  for (int j = 0; j < k; ++j)
    for (int64_t x = 0; x < C; ++x) data[j][x] = (uint8_t)rand();
  host_gemm(e, p, k, data, par, C);

  void** d_chunks = dev_rows(n, C); /* natives then parity */
  void** d_out = dev_rows(k, C);
  for (int j = 0; j < k; ++j) CHECK(gfrs_copy(d_chunks[j], data[j], (size_t)C));

  /* 1. encode through a plan */
  gfrs_plan* enc = NULL;
  CHECK(gfrs_plan_create(&enc, 0, k, p, e, (const void* const*)d_chunks, d_chunks + k, NULL, C, GFRS_ENGINE_AUTO));
  EXPECT(gfrs_plan_engine(enc) == expect_engine, "engine choice");
  CHECK(gfrs_plan_run(enc, NULL));
  CHECK(gfrs_sync(0));
  EXPECT(rows_equal_device(d_chunks + k, par, p, C), "parity mismatch");

  /* 2. device-built decode: lose natives 1, 4, 7 (and the first parity row) with nlost = 3, else
   * natives 0 .. nlost-1 */
  int surv[256], ns = 0;
  for (int r = 0; r < n && ns < k; ++r) {
    int gone = nlost == 3 ? (r == 1 || r == 4 || r == 7 || (p > 3 && r == k)) : r < nlost;
    if (!gone) surv[ns++] = r;
  }
  gfrs_decoder* dec = NULL;
  CHECK(gfrs_decoder_create(&dec, 0, k, p, e, d_chunks, d_out, C, nlost, GFRS_ENGINE_AUTO));
  EXPECT(gfrs_decoder_engine(dec) == (nlost >= 16 && k >= 64 ? GFRS_ENGINE_MFMA : GFRS_ENGINE_VALU), "decoder engine");
  CHECK(gfrs_copy(gfrs_decoder_rows(dec), surv, sizeof(int) * (size_t)k));
  CHECK(gfrs_decoder_solve(dec, NULL, NULL));
  EXPECT(gfrs_decoder_status(dec, NULL) == 0, "decoder status");
  CHECK(gfrs_decoder_run(dec, NULL));
  CHECK(gfrs_sync(0));
  EXPECT(rows_equal_device(d_out, data, k, C), "decoded rows differ from the data");

  /* 3. an invalid survivor list stores nothing and says so; a singular one is refused on the host */
  int bad[256];
  memcpy(bad, surv, sizeof(int) * (size_t)k);
  bad[1] = bad[0];
  CHECK(gfrs_copy(gfrs_decoder_rows(dec), bad, sizeof(int) * (size_t)k));
  CHECK(gfrs_decoder_solve(dec, NULL, NULL));
  EXPECT(gfrs_decoder_status(dec, NULL) == 2, "duplicate survivor not reported");
  uint8_t* dm = malloc((size_t)(k * k));
  CHECK(gfrs_decode_matrix(e, k, p, surv, dm));
  EXPECT(gfrs_decode_matrix(e, k, p, bad, dm) == GFRS_ESINGULAR, "singular pattern accepted");

  gfrs_decoder_destroy(dec);
  gfrs_plan_destroy(enc);
  free(dm);
  free(e);
  free_rows(d_chunks, NULL, n);
  free_rows(d_out, NULL, k);
  free_rows(NULL, data, k);
  free_rows(NULL, par, p);
  printf("stripe k=%d p=%d C=%lld engine=%s: encode + device-built decode of %d lost natives OK\n", k, p,
         (long long)C, expect_engine == GFRS_ENGINE_MFMA ? "mfma" : "valu", nlost);
}

static void host_pipeline(void) {
  const int k = 6, p = 3;
  const int64_t C = (3 << 20) + 77;
  uint8_t e[18];
  CHECK(gfrs_encoding_matrix(GFRS_MATRIX_CAUCHY, k, p, e));
  uint8_t** data = host_rows(k, C);
  uint8_t** got = host_rows(p, C);
  uint8_t** want = host_rows(p, C);
  for (int j = 0; j < k; ++j)
    for (int64_t x = 0; x < C; ++x) data[j][x] = (uint8_t)(x * 7 + j * 13);
  host_gemm(e, p, k, data, want, C);
  const int dev = 0;
  CHECK(gfrs_gemm_host(&dev, 1, k, p, e, (const uint8_t* const*)data, got, C, 2, 1 << 20));
  for (int i = 0; i < p; ++i) EXPECT(memcmp(got[i], want[i], (size_t)C) == 0, "host pipeline mismatch");
  free_rows(NULL, data, k);
  free_rows(NULL, got, p);
  free_rows(NULL, want, p);
  printf("host pipeline k=%d p=%d C=%lld OK\n", k, p, (long long)C);
}

int main(void) {
  gf_init();
  printf("gfrs C API v%d, %d device(s)\n", gfrs_api_version(), gfrs_device_count());
  if (gfrs_device_count() < 1) return 77;
  stripe_round_trip(10, 4, (1 << 20) + 4096 + 17, GFRS_ENGINE_VALU, 3);
  stripe_round_trip(128, 32, (1 << 18) + 256 * 3 + 96, GFRS_ENGINE_MFMA, 20);
  host_pipeline();
  CHECK(gfrs_release());
  printf("capi_demo OK\n");
  return 0;
}

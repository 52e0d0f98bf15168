// libgfrs.so: the C API of include/gfrs.h over the gfx950 kernels and the host runtime.
//
// The reference's library surface is two extern "C" functions, encode_file / decode_file
// (src/encode.h:36, src/decode.h:38), each of which sets up devices, streams and buffers, runs,
// and tears everything down. Here the same two calls exist (with the pipeline's persistent
// workspaces and the setup overlapped with the file reads), and the device-side building blocks are
// exported too: a plan is the GF-GEMM descriptor + (for wide stripes) the FP4 bit-matrix, built
// once and launched per stripe; a decoder is the device-built decode plan of ops.PatternDecoder
// (gpu_rscode_amd/ops/inverse.py), so a C caller gets the same one-launch decode with the erasure
// pattern never leaving the GPU.
#include "gfrs.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <exception>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "gfrs/async_prepare.h"
#include "gfrs/codec_file.h"
#include "gfrs/desc.h"
#include "gfrs/host_alloc.h"
#include "gfrs/host_desc.h"
#include "gfrs/kernels.h"
#include "gfrs/matrix.h"
#include "gfrs/pipeline.h"

namespace {

thread_local std::string g_err;

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw Error(GFRS_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}
void need(bool ok, const std::string& what) {
  if (!ok) throw Error(GFRS_EINVAL, what);
}

// Runs f, mapping exceptions to codes and recording the message for gfrs_last_error().
template <typename F>
int guarded(F&& f) {
  try {
    f();
    return GFRS_OK;
  } catch (const Error& e) {
    g_err = e.what();
    return e.code;
  } catch (const std::invalid_argument& e) {
    g_err = e.what();
    return GFRS_EINVAL;
  } catch (const std::exception& e) {
    g_err = e.what();
    return GFRS_EIO;  // the file codec reports format / IO problems as runtime_error
  } catch (...) {
    g_err = "unknown error";
    return GFRS_EINTERNAL;
  }
}

hipStream_t as_stream(void* s) { return static_cast<hipStream_t>(s); }

// A device buffer owned by a plan or decoder.
struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  void alloc(size_t bytes) {
    hip_check(hipMalloc(&p, std::max<size_t>(bytes, 16)), "hipMalloc");
    n = bytes;
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

constexpr int kMfmaMinK = 64, kMfmaMinM = 16, kMgCap = 8;  // as ops/gemm.py _auto_engine
// GF(2^16): as ops/gemm.py _auto_engine16 (profiles/gf65536/r08_mfma16)
constexpr int kMfma16MinK = 16, kMfma16MinM = 4, kMfma16CopyMinM = 8, kMfma16CopyMinKM = 256, kMg16Cap = 2;

class DeviceGuard {  // restores the calling thread's current device
 public:
  explicit DeviceGuard(int dev) {
    hip_check(hipGetDevice(&prev_), "hipGetDevice");
    if (dev != prev_) hip_check(hipSetDevice(dev), "hipSetDevice");
  }
  // Teardown form (the *_destroy entry points return void and must never throw into C): errors
  // from hipGetDevice/hipSetDevice are ignored, the frees still run.
  struct NoThrow {};
  DeviceGuard(int dev, NoThrow) {
    if (hipGetDevice(&prev_) != hipSuccess) prev_ = dev;
    if (dev != prev_) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() { (void)hipSetDevice(prev_); }

 private:
  int prev_ = 0;
};

gfrs::PipelineOptions pipe_opts(int streams, int64_t slice) {
  gfrs::PipelineOptions o;
  o.streams = streams > 0 ? streams : 2;
  if (slice > 0) o.slice_bytes = slice;
  return o;
}

std::vector<int> device_list(const int* devices, int ndev) {
  if (!devices || ndev <= 0) return {0};
  return std::vector<int>(devices, devices + ndev);
}

void fill_report(const gfrs::FileReport& r, gfrs_file_report* out) {
  if (!out) return;
  out->total_size = r.total_size;
  out->chunk_size = r.chunk_size;
  out->k = r.k;
  out->p = r.p;
  out->erased = r.erased;
  out->rejected = r.rejected;
  out->ms_alloc = r.ms_alloc;
  out->ms_read = r.ms_read;
  out->ms_matrix = r.ms_matrix;
  out->ms_compute = r.ms_compute;
  out->ms_write = r.ms_write;
}

}  // namespace

// ---- plan -----------------------------------------------------------------------------------
struct gfrs_plan {
  int device = 0, k = 0, m = 0, m_pad = 0, engine = GFRS_ENGINE_VALU;
  int64_t ncols = 0, in_stride = 0;
  bool bytewise = false, copies = false;
  DevBuf desc, bitmat, coeff;

  void build_bitmat(const uint8_t* c) {  // FP4 bit-matrix from host coefficients (synchronous)
    if (!coeff.p) coeff.alloc(size_t(m) * k);
    hip_check(hipMemcpy(coeff.p, c, size_t(m) * k, hipMemcpyHostToDevice), "hipMemcpy coeff");
    if (!bitmat.p) bitmat.alloc(gfrs::fp4_bitmat_bytes(k, m, kMgCap));
    hip_check(gfrs::launch_fp4_bitmat(static_cast<const uint8_t*>(coeff.p), m, k, bitmat.p, kMgCap, nullptr),
              "fp4_bitmat");
    hip_check(hipStreamSynchronize(nullptr), "hipStreamSynchronize");
  }
  void run(hipStream_t s) const {
    if (engine == GFRS_ENGINE_MFMA)
      hip_check(gfrs::launch_gf_gemm_fp4(bitmat.p, desc.p, k, m, 0, ncols, kMgCap, copies ? 0 : in_stride, copies, s),
                "gf_gemm_fp4");
    else
      hip_check(gfrs::launch_gf_gemm(desc.p, k, m_pad, 0, ncols, bytewise, 0, s, copies), "gf_gemm");
  }
};

namespace {

// Shared by gfrs_plan_create and the decoder: descriptor upload + engine choice.
void init_plan(gfrs_plan* p, int device, int k, int m, const uint8_t* coeff, const std::vector<uint64_t>& in,
               const std::vector<uint64_t>& out, const std::vector<uint64_t>& copy, int64_t ncols, int engine) {
  need(k >= 1 && k <= 256 && m >= 1 && m <= 256, "plan: 1 <= k, m <= 256");
  need(ncols >= 0, "plan: ncols must be >= 0");
  need(engine == GFRS_ENGINE_AUTO || engine == GFRS_ENGINE_VALU || engine == GFRS_ENGINE_MFMA, "plan: bad engine");
  p->device = device;
  p->k = k;
  p->m = m;
  p->m_pad = gfrs::pad_m(m);
  p->ncols = ncols;
  p->copies = !copy.empty();
  auto misaligned = [](uint64_t a) { return a % 16 != 0; };
  p->bytewise = std::any_of(in.begin(), in.end(), misaligned) || std::any_of(out.begin(), out.end(), misaligned) ||
                std::any_of(copy.begin(), copy.end(), [](uint64_t a) { return a && a % 16; });
  if (engine == GFRS_ENGINE_AUTO)
    engine = (!p->bytewise && k >= kMfmaMinK && m >= kMfmaMinM) ? GFRS_ENGINE_MFMA : GFRS_ENGINE_VALU;
  need(!(engine == GFRS_ENGINE_MFMA && p->bytewise), "plan: the matrix-core engine needs 16-byte aligned rows");
  p->engine = engine;
  const gfrs::Mat c = coeff ? gfrs::Mat(coeff, coeff + size_t(m) * k) : gfrs::Mat();
  const std::vector<uint8_t> host = gfrs::build_desc(k, m, in, copy, out, c);
  DeviceGuard g(device);
  p->desc.alloc(host.size());
  hip_check(hipMemcpy(p->desc.p, host.data(), host.size(), hipMemcpyHostToDevice), "hipMemcpy desc");
  if (engine == GFRS_ENGINE_MFMA) {
    // rows of one allocation at a fixed stride: the FP4 kernel computes its DMA addresses
    const int64_t stride = k > 1 ? int64_t(in[1] - in[0]) : 1;
    bool uniform = stride != 0;
    for (int j = 0; j < k && uniform; ++j) uniform = int64_t(in[j] - in[0]) == j * stride;
    p->in_stride = uniform ? stride : 0;
    if (coeff)
      p->build_bitmat(coeff);
    else {  // tables come later (the decoder's device solve)
      p->bitmat.alloc(gfrs::fp4_bitmat_bytes(k, m, kMgCap));
      hip_check(hipMemset(p->bitmat.p, 0, p->bitmat.n), "hipMemset");
    }
  }
}

std::vector<uint64_t> addrs(const void* const* rows, int n) {
  std::vector<uint64_t> v(static_cast<size_t>(n));
  for (int i = 0; i < n; ++i) v[size_t(i)] = reinterpret_cast<uint64_t>(rows[i]);
  return v;
}

}  // namespace

// ---- GF(2^16) plan ----------------------------------------------------------------------------
struct gfrs_plan16 {
  int device = 0, k = 0, m = 0, m_pad = 0, engine = GFRS_ENGINE_VALU;
  int64_t ncols = 0, in_stride = 0;
  bool symwise = false, copies = false;
  DevBuf desc, bitmat, coeff;

  void run(hipStream_t s) const {
    if (engine == GFRS_ENGINE_MFMA)
      hip_check(gfrs::launch_gf_gemm16_fp4(bitmat.p, desc.p, k, m, 0, ncols, kMg16Cap, copies ? 0 : in_stride, copies, s),
                "gf_gemm16_fp4");
    else
      hip_check(gfrs::launch_gf_gemm16(desc.p, k, m_pad, 0, ncols, symwise, 0, s), "gf_gemm16");
  }
};

// ---- decoder --------------------------------------------------------------------------------
struct gfrs_decoder {
  int k = 0, n = 0, e = 0;
  gfrs_plan plan;
  DevBuf g, ptrs, rows, erased, status, dm;
};

extern "C" {

int gfrs_api_version(void) { return GFRS_API_VERSION; }
const char* gfrs_last_error(void) { return g_err.c_str(); }

int gfrs_device_count(void) {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

void* gfrs_dev_alloc(int device, size_t bytes) {
  void* p = nullptr;
  const int rc = guarded([&] {
    DeviceGuard g(device);
    hip_check(hipMalloc(&p, bytes), "hipMalloc");
  });
  return rc == GFRS_OK ? p : nullptr;
}

void gfrs_dev_free(void* p) {
  if (p) (void)hipFree(p);
}

int gfrs_copy(void* dst, const void* src, size_t bytes) {
  return guarded([&] { hip_check(hipMemcpy(dst, src, bytes, hipMemcpyDefault), "hipMemcpy"); });
}

int gfrs_sync(int device) {
  return guarded([&] {
    DeviceGuard g(device);
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  });
}

int gfrs_encoding_matrix(int kind, int k, int p, uint8_t* e) {
  return guarded([&] {
    need(e && k >= 1 && p >= 1 && k + p <= 256, "encoding_matrix: 1 <= k, p and k + p <= 256");
    need(kind >= 0 && kind <= 2, "encoding_matrix: bad kind");
    const gfrs::Mat m = gfrs::encoding_matrix(static_cast<gfrs::MatrixKind>(kind), k, p);
    std::memcpy(e, m.data(), m.size());
  });
}

int gfrs_encoding_matrix16(int kind, int k, int p, uint16_t* e) {
  return guarded([&] {
    need(e && k >= 1 && p >= 1 && k + p <= 65535, "encoding_matrix16: 1 <= k, p and k + p <= 65535");
    need(kind >= 0 && kind <= 2, "encoding_matrix16: bad kind");
    const gfrs::gf16w::Mat m = gfrs::encoding_matrix16(static_cast<gfrs::MatrixKind>(kind), k, p);
    std::copy(m.begin(), m.end(), e);
  });
}

int gfrs_decode_rows16(const uint16_t* e, int k, int p, const int* survivors, const int* erased, int n_erased,
                       uint16_t* rows_out) {
  return guarded([&] {
    need(e && survivors && erased && rows_out && k >= 1 && p >= 1 && k + p <= 65535 && n_erased >= 1 &&
             n_erased <= k,
         "decode_rows16: bad arguments");
    std::vector<int> rows(survivors, survivors + k), want(erased, erased + n_erased);
    for (int r : rows) need(r >= 0 && r < k + p, "decode_rows16: survivor id out of range");
    for (int w : want) need(w >= 0 && w < k, "decode_rows16: erased native id out of range");
    const gfrs::gf16w::Mat g = gfrs::gf16w::generator(gfrs::gf16w::Mat(e, e + size_t(p) * k), k, p);
    gfrs::gf16w::Mat out;
    if (!gfrs::gf16w::decode_rows(g, k, rows, want, out)) throw Error(GFRS_ESINGULAR, "decode_rows16: pattern not recoverable");
    std::copy(out.begin(), out.end(), rows_out);
  });
}

int gfrs_plan16_create(gfrs_plan16** plan, int device, int k, int m, const uint16_t* coeff, const void* const* in,
                       void* const* out, void* const* copy, int64_t ncols, int engine) {
  return guarded([&] {
    need(plan && coeff && in && out, "plan16_create: plan, coeff, in and out are required");
    need(k >= 1 && k <= 65535 && m >= 1 && m <= 65535, "plan16_create: 1 <= k, m <= 65535");
    need(ncols >= 0 && ncols % 2 == 0, "plan16_create: ncols must be an even byte count");
    need(engine == GFRS_ENGINE_AUTO || engine == GFRS_ENGINE_VALU || engine == GFRS_ENGINE_MFMA,
         "plan16_create: bad engine");
    auto p = std::make_unique<gfrs_plan16>();
    p->device = device;
    p->k = k;
    p->m = m;
    p->m_pad = gfrs::pad_m(m);
    p->ncols = ncols;
    const std::vector<uint64_t> iv = addrs(in, k), ov = addrs(const_cast<const void* const*>(out), m);
    std::vector<uint64_t> cv;
    if (copy) cv = addrs(const_cast<const void* const*>(copy), k);
    p->copies = !cv.empty();
    auto odd = [](uint64_t a) { return a % 2 != 0; };
    need(std::none_of(iv.begin(), iv.end(), odd) && std::none_of(ov.begin(), ov.end(), odd) &&
             std::none_of(cv.begin(), cv.end(), odd),
         "plan16_create: rows must be 2-byte aligned");
    auto mis16 = [](uint64_t a) { return a % 16 != 0; };
    p->symwise = std::any_of(iv.begin(), iv.end(), mis16) || std::any_of(ov.begin(), ov.end(), mis16) ||
                 std::any_of(cv.begin(), cv.end(), [](uint64_t a) { return a && a % 16; });
    if (engine == GFRS_ENGINE_AUTO) {
      const bool wide = k >= kMfma16MinK && m >= kMfma16MinM &&
                        (!p->copies || (m >= kMfma16CopyMinM && int64_t(k) * m >= kMfma16CopyMinKM));
      engine = (!p->symwise && wide) ? GFRS_ENGINE_MFMA : GFRS_ENGINE_VALU;
    }
    need(!(engine == GFRS_ENGINE_MFMA && p->symwise), "plan16_create: the matrix-core engine needs 16-byte aligned rows");
    p->engine = engine;
    const gfrs::Mat packed = gfrs::pack16(gfrs::gf16w::Mat(coeff, coeff + size_t(m) * k));
    const std::vector<uint8_t> host = gfrs::build_desc(k, m, iv, cv, ov, packed, 16);
    DeviceGuard g(device);
    p->desc.alloc(host.size());
    hip_check(hipMemcpy(p->desc.p, host.data(), host.size(), hipMemcpyHostToDevice), "hipMemcpy desc");
    if (engine == GFRS_ENGINE_MFMA) {
      const int64_t stride = k > 1 ? int64_t(iv[1] - iv[0]) : 1;
      bool uniform = stride != 0;
      for (int j = 0; j < k && uniform; ++j) uniform = int64_t(iv[j] - iv[0]) == j * stride;
      p->in_stride = uniform ? stride : 0;
      p->coeff.alloc(size_t(m) * k * 2);
      hip_check(hipMemcpy(p->coeff.p, coeff, size_t(m) * k * 2, hipMemcpyHostToDevice), "hipMemcpy coeff");
      p->bitmat.alloc(gfrs::fp16_bitmat_bytes(k, m, kMg16Cap));
      hip_check(gfrs::launch_fp16_bitmat(static_cast<const uint16_t*>(p->coeff.p), k, nullptr, m, k, p->bitmat.p,
                                         kMg16Cap, nullptr),
                "fp16_bitmat");
      hip_check(hipStreamSynchronize(nullptr), "hipStreamSynchronize");
    }
    *plan = p.release();
  });
}

int gfrs_plan16_run(gfrs_plan16* p, void* stream) {
  return guarded([&] {
    need(p != nullptr, "plan16_run: null plan");
    DeviceGuard g(p->device);
    p->run(as_stream(stream));
  });
}

int gfrs_plan16_engine(const gfrs_plan16* p) { return p ? p->engine : GFRS_EINVAL; }

void gfrs_plan16_destroy(gfrs_plan16* p) {
  if (!p) return;
  DeviceGuard g(p->device, DeviceGuard::NoThrow{});
  delete p;
}

int gfrs_decode_matrix(const uint8_t* e, int k, int p, const int* survivors, uint8_t* dm) {
  return guarded([&] {
    need(e && survivors && dm && k >= 1 && p >= 1 && k + p <= 256, "decode_matrix: bad arguments");
    std::vector<int> rows(survivors, survivors + k);
    for (int r : rows) need(r >= 0 && r < k + p, "decode_matrix: survivor id out of range");
    const gfrs::Mat g = gfrs::generator(gfrs::Mat(e, e + size_t(p) * k), k, p);
    gfrs::Mat out;
    if (!gfrs::decode_matrix(g, k, rows, out)) throw Error(GFRS_ESINGULAR, "decode_matrix: pattern not recoverable");
    std::memcpy(dm, out.data(), out.size());
  });
}

int gfrs_plan_create(gfrs_plan** plan, int device, int k, int m, const uint8_t* coeff, const void* const* in,
                     void* const* out, void* const* copy, int64_t ncols, int engine) {
  return guarded([&] {
    need(plan && coeff && in && out, "plan_create: plan, coeff, in and out are required");
    auto p = std::make_unique<gfrs_plan>();
    std::vector<uint64_t> cp;
    if (copy) cp = addrs(const_cast<const void* const*>(copy), k);
    init_plan(p.get(), device, k, m, coeff, addrs(in, k), addrs(const_cast<const void* const*>(out), m), cp, ncols,
              engine);
    *plan = p.release();
  });
}

int gfrs_plan_set_coeff(gfrs_plan* p, const uint8_t* coeff) {
  return guarded([&] {
    need(p && coeff, "plan_set_coeff: bad arguments");
    DeviceGuard g(p->device);
    const std::vector<gfrs::PermTable> t = gfrs::perm_tables_kmajor(gfrs::Mat(coeff, coeff + size_t(p->m) * p->k),
                                                                    p->m, p->k);
    const gfrs::DescLayout l = gfrs::desc_layout(p->k, p->m_pad);
    std::vector<gfrs::PermTable> slab(size_t(p->k) * p->m_pad);
    for (int j = 0; j < p->k; ++j)
      std::copy_n(&t[size_t(j) * p->m], p->m, &slab[size_t(j) * p->m_pad]);
    hip_check(hipMemcpy(static_cast<char*>(p->desc.p) + l.tab_off, slab.data(), slab.size() * sizeof(gfrs::PermTable),
                        hipMemcpyHostToDevice),
              "hipMemcpy tables");
    if (p->engine == GFRS_ENGINE_MFMA) p->build_bitmat(coeff);
  });
}

int gfrs_plan_run(gfrs_plan* p, void* stream) {
  return guarded([&] {
    need(p != nullptr, "plan_run: null plan");
    DeviceGuard g(p->device);
    p->run(as_stream(stream));
  });
}

int gfrs_plan_engine(const gfrs_plan* p) { return p ? p->engine : GFRS_EINVAL; }

void gfrs_plan_destroy(gfrs_plan* p) {
  if (!p) return;
  DeviceGuard g(p->device, DeviceGuard::NoThrow{});
  delete p;
}

int gfrs_decoder_create(gfrs_decoder** dec, int device, int k, int p, const uint8_t* e, void* const* chunks,
                        void* const* out, int64_t ncols, int erased, int engine) {
  return guarded([&] {
    need(dec && e && chunks && out, "decoder_create: dec, e, chunks and out are required");
    need(k >= 1 && p >= 1 && k + p <= 256, "decoder_create: 1 <= k, p and k + p <= 256");
    need(erased >= 1 && erased <= std::min(k, p), "decoder_create: erased must be in [1, min(k, p)]");
    const int n = k + p;
    auto d = std::make_unique<gfrs_decoder>();
    d->k = k;
    d->n = n;
    d->e = erased;
    const std::vector<uint64_t> ch = addrs(const_cast<const void* const*>(chunks), n);
    const std::vector<uint64_t> o = addrs(const_cast<const void* const*>(out), k);
    for (uint64_t a : ch) need(a && a % 16 == 0, "decoder_create: chunk rows must be 16-byte aligned");
    for (uint64_t a : o) need(a && a % 16 == 0, "decoder_create: output rows must be 16-byte aligned");
    // placeholders until the first solve: inputs = the natives, outputs = the first e output rows,
    // copies = every output row (the solve rewrites all of them from the pattern)
    init_plan(&d->plan, device, k, erased, nullptr, std::vector<uint64_t>(ch.begin(), ch.begin() + k),
              std::vector<uint64_t>(o.begin(), o.begin() + erased), o, ncols, engine);
    if (d->plan.engine == GFRS_ENGINE_MFMA) d->plan.in_stride = 0;  // survivors are not equally spaced
    DeviceGuard g(device);
    const gfrs::Mat gen = gfrs::generator(gfrs::Mat(e, e + size_t(p) * k), k, p);
    d->g.alloc(gen.size());
    hip_check(hipMemcpy(d->g.p, gen.data(), gen.size(), hipMemcpyHostToDevice), "hipMemcpy G");
    std::vector<uint64_t> all(ch);
    all.insert(all.end(), o.begin(), o.end());
    d->ptrs.alloc(all.size() * 8);
    hip_check(hipMemcpy(d->ptrs.p, all.data(), all.size() * 8, hipMemcpyHostToDevice), "hipMemcpy ptrs");
    d->rows.alloc(size_t(k) * 4);
    d->erased.alloc(size_t(erased) * 4);
    d->status.alloc(4);
    hip_check(hipMemset(d->rows.p, 0, d->rows.n), "hipMemset");
    hip_check(hipMemset(d->status.p, 0, 4), "hipMemset");
    if (d->plan.engine == GFRS_ENGINE_MFMA) d->dm.alloc(size_t(erased) * k);
    *dec = d.release();
  });
}

int* gfrs_decoder_rows(gfrs_decoder* d) { return d ? static_cast<int*>(d->rows.p) : nullptr; }

int gfrs_decoder_solve(gfrs_decoder* d, const int* rows_dev, void* stream) {
  return guarded([&] {
    need(d != nullptr, "decoder_solve: null decoder");
    DeviceGuard g(d->plan.device);
    const hipStream_t s = as_stream(stream);
    const int* rows = rows_dev ? rows_dev : static_cast<const int*>(d->rows.p);
    const bool mfma = d->plan.engine == GFRS_ENGINE_MFMA;
    hip_check(gfrs::launch_gf_decode_system(static_cast<const uint8_t*>(d->g.p), d->k, rows,
                                            static_cast<int*>(d->erased.p), d->e,
                                            mfma ? static_cast<uint8_t*>(d->dm.p) : nullptr,
                                            static_cast<int*>(d->status.p), d->plan.desc.p, d->plan.m_pad, s,
                                            static_cast<const uint64_t*>(d->ptrs.p), d->n),
              "decode_system");
    if (mfma)
      hip_check(gfrs::launch_fp4_bitmat_sel(static_cast<const uint8_t*>(d->dm.p), d->k, nullptr, d->e, d->k,
                                            d->plan.bitmat.p, kMgCap, s),
                "fp4_bitmat_sel");
  });
}

int gfrs_decoder_run(gfrs_decoder* d, void* stream) {
  return guarded([&] {
    need(d != nullptr, "decoder_run: null decoder");
    DeviceGuard g(d->plan.device);
    d->plan.run(as_stream(stream));
  });
}

int gfrs_decoder_status(gfrs_decoder* d, void* stream) {
  int st = -1;
  const int rc = guarded([&] {
    need(d != nullptr, "decoder_status: null decoder");
    DeviceGuard g(d->plan.device);
    hip_check(hipMemcpyAsync(&st, d->status.p, 4, hipMemcpyDeviceToHost, as_stream(stream)), "hipMemcpyAsync");
    hip_check(hipStreamSynchronize(as_stream(stream)), "hipStreamSynchronize");
  });
  return rc == GFRS_OK ? st : rc;
}

int gfrs_decoder_engine(const gfrs_decoder* d) { return d ? d->plan.engine : GFRS_EINVAL; }

void gfrs_decoder_destroy(gfrs_decoder* d) {
  if (!d) return;
  DeviceGuard g(d->plan.device, DeviceGuard::NoThrow{});
  delete d;
}

int gfrs_gemm_host(const int* devices, int ndev, int k, int m, const uint8_t* coeff, const uint8_t* const* in,
                   uint8_t* const* out, int64_t ncols, int streams, int64_t slice_bytes) {
  return guarded([&] {
    need(coeff && in && out && k >= 1 && m >= 1 && k <= 256 && m <= 256 && ncols >= 0, "gemm_host: bad arguments");
    std::vector<const uint8_t*> ip(in, in + k);
    std::vector<uint8_t*> op(out, out + m);
    hip_check(gfrs::gemm_host_multi(device_list(devices, ndev), ip, op, gfrs::Mat(coeff, coeff + size_t(m) * k), ncols,
                                    pipe_opts(streams, slice_bytes), nullptr, nullptr),
              "gemm_host");
  });
}

int gfrs_encode_file_ex(const char* file, int k, int p, int matrix_kind, int field_w, unsigned flags,
                        const int* devices, int ndev, int streams, gfrs_file_report* report) {
  return guarded([&] {
    need(file && *file, "encode_file: no file");
    need(matrix_kind >= 0 && matrix_kind <= 2, "encode_file: bad matrix kind");
    need(field_w == 8 || field_w == 16, "encode_file: field width must be 8 or 16");
    const std::vector<int> devs = device_list(devices, ndev);
    gfrs::PipelineOptions opt = pipe_opts(streams, 0);
    opt.field_w = field_w;
    opt.zero_copy = (flags & GFRS_FLAG_ZERO_COPY) != 0;
    auto prep = gfrs::prepare_for_encode(devs, opt, file, k, p);  // device setup beside the reads
    const gfrs::GemmFn gemm = [&](const std::vector<const uint8_t*>& in, const std::vector<uint8_t*>& out,
                                  const gfrs::Mat& coeff, int64_t ncols, int fw) {
      if (prep) {
        prep->wait();
        prep.reset();
      }
      gfrs::PipelineOptions o = opt;
      o.field_w = fw;
      hip_check(gfrs::gemm_host_multi(devs, in, out, coeff, ncols, o, nullptr, nullptr), "GPU pipeline");
    };
    fill_report(gfrs::encode_file(file, k, p, static_cast<gfrs::MatrixKind>(matrix_kind), gemm,
                                  gfrs::thp_pinned_host_alloc(), false, field_w),
                report);
  });
}

int gfrs_encode_file(const char* file, int k, int p, int matrix_kind, const int* devices, int ndev, int streams,
                     gfrs_file_report* report) {
  return gfrs_encode_file_ex(file, k, p, matrix_kind, 8, 0u, devices, ndev, streams, report);
}

int gfrs_decode_file_ex(const char* file, const char* conf, const char* out, unsigned flags, const int* devices,
                        int ndev, int streams, gfrs_file_report* report) {
  return guarded([&] {
    need(file && *file && conf && *conf, "decode_file: file and conf are required");
    const std::vector<int> devs = device_list(devices, ndev);
    gfrs::PipelineOptions opt = pipe_opts(streams, 0);
    opt.zero_copy = (flags & GFRS_FLAG_ZERO_COPY) != 0;
    auto prep = gfrs::prepare_for_decode(devs, opt, file);
    const gfrs::GemmFn gemm = [&](const std::vector<const uint8_t*>& in, const std::vector<uint8_t*>& o,
                                  const gfrs::Mat& coeff, int64_t ncols, int fw) {
      if (prep) {
        prep->wait();
        prep.reset();
      }
      gfrs::PipelineOptions po = opt;
      po.field_w = fw;
      hip_check(gfrs::gemm_host_multi(devs, in, o, coeff, ncols, po, nullptr, nullptr), "GPU pipeline");
    };
    fill_report(gfrs::decode_file(file, conf, out ? out : "", gemm, gfrs::thp_pinned_host_alloc()), report);
  });
}

int gfrs_decode_file(const char* file, const char* conf, const char* out, const int* devices, int ndev, int streams,
                     gfrs_file_report* report) {
  return gfrs_decode_file_ex(file, conf, out, 0u, devices, ndev, streams, report);
}

int gfrs_release(void) {
  return guarded([&] { hip_check(gfrs::release_workspaces(), "release_workspaces"); });
}

}  // extern "C"

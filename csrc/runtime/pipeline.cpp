// Host<->device streaming pipeline. See gfrs/pipeline.h for the design notes.
#include "gfrs/pipeline.h"
#include "gfrs/tune.h"
#include "gfrs/trace.h"

#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

#include "gfrs/host_desc.h"
#include "gfrs/kernels.h"

namespace gfrs {
namespace {

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

#define GFRS_TRY(expr)                   \
  do {                                   \
    const hipError_t e__ = (expr);       \
    if (e__ != hipSuccess) return e__;   \
  } while (0)

constexpr int kSlots = 2;  // slice buffers per lane: H2D of one overlaps kernel + D2H of the other

// One slice buffer set: k input rows, m output rows, the GEMM descriptor pointing at them, and the
// two events that hand it between the lane's copy-in and compute streams.
struct Slot {
  uint8_t* in = nullptr;   // k x slice
  uint8_t* out = nullptr;  // m x slice
  void* desc = nullptr;
  size_t in_cap = 0, out_cap = 0, desc_cap = 0;
  std::vector<uint8_t> desc_host;  // what `desc` holds (skip identical re-uploads)
  hipEvent_t loaded = nullptr;     // H2D of the slice done (recorded on copy_in)
  hipEvent_t freed = nullptr;      // D2H of the slice done (recorded on compute)
  bool used = false;               // `freed` has been recorded at least once
};

// A lane = the reference's "stream" (-s): its own copy-in stream (H2D) and compute stream
// (kernel + D2H), and kSlots slice buffers used alternately.
struct Lane {
  hipStream_t copy_in = nullptr;
  hipStream_t compute = nullptr;
  Slot slot[kSlots];
};

// Per-device workspace kept across calls: streams, events, slice buffers and descriptors are
// allocated once and reused while large enough (the streaming file codec calls the pipeline once
// per window; re-creating streams and hipMalloc/hipFree-ing ~100s of MB each time cost ~20 ms per
// call on MI355X, more than the transfers themselves — profiles/r01_round).
struct Workspace {
  std::mutex mu;
  std::vector<Lane> lane;
  // zero-copy path: one stream and one descriptor (pointing at mapped host rows)
  hipStream_t zc_stream = nullptr;
  void* zc_desc = nullptr;
  size_t zc_cap = 0;
  std::vector<uint8_t> zc_host;
};

std::mutex g_ws_mu;
std::map<int, std::unique_ptr<Workspace>>& workspaces() {
  static auto* m = new std::map<int, std::unique_ptr<Workspace>>();  // never destroyed: no hipFree at exit
  return *m;
}
Workspace& workspace(int device) {
  std::lock_guard<std::mutex> g(g_ws_mu);
  auto& p = workspaces()[device];
  if (!p) p = std::make_unique<Workspace>();
  return *p;
}

hipError_t ensure(void** ptr, size_t& cap, size_t need) {
  if (cap >= need && *ptr) return hipSuccess;
  if (*ptr) GFRS_TRY(hipFree(*ptr));
  *ptr = nullptr;
  cap = 0;
  GFRS_TRY(hipMalloc(ptr, need));
  cap = need;
  return hipSuccess;
}

// Waits for everything queued on the lanes (also on error paths: a later call re-uploads
// descriptors with a synchronous hipMemcpy that is not ordered against these non-blocking streams).
hipError_t drain(std::vector<Lane>& lanes) {
  hipError_t first = hipSuccess;
  for (auto& L : lanes)
    for (hipStream_t s : {L.copy_in, L.compute})
      if (s) {
        const hipError_t e = hipStreamSynchronize(s);
        if (first == hipSuccess) first = e;
      }
  return first;
}

hipError_t free_lane(Lane& L) {
  for (hipStream_t s : {L.copy_in, L.compute})
    if (s) GFRS_TRY(hipStreamSynchronize(s));
  for (auto& S : L.slot) {
    if (S.in) GFRS_TRY(hipFree(S.in));
    if (S.out) GFRS_TRY(hipFree(S.out));
    if (S.desc) GFRS_TRY(hipFree(S.desc));
    if (S.loaded) GFRS_TRY(hipEventDestroy(S.loaded));
    if (S.freed) GFRS_TRY(hipEventDestroy(S.freed));
  }
  for (hipStream_t s : {L.copy_in, L.compute})
    if (s) GFRS_TRY(hipStreamDestroy(s));
  L = Lane{};
  return hipSuccess;
}

struct Geometry {
  int64_t slice = 0, nslices = 0;
  int lanes = 0;
};

Geometry geometry(int64_t ncols, const PipelineOptions& opt) {
  Geometry g;
  const int S = opt.streams;
  g.slice = std::max<int64_t>(256, (opt.slice_bytes + 255) / 256 * 256);
  // at least kSlots slices per lane when the range allows it (so every lane double-buffers), never
  // wider than needed
  const int64_t per_slot = ((ncols + int64_t(S) * kSlots - 1) / (int64_t(S) * kSlots) + 255) / 256 * 256;
  g.slice = std::min(g.slice, std::max<int64_t>(256, per_slot));
  g.nslices = (ncols + g.slice - 1) / g.slice;
  g.lanes = int(std::min<int64_t>(S, g.nslices));
  return g;
}

// Streams, events and buffers for `lanes` lanes of k x slice in / m x slice out, descriptors built
// from `coeff` (zeros when empty). Caller holds ws.mu and has set the device.
hipError_t setup_lanes(Workspace& ws, int lanes, int k, int m, int64_t slice, const Mat& coeff, bool split,
                       int field_w = 8) {
  if (int(ws.lane.size()) < lanes) ws.lane.resize(size_t(lanes));
  const Mat zero = coeff.empty() ? Mat(coeff_bytes(m, k, field_w), 0) : Mat{};
  const Mat& c = coeff.empty() ? zero : coeff;
  for (int l = 0; l < lanes; ++l) {
    Lane& L = ws.lane[size_t(l)];
    // (streams map onto a few hardware queues — 4 per process by default — so the copy-in stream
    // exists only when it is used)
    if (split && !L.copy_in) GFRS_TRY(hipStreamCreateWithFlags(&L.copy_in, hipStreamNonBlocking));
    if (!L.compute) GFRS_TRY(hipStreamCreateWithFlags(&L.compute, hipStreamNonBlocking));
    for (auto& S : L.slot) {
      if (!S.loaded) GFRS_TRY(hipEventCreateWithFlags(&S.loaded, hipEventDisableTiming));
      if (!S.freed) GFRS_TRY(hipEventCreateWithFlags(&S.freed, hipEventDisableTiming));
      GFRS_TRY(ensure(reinterpret_cast<void**>(&S.in), S.in_cap, size_t(k) * slice));
      GFRS_TRY(ensure(reinterpret_cast<void**>(&S.out), S.out_cap, size_t(m) * slice));
      std::vector<uint64_t> ip(k), op(m);
      for (int j = 0; j < k; ++j) ip[j] = reinterpret_cast<uint64_t>(S.in + size_t(j) * slice);
      for (int i = 0; i < m; ++i) op[i] = reinterpret_cast<uint64_t>(S.out + size_t(i) * slice);
      std::vector<uint8_t> d = build_desc(k, m, ip, {}, op, c, field_w);
      if (d != S.desc_host) {
        GFRS_TRY(ensure(&S.desc, S.desc_cap, d.size()));
        // every lane was drained before the previous call returned, so no kernel still reads it
        GFRS_TRY(hipMemcpy(S.desc, d.data(), d.size(), hipMemcpyHostToDevice));
        S.desc_host = std::move(d);
      }
    }
  }
  return hipSuccess;
}

// rows [first, first + count) of a host row list, `pitch` bytes apart (count == 1: pitch unused)
struct Run {
  int first = 0, count = 0;
  int64_t pitch = 0;
};

// Largest host row pitch a 2-D copy is given. hipMemcpy2DAsync's pitches are size_t, but the DMA
// engines' pitch fields are narrower than that; beyond 2^31 - 1 (a non-streamed bin/RS run of a big
// file with small k: C of several GiB) rows are copied one by one. GFRS_TUNE=max_rect_pitch=N
// lowers the cap (tests exercise the fallback with small rows).
int64_t max_rect_pitch() {
  static const int64_t cap = [] {
    const int64_t c = (int64_t(1) << 31) - 1;
    const int64_t v = tune_int("max_rect_pitch", c);
    return v > 0 && v < c ? v : c;
  }();
  return cap;
}

// Maximal runs of equally spaced rows with spacing in [min_pitch, max_rect_pitch()] (min_pitch 0:
// every row alone).
template <class Ptr>
std::vector<Run> row_runs(const std::vector<Ptr>& rows, int64_t min_pitch) {
  std::vector<Run> runs;
  auto at = [&](size_t i) { return reinterpret_cast<const uint8_t*>(rows[i]); };
  for (size_t i = 0; i < rows.size();) {
    Run r{int(i), 1, 0};
    if (min_pitch > 0 && i + 1 < rows.size()) {
      const int64_t d = at(i + 1) - at(i);
      if (d >= min_pitch && d <= max_rect_pitch()) {
        r.pitch = d;
        while (i + r.count < rows.size() && at(i + r.count) - at(i + r.count - 1) == d) ++r.count;
      }
    }
    runs.push_back(r);
    i += size_t(r.count);
  }
  return runs;
}

// One run of rows between host memory (pitch r.pitch) and a slot buffer (pitch `slot_pitch`),
// columns [0, w) of the given base pointers. `dst`/`src` point at the run's first row.
template <class Dst, class Src>
hipError_t copy_run(Dst* dst, size_t slot_pitch, const Src* src, const Run& r, int64_t w, hipMemcpyKind kind,
                    hipStream_t s) {
  const bool h2d = kind == hipMemcpyHostToDevice;
  if (r.count == 1) return hipMemcpyAsync(dst, src, size_t(w), kind, s);
  const size_t dpitch = h2d ? slot_pitch : size_t(r.pitch);
  const size_t spitch = h2d ? size_t(r.pitch) : slot_pitch;
  return hipMemcpy2DAsync(dst, dpitch, src, spitch, size_t(w), size_t(r.count), kind, s);
}

bool valid(int k, int m, size_t coeff_size, int64_t c0, int64_t c1, const PipelineOptions& opt) {
  const int cap = max_rows(opt.field_w);
  const bool whole = opt.field_w != 16 || ((c0 | c1) & 1) == 0;  // GF(2^16): whole symbols
  return k > 0 && m > 0 && k <= cap && m <= cap && (coeff_size == 0 || coeff_size == coeff_bytes(m, k, opt.field_w)) &&
         c1 >= c0 && opt.streams > 0 && whole;
}

// The slice GEMM of the pipeline's field (descriptors never carry fused copies).
hipError_t launch_slice(const void* desc, int k, int m, int64_t w, const PipelineOptions& opt, hipStream_t s) {
  if (opt.field_w == 16) return launch_gf_gemm16(desc, k, pad_m(m), 0, w, opt.bytewise, opt.max_blocks, s);
  return launch_gf_gemm(desc, k, pad_m(m), 0, w, opt.bytewise, opt.max_blocks, s, /*copies=*/false);
}

// Device-visible address of a pinned host pointer (hipHostRegister'ed or hipHostMalloc'ed): 0 when
// `p` is not host memory mapped for the current device.
uint64_t mapped_addr(const void* p) {
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  if (at.type != hipMemoryTypeHost || !at.devicePointer) return 0;
  return reinterpret_cast<uint64_t>(at.devicePointer);
}

// Device addresses of every row on the CURRENT device (each gemm_host thread has set its own), or
// empty when one is unmapped there or not 16-byte aligned (the zero-copy kernel streams 16-byte
// groups; a byte-wise pass over PCIe would be slower than staging); `why` says which.
template <class Ptr>
std::vector<uint64_t> map_rows(const std::vector<Ptr>& rows, int& why) {
  std::vector<uint64_t> a(rows.size());
  for (size_t i = 0; i < rows.size(); ++i) {
    a[i] = mapped_addr(rows[i]);
    if (!a[i] || a[i] % 16) {
      why = !a[i] ? kZcUnmapped : kZcUnaligned;
      return {};
    }
  }
  return a;
}

// Zero-copy needs the whole output set in ONE tile: each tile's lanes read all k host rows, so a
// second tile would pull every input byte over PCIe again (GF(2^8): 16 outputs per tile; GF(2^16):
// 8, gf_gemm16.hip).
bool zc_one_tile(int m, int field_w) { return pad_m(m) <= (field_w == 16 ? 8 : kMaxTile); }

// The zero-copy launches go to the null stream: every hardware queue a process creates costs it
// 8-25 ms on first use (the first stream even more), and the null stream is the one queue the
// synchronous descriptor upload uses anyway (scripts/setup_probe.cpp, profiles/host_pipeline/r07_zc2:
// a dedicated stream put 21-23 ms of stream creation plus 8 ms of null-stream bring-up into the
// setup; the null stream alone costs ~26 ms once). GFRS_TUNE=zc_stream=own restores a stream of its own.
bool zc_null_stream() {
  static const bool v = tune_str("zc_stream") != "own";
  return v;
}

hipError_t zc_stream(Workspace& ws) {
  if (!ws.zc_stream && !zc_null_stream()) GFRS_TRY(hipStreamCreateWithFlags(&ws.zc_stream, hipStreamNonBlocking));
  return hipSuccess;
}

}  // namespace

const char* zc_fallback_name(int reason) {
  switch (reason) {
    case kZcNone: return "";
    case kZcUnmapped: return "a host row is not mapped into this device";
    case kZcUnaligned: return "a host row is not 16-byte aligned";
    case kZcWideCode: return "more outputs than one kernel tile (host rows would cross PCIe once per tile)";
  }
  return "unknown";
}

hipError_t release_workspaces() {
  std::lock_guard<std::mutex> g(g_ws_mu);
  for (auto& [dev, ws] : workspaces()) {
    std::lock_guard<std::mutex> l(ws->mu);
    GFRS_TRY(hipSetDevice(dev));
    for (auto& L : ws->lane) GFRS_TRY(free_lane(L));
    ws->lane.clear();
    if (ws->zc_stream) GFRS_TRY(hipStreamSynchronize(ws->zc_stream));
    if (ws->zc_desc) GFRS_TRY(hipFree(ws->zc_desc));
    if (ws->zc_stream) GFRS_TRY(hipStreamDestroy(ws->zc_stream));
    ws->zc_stream = nullptr;
    ws->zc_desc = nullptr;
    ws->zc_cap = 0;
    ws->zc_host.clear();
  }
  return hipSuccess;
}

namespace {

// The zero-copy GEMM over columns [c0, c1) of mapped host rows: one launch on the workspace's
// stream, waited for. Returns hipErrorInvalidValue (nothing launched) when a row is not mapped.
hipError_t gemm_zero_copy(Workspace& ws, const std::vector<const uint8_t*>& in_rows,
                          const std::vector<uint8_t*>& out_rows, const Mat& coeff, int64_t c0, int64_t c1,
                          const PipelineOptions& opt, PipelineStats& st) {
  const int k = int(in_rows.size()), m = int(out_rows.size());
  const auto t0 = Clock::now();
  if (!zc_one_tile(m, opt.field_w)) {
    st.zc_fallback = kZcWideCode;
    return hipErrorInvalidValue;
  }
  int why = kZcNone;
  const std::vector<uint64_t> ip = map_rows(in_rows, why);
  const std::vector<uint64_t> op = ip.empty() ? std::vector<uint64_t>{} : map_rows(out_rows, why);
  if (ip.empty() || op.empty()) {
    st.zc_fallback = why;
    return hipErrorInvalidValue;
  }
  std::vector<uint8_t> d = build_desc(k, m, ip, {}, op, coeff, opt.field_w);
  GFRS_TRY(zc_stream(ws));
  if (d != ws.zc_host) {
    GFRS_TRY(ensure(&ws.zc_desc, ws.zc_cap, d.size()));
    GFRS_TRY(hipMemcpy(ws.zc_desc, d.data(), d.size(), hipMemcpyHostToDevice));
    ws.zc_host = std::move(d);
  }
  st.ms_setup = ms_since(t0);
  const auto t1 = Clock::now();
  {
    TraceRange tr("pipeline/zero-copy");
    const hipError_t e = opt.field_w == 16
                             ? launch_gf_gemm16(ws.zc_desc, k, pad_m(m), c0, c1 - c0, false, opt.max_blocks, ws.zc_stream,
                                                /*one_tile=*/true)
                             : launch_gf_gemm(ws.zc_desc, k, pad_m(m), c0, c1 - c0, opt.bytewise, opt.max_blocks,
                                              ws.zc_stream, /*copies=*/false);
    const hipError_t e2 = hipStreamSynchronize(ws.zc_stream);
    GFRS_TRY(e);
    GFRS_TRY(e2);
  }
  st.ms_stream = ms_since(t1);
  st.zero_copy = true;
  st.bytes_h2d = int64_t(k) * (c1 - c0);
  st.bytes_d2h = int64_t(m) * (c1 - c0);
  st.slices = 1;
  st.lanes = 0;
  return hipSuccess;
}

}  // namespace

hipError_t prepare_pipeline(int device, int k, int m, int64_t ncols, const PipelineOptions& opt,
                            PrepareStats* stats) {
  if (!valid(k, m, 0, 0, ncols, opt)) return hipErrorInvalidValue;
  if (ncols == 0) return hipSuccess;
  PrepareStats ps;
  const auto t_all = Clock::now();
  auto t = t_all;
  {
    TraceRange tr("pipeline/prepare/device");
    GFRS_TRY(hipSetDevice(device));
    GFRS_TRY(hipFree(nullptr));  // forces the device's context into existence on this thread
  }
  ps.ms_device = ms_since(t);
  const Geometry g = geometry(ncols, opt);
  Workspace& ws = workspace(device);
  std::lock_guard<std::mutex> guard(ws.mu);
  TraceRange tr("pipeline/prepare");
  if (opt.zero_copy) {
    // the zero-copy run needs only its stream and the kernel's code object: load it with one
    // launch over a small device scratch row set (no slice buffers, no copy engines)
    t = Clock::now();
    GFRS_TRY(zc_stream(ws));
    ps.ms_lanes = ms_since(t);
    t = Clock::now();
    constexpr int64_t kCols = 4096;
    uint8_t* scratch = nullptr;
    GFRS_TRY(hipMalloc(reinterpret_cast<void**>(&scratch), size_t(k + m) * kCols));
    std::vector<uint64_t> ip(k), op(m);
    for (int j = 0; j < k; ++j) ip[j] = reinterpret_cast<uint64_t>(scratch + size_t(j) * kCols);
    for (int i = 0; i < m; ++i) op[i] = reinterpret_cast<uint64_t>(scratch + size_t(k + i) * kCols);
    const std::vector<uint8_t> d = build_desc(k, m, ip, {}, op, Mat(coeff_bytes(m, k, opt.field_w), 0), opt.field_w);
    void* dd = nullptr;
    hipError_t err = hipMalloc(&dd, d.size());
    if (err == hipSuccess) err = hipMemsetAsync(scratch, 0, size_t(k + m) * kCols, ws.zc_stream);
    if (err == hipSuccess) err = hipMemcpyAsync(dd, d.data(), d.size(), hipMemcpyHostToDevice, ws.zc_stream);
    if (err == hipSuccess)
      err = opt.field_w == 16 ? launch_gf_gemm16(dd, k, pad_m(m), 0, kCols, false, 0, ws.zc_stream)
                              : launch_gf_gemm(dd, k, pad_m(m), 0, kCols, false, 0, ws.zc_stream, /*copies=*/false);
    const hipError_t e2 = hipStreamSynchronize(ws.zc_stream);
    (void)hipFree(dd);
    (void)hipFree(scratch);
    ps.ms_kernel = ms_since(t);
    ps.ms_total = ms_since(t_all);
    if (stats) *stats = ps;
    return err != hipSuccess ? err : e2;
  }
  t = Clock::now();
  {
    TraceRange tl("pipeline/prepare/lanes");
    GFRS_TRY(setup_lanes(ws, g.lanes, k, m, g.slice, {}, opt.copy_streams > 0, opt.field_w));
  }
  ps.ms_lanes = ms_since(t);
  // Before anyone's clock starts, run every path the stream loop will take once, on a few columns:
  // the kernel launch (code-object load), and H2D / D2H copies in both the 1-D and the 2-D form
  // on the streams that will issue them. The first DMA of a process sets up its copy engines and
  // blit kernels: ~15 ms of a 1 GiB encode when it lands inside the loop (profiles/r02c).
  constexpr size_t kProbe = 4096;
  const size_t probe = std::min<size_t>(kProbe, size_t(g.slice));
  void* host = nullptr;
  GFRS_TRY(hipHostMalloc(&host, 2 * kProbe, hipHostMallocDefault));
  auto* h = static_cast<uint8_t*>(host);
  hipError_t err = hipSuccess;
  t = Clock::now();
  {  // kernel first (code-object load), alone, so its cost is separable from the copies'
    TraceRange tk("pipeline/prepare/kernel");
    Lane& L = ws.lane[0];
    err = launch_slice(L.slot[0].desc, k, m, std::min<int64_t>(g.slice, int64_t(probe)), opt, L.compute);
    if (err == hipSuccess) err = hipStreamSynchronize(L.compute);
  }
  ps.ms_kernel = ms_since(t);
  t = Clock::now();
  TraceRange td("pipeline/prepare/dma");
  for (int l = 0; l < g.lanes && err == hipSuccess; ++l) {
    Lane& L = ws.lane[size_t(l)];
    hipStream_t cin = L.copy_in ? L.copy_in : L.compute;
    auto warm = [&]() -> hipError_t {
      GFRS_TRY(hipMemsetAsync(L.slot[0].in, 0, size_t(k) * g.slice, L.compute));
      GFRS_TRY(hipStreamSynchronize(L.compute));
      GFRS_TRY(hipMemcpyAsync(L.slot[0].in, h, probe, hipMemcpyHostToDevice, cin));
      GFRS_TRY(hipMemcpy2DAsync(L.slot[1].in, size_t(g.slice), h, probe, probe, 1, hipMemcpyHostToDevice, cin));
      GFRS_TRY(hipStreamSynchronize(cin));
      GFRS_TRY(launch_slice(L.slot[0].desc, k, m, std::min<int64_t>(g.slice, int64_t(probe)), opt, L.compute));
      GFRS_TRY(hipMemcpyAsync(h + kProbe, L.slot[0].out, probe, hipMemcpyDeviceToHost, L.compute));
      GFRS_TRY(hipMemcpy2DAsync(h + kProbe, probe, L.slot[1].out, size_t(g.slice), probe, 1, hipMemcpyDeviceToHost,
                                L.compute));
      return hipSuccess;
    };
    err = warm();
  }
  const hipError_t e2 = drain(ws.lane);
  const hipError_t e3 = hipHostFree(host);
  ps.ms_dma = ms_since(t);
  ps.ms_total = ms_since(t_all);
  if (stats) *stats = ps;
  if (err != hipSuccess) return err;
  if (e2 != hipSuccess) return e2;
  return e3;
}

hipError_t prepare_pipeline_multi(const std::vector<int>& devices, int k, int m, int64_t ncols,
                                  const PipelineOptions& opt, std::vector<PrepareStats>* stats) {
  const int D = int(devices.size());
  if (D <= 0) return hipErrorInvalidValue;
  std::vector<hipError_t> err(D, hipSuccess);
  std::vector<PrepareStats> ps(static_cast<size_t>(D));
  std::vector<std::thread> th;
  for (int d = 0; d < D; ++d) {
    const auto [a, b] = device_shard(ncols, D, d);
    th.emplace_back([&, d, a = a, b = b] { err[d] = prepare_pipeline(devices[d], k, m, b - a, opt, &ps[size_t(d)]); });
  }
  for (auto& t : th) t.join();
  if (stats) *stats = ps;
  for (auto e : err)
    if (e != hipSuccess) return e;
  return hipSuccess;
}

hipError_t gemm_host(int device, const std::vector<const uint8_t*>& in_rows, const std::vector<uint8_t*>& out_rows,
                     const Mat& coeff, int64_t c0, int64_t c1, const PipelineOptions& opt, PipelineStats* stats) {
  const int k = int(in_rows.size());
  const int m = int(out_rows.size());
  if (!valid(k, m, coeff.size(), c0, c1, opt) || coeff.empty()) return hipErrorInvalidValue;
  PipelineStats st;
  const auto t_all = Clock::now();
  const int64_t ncols = c1 - c0;
  if (ncols == 0) {
    if (stats) *stats = st;
    return hipSuccess;
  }
  GFRS_TRY(hipSetDevice(device));
  const Geometry g = geometry(ncols, opt);
  const int64_t slice = g.slice;
  const int lanes = g.lanes;

  Workspace& ws = workspace(device);
  std::lock_guard<std::mutex> guard(ws.mu);
  if (opt.zero_copy) {
    const hipError_t e = gemm_zero_copy(ws, in_rows, out_rows, coeff, c0, c1, opt, st);
    if (e == hipSuccess) {
      st.ms_total = ms_since(t_all);
      if (stats) *stats = st;
      return hipSuccess;
    }
    if (e != hipErrorInvalidValue) return e;
    const int why = st.zc_fallback;  // refused (reason recorded): the staged pipeline below
    st = PipelineStats{};
    st.zc_fallback = why;
  }
  {
    TraceRange tr("pipeline/setup");
    const hipError_t e = setup_lanes(ws, lanes, k, m, slice, coeff, opt.copy_streams > 0, opt.field_w);
    if (e != hipSuccess) {
      (void)drain(ws.lane);
      return e;
    }
  }
  st.ms_setup = ms_since(t_all);

  // Host rows grouped into maximal runs at one fixed distance >= the slice (e.g. the codec's k x C
  // buffer is one run; a decode's survivors are a run of natives plus a run of parity rows): each
  // run moves as ONE 2-D copy per slice. Measured on MI355X (profiles/r02b): k separate 1-D copies
  // per slice cost up to 30% of the H2D rate on 4 lanes.
  const std::vector<Run> in_runs = row_runs(in_rows, opt.rect ? slice : 0);
  const std::vector<Run> out_runs = row_runs(out_rows, opt.rect ? slice : 0);
  const auto t_stream = Clock::now();
  hipError_t err = hipSuccess;
  {
    TraceRange tr_stream("pipeline/stream-loop");
    // slice t -> lane t % lanes, slot (t / lanes) % kSlots. Copy-in waits until the slot's previous
    // D2H has drained; compute waits for the slot's H2D. No host synchronisation inside the loop.
    for (int64_t t = 0; t < g.nslices && err == hipSuccess; ++t) {
      Lane& L = ws.lane[size_t(t % lanes)];
      Slot& S = L.slot[(t / lanes) % kSlots];
      const int64_t a = c0 + t * slice;
      const int64_t w = std::min(slice, c1 - a);
      hipStream_t cin = (opt.copy_streams && L.copy_in) ? L.copy_in : L.compute;
      auto body = [&]() -> hipError_t {
        if (S.used && cin != L.compute) GFRS_TRY(hipStreamWaitEvent(cin, S.freed, 0));
        for (const Run& r : in_runs)
          GFRS_TRY(copy_run(S.in + size_t(r.first) * slice, size_t(slice), in_rows[r.first] + a, r, w,
                            hipMemcpyHostToDevice, cin));
        if (cin != L.compute) {
          GFRS_TRY(hipEventRecord(S.loaded, cin));
          GFRS_TRY(hipStreamWaitEvent(L.compute, S.loaded, 0));
        }
        GFRS_TRY(launch_slice(S.desc, k, m, w, opt, L.compute));
        for (const Run& r : out_runs)
          GFRS_TRY(copy_run(out_rows[r.first] + a, size_t(slice), S.out + size_t(r.first) * slice, r, w,
                            hipMemcpyDeviceToHost, L.compute));
        GFRS_TRY(hipEventRecord(S.freed, L.compute));
        S.used = true;
        return hipSuccess;
      };
      err = body();
      st.bytes_h2d += int64_t(k) * w;
      st.bytes_d2h += int64_t(m) * w;
    }
  }
  {
    TraceRange tr("pipeline/drain");
    const hipError_t e = drain(ws.lane);
    if (err == hipSuccess) err = e;
  }
  if (err != hipSuccess) return err;
  st.ms_stream = ms_since(t_stream);
  if (!opt.persistent) {
    const auto t_free = Clock::now();
    for (auto& L : ws.lane) GFRS_TRY(free_lane(L));
    ws.lane.clear();
    st.ms_teardown = ms_since(t_free);
  }
  st.ms_total = ms_since(t_all);
  st.slices = int(g.nslices);
  st.lanes = lanes;
  if (stats) *stats = st;
  return hipSuccess;
}

std::pair<int64_t, int64_t> device_shard(int64_t ncols, int devices, int d) {
  // contiguous column shards, 4 KiB aligned, remainder to the last device (src/encode.cu:368-381)
  const int64_t per = (ncols / devices) / 4096 * 4096;
  const int64_t a = int64_t(d) * per;
  const int64_t b = (d == devices - 1) ? ncols : a + per;
  return {a, b};
}

hipError_t gemm_host_multi(const std::vector<int>& devices, const std::vector<const uint8_t*>& in_rows,
                           const std::vector<uint8_t*>& out_rows, const Mat& coeff, int64_t ncols,
                           const PipelineOptions& opt, std::vector<PipelineStats>* stats, double* wall_ms) {
  const int D = int(devices.size());
  if (D <= 0) return hipErrorInvalidValue;
  std::vector<PipelineStats> st(D);
  std::vector<hipError_t> err(D, hipSuccess);
  const auto t0 = Clock::now();
  std::vector<std::thread> th;
  for (int d = 0; d < D; ++d) {
    const auto [a, b] = device_shard(ncols, D, d);
    th.emplace_back([&, d, a = a, b = b] {
      err[d] = gemm_host(devices[d], in_rows, out_rows, coeff, a, b, opt, &st[d]);
    });
  }
  for (auto& t : th) t.join();
  if (wall_ms) *wall_ms = ms_since(t0);
  if (stats) *stats = st;
  for (auto e : err)
    if (e != hipSuccess) return e;
  return hipSuccess;
}

}  // namespace gfrs

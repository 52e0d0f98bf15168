// Host<->device streaming pipeline. See gfrs/pipeline.h for the design notes.
#include "gfrs/pipeline.h"
#include "gfrs/trace.h"

#include <algorithm>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
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

struct Lane {
  hipStream_t stream = nullptr;
  uint8_t* in = nullptr;   // k x slice
  uint8_t* out = nullptr;  // m x slice
  void* desc = nullptr;
  size_t in_cap = 0, out_cap = 0, desc_cap = 0;
  std::vector<uint8_t> desc_host;  // what `desc` holds (skip identical re-uploads)
};

// Per-device workspace kept across calls: streams, slice buffers and the descriptor are allocated
// once and reused while they are large enough (the streaming file codec calls the pipeline once
// per window; re-creating streams and hipMalloc/hipFree-ing ~100s of MB each time cost ~20 ms per
// call on MI355X, more than the transfers themselves — profiles/r01_round).
struct Workspace {
  std::mutex mu;
  std::vector<Lane> lane;
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

hipError_t free_lane(Lane& L) {
  if (L.stream) GFRS_TRY(hipStreamSynchronize(L.stream));
  if (L.in) GFRS_TRY(hipFree(L.in));
  if (L.out) GFRS_TRY(hipFree(L.out));
  if (L.desc) GFRS_TRY(hipFree(L.desc));
  if (L.stream) GFRS_TRY(hipStreamDestroy(L.stream));
  L = Lane{};
  return hipSuccess;
}

}  // namespace

hipError_t release_workspaces() {
  std::lock_guard<std::mutex> g(g_ws_mu);
  for (auto& [dev, ws] : workspaces()) {
    std::lock_guard<std::mutex> l(ws->mu);
    GFRS_TRY(hipSetDevice(dev));
    for (auto& L : ws->lane) GFRS_TRY(free_lane(L));
    ws->lane.clear();
  }
  return hipSuccess;
}

hipError_t gemm_host(int device, const std::vector<const uint8_t*>& in_rows, const std::vector<uint8_t*>& out_rows,
                     const Mat& coeff, int64_t c0, int64_t c1, const PipelineOptions& opt, PipelineStats* stats) {
  const int k = int(in_rows.size());
  const int m = int(out_rows.size());
  if (k <= 0 || m <= 0 || coeff.size() != size_t(m) * k || c1 < c0 || opt.streams <= 0)
    return hipErrorInvalidValue;
  PipelineStats st;
  const auto t_all = Clock::now();
  const int64_t ncols = c1 - c0;
  if (ncols == 0) {
    if (stats) *stats = st;
    return hipSuccess;
  }
  GFRS_TRY(hipSetDevice(device));

  const int S = opt.streams;
  int64_t slice = std::max<int64_t>(256, (opt.slice_bytes + 255) / 256 * 256);
  // at least one slice per stream so every stream has work, never wider than needed
  const int64_t per_stream = ((ncols + S - 1) / S + 255) / 256 * 256;
  slice = std::min(slice, std::max<int64_t>(256, per_stream));
  const int64_t nslices = (ncols + slice - 1) / slice;
  const int lanes = int(std::min<int64_t>(S, nslices));
  const int m_pad = pad_m(m);

  Workspace& ws = workspace(device);
  std::lock_guard<std::mutex> guard(ws.mu);
  {
    TraceRange tr("pipeline/setup");
    if (int(ws.lane.size()) < lanes) ws.lane.resize(size_t(lanes));
    for (int l = 0; l < lanes; ++l) {
      Lane& L = ws.lane[size_t(l)];
      if (!L.stream) GFRS_TRY(hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking));
      GFRS_TRY(ensure(reinterpret_cast<void**>(&L.in), L.in_cap, size_t(k) * slice));
      GFRS_TRY(ensure(reinterpret_cast<void**>(&L.out), L.out_cap, size_t(m) * slice));
      std::vector<uint64_t> ip(k), op(m);
      for (int j = 0; j < k; ++j) ip[j] = reinterpret_cast<uint64_t>(L.in + size_t(j) * slice);
      for (int i = 0; i < m; ++i) op[i] = reinterpret_cast<uint64_t>(L.out + size_t(i) * slice);
      std::vector<uint8_t> d = build_desc(k, m, ip, {}, op, coeff);
      if (d != L.desc_host) {
        GFRS_TRY(ensure(&L.desc, L.desc_cap, d.size()));
        // (the previous call drained every lane before returning, so no kernel still reads it)
        GFRS_TRY(hipMemcpy(L.desc, d.data(), d.size(), hipMemcpyHostToDevice));
        L.desc_host = std::move(d);
      }
    }
  }
  st.ms_setup = ms_since(t_all);

  const auto t_stream = Clock::now();
  {
    TraceRange tr_stream("pipeline/stream-loop");
    for (int64_t t = 0; t < nslices; ++t) {
      Lane& L = ws.lane[size_t(t % lanes)];
      const int64_t a = c0 + t * slice;
      const int64_t w = std::min(slice, c1 - a);
      for (int j = 0; j < k; ++j)
        GFRS_TRY(hipMemcpyAsync(L.in + size_t(j) * slice, in_rows[j] + a, w, hipMemcpyHostToDevice, L.stream));
      GFRS_TRY(launch_gf_gemm(L.desc, k, m_pad, 0, w, opt.bytewise, opt.max_blocks, L.stream));
      for (int i = 0; i < m; ++i)
        GFRS_TRY(hipMemcpyAsync(out_rows[i] + a, L.out + size_t(i) * slice, w, hipMemcpyDeviceToHost, L.stream));
      st.bytes_h2d += int64_t(k) * w;
      st.bytes_d2h += int64_t(m) * w;
    }
  }
  {
    TraceRange tr("pipeline/drain");
    for (int l = 0; l < lanes; ++l) GFRS_TRY(hipStreamSynchronize(ws.lane[size_t(l)].stream));
  }
  st.ms_stream = ms_since(t_stream);
  if (!opt.persistent) {
    const auto t_free = Clock::now();
    for (auto& L : ws.lane) GFRS_TRY(free_lane(L));
    ws.lane.clear();
    st.ms_teardown = ms_since(t_free);
  }
  st.ms_total = ms_since(t_all);
  st.slices = int(nslices);
  if (stats) *stats = st;
  return hipSuccess;
}

hipError_t gemm_host_multi(const std::vector<int>& devices, const std::vector<const uint8_t*>& in_rows,
                           const std::vector<uint8_t*>& out_rows, const Mat& coeff, int64_t ncols,
                           const PipelineOptions& opt, std::vector<PipelineStats>* stats, double* wall_ms) {
  const int D = int(devices.size());
  if (D <= 0) return hipErrorInvalidValue;
  std::vector<PipelineStats> st(D);
  std::vector<hipError_t> err(D, hipSuccess);
  // contiguous column shards, 4 KiB aligned, remainder to the last device (src/encode.cu:368-381)
  const int64_t per = (ncols / D) / 4096 * 4096;
  const auto t0 = Clock::now();
  std::vector<std::thread> th;
  for (int d = 0; d < D; ++d) {
    const int64_t a = int64_t(d) * per;
    const int64_t b = (d == D - 1) ? ncols : a + per;
    th.emplace_back([&, d, a, b] { err[d] = gemm_host(devices[d], in_rows, out_rows, coeff, a, b, opt, &st[d]); });
  }
  for (auto& t : th) t.join();
  if (wall_ms) *wall_ms = ms_since(t0);
  if (stats) *stats = st;
  for (auto e : err)
    if (e != hipSuccess) return e;
  return hipSuccess;
}

}  // namespace gfrs

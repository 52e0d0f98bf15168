// bin/RS — gfx950 Reed-Solomon CLI with the reference's flags (src/main.c:32-167):
//   RS -k K -n N -e FILE [-p G] [-s S]
//   RS -d -i FILE -c CONF [-o OUT] [-p G] [-s S]
// Column-sharded across every visible GPU (one host thread per device, like src/encode.cu:357-408),
// each device streaming pinned host rows through `-s` HIP streams (gfrs/pipeline.h).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <memory>
#include <stdexcept>
#include <string>

#include "cli_common.h"
#include "gfrs/tune.h"
#include "gfrs/async_prepare.h"
#include "gfrs/codec_file.h"
#include "gfrs/format.h"
#include "gfrs/host_alloc.h"
#include "gfrs/pipeline.h"
#include "gfrs/stream_codec.h"

namespace {

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// Pinned host buffers: huge-page anonymous memory + hipHostRegister (gfrs/host_alloc.h, ~25x
// cheaper than hipHostMalloc); GFRS_HOST_ALLOC=hipHostMalloc selects the plain allocator.
gfrs::HostAlloc pinned_alloc() {
  const char* env = std::getenv("GFRS_HOST_ALLOC");
  if (!env || std::string(env) != "hipHostMalloc") return gfrs::thp_pinned_host_alloc();
  return {[](size_t n) -> uint8_t* {
            void* p = nullptr;
            if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) return nullptr;
            return static_cast<uint8_t*>(p);
          },
          [](uint8_t* p) { (void)hipHostFree(p); }};
}

}  // namespace

int main(int argc, char** argv) {
  using namespace gfrs;
  const gfrs_cli::Args a = gfrs_cli::parse(argc, argv, /*gpu=*/true);
  try {
    if (a.op == gfrs_cli::Args::kMakeConf) {
      const std::string name = "conf-" + std::to_string(a.n) + "-" + std::to_string(a.k) + "-" + a.in_file;
      write_conf(name, worst_case_conf(a.in_file, a.n, a.k));
      if (!a.quiet) std::printf("wrote %s\n", name.c_str());
      return 0;
    }
    int ndev = 0;
    const auto t_init = std::chrono::steady_clock::now();
    check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");  // first HIP call: runtime + device discovery
    const double ms_init =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_init).count();
    if (ndev <= 0) throw std::runtime_error("no GPU visible (use bin/CPU-RS for the CPU codec)");
    if (a.gpus > 0 && a.gpus < ndev) ndev = a.gpus;
    std::vector<int> devices(ndev);
    for (int d = 0; d < ndev; ++d) devices[d] = d;
    if (!a.devices.empty()) {
      for (int d : a.devices)
        if (d >= ndev) throw std::runtime_error("--devices: device " + std::to_string(d) + " is not visible");
      devices = a.devices;
      ndev = int(devices.size());
    }

    PipelineOptions opt;
    opt.streams = a.streams;
    opt.max_blocks = a.grid;
    opt.slice_bytes = a.slice;
    opt.zero_copy = a.zero_copy == 1;
    const bool enc = a.op == gfrs_cli::Args::kEncode;
    const char* verb = enc ? "encoding" : "decoding";
    // device setup overlapped with the input reads (gfrs/async_prepare.h), sized for the whole
    // stripe or, streamed, for one window of the streaming codec
    StreamOptions so;
    so.window = a.window;
    so.resume = a.resume;
    so.durable = a.sync;
    so.field_w = enc ? a.field_w : 8;
    const StreamOptions* sop = a.streaming() ? &so : nullptr;
    double gpu_ms = 0;  // stream-loop time: transfers + kernels + frees, all devices (setup excluded)
    double setup_ms = 0, setup_past_ms = 0;  // helper-thread device setup, and the part the GEMM waited for
    opt.field_w = enc ? a.field_w : 8;  // (decode: the field comes from the METADATA)
    std::unique_ptr<AsyncPrepare> prep = enc ? prepare_for_encode(devices, opt, a.in_file, a.k, a.n - a.k, sop)
                                             : prepare_for_decode(devices, opt, a.in_file, sop);
    // GFRS_TUNE=setup=serial (measurement aid): finish the device setup before the host buffers are
    // allocated and the file is read, so each phase's uncontended cost shows
    if (prep && gfrs::tune_str("setup") == "serial") {
      const double ms = prep->wait();
      if (!a.quiet) {
        std::printf("GPU pipeline setup (serial): %fms\n", ms);
        for (size_t d = 0; d < prep->stats().size(); ++d) {
          const PrepareStats& ps = prep->stats()[d];
          std::printf("Device%zu: setup breakdown: device bring-up %fms, streams+buffers %fms, kernel load %fms, "
                      "DMA warm-up %fms\n",
                      d, ps.ms_device, ps.ms_lanes, ps.ms_kernel, ps.ms_dma);
        }
      }
      setup_ms += ms;
      prep.reset();
    }
    const GemmFn gemm = [&](const std::vector<const uint8_t*>& in, const std::vector<uint8_t*>& out,
                            const Mat& coeff, int64_t ncols, int field_w) {
      if (prep) {
        const auto t0 = std::chrono::steady_clock::now();
        const double since_start = prep->ms_until(t0);
        const double ms = prep->wait();
        const double waited = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        setup_ms += ms;
        setup_past_ms += waited;
        if (!a.quiet) {
          std::printf("GPU pipeline setup: %fms on a helper thread started %fms before the GEMM was ready to run "
                      "(%fms of it past the file reads)\n",
                      ms, since_start, waited);
          for (size_t d = 0; d < prep->stats().size(); ++d) {
            const PrepareStats& ps = prep->stats()[d];
            std::printf("Device%zu: setup breakdown: device bring-up %fms, streams+buffers %fms, kernel load %fms, "
                        "DMA warm-up %fms\n",
                        d, ps.ms_device, ps.ms_lanes, ps.ms_kernel, ps.ms_dma);
          }
        }
        prep.reset();
      }
      std::vector<PipelineStats> st;
      double wall = 0;
      PipelineOptions o = opt;
      o.field_w = field_w;
      check(gemm_host_multi(devices, in, out, coeff, ncols, o, &st, &wall), "GPU pipeline");
      gpu_ms += wall;
      if (!a.quiet) {
        for (size_t d = 0; d < st.size(); ++d)
          if (st[d].zero_copy)
            std::printf("Device%zu: Total GPU %s time: %fms (zero-copy kernel %fms, row mapping + descriptor %fms)\n",
                        d, verb, st[d].ms_total, st[d].ms_stream, st[d].ms_setup);
          else
            std::printf("Device%zu: Total GPU %s time: %fms (stream loop %fms, %d slices%s%s)\n", d, verb,
                        st[d].ms_total, st[d].ms_stream, st[d].slices,
                        st[d].zc_fallback ? "; staged, zero-copy refused: " : "", zc_fallback_name(st[d].zc_fallback));
        std::printf("Total GPU %s time using multiple devices: %fms\n", verb, wall);
      }
    };
    FileReport r;
    const auto t_codec = std::chrono::steady_clock::now();
    if (a.streaming()) {
      const StreamReport sr = enc ? encode_file_stream(a.in_file, a.k, a.n - a.k, parse_matrix_kind(a.matrix),
                                                       gemm, pinned_alloc(), so, a.cpu_meta)
                                  : decode_file_stream(a.in_file, a.conf, a.out, gemm, pinned_alloc(), so);
      if (!a.quiet)
        std::printf("Streamed %d window(s) of %lld bytes per chunk (resumed at %lld)\n", sr.windows,
                    static_cast<long long>(sr.window), static_cast<long long>(sr.resumed_from));
      r = sr;
    } else {
      r = enc ? encode_file(a.in_file, a.k, a.n - a.k, parse_matrix_kind(a.matrix), gemm, pinned_alloc(), a.cpu_meta,
                            a.field_w)
              : decode_file(a.in_file, a.conf, a.out, gemm, pinned_alloc());
    }
    const double codec_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_codec).count();
    if (!a.quiet) {
      // the whole file codec call: reads, device setup left on the path, GEMMs, writes (overlapped
      // when streamed), METADATA — what the multi-process --dist codec reports as its codec time
      std::printf("File codec: %fms (%.3f GB/s of input)\n", codec_ms, r.total_size / std::max(codec_ms, 1e-9) / 1e6);
      const double mb = r.total_size / 1048576.0;
      std::printf("Host: HIP runtime init %fms, pinned buffers %fms, file read %fms\n", ms_init, r.ms_alloc,
                  r.ms_read);
      std::printf("GPU %s bandwidth: %.3f MB/s (%lld bytes in %.3f ms of GPU time: transfers + kernels, device "
                  "setup excluded; k=%d, p=%d, %zu device shard(s), %s)\n",
                  verb, mb / (std::max(gpu_ms, 1e-9) / 1e3), static_cast<long long>(r.total_size), gpu_ms, r.k, r.p,
                  devices.size(), opt.zero_copy ? "zero-copy" : (std::to_string(a.streams) + " stream(s)").c_str());
      // the reference's "Total GPU ... time" window starts before its cudaMalloc/cudaStreamCreate
      // (src/encode.cu:117-119,168-232): setup on the critical path counts, overlapped setup does not
      std::printf("GPU %s bandwidth, reference window (setup on the critical path + transfers + kernels): %.3f MB/s "
                  "(%.3f ms); with the whole setup serialised: %.3f MB/s (%.3f ms)\n",
                  verb, mb / (std::max(gpu_ms + setup_past_ms, 1e-9) / 1e3), gpu_ms + setup_past_ms,
                  mb / (std::max(gpu_ms + setup_ms, 1e-9) / 1e3), gpu_ms + setup_ms);
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "RS: %s\n", e.what());
    return 1;
  }
  return 0;
}

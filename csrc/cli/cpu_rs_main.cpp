// bin/CPU-RS — CPU reference codec CLI (the reference's `make CPU` target, src/cpu-rs.c:695-808).
// Runs without a GPU; BASELINE.json config #1 (k=4,n=6 encode+verify of 1 MiB) uses it.
#include <cstdio>
#include <exception>

#include "cli_common.h"
#include "gfrs/codec_file.h"
#include "gfrs/cpu_codec.h"
#include "gfrs/format.h"
#include "gfrs/host_desc.h"
#include "gfrs/stream_codec.h"

int main(int argc, char** argv) {
  using namespace gfrs;
  const gfrs_cli::Args a = gfrs_cli::parse(argc, argv, /*gpu=*/false);
  try {
    const CpuMul strat = parse_cpu_mul(a.mul);
    const GemmFn gemm = [&](const std::vector<const uint8_t*>& in, const std::vector<uint8_t*>& out,
                            const Mat& coeff, int64_t ncols, int field_w) {
      if (field_w == 16)
        cpu_gemm16(in, out, unpack16(coeff), ncols, a.threads);
      else
        cpu_gemm(in, out, coeff, ncols, strat, a.threads);
    };
    if (a.op == gfrs_cli::Args::kMakeConf) {
      const std::string name = "conf-" + std::to_string(a.n) + "-" + std::to_string(a.k) + "-" + a.in_file;
      write_conf(name, worst_case_conf(a.in_file, a.n, a.k));
      if (!a.quiet) std::printf("wrote %s\n", name.c_str());
    } else if (a.op == gfrs_cli::Args::kEncode) {
      StreamOptions so;
      so.window = a.window;
      so.resume = a.resume;
      so.durable = a.sync;
      so.field_w = a.field_w;
      const FileReport r = a.streaming() ? encode_file_stream(a.in_file, a.k, a.n - a.k, parse_matrix_kind(a.matrix),
                                                              gemm, default_host_alloc(), so, a.cpu_meta)
                                         : encode_file(a.in_file, a.k, a.n - a.k, parse_matrix_kind(a.matrix), gemm,
                                                       default_host_alloc(), a.cpu_meta, a.field_w);
      if (!a.quiet) {
        std::printf("Total CPU encoding time: %fms\n", r.ms_matrix + r.ms_compute);
        std::printf("CPU encoding bandwidth: %.3f MB/s (strategy %s, %d thread(s))\n",
                    r.total_size / 1048576.0 / ((r.ms_matrix + r.ms_compute) / 1e3), cpu_mul_name(strat), a.threads);
      }
    } else {
      StreamOptions so;
      so.window = a.window;
      so.resume = a.resume;
      so.durable = a.sync;
      const FileReport r = a.streaming()
                               ? decode_file_stream(a.in_file, a.conf, a.out, gemm, default_host_alloc(), so)
                               : decode_file(a.in_file, a.conf, a.out, gemm, default_host_alloc());
      if (!a.quiet) {
        std::printf("Total CPU decoding time: %fms\n", r.ms_matrix + r.ms_compute);
        std::printf("CPU decoding bandwidth: %.3f MB/s (%d erased native chunk(s))\n",
                    r.total_size / 1048576.0 / ((r.ms_matrix + r.ms_compute) / 1e3), r.erased);
      }
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "CPU-RS: %s\n", e.what());
    return 1;
  }
  return 0;
}

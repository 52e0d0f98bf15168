// Host<->device streaming pipeline (the reference's per-device `-s` stream loop,
// src/encode.cu:109-238 / src/decode.cu:89-196) and its multi-GPU data-parallel driver
// (src/encode.cu:357-432, one host thread per device).
//
// Differences from the reference, by design:
//   * no event on the legacy default stream and no host sync inside the loop (the reference's
//     encode_chunk blocks on cudaEventSynchronize every slice, src/matrix.cu:805-809, which is why
//     its authors saw multi-stream *degrade*, doc/design.tex:530);
//   * the slice ring is larger than the stream count, so copy engines (SDMA) stay busy while the
//     previous slice's kernel runs; buffers are reused round-robin in stream order;
//   * host rows are used in place (no H2H staging copies, src/encode.cu:389-398,410-429); pinned
//     rows give true async DMA;
//   * streams, slice buffers and descriptors persist per device across calls (PipelineOptions::
//     persistent), so per-window calls of the streaming file codec pay no allocation;
//   * 64-bit column ranges (the reference is int-limited to < 2 GiB, src/encode.cu:303-322).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "gfrs/matrix.h"

namespace gfrs {

struct PipelineOptions {
  int streams = 2;                 // -s
  int64_t slice_bytes = 16 << 20;  // column width per slice (rounded to 256)
  int max_blocks = 0;              // -p (grid cap), 0 = uncapped
  bool bytewise = false;           // force the byte kernel (debug/ablation)
  bool persistent = true;          // keep streams/buffers/descriptor per device for the next call
};

struct PipelineStats {
  double ms_setup = 0;    // stream/buffer/descriptor setup (alloc)
  double ms_stream = 0;   // H2D + kernel + D2H loop until the last stream drains
  double ms_teardown = 0;  // frees
  double ms_total = 0;     // everything (the reference's "Total GPU encoding time")
  int64_t bytes_h2d = 0, bytes_d2h = 0;
  int slices = 0;
};

// out_rows[i][c] = XOR_j coeff[i][j] * in_rows[j][c] for c in [c0, c1) on `device`.
hipError_t gemm_host(int device, const std::vector<const uint8_t*>& in_rows, const std::vector<uint8_t*>& out_rows,
                     const Mat& coeff, int64_t c0, int64_t c1, const PipelineOptions& opt, PipelineStats* stats);

// Frees every persistent per-device workspace (streams, slice buffers, descriptors).
hipError_t release_workspaces();

// Column-sharded data parallelism over `devices` (one host thread each). Shard boundaries are
// 4 KiB aligned; stats[d] receives device d's numbers. Returns the first error encountered.
hipError_t gemm_host_multi(const std::vector<int>& devices, const std::vector<const uint8_t*>& in_rows,
                           const std::vector<uint8_t*>& out_rows, const Mat& coeff, int64_t ncols,
                           const PipelineOptions& opt, std::vector<PipelineStats>* stats, double* wall_ms);

}  // namespace gfrs

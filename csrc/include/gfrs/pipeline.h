// Host<->device streaming pipeline (the reference's per-device `-s` stream loop,
// src/encode.cu:109-238 / src/decode.cu:89-196) and its multi-GPU data-parallel driver
// (src/encode.cu:357-432, one host thread per device).
//
// Differences from the reference, by design:
//   * no event on the legacy default stream and no host sync inside the loop (the reference's
//     encode_chunk blocks on cudaEventSynchronize every slice, src/matrix.cu:805-809, which is why
//     its authors saw multi-stream *degrade*, doc/design.tex:530);
//   * every lane ("stream" of -s) owns two slice buffers and two HIP streams — copy-in (H2D) and
//     compute (kernel + D2H) — handing slots over with events, so even -s 1 overlaps the H2D of
//     slice t+1 with the kernel and D2H of slice t (SDMA engines busy in both directions);
//   * host rows are used in place (no H2H staging copies, src/encode.cu:389-398,410-429); pinned
//     rows give true async DMA;
//   * streams, slice buffers and descriptors persist per device across calls (PipelineOptions::
//     persistent), so per-window calls of the streaming file codec pay no allocation;
//   * 64-bit column ranges (the reference is int-limited to < 2 GiB, src/encode.cu:303-322).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>
#include <vector>

#include "gfrs/matrix.h"

namespace gfrs {

struct PipelineOptions {
  int streams = 2;                 // -s
  int64_t slice_bytes = 16 << 20;  // column width per slice (rounded to 256)
  int max_blocks = 0;              // -p (grid cap), 0 = uncapped
  bool bytewise = false;           // force the byte kernel (debug/ablation)
  bool persistent = true;          // keep streams/buffers/descriptor per device for the next call
  int copy_streams = 1;            // 1: H2D on a per-lane copy-in stream; 0: everything on one stream
  bool rect = true;                // equally spaced host rows: one 2-D copy per slice instead of k / m
  int field_w = 8;                 // 8: GF(2^8) coefficients; 4: the GF(16) nibble method (doc/design.tex:190-209);
                                   // 16: GF(2^16), coefficients packed as little-endian pairs (host_desc.h pack16)
  // Zero-copy: the GEMM kernel reads the k input rows and writes the m output rows straight from/to
  // pinned, device-mapped host memory over PCIe (hipHostRegister / hipHostMalloc rows, 16-byte
  // aligned). No slice buffers, no copy engines: the per-process setup is a stream and the kernel
  // load. Falls back to the staged -s pipeline when a row is not mapped or not aligned.
  bool zero_copy = false;
};

// Why a device asked for the zero-copy kernel ran the staged pipeline instead (PipelineStats).
enum ZcFallback : int {
  kZcNone = 0,        // not asked for, or ran zero-copy
  kZcUnmapped = 1,    // a host row is not pinned / not mapped into THIS device's address space
  kZcUnaligned = 2,   // a host row is not 16-byte aligned (the kernel streams 16-byte groups)
  kZcWideCode = 3,    // more outputs than one tile: every tile would re-read the host rows over PCIe
};
const char* zc_fallback_name(int reason);

struct PipelineStats {
  bool zero_copy = false;  // ran the zero-copy kernel (else the staged -s pipeline)
  int zc_fallback = kZcNone;  // zero-copy asked for but refused on this device: why (ZcFallback)
  double ms_setup = 0;    // stream/buffer/descriptor setup (alloc)
  double ms_stream = 0;   // H2D + kernel + D2H loop until the last stream drains
  double ms_teardown = 0;  // frees
  double ms_total = 0;     // everything (the reference's "Total GPU encoding time")
  int64_t bytes_h2d = 0, bytes_d2h = 0;
  int slices = 0;
  int lanes = 0;
};

// out_rows[i][c] = XOR_j coeff[i][j] * in_rows[j][c] for c in [c0, c1) on `device`.
hipError_t gemm_host(int device, const std::vector<const uint8_t*>& in_rows, const std::vector<uint8_t*>& out_rows,
                     const Mat& coeff, int64_t c0, int64_t c1, const PipelineOptions& opt, PipelineStats* stats);

// Where a prepare_pipeline call spends its time (bin/RS prints it; roctx ranges of the same names).
struct PrepareStats {
  double ms_device = 0;  // hipSetDevice: the runtime's device/context bring-up on this thread
  double ms_lanes = 0;   // streams, events, hipMalloc of the slice buffers, descriptor uploads
  double ms_kernel = 0;  // first GEMM launch + completion: code-object load
  double ms_dma = 0;     // first H2D / D2H (1-D and 2-D) per lane: copy engines and blit kernels
  double ms_total = 0;
};

// Creates the device's streams, events and slice buffers for a later gemm_host over `ncols` columns
// of k inputs / m outputs with `opt` (persistent workspace), and loads the kernels — so a caller can
// overlap device setup with its file reads and keep it out of the timed GPU region.
hipError_t prepare_pipeline(int device, int k, int m, int64_t ncols, const PipelineOptions& opt,
                            PrepareStats* stats = nullptr);
// prepare_pipeline on every device for the shards gemm_host_multi will give it (stats per device).
hipError_t prepare_pipeline_multi(const std::vector<int>& devices, int k, int m, int64_t ncols,
                                  const PipelineOptions& opt, std::vector<PrepareStats>* stats = nullptr);

// Column shard [first, second) of device index d of `devices` (4 KiB aligned, remainder last).
std::pair<int64_t, int64_t> device_shard(int64_t ncols, int devices, int d);

// Frees every persistent per-device workspace (streams, slice buffers, descriptors).
hipError_t release_workspaces();

// Column-sharded data parallelism over `devices` (one host thread each). Shard boundaries are
// 4 KiB aligned; stats[d] receives device d's numbers. Returns the first error encountered.
hipError_t gemm_host_multi(const std::vector<int>& devices, const std::vector<const uint8_t*>& in_rows,
                           const std::vector<uint8_t*>& out_rows, const Mat& coeff, int64_t ncols,
                           const PipelineOptions& opt, std::vector<PipelineStats>* stats, double* wall_ms);

}  // namespace gfrs

// Bounded-memory, resumable file codec (SURVEY §5.4 checkpoint/resume, §5.7 stripe length).
//
// The reference reads the whole input into host memory and writes every chunk only after all GPU
// work is done (src/encode.cu:319-345, :434-465): files larger than host RAM are impossible and a
// crash loses everything. Here the stripe is processed in column windows of W bytes per chunk row:
// window w covers chunk bytes [w*W, (w+1)*W) of all n chunks, so host memory is 3 x (k+p) x W
// (read / compute / write buffer sets) whatever the file size, and the three stages overlap:
// read(w+1) on one thread, the GEMM (GPU pipeline or CPU codec) of window w on the caller, and
// write(w-1) + checkpoint on another. After each window is written (and fdatasync'ed) a
// "<target>.PROGRESS" file is atomically replaced (write + rename) with the byte offset reached and
// the running per-chunk CRC-32s; a later call with resume=true validates it against the current
// parameters and continues from there. The output files are byte-identical to encode_file /
// decode_file (tests/test_cpu_codec.py::test_stream_*).
#pragma once

#include <cstdint>
#include <functional>
#include <string>

#include "gfrs/codec_file.h"

namespace gfrs {

struct StreamOptions {
  int64_t window = 0;   // bytes per chunk row per window; 0 = auto (~1 GiB of buffers in total)
  bool resume = true;   // continue from a matching <target>.PROGRESS
  bool durable = true;  // fdatasync the outputs before each checkpoint
  int stop_after = -1;  // testing: return after this many windows of this call (simulated crash)
};

struct StreamReport : FileReport {
  int64_t window = 0;
  int windows = 0;           // windows processed by this call
  int64_t resumed_from = 0;  // chunk offset this call started at (0 = fresh)
  bool complete = false;
};

StreamReport encode_file_stream(const std::string& file, int k, int p, MatrixKind kind, const GemmFn& gemm,
                                const HostAlloc& alloc, const StreamOptions& opt, bool cpu_meta = false);

StreamReport decode_file_stream(const std::string& file, const std::string& conf, const std::string& out,
                                const GemmFn& gemm, const HostAlloc& alloc, const StreamOptions& opt);

std::string progress_path(const std::string& target);

// Column window (bytes per chunk row) the streaming codecs use for `rows` buffered rows per window
// (encode: n, decode: 2k) of C-byte chunks.
int64_t stream_window(const StreamOptions& opt, int rows, int64_t C);

}  // namespace gfrs

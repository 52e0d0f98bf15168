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
#include <vector>

#include "gfrs/codec_file.h"

namespace gfrs {

struct StreamOptions {
  int64_t window = 0;   // bytes per chunk row per window; 0 = auto (~1 GiB of buffers in total)
  bool resume = true;   // continue from a matching <target>.PROGRESS
  bool durable = true;  // fdatasync the outputs before each checkpoint
  int stop_after = -1;  // testing: return after this many windows of this call (simulated crash)
  // testing: return after the last window, before the commit (chunk sizes, METADATA, checkpoint
  // removal): a crash at the last step, which a later call with resume completes
  bool stop_before_commit = false;
  int field_w = 8;      // encode: GF(2^8) or GF(2^16) symbols (decode reads it from METADATA)
  // Column shard (the multi-GPU file codec, one rank per GPU: the reference's per-device column
  // split, src/encode.cu:368-381): process chunk columns [col_lo, col_hi) only (col_hi < 0: to C;
  // GF(2^16): even offsets). With `shard`, the outputs must already exist at their full size (one
  // coordinator creates them): they are neither truncated nor resized, no METADATA is written, the
  // checkpoint is "<target>.PROGRESS.<lo>-<hi>" (shard_progress_path) and is NOT removed when the
  // shard completes (the coordinator removes it once its METADATA is committed, so a job that dies
  // before that resumes finished shards at their end), and StreamReport::crc holds the shard's
  // per-chunk CRC-32s (crc32_combine them in column order for the METADATA).
  int64_t col_lo = 0, col_hi = -1;
  bool shard = false;
  // decode: decode from exactly these survivor chunk ids, in this order (chosen and CRC-verified by
  // a coordinator, choose_survivors), instead of searching the conf; their names come from the conf.
  std::vector<int> rows;
};

struct StreamReport : FileReport {
  int64_t window = 0;
  int windows = 0;           // windows processed by this call
  int64_t resumed_from = 0;  // chunk offset this call started at (col_lo = fresh)
  bool complete = false;
  int64_t col_lo = 0, col_hi = 0;  // the column range processed
  std::vector<uint32_t> crc;       // encode: per-chunk CRC-32 of columns [col_lo, col_hi)
  std::vector<int> rows;           // decode: the survivor chunk ids used, in system order
};

// Decode survivors for `file` + `conf`: the first recoverable k-subset, in conf order, of the chunks
// that exist and match their METADATA CRC-32 (the aggressive read of decode_file). Streams every
// candidate through its CRC in bounded windows. `rejected` counts CRC mismatches.
std::vector<int> choose_survivors(const std::string& file, const std::string& conf, int* rejected = nullptr);

// A survivor check split over ranks (the multi-GPU decode): each rank reads only its column range
// [lo, hi) of every conf candidate (on parallel threads) and reports whether the chunk file is there
// in full and the CRC-32 of those bytes; the coordinator combines the ranks' CRCs in column order
// (crc32_combine), compares them with the METADATA, and picks the survivors from the verdicts.
struct ShardCrc {
  int index = -1;        // chunk index of the candidate (conf order)
  bool present = false;  // the file exists and holds the whole chunk
  uint32_t crc = 0;      // CRC-32 of its bytes [lo, hi)
};
// Only candidates [first, first + count) are read (count < 0: to the end); the others are reported
// absent. The coordinator asks for the first k (all a clean decode needs) and reads further ones only
// when those are short of a recoverable set.
std::vector<ShardCrc> shard_crcs(const std::string& file, const std::string& conf, int64_t lo, int64_t hi,
                                 int first = 0, int count = -1);
// choose_survivors with every candidate's verdict known (intact[ci] != 0: usable), conf order
std::vector<int> choose_survivors_given(const std::string& file, const std::string& conf,
                                        const std::vector<int>& intact);

StreamReport encode_file_stream(const std::string& file, int k, int p, MatrixKind kind, const GemmFn& gemm,
                                const HostAlloc& alloc, const StreamOptions& opt, bool cpu_meta = false);

StreamReport decode_file_stream(const std::string& file, const std::string& conf, const std::string& out,
                                const GemmFn& gemm, const HostAlloc& alloc, const StreamOptions& opt);

std::string progress_path(const std::string& target);
// a column shard's checkpoint: "<target>.PROGRESS.<lo>-<hi>"
std::string shard_progress_path(const std::string& target, int64_t lo, int64_t hi);

// Column window (bytes per chunk row) the streaming codecs use for `rows` buffered rows per window
// (encode: n, decode: 2k) of C-byte chunks.
int64_t stream_window(const StreamOptions& opt, int rows, int64_t C);

}  // namespace gfrs

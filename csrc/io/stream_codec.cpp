// Bounded-memory, resumable file codec (see gfrs/stream_codec.h).
#include "gfrs/stream_codec.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <future>
#include <set>
#include <sstream>
#include <stdexcept>
#include <thread>

#include "gfrs/format.h"
#include "gfrs/host_desc.h"
#include "gfrs/trace.h"

namespace gfrs {
namespace {

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); }

struct Fd {
  int fd = -1;
  Fd() = default;
  explicit Fd(int f) : fd(f) {}
  Fd(Fd&& o) noexcept : fd(o.fd) { o.fd = -1; }
  Fd& operator=(Fd&& o) noexcept {
    std::swap(fd, o.fd);
    return *this;
  }
  Fd(const Fd&) = delete;
  ~Fd() {
    if (fd >= 0) ::close(fd);
  }
};

Fd open_or_throw(const std::string& path, int flags) {
  const int fd = ::open(path.c_str(), flags | O_CLOEXEC, 0644);
  if (fd < 0) throw std::runtime_error("cannot open " + path + ": " + std::strerror(errno));
  return Fd(fd);
}

// reads len bytes at off; what the file does not cover is zero-filled (the padded tail)
void pread_full(int fd, uint8_t* dst, int64_t len, int64_t off) {
  int64_t got = 0;
  while (got < len) {
    const ssize_t r = ::pread(fd, dst + got, size_t(len - got), off + got);
    if (r < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("read failed: ") + std::strerror(errno));
    }
    if (r == 0) break;
    got += r;
  }
  if (got < len) std::memset(dst + got, 0, size_t(len - got));
}

void pwrite_full(int fd, const uint8_t* src, int64_t len, int64_t off) {
  int64_t put = 0;
  while (put < len) {
    const ssize_t w = ::pwrite(fd, src + put, size_t(len - put), off + put);
    if (w < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("write failed: ") + std::strerror(errno));
    }
    put += w;
  }
}

bool file_at_least(const std::string& path, int64_t n) {
  struct stat sb;
  return ::stat(path.c_str(), &sb) == 0 && int64_t(sb.st_size) >= n;
}

int64_t pick_window(const StreamOptions& opt, int rows, int64_t C) {
  int64_t w = opt.window;
  if (w <= 0) {  // ~1 GiB of host buffers in total (3 sets x rows x W), 1..64 MiB per row
    w = (int64_t(1) << 30) / (3 * int64_t(rows));
    w = std::clamp<int64_t>(w, int64_t(1) << 20, int64_t(64) << 20) / 4096 * 4096;
  }
  return std::max<int64_t>(1, std::min(w, C));
}

// Atomic checkpoint: temp file, checked writes, fsync, rename over the old one (format.h).
void write_progress(const std::string& path, const std::string& line, bool durable) {
  commit_file(path, reinterpret_cast<const uint8_t*>(line.data()), int64_t(line.size()), durable);
}

// modification time (ns) of a file the output bytes depend on: part of a checkpoint's key, so a
// checkpoint never resumes over an input that changed since it was written
long long mtime_ns(const std::string& path) {
  struct stat sb;
  if (::stat(path.c_str(), &sb) != 0) return -1;
  return static_cast<long long>(sb.st_mtim.tv_sec) * 1000000000LL + sb.st_mtim.tv_nsec;
}

// fsync every output (the windows were fdatasync'ed; the final size change was not)
void sync_all(const std::vector<Fd>& fds, const std::string& what) {
  for (const Fd& f : fds)
    if (::fsync(f.fd) != 0) throw std::runtime_error("fsync failed on " + what + ": " + std::strerror(errno));
}

std::vector<std::string> read_progress(const std::string& path) {
  std::ifstream in(path);
  std::vector<std::string> tok;
  std::string t;
  while (in >> t) tok.push_back(t);
  return tok;
}

// Host buffer block: `rows` rows of W bytes.
struct Block {
  const HostAlloc* a = nullptr;
  uint8_t* p = nullptr;
  Block(const HostAlloc& al, size_t bytes) : a(&al), p(al.alloc(bytes ? bytes : 1)) {
    if (!p) throw std::runtime_error("host allocation failed");
  }
  ~Block() {
    if (p) a->release(p);
  }
  Block(const Block&) = delete;
};

// Three-stage window pipeline over chunk offsets [start, C): read(w+1) || compute(w) || write(w-1).
// Buffer set w % 3 belongs to window w; write(w) checkpoints after its data is on disk.
template <class Read, class Compute, class Write>
void run_windows(int64_t start, int64_t C, int64_t W, int stop_after, Read read, Compute compute, Write write,
                 StreamReport& rep) {
  const int64_t nw = (C - start + W - 1) / W;
  const int64_t limit = stop_after >= 0 ? std::min<int64_t>(nw, stop_after) : nw;
  if (limit <= 0) return;
  auto win = [&](int64_t w, int64_t& off, int64_t& len) {
    off = start + w * W;
    len = std::min(W, C - off);
  };
  auto do_read = [&](int64_t w) {
    int64_t off, len;
    win(w, off, len);
    const auto t = Clock::now();
    TraceRange tr("stream/read");
    read(int(w % 3), off, len);
    return ms_since(t);
  };
  std::future<double> rd = std::async(std::launch::async, do_read, int64_t(0));
  std::future<double> wr;
  for (int64_t w = 0; w < limit; ++w) {
    rep.ms_read += rd.get();
    if (w + 1 < limit) rd = std::async(std::launch::async, do_read, w + 1);  // set (w+1)%3: write(w-2) joined
    int64_t off, len;
    win(w, off, len);
    const auto t = Clock::now();
    {
      TraceRange tr("stream/compute");
      compute(int(w % 3), off, len);
    }
    rep.ms_compute += ms_since(t);
    if (wr.valid()) rep.ms_write += wr.get();  // write(w-1) + its checkpoint
    wr = std::async(std::launch::async, [&, w, off, len] {
      const auto tw = Clock::now();
      TraceRange tr("stream/write+checkpoint");
      write(int(w % 3), off, len);
      return ms_since(tw);
    });
    ++rep.windows;
  }
  rep.ms_write += wr.get();
}

// rows handled by a small thread team (per-row CRC + pwrite)
template <class F>
void for_rows(int n, F f) {
  const int T = std::min(n, 16);
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t)
    th.emplace_back([&, t] {
      for (int i = t; i < n; i += T) f(i);
    });
  for (int i = 0; i < n; i += T) f(i);
  for (auto& x : th) x.join();
}

std::string join_u32(const std::vector<uint32_t>& v) {
  std::ostringstream s;
  for (auto x : v) s << ' ' << x;
  return s.str();
}

}  // namespace

int64_t stream_window(const StreamOptions& opt, int rows, int64_t C) { return pick_window(opt, rows, C); }

std::string progress_path(const std::string& target) { return target + ".PROGRESS"; }

std::string shard_progress_path(const std::string& target, int64_t lo, int64_t hi) {
  return progress_path(target) + "." + std::to_string(lo) + "-" + std::to_string(hi);
}

namespace {

// The column range [lo, hi) of a call (validated), the checkpoint path and the window.
struct Range {
  int64_t lo = 0, hi = 0, W = 0;
  std::string prog;
};

Range column_range(const StreamOptions& opt, const std::string& target, int rows, int64_t C, int field_w) {
  Range r;
  r.lo = opt.col_lo;
  r.hi = opt.col_hi < 0 ? C : std::min<int64_t>(opt.col_hi, C);
  if (r.lo < 0 || r.lo > r.hi) throw std::invalid_argument("stream codec: bad column range");
  if (field_w == 16 && (r.lo % 2 || r.hi % 2)) throw std::invalid_argument("stream codec: GF(2^16) columns are whole symbols");
  r.W = pick_window(opt, rows, std::max<int64_t>(1, r.hi - r.lo));
  if (field_w == 16) r.W += r.W % 2;  // whole 16-bit symbols per window
  r.prog = opt.shard ? shard_progress_path(target, r.lo, r.hi) : progress_path(target);
  return r;
}

// Checkpoint "<key> <offset> [crc ...]": the offset reached (in [lo, hi]) when the key matches.
bool resume_point(const std::string& prog, const std::string& key, size_t extra, int64_t lo, int64_t hi,
                  int64_t& off, std::vector<std::string>& rest) {
  const auto tok = read_progress(prog);
  std::istringstream ks(key);
  std::vector<std::string> kt;
  for (std::string x; ks >> x;) kt.push_back(x);
  if (tok.size() != kt.size() + 1 + extra || !std::equal(kt.begin(), kt.end(), tok.begin())) return false;
  off = std::stoll(tok[kt.size()]);
  if (off < lo || off > hi) return false;
  rest.assign(tok.begin() + long(kt.size()) + 1, tok.end());
  return true;
}

}  // namespace

StreamReport encode_file_stream(const std::string& file, int k, int p, MatrixKind kind, const GemmFn& gemm,
                                const HostAlloc& alloc, const StreamOptions& opt, bool cpu_meta) {
  const int fw = opt.field_w;
  if (fw != 8 && fw != 16) throw std::invalid_argument("encode: field width must be 8 or 16");
  if (k <= 0 || p < 0 || k + p > max_rows(fw))
    throw std::invalid_argument(fw == 16 ? "encode: need k >= 1, p >= 0, k + p <= 65535 (GF(2^16))"
                                         : "encode: need k >= 1, p >= 0, k + p <= 256");
  if (fw == 16 && cpu_meta) throw std::invalid_argument("encode: the 2-line CPU METADATA has no GF(2^16) form");
  StreamReport rep;
  rep.k = k;
  rep.p = p;
  rep.total_size = file_size(file);
  const int64_t C = std::max<int64_t>(fw == 16 ? 2 : 1, chunk_size(rep.total_size, k, fw));
  rep.chunk_size = C;
  const int n = k + p;
  const Range rg = column_range(opt, file, n, C, fw);
  const int64_t W = rg.W;
  rep.window = W;
  rep.col_lo = rg.lo;
  rep.col_hi = rg.hi;
  auto t = Clock::now();
  gf16w::Mat e16;
  Mat e;
  if (p && fw == 16) {
    e16 = encoding_matrix16(kind, k, p);
    e = pack16(e16);
  } else if (p) {
    e = encoding_matrix(kind, k, p);
  }
  rep.ms_matrix = ms_since(t);

  // resume point (the key names everything the bytes depend on, the column range included)
  std::ostringstream key;
  key << "gfrs-progress 2 encode " << rep.total_size << ' ' << k << ' ' << p << ' ' << int(kind) << ' '
      << int(cpu_meta) << ' ' << C << ' ' << fw << ' ' << rg.lo << ' ' << rg.hi << ' ' << mtime_ns(file);
  int64_t start = rg.lo;
  std::vector<uint32_t> crc(size_t(n), 0);
  if (opt.resume) {
    int64_t off;
    std::vector<std::string> rest;
    if (resume_point(rg.prog, key.str(), size_t(n), rg.lo, rg.hi, off, rest)) {
      bool ok = true;
      for (int i = 0; ok && i < n; ++i) ok = file_at_least(chunk_path(file, i), opt.shard ? C : off);
      if (ok) {
        start = off;
        for (int i = 0; i < n; ++i) crc[size_t(i)] = uint32_t(std::stoul(rest[size_t(i)]));
      }
    }
  }
  rep.resumed_from = start;
  // an older METADATA goes before the first chunk byte changes (a shard's coordinator removes it)
  if (!opt.shard) remove_file(metadata_path(file), opt.durable);

  Fd in = open_or_throw(file, O_RDONLY);
  std::vector<Fd> outs;
  const int oflags = opt.shard ? O_WRONLY : (O_WRONLY | O_CREAT | (start > rg.lo || rg.lo > 0 ? 0 : O_TRUNC));
  for (int i = 0; i < n; ++i) outs.push_back(open_or_throw(chunk_path(file, i), oflags));
  Block buf(alloc, size_t(3) * n * size_t(W));
  auto row = [&](int set, int i) { return buf.p + (size_t(set) * n + size_t(i)) * size_t(W); };

  run_windows(
      start, rg.hi, W, opt.stop_after,
      [&](int set, int64_t off, int64_t len) {
        for_rows(k, [&](int j) { pread_full(in.fd, row(set, j), len, int64_t(j) * C + off); });
      },
      [&](int set, int64_t, int64_t len) {
        if (!p) return;
        std::vector<const uint8_t*> ip(k);
        std::vector<uint8_t*> op(p);
        for (int j = 0; j < k; ++j) ip[j] = row(set, j);
        for (int i = 0; i < p; ++i) op[i] = row(set, k + i);
        gemm(ip, op, e, len, fw);
      },
      [&](int set, int64_t off, int64_t len) {
        for_rows(n, [&](int i) {
          if (!cpu_meta) crc[size_t(i)] = crc32(row(set, i), len, crc[size_t(i)]);
          pwrite_full(outs[size_t(i)].fd, row(set, i), len, off);
          if (opt.durable) ::fdatasync(outs[size_t(i)].fd);
        });
        write_progress(rg.prog, key.str() + ' ' + std::to_string(off + len) + join_u32(crc) + '\n', opt.durable);
      },
      rep);

  const int64_t done = start + int64_t(rep.windows) * W;
  if (done < rg.hi) return rep;  // stopped early (stop_after): the checkpoint says where to resume
  rep.crc = crc;
  if (opt.shard) {
    // The coordinator combines the shards' CRCs and commits the METADATA; this shard's checkpoint
    // (offset = hi, its CRCs) stays until then, so a job that dies before the commit resumes every
    // finished shard at its end instead of re-encoding it (the caller removes it afterwards).
    rep.complete = true;
    return rep;
  }
  if (rg.lo != 0 || rg.hi != C) throw std::invalid_argument("encode: a partial column range needs shard mode");
  if (opt.stop_before_commit) return rep;  // (testing: a crash between the last window and the commit)
  // commit: sized and synced chunks, then the METADATA (atomic), then the checkpoint goes
  for (int i = 0; i < n; ++i)
    if (::ftruncate(outs[size_t(i)].fd, C) != 0) throw std::runtime_error("cannot size chunk file");
  if (opt.durable) sync_all(outs, "chunk file");
  if (fw == 16)
    write_metadata16(metadata_path(file), rep.total_size, p, k, e16, crc);
  else
    write_metadata(metadata_path(file), rep.total_size, p, k, e, !cpu_meta, cpu_meta ? std::vector<uint32_t>{} : crc);
  remove_file(rg.prog, opt.durable);
  rep.complete = true;
  return rep;
}

namespace {

struct Candidates {
  std::vector<int> idx;
  std::vector<std::string> path;
};

Candidates conf_candidates(const std::string& file, const std::string& conf, const Metadata& md) {
  const int k = md.k, n = md.k + md.p;
  const std::vector<std::string> names = read_conf(conf);
  if (int(names.size()) < k)
    throw std::runtime_error("configuration lists " + std::to_string(names.size()) + " chunks, need k = " +
                             std::to_string(k));
  Candidates c;
  std::set<int> seen;
  for (const auto& nm : names) {
    const int idx = chunk_index(nm);
    if (idx < 0 || idx >= n) throw std::runtime_error("bad chunk name in configuration: " + nm);
    if (!seen.insert(idx).second) throw std::runtime_error("duplicate chunk in configuration: " + nm);
    c.idx.push_back(idx);
    c.path.push_back(resolve_chunk(nm, file));
  }
  return c;
}

int64_t stripe_chunk(const Metadata& md) {
  return std::max<int64_t>(md.w == 16 ? 2 : 1, chunk_size(md.total_size, md.k, md.w));
}

// First recoverable k-subset (conf order) of the candidates that exist and pass their CRC; returns
// positions into the candidate list.
std::vector<int> pick_survivors(const Metadata& md, const Candidates& cand, int64_t C, int* rejected,
                                const std::vector<int>* given = nullptr) {
  const int k = md.k;
  const size_t scratch_bytes = size_t(std::min<int64_t>(std::max<int64_t>(C, 1), int64_t(16) << 20));
  // 1 = intact, 0 = missing, short or failing its CRC (*rej counts the CRC failures)
  auto check = [&](int ci, std::vector<uint8_t>& scratch, int* rej) -> bool {
    try {
      const std::string& path = cand.path[size_t(ci)];
      if (!file_at_least(path, md.total_size > 0 ? C : 0)) return false;
      if (md.crc.empty()) return true;
      Fd f(::open(path.c_str(), O_RDONLY | O_CLOEXEC));
      if (f.fd < 0) return false;
      scratch.resize(scratch_bytes);
      uint32_t c = 0;
      for (int64_t off = 0; off < C; off += int64_t(scratch.size())) {
        const int64_t len = std::min<int64_t>(int64_t(scratch.size()), C - off);
        pread_full(f.fd, scratch.data(), len, off);
        c = crc32(scratch.data(), len, c);
      }
      if (c != md.crc[size_t(cand.idx[size_t(ci)])]) {
        ++*rej;
        return false;
      }
      return true;
    } catch (const std::exception&) {
      return false;
    }
  };
  // the first k candidates (all a clean decode needs) are read and checked at once
  const int ncand = int(cand.idx.size());
  const int first = std::min(ncand, k);
  std::vector<signed char> pre(size_t(ncand), -1);
  std::vector<int> rej(size_t(ncand), 0);
  if (given) {  // verdicts known already (a distributed check: combined shard CRCs)
    for (int ci = 0; ci < ncand; ++ci) pre[size_t(ci)] = ci < int(given->size()) && (*given)[size_t(ci)] ? 1 : 0;
  } else {
    parallel_indices(first, verify_threads(), [&](int ci) {
      std::vector<uint8_t> scratch;
      pre[size_t(ci)] = check(ci, scratch, &rej[size_t(ci)]) ? 1 : 0;
    });
  }
  std::vector<uint8_t> scratch;
  auto verified_ok = [&](int ci) -> bool {
    const bool ok = pre[size_t(ci)] >= 0 ? pre[size_t(ci)] == 1 : check(ci, scratch, &rej[size_t(ci)]);
    if (rejected) *rejected += rej[size_t(ci)];
    return ok;
  };
  std::vector<int> verified;
  for (int ci = 0; ci < ncand; ++ci) {
    if (!verified_ok(ci)) continue;
    verified.push_back(ci);
    if (int(verified.size()) < k) continue;
    // recoverable k-subset among the verified chunks, earliest in conf order first
    std::vector<int> pick(k);
    for (int i = 0; i < k; ++i) pick[i] = i;
    const int V = int(verified.size());
    for (long tries = 0; tries < 100000; ++tries) {
      std::vector<int> rr(k);
      for (int i = 0; i < k; ++i) rr[i] = cand.idx[size_t(verified[size_t(pick[i])])];
      if (decode_coefficients(md, rr, nullptr, nullptr)) {
        std::vector<int> chosen(k);
        for (int i = 0; i < k; ++i) chosen[i] = verified[size_t(pick[i])];
        return chosen;
      }
      int i = k - 1;
      while (i >= 0 && pick[i] == V - k + i) --i;
      if (i < 0) break;
      ++pick[i];
      for (int j = i + 1; j < k; ++j) pick[j] = pick[j - 1] + 1;
    }
  }
  if (int(verified.size()) < k)
    throw std::runtime_error("only " + std::to_string(verified.size()) + " intact chunks available, need k = " +
                             std::to_string(k));
  throw std::runtime_error("unrecoverable erasure pattern: the selected rows of the generator are singular");
}

}  // namespace

std::vector<int> choose_survivors(const std::string& file, const std::string& conf, int* rejected) {
  const Metadata md = read_metadata(metadata_path(file));
  const Candidates cand = conf_candidates(file, conf, md);
  const std::vector<int> pos = pick_survivors(md, cand, stripe_chunk(md), rejected);
  std::vector<int> rows;
  for (int ci : pos) rows.push_back(cand.idx[size_t(ci)]);
  return rows;
}

std::vector<ShardCrc> shard_crcs(const std::string& file, const std::string& conf, int64_t lo, int64_t hi, int first,
                                 int count) {
  const Metadata md = read_metadata(metadata_path(file));
  const Candidates cand = conf_candidates(file, conf, md);
  const int64_t C = stripe_chunk(md);
  lo = std::max<int64_t>(0, std::min(lo, C));
  hi = std::max<int64_t>(lo, std::min(hi, C));
  const int ncand = int(cand.idx.size());
  first = std::max(0, std::min(first, ncand));
  const int end = count < 0 ? ncand : std::min(ncand, first + count);
  std::vector<ShardCrc> out(cand.idx.size());
  for (int ci = 0; ci < ncand; ++ci) out[size_t(ci)].index = cand.idx[size_t(ci)];
  parallel_indices(end - first, verify_threads(), [&](int i) {
    const int ci = first + i;
    ShardCrc& r = out[size_t(ci)];
    try {
      const std::string& path = cand.path[size_t(ci)];
      if (!file_at_least(path, md.total_size > 0 ? C : 0)) return;
      Fd f(::open(path.c_str(), O_RDONLY | O_CLOEXEC));
      if (f.fd < 0) return;
      std::vector<uint8_t> scratch(size_t(std::min<int64_t>(std::max<int64_t>(hi - lo, 1), int64_t(16) << 20)));
      uint32_t c = 0;
      for (int64_t off = lo; off < hi; off += int64_t(scratch.size())) {
        const int64_t len = std::min<int64_t>(int64_t(scratch.size()), hi - off);
        pread_full(f.fd, scratch.data(), len, off);
        c = crc32(scratch.data(), len, c);
      }
      r.crc = c;
      r.present = true;
    } catch (const std::exception&) {
      r.present = false;
    }
  });
  return out;
}

std::vector<int> choose_survivors_given(const std::string& file, const std::string& conf,
                                        const std::vector<int>& intact) {
  const Metadata md = read_metadata(metadata_path(file));
  const Candidates cand = conf_candidates(file, conf, md);
  const std::vector<int> pos = pick_survivors(md, cand, stripe_chunk(md), nullptr, &intact);
  std::vector<int> rows;
  for (int ci : pos) rows.push_back(cand.idx[size_t(ci)]);
  return rows;
}

StreamReport decode_file_stream(const std::string& file, const std::string& conf, const std::string& out,
                                const GemmFn& gemm, const HostAlloc& alloc, const StreamOptions& opt) {
  StreamReport rep;
  const Metadata md = read_metadata(metadata_path(file));
  const int k = md.k;
  rep.k = k;
  rep.p = md.p;
  rep.total_size = md.total_size;
  const int64_t C = stripe_chunk(md);
  rep.chunk_size = C;
  const std::string dst = out.empty() ? file : out;
  const Range rg = column_range(opt, dst, 2 * k, C, md.w);
  const int64_t W = rg.W;
  rep.window = W;
  rep.col_lo = rg.lo;
  rep.col_hi = rg.hi;

  // survivors: the coordinator's choice (opt.rows), else the aggressive read over the conf (every
  // candidate streamed through its CRC-32 in windows, so no chunk is ever held whole in memory)
  auto t = Clock::now();
  const Candidates cand = conf_candidates(file, conf, md);
  std::vector<int> rows;
  std::vector<std::string> paths;
  if (!opt.rows.empty()) {
    if (int(opt.rows.size()) != k) throw std::runtime_error("decode: the given survivor list needs k entries");
    for (int r : opt.rows) {
      const auto it = std::find(cand.idx.begin(), cand.idx.end(), r);
      if (it == cand.idx.end()) throw std::runtime_error("decode: survivor chunk " + std::to_string(r) + " is not in the configuration");
      const std::string& path = cand.path[size_t(it - cand.idx.begin())];
      if (!file_at_least(path, md.total_size > 0 ? C : 0)) throw std::runtime_error("decode: chunk missing or short: " + path);
      rows.push_back(r);
      paths.push_back(path);
    }
  } else {
    for (int ci : pick_survivors(md, cand, C, &rep.rejected)) {
      rows.push_back(cand.idx[size_t(ci)]);
      paths.push_back(cand.path[size_t(ci)]);
    }
  }
  std::vector<int> pos_of_native(k, -1);
  for (int i = 0; i < k; ++i)
    if (rows[i] < k) pos_of_native[rows[i]] = i;
  std::vector<int> erased;
  for (int i = 0; i < k; ++i)
    if (pos_of_native[i] < 0) erased.push_back(i);
  rep.erased = int(erased.size());
  rep.rows = rows;
  const int ne = int(erased.size());
  Mat coeff;
  if (!decode_coefficients(md, rows, &erased, &coeff))
    throw std::runtime_error("unrecoverable erasure pattern: the selected rows of the generator are singular");
  rep.ms_matrix = ms_since(t);

  std::ostringstream key;
  key << "gfrs-progress 2 decode " << md.total_size << ' ' << k << ' ' << md.p << ' ' << C << ' ' << md.w << ' '
      << rg.lo << ' ' << rg.hi << ' ' << mtime_ns(metadata_path(file));
  for (int r : rows) key << ' ' << r;
  int64_t start = rg.lo;
  if (opt.resume) {
    int64_t off;
    std::vector<std::string> rest;
    if (resume_point(rg.prog, key.str(), 0, rg.lo, rg.hi, off, rest) && ::access(dst.c_str(), F_OK) == 0) start = off;
  }
  rep.resumed_from = start;

  std::vector<Fd> ins;
  for (int i = 0; i < k; ++i) ins.push_back(open_or_throw(paths[size_t(i)], O_RDONLY));
  const int oflags = opt.shard ? O_WRONLY : (O_WRONLY | O_CREAT | (start > rg.lo || rg.lo > 0 ? 0 : O_TRUNC));
  Fd of = open_or_throw(dst, oflags);
  const int R = k + std::max(ne, 1);
  Block buf(alloc, size_t(3) * R * size_t(W));
  auto row = [&](int set, int i) { return buf.p + (size_t(set) * R + size_t(i)) * size_t(W); };

  run_windows(
      start, rg.hi, W, opt.stop_after,
      [&](int set, int64_t off, int64_t len) {
        for_rows(k, [&](int j) { pread_full(ins[size_t(j)].fd, row(set, j), len, off); });
      },
      [&](int set, int64_t, int64_t len) {
        if (!ne) return;
        std::vector<const uint8_t*> ip(k);
        std::vector<uint8_t*> op(ne);
        for (int j = 0; j < k; ++j) ip[j] = row(set, j);
        for (int e = 0; e < ne; ++e) op[e] = row(set, k + e);
        gemm(ip, op, coeff, len, md.w);
      },
      [&](int set, int64_t off, int64_t len) {
        int e = 0;
        for (int i = 0; i < k; ++i) {
          const uint8_t* src = pos_of_native[i] >= 0 ? row(set, pos_of_native[i]) : row(set, k + e++);
          const int64_t foff = int64_t(i) * C + off;
          const int64_t w = std::min(len, md.total_size - foff);
          if (w > 0) pwrite_full(of.fd, src, w, foff);
        }
        if (opt.durable) ::fdatasync(of.fd);
        write_progress(rg.prog, key.str() + ' ' + std::to_string(off + len) + '\n', opt.durable);
      },
      rep);

  const int64_t done = start + int64_t(rep.windows) * W;
  if (done < rg.hi) return rep;
  if (opt.shard) {  // (the checkpoint stays until the coordinator's final barrier, as for encode)
    rep.complete = true;
    return rep;
  }
  if (rg.lo != 0 || rg.hi != C) throw std::invalid_argument("decode: a partial column range needs shard mode");
  if (opt.stop_before_commit) return rep;
  if (::ftruncate(of.fd, md.total_size) != 0) throw std::runtime_error("cannot size output file " + dst);
  if (opt.durable && ::fsync(of.fd) != 0) throw std::runtime_error("fsync failed on " + dst + ": " + std::strerror(errno));
  remove_file(rg.prog, opt.durable);
  rep.complete = true;
  return rep;
}

}  // namespace gfrs

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

// Atomic checkpoint: write a temp file, fsync it, rename over the old one.
void write_progress(const std::string& path, const std::string& line, bool durable) {
  const std::string tmp = path + ".tmp";
  {
    Fd f = open_or_throw(tmp, O_WRONLY | O_CREAT | O_TRUNC);
    pwrite_full(f.fd, reinterpret_cast<const uint8_t*>(line.data()), int64_t(line.size()), 0);
    if (durable) ::fsync(f.fd);
  }
  if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("cannot write checkpoint " + path);
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

StreamReport encode_file_stream(const std::string& file, int k, int p, MatrixKind kind, const GemmFn& gemm,
                                const HostAlloc& alloc, const StreamOptions& opt, bool cpu_meta) {
  if (k <= 0 || p < 0 || k + p > 256) throw std::invalid_argument("encode: need k >= 1, p >= 0, k + p <= 256");
  StreamReport rep;
  rep.k = k;
  rep.p = p;
  rep.total_size = file_size(file);
  const int64_t C = std::max<int64_t>(1, chunk_size(rep.total_size, k));
  rep.chunk_size = C;
  const int n = k + p;
  const int64_t W = pick_window(opt, n, C);
  rep.window = W;
  auto t = Clock::now();
  const Mat e = p ? encoding_matrix(kind, k, p) : Mat{};
  rep.ms_matrix = ms_since(t);

  // resume point
  const std::string prog = progress_path(file);
  std::ostringstream key;
  key << "gfrs-progress 1 encode " << rep.total_size << ' ' << k << ' ' << p << ' ' << int(kind) << ' '
      << int(cpu_meta) << ' ' << C;
  int64_t start = 0;
  std::vector<uint32_t> crc(size_t(n), 0);
  if (opt.resume) {
    const auto tok = read_progress(prog);
    std::istringstream ks(key.str());
    std::vector<std::string> kt;
    for (std::string x; ks >> x;) kt.push_back(x);
    if (tok.size() == kt.size() + 1 + size_t(n) && std::equal(kt.begin(), kt.end(), tok.begin())) {
      const int64_t off = std::stoll(tok[kt.size()]);
      bool ok = off >= 0 && off <= C;
      for (int i = 0; ok && i < n; ++i) ok = file_at_least(chunk_path(file, i), off);
      if (ok) {
        start = off;
        for (int i = 0; i < n; ++i) crc[size_t(i)] = uint32_t(std::stoul(tok[kt.size() + 1 + size_t(i)]));
      }
    }
  }
  rep.resumed_from = start;

  Fd in = open_or_throw(file, O_RDONLY);
  std::vector<Fd> outs;
  for (int i = 0; i < n; ++i)
    outs.push_back(open_or_throw(chunk_path(file, i), O_WRONLY | O_CREAT | (start ? 0 : O_TRUNC)));
  Block buf(alloc, size_t(3) * n * size_t(W));
  auto row = [&](int set, int i) { return buf.p + (size_t(set) * n + size_t(i)) * size_t(W); };

  run_windows(
      start, C, W, opt.stop_after,
      [&](int set, int64_t off, int64_t len) {
        for_rows(k, [&](int j) { pread_full(in.fd, row(set, j), len, int64_t(j) * C + off); });
      },
      [&](int set, int64_t, int64_t len) {
        if (!p) return;
        std::vector<const uint8_t*> ip(k);
        std::vector<uint8_t*> op(p);
        for (int j = 0; j < k; ++j) ip[j] = row(set, j);
        for (int i = 0; i < p; ++i) op[i] = row(set, k + i);
        gemm(ip, op, e, len, 8);
      },
      [&](int set, int64_t off, int64_t len) {
        for_rows(n, [&](int i) {
          if (!cpu_meta) crc[size_t(i)] = crc32(row(set, i), len, crc[size_t(i)]);
          pwrite_full(outs[size_t(i)].fd, row(set, i), len, off);
          if (opt.durable) ::fdatasync(outs[size_t(i)].fd);
        });
        write_progress(prog, key.str() + ' ' + std::to_string(off + len) + join_u32(crc) + '\n', opt.durable);
      },
      rep);

  const int64_t done = start + int64_t(rep.windows) * W;
  if (done < C) return rep;  // stopped early (stop_after): the checkpoint says where to resume
  for (int i = 0; i < n; ++i)
    if (::ftruncate(outs[size_t(i)].fd, C) != 0) throw std::runtime_error("cannot size chunk file");
  write_metadata(metadata_path(file), rep.total_size, p, k, e, !cpu_meta, cpu_meta ? std::vector<uint32_t>{} : crc);
  std::remove(prog.c_str());
  rep.complete = true;
  return rep;
}

StreamReport decode_file_stream(const std::string& file, const std::string& conf, const std::string& out,
                                const GemmFn& gemm, const HostAlloc& alloc, const StreamOptions& opt) {
  StreamReport rep;
  const Metadata md = read_metadata(metadata_path(file));
  if (md.w != 8)
    throw std::runtime_error("the windowed codec handles GF(2^8) stripes; decode a GF(2^16) stripe without --window");
  const int k = md.k, n = md.k + md.p;
  rep.k = k;
  rep.p = md.p;
  rep.total_size = md.total_size;
  const int64_t C = std::max<int64_t>(1, chunk_size(md.total_size, k));
  rep.chunk_size = C;
  const int64_t W = pick_window(opt, 2 * k, C);
  rep.window = W;

  // candidate chunks in conf order (see decode_file: aggressive read); verification streams each
  // chunk through its CRC-32 in windows, so no chunk is ever held whole in memory
  auto t = Clock::now();
  const std::vector<std::string> names = read_conf(conf);
  if (int(names.size()) < k)
    throw std::runtime_error("configuration lists " + std::to_string(names.size()) + " chunks, need k = " +
                             std::to_string(k));
  std::vector<int> cand_idx;
  std::vector<std::string> cand_path;
  std::set<int> seen;
  for (const auto& nm : names) {
    const int idx = chunk_index(nm);
    if (idx < 0 || idx >= n) throw std::runtime_error("bad chunk name in configuration: " + nm);
    if (!seen.insert(idx).second) throw std::runtime_error("duplicate chunk in configuration: " + nm);
    cand_idx.push_back(idx);
    cand_path.push_back(resolve_chunk(nm, file));
  }
  std::vector<uint8_t> scratch(static_cast<size_t>(std::min<int64_t>(W, int64_t(16) << 20)));
  auto verified_ok = [&](int ci) -> bool {
    const std::string& path = cand_path[size_t(ci)];
    if (!file_at_least(path, md.total_size > 0 ? C : 0)) return false;
    if (md.crc.empty()) return true;
    Fd f(::open(path.c_str(), O_RDONLY | O_CLOEXEC));
    if (f.fd < 0) return false;
    uint32_t c = 0;
    for (int64_t off = 0; off < C; off += int64_t(scratch.size())) {
      const int64_t len = std::min<int64_t>(int64_t(scratch.size()), C - off);
      pread_full(f.fd, scratch.data(), len, off);
      c = crc32(scratch.data(), len, c);
    }
    if (c != md.crc[size_t(cand_idx[size_t(ci)])]) {
      ++rep.rejected;
      return false;
    }
    return true;
  };
  std::vector<int> verified, rows;
  Mat dm;
  bool found = false;
  for (int ci = 0; ci < int(cand_idx.size()) && !found; ++ci) {
    if (!verified_ok(ci)) continue;
    verified.push_back(ci);
    if (int(verified.size()) < k) continue;
    // recoverable k-subset among the verified chunks, earliest in conf order first
    std::vector<int> pick(k);
    for (int i = 0; i < k; ++i) pick[i] = i;
    const int V = int(verified.size());
    for (long tries = 0; tries < 100000; ++tries) {
      std::vector<int> rr(k);
      for (int i = 0; i < k; ++i) rr[i] = cand_idx[size_t(verified[size_t(pick[i])])];
      if (decode_matrix(md.g, k, rr, dm)) {
        rows = rr;
        std::vector<int> chosen(k);
        for (int i = 0; i < k; ++i) chosen[i] = verified[size_t(pick[i])];
        verified = chosen;
        found = true;
        break;
      }
      int i = k - 1;
      while (i >= 0 && pick[i] == V - k + i) --i;
      if (i < 0) break;
      ++pick[i];
      for (int j = i + 1; j < k; ++j) pick[j] = pick[j - 1] + 1;
    }
  }
  if (!found) {
    if (int(verified.size()) < k)
      throw std::runtime_error("only " + std::to_string(verified.size()) + " intact chunks available, need k = " +
                               std::to_string(k));
    throw std::runtime_error("unrecoverable erasure pattern: the selected rows of the generator are singular");
  }
  std::vector<int> pos_of_native(k, -1);
  for (int i = 0; i < k; ++i)
    if (rows[i] < k) pos_of_native[rows[i]] = i;
  std::vector<int> erased;
  for (int i = 0; i < k; ++i)
    if (pos_of_native[i] < 0) erased.push_back(i);
  rep.erased = int(erased.size());
  const int ne = int(erased.size());
  Mat coeff(size_t(ne) * k);
  for (int e = 0; e < ne; ++e) std::memcpy(&coeff[size_t(e) * k], &dm[size_t(erased[e]) * k], size_t(k));
  rep.ms_matrix = ms_since(t);

  const std::string dst = out.empty() ? file : out;
  const std::string prog = progress_path(dst);
  std::ostringstream key;
  key << "gfrs-progress 1 decode " << md.total_size << ' ' << k << ' ' << md.p << ' ' << C;
  for (int r : rows) key << ' ' << r;
  int64_t start = 0;
  if (opt.resume) {
    const auto tok = read_progress(prog);
    std::istringstream ks(key.str());
    std::vector<std::string> kt;
    for (std::string x; ks >> x;) kt.push_back(x);
    if (tok.size() == kt.size() + 1 && std::equal(kt.begin(), kt.end(), tok.begin())) {
      const int64_t off = std::stoll(tok.back());
      if (off >= 0 && off <= C && ::access(dst.c_str(), F_OK) == 0) start = off;
    }
  }
  rep.resumed_from = start;

  std::vector<Fd> ins;
  for (int i = 0; i < k; ++i) ins.push_back(open_or_throw(cand_path[size_t(verified[size_t(i)])], O_RDONLY));
  Fd of = open_or_throw(dst, O_WRONLY | O_CREAT | (start ? 0 : O_TRUNC));
  const int R = k + std::max(ne, 1);
  Block buf(alloc, size_t(3) * R * size_t(W));
  auto row = [&](int set, int i) { return buf.p + (size_t(set) * R + size_t(i)) * size_t(W); };

  run_windows(
      start, C, W, opt.stop_after,
      [&](int set, int64_t off, int64_t len) {
        for_rows(k, [&](int j) { pread_full(ins[size_t(j)].fd, row(set, j), len, off); });
      },
      [&](int set, int64_t, int64_t len) {
        if (!ne) return;
        std::vector<const uint8_t*> ip(k);
        std::vector<uint8_t*> op(ne);
        for (int j = 0; j < k; ++j) ip[j] = row(set, j);
        for (int e = 0; e < ne; ++e) op[e] = row(set, k + e);
        gemm(ip, op, coeff, len, 8);
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
        write_progress(prog, key.str() + ' ' + std::to_string(off + len) + '\n', opt.durable);
      },
      rep);

  const int64_t done = start + int64_t(rep.windows) * W;
  if (done < C) return rep;
  if (::ftruncate(of.fd, md.total_size) != 0) throw std::runtime_error("cannot size output file " + dst);
  std::remove(prog.c_str());
  rep.complete = true;
  return rep;
}

}  // namespace gfrs

// File-level codec (see gfrs/codec_file.h).
#include "gfrs/codec_file.h"

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <set>
#include <thread>
#include <stdexcept>

#include "gfrs/format.h"
#include "gfrs/host_desc.h"
#include "gfrs/trace.h"

namespace gfrs {
namespace {

using Clock = std::chrono::steady_clock;

// Host row pitch of the codec's buffers: chunk rows start on 4 KiB boundaries (an odd C, e.g.
// 2^30 / 10, would otherwise leave every row but the first unaligned), so the zero-copy pipeline
// streams them with 16-byte vector loads and the staged one with 2-D copies.
int64_t row_pitch(int64_t C) { return (C + 4095) / 4096 * 4096; }
double ms_since(Clock::time_point t0) { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); }

struct Buf {
  const HostAlloc* a = nullptr;
  uint8_t* p = nullptr;
  Buf(const HostAlloc& al, size_t n) : a(&al), p(al.alloc(n ? n : 1)) {
    if (!p) throw std::runtime_error("host allocation failed");
  }
  ~Buf() {
    if (p) a->release(p);
  }
  Buf(const Buf&) = delete;
  Buf& operator=(const Buf&) = delete;
};

}  // namespace

// GF(2^16) coding blocks (gfrs/gf65536.h): the reference Vandermonde and Cauchy, and the
// systematic Vandermonde V[k:] . inv(V[:k]) over the points 0..n-1.
gf16w::Mat encoding_matrix16(MatrixKind kind, int k, int p) {
  switch (kind) {
    case MatrixKind::kVandermondeRef: return gf16w::vandermonde_ref(k, p);
    case MatrixKind::kCauchy: return gf16w::cauchy(k, p);
    case MatrixKind::kSysVandermonde: {
      const int n = k + p;
      gf16w::Mat v(size_t(n) * k);
      for (int r = 0; r < n; ++r)
        for (int j = 0; j < k; ++j) v[size_t(r) * k + j] = gf16w::pow(static_cast<uint16_t>(r), unsigned(j));
      gf16w::Mat top(v.begin(), v.begin() + size_t(k) * k), top_inv;
      if (!gf16w::invert(top, k, top_inv)) throw std::runtime_error("sys_vandermonde: singular top block");
      return gf16w::matmul(gf16w::Mat(v.begin() + size_t(k) * k, v.end()), top_inv, p, k, k);
    }
  }
  throw std::invalid_argument("bad matrix kind");
}

namespace {

// Decode system of either field: rows of the inverse of G[rows], packed as GemmFn coefficients
// (one byte per GF(2^8) entry, two per GF(2^16) entry). False when the pattern is singular.
struct Solver {
  const Metadata& md;
  bool solve(const std::vector<int>& rows, const std::vector<int>* erased, Mat* coeff) const {
    const int k = md.k;
    if (md.w == 16) {  // the e x e systematic solve of the erased rows only (gf16w::decode_rows)
      std::vector<int> want;
      if (erased) {
        want = *erased;
      } else {
        std::vector<char> seen(size_t(k), 0);
        for (int r : rows)
          if (r >= 0 && r < k) seen[size_t(r)] = 1;
        for (int i = 0; i < k; ++i)
          if (!seen[size_t(i)]) want.push_back(i);
      }
      gf16w::Mat sel;
      if (!gf16w::decode_rows(md.g16, k, rows, want, sel)) return false;
      if (erased && coeff) *coeff = pack16(sel);
      return true;
    }
    Mat dm;
    if (!decode_matrix(md.g, k, rows, dm)) return false;
    if (erased && coeff) {
      coeff->clear();
      for (int e : *erased) coeff->insert(coeff->end(), dm.begin() + size_t(e) * k, dm.begin() + size_t(e + 1) * k);
    }
    return true;
  }
};

}  // namespace

bool decode_coefficients(const Metadata& md, const std::vector<int>& rows, const std::vector<int>* erased, Mat* coeff) {
  return Solver{md}.solve(rows, erased, coeff);
}

HostAlloc default_host_alloc() {
  return {[](size_t n) -> uint8_t* {
            void* p = nullptr;
            if (posix_memalign(&p, 4096, (n + 4095) / 4096 * 4096) != 0) return nullptr;
            return static_cast<uint8_t*>(p);
          },
          [](uint8_t* p) { std::free(p); }};
}

FileReport encode_file(const std::string& file, int k, int p, MatrixKind kind, const GemmFn& gemm,
                       const HostAlloc& alloc, bool cpu_meta, int field_w) {
  if (field_w != 8 && field_w != 16) throw std::invalid_argument("encode: field width must be 8 or 16");
  if (k <= 0 || p < 0 || k + p > max_rows(field_w))
    throw std::invalid_argument(field_w == 16 ? "encode: need k >= 1, p >= 0, k + p <= 65535 (GF(2^16))"
                                              : "encode: need k >= 1, p >= 0, k + p <= 256");
  if (field_w == 16 && cpu_meta) throw std::invalid_argument("encode: the 2-line CPU METADATA has no GF(2^16) form");
  FileReport r;
  r.k = k;
  r.p = p;
  auto t = Clock::now();
  r.total_size = file_size(file);
  r.chunk_size = std::max<int64_t>(field_w == 16 ? 2 : 1, chunk_size(r.total_size, k, field_w));
  const int64_t C = r.chunk_size;
  const int64_t P = row_pitch(C);
  std::unique_ptr<Buf> data_b, parity_b;
  {
    TraceRange tr("encode/alloc");
    data_b = std::make_unique<Buf>(alloc, size_t(k) * P);
    parity_b = std::make_unique<Buf>(alloc, size_t(std::max(p, 1)) * P);
  }
  Buf& data = *data_b;
  Buf& parity = *parity_b;
  r.ms_alloc = ms_since(t);
  t = Clock::now();
  {
    TraceRange tr("encode/read");
    for (int j = 0; j < k; ++j) read_into(file, int64_t(j) * C, data.p + size_t(j) * P, C);
  }  // one read per chunk row; tail zero-padded
  r.ms_read = ms_since(t);

  t = Clock::now();
  gf16w::Mat e16;
  Mat e;
  if (p && field_w == 16) {
    e16 = encoding_matrix16(kind, k, p);
    e = pack16(e16);
  } else if (p) {
    e = encoding_matrix(kind, k, p);
  }
  r.ms_matrix = ms_since(t);

  t = Clock::now();
  if (p) {
    TraceRange tr("encode/gemm");
    std::vector<const uint8_t*> in(k);
    std::vector<uint8_t*> out(p);
    for (int j = 0; j < k; ++j) in[j] = data.p + size_t(j) * P;
    for (int i = 0; i < p; ++i) out[i] = parity.p + size_t(i) * P;
    gemm(in, out, e, C, field_w);
  }
  r.ms_compute = ms_since(t);

  t = Clock::now();
  TraceRange tr_write("encode/crc+write");
  std::vector<uint32_t> crc;
  if (!cpu_meta) {  // per-chunk CRC-32 (METADATA extension): lets decode reject corrupted chunks
    crc.resize(size_t(k + p));
    std::vector<std::thread> th;
    for (int i = 0; i < k + p; ++i)
      th.emplace_back([&, i] {
        const uint8_t* row = i < k ? data.p + size_t(i) * P : parity.p + size_t(i - k) * P;
        crc[size_t(i)] = crc32(row, C);
      });
    for (auto& x : th) x.join();
  }
  // commit order: an older METADATA goes first, then the chunks, then the new METADATA (atomic) — a
  // failure anywhere (ENOSPC at a chunk, at the METADATA) leaves no METADATA claiming the stripe
  remove_file(metadata_path(file));
  for (int i = 0; i < k; ++i) write_from(chunk_path(file, i), data.p + size_t(i) * P, C);
  for (int i = 0; i < p; ++i) write_from(chunk_path(file, k + i), parity.p + size_t(i) * P, C);
  if (field_w == 16)
    write_metadata16(metadata_path(file), r.total_size, p, k, e16, crc);
  else
    write_metadata(metadata_path(file), r.total_size, p, k, e, !cpu_meta, crc);
  r.ms_write = ms_since(t);
  return r;
}

FileReport decode_file(const std::string& file, const std::string& conf, const std::string& out,
                       const GemmFn& gemm, const HostAlloc& alloc) {
  FileReport r;
  auto t = Clock::now();
  const Metadata md = read_metadata(metadata_path(file));
  const int k = md.k, n = md.k + md.p;
  r.k = k;
  r.p = md.p;
  r.total_size = md.total_size;
  r.chunk_size = std::max<int64_t>(md.w == 16 ? 2 : 1, chunk_size(md.total_size, k, md.w));
  const int64_t C = r.chunk_size;
  const int64_t P = row_pitch(C);
  const Solver solver{md};

  // The reference uses exactly the first k names (src/decode.cu:302-318). Here the conf may list
  // more: chunks that are missing or fail their METADATA CRC-32 are skipped, and the first
  // recoverable k-subset (in conf order) is used — the "aggressive read" the reference's design
  // notes list as future work (doc/design.tex:529).
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
  double ms_meta = ms_since(t);
  t = Clock::now();
  std::unique_ptr<Buf> surv_b;
  {
    TraceRange tr("decode/alloc");
    surv_b = std::make_unique<Buf>(alloc, size_t(k) * P);
  }
  Buf& surv = *surv_b;
  r.ms_alloc = ms_since(t);
  t = Clock::now();
  std::vector<int> rows;
  std::vector<std::vector<uint8_t>> spare;  // verified chunks beyond the first k (rarely needed)
  auto row_ok = [&](int ci, uint8_t* dst) -> bool {
    try {
      if (file_size(cand_path[size_t(ci)]) < C && md.total_size > 0) return false;
      read_into(cand_path[size_t(ci)], 0, dst, C);
    } catch (const std::exception&) {
      return false;  // missing chunk
    }
    if (!md.crc.empty() && crc32(dst, C) != md.crc[size_t(cand_idx[size_t(ci)])]) {
      ++r.rejected;
      return false;
    }
    return true;
  };
  // fill k slots in conf order, then search for a recoverable subset among the verified chunks.
  // The first k candidates (all a clean decode needs) are read into slots 0..k-1 and checked at
  // once; a failed one leaves a gap that the verified rows after it close by moving down.
  const int first = std::min(int(cand_idx.size()), k);
  std::vector<signed char> pre(size_t(first), 0);
  std::vector<int> rej(size_t(first), 0);
  {
    const int r0 = r.rejected;
    parallel_indices(first, verify_threads(), [&](int ci) {
      try {
        if (file_size(cand_path[size_t(ci)]) < C && md.total_size > 0) return;
        read_into(cand_path[size_t(ci)], 0, surv.p + size_t(ci) * P, C);
      } catch (const std::exception&) {
        return;  // missing chunk
      }
      if (!md.crc.empty() && crc32(surv.p + size_t(ci) * P, C) != md.crc[size_t(cand_idx[size_t(ci)])]) {
        rej[size_t(ci)] = 1;
        return;
      }
      pre[size_t(ci)] = 1;
    });
    r.rejected = r0;
    for (int ci = 0; ci < first; ++ci) r.rejected += rej[size_t(ci)];
  }
  std::vector<int> verified;
  for (int ci = 0; ci < first; ++ci) {
    if (!pre[size_t(ci)]) continue;
    const size_t slot = verified.size();
    if (slot != size_t(ci)) std::memcpy(surv.p + slot * P, surv.p + size_t(ci) * P, size_t(C));
    verified.push_back(ci);
  }
  for (int ci = first; ci < int(cand_idx.size()); ++ci) {
    if (int(verified.size()) < k) {
      if (row_ok(ci, surv.p + size_t(verified.size()) * P)) verified.push_back(ci);
    } else {
      std::vector<uint8_t> tmp(static_cast<size_t>(C));
      if (row_ok(ci, tmp.data())) {
        verified.push_back(ci);
        spare.push_back(std::move(tmp));
      }
    }
  }
  if (int(verified.size()) < k)
    throw std::runtime_error("only " + std::to_string(verified.size()) + " intact chunks available, need k = " +
                             std::to_string(k));
  std::vector<int> pick(k);
  for (int i = 0; i < k; ++i) pick[i] = i;  // positions into `verified`
  auto rows_of = [&](const std::vector<int>& pk) {
    std::vector<int> rr(k);
    for (int i = 0; i < k; ++i) rr[i] = cand_idx[size_t(verified[size_t(pk[i])])];
    return rr;
  };
  bool found = solver.solve(rows_of(pick), nullptr, nullptr);
  for (long tries = 0; !found && tries < 100000; ++tries) {  // next k-combination of the verified set
    int i = k - 1;
    const int V = int(verified.size());
    while (i >= 0 && pick[i] == V - k + i) --i;
    if (i < 0) break;
    ++pick[i];
    for (int j = i + 1; j < k; ++j) pick[j] = pick[j - 1] + 1;
    found = solver.solve(rows_of(pick), nullptr, nullptr);
  }
  if (!found)
    throw std::runtime_error("unrecoverable erasure pattern: the selected rows of the generator are singular");
  // gather the chosen rows into the first k slots of `surv` (slot order = pick order)
  for (int i = 0; i < k; ++i) {
    const int pos = pick[i];
    if (pos == i) continue;
    const uint8_t* src = pos < k ? surv.p + size_t(pos) * P : spare[size_t(pos - k)].data();
    std::memcpy(surv.p + size_t(i) * P, src, size_t(C));  // pick is increasing: slot i <= pos, no clobber of later picks
  }
  rows = rows_of(pick);
  r.ms_read = ms_meta + ms_since(t);

  t = Clock::now();
  // survivors that are natives pass through; only erased natives are reconstructed
  std::vector<int> pos_of_native(k, -1);
  for (int i = 0; i < k; ++i)
    if (rows[i] < k) pos_of_native[rows[i]] = i;
  std::vector<int> erased;
  for (int i = 0; i < k; ++i)
    if (pos_of_native[i] < 0) erased.push_back(i);
  Mat coeff;  // the erased natives' rows of the inverse (packed for the field)
  if (!solver.solve(rows, &erased, &coeff))
    throw std::runtime_error("unrecoverable erasure pattern: the selected rows of the generator are singular");
  r.erased = int(erased.size());
  r.ms_matrix = ms_since(t);
  // (the output rows are allocated outside the timed GEMM region and outside the matrix time, like
  // encode's parity buffer: a pinned hipHostMalloc of ~GBs takes tens of ms)
  t = Clock::now();
  Buf rec(alloc, size_t(std::max<size_t>(erased.size(), 1)) * P);
  r.ms_alloc += ms_since(t);

  t = Clock::now();
  if (!erased.empty()) {
    TraceRange tr("decode/gemm");
    std::vector<const uint8_t*> in(k);
    std::vector<uint8_t*> o(erased.size());
    for (int j = 0; j < k; ++j) in[j] = surv.p + size_t(j) * P;
    for (size_t e = 0; e < erased.size(); ++e) o[e] = rec.p + e * P;
    gemm(in, o, coeff, C, md.w);
  }
  r.ms_compute = ms_since(t);

  t = Clock::now();
  const std::string dst = out.empty() ? file : out;
  // the decoded file is written next to its target and renamed over it (a failed write, e.g. ENOSPC,
  // leaves the target as it was; decoding in place over the input file never truncates it first).
  // Not fsync'ed: the reference's decode writes without a sync too (src/decode.cu:410-427); the
  // windowed codec is the durable path (--window).
  std::vector<Piece> pieces;
  int64_t left = md.total_size;
  size_t e_idx = 0;
  for (int i = 0; i < k && left > 0; ++i) {
    const uint8_t* row = pos_of_native[i] >= 0 ? surv.p + size_t(pos_of_native[i]) * P : rec.p + (e_idx++) * P;
    const int64_t w = std::min(C, left);
    pieces.push_back({row, w});
    left -= w;
  }
  commit_file(dst, pieces, false);
  r.ms_write = ms_since(t);
  return r;
}

std::vector<std::string> worst_case_conf(const std::string& file, int n, int k) {
  std::vector<std::string> names;
  for (int i = n - k; i < n; ++i) names.push_back(chunk_path(file, i));
  return names;
}

}  // namespace gfrs

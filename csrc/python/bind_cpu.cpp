// _cpu extension: CPU reference codec, GF(2^8) scalar ops, formats, file-level codec.
#include <cstring>

#include "bind_common.h"
#include "gfrs/cpu_codec.h"
#include "gfrs/format.h"
#include "gfrs/host_desc.h"

PYBIND11_MODULE(_cpu, m) {
  using namespace gfrs;
  using namespace gfrs_py;
  m.doc() = "gpu_rscode_amd CPU reference codec (C++)";
  bind_common(m);

  m.def("tables", [] {
    py::dict d;
    d["exp"] = py::bytes(reinterpret_cast<const char*>(kTables.exp), kExpLen);
    d["log"] = std::vector<int>(kTables.log, kTables.log + 256);
    d["inv"] = py::bytes(reinterpret_cast<const char*>(kTables.inv), 256);
    return d;
  });
  m.def("mul", [](int a, int b) { return int(mul(uint8_t(a), uint8_t(b))); });
  m.def("div", [](int a, int b) { return int(div(uint8_t(a), uint8_t(b))); });
  m.def("pow_ref", [](int a, unsigned e) { return int(pow_ref(uint8_t(a), e)); });
  m.def("mul_strategy", [](const std::string& s, int a, int b) { return int(cpu_mul(parse_cpu_mul(s), uint8_t(a), uint8_t(b))); });
  m.def(
      "gemm",
      [](const std::vector<uint64_t>& in, const std::vector<uint64_t>& out, const py::bytes& coeff, int64_t ncols,
         const std::string& strategy, int threads) {
        const Mat c = to_mat(coeff);
        const CpuMul s = parse_cpu_mul(strategy);
        auto ip = ptrs<const uint8_t*>(in);
        auto op = ptrs<uint8_t*>(out);
        py::gil_scoped_release nogil;
        cpu_gemm(ip, op, c, ncols, s, threads);
      },
      py::arg("in_ptrs"), py::arg("out_ptrs"), py::arg("coeff"), py::arg("ncols"), py::arg("strategy") = "simd",
      py::arg("threads") = 1);

  m.def(
      "gemm16",
      [](const std::vector<uint64_t>& in, const std::vector<uint64_t>& out, const std::vector<int>& coeff,
         int64_t ncols, int threads) {
        const gf16w::Mat c(coeff.begin(), coeff.end());
        auto ip = ptrs<const uint8_t*>(in);
        auto op = ptrs<uint8_t*>(out);
        py::gil_scoped_release nogil;
        cpu_gemm16(ip, op, c, ncols, threads);
      },
      py::arg("in_ptrs"), py::arg("out_ptrs"), py::arg("coeff"), py::arg("ncols"), py::arg("threads") = 1);
  // GF(2^16) host linear algebra (gfrs/gf65536.h): the decode system of a w = 16 code
  m.def("gf16_mul", [](int a, int b) { return int(gf16w::mul(uint16_t(a), uint16_t(b))); });
  m.def("gf16_invert", [](const std::vector<int>& a, int n) {
    if (n <= 0 || a.size() != size_t(n) * size_t(n)) throw py::value_error("gf16_invert: need n * n entries");
    for (int v : a)
      if (v < 0 || v > 0xFFFF) throw py::value_error("gf16_invert: entries are 16-bit symbols");
    gf16w::Mat out;
    if (!gf16w::invert(gf16w::Mat(a.begin(), a.end()), n, out)) throw py::value_error("singular matrix");
    return std::vector<int>(out.begin(), out.end());
  });
  // rows `want` of inv(G[rows]) (gfrs/gf65536.h decode_rows: the e x e systematic solve); G and
  // the result as little-endian uint16 bytes (no per-element Python objects: k = 300 is 90 k entries)
  m.def("gf16_decode_rows", [](const py::bytes& g, int k, const std::vector<int>& rows, const std::vector<int>& want) {
    const std::string gs = g;
    if (k <= 0 || gs.size() % (2 * size_t(k)) != 0) throw py::value_error("G must be n x k uint16");
    const size_t n = gs.size() / (2 * size_t(k));
    for (int r : rows)
      if (r < 0 || size_t(r) >= n) throw py::value_error("chunk id out of range");
    gf16w::Mat gm(n * size_t(k));
    std::memcpy(gm.data(), gs.data(), gs.size());
    gf16w::Mat out;
    bool ok;
    {
      py::gil_scoped_release nogil;
      ok = gf16w::decode_rows(gm, k, rows, want, out);
    }
    if (!ok) throw py::value_error("singular matrix");
    return py::bytes(reinterpret_cast<const char*>(out.data()), out.size() * 2);
  });
  m.def("gf16_perm_quad", [](int c) {
    const auto q = gf16w::perm_quad(uint16_t(c));
    std::vector<uint32_t> w;
    for (const auto& t : q) w.insert(w.end(), t.w, t.w + kPermStride);
    return w;
  });

  auto gemm_fn = [](const std::string& strategy, int threads) -> GemmFn {
    const CpuMul s = parse_cpu_mul(strategy);
    return [s, threads](const std::vector<const uint8_t*>& in, const std::vector<uint8_t*>& out, const Mat& coeff,
                        int64_t ncols, int field_w) {
      if (field_w == 16)
        cpu_gemm16(in, out, unpack16(coeff), ncols, threads);
      else
        cpu_gemm(in, out, coeff, ncols, s, threads);
    };
  };
  m.def(
      "encode_file",
      [gemm_fn](const std::string& file, int k, int p, const std::string& matrix, bool cpu_meta,
                const std::string& strategy, int threads, int field_w) {
        const GemmFn g = gemm_fn(strategy, threads);
        FileReport r;
        {
          py::gil_scoped_release nogil;
          r = encode_file(file, k, p, parse_matrix_kind(matrix), g, default_host_alloc(), cpu_meta, field_w);
        }
        return report(r);
      },
      py::arg("file"), py::arg("k"), py::arg("p"), py::arg("matrix") = "vandermonde", py::arg("cpu_meta") = false,
      py::arg("strategy") = "simd", py::arg("threads") = 1, py::arg("field_w") = 8);
  m.def(
      "decode_file",
      [gemm_fn](const std::string& file, const std::string& conf, const std::string& out, const std::string& strategy,
                int threads) {
        const GemmFn g = gemm_fn(strategy, threads);
        FileReport r;
        {
          py::gil_scoped_release nogil;
          r = decode_file(file, conf, out, g, default_host_alloc());
        }
        return report(r);
      },
      py::arg("file"), py::arg("conf"), py::arg("out") = "", py::arg("strategy") = "simd", py::arg("threads") = 1);

  m.def(
      "encode_file_stream",
      [gemm_fn](const std::string& file, int k, int p, const std::string& matrix, bool cpu_meta,
                const std::string& strategy, int threads, int64_t window, bool resume, bool durable, int stop_after, bool stop_before_commit,
                int field_w, int64_t col_lo, int64_t col_hi, bool shard) {
        const GemmFn g = gemm_fn(strategy, threads);
        StreamReport r;
        {
          py::gil_scoped_release nogil;
          StreamOptions so = stream_options(window, resume, durable, stop_after, field_w, col_lo, col_hi, shard);
          so.stop_before_commit = stop_before_commit;
          r = encode_file_stream(file, k, p, parse_matrix_kind(matrix), g, default_host_alloc(), so, cpu_meta);
        }
        return stream_report(r);
      },
      py::arg("file"), py::arg("k"), py::arg("p"), py::arg("matrix") = "vandermonde", py::arg("cpu_meta") = false,
      py::arg("strategy") = "simd", py::arg("threads") = 1, py::arg("window") = 0, py::arg("resume") = true,
      py::arg("durable") = true, py::arg("stop_after") = -1, py::arg("stop_before_commit") = false, py::arg("field_w") = 8, py::arg("col_lo") = 0,
      py::arg("col_hi") = -1, py::arg("shard") = false);
  m.def(
      "decode_file_stream",
      [gemm_fn](const std::string& file, const std::string& conf, const std::string& out, const std::string& strategy,
                int threads, int64_t window, bool resume, bool durable, int stop_after, bool stop_before_commit, int64_t col_lo, int64_t col_hi,
                bool shard, const std::vector<int>& rows) {
        const GemmFn g = gemm_fn(strategy, threads);
        StreamReport r;
        {
          py::gil_scoped_release nogil;
          StreamOptions so = stream_options(window, resume, durable, stop_after, 8, col_lo, col_hi, shard, rows);
          so.stop_before_commit = stop_before_commit;
          r = decode_file_stream(file, conf, out, g, default_host_alloc(), so);
        }
        return stream_report(r);
      },
      py::arg("file"), py::arg("conf"), py::arg("out") = "", py::arg("strategy") = "simd", py::arg("threads") = 1,
      py::arg("window") = 0, py::arg("resume") = true, py::arg("durable") = true, py::arg("stop_after") = -1, py::arg("stop_before_commit") = false,
      py::arg("col_lo") = 0, py::arg("col_hi") = -1, py::arg("shard") = false, py::arg("rows") = std::vector<int>{});
  m.def("progress_path", &progress_path);
  m.def("shard_progress_path", &shard_progress_path, py::arg("target"), py::arg("lo"), py::arg("hi"));
  m.def("commit_file", [](const std::string& path, const py::bytes& data, bool durable) {
    const std::string s = data;
    py::gil_scoped_release nogil;
    commit_file(path, reinterpret_cast<const uint8_t*>(s.data()), int64_t(s.size()), durable);
  }, py::arg("path"), py::arg("data"), py::arg("durable") = true,
     "write `data` to path.gfrs-tmp, fsync, rename over `path`, fsync the directory (errors raise)");
  m.def("remove_file", [](const std::string& path, bool durable) { remove_file(path, durable); }, py::arg("path"),
        py::arg("durable") = true);
  m.def("choose_survivors", [](const std::string& file, const std::string& conf) {
    int rejected = 0;
    std::vector<int> rows;
    {
      py::gil_scoped_release nogil;
      rows = choose_survivors(file, conf, &rejected);
    }
    return py::make_tuple(rows, rejected);
  });
  m.def("crc32", [](const py::bytes& b, uint32_t crc) {
    const std::string s = b;
    return crc32(reinterpret_cast<const uint8_t*>(s.data()), int64_t(s.size()), crc);
  }, py::arg("data"), py::arg("crc") = 0);
  m.def("crc32_combine", &crc32_combine);
  m.def(
      "shard_crcs",
      [](const std::string& file, const std::string& conf, int64_t lo, int64_t hi, int first, int count) {
        std::vector<ShardCrc> r;
        {
          py::gil_scoped_release nogil;
          r = shard_crcs(file, conf, lo, hi, first, count);
        }
        py::list out;
        for (const auto& x : r) out.append(py::make_tuple(x.index, x.present, x.crc));
        return out;
      },
      py::arg("file"), py::arg("conf"), py::arg("lo"), py::arg("hi"), py::arg("first") = 0, py::arg("count") = -1,
      "One rank's part of a split survivor check: (chunk index, present, CRC-32 of bytes [lo, hi)) per conf "
      "candidate; candidates [first, first + count) only (count < 0: to the end) are read, the others come back "
      "as (index, False, 0)");
  m.def(
      "choose_survivors_given",
      [](const std::string& file, const std::string& conf, const std::vector<int>& intact) {
        py::gil_scoped_release nogil;
        return choose_survivors_given(file, conf, intact);
      },
      py::arg("file"), py::arg("conf"), py::arg("intact"),
      "The decode survivors (chunk indices) given every conf candidate's verdict (1 = intact)");

  m.def("chunk_path", &chunk_path);
  m.def("chunk_index", &chunk_index);
  m.def("metadata_path", &metadata_path);
  m.def("read_conf", &read_conf);
  m.def("write_conf", &write_conf);
  m.def("worst_case_conf", &worst_case_conf);
  m.def("write_metadata", [](const std::string& path, int64_t total, int p, int k, const py::bytes& e, bool full) {
    write_metadata(path, total, p, k, to_mat(e), full);
  });
  m.def("read_metadata", [](const std::string& path) {
    const Metadata md = read_metadata(path);
    py::dict d;
    d["total_size"] = md.total_size;
    d["p"] = md.p;
    d["k"] = md.k;
    d["w"] = md.w;
    d["g"] = md.w == 16 ? py::object(py::cast(std::vector<int>(md.g16.begin(), md.g16.end()))) : py::object(from_mat(md.g));
    d["has_matrix"] = md.has_matrix;
    return d;
  });
}

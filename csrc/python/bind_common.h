// pybind11 helpers shared by the CPU (_cpu) and HIP (_hip) extension modules.
#pragma once

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <string>
#include <vector>

#include "gfrs/codec_file.h"
#include "gfrs/stream_codec.h"
#include "gfrs/trace.h"
#include "gfrs/host_desc.h"
#include "gfrs/matrix.h"

namespace py = pybind11;

namespace gfrs_py {

inline gfrs::Mat to_mat(const py::bytes& b) {
  const std::string s = b;
  return gfrs::Mat(s.begin(), s.end());
}
inline py::bytes from_mat(const gfrs::Mat& m) {
  return py::bytes(reinterpret_cast<const char*>(m.data()), m.size());
}

template <typename T>
std::vector<T> ptrs(const std::vector<uint64_t>& v) {
  std::vector<T> out(v.size());
  for (size_t i = 0; i < v.size(); ++i) out[i] = reinterpret_cast<T>(v[i]);
  return out;
}

inline py::dict report(const gfrs::FileReport& r) {
  py::dict d;
  d["total_size"] = r.total_size;
  d["chunk_size"] = r.chunk_size;
  d["k"] = r.k;
  d["p"] = r.p;
  d["erased"] = r.erased;
  d["rejected"] = r.rejected;
  d["ms_alloc"] = r.ms_alloc;
  d["ms_read"] = r.ms_read;
  d["ms_matrix"] = r.ms_matrix;
  d["ms_compute"] = r.ms_compute;
  d["ms_write"] = r.ms_write;
  return d;
}

inline py::dict stream_report(const gfrs::StreamReport& r) {
  py::dict d = report(r);
  d["window"] = r.window;
  d["windows"] = r.windows;
  d["resumed_from"] = r.resumed_from;
  d["complete"] = r.complete;
  d["col_lo"] = r.col_lo;
  d["col_hi"] = r.col_hi;
  d["crc"] = r.crc;
  d["rows"] = r.rows;
  return d;
}

inline gfrs::StreamOptions stream_options(int64_t window, bool resume, bool durable, int stop_after, int field_w = 8,
                                          int64_t col_lo = 0, int64_t col_hi = -1, bool shard = false,
                                          const std::vector<int>& rows = {}) {
  gfrs::StreamOptions o;
  o.window = window;
  o.resume = resume;
  o.durable = durable;
  o.stop_after = stop_after;
  o.field_w = field_w;
  o.col_lo = col_lo;
  o.col_hi = col_hi;
  o.shard = shard;
  o.rows = rows;
  return o;
}

// Bindings common to both modules: descriptors and matrix algebra.
inline void bind_common(py::module_& m) {
  m.def("roctx_available", &gfrs::Roctx::available);
  m.def("trace_mark", [](const std::string& s) { gfrs::trace_mark(s.c_str()); });
  m.def("trace_push", [](const std::string& s) {
    if (gfrs::Roctx::get().push) gfrs::Roctx::get().push(s.c_str());
  });
  m.def("trace_pop", [] {
    if (gfrs::Roctx::get().pop) gfrs::Roctx::get().pop();
  });
  m.def("pad_m", &gfrs::pad_m);
  m.def("tile_for", &gfrs::tile_for);
  m.def("desc_layout", [](int k, int m_pad, int batch) {
    const gfrs::DescLayout l = gfrs::desc_layout(k, m_pad, batch);
    py::dict d;
    d["in_off"] = l.in_off;
    d["copy_off"] = l.copy_off;
    d["out_off"] = l.out_off;
    d["tab_off"] = l.tab_off;
    d["bytes"] = l.bytes;
    return d;
  }, py::arg("k"), py::arg("m_pad"), py::arg("batch") = 1);
  m.def("desc_layout16", [](int k, int m_pad, int batch) {
    const gfrs::DescLayout l = gfrs::desc_layout16(k, m_pad, batch);
    py::dict d;
    d["in_off"] = l.in_off;
    d["copy_off"] = l.copy_off;
    d["out_off"] = l.out_off;
    d["tab_off"] = l.tab_off;
    d["bytes"] = l.bytes;
    return d;
  }, py::arg("k"), py::arg("m_pad"), py::arg("batch") = 1);
  m.def(
      "build_desc",
      [](int k, int mm, const std::vector<uint64_t>& in, const std::vector<uint64_t>& copy,
         const std::vector<uint64_t>& out, const py::object& coeff) {
        gfrs::Mat c;
        if (!coeff.is_none()) c = to_mat(coeff.cast<py::bytes>());
        const std::vector<uint8_t> d = gfrs::build_desc(k, mm, in, copy, out, c);
        return py::bytes(reinterpret_cast<const char*>(d.data()), d.size());
      },
      py::arg("k"), py::arg("m"), py::arg("in_ptrs"), py::arg("copy_ptrs"), py::arg("out_ptrs"),
      py::arg("coeff") = py::none());
  m.def("encoding_matrix", [](const std::string& kind, int k, int p) {
    return from_mat(gfrs::encoding_matrix(gfrs::parse_matrix_kind(kind), k, p));
  });
  m.def("invert", [](const py::bytes& a, int n) -> py::object {
    gfrs::Mat out;
    if (!gfrs::invert(to_mat(a), n, out)) return py::none();
    return from_mat(out);
  });
  m.def("decode_matrix", [](const py::bytes& g, int k, const std::vector<int>& rows) -> py::object {
    gfrs::Mat out;
    if (!gfrs::decode_matrix(to_mat(g), k, rows, out)) return py::none();
    return from_mat(out);
  });
  m.def("perm_table", [](int c) {
    const gfrs::PermTable t = gfrs::perm_for_coeff(uint8_t(c));
    return std::vector<uint32_t>(t.w, t.w + gfrs::kPermStride);
  });
  m.def("perm_apply", [](int c, int x) { return int(gfrs::perm_apply(gfrs::perm_for_coeff(uint8_t(c)), uint8_t(x))); });
}

}  // namespace gfrs_py

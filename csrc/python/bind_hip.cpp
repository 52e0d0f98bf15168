// _hip extension: gfx950 kernels and the device runtime. Device pointers and hipStream_t are passed
// as integers (torch tensors' data_ptr() and torch.cuda.current_stream().cuda_stream), so the
// extension has no libtorch build dependency and shares the process' single HIP runtime.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

#include <stdexcept>

#include "bind_common.h"
#include "gfrs/async_prepare.h"
#include "gfrs/kernels.h"
#include "gfrs/host_alloc.h"
#include "gfrs/pipeline.h"

namespace {

// A device setup running on a helper thread (gfrs/async_prepare.h), handed to a later file-codec
// call: `--dist` starts it before its file creation / survivor choice so it overlaps them.
struct PrepareHandle {
  std::unique_ptr<gfrs::AsyncPrepare> prep;
};

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
hipStream_t as_stream(uint64_t s) { return reinterpret_cast<hipStream_t>(s); }

py::dict stats_dict(const gfrs::PipelineStats& s) {
  py::dict d;
  d["ms_setup"] = s.ms_setup;
  d["ms_stream"] = s.ms_stream;
  d["ms_teardown"] = s.ms_teardown;
  d["ms_total"] = s.ms_total;
  d["bytes_h2d"] = s.bytes_h2d;
  d["bytes_d2h"] = s.bytes_d2h;
  d["slices"] = s.slices;
  d["lanes"] = s.lanes;
  d["zero_copy"] = s.zero_copy;
  d["zero_copy_refused"] = std::string(gfrs::zc_fallback_name(s.zc_fallback));
  return d;
}

gfrs::PipelineOptions pipeline_options(int streams, int64_t slice, int max_blocks) {
  gfrs::PipelineOptions opt;
  opt.streams = streams;
  opt.slice_bytes = slice;
  opt.max_blocks = max_blocks;
  return opt;
}

// Pinned host buffers: huge-page anonymous memory + hipHostRegister (gfrs/host_alloc.h, ~25x
// cheaper than hipHostMalloc); GFRS_HOST_ALLOC=hipHostMalloc selects the plain allocator.
gfrs::HostAlloc pinned_alloc() {
  const char* env = std::getenv("GFRS_HOST_ALLOC");
  if (!env || std::string(env) != "hipHostMalloc") return gfrs::thp_pinned_host_alloc();
  return {[](size_t n) -> uint8_t* {
            void* p = nullptr;
            if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) return nullptr;
            return static_cast<uint8_t*>(p);
          },
          [](uint8_t* p) { (void)hipHostFree(p); }};
}

}  // namespace

PYBIND11_MODULE(_hip, m) {
  using namespace gfrs;
  using namespace gfrs_py;
  m.doc() = "gpu_rscode_amd gfx950 HIP kernels and runtime";
  bind_common(m);

  m.def("device_count", [] {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });
  m.def(
      "gemm",
      [](uint64_t desc, int k, int m_pad, int64_t col0, int64_t ncols, bool bytewise, int max_blocks, uint64_t stream,
         bool copies) {
        check(launch_gf_gemm(reinterpret_cast<const void*>(desc), k, m_pad, col0, ncols, bytewise, max_blocks,
                             as_stream(stream), copies),
              "gf_gemm");
      },
      py::arg("desc"), py::arg("k"), py::arg("m_pad"), py::arg("col0"), py::arg("ncols"), py::arg("bytewise") = false,
      py::arg("max_blocks") = 0, py::arg("stream") = 0, py::arg("copies") = true);
  m.def(
      "gemm_batched",
      [](uint64_t desc, int k, int m_pad, int batch, int64_t col0, int64_t ncols, bool bytewise, uint64_t stream,
         bool copies) {
        check(launch_gf_gemm_batched(reinterpret_cast<const void*>(desc), k, m_pad, batch, col0, ncols, bytewise,
                                     as_stream(stream), copies),
              "gf_gemm_batched");
      },
      py::arg("desc"), py::arg("k"), py::arg("m_pad"), py::arg("batch"), py::arg("col0"), py::arg("ncols"),
      py::arg("bytewise") = false, py::arg("stream") = 0, py::arg("copies") = true);
  m.def(
      "gemm_variant",
      [](uint64_t desc, int k, int m_pad, int64_t col0, int64_t ncols, int vec, int pf, bool nt, int max_blocks,
         uint64_t stream) {
        check(launch_gf_gemm_variant(reinterpret_cast<const void*>(desc), k, m_pad, col0, ncols, vec, pf, nt,
                                     max_blocks, as_stream(stream)),
              "gf_gemm_variant");
      },
      py::arg("desc"), py::arg("k"), py::arg("m_pad"), py::arg("col0"), py::arg("ncols"), py::arg("vec"),
      py::arg("pf") = 2, py::arg("nt") = false, py::arg("max_blocks") = 0, py::arg("stream") = 0);
  m.def(
      "invert",
      [](uint64_t a, uint64_t a_inv, int n, int batch, uint64_t status, uint64_t desc, uint64_t sel_rows, int mm,
         int m_pad, uint64_t stream) {
        check(launch_gf_invert(reinterpret_cast<const uint8_t*>(a), reinterpret_cast<uint8_t*>(a_inv), n, batch,
                               reinterpret_cast<int*>(status), reinterpret_cast<void*>(desc),
                               reinterpret_cast<const int*>(sel_rows), mm, m_pad, as_stream(stream)),
              "gf_invert");
      },
      py::arg("a"), py::arg("a_inv"), py::arg("n"), py::arg("batch") = 1, py::arg("status") = 0, py::arg("desc") = 0,
      py::arg("sel_rows") = 0, py::arg("m") = 0, py::arg("m_pad") = 0, py::arg("stream") = 0);
  m.def(
      "gemm16",
      [](uint64_t desc, int k, int m_pad, int64_t col0, int64_t ncols, bool symwise, int max_blocks, uint64_t stream) {
        check(launch_gf_gemm16(reinterpret_cast<const void*>(desc), k, m_pad, col0, ncols, symwise, max_blocks,
                               as_stream(stream)),
              "gf_gemm16");
      },
      py::arg("desc"), py::arg("k"), py::arg("m_pad"), py::arg("col0"), py::arg("ncols"), py::arg("symwise") = false,
      py::arg("max_blocks") = 0, py::arg("stream") = 0);
  m.def("gemm_lut", [](uint64_t desc, int k, int m_pad, int64_t col0, int64_t ncols, uint64_t stream) {
    check(launch_gf_gemm_lut(reinterpret_cast<const void*>(desc), k, m_pad, col0, ncols, as_stream(stream)),
          "gf_gemm_lut");
  });
  m.def("mfma_bitmat_bytes", &mfma_bitmat_bytes);
  m.def("mfma_bitmat", [](uint64_t coeff, int mm, int k, uint64_t bitmat, uint64_t stream) {
    check(launch_mfma_bitmat(reinterpret_cast<const uint8_t*>(coeff), mm, k, reinterpret_cast<void*>(bitmat),
                             as_stream(stream)),
          "mfma_bitmat");
  });
  m.def("gemm_mfma", [](uint64_t bitmat, uint64_t desc, int k, int mm, int64_t col0, int64_t ncols, uint64_t stream) {
    check(launch_gf_gemm_mfma(reinterpret_cast<const void*>(bitmat), reinterpret_cast<const void*>(desc), k, mm, col0,
                              ncols, as_stream(stream)),
          "gf_gemm_mfma");
  });
  m.def("fp4_bitmat_bytes", &fp4_bitmat_bytes);
  m.def("fp4_bitmat", [](uint64_t coeff, int mm, int k, uint64_t bitmat, int mg_cap, uint64_t stream) {
    check(launch_fp4_bitmat(reinterpret_cast<const uint8_t*>(coeff), mm, k, reinterpret_cast<void*>(bitmat), mg_cap,
                            as_stream(stream)),
          "fp4_bitmat");
  });
  m.def(
      "decode_system",
      [](uint64_t g, int k, uint64_t rows, uint64_t erased, int e, uint64_t dm, uint64_t status, uint64_t desc,
         int m_pad, uint64_t stream, uint64_t ptrs, int n_chunks) {
        check(launch_gf_decode_system(reinterpret_cast<const uint8_t*>(g), k, reinterpret_cast<const int*>(rows),
                                      reinterpret_cast<int*>(erased), e, reinterpret_cast<uint8_t*>(dm),
                                      reinterpret_cast<int*>(status), reinterpret_cast<void*>(desc), m_pad,
                                      as_stream(stream), reinterpret_cast<const uint64_t*>(ptrs), n_chunks),
              "decode_system");
      },
      py::arg("g"), py::arg("k"), py::arg("rows"), py::arg("erased"), py::arg("e"), py::arg("dm"), py::arg("status"),
      py::arg("desc"), py::arg("m_pad"), py::arg("stream"), py::arg("ptrs") = 0, py::arg("n_chunks") = 0);
  m.def(
      "decode_system16",
      [](uint64_t g, int n, int k, uint64_t rows, uint64_t erased, int e, uint64_t dm, uint64_t status, uint64_t desc,
         int m_pad, uint64_t stream, uint64_t ptrs, uint64_t workspace, bool force_blocked) {
        check(launch_gf_decode_system16(reinterpret_cast<const uint16_t*>(g), n, k, reinterpret_cast<const int*>(rows),
                                        reinterpret_cast<int*>(erased), e, reinterpret_cast<uint16_t*>(dm),
                                        reinterpret_cast<int*>(status), reinterpret_cast<void*>(desc), m_pad,
                                        as_stream(stream), reinterpret_cast<const uint64_t*>(ptrs),
                                        reinterpret_cast<void*>(workspace), force_blocked),
              "decode_system16");
      },
      py::arg("g"), py::arg("n"), py::arg("k"), py::arg("rows"), py::arg("erased"), py::arg("e"), py::arg("dm"),
      py::arg("status"), py::arg("desc"), py::arg("m_pad"), py::arg("stream"), py::arg("ptrs") = 0,
      py::arg("workspace") = 0, py::arg("force_blocked") = false);
  m.def("decode_system16_supported", &decode_system16_supported);
  m.def("decode_system16_workspace", &decode_system16_workspace,
        "device workspace bytes of the blocked GF(2^16) decode solve (-1: too large)");
  m.def("fp4_bitmat_sel",[](uint64_t coeff, int ld, uint64_t sel, int mm, int k, uint64_t bitmat, int mg_cap,
                             uint64_t stream) {
    check(launch_fp4_bitmat_sel(reinterpret_cast<const uint8_t*>(coeff), ld, reinterpret_cast<const int*>(sel), mm, k,
                                reinterpret_cast<void*>(bitmat), mg_cap, as_stream(stream)),
          "fp4_bitmat_sel");
  });
  m.def("gemm_fp4", [](uint64_t bitmat, uint64_t desc, int k, int mm, int64_t col0, int64_t ncols, int mg_cap,
                       int64_t in_stride, bool copies, uint64_t stream) {
    check(launch_gf_gemm_fp4(reinterpret_cast<const void*>(bitmat), reinterpret_cast<const void*>(desc), k, mm, col0,
                             ncols, mg_cap, in_stride, copies, as_stream(stream)),
          "gf_gemm_fp4");
  });
  m.def("fp4_route", [](int k, int mm, bool copies, int mg_cap) { return std::string(fp4_route_name(k, mm, copies, mg_cap)); },
        py::arg("k"), py::arg("m"), py::arg("copies") = false, py::arg("mg_cap") = 8,
        "the FP4 kernel form (v1 / ar / tm) launch_gf_gemm_fp4 runs for this shape");
  m.def("gemm_fp4_batched", [](uint64_t bitmat, uint64_t desc, int k, int mm, int batch, int64_t col0, int64_t ncols,
                               int mg_cap, int64_t in_stride, int64_t in_bstride, int64_t out_bstride, bool copies,
                               uint64_t stream) {
    check(launch_gf_gemm_fp4_batched(reinterpret_cast<const void*>(bitmat), reinterpret_cast<const void*>(desc), k, mm,
                                     batch, col0, ncols, mg_cap, in_stride, in_bstride, out_bstride, copies,
                                     as_stream(stream)),
          "gf_gemm_fp4_batched");
  });
  m.def("fp4_batched_supported", [](int k, int mm, int mg_cap) {
    // (the A-resident kernel: k in (112, 128] and every M-tile in one group)
    const int mtiles = (mm + 3) / 4;
    int mg = 1;
    while (mg < mtiles && mg < mg_cap) mg <<= 1;
    return k > 112 && k <= 128 && mtiles <= mg && fp4ar_supported(k, mg);
  });
  m.def("fp16_bitmat_bytes", &fp16_bitmat_bytes);
  m.def("fp16_bitmat", [](uint64_t coeff, int ld, uint64_t sel, int mm, int k, uint64_t bitmat, int mg_cap,
                          uint64_t stream) {
    check(launch_fp16_bitmat(reinterpret_cast<const uint16_t*>(coeff), ld, reinterpret_cast<const int*>(sel), mm, k,
                             reinterpret_cast<void*>(bitmat), mg_cap, as_stream(stream)),
          "fp16_bitmat");
  });
  m.def("gemm16_batched", [](uint64_t desc, int k, int m_pad, int batch, int64_t col0, int64_t ncols, bool symwise,
                             uint64_t stream) {
    check(launch_gf_gemm16_batched(reinterpret_cast<const void*>(desc), k, m_pad, batch, col0, ncols, symwise, 0,
                                   as_stream(stream)),
          "gf_gemm16_batched");
  });
  m.def("gemm16_fp4_batched", [](uint64_t bitmat, uint64_t desc, int k, int mm, int batch, int64_t col0, int64_t ncols,
                                 int mg_cap, int64_t in_stride, int64_t in_bstride, int64_t out_bstride, bool copies,
                                 uint64_t stream) {
    check(launch_gf_gemm16_fp4_batched(reinterpret_cast<const void*>(bitmat), reinterpret_cast<const void*>(desc), k,
                                       mm, batch, col0, ncols, mg_cap, in_stride, in_bstride, out_bstride, copies,
                                       as_stream(stream)),
          "gf_gemm16_fp4_batched");
  });
  m.def("gemm16_fp4", [](uint64_t bitmat, uint64_t desc, int k, int mm, int64_t col0, int64_t ncols, int mg_cap,
                         int64_t in_stride, bool copies, uint64_t stream) {
    check(launch_gf_gemm16_fp4(reinterpret_cast<const void*>(bitmat), reinterpret_cast<const void*>(desc), k, mm, col0,
                               ncols, mg_cap, in_stride, copies, as_stream(stream)),
          "gf_gemm16_fp4");
  });
  m.def("gen_matrix", [](uint64_t e, int k, int p, int kind, uint64_t stream) {
    check(launch_gen_matrix(reinterpret_cast<uint8_t*>(e), k, p, kind, as_stream(stream)), "gen_matrix");
  });
  m.def("perm_tables", [](uint64_t coeff, int mm, int k, uint64_t desc, int m_pad, uint64_t stream) {
    check(launch_perm_tables(reinterpret_cast<const uint8_t*>(coeff), mm, k, reinterpret_cast<void*>(desc), m_pad,
                             as_stream(stream)),
          "perm_tables");
  });
  m.def("fill_random", [](uint64_t dst, int64_t bytes, uint64_t seed, uint64_t stream) {
    check(launch_fill_random(reinterpret_cast<uint8_t*>(dst), bytes, seed, as_stream(stream)), "fill_random");
  });
  m.def("gather_rows", [](uint64_t g, uint64_t rows, uint64_t out, int mm, int k, uint64_t stream) {
    check(launch_gather_rows(reinterpret_cast<const uint8_t*>(g), reinterpret_cast<const int*>(rows),
                             reinterpret_cast<uint8_t*>(out), mm, k, as_stream(stream)),
          "gather_rows");
  });

  m.def(
      "gemm_host",
      [](const std::vector<int>& devices, const std::vector<uint64_t>& in, const std::vector<uint64_t>& out,
         const py::bytes& coeff, int64_t ncols, int streams, int64_t slice, int max_blocks, bool bytewise,
         int copy_streams, bool rect, int field_w, bool zero_copy) {
        PipelineOptions opt;
        opt.field_w = field_w;
        opt.zero_copy = zero_copy;
        opt.streams = streams;
        opt.slice_bytes = slice;
        opt.max_blocks = max_blocks;
        opt.bytewise = bytewise;
        opt.copy_streams = copy_streams;
        opt.rect = rect;
        const Mat c = to_mat(coeff);
        auto ip = ptrs<const uint8_t*>(in);
        auto op = ptrs<uint8_t*>(out);
        std::vector<PipelineStats> st;
        double wall = 0;
        hipError_t e;
        {
          py::gil_scoped_release nogil;
          e = gemm_host_multi(devices, ip, op, c, ncols, opt, &st, &wall);
        }
        check(e, "gemm_host");
        py::dict d;
        d["wall_ms"] = wall;
        py::list per;
        for (const auto& s : st) per.append(stats_dict(s));
        d["devices"] = per;
        return d;
      },
      py::arg("devices"), py::arg("in_ptrs"), py::arg("out_ptrs"), py::arg("coeff"), py::arg("ncols"),
      py::arg("streams") = 2, py::arg("slice") = 16 << 20, py::arg("max_blocks") = 0, py::arg("bytewise") = false,
      py::arg("copy_streams") = 1, py::arg("rect") = true, py::arg("field_w") = 8, py::arg("zero_copy") = false);

  // `prep` (optional): setup started before the file reads; waited for on the first call
  m.def(
      "prepare_pipeline",
      [](const std::vector<int>& devices, int k, int mm, int64_t ncols, int streams, int64_t slice, bool zero_copy) {
        hipError_t e;
        PipelineOptions opt = pipeline_options(streams, slice, 0);
        opt.zero_copy = zero_copy;
        {
          py::gil_scoped_release nogil;
          e = prepare_pipeline_multi(devices, k, mm, ncols, opt);
        }
        check(e, "prepare_pipeline");
      },
      py::arg("devices"), py::arg("k"), py::arg("m"), py::arg("ncols"), py::arg("streams") = 2,
      py::arg("slice") = 16 << 20, py::arg("zero_copy") = false);
  // pinned host memory with explicit hipHostMalloc flags (pipeline experiments: cold vs warm DMA)
  m.def("host_alloc", [](int64_t bytes, unsigned flags) {
    void* p = nullptr;
    check(hipHostMalloc(&p, size_t(bytes), flags), "hipHostMalloc");
    return reinterpret_cast<uint64_t>(p);
  });
  m.def("host_free", [](uint64_t p) { check(hipHostFree(reinterpret_cast<void*>(p)), "hipHostFree"); });
  m.def("device_shard", [](int64_t ncols, int devices, int d) { return device_shard(ncols, devices, d); });

  auto gpu_gemm = [](const std::vector<int>& devices, int streams, int64_t slice, int max_blocks,
                     std::unique_ptr<AsyncPrepare>* prep = nullptr, bool zero_copy = false) -> GemmFn {
    return [=](const std::vector<const uint8_t*>& in, const std::vector<uint8_t*>& out, const Mat& coeff,
               int64_t ncols, int field_w) {
      if (prep && *prep) {
        (*prep)->wait();
        prep->reset();
      }
      PipelineOptions opt = pipeline_options(streams, slice, max_blocks);
      opt.field_w = field_w;
      opt.zero_copy = zero_copy;
      check(gemm_host_multi(devices, in, out, coeff, ncols, opt, nullptr, nullptr), "GPU pipeline");
    };
  };
  m.def(
      "encode_file",
      [gpu_gemm](const std::string& file, int k, int p, const std::string& matrix, bool cpu_meta,
                 const std::vector<int>& devices, int streams, int64_t slice, int max_blocks, int field_w,
                 bool zero_copy) {
        FileReport r;
        {
          py::gil_scoped_release nogil;
          PipelineOptions popt = pipeline_options(streams, slice, max_blocks);
          popt.field_w = field_w;
          popt.zero_copy = zero_copy;
          auto prep = prepare_for_encode(devices, popt, file, k, p);
          r = encode_file(file, k, p, parse_matrix_kind(matrix),
                          gpu_gemm(devices, streams, slice, max_blocks, &prep, zero_copy), pinned_alloc(), cpu_meta,
                          field_w);
        }
        return report(r);
      },
      py::arg("file"), py::arg("k"), py::arg("p"), py::arg("matrix") = "vandermonde", py::arg("cpu_meta") = false,
      py::arg("devices") = std::vector<int>{0}, py::arg("streams") = 2, py::arg("slice") = 16 << 20,
      py::arg("max_blocks") = 0, py::arg("field_w") = 8, py::arg("zero_copy") = false);
  m.def(
      "decode_file",
      [gpu_gemm](const std::string& file, const std::string& conf, const std::string& out,
                 const std::vector<int>& devices, int streams, int64_t slice, int max_blocks, bool zero_copy) {
        FileReport r;
        {
          py::gil_scoped_release nogil;
          PipelineOptions popt = pipeline_options(streams, slice, max_blocks);
          popt.zero_copy = zero_copy;
          auto prep = prepare_for_decode(devices, popt, file);
          r = decode_file(file, conf, out, gpu_gemm(devices, streams, slice, max_blocks, &prep, zero_copy),
                          pinned_alloc());
        }
        return report(r);
      },
      py::arg("file"), py::arg("conf"), py::arg("out") = "", py::arg("devices") = std::vector<int>{0},
      py::arg("streams") = 2, py::arg("slice") = 16 << 20, py::arg("max_blocks") = 0, py::arg("zero_copy") = false);
  m.def("release_workspaces", [] { check(release_workspaces(), "release_workspaces"); });
  py::class_<PrepareHandle>(m, "PrepareHandle")
      .def("wait", [](PrepareHandle& h) {
        double ms = 0;
        if (h.prep) {
          py::gil_scoped_release nogil;
          ms = h.prep->wait();
        }
        return ms;
      });
  // the setup an encode / decode of `file` will need, started now on a helper thread
  m.def(
      "prepare_encode_async",
      [](const std::string& file, int k, int p, const std::vector<int>& devices, int streams, int64_t slice,
         int max_blocks, int field_w, bool zero_copy, int64_t window) {
        PipelineOptions popt = pipeline_options(streams, slice, max_blocks);
        popt.field_w = field_w;
        popt.zero_copy = zero_copy;
        StreamOptions so;
        so.window = window;
        so.field_w = field_w;
        return PrepareHandle{prepare_for_encode(devices, popt, file, k, p, &so)};
      },
      py::arg("file"), py::arg("k"), py::arg("p"), py::arg("devices") = std::vector<int>{0}, py::arg("streams") = 2,
      py::arg("slice") = 16 << 20, py::arg("max_blocks") = 0, py::arg("field_w") = 8, py::arg("zero_copy") = false,
      py::arg("window") = 0);
  m.def(
      "prepare_decode_async",
      [](const std::string& file, const std::vector<int>& devices, int streams, int64_t slice, int max_blocks,
         bool zero_copy, int64_t window) {
        PipelineOptions popt = pipeline_options(streams, slice, max_blocks);
        popt.zero_copy = zero_copy;
        StreamOptions so;
        so.window = window;
        return PrepareHandle{prepare_for_decode(devices, popt, file, &so)};
      },
      py::arg("file"), py::arg("devices") = std::vector<int>{0}, py::arg("streams") = 2, py::arg("slice") = 16 << 20,
      py::arg("max_blocks") = 0, py::arg("zero_copy") = false, py::arg("window") = 0);
  // (prep: a PrepareHandle from prepare_*_async, consumed; None: the call starts its own)
  auto take_prep = [](py::object prep) -> std::unique_ptr<AsyncPrepare> {
    if (prep.is_none()) return nullptr;
    return std::move(prep.cast<PrepareHandle&>().prep);
  };
  m.def(
      "encode_file_stream",
      [gpu_gemm, take_prep](const std::string& file, int k, int p, const std::string& matrix, bool cpu_meta,
                            const std::vector<int>& devices, int streams, int64_t slice, int max_blocks,
                            int64_t window, bool resume, bool durable, int stop_after, bool stop_before_commit, int field_w, int64_t col_lo,
                            int64_t col_hi, bool shard, bool zero_copy, py::object prep_handle) {
        StreamReport r;
        std::unique_ptr<AsyncPrepare> given = take_prep(prep_handle);
        const bool have = bool(given) || !prep_handle.is_none();
        {
          py::gil_scoped_release nogil;
          // device setup on a helper thread during the first window's reads, as bin/RS does
          StreamOptions so = stream_options(window, resume, durable, stop_after, field_w, col_lo, col_hi, shard);
          so.stop_before_commit = stop_before_commit;
          PipelineOptions popt = pipeline_options(streams, slice, max_blocks);
          popt.field_w = field_w;
          popt.zero_copy = zero_copy;
          auto prep = have ? std::move(given) : prepare_for_encode(devices, popt, file, k, p, &so);
          const GemmFn g = gpu_gemm(devices, streams, slice, max_blocks, &prep, zero_copy);
          r = encode_file_stream(file, k, p, parse_matrix_kind(matrix), g, pinned_alloc(), so, cpu_meta);
        }
        return stream_report(r);
      },
      py::arg("file"), py::arg("k"), py::arg("p"), py::arg("matrix") = "vandermonde", py::arg("cpu_meta") = false,
      py::arg("devices") = std::vector<int>{0}, py::arg("streams") = 2, py::arg("slice") = 16 << 20,
      py::arg("max_blocks") = 0, py::arg("window") = 0, py::arg("resume") = true, py::arg("durable") = true,
      py::arg("stop_after") = -1, py::arg("stop_before_commit") = false, py::arg("field_w") = 8, py::arg("col_lo") = 0, py::arg("col_hi") = -1,
      py::arg("shard") = false, py::arg("zero_copy") = false, py::arg("prep") = py::none());
  m.def(
      "decode_file_stream",
      [gpu_gemm, take_prep](const std::string& file, const std::string& conf, const std::string& out,
                            const std::vector<int>& devices, int streams, int64_t slice, int max_blocks,
                            int64_t window, bool resume, bool durable, int stop_after, bool stop_before_commit, int64_t col_lo,
                            int64_t col_hi, bool shard, const std::vector<int>& rows, bool zero_copy,
                            py::object prep_handle) {
        StreamReport r;
        std::unique_ptr<AsyncPrepare> given = take_prep(prep_handle);
        const bool have = bool(given) || !prep_handle.is_none();
        {
          py::gil_scoped_release nogil;
          StreamOptions so = stream_options(window, resume, durable, stop_after, 8, col_lo, col_hi, shard, rows);
          so.stop_before_commit = stop_before_commit;
          PipelineOptions popt = pipeline_options(streams, slice, max_blocks);
          popt.zero_copy = zero_copy;
          auto prep = have ? std::move(given) : prepare_for_decode(devices, popt, file, &so);
          const GemmFn g = gpu_gemm(devices, streams, slice, max_blocks, &prep, zero_copy);
          r = decode_file_stream(file, conf, out, g, pinned_alloc(), so);
        }
        return stream_report(r);
      },
      py::arg("file"), py::arg("conf"), py::arg("out") = "", py::arg("devices") = std::vector<int>{0},
      py::arg("streams") = 2, py::arg("slice") = 16 << 20, py::arg("max_blocks") = 0, py::arg("window") = 0,
      py::arg("resume") = true, py::arg("durable") = true, py::arg("stop_after") = -1, py::arg("stop_before_commit") = false, py::arg("col_lo") = 0,
      py::arg("col_hi") = -1, py::arg("shard") = false, py::arg("rows") = std::vector<int>{},
      py::arg("zero_copy") = false, py::arg("prep") = py::none());
}

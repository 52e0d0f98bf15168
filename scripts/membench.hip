// HBM streaming microbenchmark for the GF-GEMM access pattern: read R rows, write W rows, no math
// (an XOR fold keeps the loads live). Answers "what does the memory system give THIS pattern?" so
// the GF-GEMM kernels can be priced against it rather than against a 1-in/1-out copy.
//
// Build: hipcc -O3 --offload-arch=gfx950 -o build/membench scripts/membench.hip
// Run:   build/membench [REPS]     (prints one JSON object)
//        build/membench sdma [ROWS WIDTH]   (copy engines vs blit copies, one JSON line per case)
//        build/membench pitch [REPS]        (enc / dec patterns at different row pitches)
//        build/membench k16 [REPS [ROW_MiB [PITCH_MiB...]]]   (config #4's k = 16 patterns, 512 MiB rows)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
template <typename T>
using gptr = __attribute__((address_space(1))) T*;

template <bool NT>
__device__ __forceinline__ u32x4 ld(gptr<const u32x4> p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(gptr<u32x4> p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// V 16-byte groups per lane, wave-strided (lane l, group v -> byte 16*l + 1024*v of the wave's span)
// PERSIST: grid-stride over wave spans; otherwise one span per wave.
template <int R, int W, int V, bool NT, bool PERSIST, int BS>
__global__ __launch_bounds__(BS) void stream_kernel(const uint8_t* in, uint8_t* out, int64_t pitch, int64_t nspans) {
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = int64_t(blockIdx.x) * (BS / 64) + (threadIdx.x >> 6);
  const int64_t wstride = PERSIST ? int64_t(gridDim.x) * (BS / 64) : nspans;
  for (int64_t w = wave0; w < nspans; w += wstride) {
    const int64_t off = w * (1024 * V) + 16 * lane;
    u32x4 x[R][V];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int v = 0; v < V; ++v) x[r][v] = ld<NT>((gptr<const u32x4>)(in + r * pitch + off + 1024 * v));
    u32x4 acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      acc[v] = x[0][v];
#pragma unroll
      for (int r = 1; r < R; ++r) acc[v] ^= x[r][v];
    }
#pragma unroll
    for (int o = 0; o < W; ++o)
#pragma unroll
      for (int v = 0; v < V; ++v) {
        u32x4 y = acc[v];
        y.x ^= o;
        st<NT>((gptr<u32x4>)(out + o * pitch + off + 1024 * v), o < R ? x[o][v] ^ y : y);
      }
  }
}

struct Case {
  std::string name;
  int R, W;
  void (*fn)(const uint8_t*, uint8_t*, int64_t, int64_t);
  int V, BS;
  bool persist;
};

template <int R, int W, int V, bool NT, bool P, int BS>
Case mk(const char* tag) {
  Case c;
  c.name = std::string(tag) + "_r" + std::to_string(R) + "w" + std::to_string(W) + "_v" + std::to_string(V) +
           (NT ? "_nt" : "_plain") + (P ? "_persist" : "_grid") + "_bs" + std::to_string(BS);
  c.R = R;
  c.W = W;
  c.fn = stream_kernel<R, W, V, NT, P, BS>;
  c.V = V;
  c.BS = BS;
  c.persist = P;
  return c;
}

int pattern_main(int argc, char** argv) {
  const int64_t C = 107374183;            // the headline chunk size (1 GiB / 10)
  const int64_t pitch = (C + 255) / 256 * 256;
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint8_t *in, *out;
  CHECK(hipMalloc(&in, 10 * pitch));
  CHECK(hipMalloc(&out, 10 * pitch));
  CHECK(hipMemset(in, 0x5a, 10 * pitch));
  CHECK(hipMemset(out, 0, 10 * pitch));

  std::vector<Case> cases = {
      mk<1, 1, 1, true, false, 256>("copy"),     mk<1, 1, 4, true, false, 256>("copy"),
      mk<1, 1, 4, false, false, 256>("copy"),    mk<1, 1, 4, true, true, 256>("copy"),
      mk<10, 4, 1, true, false, 256>("enc"),     mk<10, 4, 1, false, false, 256>("enc"),
      mk<10, 4, 2, true, false, 256>("enc"),     mk<10, 4, 1, true, true, 256>("enc"),
      mk<10, 4, 2, true, true, 256>("enc"),      mk<10, 4, 1, true, false, 512>("enc"),
      mk<10, 4, 4, true, true, 256>("enc"),      mk<10, 10, 1, true, false, 256>("dec"),
      mk<10, 10, 1, false, false, 256>("dec"),   mk<10, 10, 2, true, false, 256>("dec"),
      mk<10, 10, 1, true, true, 256>("dec"),     mk<10, 10, 2, true, true, 256>("dec"),
      mk<10, 10, 4, true, true, 256>("dec"),
  };
  std::vector<std::vector<float>> t(cases.size());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int round = 0; round < 5; ++round) {
    for (size_t i = 0; i < cases.size(); ++i) {
      const Case& c = cases[i];
      const int64_t nspans = (C / 16) / (64 * c.V);
      const int64_t waves_per_block = c.BS / 64;
      int64_t blocks = (nspans + waves_per_block - 1) / waves_per_block;
      if (c.persist) {
        int occ = 0;
        CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(c.fn), c.BS, 0));
        blocks = std::min<int64_t>(blocks, int64_t(cus) * occ);
      }
      hipLaunchKernelGGL(c.fn, dim3(unsigned(blocks)), dim3(c.BS), 0, 0, in, out, pitch, nspans);
      CHECK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(c.fn, dim3(unsigned(blocks)), dim3(c.BS), 0, 0, in, out, pitch, nspans);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipGetLastError());
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      t[i].push_back(ms / reps * 1e3f);
    }
  }
  printf("{\n");
  for (size_t i = 0; i < cases.size(); ++i) {
    std::vector<float> v = t[i];
    std::sort(v.begin(), v.end());
    const Case& c = cases[i];
    const int64_t nspans = (C / 16) / (64 * c.V);
    const double bytes = double(c.R + c.W) * nspans * 64 * 16 * c.V;
    printf("  \"%s\": {\"us_median\": %.2f, \"us_min\": %.2f, \"TBps\": %.3f}%s\n", c.name.c_str(), v[v.size() / 2],
           v[0], bytes / (v[v.size() / 2] * 1e-6) / 1e12, i + 1 < cases.size() ? "," : "");
  }
  printf("}\n");
  return 0;
}

// ---- config #4's pattern: `membench k16 [REPS]` ----------------------------------------------
// The k16n20_8g step's access patterns with no math, at its row size (8 GiB / 16 = 512 MiB rows,
// 2 MiB pitch as alloc_rows lays them out): encode 16 rows in / 4 out, decode 16 in / 16 out (the
// rebuilt natives plus the fused survivor copies), one span per wave (grid) and persistent. One
// JSON line per case: the ceiling the k = 16 kernels are priced against.
int k16_main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  // row length (MiB, default 512 = config #4's 8 GiB / 16) and the row pitches to compare (MiB,
  // >= the row): a power-of-two pitch puts row j's byte x at j * 2^29 + x, the same offset inside
  // every large power-of-two block; default: only the row length itself
  const int64_t C = (argc > 2 ? int64_t(atoi(argv[2])) : 512) << 20;
  std::vector<int64_t> pitches;
  for (int i = 3; i < argc; ++i) pitches.push_back(int64_t(atoi(argv[i])) << 20);
  if (pitches.empty()) pitches.push_back(C);
  int64_t maxp = 0;
  for (int64_t p : pitches) {
    if (p < C) {
      fprintf(stderr, "pitch below the row length\n");
      return 2;
    }
    maxp = std::max(maxp, p);
  }
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint8_t *in, *out;
  CHECK(hipMalloc(&in, 16 * maxp + (2 << 20)));
  CHECK(hipMalloc(&out, 16 * maxp + (2 << 20)));
  CHECK(hipMemset(in, 0x5a, 16 * maxp));
  CHECK(hipMemset(out, 0, 16 * maxp));
  uint8_t* in0 = reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(in) + (2 << 20) - 1) & ~uintptr_t((2 << 20) - 1));
  uint8_t* out0 = reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(out) + (2 << 20) - 1) & ~uintptr_t((2 << 20) - 1));
  std::vector<Case> cases = {mk<16, 4, 1, true, false, 256>("enc"), mk<16, 16, 1, true, false, 256>("dec"),
                             mk<16, 16, 1, true, true, 256>("dec")};
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<std::vector<float>> t(cases.size() * pitches.size());
  for (int round = 0; round < 5; ++round)
    for (size_t pi = 0; pi < pitches.size(); ++pi)
      for (size_t i = 0; i < cases.size(); ++i) {
        const Case& c = cases[i];
        const int64_t nspans = (C / 16) / (64 * c.V);
        int64_t blocks = (nspans + 3) / 4;
        if (c.persist) {
          int occ = 0;
          CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(c.fn), c.BS, 0));
          blocks = std::min<int64_t>(blocks, int64_t(cus) * occ);
        }
        hipLaunchKernelGGL(c.fn, dim3(unsigned(blocks)), dim3(c.BS), 0, 0, in0, out0, pitches[pi], nspans);
        CHECK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r)
          hipLaunchKernelGGL(c.fn, dim3(unsigned(blocks)), dim3(c.BS), 0, 0, in0, out0, pitches[pi], nspans);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipGetLastError());
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        t[pi * cases.size() + i].push_back(ms / reps * 1e3f);
      }
  for (size_t pi = 0; pi < pitches.size(); ++pi)
    for (size_t i = 0; i < cases.size(); ++i) {
      std::vector<float> v = t[pi * cases.size() + i];
      std::sort(v.begin(), v.end());
      const Case& c = cases[i];
      const double bytes = double(c.R + c.W) * C;
      printf("{\"case\": \"%s\", \"row_mib\": %lld, \"pitch_mib\": %lld, \"us_median\": %.1f, \"us_min\": %.1f, "
             "\"TBps\": %.3f}\n",
             c.name.c_str(), (long long)(C >> 20), (long long)(pitches[pi] >> 20), v[v.size() / 2], v[0],
             bytes / (v[v.size() / 2] * 1e-6) / 1e12);
    }
  return 0;
}

// ---- copy engines: `membench sdma [ROWS WIDTH]` -----------------------------------------------
// Device-to-device bandwidth of hipMemcpyDeviceToDeviceNoCU (SDMA, no compute units) against the
// blit-kernel copy, alone and beside a compute-bound kernel that holds every CU. Question it
// answers: can the wide decode's survivor copy (102 rows x 8 MiB at k=128) run on the copy engines
// under the MFMA-bound GEMM instead of inside it? (profiles/wide_stripe/r05_sdma: no, ~0.12 TB/s per engine.)
// ALU-bound spin: every lane runs `iters` dependent FMAs; the result is stored so it is kept.
__global__ void spin_kernel(float* out, int iters) {
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  for (int i = 0; i < iters; ++i) a = __builtin_fmaf(a, b, 1e-7f);
  if (a == 12345.0f) out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

static float elapsed(hipEvent_t a, hipEvent_t b) {
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

int sdma_main(int argc, char** argv) {
  const size_t rows = argc > 1 ? std::atoll(argv[1]) : 102;
  const size_t width = argc > 2 ? std::atoll(argv[2]) : 8388608;  // 1 GiB / 128
  const size_t pitch_src = width + 256, pitch_dst = width + 512;   // pitched rows, as the codec's
  const size_t bytes = rows * width;
  char *src, *dst;
  float* sink;
  CHECK(hipMalloc(&src, rows * pitch_src));
  CHECK(hipMalloc(&dst, rows * pitch_dst));
  CHECK(hipMalloc(&sink, 1 << 24));
  CHECK(hipMemset(src, 7, rows * pitch_src));
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1, e2;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventCreate(&e2));
  std::vector<hipStream_t> st(9);
  for (auto& s : st) CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));

  // mode 0: one 2-D copy per stream; mode 1: one 1-D copy per row; mode 2: one 1-D copy of the
  // stream's whole span (contiguous bytes, pitches included)
  int mode = 0;
  auto copy2d = [&](hipStream_t s, size_t r0, size_t r1, hipMemcpyKind kind) {
    if (mode == 0) {
      CHECK(hipMemcpy2DAsync(dst + r0 * pitch_dst, pitch_dst, src + r0 * pitch_src, pitch_src, width, r1 - r0, kind, s));
    } else if (mode == 1) {
      for (size_t r = r0; r < r1; ++r) CHECK(hipMemcpyAsync(dst + r * pitch_dst, src + r * pitch_src, width, kind, s));
    } else {
      CHECK(hipMemcpyAsync(dst + r0 * pitch_src, src + r0 * pitch_src, (r1 - r0) * pitch_src, kind, s));
    }
  };
  // split the rows over `ns` streams, all joined into st[0] via events
  auto copy_split = [&](int ns, hipMemcpyKind kind) {
    std::vector<hipEvent_t> done(ns);
    CHECK(hipEventRecord(e0, st[0]));
    for (int i = 0; i < ns; ++i) {
      CHECK(hipStreamWaitEvent(st[1 + i], e0, 0));
      copy2d(st[1 + i], rows * i / ns, rows * (i + 1) / ns, kind);
      CHECK(hipEventCreateWithFlags(&done[i], hipEventDisableTiming));
      CHECK(hipEventRecord(done[i], st[1 + i]));
      CHECK(hipStreamWaitEvent(st[0], done[i], 0));
    }
    CHECK(hipEventRecord(e1, st[0]));
    CHECK(hipStreamSynchronize(st[0]));
    for (auto& d : done) CHECK(hipEventDestroy(d));
    return elapsed(e0, e1);
  };

  // calibrate the spin kernel to ~1 ms on every CU (4 waves per CU)
  int iters = 1 << 14;
  for (int t = 0; t < 3; ++t) {
    CHECK(hipEventRecord(e0, st[0]));
    spin_kernel<<<cus, 256, 0, st[0]>>>(sink, iters);
    CHECK(hipEventRecord(e1, st[0]));
    CHECK(hipStreamSynchronize(st[0]));
    float ms = elapsed(e0, e1);
    iters = int(iters * (1.0f / ms));
  }

  std::printf("{\"rows\": %zu, \"width\": %zu, \"bytes\": %zu, \"cus\": %d}\n", rows, width, bytes, cus);
  const struct {
    const char* name;
    hipMemcpyKind kind;
  } kinds[] = {{"blit", hipMemcpyDeviceToDevice}, {"nocu", hipMemcpyDeviceToDeviceNoCU}};
  for (mode = 0; mode < 3; ++mode)
  for (auto& kd : kinds) {
    for (int ns : {1, 2, 4, 8}) {
      copy_split(ns, kd.kind);  // warm
      float best = 1e9f;
      for (int r = 0; r < 3; ++r) best = std::min(best, copy_split(ns, kd.kind));
      std::printf("{\"mode\": %d, \"copy\": \"%s\", \"streams\": %d, \"ms\": %.3f, \"GBps\": %.1f}\n", mode, kd.name, ns, best,
                  2.0 * bytes / best / 1e6);
    }
  }
  // overlap: spin on st[0] (every CU, ~1 ms) while the copy runs on st[1..ns]
  for (mode = 0; mode < 3; ++mode)
  for (auto& kd : kinds) {
    for (int ns : {1, 4}) {
      float best_spin = 1e9f, best_both = 1e9f;
      for (int r = 0; r < 3; ++r) {
        CHECK(hipEventRecord(e0, st[0]));
        spin_kernel<<<cus, 256, 0, st[0]>>>(sink, iters);
        CHECK(hipEventRecord(e1, st[0]));
        CHECK(hipStreamSynchronize(st[0]));
        best_spin = std::min(best_spin, elapsed(e0, e1));
        std::vector<hipEvent_t> done(ns);
        CHECK(hipEventRecord(e0, st[0]));
        for (int i = 0; i < ns; ++i) {
          CHECK(hipStreamWaitEvent(st[1 + i], e0, 0));
          copy2d(st[1 + i], rows * i / ns, rows * (i + 1) / ns, kd.kind);
          CHECK(hipEventCreateWithFlags(&done[i], hipEventDisableTiming));
          CHECK(hipEventRecord(done[i], st[1 + i]));
        }
        spin_kernel<<<cus, 256, 0, st[0]>>>(sink, iters);
        for (int i = 0; i < ns; ++i) CHECK(hipStreamWaitEvent(st[0], done[i], 0));
        CHECK(hipEventRecord(e2, st[0]));
        CHECK(hipStreamSynchronize(st[0]));
        best_both = std::min(best_both, elapsed(e0, e2));
        for (auto& d : done) CHECK(hipEventDestroy(d));
      }
      std::printf("{\"mode\": %d, \"overlap\": \"%s\", \"streams\": %d, \"spin_ms\": %.3f, \"spin_plus_copy_ms\": %.3f}\n", mode, kd.name, ns,
                  best_spin, best_both);
    }
  }
  CHECK(hipFree(src));
  CHECK(hipFree(dst));
  CHECK(hipFree(sink));
  return 0;
}

// `membench pitch`: the enc (10 in / 4 out) and dec (10 in / 10 out) patterns at different row
// pitches and output-buffer offsets — does the placement of the rows in HBM's channel interleave
// move the ceiling? Pitch = C rounded up to `align`, plus `extra` bytes; the output rows start
// `ooff` bytes after a 2 MiB-aligned base. One JSON line per case.
int pitch_main(int argc, char** argv) {
  const int64_t C = 107374183;
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  struct P {
    int64_t align, extra, ooff;
  };
  std::vector<P> ps = {
      {256, 0, 0},          {4096, 2048, 0},        {2 << 20, 0, 0},        {2 << 20, 256, 0},
      {2 << 20, 512, 0},    {2 << 20, 1024, 0},     {2 << 20, 2048, 0},     {2 << 20, 65536, 0},
      {2 << 20, 1 << 20, 0}, {1 << 20, 0, 0},       {512 << 10, 0, 0},      {4 << 20, 0, 0},
      {8 << 20, 0, 0},      {2 << 20, 0, 1 << 20},  {2 << 20, 0, 256 << 10}, {2 << 20, 0, 4096},
      {2 << 20, 0, 256}};
  // `membench pitch REPS MiB...`: explicit pitches in MiB instead (align 1 MiB, extra = the rest)
  if (argc > 2) {
    ps.clear();
    for (int i = 2; i < argc; ++i) {
      const int64_t p = int64_t(atoi(argv[i])) << 20;
      if (p < C || p > (int64_t(160) << 20)) {
        fprintf(stderr, "pitch %s MiB: need C <= pitch <= 160 MiB\n", argv[i]);
        return 2;
      }
      ps.push_back({1 << 20, p - (C + (1 << 20) - 1) / (1 << 20) * (1 << 20), 0});
    }
  }
  const Case cs[2] = {mk<10, 4, 1, true, false, 256>("enc"), mk<10, 10, 1, true, false, 256>("dec")};
  const int64_t maxpitch = int64_t(161) << 20;
  uint8_t *in, *out;
  CHECK(hipMalloc(&in, 10 * maxpitch + (4 << 20)));
  CHECK(hipMalloc(&out, 10 * maxpitch + (4 << 20)));
  CHECK(hipMemset(in, 0x5a, 10 * maxpitch));
  uint8_t* in0 = reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(in) + (2 << 20) - 1) & ~uintptr_t((2 << 20) - 1));
  uint8_t* out0 = reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(out) + (2 << 20) - 1) & ~uintptr_t((2 << 20) - 1));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<std::vector<float>> t(ps.size() * 2);
  for (int round = 0; round < 5; ++round)
    for (size_t i = 0; i < ps.size(); ++i)
      for (int c = 0; c < 2; ++c) {
        const int64_t pitch = (C + ps[i].align - 1) / ps[i].align * ps[i].align + ps[i].extra;
        const int64_t nspans = (C / 16) / 64;
        const int64_t blocks = (nspans + 3) / 4;
        uint8_t* o = out0 + ps[i].ooff;
        hipLaunchKernelGGL(cs[c].fn, dim3(unsigned(blocks)), dim3(256), 0, 0, in0, o, pitch, nspans);
        CHECK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r)
          hipLaunchKernelGGL(cs[c].fn, dim3(unsigned(blocks)), dim3(256), 0, 0, in0, o, pitch, nspans);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipGetLastError());
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        t[2 * i + c].push_back(ms / reps * 1e3f);
      }
  for (size_t i = 0; i < ps.size(); ++i)
    for (int c = 0; c < 2; ++c) {
      std::vector<float> v = t[2 * i + c];
      std::sort(v.begin(), v.end());
      const int64_t pitch = (C + ps[i].align - 1) / ps[i].align * ps[i].align + ps[i].extra;
      const double bytes = double(cs[c].R + cs[c].W) * ((C / 16) / 64) * 64 * 16;
      printf("{\"case\": \"%s\", \"align\": %lld, \"extra\": %lld, \"out_offset\": %lld, \"pitch_mod_64k\": %lld, "
             "\"us_median\": %.2f, \"us_min\": %.2f, \"TBps\": %.3f}\n",
             c ? "dec" : "enc", (long long)ps[i].align, (long long)ps[i].extra, (long long)ps[i].ooff,
             (long long)(pitch % 65536), v[v.size() / 2], v[0], bytes / (v[v.size() / 2] * 1e-6) / 1e12);
    }
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::string(argv[1]) == "sdma") return sdma_main(argc - 1, argv + 1);
  if (argc > 1 && std::string(argv[1]) == "pitch") return pitch_main(argc - 1, argv + 1);
  if (argc > 1 && std::string(argv[1]) == "k16") return k16_main(argc - 1, argv + 1);
  return pattern_main(argc, argv);
}

// HBM streaming microbenchmark for the GF-GEMM access pattern: read R rows, write W rows, no math
// (an XOR fold keeps the loads live). Answers "what does the memory system give THIS pattern?" so
// the GF-GEMM kernels can be priced against it rather than against a 1-in/1-out copy.
//
// Build: hipcc -O3 --offload-arch=gfx950 -o build/membench scripts/membench.hip
// Run:   build/membench            (prints one JSON object)
#include <hip/hip_runtime.h>

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

int main(int argc, char** argv) {
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

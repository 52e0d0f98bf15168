// Does streaming the GF-GEMM's input rows through LDS-DMA (global_load_lds_dwordx4) beat register
// loads for the narrow-code pattern? Same pattern as membench.hip — read R rows, write W rows, an
// XOR fold instead of the math — with the reads as LDS-DMA into a per-wave ring of D spans (R KiB
// each), consumed by ds_read_b128. MI355X_MICROARCH.md measures LDS-DMA streams at 6.5-6.8 TB/s
// (nt) against ~6.0 for register loads.
//
// Build: hipcc -O3 --offload-arch=gfx950 -o bin/membench_lds scripts/membench_lds.hip
// Run:   bin/membench_lds [reps]        (prints one JSON object)
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
using lds_u8 = __attribute__((address_space(3))) uint8_t;
using lds_v4 = __attribute__((address_space(3))) u32x4;

// register loads (the GEMM kernel's current scheme): one wave span = 64 lanes x 16 B per row
template <int R, int W>
__global__ __launch_bounds__(256) void reg_kernel(const uint8_t* in, uint8_t* out, int64_t pitch, int64_t nspans) {
  const int lane = threadIdx.x & 63;
  const int64_t wstride = int64_t(gridDim.x) * 4;
  for (int64_t w = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); w < nspans; w += wstride) {
    const int64_t off = w * 1024 + 16 * lane;
    u32x4 x[R];
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = __builtin_nontemporal_load((gptr<const u32x4>)(in + r * pitch + off));
    u32x4 acc = x[0];
#pragma unroll
    for (int r = 1; r < R; ++r) acc ^= x[r];
#pragma unroll
    for (int o = 0; o < W; ++o) {
      u32x4 y = acc;
      y.x ^= o;
      __builtin_nontemporal_store(o < R ? x[o] ^ y : y, (gptr<u32x4>)(out + o * pitch + off));
    }
  }
}

// LDS-DMA: each wave owns a ring of D slots x R KiB; span i lands in slot i % D. The stores of a span
// are counted in vmcnt (in issue order with the DMAs), so every wait is the exact constant
// (D-1)(R+W); the prologue issues dummy stores to a sink to keep the pattern from span 0.
template <int R, int W, int D>
__global__ __launch_bounds__(256) void lds_kernel(const uint8_t* in, uint8_t* out, uint8_t* sink, int64_t pitch,
                                                  int64_t nspans) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  lds_u8* ring = (lds_u8*)smem + size_t(wave) * D * R * 1024;
  const int64_t wstride = int64_t(gridDim.x) * 4;
  const int64_t w0 = int64_t(blockIdx.x) * 4 + wave;
  const int64_t my = w0 < nspans ? (nspans - 1 - w0) / wstride + 1 : 0;
  const gptr<u32x4> sk = (gptr<u32x4>)(sink + 16 * (threadIdx.x + 256 * (blockIdx.x & 255)));
  auto issue = [&](int64_t i) __attribute__((always_inline)) {
    const bool live = i < my;
    const int64_t off = (w0 + (live ? i : 0) * wstride) * 1024 + 16 * lane;
    const int slot = int(i % D);
#pragma unroll
    for (int r = 0; r < R; ++r)
      __builtin_amdgcn_global_load_lds((gptr<const void>)(in + r * pitch + off), ring + (slot * R + r) * 1024, 16, 0, 0);
  };
  if (my == 0) return;
#pragma unroll
  for (int j = 0; j < D; ++j) {
    issue(j);
    if (j < D - 1) {
#pragma unroll
      for (int o = 0; o < W; ++o) __builtin_nontemporal_store(u32x4{0, 0, 0, 0}, sk);
    }
  }
  for (int64_t i = 0; i < my; ++i) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 1) * (R + W) < 63 ? (D - 1) * (R + W) : 63) : "memory");
    const int slot = int(i % D);
    u32x4 x[R];
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = *(const lds_v4*)(ring + (slot * R + r) * 1024 + 16 * lane);
    u32x4 acc = x[0];
#pragma unroll
    for (int r = 1; r < R; ++r) acc ^= x[r];
    const int64_t off = (w0 + i * wstride) * 1024 + 16 * lane;
#pragma unroll
    for (int o = 0; o < W; ++o) {
      u32x4 y = acc;
      y.x ^= o;
      __builtin_nontemporal_store(o < R ? x[o] ^ y : y, (gptr<u32x4>)(out + o * pitch + off));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's LDS reads are done before it is refilled
    issue(i + D);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

struct Case {
  std::string name;
  int R, W;
  int kind;  // 0 reg, 1 lds
  const void* fn;
  size_t lds;
};

int main(int argc, char** argv) {
  const int64_t C = 107374183;
  const int64_t pitch = (C + 255) / 256 * 256;
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint8_t *in, *out, *sink;
  CHECK(hipMalloc(&in, 10 * pitch));
  CHECK(hipMalloc(&out, 10 * pitch));
  CHECK(hipMalloc(&sink, 256 * 256 * 16));
  CHECK(hipMemset(in, 0x5a, 10 * pitch));
  CHECK(hipMemset(out, 0, 10 * pitch));
  const int64_t nspans = (C / 16) / 64;

  std::vector<Case> cases;
  cases.push_back({"enc_reg_r10w4", 10, 4, 0, (const void*)reg_kernel<10, 4>, 0});
  cases.push_back({"enc_lds_r10w4_d2", 10, 4, 1, (const void*)lds_kernel<10, 4, 2>, 4 * 2 * 10 * 1024});
  cases.push_back({"enc_lds_r10w4_d3", 10, 4, 1, (const void*)lds_kernel<10, 4, 3>, 4 * 3 * 10 * 1024});
  cases.push_back({"dec_reg_r10w10", 10, 10, 0, (const void*)reg_kernel<10, 10>, 0});
  cases.push_back({"dec_lds_r10w10_d2", 10, 10, 1, (const void*)lds_kernel<10, 10, 2>, 4 * 2 * 10 * 1024});
  cases.push_back({"dec_lds_r10w10_d3", 10, 10, 1, (const void*)lds_kernel<10, 10, 3>, 4 * 3 * 10 * 1024});
  cases.push_back({"copy_reg_r1w1", 1, 1, 0, (const void*)reg_kernel<1, 1>, 0});
  cases.push_back({"copy_lds_r1w1_d4", 1, 1, 1, (const void*)lds_kernel<1, 1, 4>, 4 * 4 * 1024});
  for (auto& c : cases)
    if (c.lds > 65536) CHECK(hipFuncSetAttribute(c.fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(c.lds)));

  std::vector<std::vector<float>> t(cases.size());
  std::vector<int> grids(cases.size());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (size_t i = 0; i < cases.size(); ++i) {
    int occ = 0;
    CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, cases[i].fn, 256, cases[i].lds));
    grids[i] = int(std::min<int64_t>((nspans + 3) / 4, int64_t(cus) * std::max(occ, 1)));
  }
  auto launch = [&](size_t i) {
    const Case& c = cases[i];
    void* args_reg[] = {(void*)&in, (void*)&out, (void*)&pitch, (void*)&nspans};
    void* args_lds[] = {(void*)&in, (void*)&out, (void*)&sink, (void*)&pitch, (void*)&nspans};
    CHECK(hipLaunchKernel(c.fn, dim3(grids[i]), dim3(256), c.kind ? args_lds : args_reg, c.lds, 0));
  };
  for (int round = 0; round < 5; ++round)
    for (size_t i = 0; i < cases.size(); ++i) {
      launch(i);
      CHECK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) launch(i);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      t[i].push_back(ms / reps * 1e3f);
    }
  // correctness of the LDS path against the register path (same pattern, same output)
  std::vector<uint8_t> a(4096), b(4096);
  printf("{\n");
  for (size_t i = 0; i < cases.size(); ++i) {
    std::vector<float> v = t[i];
    std::sort(v.begin(), v.end());
    const Case& c = cases[i];
    const double bytes = double(c.R + c.W) * nspans * 1024;
    printf("  \"%s\": {\"us_median\": %.2f, \"us_min\": %.2f, \"TBps\": %.3f, \"grid\": %d}%s\n", c.name.c_str(),
           v[v.size() / 2], v[0], bytes / (v[v.size() / 2] * 1e-6) / 1e12, grids[i], i + 1 < cases.size() ? "," : "");
  }
  // check: enc_reg then enc_lds write the same bytes
  launch(0);
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(a.data(), out + 3 * pitch + 12345 * 16, 4096, hipMemcpyDeviceToHost));
  CHECK(hipMemset(out, 0, 10 * pitch));
  launch(2);
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(b.data(), out + 3 * pitch + 12345 * 16, 4096, hipMemcpyDeviceToHost));
  printf("}\nlds_matches_reg: %s\n", a == b ? "yes" : "NO");
  return a == b ? 0 : 1;
}

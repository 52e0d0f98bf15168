// FP4 block-scaled MFMA rate by shape: v_mfma_scale_f32_32x32x64_f8f6f4 against _16x16x128_ on the
// same FLOPs, one wave per SIMD (the wide-stripe kernels' occupancy), operands in registers.
// MI355X_MICROARCH.md measures bf16 16x16x32 at ~1.15x the FLOP/s of 32x32x16 on random data at equal
// cycles per FLOP (lower power, higher clock); the wide-stripe GF(2) bit-matrix kernels are
// clock-bound on 32x32x64, so this asks whether the FP4 16x16x128 form would carry the same clock
// advantage before any kernel is rewritten for it. Operand density: the GF(2) kernels feed {0, 1}
// e2m1 codes (one bit per nibble) at ~50 % ones; `dense` = random nibbles, `gf2` = that pattern,
// `zero` = all zero.
//
// Build: hipcc -O3 --offload-arch=gfx950 -o bin/mfma_rate scripts/mfma_rate.hip
// Run:   bin/mfma_rate [iters]      (one JSON line per shape x operands)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

using i32x8 = int __attribute__((ext_vector_type(8)));
using f32x16 = float __attribute__((ext_vector_type(16)));
using f32x4 = float __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  return x ^ (x >> 16);
}

// 8 independent accumulator chains of 32x32x64 per iteration (8 x 65536 MACs)
__global__ __launch_bounds__(256, 1) void rate32(int iters, int mode, float* out, long long* cyc) {
  const uint32_t seed = mix(blockIdx.x * 256 + threadIdx.x);
  i32x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, b = a;
  for (int i = 0; i < 4; ++i) {
    uint32_t ra = mix(seed + 17 * i), rb = mix(seed + 91 * i + 5);
    if (mode == 1) {  // gf2: one bit per nibble, ~50 % ones
      ra &= 0x22222222u;
      rb &= 0x22222222u;
    } else if (mode == 2) {
      ra = rb = 0;
    }
    a[i] = int(ra);
    b[i] = int(rb);
  }
  f32x16 acc[8];
  for (int j = 0; j < 8; ++j) acc[j] = (f32x16)(0.0f);
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      acc[j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc[j], 4, 4, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
  }
  const long long t1 = clock64();
  float s = 0.f;
  for (int j = 0; j < 8; ++j)
    for (int v = 0; v < 16; ++v) s += acc[j][v];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// 16 independent chains of 16x16x128 per iteration (16 x 32768 MACs: the same FLOPs)
__global__ __launch_bounds__(256, 1) void rate16(int iters, int mode, float* out, long long* cyc) {
  const uint32_t seed = mix(blockIdx.x * 256 + threadIdx.x);
  i32x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, b = a;
  for (int i = 0; i < 4; ++i) {
    uint32_t ra = mix(seed + 17 * i), rb = mix(seed + 91 * i + 5);
    if (mode == 1) {
      ra &= 0x22222222u;
      rb &= 0x22222222u;
    } else if (mode == 2) {
      ra = rb = 0;
    }
    a[i] = int(ra);
    b[i] = int(rb);
  }
  f32x4 acc[16];
  for (int j = 0; j < 16; ++j) acc[j] = (f32x4)(0.0f);
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      acc[j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc[j], 4, 4, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
  }
  const long long t1 = clock64();
  float s = 0.f;
  for (int j = 0; j < 16; ++j)
    for (int v = 0; v < 4; ++v) s += acc[j][v];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  float* out;
  long long* cyc;
  CHECK(hipMalloc(&out, sizeof(float) * 256 * cus));
  CHECK(hipMalloc(&cyc, sizeof(long long) * cus));
  long long* hc = new long long[cus];
  const char* names[3] = {"dense", "gf2", "zero"};
  for (int rep = 0; rep < 2; ++rep)
    for (int shape = 0; shape < 2; ++shape)
      for (int mode = 0; mode < 3; ++mode) {
        auto launch = [&](int n) {
          if (shape == 0)
            rate32<<<cus, 256>>>(n, mode, out, cyc);
          else
            rate16<<<cus, 256>>>(n, mode, out, cyc);
        };
        launch(iters / 10);  // warm + clocks up
        CHECK(hipDeviceSynchronize());
        const auto t0 = std::chrono::steady_clock::now();
        launch(iters);
        CHECK(hipDeviceSynchronize());
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        CHECK(hipMemcpy(hc, cyc, sizeof(long long) * cus, hipMemcpyDeviceToHost));
        double mc = 0;
        for (int i = 0; i < cus; ++i) mc += double(hc[i]) / cus;
        const double flops = 2.0 * 8 * 65536.0 * iters * 4 * cus;  // 4 waves per CU
        const double mfmas = double(shape == 0 ? 8 : 16) * iters;  // per wave
        printf("{\"rep\": %d, \"shape\": \"%s\", \"operands\": \"%s\", \"tflops\": %.1f, \"ms\": %.3f, "
               "\"cycles_per_mfma\": %.2f, \"clock_ghz_est\": %.3f}\n",
               rep, shape == 0 ? "32x32x64" : "16x16x128", names[mode], flops / s / 1e12, s * 1e3, mc / mfmas,
               mc / s / 1e9);
      }
  return 0;
}

// Per-process HIP setup costs on one MI355X: what a fresh bin/RS pays before its first GEMM.
//
//   make -C csrc probe && bin/setup_probe            (HSA_ENABLE_SDMA=0 bin/setup_probe: blit copies)
//
// Times, in order, in a fresh process: runtime init (hipGetDeviceCount), context (hipFree(0)), the
// first and a second stream creation, the first kernel launch (code object load), the first and a
// second small H2D hipMemcpy (copy-engine / blit set-up), hipHostRegister of 64 MiB of huge-page
// memory, and hipPointerGetAttributes on 14 rows of it. One JSON line.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace {

using Clock = std::chrono::steady_clock;
double ms(Clock::time_point a) { return std::chrono::duration<double, std::milli>(Clock::now() - a).count(); }

__global__ void touch(int* p) {
  if (threadIdx.x == 0) p[0] = 1;
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

}  // namespace

int main() {
  auto t = Clock::now();
  int n = 0;
  CK(hipGetDeviceCount(&n));
  const double t_init = ms(t);
  t = Clock::now();
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  const double t_ctx = ms(t);
  hipStream_t s1, s2;
  t = Clock::now();
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  const double t_s1 = ms(t);
  t = Clock::now();
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  const double t_s2 = ms(t);
  int* d = nullptr;
  t = Clock::now();
  CK(hipMalloc(&d, 1 << 20));
  const double t_malloc = ms(t);
  t = Clock::now();
  touch<<<1, 64, 0, s1>>>(d);
  CK(hipStreamSynchronize(s1));
  const double t_kernel = ms(t);
  t = Clock::now();
  touch<<<1, 64, 0, nullptr>>>(d);
  CK(hipStreamSynchronize(nullptr));
  const double t_null_kernel = ms(t);
  std::vector<char> h(2048, 1);
  t = Clock::now();
  CK(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
  const double t_copy1 = ms(t);
  t = Clock::now();
  CK(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
  const double t_copy2 = ms(t);
  const size_t len = 64u << 20;
  void* m = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  (void)madvise(m, len, MADV_HUGEPAGE);
  for (size_t o = 0; o < len; o += 4096) static_cast<char*>(m)[o] = 0;
  t = Clock::now();
  CK(hipHostRegister(m, len, hipHostRegisterDefault));
  const double t_reg = ms(t);
  t = Clock::now();
  int mapped = 0;
  for (int r = 0; r < 14; ++r) {
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, static_cast<char*>(m) + size_t(r) * (4u << 20)) == hipSuccess && at.devicePointer)
      ++mapped;
  }
  const double t_attr = ms(t);
  const char* sdma = std::getenv("HSA_ENABLE_SDMA");
  std::printf("{\"HSA_ENABLE_SDMA\": \"%s\", \"runtime_init_ms\": %.3f, \"context_ms\": %.3f, \"stream1_ms\": %.3f, "
              "\"stream2_ms\": %.3f, \"hipMalloc_1MiB_ms\": %.3f, \"first_kernel_ms\": %.3f, \"null_stream_kernel_ms\": "
              "%.3f, \"first_h2d_2KiB_ms\": %.3f, \"second_h2d_2KiB_ms\": %.3f, \"hostRegister_64MiB_ms\": %.3f, "
              "\"pointer_attributes_x14_ms\": %.3f, \"rows_mapped\": %d}\n",
              sdma ? sdma : "", t_init, t_ctx, t_s1, t_s2, t_malloc, t_kernel, t_null_kernel, t_copy1, t_copy2, t_reg,
              t_attr, mapped);
  CK(hipHostUnregister(m));
  munmap(m, len);
  CK(hipFree(d));
  CK(hipStreamDestroy(s1));
  CK(hipStreamDestroy(s2));
  return 0;
}

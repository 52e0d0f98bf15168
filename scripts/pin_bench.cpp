// Host-memory pinning costs on the GPU box (what bin/RS's setup pays before its first DMA).
//   hipcc --offload-arch=gfx950 -O2 -o build/pin_bench scripts/pin_bench.cpp && build/pin_bench [GiB]
// Times, for a buffer of the given size: hipHostMalloc; malloc + first touch (page faults) +
// hipHostRegister of the touched pages (whole, and in 64 MiB windows); the same with
// MADV_HUGEPAGE; and an H2D copy from each to check the pinned rate.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

using Clock = std::chrono::steady_clock;
static double ms(Clock::time_point t0) { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); }
#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e));           \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

static double h2d_gbps(void* dev, const void* host, size_t n) {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  CK(hipMemcpyAsync(dev, host, 64 << 20, hipMemcpyHostToDevice, s));
  CK(hipStreamSynchronize(s));
  const auto t = Clock::now();
  CK(hipMemcpyAsync(dev, host, n, hipMemcpyHostToDevice, s));
  CK(hipStreamSynchronize(s));
  const double t_ms = ms(t);
  CK(hipStreamDestroy(s));
  return n / (t_ms / 1e3) / 1e9;
}

static void touch(uint8_t* p, size_t n, int threads) {
  std::vector<std::thread> th;
  const size_t per = (n / threads + 4095) / 4096 * 4096;
  for (int i = 0; i < threads; ++i)
    th.emplace_back([=] {
      const size_t a = size_t(i) * per, b = std::min(n, a + per);
      if (a < b) std::memset(p + a, i + 1, b - a);
    });
  for (auto& t : th) t.join();
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? std::atof(argv[1]) : 1.4;
  const size_t n = size_t(gib * double(1ull << 30)) / 4096 * 4096;
  auto t = Clock::now();
  int ndev = 0;
  CK(hipGetDeviceCount(&ndev));
  std::printf("hip init %.1f ms (%d devices), buffer %.2f GiB\n", ms(t), ndev, n / double(1ull << 30));
  void* dev = nullptr;
  t = Clock::now();
  CK(hipMalloc(&dev, n));
  std::printf("hipMalloc %.1f ms\n", ms(t));

  {
    t = Clock::now();
    void* p = nullptr;
    CK(hipHostMalloc(&p, n, hipHostMallocDefault));
    const double a = ms(t);
    std::printf("hipHostMalloc %.1f ms (%.1f GB/s); H2D %.1f GB/s\n", a, n / (a / 1e3) / 1e9, h2d_gbps(dev, p, n));
    t = Clock::now();
    CK(hipHostFree(p));
    std::printf("  hipHostFree %.1f ms\n", ms(t));
  }
  for (int huge = 0; huge < 2; ++huge)
    for (int threads : {1, 8}) {
      uint8_t* p = static_cast<uint8_t*>(mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
      if (huge) madvise(p, n, MADV_HUGEPAGE);
      t = Clock::now();
      touch(p, n, threads);
      const double a = ms(t);
      t = Clock::now();
      CK(hipHostRegister(p, n, hipHostRegisterDefault));
      const double b = ms(t);
      std::printf("%s touch x%d %.1f ms + hipHostRegister(whole) %.1f ms (%.1f GB/s); H2D %.1f GB/s\n",
                  huge ? "THP " : "4KiB", threads, a, b, n / (b / 1e3) / 1e9, h2d_gbps(dev, p, n));
      CK(hipHostUnregister(p));
      munmap(p, n);
    }
  {
    uint8_t* p = static_cast<uint8_t*>(mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
    madvise(p, n, MADV_HUGEPAGE);
    touch(p, n, 8);
    const size_t w = 64ull << 20;
    t = Clock::now();
    for (size_t a = 0; a < n; a += w) CK(hipHostRegister(p + a, std::min(w, n - a), hipHostRegisterDefault));
    const double b = ms(t);
    std::printf("THP  hipHostRegister in 64 MiB windows %.1f ms (%.1f GB/s)\n", b, n / (b / 1e3) / 1e9);
    for (size_t a = 0; a < n; a += w) CK(hipHostUnregister(p + a));
    munmap(p, n);
  }
  CK(hipFree(dev));
  return 0;
}

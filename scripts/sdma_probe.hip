// Copy-engine probe: device-to-device bandwidth of hipMemcpyDeviceToDeviceNoCU (SDMA, no compute
// units) against the blit-kernel copy, alone and beside a compute-bound kernel that holds every CU.
// Question it answers: can the wide decode's survivor copy (102 rows x 8.4 MB at k=128) run on the
// copy engines under the MFMA-bound GEMM instead of inside it?
//   hipcc --offload-arch=gfx950 -O2 scripts/sdma_probe.hip -o /tmp/sdma_probe && /tmp/sdma_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

// ALU-bound spin: every lane runs `iters` dependent FMAs; the result is stored so it is kept.
__global__ void spin_kernel(float* out, int iters) {
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  for (int i = 0; i < iters; ++i) a = __builtin_fmaf(a, b, 1e-7f);
  if (a == 12345.0f) out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

static float elapsed(hipEvent_t a, hipEvent_t b) {
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

int main(int argc, char** argv) {
  const size_t rows = argc > 1 ? std::atoll(argv[1]) : 102;
  const size_t width = argc > 2 ? std::atoll(argv[2]) : 8388608;  // 1 GiB / 128
  const size_t pitch_src = width + 256, pitch_dst = width + 512;   // pitched rows, as the codec's
  const size_t bytes = rows * width;
  char *src, *dst;
  float* sink;
  CK(hipMalloc(&src, rows * pitch_src));
  CK(hipMalloc(&dst, rows * pitch_dst));
  CK(hipMalloc(&sink, 1 << 24));
  CK(hipMemset(src, 7, rows * pitch_src));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  std::vector<hipStream_t> st(9);
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));

  // mode 0: one 2-D copy per stream; mode 1: one 1-D copy per row; mode 2: one 1-D copy of the
  // stream's whole span (contiguous bytes, pitches included)
  int mode = 0;
  auto copy2d = [&](hipStream_t s, size_t r0, size_t r1, hipMemcpyKind kind) {
    if (mode == 0) {
      CK(hipMemcpy2DAsync(dst + r0 * pitch_dst, pitch_dst, src + r0 * pitch_src, pitch_src, width, r1 - r0, kind, s));
    } else if (mode == 1) {
      for (size_t r = r0; r < r1; ++r) CK(hipMemcpyAsync(dst + r * pitch_dst, src + r * pitch_src, width, kind, s));
    } else {
      CK(hipMemcpyAsync(dst + r0 * pitch_src, src + r0 * pitch_src, (r1 - r0) * pitch_src, kind, s));
    }
  };
  // split the rows over `ns` streams, all joined into st[0] via events
  auto copy_split = [&](int ns, hipMemcpyKind kind) {
    std::vector<hipEvent_t> done(ns);
    CK(hipEventRecord(e0, st[0]));
    for (int i = 0; i < ns; ++i) {
      CK(hipStreamWaitEvent(st[1 + i], e0, 0));
      copy2d(st[1 + i], rows * i / ns, rows * (i + 1) / ns, kind);
      CK(hipEventCreateWithFlags(&done[i], hipEventDisableTiming));
      CK(hipEventRecord(done[i], st[1 + i]));
      CK(hipStreamWaitEvent(st[0], done[i], 0));
    }
    CK(hipEventRecord(e1, st[0]));
    CK(hipStreamSynchronize(st[0]));
    for (auto& d : done) CK(hipEventDestroy(d));
    return elapsed(e0, e1);
  };

  // calibrate the spin kernel to ~1 ms on every CU (4 waves per CU)
  int iters = 1 << 14;
  for (int t = 0; t < 3; ++t) {
    CK(hipEventRecord(e0, st[0]));
    spin_kernel<<<cus, 256, 0, st[0]>>>(sink, iters);
    CK(hipEventRecord(e1, st[0]));
    CK(hipStreamSynchronize(st[0]));
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
        CK(hipEventRecord(e0, st[0]));
        spin_kernel<<<cus, 256, 0, st[0]>>>(sink, iters);
        CK(hipEventRecord(e1, st[0]));
        CK(hipStreamSynchronize(st[0]));
        best_spin = std::min(best_spin, elapsed(e0, e1));
        std::vector<hipEvent_t> done(ns);
        CK(hipEventRecord(e0, st[0]));
        for (int i = 0; i < ns; ++i) {
          CK(hipStreamWaitEvent(st[1 + i], e0, 0));
          copy2d(st[1 + i], rows * i / ns, rows * (i + 1) / ns, kd.kind);
          CK(hipEventCreateWithFlags(&done[i], hipEventDisableTiming));
          CK(hipEventRecord(done[i], st[1 + i]));
        }
        spin_kernel<<<cus, 256, 0, st[0]>>>(sink, iters);
        for (int i = 0; i < ns; ++i) CK(hipStreamWaitEvent(st[0], done[i], 0));
        CK(hipEventRecord(e2, st[0]));
        CK(hipStreamSynchronize(st[0]));
        best_both = std::min(best_both, elapsed(e0, e2));
        for (auto& d : done) CK(hipEventDestroy(d));
      }
      std::printf("{\"mode\": %d, \"overlap\": \"%s\", \"streams\": %d, \"spin_ms\": %.3f, \"spin_plus_copy_ms\": %.3f}\n", mode, kd.name, ns,
                  best_spin, best_both);
    }
  }
  CK(hipFree(src));
  CK(hipFree(dst));
  CK(hipFree(sink));
  return 0;
}

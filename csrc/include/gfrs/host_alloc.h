// Pinned host buffers for the file codecs without hipHostMalloc's cost.
//
// Measured on the MI355X box (scripts/pin_bench.cpp, profiles/host_pipeline/r03_setup): pinning 1.4 GiB with
// hipHostMalloc takes ~360 ms (and hipHostFree ~230 ms) — 4 GB/s of page zeroing, pinning and IOMMU
// mapping in 4 KiB pages, on the critical path of every bin/RS run before its first DMA. The same
// bytes as anonymous memory backed by transparent huge pages (MADV_HUGEPAGE), first-touched by 8
// threads (12 ms), then hipHostRegister'ed (3 ms: 2 MiB pages pin and map ~100x faster) reach the
// same H2D rate (57 GB/s). The reference pins with cudaMallocHost (src/encode.cu:389-398).
#pragma once

#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "gfrs/codec_file.h"

namespace gfrs {

namespace host_alloc_detail {
inline std::mutex& mu() {
  static std::mutex m;
  return m;
}
inline std::map<uint8_t*, size_t>& sizes() {
  static auto* m = new std::map<uint8_t*, size_t>();
  return *m;
}
}  // namespace host_alloc_detail

// Zero-filled, hipHostRegister'ed, huge-page backed buffer of >= n bytes (nullptr on failure).
inline uint8_t* thp_pinned_alloc(size_t n, int touch_threads = 8) {
  constexpr size_t kHuge = 2u << 20;
  const size_t len = std::max<size_t>(kHuge, (n + kHuge - 1) / kHuge * kHuge);
  void* m = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (m == MAP_FAILED) return nullptr;
  auto* p = static_cast<uint8_t*>(m);
  (void)madvise(p, len, MADV_HUGEPAGE);  // best effort: 4 KiB pages still work, just slower
  // first touch in parallel: the kernel zeroes (and THP-allocates) the pages on these threads
  const int T = len >= (256u << 20) ? std::max(1, touch_threads) : 1;
  const size_t per = (len / size_t(T) + kHuge - 1) / kHuge * kHuge;
  std::vector<std::thread> th;
  for (int i = 0; i < T; ++i)
    th.emplace_back([=] {
      const size_t a = size_t(i) * per, b = std::min(len, a + per);
      for (size_t o = a; o < b; o += 4096) p[o] = 0;  // one store per 4 KiB page faults it in
    });
  for (auto& t : th) t.join();
  // portable + mapped: every device of the process sees the rows (the multi-device zero-copy
  // pipeline maps them per device, gemm_host_multi)
  if (hipHostRegister(p, len, hipHostRegisterPortable | hipHostRegisterMapped) != hipSuccess) {
    // registration refused (e.g. a locked-memory limit): fall back to the runtime's own pinned
    // allocator rather than failing the codec
    munmap(p, len);
    void* q = nullptr;
    if (hipHostMalloc(&q, n ? n : 1, hipHostMallocPortable | hipHostMallocMapped) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> g(host_alloc_detail::mu());
    host_alloc_detail::sizes()[static_cast<uint8_t*>(q)] = 0;  // 0: hipHostFree on release
    return static_cast<uint8_t*>(q);
  }
  std::lock_guard<std::mutex> g(host_alloc_detail::mu());
  host_alloc_detail::sizes()[p] = len;
  return p;
}

inline void thp_pinned_free(uint8_t* p) {
  size_t len = 0;
  {
    std::lock_guard<std::mutex> g(host_alloc_detail::mu());
    auto it = host_alloc_detail::sizes().find(p);
    if (it == host_alloc_detail::sizes().end()) return;
    len = it->second;
    host_alloc_detail::sizes().erase(it);
  }
  if (len == 0) {  // the hipHostMalloc fallback
    (void)hipHostFree(p);
    return;
  }
  (void)hipHostUnregister(p);
  munmap(p, len);
}

// HostAlloc for the file codecs (gfrs/codec_file.h, gfrs/stream_codec.h).
inline HostAlloc thp_pinned_host_alloc() { return {[](size_t n) { return thp_pinned_alloc(n); }, thp_pinned_free}; }

}  // namespace gfrs

// Per-device, thread-safe launch-time caches.
//
// One process may drive several GPUs from several host threads (gemm_host_multi, one thread per
// device like the reference's GPU_thread_func, src/encode.cu:240-292), so anything a launcher
// learns about "the device" — the >64 KiB dynamic-LDS opt-in of a kernel, the CU count, an
// occupancy-driven variant choice — is keyed by the HIP device that is current on the calling
// thread and guarded by a mutex. Lookups after the first are a map probe under an uncontended lock.
#pragma once

#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <utility>

namespace gfrs {

inline int current_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  return dev;
}

// Opts kernel `fn` into `bytes` of dynamic LDS on the current device, once per (fn, device).
inline hipError_t ensure_lds_optin(const void* fn, int bytes = 160 * 1024) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int>* done = new std::map<std::pair<const void*, int>, int>();
  const std::pair<const void*, int> key{fn, current_device()};
  std::lock_guard<std::mutex> g(mu);
  auto it = done->find(key);
  if (it != done->end() && it->second >= bytes) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) (*done)[key] = bytes;
  return e;
}

// Compute units of the current device (256 on MI355X), cached per device.
inline int device_cu_count() {
  static std::mutex mu;
  static std::map<int, int>* cache = new std::map<int, int>();
  const int dev = current_device();
  std::lock_guard<std::mutex> g(mu);
  auto it = cache->find(dev);
  if (it != cache->end()) return it->second;
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  (*cache)[dev] = n;
  return n;
}

// A small per-(device, key) memo: `get_or(key, make)` runs `make()` once per device and key.
// `make` runs under the lock (it only queries the runtime, e.g. occupancy).
template <class Key, class Value>
class DeviceMemo {
 public:
  template <class F>
  Value get_or(const Key& key, F&& make) {
    const std::pair<int, Key> k{current_device(), key};
    std::lock_guard<std::mutex> g(mu_);
    auto it = map_.find(k);
    if (it != map_.end()) return it->second;
    Value v = make();
    map_.emplace(k, v);
    return v;
  }

 private:
  std::mutex mu_;
  std::map<std::pair<int, Key>, Value> map_;
};

}  // namespace gfrs

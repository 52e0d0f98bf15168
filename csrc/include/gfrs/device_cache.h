// Per-device, thread-safe launch-time caches.
//
// One process may drive several GPUs from several host threads (gemm_host_multi, one thread per
// device like the reference's GPU_thread_func, src/encode.cu:240-292), so anything a launcher
// learns about "the device" — the >64 KiB dynamic-LDS opt-in of a kernel, the CU count, an
// occupancy-driven variant choice — is keyed by the HIP device that is current on the calling
// thread and guarded by a mutex. Lookups after the first are a map probe under an uncontended lock.
#pragma once

#include "gfrs/tune.h"
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
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

// Chunk slots of a persistent FP4 grid (blocks = slots x groups). With several M-groups a slot's
// blocks must share an XCD, so slots are a multiple of 8. With one group every block owns its chunk
// stream outright and the slot count is free: the grid then leaves GFRS_TUNE=fp4_free_cus=N compute units
// (default 0) without a block, so a one-workgroup side kernel — the decode-system solve of the next
// step — finds an empty CU instead of holding one of the GEMM's blocks back (a persistent GEMM with
// one block per CU ends when its last block does: a 50 us solve in front of one block delays the
// whole kernel by 50 us).
inline int64_t persistent_slots(int occ, int groups, int64_t nchunks) {
  static const int free_cus = int(std::max<int64_t>(0, tune_int("fp4_free_cus", 0)));
  const int64_t full = int64_t(device_cu_count()) * occ / groups;
  if (groups == 1 && free_cus > 0) {
    const int64_t s = std::max<int64_t>(1, full - free_cus);
    return std::min<int64_t>(s, nchunks);
  }
  const int64_t s = std::max<int64_t>(8, full / 8 * 8);
  return std::min<int64_t>(s, (nchunks + 7) / 8 * 8);
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

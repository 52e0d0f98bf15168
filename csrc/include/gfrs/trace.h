// roctx ranges for rocprofv3 --marker-trace (the reference has only CUDA events and
// printf; here every pipeline stage is a named range on the timeline). The roctx library is
// dlopen'ed on first use, so binaries carry no hard dependency: without it, or without a profiler
// attached, a range costs one predictable branch / one cheap library call.
#pragma once

#include <dlfcn.h>

namespace gfrs {

struct Roctx {
  using PushFn = int (*)(const char*);
  using PopFn = int (*)();
  using MarkFn = void (*)(const char*);
  PushFn push = nullptr;
  PopFn pop = nullptr;
  MarkFn mark = nullptr;
  static const Roctx& get() {
    static const Roctx r = [] {
      Roctx x;
      void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
      if (!h) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
      if (h) {
        x.push = reinterpret_cast<PushFn>(dlsym(h, "roctxRangePushA"));
        x.pop = reinterpret_cast<PopFn>(dlsym(h, "roctxRangePop"));
        x.mark = reinterpret_cast<MarkFn>(dlsym(h, "roctxMarkA"));
        if (!x.push || !x.pop) x.push = nullptr, x.pop = nullptr;
      }
      return x;
    }();
    return r;
  }
  static bool available() { return get().push != nullptr; }
};

// RAII range: TraceRange r("encode/window");
class TraceRange {
 public:
  explicit TraceRange(const char* name) : on_(Roctx::get().push != nullptr) {
    if (on_) Roctx::get().push(name);
  }
  ~TraceRange() {
    if (on_) Roctx::get().pop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;

 private:
  bool on_;
};

inline void trace_mark(const char* name) {
  if (Roctx::get().mark) Roctx::get().mark(name);
}

}  // namespace gfrs

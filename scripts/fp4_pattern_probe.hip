// No-math probe of the wide FP4 kernels' memory pattern (k = 128 decode shape, 1 GiB): is the
// decode's time set by its access pattern rather than by its matrix-core work?
//
// Same persistent grid (one 256-thread block per CU, LDS-DMA rings), same per-wave access as
// gf_mfma_fp4tm.hip: each wave moves 64 columns of a 256-column chunk; one global_load_lds_dwordx4
// per 1-KiB ring slot reads 16 rows x 64 B; the fused copy stores 16 B per lane of each slot; the
// outputs are 2-byte stores per lane (rows 4t + 2h + u). The next chunk's 8 DMAs are issued before
// the current chunk's stores, and the wait counts exactly the ops issued after them.
//   mode 0: reads only; mode 1: + copies (rows >= ncopy to a sink); mode 2: + the output stores;
//   mode 3: mode 1 with block-wide copies (each store instruction 4 rows x 256 B from the four
//   waves' rings, two barriers per chunk); mode 4: mode 3 + the output stores.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o bin/fp4_pattern_probe scripts/fp4_pattern_probe.hip
//   bin/fp4_pattern_probe [k=128] [m=26] [ncopy=102] [reps=15]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

using u32x4 = unsigned __attribute__((ext_vector_type(4)));
template <typename T>
using gptr = __attribute__((address_space(1))) T*;
using lds_u8 = __attribute__((address_space(3))) uint8_t;

constexpr int kSlots = 8;
constexpr int kTiles = 7;

template <int MODE>
__global__ __launch_bounds__(256, 1) void probe_kernel(const uint64_t* __restrict__ inp, const uint64_t* __restrict__ cpy,
                                                       const uint64_t* __restrict__ outp, uint64_t sink,
                                                       int64_t nchunks, int64_t slots) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  const int drow = lane >> 2, dcol = wave * 64 + 16 * (lane & 3);
  lds_u8* ring = (lds_u8*)smem + size_t(wave) * 2 * kSlots * 1024;  // two chunk buffers per wave
  const uint64_t snk = sink + uint64_t((blockIdx.x * 4 + wave) % 256) * 1024 + 16 * lane;
  uint64_t rp[kSlots], cp[kSlots];
  for (int p = 0; p < kSlots; ++p) {
    rp[p] = inp[16 * p + drow];
    cp[p] = cpy[16 * p + drow];
  }
  const int64_t first = blockIdx.x;
  if (first >= nchunks) return;
  auto dma = [&](int64_t ch, int buf) {
    const int64_t col = (ch < nchunks ? ch : first) * 256 + dcol;
#pragma unroll
    for (int p = 0; p < kSlots; ++p)
      __builtin_amdgcn_global_load_lds((gptr<const void>)(rp[p] + uint64_t(col)), ring + (buf * kSlots + p) * 1024, 16,
                                       0, 0);
  };
  dma(first, 0);
  int buf = 0;
  // stores per chunk and wave (copies, outputs): issued after the next chunk's DMAs
  constexpr int kStores = (MODE >= 1 ? kSlots : 0) + (MODE == 2 || MODE == 4 ? 2 * kTiles : 0);
  constexpr bool kWide = MODE >= 3;
  // block-wide copy: this lane's row 4 * wave + lane / 16 of a slot, columns 16 * (lane % 16) of the
  // block's 256, found in the ring of wave (lane % 16) / 4
  const int wrow = 4 * wave + (lane >> 4), wcol = 16 * (lane & 15);
  lds_u8* wring = (lds_u8*)smem + size_t((lane & 15) >> 2) * 2 * kSlots * 1024 + wrow * 64 + 16 * (lane & 3);
  uint64_t wcp[kSlots];
  for (int p = 0; p < kSlots; ++p) wcp[p] = cpy[16 * p + wrow];
  for (int64_t ch = first; ch < nchunks; ch += slots) {
    if constexpr (kWide) __syncthreads();  // every wave is done reading the buffer refilled now
    dma(ch + slots, buf ^ 1);
    // this chunk's DMAs have landed: younger are the previous chunk's stores and the next chunk's 8
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kSlots + kStores) : "memory");
    if constexpr (kWide) __syncthreads();  // ... in every wave's ring
    const int64_t col = ch * 256 + dcol;
    u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int p = 0; p < kSlots; ++p) {
      u32x4 v;
      const uint32_t addr = uint32_t(reinterpret_cast<uintptr_t>(ring + (buf * kSlots + p) * 1024 + 16 * lane));
      asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
      acc ^= v;
      if constexpr (MODE >= 1 && !kWide) {
        const uint64_t d = cp[p];
        __builtin_nontemporal_store(v, (gptr<u32x4>)(d ? d + uint64_t(col) : snk));
      }
      if constexpr (kWide) {
        u32x4 wv;
        const uint32_t waddr = uint32_t(reinterpret_cast<uintptr_t>(wring + (buf * kSlots + p) * 1024));
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(wv) : "v"(waddr) : "memory");
        const uint64_t d = wcp[p];
        __builtin_nontemporal_store(wv, (gptr<u32x4>)(d ? d + uint64_t(ch * 256 + wcol) : snk));
      }
    }
    if constexpr (MODE == 2 || MODE == 4) {
      const int64_t colw = ch * 256 + wave * 64 + 2 * c;
#pragma unroll
      for (int t = 0; t < kTiles; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const uint64_t o = outp[4 * t + 2 * h + u];
          *(gptr<uint16_t>)(o ? o + uint64_t(colw) : snk) = uint16_t(acc[u] >> (4 * t));
        }
    }
    buf ^= 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int main(int argc, char** argv) {
  const int k = argc > 1 ? std::atoi(argv[1]) : 128;
  const int m = argc > 2 ? std::atoi(argv[2]) : 26;
  const int ncopy = argc > 3 ? std::atoi(argv[3]) : 102;
  const int reps = argc > 4 ? std::atoi(argv[4]) : 15;
  const int64_t C = (int64_t(1) << 30) / k / 256 * 256;  // bytes per row, whole chunks
  const int64_t nchunks = C / 256;
  std::vector<uint64_t> hin(128, 0), hcp(128, 0), hout(32, 0);
  std::vector<void*> bufs;
  for (int j = 0; j < 128; ++j) {
    void* p;
    CHECK(hipMalloc(&p, size_t(C)));
    CHECK(hipMemset(p, j, size_t(C)));
    bufs.push_back(p);
    hin[j] = uint64_t(p);
  }
  for (int j = 0; j < ncopy && j < 128; ++j) {
    void* p;
    CHECK(hipMalloc(&p, size_t(C)));
    bufs.push_back(p);
    hcp[j] = uint64_t(p);
  }
  for (int i = 0; i < m && i < 28; ++i) {
    void* p;
    CHECK(hipMalloc(&p, size_t(C)));
    bufs.push_back(p);
    hout[i] = uint64_t(p);
  }
  (void)k;
  uint64_t *din, *dcp, *dout;
  void* sink;
  CHECK(hipMalloc(&din, 128 * 8));
  CHECK(hipMalloc(&dcp, 128 * 8));
  CHECK(hipMalloc(&dout, 32 * 8));
  CHECK(hipMalloc(&sink, 256 * 1024));
  CHECK(hipMemcpy(din, hin.data(), 128 * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dcp, hcp.data(), 128 * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dout, hout.data(), 32 * 8, hipMemcpyHostToDevice));
  int cus = 256;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t lds = 150 * 1024;  // one block per CU, as the FP4 kernels
  const void* fns[5] = {(const void*)&probe_kernel<0>, (const void*)&probe_kernel<1>, (const void*)&probe_kernel<2>,
                        (const void*)&probe_kernel<3>, (const void*)&probe_kernel<4>};
  for (auto f : fns) CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const int64_t slots = std::min<int64_t>(cus, nchunks);
  for (int mode = 0; mode < 5; ++mode) {
    std::vector<float> ts;
    for (int r = 0; r < reps + 2; ++r) {
      CHECK(hipEventRecord(a));
      if (mode == 0)
        probe_kernel<0><<<unsigned(slots), 256, lds>>>(din, dcp, dout, uint64_t(sink), nchunks, slots);
      else if (mode == 1)
        probe_kernel<1><<<unsigned(slots), 256, lds>>>(din, dcp, dout, uint64_t(sink), nchunks, slots);
      else if (mode == 2)
        probe_kernel<2><<<unsigned(slots), 256, lds>>>(din, dcp, dout, uint64_t(sink), nchunks, slots);
      else if (mode == 3)
        probe_kernel<3><<<unsigned(slots), 256, lds>>>(din, dcp, dout, uint64_t(sink), nchunks, slots);
      else
        probe_kernel<4><<<unsigned(slots), 256, lds>>>(din, dcp, dout, uint64_t(sink), nchunks, slots);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      if (r >= 2) ts.push_back(ms * 1000.f);
    }
    std::sort(ts.begin(), ts.end());
    const double bytes = double(C) * (128 + (mode >= 1 ? ncopy : 0) + (mode == 2 || mode == 4 ? m : 0));
    std::printf("{\"mode\": %d, \"median_us\": %.1f, \"min_us\": %.1f, \"TBps\": %.2f}\n", mode, ts[ts.size() / 2],
                ts[0], bytes / (ts[ts.size() / 2] * 1e-6) / 1e12);
  }
  for (void* p : bufs) CHECK(hipFree(p));
  return 0;
}

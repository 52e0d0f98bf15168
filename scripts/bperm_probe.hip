// Lookup-rate probe for a GF(2^16) multiply-by-constant engine built on cross-lane table lookups.
//
// Multiplying a 16-bit symbol by a constant c is GF(2)-linear, so c*s = XOR over the symbol's bit
// chunks of c*(chunk << shift). With 64-entry tables held one entry per lane in a VGPR,
// ds_bpermute_b32 looks up a 6-bit chunk per lane and returns 32 bits: the 16-bit products of two
// output coefficients at once. A symbol then costs 3 lookups (chunks of 6, 6, 4 bits) per pair of
// outputs, against the v_perm engine's 3-bit lookups (gf_gemm16.hip: 23 VALU per symbol and
// 4 outputs). The alternative is an LDS table indexed by a whole byte (ds_read_b32, 2 lookups per
// pair, random banks).
//
// Build: hipcc -O3 --offload-arch=gfx950 -o build/bperm_probe scripts/bperm_probe.hip
// Run:   build/bperm_probe        (one JSON line per case; "sem" checks the address masking first)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

// lane l reads data[(addr >> 2) & 63]? addr carries garbage above bit 7 and in bits 0..1
__global__ void sem_kernel(const unsigned* garbage, unsigned* out) {
  const int l = threadIdx.x;
  const unsigned data = 1000u * l + 7u;
  const unsigned idx = (l * 37u + 11u) & 63u;
  const unsigned addr = (garbage[l] & ~0xFFu) | (idx << 2) | (garbage[l] & 3u);
  out[l] = unsigned(__builtin_amdgcn_ds_bpermute(int(addr), int(data)));
  out[64 + l] = 1000u * idx + 7u;
}

// U independent symbol dwords per lane (2 symbols each), 4 outputs as 2 pairs: per symbol 3 shifts,
// 6 bpermutes, 4 XOR (acc ^ a ^ b, acc ^ c); the data word is stepped by an LCG (2 VALU) so no
// lookup can be hoisted. Returns an XOR of everything so nothing is dead.
template <int U>
__global__ __launch_bounds__(256) void bperm_rate(unsigned seed, int iters, unsigned* sink) {
  const int l = threadIdx.x & 63;
  unsigned tab[6];
#pragma unroll
  for (int t = 0; t < 6; ++t) tab[t] = (l * 2654435761u) ^ (t * 40503u) ^ seed;
  unsigned x[U], acc[U][4];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    x[u] = seed * (threadIdx.x + 1) + u * 977u + blockIdx.x;
    acc[u][0] = acc[u][1] = acc[u][2] = acc[u][3] = 0;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned v = x[u];
      // low symbol: chunks [0,6) [6,12) [12,16); high symbol: [16,22) [22,28) [28,32)
      const int s0 = int(v << 2), s1 = int(v >> 4), s2 = int(v >> 10);
      const int s3 = int(v >> 14), s4 = int(v >> 20), s5 = int(v >> 26);
      const int sel[6] = {s0, s1, s2, s3, s4, s5};
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
          const unsigned a = unsigned(__builtin_amdgcn_ds_bpermute(sel[3 * h + 0], int(tab[3 * pr + 0])));
          const unsigned b = unsigned(__builtin_amdgcn_ds_bpermute(sel[3 * h + 1], int(tab[3 * pr + 1])));
          const unsigned c = unsigned(__builtin_amdgcn_ds_bpermute(sel[3 * h + 2], int(tab[3 * pr + 2])));
          acc[u][2 * h + pr] = __builtin_amdgcn_bitop3_b32(acc[u][2 * h + pr], a, b, 0x96) ^ c;
        }
      x[u] = v * 1664525u + 1013904223u;
    }
  }
  unsigned r = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) r ^= acc[u][0] ^ acc[u][1] ^ acc[u][2] ^ acc[u][3];
  if (r == 0x12345678u) sink[0] = r;
}

// Byte-indexed LDS tables: per symbol 2 byte lookups per output pair (ds_read_b32 at 4 * byte).
template <int U>
__global__ __launch_bounds__(256) void lds_rate(unsigned seed, int iters, unsigned* sink) {
  __shared__ unsigned tab[4][256];  // [chunk (lo, hi byte) x pair][byte]
  for (int i = threadIdx.x; i < 4 * 256; i += 256) (&tab[0][0])[i] = i * 2654435761u ^ seed;
  __syncthreads();
  unsigned x[U], acc[U][4];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    x[u] = seed * (threadIdx.x + 1) + u * 977u + blockIdx.x;
    acc[u][0] = acc[u][1] = acc[u][2] = acc[u][3] = 0;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned v = x[u];
      const unsigned b[4] = {v & 255u, (v >> 8) & 255u, (v >> 16) & 255u, v >> 24};
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr)
          acc[u][2 * h + pr] ^= tab[2 * pr + 0][b[2 * h]] ^ tab[2 * pr + 1][b[2 * h + 1]];
      x[u] = v * 1664525u + 1013904223u;
    }
  }
  unsigned r = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) r ^= acc[u][0] ^ acc[u][1] ^ acc[u][2] ^ acc[u][3];
  if (r == 0x12345678u) sink[0] = r;
}

template <typename K>
double time_ms(K launch, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  launch();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) launch();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  unsigned *g, *o, *sink;
  CHECK(hipMalloc(&g, 64 * 4));
  CHECK(hipMalloc(&o, 128 * 4));
  CHECK(hipMalloc(&sink, 4));
  std::vector<unsigned> gh(64);
  for (int i = 0; i < 64; ++i) gh[i] = 0xA5A5A5A5u * (i + 3) ^ 0x5C3u * i;
  CHECK(hipMemcpy(g, gh.data(), 64 * 4, hipMemcpyHostToDevice));
  sem_kernel<<<1, 64>>>(g, o);
  std::vector<unsigned> oh(128);
  CHECK(hipMemcpy(oh.data(), o, 128 * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < 64; ++i) bad += oh[i] != oh[64 + i];
  printf("{\"case\": \"sem\", \"mismatches\": %d, \"lane0\": [%u, %u]}\n", bad, oh[0], oh[64]);

  const int iters = 4096;
  for (int wpc : {4, 8, 16}) {  // waves per CU (256-thread blocks)
    const int blocks = cus * wpc / 4;
    auto run_b = [&] { bperm_rate<4><<<blocks, 256>>>(0x1234u, iters, sink); };
    auto run_l = [&] { lds_rate<4><<<blocks, 256>>>(0x1234u, iters, sink); };
    const double mb = time_ms(run_b, 5), ml = time_ms(run_l, 5);
    // symbol-rows (one symbol x one input row, 4 outputs) per launch
    const double syms = double(blocks) * 256 * iters * 4 * 2;
    printf("{\"case\": \"rate\", \"waves_per_cu\": %d, \"bperm_ms\": %.3f, \"bperm_Tsym_rows_s\": %.3f, "
           "\"lds_ms\": %.3f, \"lds_Tsym_rows_s\": %.3f}\n",
           wpc, mb, syms / mb / 1e9, ml, syms / ml / 1e9);
  }
  CHECK(hipGetLastError());
  return 0;
}

// Device helpers of the v_perm GF(2)-linear byte-map kernels (gf_gemm.hip: GF(2^8) / GF(16)
// nibble method; gf_gemm16.hip: GF(2^16)). Included only by .hip translation units.
//
// A byte map L is applied to 4 packed bytes with 3 v_perm_b32 (gfrs/gf256.h: T0[x&7], T1[(x>>3)&7],
// T2[x>>6]); the selectors depend only on the input bytes and are shared by every output.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "gfrs/desc.h"

namespace gfrs {
namespace permdev {

constexpr int kBlock = 256;

struct Sel {
  uint32_t s0, s1, s2;
};

__device__ __forceinline__ Sel make_sel(uint32_t w) {
  return {w & 0x07070707u, (w >> 3) & 0x07070707u, (w >> 6) & 0x03030303u};
}

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));

// 3-input XOR in one VALU op: gfx950's v_bitop3_b32 with truth table 0x96 (a ^ b ^ c).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// acc ^= L0(x0) ^ L1(x1) for two rows: 6 v_perm_b32 + 3 v_bitop3.
template <typename P>
__device__ __forceinline__ uint32_t mac_pair(uint32_t acc, P t0, const Sel& s0, P t1, const Sel& s1) {
  const uint32_t a0 = __builtin_amdgcn_perm(t0[1], t0[0], s0.s0);
  const uint32_t b0 = __builtin_amdgcn_perm(t0[3], t0[2], s0.s1);
  const uint32_t c0 = __builtin_amdgcn_perm(0u, t0[4], s0.s2);
  const uint32_t a1 = __builtin_amdgcn_perm(t1[1], t1[0], s1.s0);
  const uint32_t b1 = __builtin_amdgcn_perm(t1[3], t1[2], s1.s1);
  const uint32_t c1 = __builtin_amdgcn_perm(0u, t1[4], s1.s2);
  return xor3(xor3(xor3(acc, a0, b0), c0, a1), b1, c1);
}

// A byte map's five table words with two of them copied to VGPRs once: a v_perm can read only one
// SGPR (the gfx9 constant bus), and left to itself the compiler re-copies a table word before every
// v_perm that reads it (0.6 v_mov per v_perm in the w = 16 kernel). The asm copy is opaque, so it
// is made once and shared by every word the map is applied to.
struct MapV {
  uint32_t s1, s3, s4;  // (scalar)
  uint32_t v0, v2;      // (vector copies)
};
__device__ __forceinline__ uint32_t vcopy(uint32_t s) {
  uint32_t v;
  asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(s));
  return v;
}
template <typename P>
__device__ __forceinline__ MapV map_v(P t) {
  return {t[1], t[3], t[4], vcopy(t[0]), vcopy(t[2])};
}
// acc ^= L0(x0) ^ L1(x1) for two rows, tables in MapV form: 6 v_perm_b32 + 3 v_bitop3.
__device__ __forceinline__ uint32_t mac_pair_v(uint32_t acc, const MapV& t0, const Sel& s0, const MapV& t1,
                                               const Sel& s1) {
  const uint32_t a0 = __builtin_amdgcn_perm(t0.s1, t0.v0, s0.s0);
  const uint32_t b0 = __builtin_amdgcn_perm(t0.s3, t0.v2, s0.s1);
  const uint32_t c0 = __builtin_amdgcn_perm(0u, t0.s4, s0.s2);
  const uint32_t a1 = __builtin_amdgcn_perm(t1.s1, t1.v0, s1.s0);
  const uint32_t b1 = __builtin_amdgcn_perm(t1.s3, t1.v2, s1.s1);
  const uint32_t c1 = __builtin_amdgcn_perm(0u, t1.s4, s1.s2);
  return xor3(xor3(xor3(acc, a0, b0), c0, a1), b1, c1);
}

// acc ^= L(x) for one GF(2)-linear byte map L on 4 packed bytes: 3 v_perm_b32 + 2 v_bitop3.
template <typename P>
__device__ __forceinline__ uint32_t mac_map(uint32_t acc, P t, const Sel& s) {
  const uint32_t a = __builtin_amdgcn_perm(t[1], t[0], s.s0);
  const uint32_t b = __builtin_amdgcn_perm(t[3], t[2], s.s1);
  const uint32_t c = __builtin_amdgcn_perm(0u, t[4], s.s2);
  return xor3(xor3(acc, a, b), c, 0u);
}

// Descriptor words are wave-uniform and read-only for the kernel's lifetime: reading them through
// the constant address space (4) makes hipcc emit s_load (scalar cache, lgkmcnt) instead of vector
// loads that would share vmcnt with the data stream and serialise the prefetch.
template <typename T>
using cptr = const __attribute__((address_space(4))) T*;
// Data rows through the global address space (1): global_load/store instead of flat_*.
template <typename T>
using gptr = __attribute__((address_space(1))) T*;

struct DescView {
  cptr<uint64_t> in;
  cptr<uint64_t> copy;
  cptr<uint64_t> out;
  cptr<uint32_t> tab;
};

inline DescView view(const void* desc, int k, int m_pad, int batch = 1) {
  const DescLayout l = desc_layout(k, m_pad, batch);
  const char* b = static_cast<const char*>(desc);
  return {(cptr<uint64_t>)(b + l.in_off), (cptr<uint64_t>)(b + l.copy_off), (cptr<uint64_t>)(b + l.out_off),
          (cptr<uint32_t>)(b + l.tab_off)};
}

__device__ __forceinline__ gptr<const u32x4> row_vec(uint64_t base, int64_t off) {
  return (gptr<const u32x4>)(base + uint64_t(off));
}
__device__ __forceinline__ gptr<u32x4> row_vec_w(uint64_t base, int64_t off) {
  return (gptr<u32x4>)(base + uint64_t(off));
}

// A wave-uniform int that the compiler computed on the VALU (e.g. the output tile, which comes out
// of a runtime division: AMDGPU divides in float on the VALU) moved into an SGPR once. Left in a
// VGPR, every table address formed from it is built with 64-bit VALU adds and read back with
// v_readfirstlane before each s_load (32 + 16 VALU per 16-byte group in the k=10 rows kernel).
// The empty asm hides the value's uniformity so the compiler keeps the readfirstlane builtin (it
// drops it for a value it knows is uniform) and inserts the wait states the VALU-write ->
// v_readfirstlane hazard needs itself. (A v_readfirstlane written as inline asm got none: it read
// a stale VGPR and the table s_loads fed by it faulted, gf_gemm_vec_kernel<2,1,2>, round 4.)
// Called at the top of a kernel, before any divergent branch.
__device__ __forceinline__ int sgpr_int(int v) {
  asm volatile("" : "+v"(v));
  return __builtin_amdgcn_readfirstlane(v);
}

// Block -> (column block, output tile) mapping. Blocks b and b+8 share an XCD under the observed
// round-robin dispatch; consecutive `local` ids of one XCD sweep the tiles of one column block.
// Placement only affects speed, never correctness. Grids of fewer than 8 column blocks are not
// padded to 8 (make_grid) and map plainly: padded, their live blocks sat on the first ncb XCDs
// only — for every stripe of a batch, since a row of 8 x ntiles blocks keeps x & 7 = XCD.
struct TileMap {
  int tile;
  int64_t cb0;
};
__device__ __forceinline__ TileMap map_block(int ntiles) {
  const int bid = blockIdx.x;
  if (gridDim.x % (8u * unsigned(ntiles)) != 0) return {bid % ntiles, int64_t(bid / ntiles)};
  const int xcd = bid & 7;
  const int local = bid >> 3;
  return {local % ntiles, int64_t(local / ntiles) * 8 + xcd};
}

template <bool NT>
__device__ __forceinline__ u32x4 ld16(gptr<const u32x4> p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st16(gptr<u32x4> p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

}  // namespace permdev
}  // namespace gfrs

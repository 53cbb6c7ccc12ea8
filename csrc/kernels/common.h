// Shared device helpers for the gfx950 kernels (wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../include/records.h"

#define IGP_WAVE 64

namespace igp {

// Hide a wave-uniform value's uniformity from the compiler, so loads addressed by it are
// issued as vector memory ops: random per-wave gathers (account rows) miss the small scalar
// cache and serialise on it, while a vector load of a broadcast address is one request.
__device__ __forceinline__ int as_vgpr(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

// A kernel's argument struct read with VECTOR loads from the kernarg segment (one dword per
// lane, issued with the kernel's first loads) and rebuilt in SGPRs by v_readlane. The default
// lowering reads it with scalar loads that the compiler re-issues whenever SGPR pressure evicts
// a field (K1: 15 kernarg loads, 39 SGPR spills), each an s_waitcnt lgkmcnt(0) round trip to the
// kernarg segment - measured at ~1,700-2,700 cycles per scalar load on MI355X (SmemLatency,
// profiles/r5/NOTES: "K1's fixed cost"). Here the words stay in one or two VGPRs and a field the
// compiler drops is re-read by v_readlane, not from memory. T must be <= 512 bytes.
template <class T>
__device__ __forceinline__ T kernarg_vgpr() {
  static_assert(sizeof(T) % 4 == 0 && sizeof(T) <= 512, "kernarg_vgpr: 4-byte multiple, <= 512 B");
  constexpr int NW = (int)(sizeof(T) / 4);
  typedef const uint32_t __attribute__((address_space(4)))* kptr_t;  // the constant address space
  const kptr_t kp = (kptr_t)__builtin_amdgcn_kernarg_segment_ptr();
  const int lane = (int)(threadIdx.x & 63);
  uint32_t w[(NW + 63) / 64];
#pragma unroll
  for (int r = 0; r < (NW + 63) / 64; ++r) {
    const int i = as_vgpr(64 * r + lane);
    w[r] = kp[i < NW ? i : 0];
  }
  T out;
  uint32_t* ow = reinterpret_cast<uint32_t*>(&out);
#pragma unroll
  for (int k = 0; k < NW; ++k) ow[k] = (uint32_t)__builtin_amdgcn_readlane((int)w[k >> 6], k & 63);
  return out;
}

// A generic pointer re-derived from a global (address space 1) one: pointers rebuilt from
// integer words (kernarg_vgpr) lose the address space the compiler infers for kernel arguments,
// and their loads / stores would be issued as flat_* instructions (out of order, counted in both
// vmcnt and lgkmcnt); this cast lets the address-space inference see them as global again.
template <class P>
__device__ __forceinline__ void as_global(P*& p) {
  typedef __attribute__((address_space(1))) P* gptr_t;
  p = (P*)(gptr_t)(uintptr_t)(p);  // int -> global -> generic: the inference sees the global origin
}

// Mark a loaded value as used here: keeps the compiler from sinking its load below a branch
// (the load then issues together with the other first-level loads).
__device__ __forceinline__ void keep_issued(int x) { asm volatile("" ::"v"(x)); }

template <class T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, IGP_WAVE);
  return v;
}

template <class T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T u = __shfl_xor(v, o, IGP_WAVE);
    v = u > v ? u : v;
  }
  return v;
}

// exact 2^-r for r in [0, 64] (HLL harmonic terms)
__device__ __forceinline__ double exp2_neg(int r) {
  return __longlong_as_double((long long)(1023 - r) << 52);
}

__device__ __forceinline__ float minmax_scale(float x, float lo, float hi) {
  if (x < lo) return 0.f;
  if (x > hi) return 1.f;
  return (x - lo) / (hi - lo);
}

// onnx_model.go:187-195; identity = the reference's stub log1p (quirk Q1)
__device__ __forceinline__ float log_transform(float x, int identity) {
  if (x <= 0.f) return 0.f;
  if (identity) return x;
  return (float)log1p((double)x);
}

__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

// precise variant (matches the CPU executor to ~1 ulp)
__device__ __forceinline__ float sigmoid_precise(float x) { return 1.f / (1.f + expf(-x)); }

// request ownership (multi-GPU broadcast serving): the row belongs to this rank's shard
__device__ __forceinline__ bool row_owned(const ReqRec& r, const ScoreCfg& c) {
  return !c.owner_filter || ((r.tx_type >> 8) & 0xff) == c.my_rank;
}

}  // namespace igp

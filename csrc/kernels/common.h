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

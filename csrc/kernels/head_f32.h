// Shared pieces of the f32 MLP head (gemm.hip mlp_head_f32_* and the tree->head fused kernel in
// trees.hip): the activation switch and four chained v_mfma_f32_16x16x4_f32.
#pragma once
#include "common.h"

namespace igp {

typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ float act_fn(float v, int act) {
  switch (act) {
    case 1: return v > 0.f ? v : 0.f;
    case 2: return 1.f / (1.f + expf(-v));
    case 3: return tanhf(v);
    default: return v;
  }
}

// lane l supplies A[l & 15][k] and B[k][l & 15] with k = 4 (l >> 4) + j for the j-th of four
// consecutive MFMAs: one 16-B read per operand feeds four MFMAs covering 16 k
__device__ __forceinline__ f32x4 mfma4_f32(const float4& av, const float4& bv, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv.x, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv.y, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bv.z, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bv.w, acc, 0, 0, 0);
  return acc;
}

}  // namespace igp

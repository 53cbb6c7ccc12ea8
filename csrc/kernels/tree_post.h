// TreeEnsemble post transforms on the device, operation for operation the CPU executor's
// (csrc/runtime/trees.cpp post_transform): NONE, LOGISTIC, SOFTMAX, SOFTMAX_ZERO, PROBIT, with
// the binary-classifier expansion of one score into two probability columns.
#pragma once
#include <hip/hip_runtime.h>

namespace igp {

enum TreePostKind : int { TP_NONE = 0, TP_LOGISTIC = 1, TP_SOFTMAX = 2, TP_SOFTMAX_ZERO = 3, TP_PROBIT = 4 };

// Giles' single-precision erfinv (same coefficients and order as the executor)
__device__ __forceinline__ float tp_erfinv(float x) {
  if (!(fabsf(x) < 1.0f)) return isnan(x) ? x : copysignf(INFINITY, x);  // the domain edge (p = 0 or 1)
  float w = -logf((1.0f - x) * (1.0f + x)), p;
  if (w < 5.0f) {
    w -= 2.5f;
    p = 2.81022636e-08f; p = 3.43273939e-07f + p * w; p = -3.5233877e-06f + p * w;
    p = -4.39150654e-06f + p * w; p = 0.00021858087f + p * w; p = -0.00125372503f + p * w;
    p = -0.00417768164f + p * w; p = 0.246640727f + p * w; p = 1.50140941f + p * w;
  } else {
    w = sqrtf(w) - 3.0f;
    p = -0.000200214257f; p = 0.000100950558f + p * w; p = 0.00134934322f + p * w;
    p = -0.00367342844f + p * w; p = 0.00573950773f + p * w; p = -0.0076224613f + p * w;
    p = 0.00943887047f + p * w; p = 1.00167406f + p * w; p = 2.83297682f + p * w;
  }
  return p * x;
}

// binary classifier: aggregated score v (base added) -> o[0..1]; c = the class the trees score
__device__ __forceinline__ void tree_post_binary(int post, int c, int all_positive, float v, float* o) {
  if (post == TP_LOGISTIC) {
    o[c] = 1.f / (1.f + expf(-v));
    o[1 - c] = 1.f / (1.f + expf(v));
    return;
  }
  float z[2];
  z[c] = v;
  z[1 - c] = all_positive ? 1.f - v : -v;
  if (post == TP_PROBIT) {
    z[c] = 1.41421356f * tp_erfinv(2 * z[c] - 1);
    z[1 - c] = 1.41421356f * tp_erfinv(2 * z[1 - c] - 1);
  } else if (post == TP_SOFTMAX || post == TP_SOFTMAX_ZERO) {
    const float m = fmaxf(z[0], z[1]);
    const float a = expf(z[0] - m), b = expf(z[1] - m);
    z[0] = a / (a + b);
    z[1] = b / (a + b);
  }
  o[0] = z[0];
  o[1] = z[1];
}

// multi-column scores already in o[0..n) (base added) -> transformed in place
__device__ __forceinline__ void tree_post_inplace(int post, int n, float* o) {
  if (post == TP_LOGISTIC) {
    for (int k = 0; k < n; ++k) o[k] = 1.f / (1.f + expf(-o[k]));
  } else if (post == TP_SOFTMAX || post == TP_SOFTMAX_ZERO) {
    const bool zero = post == TP_SOFTMAX_ZERO;
    float m = -INFINITY;
    for (int k = 0; k < n; ++k)
      if (!(zero && o[k] == 0.f)) m = fmaxf(m, o[k]);
    float sum = 0.f;
    for (int k = 0; k < n; ++k) {
      if (zero && o[k] == 0.f) continue;
      o[k] = expf(o[k] - m);
      sum += o[k];
    }
    for (int k = 0; k < n; ++k) o[k] = sum > 0 ? o[k] / sum : 0.f;
  } else if (post == TP_PROBIT) {
    for (int k = 0; k < n; ++k) o[k] = 1.41421356f * tp_erfinv(2 * o[k] - 1);
  }
}

}  // namespace igp

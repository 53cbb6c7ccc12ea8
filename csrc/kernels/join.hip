// Join of two branches of a DAG-shaped ONNX model (models/plan.py JoinStep): the Add or
// Concat that brings two chains back together (residual blocks, wide & deep towers).
//
//   op 0 (add)     Y[:, 0:N]         = A[:, 0:N] + B[:, 0:N]
//   op 1 (concat)  Y[:, 0:na]        = A[:, 0:na]
//                  Y[:, na:na + nb]  = B[:, 0:nb]
//
// Memory-bound and small (rows x a few hundred columns): one thread per output element,
// consecutive threads on consecutive columns of a row so every wave reads / writes whole
// 256-byte runs. A, B and Y are f32 or bf16 (the producer's / consumer's activation dtype);
// the add runs in f32. Live rows come from m_ptr when the step is replayed from a graph.
#include "common.h"
#include "launch.h"

namespace igp {

namespace {

__device__ __forceinline__ float load_act(const void* p, int bf16, long i) {
  return bf16 ? bf16_to_f32(static_cast<const uint16_t*>(p)[i]) : static_cast<const float*>(p)[i];
}

__global__ void __launch_bounds__(256) join_kernel(JoinArgs a) {
  const int M = a.m_ptr ? min(*a.m_ptr, a.M) : a.M;
  const int N = a.op == 0 ? a.na : a.na + a.nb;
  const long e = long(blockIdx.x) * 256 + threadIdx.x;
  const int r = int(e / N), c = int(e - long(r) * N);
  if (r >= M) return;
  float v;
  if (a.op == 0) {
    v = load_act(a.A, a.a_bf16, long(r) * a.lda + c) + load_act(a.B, a.b_bf16, long(r) * a.ldb + c);
  } else {
    v = c < a.na ? load_act(a.A, a.a_bf16, long(r) * a.lda + c) : load_act(a.B, a.b_bf16, long(r) * a.ldb + c - a.na);
  }
  const long o = long(r) * a.ldy + c;
  if (a.y_bf16) static_cast<uint16_t*>(a.Y)[o] = f32_to_bf16(v);
  else static_cast<float*>(a.Y)[o] = v;
}

}  // namespace

void launch_join(const JoinArgs& a, hipStream_t st) {
  const long n = long(a.M) * (a.op == 0 ? a.na : a.na + a.nb);
  if (n <= 0) return;
  IGP_LAUNCH(join_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, st, a);
}

}  // namespace igp

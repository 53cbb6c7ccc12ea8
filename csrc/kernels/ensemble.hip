// K5 rules_ensemble tail + K10 metrics histogram.
//
// The rule predicates run inside feature_assemble (they need only raw features); this
// kernel combines the rule score with the ML score (engine.go:276-310):
//   final = int(RuleWeight*rule + MLWeight*(ml*100)), cap 100; action by thresholds;
//   ML_HIGH_RISK appended when ml > 0.7 (its weight is not added, quirk Q13).
// The heuristic model (mockPredict, onnx_model.go:258-308) is evaluated here in float64
// with the reference's addition order, so scores match the Go arithmetic bit-for-bit.
// Metrics (score histogram, action counts) are aggregated per block in LDS, then one
// global atomic per bucket per block.
#include "ensemble.h"

namespace igp {

__global__ void __launch_bounds__(256) ensemble_kernel(EnsembleArgs a) {
  __shared__ unsigned int cnt[MET_N];
  const int tid = threadIdx.x;
  if (a.metrics) {
    for (int i = tid; i < MET_N; i += 256) cnt[i] = 0;
    __syncthreads();
  }
  const int row = blockIdx.x * 256 + tid;
  if (row < a.n_rows) ensemble_row(a, row, false, 0.f, a.metrics ? cnt : nullptr);
  if (a.metrics) {
    __syncthreads();
    ensemble_metrics_flush(a, cnt, tid, 256);
  }
}

void launch_ensemble(const EnsembleArgs& a, hipStream_t st) {
  if (a.n_rows <= 0) return;
  IGP_LAUNCH(ensemble_kernel, dim3((a.n_rows + 255) / 256), dim3(256), 0, st, a);
}

}  // namespace igp

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
#include "common.h"
#include "launch.h"

namespace igp {

__device__ __forceinline__ double heuristic_ml(const float* x) {
  double s = 0.0;
  if (x[0] > 0.5f) s += 0.2;
  if (x[2] > 0.5f) s += 0.15;
  if (x[5] > 0.3f) s += 0.15;
  if (x[6] > 0.25f) s += 0.1;
  if (x[19] > 0.f || x[20] > 0.f) s += 0.15;
  if (x[21] > 0.f) s += 0.25;
  if (x[9] < 0.02f && x[26] > 0.5f) s += 0.2;
  if (x[25] > 0.f) s += 0.15;
  if (x[15] < 0.01f && x[28] > 0.f) {
    if (x[11] > x[10] * 0.8f) s += 0.2;
  }
  return s > 1.0 ? 1.0 : s;
}

constexpr int MET_HIST = 0, MET_ACTION = 101, MET_MLHIGH = 105, MET_ROWS = 106, MET_BLACKLIST = 107,
              MET_N = 128;

__global__ void __launch_bounds__(256) ensemble_kernel(EnsembleArgs a) {
  __shared__ unsigned int cnt[MET_N];
  const int tid = threadIdx.x;
  if (a.metrics) {
    for (int i = tid; i < MET_N; i += 256) cnt[i] = 0;
    __syncthreads();
  }
  const int row = blockIdx.x * 256 + tid;
  const int n_live = a.hdr->n;
  if (row < a.n_rows) {
    if (row >= n_live || (a.feat[row].flags & FR_NOT_OWNED)) {
      a.out[row] = ResultRec{0u, 0.f};  // padding / another rank's request: zero (merge by sum)
    } else {
      const ScoreCfg& cfg = *a.cfg;
      const FeatRec& f = a.feat[row];
      uint32_t reasons = (uint32_t)f.reserved0;
      const int rule = f.reserved1;
      double ml = 0.0;
      if (cfg.model_kind == 1) {
        ml = heuristic_ml(a.X + (size_t)row * a.x_stride);
      } else if (cfg.model_kind == 2) {
        float v = a.ml[(size_t)row * cfg.ml_stride + cfg.ml_col];
        if (isnan(v)) {
          ml = cfg.ml_error_score;  // model error -> neutral score (engine.go:279-282)
        } else {
          if (v < 0.f) v = 0.f;
          if (v > 1.f) v = 1.f;
          ml = (double)v;
        }
      }
      if (cfg.model_kind != 0 && ml > cfg.ml_high_risk) reasons |= 1u << 8;
      int fin = (int)(cfg.rule_weight * (double)rule + cfg.ml_weight * (ml * 100.0));
      if (fin > 100) fin = 100;
      const int action = fin >= cfg.block_threshold ? 3 : fin >= cfg.review_threshold ? 2 : 1;
      const uint32_t packed = (uint32_t)(fin & 0xff) | ((uint32_t)(rule & 0xff) << 8) |
                              ((uint32_t)action << 16) | ((cfg.model_kind != 0 ? 1u : 0u) << 18) |
                              (reasons << 20);
      a.out[row] = ResultRec{packed, (float)ml};
      if (a.metrics) {
        atomicAdd(&cnt[MET_HIST + (fin < 0 ? 0 : fin)], 1u);
        atomicAdd(&cnt[MET_ACTION + action], 1u);
        if (reasons & (1u << 8)) atomicAdd(&cnt[MET_MLHIGH], 1u);
        if (f.flags & FR_BLACKLISTED) atomicAdd(&cnt[MET_BLACKLIST], 1u);
        atomicAdd(&cnt[MET_ROWS], 1u);
      }
    }
  }
  if (a.metrics) {
    __syncthreads();
    for (int i = tid; i < MET_N; i += 256)
      if (cnt[i]) atomicAdd(&a.metrics[i], (unsigned long long)cnt[i]);
  }
}

void launch_ensemble(const EnsembleArgs& a, hipStream_t st) {
  if (a.n_rows <= 0) return;
  hipLaunchKernelGGL(ensemble_kernel, dim3((a.n_rows + 255) / 256), dim3(256), 0, st, a);
}

}  // namespace igp

// K5 per-row ensemble (engine.go:276-310), shared by the standalone ensemble kernel and the
// fused MLP-head epilogue (gemm.hip): rule score + ML score -> final score, action, reasons;
// metrics counted into a workgroup LDS histogram and flushed with one global atomic per
// non-empty bucket.
#pragma once
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

// row's result. ml_in: the model output for this row when the caller already holds it
// (fused head epilogue), else NaN-free read from a.ml. cnt: LDS [MET_N] (nullable)
__device__ __forceinline__ void ensemble_row(const EnsembleArgs& a, int row, bool have_ml, float ml_in,
                                             unsigned int* cnt) {
  const int n_live = a.hdr->n;
  if (row >= n_live || (a.feat[row].flags & FR_NOT_OWNED)) {
    a.out[row] = ResultRec{0u, 0.f};  // padding / another rank's request: zero (merge by sum)
    if (a.host_out && !a.route) a.host_out[row] = ResultRec{0u, 0.f};
    return;
  }
  const ScoreCfg& cfg = *a.cfg;
  const FeatRec& f = a.feat[row];
  uint32_t reasons = (uint32_t)f.reserved0;
  const int rule = f.reserved1;
  double ml = 0.0;
  if (cfg.model_kind == 1) {
    ml = heuristic_ml(a.X + (size_t)row * a.x_stride);
  } else if (cfg.model_kind == 2) {
    float v = have_ml ? ml_in : a.ml[(size_t)row * cfg.ml_stride + cfg.ml_col];
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
  const uint32_t packed = (uint32_t)(fin & 0xff) | ((uint32_t)(rule & 0xff) << 8) | ((uint32_t)action << 16) |
                          ((cfg.model_kind != 0 ? 1u : 0u) << 18) | (reasons << 20);
  a.out[row] = ResultRec{packed, (float)ml};
  // host copy: 8-B stores over the bus, visible to the host once the kernel's completion
  // signal (system-scope release) is
  if (a.host_out) {
    ResultRec* dst = a.host_out + row;
    if (a.route) {  // the row's place in its sender's chunk of the results region
      const int d = a.route[row];
      const int p = d / a.route_c;
      dst = reinterpret_cast<ResultRec*>(reinterpret_cast<char*>(a.host_out) + (size_t)p * a.route_stride) +
            (d - p * a.route_c);
    }
    *dst = ResultRec{packed, (float)ml};
  }
  if (cnt) {
    atomicAdd(&cnt[MET_HIST + (fin < 0 ? 0 : fin)], 1u);
    atomicAdd(&cnt[MET_ACTION + action], 1u);
    if (reasons & (1u << 8)) atomicAdd(&cnt[MET_MLHIGH], 1u);
    if (f.flags & FR_BLACKLISTED) atomicAdd(&cnt[MET_BLACKLIST], 1u);
    atomicAdd(&cnt[MET_ROWS], 1u);
  }
}

__device__ __forceinline__ void ensemble_metrics_flush(const EnsembleArgs& a, const unsigned int* cnt, int tid,
                                                       int nthreads) {
  for (int i = tid; i < MET_N; i += nthreads)
    if (cnt[i]) atomicAdd(&a.metrics[i], (unsigned long long)cnt[i]);
}

}  // namespace igp

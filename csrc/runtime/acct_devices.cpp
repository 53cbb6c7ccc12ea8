#include "acct_devices.h"

#include <cmath>
#include <cstring>
#include <stdexcept>

#define IGP_LTV_FN inline
#include "../include/ltv_logic.h"

namespace igp {

namespace {

void copy_err(char* err, int32_t errlen, const char* msg) {
  if (!err || errlen <= 0) return;
  std::strncpy(err, msg, size_t(errlen) - 1);
  err[errlen - 1] = 0;
}

// the executor output named `want`, or the graph's last output (engine/ltv.py, engine/abuse.py:
// y.get(output_name, last value))
const onnx::Tensor& pick_output(const exec::Executor& ex, const std::map<std::string, onnx::Tensor>& y,
                                const std::string& want) {
  auto it = y.find(want);
  if (it != y.end()) return it->second;
  const auto& outs = ex.model().graph.outputs;
  if (!outs.empty()) {
    it = y.find(outs.back().name);
    if (it != y.end()) return it->second;
  }
  if (y.empty()) throw std::runtime_error("model produced no output");
  return y.rbegin()->second;
}

}  // namespace

// ============================================================================ LTV
CpuLtvDevice::CpuLtvDevice(const float* rows, const uint8_t* present, const float* ext, int ext_w, int64_t capacity,
                           std::shared_ptr<exec::Executor> model, std::string in_name, std::string out_name,
                           int model_width, int depth, int cap)
    : rows_(rows), present_(present), ext_(ext), ext_w_(ext_w), cap_rows_(capacity), model_(std::move(model)),
      in_(std::move(in_name)), out_(std::move(out_name)), width_(model_width) {
  if (!rows_ || !present_ || capacity < 1 || depth < 1 || cap < 1) throw std::runtime_error("CpuLtvDevice: arguments");
  if (model_ && width_ < P_NCOLS) throw std::runtime_error("CpuLtvDevice: model input narrower than the profile");
  slots_.resize(size_t(depth));
  for (auto& s : slots_) {
    s.slots.assign(size_t(cap), -1);
    s.out.assign(size_t(cap) * 6, 0.f);
  }
  ops_.abi = IGP_MODEL_OPS_ABI;
  ops_.kind = IGP_MODEL_LTV;
  ops_.depth = depth;
  ops_.cap = cap;
  ops_.has_model = model_ ? 1 : 0;
  ops_.ctx = this;
  ops_.slots = [](void* ctx, int32_t slot) { return static_cast<CpuLtvDevice*>(ctx)->slots_[size_t(slot)].slots.data(); };
  ops_.submit = [](void* ctx, int32_t slot, int32_t n, int64_t, char* err, int32_t errlen) -> int32_t {
    auto* d = static_cast<CpuLtvDevice*>(ctx);
    try {
      d->run(d->slots_[size_t(slot)], n);
    } catch (const std::exception& e) {
      copy_err(err, errlen, e.what());
      return -1;
    }
    return 0;
  };
  ops_.wait = [](void*, int32_t, int64_t, char*, int32_t) -> int32_t { return 0; };
  ops_.out0 = [](void* ctx, int32_t slot) -> const void* {
    return static_cast<CpuLtvDevice*>(ctx)->slots_[size_t(slot)].out.data();
  };
  ops_.out1 = [](void*, int32_t) -> const void* { return nullptr; };
}

void CpuLtvDevice::run(Slot& s, int n) {
  std::vector<float> prof(size_t(n) * P_NCOLS, 0.f);
  for (int i = 0; i < n; ++i) {
    const int32_t sl = s.slots[size_t(i)];
    if (sl >= 0 && sl < cap_rows_ && present_[sl])
      std::memcpy(&prof[size_t(i) * P_NCOLS], rows_ + size_t(sl) * P_NCOLS, sizeof(float) * P_NCOLS);
  }
  std::vector<float> ml;
  if (model_ && n > 0) {
    // engine/ltv.py ltv_model_input: signed log1p of the 25 profile columns, then the account's
    // extra LTV features (zero for an empty profile)
    onnx::Tensor x;
    x.name = in_;
    x.dtype = onnx::FLOAT;
    x.dims = {n, width_};
    x.f.assign(size_t(n) * size_t(width_), 0.f);
    for (int i = 0; i < n; ++i) {
      float* xr = &x.f[size_t(i) * size_t(width_)];
      const float* p = &prof[size_t(i) * P_NCOLS];
      for (int c = 0; c < P_NCOLS; ++c) {
        const float v = p[c];
        xr[c] = (v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f)) * std::log1p(std::fabs(v));
      }
      const int32_t sl = s.slots[size_t(i)];
      if (ext_ && ext_w_ > 0 && sl >= 0 && sl < cap_rows_ && present_[sl]) {
        const int w = std::min(ext_w_, width_ - P_NCOLS);
        std::memcpy(xr + P_NCOLS, ext_ + size_t(sl) * size_t(ext_w_), sizeof(float) * size_t(w));
      }
    }
    std::map<std::string, onnx::Tensor> in;
    in.emplace(in_, std::move(x));
    const auto y = model_->run(in);
    const onnx::Tensor& t = pick_output(*model_, y, out_);
    if (int64_t(t.f.size()) < n) throw std::runtime_error("CpuLtvDevice: model output too short");
    const size_t stride = t.f.size() / size_t(n);
    ml.resize(size_t(n));
    for (int i = 0; i < n; ++i) ml[size_t(i)] = t.f[size_t(i) * stride];
  }
  for (int i = 0; i < n; ++i)
    ltv_row(&prof[size_t(i) * P_NCOLS], ml.empty() ? nullptr : &ml[size_t(i)], &s.out[size_t(i) * 6]);
}

// ============================================================================ abuse
CpuAbuseDevice::CpuAbuseDevice(std::shared_ptr<CpuScorer> sc, std::shared_ptr<exec::Executor> model,
                               std::string in_name, std::string out_name, int depth, int cap)
    : sc_(std::move(sc)), model_(std::move(model)), in_(std::move(in_name)), out_(std::move(out_name)) {
  if (!sc_ || depth < 1 || cap < 1) throw std::runtime_error("CpuAbuseDevice: arguments");
  slots_.resize(size_t(depth));
  for (auto& s : slots_) {
    s.slots.assign(size_t(cap), -1);
    s.score.assign(size_t(cap), 0.f);
    s.feat.assign(size_t(cap), FeatRec{});
  }
  ops_.abi = IGP_MODEL_OPS_ABI;
  ops_.kind = IGP_MODEL_ABUSE;
  ops_.depth = depth;
  ops_.cap = cap;
  ops_.has_model = model_ ? 1 : 0;
  ops_.ctx = this;
  ops_.slots = [](void* ctx, int32_t slot) {
    return static_cast<CpuAbuseDevice*>(ctx)->slots_[size_t(slot)].slots.data();
  };
  ops_.submit = [](void* ctx, int32_t slot, int32_t n, int64_t now, char* err, int32_t errlen) -> int32_t {
    auto* d = static_cast<CpuAbuseDevice*>(ctx);
    try {
      d->run(d->slots_[size_t(slot)], n, now);
    } catch (const std::exception& e) {
      copy_err(err, errlen, e.what());
      return -1;
    }
    return 0;
  };
  ops_.wait = [](void*, int32_t, int64_t, char*, int32_t) -> int32_t { return 0; };
  ops_.out0 = [](void* ctx, int32_t slot) -> const void* {
    return static_cast<CpuAbuseDevice*>(ctx)->slots_[size_t(slot)].score.data();
  };
  ops_.out1 = [](void* ctx, int32_t slot) -> const void* {
    return static_cast<CpuAbuseDevice*>(ctx)->slots_[size_t(slot)].feat.data();
  };
}

void CpuAbuseDevice::run(Slot& s, int n, int64_t now) {
  for (int i = 0; i < n; ++i) {
    const int32_t sl = s.slots[size_t(i)];
    s.feat[size_t(i)] = sl >= 0 ? sc_->features(sl, now) : FeatRec{};
  }
  if (!model_ || n == 0) return;
  // engine/abuse.py model_scores (executor path): X [event_ring][n][event_dim], each account's
  // history oldest first, right-aligned (zeros for an unknown account)
  const int T = sc_->event_ring(), D = sc_->event_dim();
  onnx::Tensor x;
  x.name = in_;
  x.dtype = onnx::FLOAT;
  x.dims = {T, n, D};
  x.f.assign(size_t(T) * size_t(n) * size_t(D), 0.f);
  std::vector<float> h(size_t(T) * size_t(D));
  for (int i = 0; i < n; ++i) {
    const int32_t sl = s.slots[size_t(i)];
    if (sl < 0) continue;
    sc_->event_history(sl, h.data());
    for (int t = 0; t < T; ++t)
      std::memcpy(&x.f[(size_t(t) * size_t(n) + size_t(i)) * size_t(D)], &h[size_t(t) * size_t(D)],
                  sizeof(float) * size_t(D));
  }
  std::map<std::string, onnx::Tensor> in;
  in.emplace(in_, std::move(x));
  const auto y = model_->run(in);
  const onnx::Tensor& t = pick_output(*model_, y, out_);
  if (int64_t(t.f.size()) < n) throw std::runtime_error("CpuAbuseDevice: model output too short");
  for (int i = 0; i < n; ++i) s.score[size_t(i)] = t.f[size_t(i)];
}

}  // namespace igp

// CPU reference executor: float32 tensors, double accumulation for matrix products.
#include "executor.h"

#include <algorithm>
#include <cmath>
#include <functional>
#include <numeric>
#include <set>
#include <stdexcept>

namespace igp::exec {
namespace {

using onnx::FLOAT;
using onnx::INT64;

Tensor make(const std::vector<int64_t>& dims, int32_t dtype = FLOAT) {
  Tensor t;
  t.dims = dims;
  t.dtype = dtype;
  if (dtype == FLOAT) t.f.assign(t.numel(), 0.f);
  else t.i.assign(t.numel(), 0);
  return t;
}

std::vector<float> as_float(const Tensor& t) {
  if (t.dtype == FLOAT) return t.f;
  return std::vector<float>(t.i.begin(), t.i.end());
}

std::vector<int64_t> as_int(const Tensor& t) {
  if (t.dtype == INT64) return t.i;
  std::vector<int64_t> r;
  for (float v : t.f) r.push_back(int64_t(v));
  return r;
}

int64_t norm_axis(int64_t a, size_t rank) {
  if (a < 0) a += int64_t(rank);
  if (a < 0 || a >= int64_t(rank) + 1) throw std::runtime_error("axis out of range");
  return a;
}

// numpy-style broadcasting elementwise binary op on float tensors
Tensor binary(const Tensor& A, const Tensor& B, const std::function<float(float, float)>& op) {
  const auto a = as_float(A), b = as_float(B);
  size_t r = std::max(A.dims.size(), B.dims.size());
  std::vector<int64_t> da(r, 1), db(r, 1), dout(r);
  std::copy(A.dims.begin(), A.dims.end(), da.begin() + (r - A.dims.size()));
  std::copy(B.dims.begin(), B.dims.end(), db.begin() + (r - B.dims.size()));
  for (size_t k = 0; k < r; ++k) {
    if (da[k] != db[k] && da[k] != 1 && db[k] != 1) throw std::runtime_error("broadcast: incompatible shapes");
    dout[k] = std::max(da[k], db[k]);
  }
  Tensor out = make(dout);
  std::vector<int64_t> sa(r), sb(r);
  int64_t ma = 1, mb = 1;
  for (int k = int(r) - 1; k >= 0; --k) {
    sa[k] = da[k] == 1 ? 0 : ma; ma *= da[k];
    sb[k] = db[k] == 1 ? 0 : mb; mb *= db[k];
  }
  std::vector<int64_t> idx(r, 0);
  const int64_t n = out.numel();
  for (int64_t e = 0; e < n; ++e) {
    int64_t oa = 0, ob = 0;
    for (size_t k = 0; k < r; ++k) { oa += idx[k] * sa[k]; ob += idx[k] * sb[k]; }
    out.f[e] = op(a[oa], b[ob]);
    for (int k = int(r) - 1; k >= 0; --k) {
      if (++idx[k] < dout[k]) break;
      idx[k] = 0;
    }
  }
  return out;
}

Tensor unary(const Tensor& A, const std::function<float(float)>& op) {
  Tensor out = make(A.dims);
  auto a = as_float(A);
  for (size_t k = 0; k < a.size(); ++k) out.f[k] = op(a[k]);
  return out;
}

inline float sigmoid(float x) { return 1.f / (1.f + std::exp(-x)); }

Tensor gemm(const onnx::Node& n, const Tensor& A, const Tensor& B, const Tensor* C) {
  const float alpha = n.getf("alpha", 1.f), beta = n.getf("beta", 1.f);
  const bool ta = n.geti("transA", 0), tb = n.geti("transB", 0);
  if (A.dims.size() != 2 || B.dims.size() != 2) throw std::runtime_error("Gemm: 2-D inputs required");
  const int64_t M = ta ? A.dims[1] : A.dims[0], K = ta ? A.dims[0] : A.dims[1];
  const int64_t K2 = tb ? B.dims[1] : B.dims[0], N = tb ? B.dims[0] : B.dims[1];
  if (K != K2) throw std::runtime_error("Gemm: inner dimensions differ");
  Tensor Y = make({M, N});
  const auto& a = A.f;
  const auto& b = B.f;
  for (int64_t i = 0; i < M; ++i)
    for (int64_t j = 0; j < N; ++j) {
      double s = 0;
      for (int64_t k = 0; k < K; ++k) {
        float av = ta ? a[k * M + i] : a[i * K + k];
        float bv = tb ? b[j * K + k] : b[k * N + j];
        s += double(av) * double(bv);
      }
      Y.f[i * N + j] = float(alpha * s);
    }
  if (C && beta != 0.f) {
    Tensor c = *C;
    Y = binary(Y, c, [beta](float y, float cv) { return y + beta * cv; });
  }
  return Y;
}

Tensor matmul(const Tensor& A, const Tensor& B) {
  if (B.dims.size() != 2 || A.dims.size() < 1) throw std::runtime_error("MatMul: B must be 2-D");
  const int64_t K = A.dims.back(), N = B.dims[1];
  if (B.dims[0] != K) throw std::runtime_error("MatMul: inner dimensions differ");
  const int64_t M = A.numel() / K;
  std::vector<int64_t> od = A.dims;
  od.back() = N;
  Tensor Y = make(od);
  for (int64_t i = 0; i < M; ++i)
    for (int64_t j = 0; j < N; ++j) {
      double s = 0;
      for (int64_t k = 0; k < K; ++k) s += double(A.f[i * K + k]) * double(B.f[k * N + j]);
      Y.f[i * N + j] = float(s);
    }
  return Y;
}

// ONNX GRU (gates z, r, h), activations sigmoid/tanh, directions forward / reverse /
// bidirectional. layout 0: X [S][B][I], Y [S][D][B][H], Y_h / initial_h [D][B][H];
// layout 1 (batch-major): X [B][S][I], Y [B][S][D][H], Y_h / initial_h [B][D][H].
void gru(const onnx::Node& n, const Tensor& X, const Tensor& W, const Tensor& R, const Tensor* Bp,
         const Tensor* h0, Tensor& Y, Tensor& Yh) {
  const int64_t H = n.geti("hidden_size", R.dims.back());
  const bool lbr = n.geti("linear_before_reset", 0);
  const int64_t layout = n.geti("layout", 0);
  if (layout != 0 && layout != 1) throw std::runtime_error("GRU: layout must be 0 or 1");
  std::string dir = n.gets("direction", "forward");
  if (dir != "forward" && dir != "reverse" && dir != "bidirectional") throw std::runtime_error("GRU: direction");
  const int64_t D = dir == "bidirectional" ? 2 : 1;
  if (X.dims.size() != 3) throw std::runtime_error("GRU: X must be rank 3");
  const int64_t S = layout ? X.dims[1] : X.dims[0], Bn = layout ? X.dims[0] : X.dims[1], I = X.dims[2];
  if (W.dims[0] != D || W.dims[1] != 3 * H || W.dims[2] != I) throw std::runtime_error("GRU: W shape");
  if (R.dims[0] != D || R.dims[1] != 3 * H || R.dims[2] != H) throw std::runtime_error("GRU: R shape");
  Y = layout ? make({Bn, S, D, H}) : make({S, D, Bn, H});
  Yh = layout ? make({Bn, D, H}) : make({D, Bn, H});
  // element offsets of (t, b) in X, (t, d, b) in Y and (d, b) in Y_h / initial_h
  auto xo = [&](int64_t t, int64_t b) { return (layout ? b * S + t : t * Bn + b) * I; };
  auto yo = [&](int64_t t, int64_t d, int64_t b) { return (layout ? (b * S + t) * D + d : (t * D + d) * Bn + b) * H; };
  auto ho = [&](int64_t d, int64_t b) { return (layout ? b * D + d : d * Bn + b) * H; };
  std::vector<double> hz(H), hr(H), hh(H), xz(H), xr(H), xh(H);
  for (int64_t d = 0; d < D; ++d) {
    const bool rev = dir == "reverse" || (D == 2 && d == 1);
    const float* w = &W.f[d * 3 * H * I];
    const float* r = &R.f[d * 3 * H * H];
    std::vector<float> bias(6 * H, 0.f);
    if (Bp) std::copy(Bp->f.begin() + d * 6 * H, Bp->f.begin() + (d + 1) * 6 * H, bias.begin());
    for (int64_t b = 0; b < Bn; ++b) {
      std::vector<float> h(H, 0.f);
      if (h0) std::copy(h0->f.begin() + ho(d, b), h0->f.begin() + ho(d, b) + H, h.begin());
      for (int64_t st = 0; st < S; ++st) {
        const int64_t t = rev ? S - 1 - st : st;
        const float* x = &X.f[xo(t, b)];
        for (int64_t j = 0; j < H; ++j) {
          double az = 0, ar = 0, ah = 0, bz = 0, br = 0, bh = 0;
          for (int64_t k = 0; k < I; ++k) {
            az += double(w[j * I + k]) * x[k];
            ar += double(w[(H + j) * I + k]) * x[k];
            ah += double(w[(2 * H + j) * I + k]) * x[k];
          }
          for (int64_t k = 0; k < H; ++k) {
            bz += double(r[j * H + k]) * h[k];
            br += double(r[(H + j) * H + k]) * h[k];
          }
          xz[j] = az; xr[j] = ar; xh[j] = ah; hz[j] = bz; hr[j] = br;
          (void)bh;
        }
        std::vector<float> rg(H), zg(H);
        for (int64_t j = 0; j < H; ++j) {
          zg[j] = sigmoid(float(xz[j] + hz[j] + bias[j] + bias[3 * H + j]));
          rg[j] = sigmoid(float(xr[j] + hr[j] + bias[H + j] + bias[4 * H + j]));
        }
        for (int64_t j = 0; j < H; ++j) {
          double acc = 0;
          if (lbr) {
            for (int64_t k = 0; k < H; ++k) acc += double(r[(2 * H + j) * H + k]) * h[k];
            hh[j] = rg[j] * (acc + bias[5 * H + j]);
          } else {
            for (int64_t k = 0; k < H; ++k) acc += double(r[(2 * H + j) * H + k]) * (rg[k] * h[k]);
            hh[j] = acc + bias[5 * H + j];
          }
        }
        for (int64_t j = 0; j < H; ++j) {
          float nt = std::tanh(float(xh[j] + bias[2 * H + j] + hh[j]));
          h[j] = (1.f - zg[j]) * nt + zg[j] * h[j];
        }
        std::copy(h.begin(), h.end(), Y.f.begin() + yo(t, d, b));
      }
      std::copy(h.begin(), h.end(), Yh.f.begin() + ho(d, b));
    }
  }
}

// ---- ai.onnx.ml linear models and preprocessing (sklearn-style pipelines: Scaler ->
// LinearClassifier -> ZipMap; Normalizer; LinearRegressor). Semantics follow the ai.onnx.ml
// operator definitions; ORT itself is not available offline, so exact ORT parity is unpinned
// (tests compare against numpy references of the definitions below).

int32_t post_code(const onnx::Node& n) {
  const std::string p = n.gets("post_transform", "NONE");
  if (p == "NONE") return trees::NONE;
  if (p == "LOGISTIC") return trees::LOGISTIC;
  if (p == "SOFTMAX") return trees::SOFTMAX;
  if (p == "SOFTMAX_ZERO") return trees::SOFTMAX_ZERO;
  if (p == "PROBIT") return trees::PROBIT;
  throw std::runtime_error(n.op_type + ": unknown post_transform " + p);
}

// one row of K scores through a post transform, in place
void post_row(int32_t post, float* z, int64_t k) {
  if (post == trees::LOGISTIC) {
    for (int64_t c = 0; c < k; ++c) z[c] = sigmoid(z[c]);
  } else if (post == trees::SOFTMAX || post == trees::SOFTMAX_ZERO) {
    const bool zero = post == trees::SOFTMAX_ZERO;
    float m = -INFINITY;
    for (int64_t c = 0; c < k; ++c) if (!(zero && z[c] == 0.f)) m = std::max(m, z[c]);
    double s = 0;
    for (int64_t c = 0; c < k; ++c) {
      if (zero && z[c] == 0.f) continue;
      z[c] = std::exp(z[c] - m);
      s += z[c];
    }
    for (int64_t c = 0; c < k; ++c) z[c] = (zero && z[c] == 0.f) || s <= 0 ? 0.f : float(z[c] / s);
  } else if (post == trees::PROBIT) {
    for (int64_t c = 0; c < k; ++c) z[c] = 1.41421356f * trees::erfinv(2 * z[c] - 1);
  }
}

// rows of X ([N][C], or one row [C]) times coefficient rows W [E][C] plus intercepts: [N][E]
std::vector<float> linear_rows(const std::string& op, const Tensor& X, const std::vector<float>& W,
                               const std::vector<float>& b, int64_t E, int64_t& N) {
  const auto x = as_float(X);
  const int64_t C = X.dims.empty() ? 1 : X.dims.back();
  N = X.dims.size() <= 1 ? 1 : X.numel() / std::max<int64_t>(C, 1);
  if (E < 1 || int64_t(W.size()) != E * C) throw std::runtime_error(op + ": coefficients do not match [E][C]");
  if (!b.empty() && int64_t(b.size()) != E) throw std::runtime_error(op + ": intercepts do not match E");
  std::vector<float> y(size_t(N * E));
  for (int64_t i = 0; i < N; ++i)
    for (int64_t e = 0; e < E; ++e) {
      double s = b.empty() ? 0.0 : double(b[e]);
      for (int64_t c = 0; c < C; ++c) s += double(W[e * C + c]) * double(x[i * C + c]);
      y[i * E + e] = float(s);
    }
  return y;
}

const std::vector<float>& attr_floats(const onnx::Node& n, const char* name) {
  static const std::vector<float> none;
  auto a = n.attr(name);
  return a ? a->floats : none;
}

// LinearClassifier: outputs (label [N] int64, scores [N][K]). One coefficient row is the binary
// case: raw score s becomes the two columns [-s, s] before the post transform (LOGISTIC then
// gives [sigmoid(-s), sigmoid(s)]) and the label is classlabels[s > 0]. E rows: label =
// classlabels[argmax raw]. String class labels yield the class index as the label.
void linear_classifier(const onnx::Node& n, const Tensor& X, Tensor& labels, Tensor& scores) {
  const auto& W = attr_floats(n, "coefficients");
  const auto& b = attr_floats(n, "intercepts");
  const int64_t C = X.dims.empty() ? 1 : X.dims.back();
  const int64_t E = !b.empty() ? int64_t(b.size()) : int64_t(W.size()) / std::max<int64_t>(C, 1);
  std::vector<int64_t> cl;
  if (auto a = n.attr("classlabels_ints")) cl = a->ints;
  else if (auto s = n.attr("classlabels_strings"))
    for (size_t k = 0; k < s->strings.size(); ++k) cl.push_back(int64_t(k));
  int64_t N = 0;
  auto raw = linear_rows(n.op_type, X, W, b, E, N);
  const int32_t post = post_code(n);
  const int64_t K = E == 1 ? 2 : E;
  labels = make({N}, INT64);
  scores = make({N, K});
  for (int64_t i = 0; i < N; ++i) {
    float* z = &scores.f[i * K];
    int64_t best = 0;
    if (E == 1) {
      z[0] = -raw[i];
      z[1] = raw[i];
      best = raw[i] > 0.f ? 1 : 0;
    } else {
      for (int64_t e = 0; e < E; ++e) {
        z[e] = raw[i * E + e];
        if (z[e] > z[best]) best = e;
      }
    }
    post_row(post, z, K);
    labels.i[i] = best < int64_t(cl.size()) ? cl[best] : best;
  }
}

}  // namespace

Executor::Executor(onnx::Model model) : model_(std::move(model)) {
  auto& g = model_.graph;
  std::set<std::string> avail;
  for (auto& kv : g.initializers) avail.insert(kv.first);
  for (auto& v : g.inputs) avail.insert(v.name);
  avail.insert("");
  std::vector<bool> done(g.nodes.size(), false);
  for (size_t pass = 0; pass < g.nodes.size(); ++pass) {
    bool progress = false;
    for (size_t k = 0; k < g.nodes.size(); ++k) {
      if (done[k]) continue;
      bool ready = true;
      for (auto& in : g.nodes[k].inputs) ready &= avail.count(in) > 0;
      if (!ready) continue;
      done[k] = true;
      progress = true;
      order_.push_back(k);
      for (auto& o : g.nodes[k].outputs) avail.insert(o);
    }
    if (!progress) break;
  }
  if (order_.size() != g.nodes.size()) throw std::runtime_error("onnx: graph has unresolvable inputs or a cycle");
  for (size_t k = 0; k < g.nodes.size(); ++k) {
    const auto& op = g.nodes[k].op_type;
    if (op == "TreeEnsembleClassifier" || op == "TreeEnsembleRegressor")
      ensembles_[k] = std::make_shared<trees::Ensemble>(trees::compile(g.nodes[k]));
  }
}

const trees::Ensemble* Executor::ensemble(size_t node_index) const {
  auto it = ensembles_.find(node_index);
  return it == ensembles_.end() ? nullptr : it->second.get();
}

std::map<std::string, Tensor> Executor::run(const std::map<std::string, Tensor>& inputs) const {
  const auto& g = model_.graph;
  std::map<std::string, Tensor> vals;
  for (auto& kv : g.initializers) vals[kv.first] = kv.second;
  for (auto& v : g.inputs) {
    auto it = inputs.find(v.name);
    if (it == inputs.end()) throw std::runtime_error("executor: missing input " + v.name);
    vals[v.name] = it->second;
  }
  auto get = [&](const std::string& name) -> const Tensor& {
    auto it = vals.find(name);
    if (it == vals.end()) throw std::runtime_error("executor: value not computed: " + name);
    return it->second;
  };
  auto opt = [&](const onnx::Node& n, size_t i) -> const Tensor* {
    if (i >= n.inputs.size() || n.inputs[i].empty()) return nullptr;
    return &get(n.inputs[i]);
  };
  for (size_t k : order_) {
    const auto& n = g.nodes[k];
    const std::string& op = n.op_type;
    Tensor out;
    if (op == "Gemm") out = gemm(n, get(n.inputs[0]), get(n.inputs[1]), opt(n, 2));
    else if (op == "MatMul") out = matmul(get(n.inputs[0]), get(n.inputs[1]));
    else if (op == "Add") out = binary(get(n.inputs[0]), get(n.inputs[1]), [](float a, float b) { return a + b; });
    else if (op == "Sub") out = binary(get(n.inputs[0]), get(n.inputs[1]), [](float a, float b) { return a - b; });
    else if (op == "Mul") out = binary(get(n.inputs[0]), get(n.inputs[1]), [](float a, float b) { return a * b; });
    else if (op == "Div") out = binary(get(n.inputs[0]), get(n.inputs[1]), [](float a, float b) { return a / b; });
    else if (op == "Max") out = binary(get(n.inputs[0]), get(n.inputs[1]), [](float a, float b) { return std::max(a, b); });
    else if (op == "Min") out = binary(get(n.inputs[0]), get(n.inputs[1]), [](float a, float b) { return std::min(a, b); });
    else if (op == "Relu") out = unary(get(n.inputs[0]), [](float x) { return x > 0 ? x : 0.f; });
    else if (op == "LeakyRelu") { float a = n.getf("alpha", 0.01f); out = unary(get(n.inputs[0]), [a](float x) { return x > 0 ? x : a * x; }); }
    else if (op == "Sigmoid") out = unary(get(n.inputs[0]), sigmoid);
    else if (op == "Tanh") out = unary(get(n.inputs[0]), [](float x) { return std::tanh(x); });
    else if (op == "Exp") out = unary(get(n.inputs[0]), [](float x) { return std::exp(x); });
    else if (op == "Log") out = unary(get(n.inputs[0]), [](float x) { return std::log(x); });
    else if (op == "Abs") out = unary(get(n.inputs[0]), [](float x) { return std::fabs(x); });
    else if (op == "Neg") out = unary(get(n.inputs[0]), [](float x) { return -x; });
    else if (op == "Sqrt") out = unary(get(n.inputs[0]), [](float x) { return std::sqrt(x); });
    else if (op == "Identity") out = get(n.inputs[0]);
    else if (op == "Clip") {
      float lo = -INFINITY, hi = INFINITY;
      if (auto t = opt(n, 1)) lo = as_float(*t)[0];
      if (auto t = opt(n, 2)) hi = as_float(*t)[0];
      if (n.attr("min")) lo = n.getf("min", lo);
      if (n.attr("max")) hi = n.getf("max", hi);
      out = unary(get(n.inputs[0]), [lo, hi](float x) { return std::min(std::max(x, lo), hi); });
    } else if (op == "Cast") {
      int64_t to = n.geti("to", FLOAT);
      const Tensor& x = get(n.inputs[0]);
      out.dims = x.dims;
      if (to == INT64 || to == onnx::INT32) { out.dtype = INT64; out.i = as_int(x); }
      else { out.dtype = FLOAT; out.f = as_float(x); }
    } else if (op == "Softmax") {
      const Tensor& x = get(n.inputs[0]);
      int64_t ax = norm_axis(n.geti("axis", -1), x.dims.size());
      int64_t inner = 1;
      for (size_t d = ax + 1; d < x.dims.size(); ++d) inner *= x.dims[d];
      int64_t len = x.dims[ax], outer = x.numel() / (len * inner);
      out = make(x.dims);
      for (int64_t o = 0; o < outer; ++o)
        for (int64_t i = 0; i < inner; ++i) {
          float m = -INFINITY;
          for (int64_t l = 0; l < len; ++l) m = std::max(m, x.f[(o * len + l) * inner + i]);
          double s = 0;
          for (int64_t l = 0; l < len; ++l) s += std::exp(double(x.f[(o * len + l) * inner + i] - m));
          for (int64_t l = 0; l < len; ++l)
            out.f[(o * len + l) * inner + i] = float(std::exp(double(x.f[(o * len + l) * inner + i] - m)) / s);
        }
    } else if (op == "Flatten") {
      const Tensor& x = get(n.inputs[0]);
      int64_t ax = norm_axis(n.geti("axis", 1), x.dims.size());
      int64_t a = 1;
      for (int64_t d = 0; d < ax; ++d) a *= x.dims[d];
      out = x;
      out.dims = {a, x.numel() / std::max<int64_t>(a, 1)};
    } else if (op == "Reshape") {
      const Tensor& x = get(n.inputs[0]);
      auto shp = as_int(get(n.inputs[1]));
      int64_t known = 1, neg = -1;
      for (size_t d = 0; d < shp.size(); ++d) {
        if (shp[d] == 0) shp[d] = x.dims.at(d);
        if (shp[d] == -1) neg = int64_t(d); else known *= shp[d];
      }
      if (neg >= 0) shp[neg] = x.numel() / known;
      out = x;
      out.dims = shp;
      if (out.numel() != x.numel()) throw std::runtime_error("Reshape: element count mismatch");
    } else if (op == "Squeeze" || op == "Unsqueeze") {
      const Tensor& x = get(n.inputs[0]);
      std::vector<int64_t> axes;
      if (auto t = opt(n, 1)) axes = as_int(*t);
      else if (auto a = n.attr("axes")) axes = a->ints;
      out = x;
      if (op == "Squeeze") {
        std::vector<int64_t> d;
        for (size_t k2 = 0; k2 < x.dims.size(); ++k2) {
          bool drop = axes.empty() ? x.dims[k2] == 1 : false;
          for (auto a : axes) drop |= norm_axis(a, x.dims.size()) == int64_t(k2);
          if (!drop) d.push_back(x.dims[k2]);
        }
        out.dims = d;
      } else {
        size_t r = x.dims.size() + axes.size();
        std::vector<int64_t> d;
        std::set<int64_t> ax;
        for (auto a : axes) ax.insert(a < 0 ? a + int64_t(r) : a);
        size_t src = 0;
        for (size_t k2 = 0; k2 < r; ++k2) d.push_back(ax.count(k2) ? 1 : x.dims[src++]);
        out.dims = d;
      }
    } else if (op == "Concat") {
      std::vector<const Tensor*> ts;
      for (auto& in : n.inputs) ts.push_back(&get(in));
      int64_t ax = norm_axis(n.geti("axis", 0), ts[0]->dims.size());
      std::vector<int64_t> d = ts[0]->dims;
      d[ax] = 0;
      for (auto t : ts) d[ax] += t->dims[ax];
      out = make(d);
      int64_t outer = 1, inner = 1;
      for (int64_t k2 = 0; k2 < ax; ++k2) outer *= d[k2];
      for (size_t k2 = ax + 1; k2 < d.size(); ++k2) inner *= d[k2];
      int64_t off = 0;
      for (auto t : ts) {
        auto tf = as_float(*t);
        int64_t len = t->dims[ax];
        for (int64_t o = 0; o < outer; ++o)
          std::copy(tf.begin() + o * len * inner, tf.begin() + (o + 1) * len * inner,
                    out.f.begin() + (o * d[ax] + off) * inner);
        off += len;
      }
    } else if (op == "Transpose") {
      const Tensor& x = get(n.inputs[0]);
      size_t r = x.dims.size();
      std::vector<int64_t> perm(r);
      if (auto a = n.attr("perm")) perm = a->ints;
      else for (size_t k2 = 0; k2 < r; ++k2) perm[k2] = int64_t(r - 1 - k2);
      std::vector<int64_t> d(r), st(r, 1);
      for (int k2 = int(r) - 2; k2 >= 0; --k2) st[k2] = st[k2 + 1] * x.dims[k2 + 1];
      for (size_t k2 = 0; k2 < r; ++k2) d[k2] = x.dims[perm[k2]];
      out = make(d);
      std::vector<int64_t> idx(r, 0);
      for (int64_t e = 0; e < out.numel(); ++e) {
        int64_t src = 0;
        for (size_t k2 = 0; k2 < r; ++k2) src += idx[k2] * st[perm[k2]];
        out.f[e] = x.f[src];
        for (int k2 = int(r) - 1; k2 >= 0; --k2) { if (++idx[k2] < d[k2]) break; idx[k2] = 0; }
      }
    } else if (op == "TreeEnsembleClassifier" || op == "TreeEnsembleRegressor") {
      const auto* e = ensemble(k);
      const Tensor& x = get(n.inputs[0]);
      auto xf = as_float(x);
      int64_t N = x.dims.size() == 1 ? 1 : x.dims[0];
      int64_t F = x.numel() / std::max<int64_t>(N, 1);
      std::vector<float> sc(size_t(N) * e->n_targets);
      trees::eval_raw(*e, xf.data(), N, F, sc.data());
      Tensor probs = make({N, e->n_outputs});
      if (e->classifier) {
        Tensor labels = make({N}, INT64);
        trees::post_transform(*e, sc.data(), N, probs.f.data(), labels.i.data());
        vals[n.outputs[0]] = labels;
        if (n.outputs.size() > 1) vals[n.outputs[1]] = probs;
      } else {
        trees::post_transform(*e, sc.data(), N, probs.f.data(), nullptr);
        vals[n.outputs[0]] = probs;
      }
      continue;
    } else if (op == "LinearClassifier") {
      Tensor labels, scores;
      linear_classifier(n, get(n.inputs[0]), labels, scores);
      vals[n.outputs[0]] = std::move(labels);
      if (n.outputs.size() > 1) vals[n.outputs[1]] = std::move(scores);
      continue;
    } else if (op == "LinearRegressor") {
      const Tensor& x = get(n.inputs[0]);
      const int64_t E = n.geti("targets", 1);
      int64_t N = 0;
      auto y = linear_rows(op, x, attr_floats(n, "coefficients"), attr_floats(n, "intercepts"), E, N);
      const int32_t post = post_code(n);
      out = make({N, E});
      out.f = std::move(y);
      for (int64_t i = 0; i < N; ++i) post_row(post, &out.f[i * E], E);
    } else if (op == "Scaler") {
      // Y = (X - offset) * scale, offset / scale per column (or one value for all)
      const Tensor& x = get(n.inputs[0]);
      const auto& off = attr_floats(n, "offset");
      const auto& sc = attr_floats(n, "scale");
      const int64_t C = x.dims.empty() ? 1 : x.dims.back();
      auto ok = [C](size_t s) { return s == 0 || s == 1 || int64_t(s) == C; };
      if (!ok(off.size()) || !ok(sc.size())) throw std::runtime_error("Scaler: offset / scale length must be 1 or C");
      auto xf = as_float(x);
      out = make(x.dims);
      for (int64_t e = 0; e < x.numel(); ++e) {
        const int64_t c = e % C;
        const float o = off.empty() ? 0.f : off[off.size() == 1 ? 0 : c];
        const float s = sc.empty() ? 1.f : sc[sc.size() == 1 ? 0 : c];
        out.f[e] = (xf[e] - o) * s;
      }
    } else if (op == "Normalizer") {
      // per row (last axis): MAX divides by the row maximum, L1 by sum |x|, L2 by sqrt(sum x^2);
      // a zero denominator leaves the row unchanged
      const Tensor& x = get(n.inputs[0]);
      const std::string norm = n.gets("norm", "MAX");
      if (norm != "MAX" && norm != "L1" && norm != "L2") throw std::runtime_error("Normalizer: norm " + norm);
      const int64_t C = x.dims.empty() ? 1 : x.dims.back();
      out = make(x.dims);
      out.f = as_float(x);
      for (int64_t r = 0; r < x.numel() / std::max<int64_t>(C, 1); ++r) {
        float* z = &out.f[r * C];
        double d = norm == "MAX" ? -INFINITY : 0.0;
        for (int64_t c = 0; c < C; ++c)
          d = norm == "MAX" ? std::max(d, double(z[c])) : norm == "L1" ? d + std::fabs(double(z[c]))
                                                                        : d + double(z[c]) * z[c];
        if (norm == "L2") d = std::sqrt(d);
        if (d != 0.0 && std::isfinite(d))
          for (int64_t c = 0; c < C; ++c) z[c] = float(double(z[c]) / d);
      }
    } else if (op == "ZipMap") {
      // seq(map(label -> probability)) is represented densely: the [N][K] probability tensor,
      // columns in classlabels order (what every consumer of the model output reads)
      const Tensor& x = get(n.inputs[0]);
      out = make(x.dims);
      out.f = as_float(x);
    } else if (op == "GRU") {
      Tensor Y, Yh;
      gru(n, get(n.inputs[0]), get(n.inputs[1]), get(n.inputs[2]), opt(n, 3),
          opt(n, 5), Y, Yh);
      if (opt(n, 4)) throw std::runtime_error("GRU: sequence_lens is not supported");
      if (!n.outputs.empty() && !n.outputs[0].empty()) vals[n.outputs[0]] = Y;
      if (n.outputs.size() > 1 && !n.outputs[1].empty()) vals[n.outputs[1]] = Yh;
      continue;
    } else {
      throw std::runtime_error("executor: unsupported op " + op + " (node " + n.name + ")");
    }
    vals[n.outputs[0]] = std::move(out);
  }
  std::map<std::string, Tensor> res;
  for (auto& v : g.outputs) res[v.name] = get(v.name);
  return res;
}

}  // namespace igp::exec

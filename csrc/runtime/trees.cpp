// TreeEnsemble compilation and CPU evaluation (semantics: ONNX-ML TreeEnsemble{Classifier,
// Regressor}; binary-classifier conventions follow ONNX Runtime's tree aggregator).
#include "trees.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <stdexcept>

namespace igp::trees {
namespace {

uint8_t parse_mode(const std::string& m) {
  if (m == "BRANCH_LEQ") return LEQ;
  if (m == "BRANCH_LT") return LT;
  if (m == "BRANCH_GTE") return GTE;
  if (m == "BRANCH_GT") return GT;
  if (m == "BRANCH_EQ") return EQ;
  if (m == "BRANCH_NEQ") return NEQ;
  if (m == "LEAF") return LEAF;
  throw std::runtime_error("TreeEnsemble: unknown node mode " + m);
}

const std::vector<int64_t>& ints(const onnx::Node& n, const char* name, bool required = true) {
  static const std::vector<int64_t> empty;
  auto a = n.attr(name);
  if (!a) {
    if (required) throw std::runtime_error(std::string("TreeEnsemble: missing attribute ") + name);
    return empty;
  }
  return a->ints;
}

std::vector<float> floats(const onnx::Node& n, const char* name, const char* tensor_name) {
  if (auto a = n.attr(name)) return a->floats;
  if (auto t = n.attr(tensor_name)) {
    if (t->t) return t->t->f;
  }
  return {};
}

inline bool go_true(float x, float thr, uint8_t mode, uint8_t miss) {
  bool c;
  switch (mode) {
    case LEQ: c = x <= thr; break;
    case LT: c = x < thr; break;
    case GTE: c = x >= thr; break;
    case GT: c = x > thr; break;
    case EQ: c = x == thr; break;
    default: c = x != thr; break;  // NEQ
  }
  return c || (miss && std::isnan(x));
}


}  // namespace

float erfinv(float x) {  // Giles' single-precision approximation (PROBIT post transform)
  if (!(std::fabs(x) < 1.0f)) return std::isnan(x) ? x : std::copysign(INFINITY, x);
  float w = -std::log((1.0f - x) * (1.0f + x)), p;
  if (w < 5.0f) {
    w -= 2.5f;
    p = 2.81022636e-08f; p = 3.43273939e-07f + p * w; p = -3.5233877e-06f + p * w;
    p = -4.39150654e-06f + p * w; p = 0.00021858087f + p * w; p = -0.00125372503f + p * w;
    p = -0.00417768164f + p * w; p = 0.246640727f + p * w; p = 1.50140941f + p * w;
  } else {
    w = std::sqrt(w) - 3.0f;
    p = -0.000200214257f; p = 0.000100950558f + p * w; p = 0.00134934322f + p * w;
    p = -0.00367342844f + p * w; p = 0.00573950773f + p * w; p = -0.0076224613f + p * w;
    p = 0.00943887047f + p * w; p = 1.00167406f + p * w; p = 2.83297682f + p * w;
  }
  return p * x;
}

Ensemble compile(const onnx::Node& node) {
  Ensemble e;
  e.classifier = node.op_type == "TreeEnsembleClassifier";
  if (!e.classifier && node.op_type != "TreeEnsembleRegressor")
    throw std::runtime_error("trees::compile: not a TreeEnsemble node: " + node.op_type);
  const auto& tids = ints(node, "nodes_treeids");
  const auto& nids = ints(node, "nodes_nodeids");
  const auto& fids = ints(node, "nodes_featureids");
  const auto& tnodes = ints(node, "nodes_truenodeids");
  const auto& fnodes = ints(node, "nodes_falsenodeids");
  const auto& miss = ints(node, "nodes_missing_value_tracks_true", false);
  auto vals = floats(node, "nodes_values", "nodes_values_as_tensor");
  auto modes_a = node.attr("nodes_modes");
  if (!modes_a) throw std::runtime_error("TreeEnsemble: missing nodes_modes");
  const size_t nn = tids.size();
  if (nids.size() != nn || fids.size() != nn || tnodes.size() != nn || fnodes.size() != nn ||
      vals.size() != nn || modes_a->strings.size() != nn)
    throw std::runtime_error("TreeEnsemble: node attribute lengths differ");

  // dense tree ordering by tree id
  std::map<int64_t, int32_t> tree_of;
  for (auto t : tids) tree_of.emplace(t, 0);
  int32_t ti = 0;
  for (auto& kv : tree_of) kv.second = ti++;
  e.trees.resize(tree_of.size());
  std::vector<std::map<int64_t, int32_t>> idx(tree_of.size());
  for (size_t k = 0; k < nn; ++k) {
    int32_t t = tree_of[tids[k]];
    if (idx[t].count(nids[k])) throw std::runtime_error("TreeEnsemble: duplicate node id");
    idx[t][nids[k]] = int32_t(e.trees[t].size());
    GNode g;
    g.thr = vals[k];
    g.feat = int32_t(fids[k]);
    g.mode = parse_mode(modes_a->strings[k]);
    g.miss = miss.empty() ? 0 : uint8_t(miss[k] != 0);
    e.trees[t].push_back(g);
  }
  for (size_t k = 0; k < nn; ++k) {
    int32_t t = tree_of[tids[k]];
    GNode& g = e.trees[t][idx[t][nids[k]]];
    if (g.mode == LEAF) continue;
    auto it = idx[t].find(tnodes[k]);
    auto jt = idx[t].find(fnodes[k]);
    if (it == idx[t].end() || jt == idx[t].end()) throw std::runtime_error("TreeEnsemble: dangling child id");
    g.t = it->second;
    g.f = jt->second;
    e.max_feature = std::max(e.max_feature, g.feat);
  }
  // put each root at index 0
  for (auto& tr : e.trees) {
    std::vector<uint8_t> is_child(tr.size(), 0);
    for (auto& g : tr)
      if (g.mode != LEAF) { is_child[g.t] = 1; is_child[g.f] = 1; }
    int32_t root = -1;
    for (size_t k = 0; k < tr.size(); ++k)
      if (!is_child[k]) { if (root >= 0) throw std::runtime_error("TreeEnsemble: tree has several roots"); root = int32_t(k); }
    if (root < 0) throw std::runtime_error("TreeEnsemble: cyclic tree");
    if (root != 0) {
      std::swap(tr[0], tr[root]);
      for (auto& g : tr) {
        if (g.mode == LEAF) continue;
        for (int32_t* c : {&g.t, &g.f}) {
          if (*c == 0) *c = root; else if (*c == root) *c = 0;
        }
      }
    }
  }

  // leaves
  const char* pre = e.classifier ? "class" : "target";
  std::string p(pre);
  const auto& lt = ints(node, (p + "_treeids").c_str());
  const auto& ln = ints(node, (p + "_nodeids").c_str());
  const auto& lid = ints(node, (p + "_ids").c_str());
  auto lw = floats(node, (p + "_weights").c_str(), (p + "_weights_as_tensor").c_str());
  if (ln.size() != lt.size() || lid.size() != lt.size() || lw.size() != lt.size())
    throw std::runtime_error("TreeEnsemble: leaf attribute lengths differ");
  e.base_values = floats(node, "base_values", "base_values_as_tensor");
  std::string post = node.gets("post_transform", "NONE");
  e.post = post == "NONE" ? NONE : post == "LOGISTIC" ? LOGISTIC : post == "SOFTMAX" ? SOFTMAX
           : post == "SOFTMAX_ZERO" ? SOFTMAX_ZERO : post == "PROBIT" ? PROBIT : -1;
  if (e.post < 0) throw std::runtime_error("TreeEnsemble: unknown post_transform " + post);

  bool all_positive = true;
  if (e.classifier) {
    if (auto a = node.attr("classlabels_int64s")) e.classlabels = a->ints;
    else if (auto b = node.attr("classlabels_strings")) {
      for (size_t k = 0; k < b->strings.size(); ++k) e.classlabels.push_back(int64_t(k));
    }
    int32_t ncls = int32_t(e.classlabels.size());
    if (ncls < 2) throw std::runtime_error("TreeEnsembleClassifier: needs >= 2 class labels");
    int64_t first = lid.empty() ? 0 : lid[0];
    bool single = true;
    for (auto c : lid) single &= (c == first);
    for (auto w : lw) all_positive &= (w >= 0);
    e.binary_case = ncls == 2 && single;
    e.binary_class = int32_t(first);
    e.n_targets = e.binary_case ? 1 : ncls;
    e.n_outputs = ncls;
  } else {
    e.n_targets = int32_t(node.geti("n_targets", 1));
    e.n_outputs = e.n_targets;
    std::string agg = node.gets("aggregate_function", "SUM");
    e.aggregate = agg == "SUM" ? SUM : agg == "AVERAGE" ? AVERAGE : agg == "MIN" ? MIN : agg == "MAX" ? MAX : -1;
    if (e.aggregate < 0) throw std::runtime_error("TreeEnsembleRegressor: unknown aggregate " + agg);
  }
  // weights_are_all_positive only matters for the binary NONE case (stored in binary_class sign)
  if (e.binary_case && !all_positive) e.binary_class |= 0x100;

  const int32_t K = e.n_targets;
  int32_t n_leaves = 0;
  for (auto& tr : e.trees)
    for (auto& g : tr)
      if (g.mode == LEAF) g.leaf = n_leaves++;
  e.leaf_w.assign(size_t(n_leaves) * K, 0.f);
  e.leaf_has.assign(size_t(n_leaves) * K, 0);
  for (size_t k = 0; k < lt.size(); ++k) {
    auto tt = tree_of.find(lt[k]);
    if (tt == tree_of.end()) throw std::runtime_error("TreeEnsemble: leaf refers to unknown tree");
    auto& m = idx[tt->second];
    auto it = m.find(ln[k]);
    if (it == m.end()) throw std::runtime_error("TreeEnsemble: leaf refers to unknown node");
    GNode& g = e.trees[tt->second][it->second];
    if (g.mode != LEAF) throw std::runtime_error("TreeEnsemble: weight on a non-leaf node");
    int64_t col = e.binary_case ? 0 : lid[k];
    if (col < 0 || col >= K) throw std::runtime_error("TreeEnsemble: target/class id out of range");
    e.leaf_w[size_t(g.leaf) * K + col] += lw[k];
    e.leaf_has[size_t(g.leaf) * K + col] = 1;
  }
  // max depth
  for (auto& tr : e.trees) {
    std::function<int32_t(int32_t)> depth = [&](int32_t i) -> int32_t {
      if (tr[i].mode == LEAF) return 0;
      return 1 + std::max(depth(tr[i].t), depth(tr[i].f));
    };
    e.max_depth = std::max(e.max_depth, depth(0));
  }
  return e;
}

void eval_raw(const Ensemble& e, const float* X, int64_t n, int64_t n_feat, float* scores) {
  if (e.max_feature >= n_feat) throw std::runtime_error("TreeEnsemble: input has too few features");
  const int32_t K = e.n_targets;
  const int32_t T = e.n_trees();
  std::vector<float> acc(K);
  std::vector<uint8_t> has(K);
  for (int64_t s = 0; s < n; ++s) {
    const float* x = X + s * n_feat;
    std::fill(acc.begin(), acc.end(), 0.f);
    std::fill(has.begin(), has.end(), 0);
    for (int32_t t = 0; t < T; ++t) {
      const auto& tr = e.trees[t];
      int32_t i = 0;
      while (tr[i].mode != LEAF) {
        const GNode& g = tr[i];
        i = go_true(x[g.feat], g.thr, g.mode, g.miss) ? g.t : g.f;
      }
      const float* w = &e.leaf_w[size_t(tr[i].leaf) * K];
      const uint8_t* h = &e.leaf_has[size_t(tr[i].leaf) * K];
      for (int32_t k = 0; k < K; ++k) {
        if (e.aggregate == SUM || e.aggregate == AVERAGE) acc[k] += w[k];
        else if (h[k]) {
          if (!has[k]) acc[k] = w[k];
          else acc[k] = e.aggregate == MIN ? std::min(acc[k], w[k]) : std::max(acc[k], w[k]);
          has[k] = 1;
        }
      }
    }
    for (int32_t k = 0; k < K; ++k) {
      float v = acc[k];
      if (e.aggregate == AVERAGE) v /= float(T);
      float b = 0.f;
      if (e.binary_case) {
        if (e.base_values.size() == 1) b = e.base_values[0];
        else if (e.base_values.size() == 2) b = e.base_values[e.binary_class & 1];
      } else if (size_t(k) < e.base_values.size()) {
        b = e.base_values[k];
      }
      scores[s * K + k] = v + b;
    }
  }
}

void post_transform(const Ensemble& e, const float* scores, int64_t n, float* out, int64_t* labels) {
  const int32_t K = e.n_targets;
  const int32_t O = e.n_outputs;
  std::vector<float> z(O);
  for (int64_t s = 0; s < n; ++s) {
    const float* sc = scores + s * K;
    if (e.binary_case) {
      const int c = e.binary_class & 1;
      const float v = sc[0];
      if (e.post == LOGISTIC) {
        z[c] = 1.f / (1.f + std::exp(-v));
        z[1 - c] = 1.f / (1.f + std::exp(v));
      } else {
        const bool all_pos = !(e.binary_class & 0x100);
        z[c] = v;
        z[1 - c] = all_pos ? 1.f - v : -v;
        if (e.post == PROBIT) { z[c] = 1.41421356f * erfinv(2 * z[c] - 1); z[1 - c] = 1.41421356f * erfinv(2 * z[1 - c] - 1); }
        else if (e.post == SOFTMAX || e.post == SOFTMAX_ZERO) {
          float m = std::max(z[0], z[1]);
          float a = std::exp(z[0] - m), b = std::exp(z[1] - m);
          z[0] = a / (a + b); z[1] = b / (a + b);
        }
      }
    } else {
      for (int32_t k = 0; k < O; ++k) z[k] = sc[k];
      if (e.post == LOGISTIC) {
        for (auto& v : z) v = 1.f / (1.f + std::exp(-v));
      } else if (e.post == SOFTMAX || e.post == SOFTMAX_ZERO) {
        float m = -std::numeric_limits<float>::infinity();
        for (auto v : z) if (!(e.post == SOFTMAX_ZERO && v == 0.f)) m = std::max(m, v);
        float sum = 0.f;
        for (auto& v : z) {
          if (e.post == SOFTMAX_ZERO && v == 0.f) { v = 0.f; continue; }
          v = std::exp(v - m); sum += v;
        }
        for (auto& v : z) v = sum > 0 ? v / sum : 0.f;
      } else if (e.post == PROBIT) {
        for (auto& v : z) v = 1.41421356f * erfinv(2 * v - 1);
      }
    }
    for (int32_t k = 0; k < O; ++k) out[s * O + k] = z[k];
    if (labels && e.classifier) {
      int32_t best = 0;
      for (int32_t k = 1; k < O; ++k)
        if (z[k] > z[best]) best = k;
      labels[s] = e.classlabels.empty() ? best : e.classlabels[best];
    }
  }
}

uint32_t node_meta(uint32_t feat, uint32_t mode, uint32_t miss) {
  return (feat & 0xffff) | (mode << 16) | (miss << 19);
}

Sparse to_sparse(const Ensemble& e) {
  Sparse sp;
  sp.depth = std::max<int32_t>(e.max_depth, 0);
  sp.n_trees = e.n_trees();
  sp.k = e.n_targets;
  size_t total = 0;
  for (auto& tr : e.trees) total += tr.size();
  if (total >= (size_t(1) << 31)) throw std::runtime_error("TreeEnsemble: too many nodes for 32-bit indices");
  sp.nodes.assign(total * 4, 0);
  sp.roots.resize(e.trees.size());
  int32_t off = 0;
  for (size_t t = 0; t < e.trees.size(); ++t) {
    const auto& tr = e.trees[t];
    sp.roots[t] = off;  // compile() puts each root at index 0
    for (size_t i = 0; i < tr.size(); ++i) {
      const GNode& g = tr[i];
      int32_t* o = &sp.nodes[(size_t(off) + i) * 4];
      if (g.mode == LEAF) {
        o[0] = int32_t(node_meta(0, LEAF, 0));
        o[2] = g.leaf;
        continue;
      }
      if (g.feat < 0 || g.feat > 0xffff) throw std::runtime_error("TreeEnsemble: feature id out of the device range");
      o[0] = int32_t(node_meta(uint32_t(g.feat), g.mode, g.miss));
      std::memcpy(&o[1], &g.thr, 4);
      o[2] = off + g.t;
      o[3] = off + g.f;
    }
    off += int32_t(tr.size());
  }
  sp.leaf_w = e.leaf_w;
  sp.leaf_has = e.leaf_has;
  return sp;
}

Complete to_complete(const Ensemble& e, int32_t max_depth_limit) {
  if (e.max_depth > max_depth_limit)
    throw std::runtime_error("TreeEnsemble: depth " + std::to_string(e.max_depth) +
                             " exceeds the complete-layout limit " + std::to_string(max_depth_limit));
  Complete c;
  c.depth = std::max<int32_t>(e.max_depth, 1);
  c.n_trees = e.n_trees();
  c.k = e.n_targets;
  const int32_t D = c.depth;
  const int64_t n_int = (int64_t(1) << D) - 1;
  const int64_t n_leaf = int64_t(1) << D;
  c.nodes.assign(size_t(c.n_trees) * n_int * 2, 0.f);
  c.leaves.assign(size_t(c.n_trees) * n_leaf * c.k, 0.f);
  auto meta_bits = [](uint32_t feat, uint32_t mode, uint32_t miss) {
    uint32_t m = node_meta(feat, mode, miss);
    float f;
    std::memcpy(&f, &m, 4);
    return f;
  };
  const float dummy_meta = meta_bits(0, LEQ, 1);
  const float inf = std::numeric_limits<float>::infinity();
  for (int32_t t = 0; t < c.n_trees; ++t) {
    float* nodes = &c.nodes[size_t(t) * n_int * 2];
    float* leaves = &c.leaves[size_t(t) * n_leaf * c.k];
    const auto& tr = e.trees[t];
    std::function<void(int64_t, int32_t, int32_t)> fill_leaf = [&](int64_t pos, int32_t d, int32_t leaf) {
      if (d == D) {
        std::memcpy(leaves + (pos - n_int) * c.k, &e.leaf_w[size_t(leaf) * c.k], sizeof(float) * c.k);
        return;
      }
      nodes[pos * 2] = inf;
      nodes[pos * 2 + 1] = dummy_meta;
      fill_leaf(2 * pos + 1, d + 1, leaf);
      fill_leaf(2 * pos + 2, d + 1, leaf);
    };
    std::function<void(int32_t, int64_t, int32_t)> place = [&](int32_t gi, int64_t pos, int32_t d) {
      const GNode& g = tr[gi];
      if (g.mode == LEAF) { fill_leaf(pos, d, g.leaf); return; }
      nodes[pos * 2] = g.thr;
      nodes[pos * 2 + 1] = meta_bits(uint32_t(g.feat), g.mode, g.miss);
      place(g.t, 2 * pos + 1, d + 1);
      place(g.f, 2 * pos + 2, d + 1);
    };
    place(0, 0, 0);
  }
  return c;
}

}  // namespace igp::trees

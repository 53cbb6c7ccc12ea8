// TreeEnsemble{Classifier,Regressor} (ai.onnx.ml) compiled from node attributes into
//  (a) a general pointer layout, evaluated by the CPU executor, and
//  (b) the implicit complete-tree layout streamed/staged by the HIP tree kernel:
//      node i -> children 2i+1 (true) / 2i+2 (false); shallower leaves are padded by
//      "don't-care" nodes whose two subtrees carry the same leaf vector, so results are
//      identical for every input (NaN included).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "onnx_model.h"

namespace igp::trees {

enum Mode : uint8_t { LEQ = 0, LT = 1, GTE = 2, GT = 3, EQ = 4, NEQ = 5, LEAF = 7 };
enum Aggregate : int32_t { SUM = 0, AVERAGE = 1, MIN = 2, MAX = 3 };
enum Post : int32_t { NONE = 0, LOGISTIC = 1, SOFTMAX = 2, SOFTMAX_ZERO = 3, PROBIT = 4 };

struct GNode {
  float thr = 0;
  int32_t feat = 0;
  uint8_t mode = LEAF;
  uint8_t miss = 0;  // missing_value_tracks_true
  int32_t t = -1, f = -1;  // child node indices within the tree
  int32_t leaf = -1;       // leaf index into Ensemble::leaf_w (rows of K)
};

struct Ensemble {
  bool classifier = false;
  int32_t n_targets = 1;   // K (targets, or score columns for classifiers)
  int32_t n_outputs = 1;   // classifier probability columns (2 in the binary case)
  int32_t aggregate = SUM;
  int32_t post = NONE;
  bool binary_case = false;
  int32_t binary_class = 1;
  std::vector<float> base_values;
  std::vector<int64_t> classlabels;
  std::vector<std::vector<GNode>> trees;  // roots at index 0
  std::vector<float> leaf_w;              // [n_leaves][K]
  std::vector<uint8_t> leaf_has;          // [n_leaves][K]: target touched (for MIN/MAX)
  int32_t max_depth = 0;
  int32_t max_feature = -1;

  int32_t n_trees() const { return int32_t(trees.size()); }
};

Ensemble compile(const onnx::Node& node);
// single-precision inverse error function (the PROBIT post transform: sqrt(2) * erfinv(2p - 1))
float erfinv(float x);

// Per-sample raw scores [N][K] (aggregated, + base values, before post transform).
void eval_raw(const Ensemble& e, const float* X, int64_t n, int64_t n_feat, float* scores);
// Apply post transform; classifier binary case expands K=1 scores to 2 probability columns.
void post_transform(const Ensemble& e, const float* scores, int64_t n, float* out, int64_t* labels);

// Complete layout for device kernels.
struct Complete {
  int32_t depth = 0;
  int32_t n_trees = 0;
  int32_t k = 1;
  std::vector<float> nodes;   // [T][2^D - 1][2]: (threshold, meta bits) meta = feat | mode<<16 | miss<<19
  std::vector<float> leaves;  // [T][2^D][K]
};
Complete to_complete(const Ensemble& e, int32_t max_depth_limit = 12);

// Pointer layout for the device's general tree kernel (any depth, any shape): all trees'
// nodes in one array, 16 B each {meta, threshold bits, true child, false child}; a leaf has
// mode LEAF and its leaf row in the "true child" slot. Children / leaf rows are global indices.
struct Sparse {
  int32_t depth = 0;   // longest root-to-leaf path (edges)
  int32_t n_trees = 0;
  int32_t k = 1;
  std::vector<int32_t> nodes;    // [N][4]
  std::vector<int32_t> roots;    // [T]
  std::vector<float> leaf_w;     // [L][K]
  std::vector<uint8_t> leaf_has; // [L][K]
};
Sparse to_sparse(const Ensemble& e);
uint32_t node_meta(uint32_t feat, uint32_t mode, uint32_t miss);

}  // namespace igp::trees

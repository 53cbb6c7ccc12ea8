// CPU executor for ONNX graphs of the supported model families.
//
// Plays two roles: (1) the CPU scoring path of config 1 (BASELINE: "CPU ONNX Runtime,
// 32-feature logistic, batch=1"), standing in for ONNX Runtime, which the reference uses
// through cgo (onnx_model.go:63-68, 222-238) and which cannot be installed offline;
// (2) the golden reference every HIP model kernel is tested against.
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "onnx_model.h"
#include "trees.h"

namespace igp::exec {

using onnx::Tensor;

class Executor {
 public:
  explicit Executor(onnx::Model model);
  // Run with named float inputs; returns every graph output.
  std::map<std::string, Tensor> run(const std::map<std::string, Tensor>& inputs) const;
  const onnx::Model& model() const { return model_; }
  // compiled tree ensembles by node index (shared with the device plan compiler)
  const trees::Ensemble* ensemble(size_t node_index) const;

 private:
  onnx::Model model_;
  std::map<size_t, std::shared_ptr<trees::Ensemble>> ensembles_;
  std::vector<size_t> order_;  // topological node order
};

}  // namespace igp::exec

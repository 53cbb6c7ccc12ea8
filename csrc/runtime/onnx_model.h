// ONNX ModelProto reader (the subset needed for fraud/LTV/abuse model families) and the
// graph data structures shared by the CPU executor and the device plan compiler.
//
// Replaces the ONNX Runtime session load of the reference
// (services/risk/internal/ml/onnx_model.go:44-82), which we cannot link (no ORT offline).
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace igp::onnx {

enum DType : int32_t { FLOAT = 1, UINT8 = 2, INT8 = 3, INT32 = 6, INT64 = 7, STRING = 8, BOOL = 9,
                       FLOAT16 = 10, DOUBLE = 11, BFLOAT16 = 16 };

// Host tensor: float32 or int64 payloads (everything the supported ops need).
struct Tensor {
  std::string name;
  int32_t dtype = FLOAT;
  std::vector<int64_t> dims;
  std::vector<float> f;
  std::vector<int64_t> i;
  int64_t numel() const {
    int64_t n = 1;
    for (auto d : dims) n *= d;
    return n;
  }
};

enum AttrType : int32_t { A_UNDEF = 0, A_FLOAT = 1, A_INT = 2, A_STRING = 3, A_TENSOR = 4,
                          A_GRAPH = 5, A_FLOATS = 6, A_INTS = 7, A_STRINGS = 8, A_TENSORS = 9 };

struct Attribute {
  std::string name;
  int32_t type = A_UNDEF;
  float f = 0;
  int64_t i = 0;
  std::string s;
  std::vector<float> floats;
  std::vector<int64_t> ints;
  std::vector<std::string> strings;
  std::shared_ptr<Tensor> t;
};

struct Node {
  std::string name, op_type, domain;
  std::vector<std::string> inputs, outputs;
  std::map<std::string, Attribute> attrs;

  const Attribute* attr(const std::string& n) const {
    auto it = attrs.find(n);
    return it == attrs.end() ? nullptr : &it->second;
  }
  int64_t geti(const std::string& n, int64_t d) const { auto a = attr(n); return a ? a->i : d; }
  float getf(const std::string& n, float d) const { auto a = attr(n); return a ? a->f : d; }
  std::string gets(const std::string& n, const std::string& d) const { auto a = attr(n); return a ? a->s : d; }
};

struct ValueInfo {
  std::string name;
  int32_t elem_type = 0;
  std::vector<int64_t> dims;       // -1 for symbolic
  std::vector<std::string> params; // symbolic names ("" when fixed)
};

struct Graph {
  std::string name;
  std::vector<Node> nodes;
  std::map<std::string, Tensor> initializers;
  std::vector<ValueInfo> inputs, outputs;
};

struct Model {
  int64_t ir_version = 0;
  std::string producer_name, producer_version;
  std::map<std::string, int64_t> opsets;  // domain -> version
  std::map<std::string, std::string> metadata;
  Graph graph;
};

Model parse_model(const std::string& bytes);
Model load_model(const std::string& path);

}  // namespace igp::onnx

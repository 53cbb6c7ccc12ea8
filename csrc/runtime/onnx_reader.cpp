// ONNX protobuf decoder (field numbers from onnx.proto, IR v3..v10).
#include <fstream>
#include <sstream>

#include "onnx_model.h"
#include "pb.h"

namespace igp::onnx {
namespace {

using pb::Reader;

void parse_tensor(std::string_view buf, Tensor& t) {
  Reader r(buf);
  uint32_t f, w;
  std::string raw;
  std::vector<double> dbl;
  std::vector<int64_t> i32;
  while (r.tag(f, w)) {
    switch (f) {
      case 1: r.repeated(w, t.dims, [](Reader& x) { return int64_t(x.varint()); }); break;
      case 2: t.dtype = int32_t(r.varint()); break;
      case 4: r.repeated(w, t.f, [](Reader& x) { return x.f32(); }); break;
      case 5: r.repeated(w, i32, [](Reader& x) { return int64_t(int32_t(x.varint())); }); break;
      case 7: r.repeated(w, t.i, [](Reader& x) { return int64_t(x.varint()); }); break;
      case 8: t.name = std::string(r.bytes()); break;
      case 9: raw = std::string(r.bytes()); break;
      case 10: r.repeated(w, dbl, [](Reader& x) { return x.f64(); }); break;
      case 13: throw std::runtime_error("onnx: external tensor data is not supported (" + t.name + ")");
      default: r.skip(w);
    }
  }
  const int64_t n = t.numel();
  auto need = [&](size_t bytes) {
    if (raw.size() != bytes)
      throw std::runtime_error("onnx: raw_data size mismatch for tensor " + t.name);
  };
  switch (t.dtype) {
    case FLOAT:
      if (!raw.empty()) { need(n * 4); t.f.resize(n); std::memcpy(t.f.data(), raw.data(), n * 4); }
      break;
    case DOUBLE:
      if (!raw.empty()) { need(n * 8); dbl.resize(n); std::memcpy(dbl.data(), raw.data(), n * 8); }
      t.f.assign(dbl.begin(), dbl.end());
      t.dtype = FLOAT;
      break;
    case INT64:
      if (!raw.empty()) { need(n * 8); t.i.resize(n); std::memcpy(t.i.data(), raw.data(), n * 8); }
      break;
    case INT32: case INT8: case UINT8: case BOOL: {
      if (!raw.empty()) {
        size_t es = t.dtype == INT32 ? 4 : 1;
        need(n * es);
        i32.resize(n);
        for (int64_t k = 0; k < n; ++k) {
          if (t.dtype == INT32) { int32_t v; std::memcpy(&v, raw.data() + 4 * k, 4); i32[k] = v; }
          else if (t.dtype == INT8) i32[k] = int8_t(raw[k]);
          else i32[k] = uint8_t(raw[k]);
        }
      }
      t.i.assign(i32.begin(), i32.end());
      t.dtype = INT64;
      break;
    }
    default:
      throw std::runtime_error("onnx: unsupported tensor dtype " + std::to_string(t.dtype) + " for " + t.name);
  }
  if (t.dtype == FLOAT && int64_t(t.f.size()) != n) throw std::runtime_error("onnx: float tensor size mismatch " + t.name);
  if (t.dtype == INT64 && int64_t(t.i.size()) != n) throw std::runtime_error("onnx: int tensor size mismatch " + t.name);
}

void parse_attr(std::string_view buf, Attribute& a) {
  Reader r(buf);
  uint32_t f, w;
  while (r.tag(f, w)) {
    switch (f) {
      case 1: a.name = std::string(r.bytes()); break;
      case 2: a.f = r.f32(); break;
      case 3: a.i = int64_t(r.varint()); break;
      case 4: a.s = std::string(r.bytes()); break;
      case 5: a.t = std::make_shared<Tensor>(); parse_tensor(r.bytes(), *a.t); break;
      case 7: r.repeated(w, a.floats, [](Reader& x) { return x.f32(); }); break;
      case 8: r.repeated(w, a.ints, [](Reader& x) { return int64_t(x.varint()); }); break;
      case 9: a.strings.emplace_back(r.bytes()); break;
      case 20: a.type = int32_t(r.varint()); break;
      default: r.skip(w);
    }
  }
  if (a.type == A_UNDEF) {  // IR < 0.0.2 style: infer from payload
    if (!a.floats.empty()) a.type = A_FLOATS;
    else if (!a.ints.empty()) a.type = A_INTS;
    else if (!a.strings.empty()) a.type = A_STRINGS;
    else if (a.t) a.type = A_TENSOR;
    else if (!a.s.empty()) a.type = A_STRING;
  }
}

void parse_node(std::string_view buf, Node& n) {
  Reader r(buf);
  uint32_t f, w;
  while (r.tag(f, w)) {
    switch (f) {
      case 1: n.inputs.emplace_back(r.bytes()); break;
      case 2: n.outputs.emplace_back(r.bytes()); break;
      case 3: n.name = std::string(r.bytes()); break;
      case 4: n.op_type = std::string(r.bytes()); break;
      case 5: { Attribute a; parse_attr(r.bytes(), a); n.attrs[a.name] = std::move(a); break; }
      case 7: n.domain = std::string(r.bytes()); break;
      default: r.skip(w);
    }
  }
}

void parse_value_info(std::string_view buf, ValueInfo& v) {
  Reader r(buf);
  uint32_t f, w;
  while (r.tag(f, w)) {
    if (f == 1) { v.name = std::string(r.bytes()); continue; }
    if (f != 2) { r.skip(w); continue; }
    Reader tp(r.bytes());  // TypeProto
    uint32_t f2, w2;
    while (tp.tag(f2, w2)) {
      if (f2 != 1) { tp.skip(w2); continue; }
      Reader tt(tp.bytes());  // TypeProto.Tensor
      uint32_t f3, w3;
      while (tt.tag(f3, w3)) {
        if (f3 == 1) v.elem_type = int32_t(tt.varint());
        else if (f3 == 2) {
          Reader sh(tt.bytes());  // TensorShapeProto
          uint32_t f4, w4;
          while (sh.tag(f4, w4)) {
            if (f4 != 1) { sh.skip(w4); continue; }
            Reader dim(sh.bytes());
            uint32_t f5, w5;
            int64_t dv = -1;
            std::string dp;
            while (dim.tag(f5, w5)) {
              if (f5 == 1) dv = int64_t(dim.varint());
              else if (f5 == 2) dp = std::string(dim.bytes());
              else dim.skip(w5);
            }
            v.dims.push_back(dv);
            v.params.push_back(dp);
          }
        } else tt.skip(w3);
      }
    }
  }
}

void parse_graph(std::string_view buf, Graph& g) {
  Reader r(buf);
  uint32_t f, w;
  while (r.tag(f, w)) {
    switch (f) {
      case 1: { Node n; parse_node(r.bytes(), n); g.nodes.push_back(std::move(n)); break; }
      case 2: g.name = std::string(r.bytes()); break;
      case 5: { Tensor t; parse_tensor(r.bytes(), t); std::string nm = t.name; g.initializers[nm] = std::move(t); break; }
      case 11: { ValueInfo v; parse_value_info(r.bytes(), v); g.inputs.push_back(std::move(v)); break; }
      case 12: { ValueInfo v; parse_value_info(r.bytes(), v); g.outputs.push_back(std::move(v)); break; }
      default: r.skip(w);
    }
  }
  // graph inputs that are initializers are constants, not runtime inputs (IR < 4 convention)
  std::vector<ValueInfo> real;
  for (auto& v : g.inputs)
    if (!g.initializers.count(v.name)) real.push_back(v);
  g.inputs = std::move(real);
}

}  // namespace

Model parse_model(const std::string& bytes) {
  Model m;
  Reader r(bytes);
  uint32_t f, w;
  bool has_graph = false;
  while (r.tag(f, w)) {
    switch (f) {
      case 1: m.ir_version = int64_t(r.varint()); break;
      case 2: m.producer_name = std::string(r.bytes()); break;
      case 3: m.producer_version = std::string(r.bytes()); break;
      case 7: parse_graph(r.bytes(), m.graph); has_graph = true; break;
      case 8: {
        Reader o(r.bytes());
        uint32_t f2, w2;
        std::string dom;
        int64_t ver = 0;
        while (o.tag(f2, w2)) {
          if (f2 == 1) dom = std::string(o.bytes());
          else if (f2 == 2) ver = int64_t(o.varint());
          else o.skip(w2);
        }
        m.opsets[dom] = ver;
        break;
      }
      case 14: {
        Reader o(r.bytes());
        uint32_t f2, w2;
        std::string k, v;
        while (o.tag(f2, w2)) {
          if (f2 == 1) k = std::string(o.bytes());
          else if (f2 == 2) v = std::string(o.bytes());
          else o.skip(w2);
        }
        m.metadata[k] = v;
        break;
      }
      default: r.skip(w);
    }
  }
  if (!has_graph) throw std::runtime_error("onnx: model has no graph");
  return m;
}

Model load_model(const std::string& path) {
  std::ifstream in(path, std::ios::binary);
  if (!in) throw std::runtime_error("onnx: cannot open " + path);
  std::stringstream ss;
  ss << in.rdbuf();
  return parse_model(ss.str());
}

}  // namespace igp::onnx

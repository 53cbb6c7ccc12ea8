// Minimal protobuf wire-format reader/writer used by the ONNX reader and the risk.v1 codec.
// No protoc / libprotobuf in the image: both formats are decoded directly from the wire.
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

namespace igp::pb {

enum Wire : uint32_t { VARINT = 0, I64 = 1, LEN = 2, I32 = 5 };

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  Reader(const void* data, size_t n) : p((const uint8_t*)data), end((const uint8_t*)data + n) {}
  explicit Reader(std::string_view s) : Reader(s.data(), s.size()) {}
  bool done() const { return p >= end; }

  uint64_t varint() {
    uint64_t v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      if (p >= end) throw std::runtime_error("pb: truncated varint");
      uint8_t b = *p++;
      v |= uint64_t(b & 0x7f) << shift;
      if (!(b & 0x80)) return v;
    }
    throw std::runtime_error("pb: varint too long");
  }
  // returns false at end of message
  bool tag(uint32_t& field, uint32_t& wire) {
    if (p >= end) return false;
    uint64_t t = varint();
    field = uint32_t(t >> 3);
    wire = uint32_t(t & 7);
    if (field == 0) throw std::runtime_error("pb: field 0");
    return true;
  }
  std::string_view bytes() {
    uint64_t n = varint();
    if (n > uint64_t(end - p)) throw std::runtime_error("pb: truncated length-delimited field");
    std::string_view s((const char*)p, n);
    p += n;
    return s;
  }
  uint32_t fixed32() {
    if (end - p < 4) throw std::runtime_error("pb: truncated fixed32");
    uint32_t v;
    std::memcpy(&v, p, 4);
    p += 4;
    return v;
  }
  uint64_t fixed64() {
    if (end - p < 8) throw std::runtime_error("pb: truncated fixed64");
    uint64_t v;
    std::memcpy(&v, p, 8);
    p += 8;
    return v;
  }
  float f32() { uint32_t u = fixed32(); float f; std::memcpy(&f, &u, 4); return f; }
  double f64() { uint64_t u = fixed64(); double d; std::memcpy(&d, &u, 8); return d; }
  void skip(uint32_t wire) {
    switch (wire) {
      case VARINT: varint(); break;
      case I64: fixed64(); break;
      case LEN: bytes(); break;
      case I32: fixed32(); break;
      default: throw std::runtime_error("pb: unsupported wire type " + std::to_string(wire));
    }
  }
  // repeated scalar, packed or not
  template <class T, class F>
  void repeated(uint32_t wire, std::vector<T>& out, F one) {
    if (wire == LEN) {
      Reader sub(bytes());
      while (!sub.done()) out.push_back(one(sub));
    } else {
      out.push_back(one(*this));
    }
  }
};

struct Writer {
  std::string buf;
  void varint(uint64_t v) {
    while (v >= 0x80) { buf.push_back(char(v | 0x80)); v >>= 7; }
    buf.push_back(char(v));
  }
  void tag(uint32_t field, uint32_t wire) { varint((uint64_t(field) << 3) | wire); }
  void u64(uint32_t field, uint64_t v) { if (v) { tag(field, VARINT); varint(v); } }
  void i64(uint32_t field, int64_t v) { if (v) { tag(field, VARINT); varint(uint64_t(v)); } }
  void i32(uint32_t field, int32_t v) { if (v) { tag(field, VARINT); varint(uint64_t(int64_t(v))); } }
  void boolean(uint32_t field, bool v) { if (v) { tag(field, VARINT); varint(1); } }
  void f32(uint32_t field, float v) {
    uint32_t u; std::memcpy(&u, &v, 4);
    if (u == 0) return;  // proto3: +0.0 is the default and is not emitted
    tag(field, I32);
    buf.append((const char*)&u, 4);
  }
  void str(uint32_t field, std::string_view s) {
    if (s.empty()) return;
    tag(field, LEN); varint(s.size()); buf.append(s.data(), s.size());
  }
  void str_always(uint32_t field, std::string_view s) {
    tag(field, LEN); varint(s.size()); buf.append(s.data(), s.size());
  }
  // length-delimited sub-message: write into tmp then append
  void msg(uint32_t field, const std::string& body) {
    tag(field, LEN); varint(body.size()); buf.append(body);
  }
  // header of a sub-message whose body (of `size` bytes) the caller writes next
  void msg_header(uint32_t field, size_t size) { tag(field, LEN); varint(size); }
  static size_t varint_size(uint64_t v) { size_t n = 1; while (v >= 0x80) { v >>= 7; ++n; } return n; }
};

// Same field API as Writer, counting bytes only (sizes nested messages before writing them).
struct Sizer {
  size_t n = 0;
  void varint(uint64_t v) { n += Writer::varint_size(v); }
  void tag(uint32_t field, uint32_t wire) { varint((uint64_t(field) << 3) | wire); }
  void u64(uint32_t field, uint64_t v) { if (v) { tag(field, VARINT); varint(v); } }
  void i64(uint32_t field, int64_t v) { if (v) { tag(field, VARINT); varint(uint64_t(v)); } }
  void i32(uint32_t field, int32_t v) { if (v) { tag(field, VARINT); varint(uint64_t(int64_t(v))); } }
  void boolean(uint32_t field, bool v) { if (v) { tag(field, VARINT); varint(1); } }
  void f32(uint32_t field, float v) {
    uint32_t u; std::memcpy(&u, &v, 4);
    if (u == 0) return;
    tag(field, I32);
    n += 4;
  }
  void str(uint32_t field, std::string_view s) { if (!s.empty()) str_always(field, s); }
  void str_always(uint32_t field, std::string_view s) { tag(field, LEN); varint(s.size()); n += s.size(); }
  void msg_header(uint32_t field, size_t size) { tag(field, LEN); varint(size); }
};

}  // namespace igp::pb

#include "wire.h"

#include <cstring>

#include "pb.h"
#include "xxh64.h"

namespace igp::wire {

const char* const kReasonCodes[12] = {
    "HIGH_VELOCITY", "NEW_ACCOUNT_LARGE_TX", "MULTIPLE_DEVICES", "IP_COUNTRY_MISMATCH",
    "VPN_DETECTED", "RAPID_DEPOSIT_WITHDRAW", "BONUS_ABUSE", "KNOWN_FRAUDSTER",
    "ML_HIGH_RISK", "SUSPICIOUS_PATTERN", "MULTI_ACCOUNT", "DEVICE_FINGERPRINT_MISMATCH"};

void RequestBatch::clear() {
  account_id.clear(); account_hash.clear(); amount.clear(); tx_type.clear();
  device_hash.clear(); fp_hash.clear(); ip_hash.clear(); arena.clear();
}

void RequestBatch::reserve(size_t n) {
  account_id.reserve(n); account_hash.reserve(n); amount.reserve(n); tx_type.reserve(n);
  device_hash.reserve(n); fp_hash.reserve(n); ip_hash.reserve(n);
}

const std::string& RequestBatch::own(const char* data, size_t n) {
  arena.emplace_back(std::make_unique<std::string>(data, n));
  return *arena.back();
}

uint8_t tx_type_id(const char* s, size_t n) {
  auto eq = [&](const char* lit, size_t ln) { return ln == n && std::memcmp(s, lit, n) == 0; };
  switch (n) {
    case 3:
      if (eq("bet", 3)) return TX_BET;
      if (eq("win", 3)) return TX_WIN;
      break;
    case 5:
      if (eq("bonus", 5)) return TX_BONUS;
      break;
    case 6:
      if (eq("refund", 6)) return TX_REFUND;
      break;
    case 7:
      if (eq("deposit", 7)) return TX_DEPOSIT;
      break;
    case 8:
      if (eq("withdraw", 8)) return TX_WITHDRAW;
      break;
  }
  return TX_UNKNOWN;
}

void parse_tx_row(const char* data, size_t n, TxRow& out) {
  // Fast path for the shape every client sends: one-byte tags (fields 1..15) and one-byte
  // lengths; anything else (multi-byte tags or lengths, unknown wire types) goes through the
  // general pb::Reader. Truncation throws on both paths.
  const uint8_t* p = (const uint8_t*)data;
  const uint8_t* const end = p + n;
  std::string_view acct, type, ip, dev, fp;
  int64_t amount = 0;
  while (p < end) {
    const uint32_t t = *p;
    if (__builtin_expect(t >= 0x80, 0)) {  // multi-byte tag: general reader for the rest
      pb::Reader r(p, size_t(end - p));
      uint32_t f, w;
      while (r.tag(f, w)) {
        switch (f) {
          case 1: acct = r.bytes(); break;
          case 3: amount = int64_t(r.varint()); break;
          case 4: type = r.bytes(); break;
          case 8: ip = r.bytes(); break;
          case 9: dev = r.bytes(); break;
          case 10: fp = r.bytes(); break;
          default: r.skip(w);
        }
      }
      break;
    }
    ++p;
    const uint32_t f = t >> 3, w = t & 7;
    if (f == 0) throw std::runtime_error("pb: field 0");
    if (w == pb::LEN) {
      if (p >= end) throw std::runtime_error("pb: truncated varint");
      uint64_t len = *p;
      if (__builtin_expect(len < 0x80, 1)) {
        ++p;
      } else {
        pb::Reader r(p, size_t(end - p));
        len = r.varint();
        p = r.p;
      }
      if (len > uint64_t(end - p)) throw std::runtime_error("pb: truncated length-delimited field");
      const std::string_view v((const char*)p, len);
      p += len;
      switch (f) {
        case 1: acct = v; break;
        case 4: type = v; break;
        case 8: ip = v; break;
        case 9: dev = v; break;
        case 10: fp = v; break;
        default: break;  // player_id, currency, game/round, user_agent, session, metadata
      }
    } else if (w == pb::VARINT) {
      pb::Reader r(p, size_t(end - p));
      const uint64_t v = r.varint();
      p = r.p;
      if (f == 3) amount = int64_t(v);
    } else {
      pb::Reader r(p, size_t(end - p));
      r.skip(w);
      p = r.p;
    }
  }
  out.account = acct;
  out.account_hash = id_hash(acct, SEED_ACCOUNT);
  ReqRec& q = out.rec;
  q.slot = -1;
  q.tx_type = tx_type_id(type.data(), type.size());
  q.amount = amount;
  q.dev_hash = id_hash(dev, SEED_DEVICE);
  q.fp_hash = id_hash(fp, SEED_FINGERPRINT);
  q.ip_hash = id_hash(ip, SEED_IP);
  q.ts = 0;
}

void parse_batch_rows(const char* data, size_t n, std::vector<TxRow>& out) {
  pb::Reader r(data, n);
  uint32_t f, w;
  while (r.tag(f, w)) {
    if (f == 1 && w == pb::LEN) {
      auto m = r.bytes();
      out.emplace_back();
      parse_tx_row(m.data(), m.size(), out.back());
    } else {
      r.skip(w);
    }
  }
}

void parse_tx(const char* data, size_t n, RequestBatch& out) {
  TxRow row;
  parse_tx_row(data, n, row);
  out.account_id.push_back(row.account);  // a view into the batch's arena copy of the payload
  out.account_hash.push_back(row.account_hash);
  out.amount.push_back(row.rec.amount);
  out.tx_type.push_back(uint8_t(row.rec.tx_type));
  out.device_hash.push_back(row.rec.dev_hash);
  out.fp_hash.push_back(row.rec.fp_hash);
  out.ip_hash.push_back(row.rec.ip_hash);
}

void parse_batch(const char* data, size_t n, RequestBatch& out) {
  const std::string& own = out.own(data, n);
  pb::Reader r(own.data(), own.size());
  uint32_t f, w;
  while (r.tag(f, w)) {
    if (f == 1 && w == pb::LEN) {
      auto m = r.bytes();
      parse_tx(m.data(), m.size(), out);
    } else {
      r.skip(w);
    }
  }
}

// ---------------------------------------------------------------------------- serializer
// Raw-pointer writer: the caller guarantees the space (kMaxTxResponse per response body).
// Field semantics are proto3's: zero scalars are not emitted, +0.0 floats are not emitted.
namespace {

struct Out {
  char* p;
  inline void varint(uint64_t v) {
    while (v >= 0x80) {
      *p++ = char(v | 0x80);
      v >>= 7;
    }
    *p++ = char(v);
  }
  inline void tag(uint32_t field, uint32_t wire) { varint((uint64_t(field) << 3) | wire); }
  inline void i32(uint32_t field, int32_t v) {
    if (v) { tag(field, pb::VARINT); varint(uint64_t(int64_t(v))); }
  }
  inline void i64(uint32_t field, int64_t v) {
    if (v) { tag(field, pb::VARINT); varint(uint64_t(v)); }
  }
  inline void boolean(uint32_t field, bool v) {
    if (v) { tag(field, pb::VARINT); *p++ = 1; }
  }
  inline void f32(uint32_t field, float v) {
    uint32_t u;
    std::memcpy(&u, &v, 4);
    if (u == 0) return;
    tag(field, pb::I32);
    std::memcpy(p, &u, 4);
    p += 4;
  }
  inline void bytes(const char* s, size_t n) {
    std::memcpy(p, s, n);
    p += n;
  }
};

// pre-encoded "field 3, LEN, length, bytes" of every reason code (padded to 32 bytes: copied
// with one fixed-size memcpy, the pointer advanced by the real length)
struct ReasonTable {
  char enc[12][32];
  uint8_t len[12];
  ReasonTable() {
    std::memset(enc, 0, sizeof enc);
    for (int b = 0; b < 12; ++b) {
      Out o{enc[b]};
      const size_t n = std::strlen(kReasonCodes[b]);
      o.tag(3, pb::LEN);
      o.varint(n);
      o.bytes(kReasonCodes[b], n);
      len[b] = uint8_t(o.p - enc[b]);
    }
  }
};
const ReasonTable& reasons_table() {
  static const ReasonTable t;
  return t;
}

// Field writers for the response hot path. proto3 omits zero scalars, which made every field a
// data-dependent branch (~30 per row, mispredicted whenever a counter flips between 0 and not).
// Here each field is STORED unconditionally - tag and value image - and the pointer only
// advances when the value is non-zero; the remaining branches (value < 128, >= 2^56) follow a
// field's value range and predict well. The caller's buffer keeps >= 16 bytes of slack past
// any field. Values needing more than 8 varint bytes (negative integers) take the plain path.
struct FastOut {
  char* p;
  static inline uint64_t spread7(uint64_t v) {  // 7-bit groups of v into the low 7 bits of bytes 0..7
    return (v & 0x7fULL) | ((v << 1) & 0x7f00ULL) | ((v << 2) & 0x7f0000ULL) | ((v << 3) & 0x7f000000ULL) |
           ((v << 4) & 0x7f00000000ULL) | ((v << 5) & 0x7f0000000000ULL) | ((v << 6) & 0x7f000000000000ULL) |
           ((v << 7) & 0x7f00000000000000ULL);
  }
  static inline int vlen(uint64_t v) { return (70 - __builtin_clzll(v | 1)) / 7; }
  // tag (1 or 2 bytes, pre-encoded little-endian in `tag`, `tl` bytes) + varint v, skipped if v == 0
  inline void uvar(uint32_t tag, int tl, uint64_t v) {
    if (__builtin_expect(v >> 56, 0)) {  // >= 2^56 (never 0): the plain writer
      std::memcpy(p, &tag, 2);
      Out o{p + tl};
      o.varint(v);
      p = o.p;
      return;
    }
    std::memcpy(p, &tag, 2);
    if (v < 128) {  // counters, score, action: per field a well-predicted branch
      p[tl] = char(v);
      p += (v != 0) * (tl + 1);
      return;
    }
    const int n = vlen(v);
    const uint64_t cont = 0x8080808080808080ULL & ((uint64_t(1) << (8 * (n - 1))) - 1);
    const uint64_t enc = spread7(v) | cont;
    std::memcpy(p + tl, &enc, 8);
    p += tl + n;
  }
  inline void i32(uint32_t tag, int tl, int32_t v) { uvar(tag, tl, uint64_t(int64_t(v))); }
  inline void i64(uint32_t tag, int tl, int64_t v) { uvar(tag, tl, uint64_t(v)); }
  inline void f32(uint32_t tag, int tl, float v) {
    uint32_t u;
    std::memcpy(&u, &v, 4);
    std::memcpy(p, &tag, 2);
    std::memcpy(p + tl, &u, 4);
    p += (u != 0) * (tl + 4);
  }
  inline void boolean(uint32_t tag, int tl, bool v) {
    std::memcpy(p, &tag, 2);
    p[tl] = 1;
    p += v * (tl + 1);
  }
};

// the 1- or 2-byte encoding of (field << 3 | wire) as a little-endian word
constexpr uint32_t T1(uint32_t f, uint32_t w) { return (f << 3) | w; }
constexpr uint32_t T2(uint32_t f, uint32_t w) { return (((f << 3) | w) & 0x7f) | 0x80 | ((((f << 3) | w) >> 7) << 8); }

inline void write_feature_vector(FastOut& o, const FeatRec& x) {
  o.i32(T1(1, 0), 1, x.tx_count_1m);
  o.i32(T1(2, 0), 1, x.tx_count_5m);
  o.i32(T1(3, 0), 1, x.tx_count_1h);
  o.i64(T1(4, 0), 1, x.tx_sum_1h);
  o.f32(T1(5, 5), 1, x.tx_avg_1h);
  o.i32(T1(6, 0), 1, x.unique_devices_24h);
  o.i32(T1(7, 0), 1, x.unique_ips_24h);
  o.i32(T1(8, 0), 1, x.ip_country_changes_7d);
  o.i32(T1(9, 0), 1, x.device_age_days);
  o.i32(T1(10, 0), 1, x.account_age_days);
  o.i64(T1(11, 0), 1, x.total_deposits);
  o.i64(T1(12, 0), 1, x.total_withdrawals);
  o.i64(T1(13, 0), 1, x.net_deposit);
  o.i32(T1(14, 0), 1, x.deposit_count);
  o.i32(T1(15, 0), 1, x.withdraw_count);
  o.i32(T2(16, 0), 2, x.time_since_last_tx);
  o.i32(T2(17, 0), 2, x.session_duration);
  o.f32(T2(18, 5), 2, x.avg_bet_size);
  o.f32(T2(19, 5), 2, x.win_rate);
  o.boolean(T2(20, 0), 2, x.flags & FR_VPN);
  o.boolean(T2(21, 0), 2, x.flags & FR_PROXY);
  o.boolean(T2(22, 0), 2, x.flags & FR_TOR);
  o.boolean(T2(23, 0), 2, x.flags & FR_DISPOSABLE);
  o.i32(T2(24, 0), 2, x.bonus_claim_count);
  o.f32(T2(25, 5), 2, x.bonus_wager_rate);
  o.boolean(T2(26, 0), 2, x.flags & FR_BONUS_ONLY);
}

// A length-delimited body written in place after a 1-byte length slot (bodies here are almost
// always < 128 bytes); a longer one is shifted right by the extra length bytes.
inline char* close_len(char* slot, char* end) {
  const size_t n = size_t(end - slot - 1);
  if (__builtin_expect(n < 128, 1)) {
    *slot = char(n);
    return end;
  }
  char lb[10];
  Out lo{lb};
  lo.varint(n);
  const size_t ln = size_t(lo.p - lb);
  std::memmove(slot + ln, slot + 1, n);
  std::memcpy(slot, lb, ln);
  return slot + ln + n;
}

inline char* write_tx_body(char* out, const ResultRec& r, const FeatRec* f, int64_t ms) {
  FastOut o{out};
  const uint32_t p = r.packed;
  o.uvar(T1(1, 0), 1, IGP_RES_SCORE(p));
  o.uvar(T1(2, 0), 1, IGP_RES_ACTION(p));
  // response order = rule order, ML_HIGH_RISK appended after the rules (engine.go:284-287)
  uint32_t reasons = IGP_RES_REASONS(p);
  if (reasons) {
    const ReasonTable& t = reasons_table();
    while (reasons) {
      const int b = __builtin_ctz(reasons);
      std::memcpy(o.p, t.enc[b], 32);
      o.p += t.len[b];
      reasons &= reasons - 1;
    }
  }
  o.uvar(T1(4, 0), 1, IGP_RES_RULE(p));
  o.f32(T1(5, 5), 1, r.ml);
  o.i64(T1(6, 0), 1, ms);
  if (f) {
    *o.p = char(T1(7, pb::LEN));
    const uint8_t img = reinterpret_cast<const uint8_t*>(f)[sizeof(FeatRec) - 1];
    if (img & FV_IMG_ENCODED) {  // the device encoded the body (features.hip write_fenc): <= 126 bytes
      const size_t len = img & 0x7f;
      o.p[1] = char(len);
      std::memcpy(o.p + 2, f, 128);  // whole image (the buffer has the slack): one fixed-size copy
      o.p += 2 + len;
    } else {
      char* slot = o.p + 1;
      o.p = slot + 1;
      write_feature_vector(o, *f);
      o.p = close_len(slot, o.p);
    }
  }
  return o.p;
}

}  // namespace

size_t write_tx_response(char* out, const ResultRec& r, const FeatRec* f, int64_t ms) {
  return size_t(write_tx_body(out, r, f, ms) - out);
}

size_t write_batch_response(char* dst, const ResultRec* r, const FeatRec* f, const int64_t* ms, int64_t ms_all,
                            size_t n) {
  char* p = dst;
  for (size_t i = 0; i < n; ++i) {
    *p = char(T1(1, pb::LEN));
    char* slot = p + 1;
    p = close_len(slot, write_tx_body(slot + 1, r[i], f ? f + i : nullptr, ms ? ms[i] : ms_all));
  }
  return size_t(p - dst);
}

std::string_view batch_response_scratch(const ResultRec* r, const FeatRec* f, const int64_t* ms, int64_t ms_all,
                                        size_t n) {
  // worst case per row into an uninitialised, grow-only per-thread buffer (its pages stay
  // resident across requests: a fresh multi-MB buffer per response pays a page fault per 4 KB)
  thread_local std::unique_ptr<char[]> scratch;
  thread_local size_t scratch_cap = 0;
  const size_t need = n * kMaxBatchRowBytes;
  if (scratch_cap < need) {
    scratch.reset(new char[need]);
    scratch_cap = need;
  }
  return std::string_view(scratch.get(), write_batch_response(scratch.get(), r, f, ms, ms_all, n));
}

void append_batch_response(std::string& out, const ResultRec* r, const FeatRec* f, const int64_t* ms, int64_t ms_all,
                           size_t n) {
  const std::string_view v = batch_response_scratch(r, f, ms, ms_all, n);
  out.append(v.data(), v.size());
}

std::string serialize_feature_vector(const FeatRec& x) {
  char body[400];
  FastOut o{body};
  write_feature_vector(o, x);
  return std::string(body, size_t(o.p - body));
}

std::string serialize_tx_response(const ResultView& v, size_t i) {
  char body[kMaxTxResponse];
  const size_t n = write_tx_response(body, v.res[i], v.feat ? v.feat + i : nullptr, v.response_ms ? v.response_ms[i] : 0);
  return std::string(body, n);
}

std::string serialize_batch_response(const ResultView& v) {
  std::string out;
  append_batch_response(out, v.res, v.feat, v.response_ms, 0, v.n);
  return out;
}

}  // namespace igp::wire

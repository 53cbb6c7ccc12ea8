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
  pb::Reader r(data, n);
  std::string_view acct, type, ip, dev, fp;
  int64_t amount = 0;
  uint32_t f, w;
  while (r.tag(f, w)) {
    switch (f) {
      case 1: acct = r.bytes(); break;
      case 3: amount = int64_t(r.varint()); break;
      case 4: type = r.bytes(); break;
      case 8: ip = r.bytes(); break;
      case 9: dev = r.bytes(); break;
      case 10: fp = r.bytes(); break;
      default: r.skip(w);  // player_id, currency, game/round, user_agent, session, metadata
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

// pre-encoded "field 3, LEN, length, bytes" of every reason code
struct ReasonTable {
  char enc[12][40];
  uint8_t len[12];
  ReasonTable() {
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

inline void write_feature_vector(Out& o, const FeatRec& x) {
  o.i32(1, x.tx_count_1m);
  o.i32(2, x.tx_count_5m);
  o.i32(3, x.tx_count_1h);
  o.i64(4, x.tx_sum_1h);
  o.f32(5, x.tx_avg_1h);
  o.i32(6, x.unique_devices_24h);
  o.i32(7, x.unique_ips_24h);
  o.i32(8, x.ip_country_changes_7d);
  o.i32(9, x.device_age_days);
  o.i32(10, x.account_age_days);
  o.i64(11, x.total_deposits);
  o.i64(12, x.total_withdrawals);
  o.i64(13, x.net_deposit);
  o.i32(14, x.deposit_count);
  o.i32(15, x.withdraw_count);
  o.i32(16, x.time_since_last_tx);
  o.i32(17, x.session_duration);
  o.f32(18, x.avg_bet_size);
  o.f32(19, x.win_rate);
  o.boolean(20, x.flags & FR_VPN);
  o.boolean(21, x.flags & FR_PROXY);
  o.boolean(22, x.flags & FR_TOR);
  o.boolean(23, x.flags & FR_DISPOSABLE);
  o.i32(24, x.bonus_claim_count);
  o.f32(25, x.bonus_wager_rate);
  o.boolean(26, x.flags & FR_BONUS_ONLY);
}

}  // namespace

size_t write_tx_response(char* out, const ResultRec& r, const FeatRec* f, int64_t ms) {
  Out o{out};
  const uint32_t p = r.packed;
  o.i32(1, int32_t(IGP_RES_SCORE(p)));
  o.i32(2, int32_t(IGP_RES_ACTION(p)));
  // response order = rule order, ML_HIGH_RISK appended after the rules (engine.go:284-287)
  const uint32_t reasons = IGP_RES_REASONS(p);
  if (reasons) {
    const ReasonTable& t = reasons_table();
    for (int b = 0; b < 12; ++b)
      if (reasons >> b & 1u) o.bytes(t.enc[b], t.len[b]);
  }
  o.i32(4, int32_t(IGP_RES_RULE(p)));
  o.f32(5, r.ml);
  o.i64(6, ms);
  if (f) {
    char body[400];
    Out fb{body};
    write_feature_vector(fb, *f);
    const size_t n = size_t(fb.p - body);
    o.tag(7, pb::LEN);
    o.varint(n);
    o.bytes(body, n);
  }
  return size_t(o.p - out);
}

size_t write_batch_response(char* dst, const ResultRec* r, const FeatRec* f, const int64_t* ms, int64_t ms_all,
                            size_t n) {
  char* p = dst;
  char body[kMaxTxResponse];
  for (size_t i = 0; i < n; ++i) {
    const size_t len = write_tx_response(body, r[i], f ? f + i : nullptr, ms ? ms[i] : ms_all);
    Out o{p};
    o.tag(1, pb::LEN);
    o.varint(len);
    o.bytes(body, len);
    p = o.p;
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
  Out o{body};
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

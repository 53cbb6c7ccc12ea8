#include "wire.h"

#include <cstring>

#include "account_index.h"
#include "pb.h"
#include "xxh64.h"

namespace igp::wire {

const char* const kReasonCodes[12] = {
    "HIGH_VELOCITY", "NEW_ACCOUNT_LARGE_TX", "MULTIPLE_DEVICES", "IP_COUNTRY_MISMATCH",
    "VPN_DETECTED", "RAPID_DEPOSIT_WITHDRAW", "BONUS_ABUSE", "KNOWN_FRAUDSTER",
    "ML_HIGH_RISK", "SUSPICIOUS_PATTERN", "MULTI_ACCOUNT", "DEVICE_FINGERPRINT_MISMATCH"};

void RequestBatch::clear() {
  account_id.clear(); account_hash.clear(); account_check.clear(); amount.clear(); tx_type.clear();
  device_hash.clear(); fp_hash.clear(); ip_hash.clear(); arena.clear();
}

void RequestBatch::reserve(size_t n) {
  account_id.reserve(n); account_hash.reserve(n); account_check.reserve(n); amount.reserve(n); tx_type.reserve(n);
  device_hash.reserve(n); fp_hash.reserve(n); ip_hash.reserve(n);
}

const std::string& RequestBatch::own(const char* data, size_t n) {
  arena.emplace_back(std::make_unique<std::string>(data, n));
  return *arena.back();
}

uint8_t tx_type_id(const char* s, size_t n) {
  auto eq = [&](const char* lit) { return std::strlen(lit) == n && std::memcmp(s, lit, n) == 0; };
  if (eq("deposit")) return TX_DEPOSIT;
  if (eq("withdraw")) return TX_WITHDRAW;
  if (eq("bet")) return TX_BET;
  if (eq("win")) return TX_WIN;
  if (eq("refund")) return TX_REFUND;
  if (eq("bonus")) return TX_BONUS;
  return TX_UNKNOWN;
}

void parse_tx(const char* data, size_t n, RequestBatch& out) {
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
  out.account_id.push_back(acct);  // a view into the batch's arena copy of the payload
  out.account_hash.push_back(id_hash(acct, SEED_ACCOUNT));
  out.account_check.push_back(id_check(acct));
  out.amount.push_back(amount);
  out.tx_type.push_back(tx_type_id(type.data(), type.size()));
  out.device_hash.push_back(id_hash(dev, SEED_DEVICE));
  out.fp_hash.push_back(id_hash(fp, SEED_FINGERPRINT));
  out.ip_hash.push_back(id_hash(ip, SEED_IP));
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

// Field emitters templated on the sink: pb::Writer appends bytes, pb::Sizer only counts them,
// so a nested message is sized first and then written straight into the one output buffer
// (no per-row temporary strings).
template <class W>
void emit_feature_vector(W& o, const FeatRec& x) {
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

template <class W>
void emit_tx_response(W& o, const ResultView& v, size_t i) {
  const uint32_t p = v.res[i].packed;
  o.i32(1, int32_t(IGP_RES_SCORE(p)));
  o.i32(2, int32_t(IGP_RES_ACTION(p)));
  const uint32_t reasons = IGP_RES_REASONS(p);
  // response order = rule order, ML_HIGH_RISK appended after the rules (engine.go:284-287)
  for (int b = 0; b < 12; ++b)
    if (reasons >> b & 1u) o.str_always(3, kReasonCodes[b]);
  o.i32(4, int32_t(IGP_RES_RULE(p)));
  o.f32(5, v.res[i].ml);
  if (v.response_ms) o.i64(6, v.response_ms[i]);
  if (v.feat) {
    pb::Sizer fs;
    emit_feature_vector(fs, v.feat[i]);
    o.msg_header(7, fs.n);
    emit_feature_vector(o, v.feat[i]);
  }
}

std::string serialize_feature_vector(const FeatRec& x) {
  pb::Writer o;
  emit_feature_vector(o, x);
  return o.buf;
}

std::string serialize_tx_response(const ResultView& v, size_t i) {
  pb::Writer o;
  emit_tx_response(o, v, i);
  return o.buf;
}

std::string serialize_batch_response(const ResultView& v) {
  pb::Writer o;
  o.buf.reserve(v.n * (v.feat ? 112 : 28));
  for (size_t i = 0; i < v.n; ++i) {
    pb::Sizer s;
    emit_tx_response(s, v, i);
    o.msg_header(1, s.n);
    emit_tx_response(o, v, i);
  }
  return o.buf;
}

}  // namespace igp::wire

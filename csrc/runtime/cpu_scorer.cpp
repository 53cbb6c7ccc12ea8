// Host twin of the GPU scoring pipeline; see cpu_scorer.h. Arithmetic follows the kernels
// (csrc/kernels/features.hip K1, update.h K6, ensemble.hip K5) operation for operation.
#include "cpu_scorer.h"

#include <cmath>
#include <cstring>
#include <stdexcept>

namespace igp {

namespace {

constexpr int HLL_M = 256;

uint16_t f32_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

float bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

float minmax(float x, float lo, float hi) {
  if (x < lo) return 0.f;
  if (x > hi) return 1.f;
  return (x - lo) / (hi - lo);
}

float log_t(float x, int identity) {
  if (x <= 0.f) return 0.f;
  if (identity) return x;
  return (float)std::log1p((double)x);
}

int hll_rank(uint64_t h) {
  const uint64_t w = h >> 8;
  return w ? (__builtin_clzll(w) - 8 + 1) : 57;
}

int hll_count(const uint8_t* rg) {
  double z = 0;
  int v = 0;
  for (int i = 0; i < HLL_M; ++i) {
    z += std::ldexp(1.0, -(int)rg[i]);
    v += rg[i] == 0;
  }
  const double m = 256.0, alpha = 0.7213 / (1.0 + 1.079 / 256.0);
  double e = alpha * m * m / z;
  if (e <= 2.5 * m && v > 0) e = m * std::log(m / (double)v);
  return (int)std::floor(e + 0.5);
}

double heuristic(const float* x) {  // mockPredict (onnx_model.go:258-308), float64 in Go's order
  double s = 0.0;
  if (x[0] > 0.5f) s += 0.2;
  if (x[2] > 0.5f) s += 0.15;
  if (x[5] > 0.3f) s += 0.15;
  if (x[6] > 0.25f) s += 0.1;
  if (x[19] > 0.f || x[20] > 0.f) s += 0.15;
  if (x[21] > 0.f) s += 0.25;
  if (x[9] < 0.02f && x[26] > 0.5f) s += 0.2;
  if (x[25] > 0.f) s += 0.15;
  if (x[15] < 0.01f && x[28] > 0.f) {
    if (x[11] > x[10] * 0.8f) s += 0.2;
  }
  return s > 1.0 ? 1.0 : s;
}

}  // namespace

CpuScorer::CpuScorer(int64_t capacity, int ring_size, int event_ring, int event_dim, int ext_width)
    : cap_(capacity), R_(ring_size), ER_(event_ring), ED_(event_dim), EW_(ext_width) {
  if (capacity <= 0 || ring_size <= 0 || event_dim != 16) throw std::invalid_argument("CpuScorer: bad sizes");
  ring_ts.assign((size_t)cap_ * R_, 0);
  ring_amt.assign((size_t)cap_ * R_, 0);
  hll.assign((size_t)cap_ * 2 * HLL_M, 0);
  rt.assign((size_t)cap_, AcctRT{});
  batch.assign((size_t)cap_, AcctBatch{});
  ext.assign((size_t)cap_ * (EW_ > 0 ? EW_ : 0), 0.f);
  ev.assign((size_t)cap_ * ER_ * ED_, 0);
}

void CpuScorer::set_cfg(const ScoreCfg& c) {
  std::lock_guard<std::mutex> g(mu_);
  cfg_ = c;
}

void CpuScorer::set_tables(const uint64_t* bk, const uint32_t* be, size_t bn, const uint64_t* ik,
                           const uint32_t* iflags, size_t in) {
  std::lock_guard<std::mutex> g(mu_);
  bl_keys_.assign(bk, bk + bn);
  bl_exp_.assign(be, be + bn);
  ip_keys_.assign(ik, ik + in);
  ip_flags_.assign(iflags, iflags + in);
}

void CpuScorer::set_model(std::shared_ptr<exec::Executor> ex, std::string in_name, std::string out_name, int ml_col) {
  std::lock_guard<std::mutex> g(mu_);
  ex_ = std::move(ex);
  in_name_ = std::move(in_name);
  out_name_ = std::move(out_name);
  ml_col_ = ml_col;
}

void CpuScorer::set_batch(const int32_t* slots, const AcctBatch* rows, size_t n) {
  std::lock_guard<std::mutex> g(mu_);
  for (size_t k = 0; k < n; ++k)
    if (slots[k] >= 0 && slots[k] < cap_) batch[slots[k]] = rows[k];
}

void CpuScorer::set_ext(const int32_t* slots, const float* e, size_t n, int width) {
  std::lock_guard<std::mutex> g(mu_);
  if (EW_ <= 0) return;
  const int w = width < EW_ ? width : EW_;
  for (size_t k = 0; k < n; ++k) {
    if (slots[k] < 0 || slots[k] >= cap_) continue;
    float* d = ext.data() + (size_t)slots[k] * EW_;
    std::memset(d, 0, sizeof(float) * EW_);
    std::memcpy(d, e + k * (size_t)width, sizeof(float) * w);
  }
}

void CpuScorer::reset(const int32_t* slots, size_t n) {
  std::lock_guard<std::mutex> g(mu_);
  for (size_t k = 0; k < n; ++k) {
    const int64_t s = slots[k];
    if (s < 0 || s >= cap_) continue;
    std::memset(ring_ts.data() + s * R_, 0, sizeof(uint32_t) * R_);
    std::memset(ring_amt.data() + s * R_, 0, sizeof(int64_t) * R_);
    std::memset(hll.data() + s * 2 * HLL_M, 0, 2 * HLL_M);
    rt[s] = AcctRT{};
    batch[s] = AcctBatch{};
    if (EW_ > 0) std::memset(ext.data() + s * EW_, 0, sizeof(float) * EW_);
    std::memset(ev.data() + s * ER_ * ED_, 0, sizeof(uint16_t) * ER_ * ED_);
  }
}

bool CpuScorer::blacklisted(uint64_t key, int64_t now) const {
  if (!key || bl_keys_.empty()) return false;
  uint32_t i = (uint32_t)key & (uint32_t)cfg_.bl_mask;
  for (int p = 0; p < cfg_.bl_max_probe; ++p) {
    const uint64_t k = bl_keys_[i];
    if (k == 0) return false;
    if (k == key) return bl_exp_[i] == 0u || now < (int64_t)bl_exp_[i];
    i = (i + 1) & (uint32_t)cfg_.bl_mask;
  }
  return false;
}

int CpuScorer::ip_flags(uint64_t key) const {
  if (!key || ip_keys_.empty()) return 0;
  uint32_t i = (uint32_t)key & (uint32_t)cfg_.ip_mask;
  for (int p = 0; p < cfg_.ip_max_probe; ++p) {
    const uint64_t k = ip_keys_[i];
    if (k == 0) return 0;
    if (k == key) return (int)ip_flags_[i];
    i = (i + 1) & (uint32_t)cfg_.ip_mask;
  }
  return 0;
}

// K1 (features.hip:20-275): raw features, flags, rule pass, normalised model input
void CpuScorer::assemble(const ReqRec& q, int64_t now, FeatRec& f, float* x) const {
  const ScoreCfg& c = cfg_;
  const int s = (q.slot >= 0 && q.slot < cap_) ? q.slot : -1;
  const int tx = q.tx_type & 0xff;
  std::memset(&f, 0, sizeof f);
  const bool bl = blacklisted(q.dev_hash, now) || blacklisted(q.fp_hash, now) || blacklisted(q.ip_hash, now);
  const int ipf = ip_flags(q.ip_hash);
  int c1 = 0, c5 = 0, c60 = 0;
  long long s60 = 0;
  AcctRT r{};
  AcctBatch b{};
  if (s >= 0) {
    r = rt[s];
    b = batch[s];
    const uint32_t* ts = ring_ts.data() + (size_t)s * R_;
    const int64_t* am = ring_amt.data() + (size_t)s * R_;
    for (int k = 0; k < R_; ++k) {
      const int64_t t = ts[k];
      if (t == 0) continue;
      c1 += t >= now - 60;
      c5 += t >= now - 300;
      if (t >= now - 3600) {
        ++c60;
        s60 += am[k];
      }
    }
    const uint8_t* rg = hll.data() + (size_t)s * 2 * HLL_M;
    f.unique_devices_24h = now < (int64_t)r.hll_dev_exp ? hll_count(rg) : 0;
    f.unique_ips_24h = now < (int64_t)r.hll_ip_exp ? hll_count(rg + HLL_M) : 0;
  }
  f.tx_count_1m = c1;
  f.tx_count_5m = c5;
  f.tx_count_1h = c60;
  f.tx_sum_1h = c.sum_compat ? ((s >= 0 && now < (int64_t)r.sum_exp) ? r.sum_compat : 0) : s60;
  f.tx_avg_1h = c60 > 0 ? (float)((double)f.tx_sum_1h / (double)c60) : 0.f;
  if (s >= 0) {
    if (r.last_tx > 0 && now < (int64_t)r.last_tx_exp) f.time_since_last_tx = (int32_t)(now - (int64_t)r.last_tx);
    if (r.session_start > 0 && now < (int64_t)r.session_exp)
      f.session_duration = (int32_t)(now - (int64_t)r.session_start);
  }
  int flags = 0;
  if (s >= 0 && b.present) {
    f.total_deposits = b.total_deposits;
    f.total_withdrawals = b.total_withdrawals;
    f.net_deposit = b.total_deposits - b.total_withdrawals;
    f.deposit_count = b.deposit_count;
    f.withdraw_count = b.withdraw_count;
    f.avg_bet_size = b.avg_bet_size;
    f.account_age_days = (int32_t)((now - b.account_created_at) / 86400);
    f.bonus_claim_count = b.bonus_claim_count;
    f.bonus_wager_rate = b.bonus_wager_complete;
    if (b.bet_count > 0) f.win_rate = (float)((double)b.win_count / (double)b.bet_count);
    if (b.bonus_claim_count > 3 && b.total_deposits < 5000) flags |= FR_BONUS_ONLY;
  } else {
    flags |= FR_PARTIAL;
  }
  if (ipf & 1) flags |= FR_VPN;
  if (ipf & 2) flags |= FR_PROXY;
  if (ipf & 4) flags |= FR_TOR;
  if (bl) flags |= FR_BLACKLISTED;
  f.flags = flags;
  f.tx_type = tx;
  f.slot = s;
  f.amount = q.amount;
  // rules (engine.go:420-483)
  int score = 0;
  uint32_t reasons = 0;
  if (f.tx_count_1m > c.max_tx_per_minute) { score += c.w_high_velocity; reasons |= 1u << 0; }
  if (f.account_age_days < c.new_account_days && q.amount > c.large_deposit_amount) {
    score += c.w_new_account_large_tx;
    reasons |= 1u << 1;
  }
  if (f.unique_devices_24h > c.max_devices_per_day) { score += c.w_multiple_devices; reasons |= 1u << 2; }
  if (f.unique_ips_24h > c.max_ips_per_day) { score += c.w_ip_country_mismatch; reasons |= 1u << 3; }
  if (flags & (FR_VPN | FR_PROXY | FR_TOR)) { score += c.w_vpn; reasons |= 1u << 4; }
  if (f.time_since_last_tx < 300 && tx == TX_WITHDRAW && f.deposit_count > 0 &&
      f.total_withdrawals > f.total_deposits * 80 / 100) {
    score += c.w_rapid_deposit_withdraw;
    reasons |= 1u << 5;
  }
  if (flags & FR_BONUS_ONLY) { score += c.w_bonus_abuse; reasons |= 1u << 6; }
  if (bl) { score += c.w_known_fraudster; reasons |= 1u << 7; }
  f.reserved0 = (int32_t)reasons;
  f.reserved1 = score > 100 ? 100 : score;
  // model input (onnx_model.go:133-205)
  const int id = c.log_identity;
  x[0] = minmax((float)f.tx_count_1m, 0.f, 20.f);
  x[1] = minmax((float)f.tx_count_5m, 0.f, 50.f);
  x[2] = minmax((float)f.tx_count_1h, 0.f, 200.f);
  x[3] = log_t((float)f.tx_sum_1h, id);
  x[4] = f.tx_avg_1h;
  x[5] = minmax((float)f.unique_devices_24h, 0.f, 10.f);
  x[6] = minmax((float)f.unique_ips_24h, 0.f, 20.f);
  x[7] = (float)f.ip_country_changes_7d;
  x[8] = (float)f.device_age_days;
  x[9] = minmax((float)f.account_age_days, 0.f, 365.f);
  x[10] = log_t((float)f.total_deposits, id);
  x[11] = log_t((float)f.total_withdrawals, id);
  x[12] = (float)f.net_deposit;
  x[13] = (float)f.deposit_count;
  x[14] = (float)f.withdraw_count;
  x[15] = minmax((float)f.time_since_last_tx, 0.f, 86400.f);
  x[16] = (float)f.session_duration;
  x[17] = f.avg_bet_size;
  x[18] = f.win_rate;
  x[19] = (flags & FR_VPN) ? 1.f : 0.f;
  x[20] = (flags & FR_PROXY) ? 1.f : 0.f;
  x[21] = (flags & FR_TOR) ? 1.f : 0.f;
  x[22] = (flags & FR_DISPOSABLE) ? 1.f : 0.f;
  x[23] = (float)f.bonus_claim_count;
  x[24] = f.bonus_wager_rate;
  x[25] = (flags & FR_BONUS_ONLY) ? 1.f : 0.f;
  x[26] = log_t((float)q.amount, id);
  x[27] = tx == TX_DEPOSIT ? 1.f : 0.f;
  x[28] = tx == TX_WITHDRAW ? 1.f : 0.f;
  x[29] = tx == TX_BET ? 1.f : 0.f;
  for (int j = 0; j < EW_; ++j) x[30 + j] = s >= 0 ? ext[(size_t)s * EW_ + j] : 0.f;
}

// K6 apply_event (update.h): ring, compat sum, HLLs, last tx, session, event ring
void CpuScorer::apply(const ReqRec& q, int64_t now) {
  const int s = q.slot;
  if (s < 0 || s >= cap_) return;
  const ScoreCfg& c = cfg_;
  AcctRT& r = rt[s];
  const int64_t amt = q.amount;
  ring_ts[(size_t)s * R_ + r.ring_head] = (uint32_t)now;
  ring_amt[(size_t)s * R_ + r.ring_head] = amt;
  r.ring_head = r.ring_head + 1 == R_ ? 0 : r.ring_head + 1;
  if (now >= (int64_t)r.sum_exp) r.sum_compat = 0;
  r.sum_compat += amt;
  r.sum_exp = (uint32_t)(now + c.sum_ttl);
  bool new_dev = false, new_ip = false;
  uint8_t* rg = hll.data() + (size_t)s * 2 * HLL_M;
  auto hll_add = [&](uint8_t* reg, uint32_t& exp, uint64_t h, bool& changed) {
    if (now >= (int64_t)exp) std::memset(reg, 0, HLL_M);
    const int idx = (int)(h & 255u), rank = hll_rank(h);
    if (rank > reg[idx]) {
      reg[idx] = (uint8_t)rank;
      changed = true;
    }
    exp = (uint32_t)(now + c.hll_ttl);
  };
  if (q.dev_hash) hll_add(rg, r.hll_dev_exp, q.dev_hash, new_dev);
  if (q.ip_hash) hll_add(rg + HLL_M, r.hll_ip_exp, q.ip_hash, new_ip);
  // the cached estimates (AcctRT hll_dev_n / hll_ip_n) follow every raised register, as on the
  // device; the read path below still counts from the registers, so GPU / CPU parity tests check
  // the device's cache against the definition
  if (new_dev) r.hll_dev_n = hll_count(rg);
  if (new_ip) r.hll_ip_n = hll_count(rg + HLL_M);
  r.last_tx = (uint32_t)now;
  r.last_tx_exp = (uint32_t)(now + c.last_tx_ttl);
  if (now >= (int64_t)r.session_exp || r.session_start == 0) r.session_start = (uint32_t)now;
  r.session_exp = (uint32_t)(now + c.session_ttl);
  // event row (golden.features.encode_event)
  const int tt = q.tx_type & 0xff;
  const int64_t prev = r.last_event_ts;
  const int64_t dt = (prev > 0 && now >= prev) ? now - prev : 0;
  const double hour = (double)(now % 86400) / 3600.0;
  float row[16] = {(float)(std::log1p((double)(amt > 0 ? amt : 0)) / 16.0), tt == 0 ? 1.f : 0.f,
                   tt == 1 ? 1.f : 0.f, tt == 2 ? 1.f : 0.f, tt == 3 ? 1.f : 0.f, tt == 4 ? 1.f : 0.f,
                   tt == 5 ? 1.f : 0.f, (float)(std::log1p((double)dt) / 12.0),
                   (float)std::sin(2.0 * M_PI * hour / 24.0), (float)std::cos(2.0 * M_PI * hour / 24.0),
                   new_dev ? 1.f : 0.f, new_ip ? 1.f : 0.f, amt >= 100000 ? 1.f : 0.f, 1.f, 0.f, 0.f};
  uint16_t* e = ev.data() + ((size_t)s * ER_ + r.ev_head) * ED_;
  for (int k = 0; k < 16; ++k) e[k] = f32_to_bf16(row[k]);
  r.ev_head = r.ev_head + 1 == ER_ ? 0 : r.ev_head + 1;
  r.ev_count = r.ev_count + 1 > ER_ ? ER_ : r.ev_count + 1;
  r.last_event_ts = (uint32_t)now;
}

void CpuScorer::ingest(const ReqRec* evs, size_t n) {
  std::lock_guard<std::mutex> g(mu_);
  for (size_t k = 0; k < n; ++k) apply(evs[k], evs[k].ts);
}

void CpuScorer::score(const ReqRec* req, size_t n, int64_t now, bool update, ResultRec* res, FeatRec* feat) {
  std::lock_guard<std::mutex> g(mu_);
  const ScoreCfg& c = cfg_;
  const int W = 30 + (EW_ > 0 ? EW_ : 0);
  std::vector<FeatRec> fs(n);
  std::vector<float> X(n * (size_t)W);
  for (size_t k = 0; k < n; ++k) assemble(req[k], now, fs[k], X.data() + k * W);
  // model
  std::vector<double> ml(n, 0.0);
  if (c.model_kind == 1) {
    for (size_t k = 0; k < n; ++k) ml[k] = heuristic(X.data() + k * W);
  } else if (c.model_kind == 2 && ex_ && n) {
    bool err = false;
    std::vector<float> out;
    int stride = 1;
    try {
      std::map<std::string, onnx::Tensor> in;
      onnx::Tensor t;
      t.name = in_name_;
      t.dims = {(int64_t)n, (int64_t)W};
      t.f = X;
      in[in_name_] = std::move(t);
      auto o = ex_->run(in);
      auto it = o.find(out_name_);
      if (it == o.end()) it = std::prev(o.end());
      out = it->second.f;
      stride = (int)(out.size() / n);
      if (stride <= ml_col_) err = true;
    } catch (const std::exception&) {
      err = true;  // model error -> neutral score (engine.go:279-282)
    }
    for (size_t k = 0; k < n; ++k) {
      float v = err ? NAN : out[k * stride + ml_col_];
      if (std::isnan(v)) {
        ml[k] = c.ml_error_score;
      } else {
        if (v < 0.f) v = 0.f;
        if (v > 1.f) v = 1.f;
        ml[k] = (double)v;
      }
    }
  }
  // K5 ensemble (ensemble.hip)
  for (size_t k = 0; k < n; ++k) {
    uint32_t reasons = (uint32_t)fs[k].reserved0;
    const int rule = fs[k].reserved1;
    if (c.model_kind != 0 && ml[k] > c.ml_high_risk) reasons |= 1u << 8;
    int fin = (int)(c.rule_weight * (double)rule + c.ml_weight * (ml[k] * 100.0));
    if (fin > 100) fin = 100;
    const int action = fin >= c.block_threshold ? 3 : fin >= c.review_threshold ? 2 : 1;
    res[k].packed = (uint32_t)(fin & 0xff) | ((uint32_t)(rule & 0xff) << 8) | ((uint32_t)action << 16) |
                    ((c.model_kind != 0 ? 1u : 0u) << 18) | (reasons << 20);
    res[k].ml = (float)ml[k];
    if (feat) feat[k] = fs[k];
  }
  if (update)
    for (size_t k = 0; k < n; ++k) apply(req[k], now);
}

FeatRec CpuScorer::features(int32_t slot, int64_t now) {
  std::lock_guard<std::mutex> g(mu_);
  ReqRec q{};
  q.slot = slot;
  q.tx_type = TX_UNKNOWN;
  FeatRec f;
  std::vector<float> x(30 + (EW_ > 0 ? EW_ : 0));
  assemble(q, now, f, x.data());
  return f;
}

void CpuScorer::event_history(int32_t slot, float* out) const {
  std::lock_guard<std::mutex> g(mu_);
  std::memset(out, 0, sizeof(float) * ER_ * ED_);
  if (slot < 0 || slot >= cap_) return;
  const AcctRT& r = rt[slot];
  const int cnt = r.ev_count < ER_ ? r.ev_count : ER_;
  for (int i = 0; i < cnt; ++i) {
    int idx = (r.ev_head - cnt + i) % ER_;
    if (idx < 0) idx += ER_;
    const uint16_t* e = ev.data() + ((size_t)slot * ER_ + idx) * ED_;
    float* o = out + (size_t)(ER_ - cnt + i) * ED_;
    for (int k = 0; k < ED_; ++k) o[k] = bf16_to_f32(e[k]);
  }
}

}  // namespace igp

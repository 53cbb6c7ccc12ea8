// K1 feature_assemble (+K7 blacklist probe, +K8 HLL count, + rule pass, + dedup insert) and
// K6 feature_update (ordered per-account event application) for gfx950.
//
// Reference semantics (golden spec: igaming_platform_amd/golden/features.py):
//   read path   services/risk/internal/features/redis_store.go:60-116, scoring/engine.go:326-417
//   write path  redis_store.go:119-168
//   rules       scoring/engine.go:420-483
//   blacklist   redis_store.go:267-293
#include "update.h"

namespace igp {

// ---------------------------------------------------------------------------------- K1
// model input l (onnx_model.go:133-184): 1 = minMaxScale(x, 0, k1_hi[l]), 2 = logTransform
__constant__ int k1_kind[32] = {1, 1, 1, 2, 0, 1, 1, 0, 0, 1, 2, 2, 0, 0, 0, 1,
                                0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 0, 0, 0, 0, 0};
__constant__ float k1_hi[32] = {20.f, 50.f, 200.f, 1.f, 1.f, 10.f, 20.f, 1.f, 1.f, 365.f, 1.f, 1.f, 1.f, 1.f, 1.f,
                                86400.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f,
                                1.f, 1.f};

__device__ void apply_segment_wave(const UpdateArgs& a, const DedupTab& t, int h, int c, int s, AcctRT r,
                                   int lane);

// PFADD on a register file held one uint32 (4 registers) per lane: the owner lane of the
// register updates and stores its word; an expired key (TTL) is rewritten as zeros first.
__device__ __forceinline__ bool hll_add_wave(uint32_t* words, uint32_t w, uint32_t& exp, uint64_t h, int64_t now,
                                             int ttl, int lane) {
  const bool reset = now >= (int64_t)exp;
  if (reset) w = 0u;
  const int idx = (int)(h & 255u);
  const int rank = hll_rank(h);
  const int sh = 8 * (idx & 3);
  const bool mine = lane == (idx >> 2) && rank > (int)((w >> sh) & 0xffu);
  if (mine) w = (w & ~(0xffu << sh)) | ((uint32_t)rank << sh);
  if (reset || mine) words[lane] = w;
  exp = (uint32_t)(now + ttl);
  return __ballot(mine) != 0ull;
}

// apply_event (update.h) spread over a wave that already holds the account's AcctRT (uniform)
// and HLL registers (wd / wi: 4 per lane); same arithmetic, same stored bytes. The event row
// is built by lanes 0..7 (one word each) with a single double log1p pass (lane 0: amount,
// lane 3: dt) and the batch's precomputed hour-of-day word `hour_word`.
__device__ __forceinline__ void apply_event_wave(const UpdateArgs& a, const ReqRec& ev, AcctRT r, uint32_t wd,
                                                 uint32_t wi, int lane, uint32_t hour_word) {
  const int s = ev.slot;
  const int64_t now = event_ts(a, ev);
  const ScoreCfg& cfg = *a.cfg;
  const int64_t amt = ev.amount;
  const int hd = r.ring_head;
  if (lane == 0) {
    a.ring_ts[(size_t)s * a.ring_size + hd] = (uint32_t)now;
    a.ring_amt[(size_t)s * a.ring_size + hd] = amt;
  }
  r.ring_head = hd + 1 == a.ring_size ? 0 : hd + 1;
  if (now >= (int64_t)r.sum_exp) r.sum_compat = 0;
  r.sum_compat += amt;
  r.sum_exp = (uint32_t)(now + cfg.sum_ttl);
  uint32_t* regs = reinterpret_cast<uint32_t*>(a.hll + (size_t)s * 512);
  bool new_dev = false, new_ip = false;
  if (ev.dev_hash) new_dev = hll_add_wave(regs, wd, r.hll_dev_exp, ev.dev_hash, now, cfg.hll_ttl, lane);
  if (ev.ip_hash) new_ip = hll_add_wave(regs + 64, wi, r.hll_ip_exp, ev.ip_hash, now, cfg.hll_ttl, lane);
  r.last_tx = (uint32_t)now;
  r.last_tx_exp = (uint32_t)(now + cfg.last_tx_ttl);
  if (now >= (int64_t)r.session_exp || r.session_start == 0) r.session_start = (uint32_t)now;
  r.session_exp = (uint32_t)(now + cfg.session_ttl);
  if (a.ev) {
    uint32_t* e = reinterpret_cast<uint32_t*>(a.ev + ((size_t)s * a.ev_ring + r.ev_head) * a.ev_dim);
    const int tt = ev.tx_type & 0xff;
    const int64_t prev = (int64_t)r.last_event_ts;
    const int64_t dt = (prev > 0 && now >= prev) ? now - prev : 0;
    const double l = log1p(lane == 0 ? (double)(amt > 0 ? amt : 0) : (double)dt);
    float lo = 0.f, hi = 0.f;
    switch (lane) {  // bf16 pairs of golden.features.encode_event (update.h event_word)
      case 0: lo = (float)(l / 16.0); hi = tt == 0; break;
      case 1: lo = tt == 1; hi = tt == 2; break;
      case 2: lo = tt == 3; hi = tt == 4; break;
      case 3: lo = tt == 5; hi = (float)(l / 12.0); break;
      case 5: lo = new_dev; hi = new_ip; break;
      case 6: lo = amt >= 100000; hi = 1.f; break;
      default: break;
    }
    const uint32_t w = lane == 4 ? hour_word : ((uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16));
    if (lane < 8) e[lane] = w;
    r.ev_head = r.ev_head + 1 == a.ev_ring ? 0 : r.ev_head + 1;
    r.ev_count = r.ev_count + 1 > a.ev_ring ? a.ev_ring : r.ev_count + 1;
  }
  r.last_event_ts = (uint32_t)now;
  if (lane == 0) a.rt[s] = r;
}

__device__ __forceinline__ void clear_next_dedup(const AssembleArgs& a, int row, int seq, int lane) {
  if (a.dbuf) {  // clear this wave's slice of batch seq+2's dedup region (after every load:
                 // no store precedes the account loads, so uniform ones can go scalar)
    const DedupTab nt = dedup_region(a.dbuf, a.dcap, a.dmax, dedup_ring_region(seq + 2));
    const int chunk = (a.dcap + a.n_rows - 1) / a.n_rows;
    const int e0 = row * chunk;
    dedup_clear_range(nt, e0, min(a.dcap, e0 + chunk), lane);
    if (row == 0 && lane < 2) nt.ctr[lane] = 0;
  }
}

// One wave64 per request. Every independent load is issued before the first use: the
// 256-entry ts ring as one uint4 per lane (1 KiB/wave, coalesced), HLL registers (4 per
// lane), the account rows (broadcast), the ext row, and the blacklist/ip-intel probes;
// the 1h amounts are then fetched only for in-window entries (predicated, issued together).
// Score-then-update: dedup_insert_kernel registered the batch first; a wave whose account has
// no other event in the batch applies the event itself once its reads are done (AcctRT and
// the HLL registers are already in registers), and every wave clears a slice of the other
// parity's dedup table for the next batch after its loads.
__device__ __forceinline__ void feature_assemble_body(const AssembleArgs& a) {
  const int lane = threadIdx.x & 63;
  const int row = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (row >= a.n_rows) return;
  const ScoreCfg& cfg = *a.cfg;
  // ---- dependency level 1: the request row and the batch header (independent loads). Under a
  // full grid every dependent global-load level costs several microseconds, so the kernel is
  // organised as two load levels: the row, then everything the row addresses.
  const uint4* rp = reinterpret_cast<const uint4*>(a.req + as_vgpr(row));
  const uint4 q0 = rp[0], q1 = rp[1], q2 = rp[2];
  ReqRec rq;
  rq.slot = (int32_t)q0.x;
  rq.tx_type = (int32_t)q0.y;
  rq.amount = (int64_t)(((uint64_t)q0.w << 32) | q0.z);
  rq.dev_hash = ((uint64_t)q1.y << 32) | q1.x;
  rq.fp_hash = ((uint64_t)q1.w << 32) | q1.z;
  rq.ip_hash = ((uint64_t)q2.y << 32) | q2.x;
  rq.ts = (int64_t)(((uint64_t)q2.w << 32) | q2.z);
  const int4 hv = *reinterpret_cast<const int4*>(a.hdr);  // BatchHdr {n, seq, now}
  // ScoreCfg bytes 128..159 in two 16-byte loads: {., bl_mask, bl_max_probe, ip_mask} and
  // {ip_max_probe, ext_width, owner_filter, my_rank} (records.h; static_asserts there)
  const int4 c8 = reinterpret_cast<const int4*>(a.cfg)[8];
  const int4 c9 = reinterpret_cast<const int4*>(a.cfg)[9];
  const int2 own = make_int2(c9.z, c9.w);
  const int ext_w = c9.y;
  const int n_live = hv.x;
  const int seq = hv.y;
  const int64_t now = (int64_t)(((uint64_t)(uint32_t)hv.w << 32) | (uint32_t)hv.z);
  float* xr = a.X + (size_t)row * a.x_stride;
  if (row >= n_live) {  // padded row of a graph bucket: deterministic zeros
    keep_issued((int)(q0.x ^ q0.z ^ q1.x ^ q1.z ^ q2.x ^ q2.z) ^ own.x);
    clear_next_dedup(a, row, seq, lane);
    for (int j = lane; j < 30 + ext_w; j += 64) xr[j] = 0.f;
    if (lane < 32) reinterpret_cast<int32_t*>(a.feat + row)[lane] = (lane == 27) ? -1 : 0;
    return;
  }
  if (own.x && ((rq.tx_type >> 8) & 0xff) != own.y) {  // another rank's request: inert row
    clear_next_dedup(a, row, seq, lane);
    for (int j = lane; j < 30 + ext_w; j += 64) xr[j] = 0.f;
    if (lane < 32) reinterpret_cast<int32_t*>(a.feat + row)[lane] = (lane == 27) ? -1 : (lane == 3 ? FR_NOT_OWNED : 0);
    return;
  }
  const int s = __builtin_amdgcn_readfirstlane(rq.slot);  // account rows go through SGPRs
  const int64_t amount = rq.amount;
  const int tx_type = rq.tx_type & 0xff;

  // ---- dependency level 2: every load addressed by the row, branch-free (clamped addresses,
  // results masked afterwards) so the compiler issues them back to back before the first use
  const bool has = s >= 0;
  const int sc = has ? s : 0;
  const int rs = a.ring_size;  // multiple of 64; 256 = one uint4 of ts + 4 amounts per lane
  const int rl = min(lane, rs / 4 - 1);
  uint4 tsv = reinterpret_cast<const uint4*>(a.ring_ts + (size_t)sc * rs)[rl];
  const longlong2* am2 = reinterpret_cast<const longlong2*>(a.ring_amt + (size_t)sc * rs);
  const longlong2 am01 = am2[2 * rl], am23 = am2[2 * rl + 1];
  const uint32_t* hreg = reinterpret_cast<const uint32_t*>(a.hll + (size_t)sc * 512);
  uint32_t wd = hreg[lane], wi = hreg[64 + lane];
  AcctRT rt = a.rt[sc];
  AcctBatch bt = a.batch[sc];
  const float* e = a.ext + (size_t)sc * ext_w;
  float extv[2];  // ext widths up to 128 preloaded; wider rows finish in a loop at the end
#pragma unroll
  for (int u = 0; u < 2; ++u) extv[u] = e[max(0, min(lane + 64 * u, ext_w - 1))];
  // score-then-update: first probe of the batch's dedup entry
  uint32_t dh = 0, hour_word = 0;
  int dkey = -1, dfirst = -1, dcount = 0;
  if (a.dbuf) {  // kernel-uniform
    const DedupTab t = dedup_region(a.dbuf, a.dcap, a.dmax, dedup_ring_region(seq));
    dh = mix32((uint32_t)sc) & (uint32_t)(t.cap - 1);
    dkey = t.keys[dh];
    dfirst = t.first[dh];
    dcount = t.count[dh];
    hour_word = (uint32_t)t.ctr[1];
  }
  // K7: blacklist (lanes 0..2: device, fingerprint, ip) and IP intelligence (lane 3): the first
  // probe slot's key and value are loaded with the rest, collisions walk on (rare)
  uint64_t key = 0;
  if (lane == 0) key = rq.dev_hash;
  else if (lane == 1) key = rq.fp_hash;
  else if (lane == 2 || lane == 3) key = rq.ip_hash;
  const bool tabs = a.bl_keys && a.ip_keys;  // kernel-uniform
  const bool bl_lane = tabs && lane < 3 && key != 0;
  const bool ip_lane = tabs && lane == 3 && key != 0;
  const uint64_t* pkeys = lane < 3 ? a.bl_keys : a.ip_keys;
  const uint32_t* pvals = lane < 3 ? a.bl_exp : a.ip_flags;
  const uint32_t pmask = (uint32_t)(lane < 3 ? c8.y : c8.w);
  uint32_t pi = (bl_lane || ip_lane) ? ((uint32_t)key & pmask) : 0u;
  uint64_t pk = 0;
  uint32_t pv = 0;
  if (tabs) {
    pk = pkeys[pi];
    pv = pvals[pi];
  }
  // ---- mask what a missing account / short ring must not see
  if (!has) {
    tsv = make_uint4(0, 0, 0, 0);
    wd = wi = 0u;
    rt = AcctRT{};
    bt = AcctBatch{};
    extv[0] = extv[1] = 0.f;
    dkey = -1;
  }
  if (lane * 4 >= rs) tsv = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int u = 0; u < 2; ++u)
    if (lane + 64 * u >= ext_w) extv[u] = 0.f;
  bool hit = false;
  int ipf = 0;
  if (bl_lane || ip_lane) {
    const int max_probe = lane < 3 ? c8.z : c9.x;
    for (int p = 1; p < max_probe && pk != 0 && pk != key; ++p) {
      pi = (pi + 1) & pmask;
      pk = pkeys[pi];
      pv = pvals[pi];
    }
    if (pk == key && max_probe > 0) {
      if (bl_lane) hit = (pv == 0u) || (now < (int64_t)pv);
      else ipf = (int)pv;
    }
  }
  const bool blacklisted = __ballot(hit) != 0ull;
  ipf = __shfl(ipf, 3, 64);

  // ---- window counts / sums from the tx ring
  int c1 = 0, c5 = 0, c60 = 0;
  long long s60 = 0;
  int hll_dev = 0, hll_ip = 0;
  if (s >= 0) {
    const int64_t* am = a.ring_amt + (size_t)s * rs;
    const uint32_t tv[4] = {tsv.x, tsv.y, tsv.z, tsv.w};
    bool in1h[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t t = (int64_t)tv[q];
      const bool v = t != 0;
      c1 += v && t >= now - 60;
      c5 += v && t >= now - 300;
      in1h[q] = v && t >= now - 3600;
      c60 += in1h[q];
    }
    const long long amv[4] = {in1h[0] ? am01.x : 0, in1h[1] ? am01.y : 0, in1h[2] ? am23.x : 0,
                              in1h[3] ? am23.y : 0};
    for (int q = 256 + lane; q < rs; q += 64) {  // rings longer than 256 entries (rare)
      const int64_t t = (int64_t)a.ring_ts[(size_t)s * rs + q];
      if (t != 0) {
        c1 += t >= now - 60;
        c5 += t >= now - 300;
        if (t >= now - 3600) { ++c60; s60 += am[q]; }
      }
    }
    s60 += amv[0] + amv[1] + amv[2] + amv[3];
    c1 = wave_sum(c1);
    c5 = wave_sum(c5);
    c60 = wave_sum(c60);
    s60 = wave_sum(s60);
    // ---- K8: HyperLogLog counts (p = 8; 4 registers per lane)
    double zd = 0, zi = 0;
    int vd = 0, vi = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int rd = (wd >> (8 * b)) & 0xff, ri = (wi >> (8 * b)) & 0xff;
      zd += exp2_neg(rd); vd += rd == 0;
      zi += exp2_neg(ri); vi += ri == 0;
    }
    zd = wave_sum(zd); zi = wave_sum(zi);
    vd = wave_sum(vd); vi = wave_sum(vi);
    // linear counting (E <= 2.5 m, V > 0): floor(m ln(m / V) + 0.5) from the host-computed
    // table (libm log, as the golden model); otherwise the harmonic estimate
    const double m = 256.0, alpha = 0.7213 / (1.0 + 1.079 / 256.0);
    const double ed = alpha * m * m / zd, ei = alpha * m * m / zi;
    const int ld = a.hll_lc[vd], li = a.hll_lc[vi];
    const int cd = (ed <= 2.5 * m && vd > 0) ? ld : (int)floor(ed + 0.5);
    const int ci = (ei <= 2.5 * m && vi > 0) ? li : (int)floor(ei + 0.5);
    hll_dev = now < (int64_t)rt.hll_dev_exp ? cd : 0;
    hll_ip = now < (int64_t)rt.hll_ip_exp ? ci : 0;
  }

  // ---- assemble raw features (wave-uniform values)
  FeatRec f{};
  f.tx_count_1m = c1;
  f.tx_count_5m = c5;
  f.tx_count_1h = c60;
  f.tx_sum_1h = cfg.sum_compat ? ((s >= 0 && now < (int64_t)rt.sum_exp) ? rt.sum_compat : 0) : s60;
  f.tx_avg_1h = c60 > 0 ? (float)((double)f.tx_sum_1h / (double)c60) : 0.f;
  f.unique_devices_24h = hll_dev;
  f.unique_ips_24h = hll_ip;
  if (s >= 0) {
    if (rt.last_tx > 0 && now < (int64_t)rt.last_tx_exp) f.time_since_last_tx = (int32_t)(now - (int64_t)rt.last_tx);
    if (rt.session_start > 0 && now < (int64_t)rt.session_exp)
      f.session_duration = (int32_t)(now - (int64_t)rt.session_start);
  }
  int flags = 0;
  if (s >= 0 && bt.present) {
    f.total_deposits = bt.total_deposits;
    f.total_withdrawals = bt.total_withdrawals;
    f.net_deposit = bt.total_deposits - bt.total_withdrawals;
    f.deposit_count = bt.deposit_count;
    f.withdraw_count = bt.withdraw_count;
    f.avg_bet_size = bt.avg_bet_size;
    f.account_age_days = (int32_t)((now - bt.account_created_at) / 86400);
    f.bonus_claim_count = bt.bonus_claim_count;
    f.bonus_wager_rate = bt.bonus_wager_complete;
    if (bt.bet_count > 0) f.win_rate = (float)((double)bt.win_count / (double)bt.bet_count);
    if (bt.bonus_claim_count > 3 && bt.total_deposits < 5000) flags |= FR_BONUS_ONLY;
  } else {
    flags |= FR_PARTIAL;
  }
  if (ipf & 1) flags |= FR_VPN;
  if (ipf & 2) flags |= FR_PROXY;
  if (ipf & 4) flags |= FR_TOR;
  if (blacklisted) flags |= FR_BLACKLISTED;
  f.flags = flags;
  f.tx_type = tx_type;
  f.slot = s;
  f.amount = amount;

  // ---- rule pass (engine.go:420-483), raw features
  int score = 0;
  uint32_t reasons = 0;
  if (f.tx_count_1m > cfg.max_tx_per_minute) { score += cfg.w_high_velocity; reasons |= 1u << 0; }
  if (f.account_age_days < cfg.new_account_days && amount > cfg.large_deposit_amount) {
    score += cfg.w_new_account_large_tx; reasons |= 1u << 1;
  }
  if (f.unique_devices_24h > cfg.max_devices_per_day) { score += cfg.w_multiple_devices; reasons |= 1u << 2; }
  if (f.unique_ips_24h > cfg.max_ips_per_day) { score += cfg.w_ip_country_mismatch; reasons |= 1u << 3; }
  if (flags & (FR_VPN | FR_PROXY | FR_TOR)) { score += cfg.w_vpn; reasons |= 1u << 4; }
  if (f.time_since_last_tx < 300 && tx_type == TX_WITHDRAW) {
    if (f.deposit_count > 0 && f.total_withdrawals > f.total_deposits * 80 / 100) {
      score += cfg.w_rapid_deposit_withdraw; reasons |= 1u << 5;
    }
  }
  if (flags & FR_BONUS_ONLY) { score += cfg.w_bonus_abuse; reasons |= 1u << 6; }
  if (blacklisted) { score += cfg.w_known_fraudster; reasons |= 1u << 7; }
  f.reserved0 = (int32_t)reasons;
  f.reserved1 = score > 100 ? 100 : score;

  // ---- writes: the 30 normalised inputs spread over lanes 0..29, the record by lane 0
  // each lane l < 30 produces model input l: its raw value is selected into the lane from the
  // (wave-uniform) features, then one pass of the lane's transform (min-max / log / identity)
  // runs for the whole wave instead of 30 divergent cases
  const int id = cfg.log_identity;
  float raw = 0.f;
#define IGP_PUT(l, v) raw = lane == (l) ? (float)(v) : raw
  IGP_PUT(0, f.tx_count_1m); IGP_PUT(1, f.tx_count_5m); IGP_PUT(2, f.tx_count_1h); IGP_PUT(3, f.tx_sum_1h);
  IGP_PUT(4, f.tx_avg_1h); IGP_PUT(5, f.unique_devices_24h); IGP_PUT(6, f.unique_ips_24h);
  IGP_PUT(7, f.ip_country_changes_7d); IGP_PUT(8, f.device_age_days); IGP_PUT(9, f.account_age_days);
  IGP_PUT(10, f.total_deposits); IGP_PUT(11, f.total_withdrawals); IGP_PUT(12, f.net_deposit);
  IGP_PUT(13, f.deposit_count); IGP_PUT(14, f.withdraw_count); IGP_PUT(15, f.time_since_last_tx);
  IGP_PUT(16, f.session_duration); IGP_PUT(17, f.avg_bet_size); IGP_PUT(18, f.win_rate);
  IGP_PUT(19, (flags & FR_VPN) ? 1.f : 0.f); IGP_PUT(20, (flags & FR_PROXY) ? 1.f : 0.f);
  IGP_PUT(21, (flags & FR_TOR) ? 1.f : 0.f); IGP_PUT(22, (flags & FR_DISPOSABLE) ? 1.f : 0.f);
  IGP_PUT(23, f.bonus_claim_count); IGP_PUT(24, f.bonus_wager_rate); IGP_PUT(25, (flags & FR_BONUS_ONLY) ? 1.f : 0.f);
  IGP_PUT(26, amount); IGP_PUT(27, tx_type == TX_DEPOSIT ? 1.f : 0.f); IGP_PUT(28, tx_type == TX_WITHDRAW ? 1.f : 0.f);
  IGP_PUT(29, tx_type == TX_BET ? 1.f : 0.f);
#undef IGP_PUT
  const int kind = k1_kind[lane & 31];
  float xv = raw;
  if (kind == 1) xv = minmax_scale(raw, 0.f, k1_hi[lane & 31]);
  else if (kind == 2) xv = log_transform(raw, id);
  if (lane < 30) xr[lane] = xv;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int j = lane + 64 * u;
    if (j < ext_w) xr[30 + j] = extv[u];
  }
  for (int j = lane + 128; j < ext_w; j += 64) xr[30 + j] = s >= 0 ? a.ext[(size_t)s * ext_w + j] : 0.f;
  if (lane == 0) a.feat[row] = f;
  clear_next_dedup(a, row, seq, lane);

  // ---- score-then-update (engine.go:486-488). An account whose only event in the batch is
  // this request has had all its reads done (by this wave), so the event is applied here by
  // the whole wave; a multi-event account's batch is applied by its last-finishing wave.
  if (a.dbuf && s >= 0) {
    const DedupTab t = dedup_region(a.dbuf, a.dcap, a.dmax, dedup_ring_region(seq));
    int h = (int)dh;
    if (dkey != s) {  // probe collision: walk the chain
      h = dedup_find(t, s);
      if (h >= 0) { dfirst = t.first[h]; dcount = t.count[h]; }
    }
    if (h >= 0) {
      if (dcount == 1) {
        apply_event_wave(a.upd, rq, rt, wd, wi, lane, hour_word);
      } else {
        // multi-event account: queue this row, then count it as read (its loads were all
        // consumed above); the wave that completes the count applies the account's whole
        // batch in row order (no other row of it can still be reading)
        int last = 0;
        if (lane == 0) {
          const int pos = atomicAdd(&t.fill[h], 1);
          if (pos < DEDUP_LIST) t.list[(size_t)h * DEDUP_LIST + pos] = row;
          __threadfence();
          last = atomicAdd(&t.done[h], 1) == dcount - 1;
        }
        if (__shfl(last, 0, 64)) {
          __threadfence();
          apply_segment_wave(a.upd, t, h, dcount, s, rt, lane);
        }
      }
    }
  }
}

__global__ void __launch_bounds__(256) feature_assemble_kernel(AssembleArgs a) { feature_assemble_body(a); }

// ---------------------------------------------------------------------------------- K6
__device__ __forceinline__ int upd_n(const UpdateArgs& a) {
  const int n = a.hdr ? a.hdr->n : a.n;
  return n < a.n_max ? n : a.n_max;
}

__device__ __forceinline__ DedupTab upd_region(const UpdateArgs& a) {
  const int r = a.region >= 0 ? a.region : dedup_ring_region(a.hdr->seq);
  return dedup_region(a.dbuf, a.dcap, a.dmax, r);
}

__global__ void dedup_reset_kernel(UpdateArgs a) {
  const DedupTab t = upd_region(a);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < t.cap) { t.keys[i] = -1; t.first[i] = 0x7fffffff; t.count[i] = 0; t.fill[i] = 0; t.done[i] = 0; }
  if (i < 2) t.ctr[i] = 0;
}

__global__ void dedup_insert_kernel(UpdateArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  // the batch clock's hour-of-day event-row word (sin/cos in double), once per batch for K1
  if (i == 0 && a.hdr) upd_region(a).ctr[1] = (int32_t)event_word(4, 0, 0, a.hdr->now, 0, false, false);
  if (i >= upd_n(a)) return;
  const ReqRec& r = a.req[i];
  if (r.slot >= 0 && row_owned(r, *a.cfg)) dedup_insert(upd_region(a), r.slot, i);
}

__global__ void update_single_kernel(UpdateArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= upd_n(a)) return;
  const ReqRec& r = a.req[i];
  if (r.slot >= 0 && row_owned(r, *a.cfg)) update_event(a, upd_region(a), i, r.slot);
}

// account s has more events in the batch than its dedup list holds: find them in row order
// (64 rows per ballot) and apply them one by one on lane 0 (degenerate traffic only)
__device__ void apply_scan_serial(const UpdateArgs& a, int s, int lane) {
  const int n = upd_n(a);
  AcctRT r = a.rt[s];
  for (int base = 0; base < n; base += 64) {
    const int i = base + lane;
    const bool m = i < n && a.req[i].slot == s && row_owned(a.req[i], *a.cfg);
    uint64_t b = __ballot(m);
    while (b) {
      const int l = __ffsll((long long)b) - 1;
      b &= b - 1;
      if (lane == 0) apply_event(a, base + l, r);
    }
  }
  if (lane == 0) a.rt[s] = r;
}

// PFADD of up to 64 same-account events at once: the per-register winner writes the max,
// each event learns whether it raised its register (the GRU's new-device/new-ip feature)
// exactly as the sequential order would have.
__device__ __forceinline__ uint32_t hll_segment(const UpdateArgs& a, uint8_t* rg, uint32_t exp, uint64_t hq,
                                                int64_t ts, int lane, bool& changed) {
  const bool has = hq != 0;
  const uint64_t any = __ballot(has);
  if (!any) return exp;
  const int fl = __ffsll((long long)any) - 1;
  const int ll = 63 - __clzll((long long)any);
  const int64_t tfirst = __shfl(ts, fl, 64), tlast = __shfl(ts, ll, 64);
  const bool reset = tfirst >= (int64_t)exp;
  const int idx = has ? (int)(hq & 255u) : -1;
  const int rank = has ? hll_rank(hq) : 0;
  const int before = (has && !reset) ? (int)rg[idx] : 0;
  if (reset) {
    reinterpret_cast<uint32_t*>(rg)[lane] = 0u;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  }
  int pm = before;
  bool win = has;
  for (int y = 0; y < 64; ++y) {
    const int iy = __shfl(idx, y, 64), ry = __shfl(rank, y, 64);
    if (has && iy == idx && y != lane) {
      if (y < lane) pm = max(pm, ry);
      if (ry > rank || (ry == rank && y < lane)) win = false;
    }
  }
  changed = has && rank > pm;
  if (win && rank > before) rg[idx] = (uint8_t)rank;
  return (uint32_t)(tlast + a.cfg->hll_ttl);
}

// the c (>= 2) events of account s (dedup hash slot h) in row order, by one wave holding the
// account's pre-batch AcctRT `r`: events sorted in registers and applied in parallel when
// the segment spans less than the shortest TTL (then no key can expire mid-segment);
// otherwise lane 0 applies them one by one; more than DEDUP_LIST events: ordered batch scan.
__device__ void apply_segment_wave(const UpdateArgs& a, const DedupTab& t, int h, int c, int s, AcctRT r,
                                   int lane) {
  if (c > DEDUP_LIST) {
    apply_scan_serial(a, s, lane);
    return;
  }
  // sort the (distinct) row indices: rank = #smaller, then push each to lane `rank`
  const int key = lane < c ? t.list[(size_t)h * DEDUP_LIST + lane] : (0x7fffffc0 | lane);
  int rank = 0;
  for (int y = 0; y < 64; ++y) rank += __shfl(key, y, 64) < key;
  const int j = __builtin_amdgcn_ds_permute(rank * 4, key);
  const bool act = lane < c;
  ReqRec ev{};
  if (act) ev = a.req[j];
  const int64_t ts = act ? event_ts(a, ev) : 0;
  const ScoreCfg& cfg = *a.cfg;
  const int min_ttl = min(min(cfg.session_ttl, cfg.sum_ttl), min(cfg.hll_ttl, cfg.last_tx_ttl));
  const int64_t ts0 = __shfl(ts, 0, 64);
  const int64_t tsl = __shfl(ts, c - 1, 64);
  const int64_t big = 0x3fffffffffffffffLL;
  const int64_t tmx = wave_max(act ? ts : -big);
  const int64_t tmn = -wave_max(act ? -ts : -big);
  // parallel apply is exact when the segment spans less than the shortest TTL (no key can
  // expire mid-segment); otherwise lane 0 applies the sorted events one by one
  if (tmx - tmn >= (int64_t)min_ttl) {
    for (int x = 0; x < c; ++x) {
      const int jx = __shfl(j, x, 64);
      if (lane == 0) apply_event(a, jx, r);
    }
    if (lane == 0) a.rt[s] = r;
    return;
  }
  const int64_t amt = act ? ev.amount : 0;
  // tx ring: consecutive positions from the head
  if (act) {
    const int pos = (r.ring_head + lane) % a.ring_size;
    a.ring_ts[(size_t)s * a.ring_size + pos] = (uint32_t)ts;
    a.ring_amt[(size_t)s * a.ring_size + pos] = amt;
  }
  // compat sum: only the first event can find the key expired (span < TTL)
  const long long tot = wave_sum((long long)amt);
  r.sum_compat = (ts0 >= (int64_t)r.sum_exp ? 0 : r.sum_compat) + tot;
  r.sum_exp = (uint32_t)(tsl + cfg.sum_ttl);
  // HyperLogLogs
  uint8_t* regs = a.hll + (size_t)s * 512;
  bool new_dev = false, new_ip = false;
  r.hll_dev_exp = hll_segment(a, regs, r.hll_dev_exp, act ? ev.dev_hash : 0, ts, lane, new_dev);
  r.hll_ip_exp = hll_segment(a, regs + 256, r.hll_ip_exp, act ? ev.ip_hash : 0, ts, lane, new_ip);
  // last tx / session
  if (ts0 >= (int64_t)r.session_exp || r.session_start == 0) r.session_start = (uint32_t)ts0;
  r.session_exp = (uint32_t)(tsl + cfg.session_ttl);
  r.last_tx = (uint32_t)tsl;
  r.last_tx_exp = (uint32_t)(tsl + cfg.last_tx_ttl);
  // event ring: event x's predecessor is event x-1 (event 0's is the stored last event)
  const int64_t up = __shfl(ts, lane > 0 ? lane - 1 : 0, 64);
  const int64_t prev = lane == 0 ? (int64_t)r.last_event_ts : up;
  if (a.ev && act) {
    const int pos = (r.ev_head + lane) % a.ev_ring;
    write_event_row(a.ev + ((size_t)s * a.ev_ring + pos) * a.ev_dim, amt, ev.tx_type & 0xff, ts, prev, new_dev,
                    new_ip);
  }
  if (a.ev) {
    r.ev_head = (r.ev_head + c) % a.ev_ring;
    r.ev_count = r.ev_count + c > a.ev_ring ? a.ev_ring : r.ev_count + c;
  }
  r.ring_head = (r.ring_head + c) % a.ring_size;
  r.last_event_ts = (uint32_t)tsl;
  if (lane == 0) a.rt[s] = r;
}

// standalone ingestion: one wave per multi-event account listed by update_single
__global__ void __launch_bounds__(256) update_multi_kernel(UpdateArgs a) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const DedupTab t = upd_region(a);
  if (w >= min(t.ctr[0], t.nmax)) return;
  const int h = t.mlist[w];
  if (h < 0 || h >= t.cap) return;
  const int c = t.count[h];
  const int s = t.keys[h];
  if (c < 2 || s < 0) return;
  apply_segment_wave(a, t, h, c, s, a.rt[s], lane);
}

// ---------------------------------------------------------------------------------- launch
void launch_feature_assemble(const AssembleArgs& a, hipStream_t st) {
  if (a.n_rows <= 0) return;
  hipLaunchKernelGGL(feature_assemble_kernel, dim3((a.n_rows + 3) / 4), dim3(256), 0, st, a);
}

void launch_dedup_insert(const UpdateArgs& a, hipStream_t st) {
  if (a.n_max <= 0) return;
  hipLaunchKernelGGL(dedup_insert_kernel, dim3((a.n_max + 255) / 256), dim3(256), 0, st, a);
}

void launch_update_segments(const UpdateArgs& a, hipStream_t st) {
  if (a.n_max <= 0) return;
  // at most n/2 accounts can have >= 2 events: one wave each
  hipLaunchKernelGGL(update_multi_kernel, dim3((a.n_max / 2 + 3) / 4 + 1), dim3(256), 0, st, a);
}

void launch_feature_update(const UpdateArgs& a, hipStream_t st) {
  if (a.n_max <= 0) return;
  hipLaunchKernelGGL(dedup_reset_kernel, dim3((a.dcap + 255) / 256), dim3(256), 0, st, a);
  const int g = (a.n_max + 255) / 256;
  hipLaunchKernelGGL(dedup_insert_kernel, dim3(g), dim3(256), 0, st, a);
  hipLaunchKernelGGL(update_single_kernel, dim3(g), dim3(256), 0, st, a);
  launch_update_segments(a, st);
}

}  // namespace igp

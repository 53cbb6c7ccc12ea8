// K1 feature_assemble (+K7 blacklist probe, +K8 HLL count, + rule pass, + dedup insert) and
// K6 feature_update (ordered per-account event application) for gfx950.
//
// Reference semantics (golden spec: igaming_platform_amd/golden/features.py):
//   read path   services/risk/internal/features/redis_store.go:60-116, scoring/engine.go:326-417
//   write path  redis_store.go:119-168
//   rules       scoring/engine.go:420-483
//   blacklist   redis_store.go:267-293
#include <stdexcept>

#include "update.h"

namespace igp {

// ---------------------------------------------------------------------------------- K1
// model input l (onnx_model.go:133-184): minMaxScale(x, 0, hi(l)) or logTransform. Selected in
// registers: per-lane __constant__ tables were vector loads issued after the account loads, a
// dependent memory round trip in the middle of the compute phase (tools/kbench.py trace).
constexpr uint32_t K1_MINMAX = (1u << 0) | (1u << 1) | (1u << 2) | (1u << 5) | (1u << 6) | (1u << 9) | (1u << 15);
constexpr uint32_t K1_LOG = (1u << 3) | (1u << 10) | (1u << 11) | (1u << 26);
__device__ __forceinline__ float k1_hi(int l) {
  return l == 0 ? 20.f : l == 1 ? 50.f : l == 2 ? 200.f : l == 5 ? 10.f : l == 6 ? 20.f : l == 9 ? 365.f
       : l == 15 ? 86400.f : 1.f;
}

__device__ void apply_segment_wave(const UpdateArgs& a, const DedupTab& t, int h, int c, int s, AcctRT r,
                                   int lane);

// K1 runs one request per 16-lane quarter of a wave (4 requests per wave, 16 per block): the
// per-request work is either 16-wide (tx ring, HLL registers, model inputs, ext row) or scalar
// (features, rules, update bookkeeping), and scalar work computed on a quarter instead of a
// whole wave takes a quarter of the VALU issue slots. Reductions / ballots stay inside the
// quarter (xor shuffles 1..8, ballot bits of the quarter).
constexpr int K1_QL = 16;  // lanes per request

__device__ __forceinline__ uint32_t qballot(bool p, int qb) { return (uint32_t)(__ballot(p) >> qb) & 0xffffu; }

// DPP lane moves inside a 16-lane row (= one request's quarter): no LDS round trip, unlike
// __shfl_xor (ds_bpermute, ~100 cycles per dependent step; K1 had ~100 of them).
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false);
}
template <int CTRL, class T>
__device__ __forceinline__ T dpp_t(T v) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "dpp_t: 4- or 8-byte values");
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, dpp_i<CTRL>(__builtin_bit_cast(int, v)));
  } else {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = dpp_i<CTRL>((int)b), hi = dpp_i<CTRL>((int)(b >> 32));
    return __builtin_bit_cast(T, (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
  }
}
constexpr int DPP_QUAD_X1 = 0xB1;     // quad_perm [1,0,3,2]: partner lane ^ 1
constexpr int DPP_QUAD_X2 = 0x4E;     // quad_perm [2,3,0,1]: partner lane ^ 2
constexpr int DPP_HALF_MIRROR = 0x141;  // lane i <-> 7 - i within 8: the other quad
constexpr int DPP_MIRROR = 0x140;       // lane i <-> 15 - i within 16: the other half
constexpr int DPP_SHR2 = 0x112;         // lane i <- lane i - 2 (row_shr:2)
constexpr int DPP_SHL2 = 0x102;         // lane i <- lane i + 2 (row_shl:2)

// sum over the 16 lanes of a quarter; every lane gets the sum. After the two quad steps all
// lanes of a quad hold the same value, so the mirror partners add the same pairs as the xor
// butterfly (1, 2, 4, 8) did: results are bit-identical, floating point included.
template <class T>
__device__ __forceinline__ T qsum(T v) {
  v += dpp_t<DPP_QUAD_X1>(v);
  v += dpp_t<DPP_QUAD_X2>(v);
  v += dpp_t<DPP_HALF_MIRROR>(v);
  v += dpp_t<DPP_MIRROR>(v);
  return v;
}

// HLL estimate of a register file held as 4 words (16 registers) per lane of a quarter (lane ql
// holds words ql + 16 i); every lane of the quarter gets it
__device__ __forceinline__ int hll_count_q(const uint32_t (&w)[4], const int32_t* lc) {
  double z = 0;
  int v = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int r = (w[i] >> (8 * b)) & 0xff;
      z += exp2_neg(r);
      v += r == 0;
    }
  return hll_estimate(qsum(z), qsum(v), lc);
}

// PFADD by the 16 lanes of a quarter that hold only the event's register word `w1` (the same
// word in every lane: one load per account instead of the 512-byte file). An expired key (TTL)
// is rewritten as zeros first; a raised register updates the account's cached estimate `cnt`:
// after a reset directly (one non-zero register), otherwise from the file, read only then (a
// register rises on an account's first events of a device / ip, not on repeats). Returns
// whether the register rose (golden new_device).
__device__ __forceinline__ bool hll_add_q(uint32_t* words, uint32_t w1, uint32_t& exp, int32_t& cnt, uint64_t h,
                                          int64_t now, int ttl, int ql, const int32_t* lc) {
  const bool reset = now >= (int64_t)exp;
  const int idx = (int)(h & 255u);
  const int rank = hll_rank(h);
  const int wix = idx >> 2, sh = 8 * (idx & 3);
  const uint32_t cur = reset ? 0u : w1;
  const bool rise = rank > (int)((cur >> sh) & 0xffu);  // quarter-uniform
  const uint32_t nw = (cur & ~(0xffu << sh)) | ((uint32_t)rank << sh);
  if (reset) {
#pragma unroll
    for (int i = 0; i < 4; ++i) words[ql + 16 * i] = ql + 16 * i == wix ? nw : 0u;
    cnt = hll_estimate(255.0 + exp2_neg(rank), 255, lc);
  } else if (rise) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = ql + 16 * i == wix ? nw : words[ql + 16 * i];
    if (ql == (wix & 15)) words[wix] = nw;
    cnt = hll_count_q(w, lc);
  }
  exp = (uint32_t)(now + ttl);
  return rise;
}

// apply_event (update.h) by the 16 lanes of a quarter that already hold the account's AcctRT
// and HLL registers; same arithmetic, same stored bytes. The event row is built by lanes 0..7
// (one word each) with a single double log1p pass (lane 0: amount, lane 3: dt) and the
// batch's precomputed hour-of-day word `hour_word` (dedup_insert_kernel).
__device__ __forceinline__ void apply_event_q(const UpdateArgs& a, const ScoreCfg& cfg, const ReqRec& ev, AcctRT r,
                                              uint32_t wd, uint32_t wi, int ql, uint32_t hour_word, const int32_t* lc) {
  const int s = ev.slot;
  const int64_t now = event_ts(a, ev);
  const int64_t amt = ev.amount;
  const int hd = r.ring_head;
  if (ql == 0) {
    a.ring_ts[(size_t)s * a.ring_size + hd] = (uint32_t)now;
    a.ring_amt[(size_t)s * a.ring_size + hd] = amt;
  }
  r.ring_head = hd + 1 == a.ring_size ? 0 : hd + 1;
  if (now >= (int64_t)r.sum_exp) r.sum_compat = 0;
  r.sum_compat += amt;
  r.sum_exp = (uint32_t)(now + cfg.sum_ttl);
  uint32_t* regs = reinterpret_cast<uint32_t*>(a.hll + (size_t)s * 512);
  bool new_dev = false, new_ip = false;
  if (ev.dev_hash) new_dev = hll_add_q(regs, wd, r.hll_dev_exp, r.hll_dev_n, ev.dev_hash, now, cfg.hll_ttl, ql, lc);
  if (ev.ip_hash) new_ip = hll_add_q(regs + 64, wi, r.hll_ip_exp, r.hll_ip_n, ev.ip_hash, now, cfg.hll_ttl, ql, lc);
  r.last_tx = (uint32_t)now;
  r.last_tx_exp = (uint32_t)(now + cfg.last_tx_ttl);
  if (now >= (int64_t)r.session_exp || r.session_start == 0) r.session_start = (uint32_t)now;
  r.session_exp = (uint32_t)(now + cfg.session_ttl);
  if (a.ev) {
    uint32_t* e = reinterpret_cast<uint32_t*>(a.ev + ((size_t)s * a.ev_ring + r.ev_head) * a.ev_dim);
    const int tt = ev.tx_type & 0xff;
    const int64_t prev = (int64_t)r.last_event_ts;
    const int64_t dt = (prev > 0 && now >= prev) ? now - prev : 0;
    const double l = log1p(ql == 0 ? (double)(amt > 0 ? amt : 0) : (double)dt);
    float lo = 0.f, hi = 0.f;
    switch (ql) {  // bf16 pairs of golden.features.encode_event (update.h event_word)
      case 0: lo = (float)(l / 16.0); hi = tt == 0; break;
      case 1: lo = tt == 1; hi = tt == 2; break;
      case 2: lo = tt == 3; hi = tt == 4; break;
      case 3: lo = tt == 5; hi = (float)(l / 12.0); break;
      case 5: lo = new_dev; hi = new_ip; break;
      case 6: lo = amt >= 100000; hi = 1.f; break;
      default: break;
    }
    const uint32_t w = ql == 4 ? hour_word : ((uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16));
    if (ql < 8) e[ql] = w;
    r.ev_head = r.ev_head + 1 == a.ev_ring ? 0 : r.ev_head + 1;
    r.ev_count = r.ev_count + 1 > a.ev_ring ? a.ev_ring : r.ev_count + 1;
  }
  r.last_event_ts = (uint32_t)now;
  if (ql == 0) store_rt(a.rt + s, r);
}

// inert row (graph padding / another rank's request): zero inputs, FeatRec with slot -1 (also
// as the row's D2H image)
__device__ __forceinline__ void inert_row(const AssembleArgs& a, float* xr, int row, int ql, int ext_w, int flag) {
  for (int j = ql; j < 30 + ext_w; j += K1_QL) xr[j] = 0.f;
  int32_t* fr = reinterpret_cast<int32_t*>(a.feat + row);
  fr[ql] = ql == 3 ? flag : 0;
  fr[ql + 16] = ql + 16 == 27 ? -1 : 0;
  if (a.fenc && !a.fenc_route) {  // (routed images: padding rows have no sender chunk)
    int32_t* fe = reinterpret_cast<int32_t*>(a.fenc + (size_t)row * sizeof(FeatRec));
    fe[ql] = ql == 3 ? flag : 0;
    fe[ql + 16] = ql + 16 == 27 ? -1 : 0;
  }
}

// ---- risk.v1 FeatureVector body, encoded on the device (the D2H image of a row whose request
// wants response bytes: ReqRec.tx_type bit FV_ENC_BIT). The serving core then copies these bytes
// into ScoreTransactionResponse.features instead of serialising ~26 fields per row on a host
// thread. Same bytes as the host writer (wire.cpp FastOut, byte-exact with protobuf): proto3
// zero suppression, int32 sign-extended to 64-bit varints, int64 varints, fixed32 floats,
// bools as 1, one-byte tags for fields 1-15, two-byte tags for 16-26. Image: bytes [0, len),
// byte 127 = 0x80 | len; a body longer than 126 bytes (large negative values) leaves the raw
// FeatRec instead (its byte 127 is the top byte of the rule score, 0), which the host serialises.
// FeatRec words: 0-2 tx counts, 3 flags, 4-5 tx_sum_1h, 6 tx_avg_1h, 7-11 i32 fields, 12-17 the
// three i64 totals, 18-21 i32, 22-23 f32, 24 i32, 25 f32 (records.h).
__device__ __forceinline__ void fv_put(uint64_t& lo, uint64_t& hi, int& n, uint32_t byte) {
  if (n < 8) lo |= (uint64_t)byte << (8 * n);
  else hi |= (uint64_t)byte << (8 * (n - 8));
  ++n;
}

// bytes of FeatureVector field `field` (1-based) into lo / hi; returns the byte count (0: omitted)
__device__ __forceinline__ int fv_field(const uint32_t* w, int field, uint64_t& lo, uint64_t& hi) {
  int word = 0, kind = 0;  // kind 0 int32, 1 int64, 2 float, 3 bool (flag bit in `bit`)
  uint32_t bit = 0;
  switch (field) {
    case 1: word = 0; break;
    case 2: word = 1; break;
    case 3: word = 2; break;
    case 4: word = 4; kind = 1; break;
    case 5: word = 6; kind = 2; break;
    case 6: word = 7; break;
    case 7: word = 8; break;
    case 8: word = 9; break;
    case 9: word = 10; break;
    case 10: word = 11; break;
    case 11: word = 12; kind = 1; break;
    case 12: word = 14; kind = 1; break;
    case 13: word = 16; kind = 1; break;
    case 14: word = 18; break;
    case 15: word = 19; break;
    case 16: word = 20; break;
    case 17: word = 21; break;
    case 18: word = 22; kind = 2; break;
    case 19: word = 23; kind = 2; break;
    case 20: kind = 3; bit = FR_VPN; break;
    case 21: kind = 3; bit = FR_PROXY; break;
    case 22: kind = 3; bit = FR_TOR; break;
    case 23: kind = 3; bit = FR_DISPOSABLE; break;
    case 24: word = 24; break;
    case 25: word = 25; kind = 2; break;
    default: kind = 3; bit = FR_BONUS_ONLY; break;  // 26
  }
  uint64_t v;
  if (kind == 0) v = (uint64_t)(int64_t)(int32_t)w[word];
  else if (kind == 1) v = (uint64_t)w[word] | ((uint64_t)w[word + 1] << 32);
  else if (kind == 2) v = w[word];
  else v = (w[3] & bit) ? 1u : 0u;
  lo = hi = 0;
  int n = 0;
  if (v == 0) return 0;
  const uint32_t t = ((uint32_t)field << 3) | (kind == 2 ? 5u : 0u);
  if (t < 128) {
    fv_put(lo, hi, n, t);
  } else {
    fv_put(lo, hi, n, (t & 0x7f) | 0x80);
    fv_put(lo, hi, n, t >> 7);
  }
  if (kind == 2) {
#pragma unroll
    for (int i = 0; i < 4; ++i) fv_put(lo, hi, n, (uint32_t)(v >> (8 * i)) & 0xffu);
  } else {
    do {
      uint32_t byte = (uint32_t)v & 0x7fu;
      v >>= 7;
      if (v) byte |= 0x80u;
      fv_put(lo, hi, n, byte);
    } while (v);
  }
  return n;
}

// exclusive prefix sum over the 16 lanes of a quarter (lane ql gets the sum of lanes < ql)
__device__ __forceinline__ int qscan_excl(int v, int ql) {
  int s = v;
#pragma unroll
  for (int d = 1; d < 16; d <<= 1) {
    const int u = __shfl_up(s, d, 16);
    if (ql >= d) s += u;
  }
  return s - v;
}

// the row's D2H image (a.fenc): the encoded body when the request asked for it and it fits,
// else the raw FeatRec staged in LDS (fw)
__device__ __forceinline__ void write_fenc(const AssembleArgs& a, int row, int ql, bool enc, const uint32_t* fw,
                                           uint8_t* se) {
  uint8_t* base = a.fenc + (size_t)row * sizeof(FeatRec);
  if (a.fenc_route) {  // the row's place in its sender's chunk of the results region
    const int d = a.fenc_route[row];
    const int p = d / a.fenc_c;
    base = a.fenc + (size_t)p * a.fenc_stride + (size_t)(d - p * a.fenc_c) * sizeof(FeatRec);
  }
  uint2* const out = reinterpret_cast<uint2*>(base);
  if (enc) {
    uint64_t lo0, hi0, lo1 = 0, hi1 = 0;
    const int n0 = fv_field(fw, ql + 1, lo0, hi0);
    const int n1 = ql < 10 ? fv_field(fw, ql + 17, lo1, hi1) : 0;
    const int off0 = qscan_excl(n0, ql);
    const int tot0 = __shfl(off0 + n0, 15, 16);
    const int off1 = tot0 + qscan_excl(n1, ql);
    const int total = __shfl(off1 + n1, 15, 16);
    if (total <= 126) {
      for (int i = 0; i < n0; ++i) se[off0 + i] = (uint8_t)((i < 8 ? lo0 >> (8 * i) : hi0 >> (8 * (i - 8))) & 0xff);
      for (int i = 0; i < n1; ++i) se[off1 + i] = (uint8_t)((i < 8 ? lo1 >> (8 * i) : hi1 >> (8 * (i - 8))) & 0xff);
      if (ql == 0) se[127] = (uint8_t)(0x80 | total);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // only the chunks holding the body and the length byte cross the host link (the reader
      // takes [0, len) and byte 127: wire.cpp write_tx_body); a ~75-byte body is 11 of 16 chunks
      if (8 * ql < total || ql == 15) out[ql] = reinterpret_cast<const uint2*>(se)[ql];
      return;
    }
  }
  out[ql] = reinterpret_cast<const uint2*>(fw)[ql];
}

// Loads are organised in two dependency levels (under a full grid each dependent global-load
// level costs microseconds): level 1 = the request row + batch header + config words; level 2
// = everything the row addresses (ts ring, amounts, HLL registers, account rows, ext row, dedup
// probe, blacklist / ip-intel first probe slot), issued branch-free before the first use.
// Score-then-update: dedup_insert_list_kernel registered the batch first; a request whose
// account has no other event in the batch applies its event right after its own reads; the
// accounts with several events are applied after K1 by update_multi_kernel, in row order. (An
// in-kernel hand-off - the last request of an account to finish its reads applies the
// account's events - put chains of device-scope atomics and dependent loads at the end of
// K1: a 20 us tail behind 14 us of work at B=8192.)
__device__ __forceinline__ void feature_assemble_body(const AssembleArgs& a) {
  // phase trace of every wave: [wave][16] = wall_clock64 marks 0..7, [8] HW_ID, [9] XCC_ID
  const int gw = (int)((blockIdx.x * 256 + threadIdx.x) >> 6);  // launched with 256 threads
  int64_t* const trow = (a.trace && (threadIdx.x & 63) == 0) ? a.trace + (size_t)gw * 16 : nullptr;
  if (trow) {
    trow[8] = (int64_t)__builtin_amdgcn_s_getreg(0xF804);  // HW_ID
    trow[9] = (int64_t)__builtin_amdgcn_s_getreg(0xF814);  // XCC_ID
  }
#define K1_MARK(k) \
  if (trow) trow[k] = (int64_t)wall_clock64()
  K1_MARK(0);
  const int lane = threadIdx.x & 63;
  const int ql = lane & 15, qb = lane & 48;
  const int row = blockIdx.x * 16 + (threadIdx.x >> 4);
  const bool in_grid = row < a.n_rows;
  // the config block by value, loaded once at the top: through a reference, every field read
  // after a store (X, FeatRec, rings) is a fresh scalar load the compiler must re-issue (it
  // cannot prove the stores do not alias the block)
  const ScoreCfg cfg = *a.cfg;
  // HLL linear-counting table -> LDS, loaded beside the level-1 loads (a global lookup after
  // the HLL sums was a dependent round trip)
  __shared__ int s_lc[257];
  // per-request staging of the X row (30 + up to 112 ext floats) and the FeatRec
  __shared__ __attribute__((aligned(16))) float s_xst[16][144];
  __shared__ __attribute__((aligned(16))) uint2 s_fst[16][16];
  __shared__ __attribute__((aligned(16))) uint8_t s_enc[16][128];  // encoded FeatureVector bodies
  const int lc0 = a.hll_lc[threadIdx.x];
  const int lc1 = threadIdx.x == 0 ? a.hll_lc[256] : 0;
  // ---- level 1
  const uint4* rp = reinterpret_cast<const uint4*>(a.req + as_vgpr(in_grid ? row : 0));
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
  const int ext_w = c9.y;
  const int n_live = hv.x;
  const int seq = hv.y;
  const int64_t now = (int64_t)(((uint64_t)(uint32_t)hv.w << 32) | (uint32_t)hv.z);
  float* xr = a.X + (size_t)row * a.x_stride;
  s_lc[threadIdx.x] = lc0;
  if (threadIdx.x == 0) s_lc[256] = lc1;
  __syncthreads();
  if (trow) keep_issued(hv.x + (int)rq.slot);
  K1_MARK(1);
  const bool padded = in_grid && row >= n_live;
  const bool foreign = in_grid && !padded && c9.z && ((rq.tx_type >> 8) & 0xff) != c9.w;
  const bool live = in_grid && !padded && !foreign;
  if (padded || foreign) {
    inert_row(a, xr, row, ql, ext_w, foreign ? FR_NOT_OWNED : 0);
  }
  int h = -1, s = -1, dcount = 0;
  K1_MARK(6);
  if (live) {
    s = rq.slot;
    const int64_t amount = rq.amount;
    const int tx_type = rq.tx_type & 0xff;
    // ---- level 2 (clamped addresses, masked afterwards). Every load below is unconditional
    // but for the kernel-uniform table / dedup switches: a data-dependent branch around a load
    // makes the count of outstanding loads path-dependent, and the compiler then waits for all
    // of them (vmcnt(0)) at the first use of any.
    const bool has = s >= 0;
    const int sc = has ? s : 0;
    // K7 first probe slots: blacklist (lanes 0..2: device, fingerprint, ip) and IP intelligence
    // (lane 3); their addresses need only the request row and the config block
    uint64_t key = 0;
    if (ql == 0) key = rq.dev_hash;
    else if (ql == 1) key = rq.fp_hash;
    else if (ql == 2 || ql == 3) key = rq.ip_hash;
    const bool tabs = a.bl_keys && a.ip_keys;  // kernel-uniform
    const bool bl_lane = tabs && ql < 3 && key != 0;
    const bool ip_lane = tabs && ql == 3 && key != 0;
    const uint64_t* pkeys = ql < 3 ? a.bl_keys : a.ip_keys;
    const uint32_t* pvals = ql < 3 ? a.bl_exp : a.ip_flags;
    const uint32_t pmask = (uint32_t)(ql < 3 ? c8.y : c8.w);
    uint32_t pi = (bl_lane || ip_lane) ? ((uint32_t)key & pmask) : 0u;
    // without tables the probe reads the request row instead (a valid address; masked below)
    const uint64_t* pk0 = tabs ? pkeys + pi : reinterpret_cast<const uint64_t*>(a.req);
    const uint32_t* pv0 = tabs ? pvals + pi : reinterpret_cast<const uint32_t*>(a.req);
    uint64_t pk = *pk0;
    uint32_t pv = *pv0;
    if (!tabs) pk = pv = 0;
    const int rs = a.ring_size;  // multiple of 64: lane ql holds entries 4 (ql + 16 i) .. +3
    const int n4 = rs / 4;
    const uint4* ts4 = reinterpret_cast<const uint4*>(a.ring_ts + (size_t)sc * rs);
    uint4 tsv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) tsv[i] = ts4[min(ql + 16 * i, n4 - 1)];
    // HLL: the cardinalities come cached in AcctRT; only the two register words the request's
    // own PFADDs touch are read (one address per quarter), for the single-event apply below
    const uint32_t* hreg = reinterpret_cast<const uint32_t*>(a.hll + (size_t)sc * 512);
    uint32_t wd = hreg[(uint32_t)(rq.dev_hash & 255u) >> 2];
    uint32_t wi = hreg[64 + ((uint32_t)(rq.ip_hash & 255u) >> 2)];
    AcctRT rt = load_rt(a.rt + sc);
    AcctBatch bt = a.batch[sc];
    const float* e = a.ext + (size_t)sc * ext_w;
    float extv[7];  // ext widths up to 112 preloaded; wider rows finish in a loop at the end
#pragma unroll
    for (int u = 0; u < 7; ++u) extv[u] = e[max(0, min(ql + 16 * u, ext_w - 1))];
    // dedup probe (without a dedup region: the batch header, masked below)
    uint32_t dh = 0;
    const int32_t *pkey, *pfirst, *pcount, *phour;
    if (a.dbuf) {  // kernel-uniform
      const DedupTab t = dedup_region(a.dbuf, a.dcap, a.dmax, dedup_ring_region(seq));
      dh = mix32((uint32_t)sc) & (uint32_t)(t.cap - 1);
      pkey = t.keys + dh;
      pfirst = t.first + dh;
      pcount = t.count + dh;
      phour = t.ctr + 1;
    } else {
      pkey = pfirst = pcount = phour = reinterpret_cast<const int32_t*>(a.hdr);
    }
    int dkey = *pkey, dfirst = *pfirst;
    dcount = *pcount;
    uint32_t hour_word = (uint32_t)*phour;
    if (!a.dbuf) {
      dkey = dfirst = -1;
      dcount = 0;
      hour_word = 0;
    }
    K1_MARK(7);
    // ---- mask what a missing account / short ring must not see
    if (!has) {
#pragma unroll
      for (int i = 0; i < 4; ++i) tsv[i] = make_uint4(0, 0, 0, 0);
      wd = wi = 0u;
      rt = AcctRT{};
      bt = AcctBatch{};
#pragma unroll
      for (int u = 0; u < 7; ++u) extv[u] = 0.f;
      dkey = -1;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (ql + 16 * i >= n4) tsv[i] = make_uint4(0, 0, 0, 0);
    bool hit = false;
    int ipf = 0;
    if (bl_lane || ip_lane) {
      const int max_probe = ql < 3 ? c8.z : c9.x;
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
    const bool blacklisted = qballot(hit, qb) != 0u;
    if (trow) keep_issued((int)rt.ring_head + (int)tsv[0].x + (int)wd + (int)bt.present + (int)extv[0]);
    K1_MARK(2);
    ipf = __shfl(ipf, qb + 3, 64);

    // ---- window counts / sums from the tx ring
    int c1 = 0, c5 = 0, c60 = 0;
    long long s60 = 0;
    int hll_dev = 0, hll_ip = 0;
    if (has) {
      // the amount ring (2 KB per account, half the bytes K1 gathers) is read only where the ts
      // ring shows an entry inside the hour, and not at all for the compat (INCRBY) sum: a
      // third dependent level in exchange for ~half the HBM traffic of the gather (same-box
      // A/B, cfg3 bench: 109.6 vs 106.1 M scores/s for the full-ring load)
      const int64_t* amp = a.ring_amt + (size_t)s * rs;
      const bool want_amt = !cfg.sum_compat;
      // amounts as 16-byte pairs (entries 4 q + {0, 1} and {2, 3}: one load per pair with an
      // in-hour entry, half the load instructions of one 8-byte load per entry when the whole
      // ring is inside the hour - the serving bench's case)
      typedef long long k1_ll2 __attribute__((ext_vector_type(2)));
      long long av[16];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t tv[4] = {tsv[i].x, tsv[i].y, tsv[i].z, tsv[i].w};
        bool in1h[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t t = (int64_t)tv[j];
          const bool v = t != 0 && ql + 16 * i < n4;  // rings < 256 entries: clamped lanes are copies
          c1 += v && t >= now - 60;
          c5 += v && t >= now - 300;
          in1h[j] = v && t >= now - 3600;
          c60 += in1h[j];
        }
        const k1_ll2* ap = reinterpret_cast<const k1_ll2*>(amp + 4 * (ql + 16 * i));
        k1_ll2 p0 = {0, 0}, p1 = {0, 0};
        if (want_amt && (in1h[0] || in1h[1])) p0 = ap[0];
        if (want_amt && (in1h[2] || in1h[3])) p1 = ap[1];
        av[4 * i + 0] = in1h[0] ? p0.x : 0;
        av[4 * i + 1] = in1h[1] ? p0.y : 0;
        av[4 * i + 2] = in1h[2] ? p1.x : 0;
        av[4 * i + 3] = in1h[3] ? p1.y : 0;
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) s60 += av[k];
      for (int q = 256 + ql; q < rs; q += K1_QL) {  // rings longer than 256 entries (rare)
        const int64_t t = (int64_t)a.ring_ts[(size_t)s * rs + q];
        if (t != 0) {
          c1 += t >= now - 60;
          c5 += t >= now - 300;
          if (t >= now - 3600) { ++c60; s60 += amp[q]; }
        }
      }
      c1 = qsum(c1);
      c5 = qsum(c5);
      c60 = qsum(c60);
      s60 = qsum(s60);
      // ---- K8: HyperLogLog counts (PFCOUNT): the estimates every register change keeps in AcctRT
      hll_dev = now < (int64_t)rt.hll_dev_exp ? rt.hll_dev_n : 0;
      hll_ip = now < (int64_t)rt.hll_ip_exp ? rt.hll_ip_n : 0;
    }

    // ---- assemble raw features (quarter-uniform values)
    FeatRec f{};
    f.tx_count_1m = c1;
    f.tx_count_5m = c5;
    f.tx_count_1h = c60;
    f.tx_sum_1h = cfg.sum_compat ? ((has && now < (int64_t)rt.sum_exp) ? rt.sum_compat : 0) : s60;
    f.tx_avg_1h = c60 > 0 ? (float)((double)f.tx_sum_1h / (double)c60) : 0.f;
    f.unique_devices_24h = hll_dev;
    f.unique_ips_24h = hll_ip;
    if (has) {
      if (rt.last_tx > 0 && now < (int64_t)rt.last_tx_exp) f.time_since_last_tx = (int32_t)(now - (int64_t)rt.last_tx);
      if (rt.session_start > 0 && now < (int64_t)rt.session_exp)
        f.session_duration = (int32_t)(now - (int64_t)rt.session_start);
    }
    int flags = 0;
    if (has && bt.present) {
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

    // ---- the 30 model inputs: lane ql produces inputs ql and ql + 16 (raw value selected
    // from the quarter-uniform features, then one pass of each transform for the quarter)
    const int id = cfg.log_identity;
    float r0 = 0.f, r1 = 0.f;
#define IGP_PUT(l, v) \
  if ((l) < 16) r0 = ql == (l) ? (float)(v) : r0; else r1 = ql == (l) - 16 ? (float)(v) : r1
    IGP_PUT(0, f.tx_count_1m); IGP_PUT(1, f.tx_count_5m); IGP_PUT(2, f.tx_count_1h); IGP_PUT(3, f.tx_sum_1h);
    IGP_PUT(4, f.tx_avg_1h); IGP_PUT(5, f.unique_devices_24h); IGP_PUT(6, f.unique_ips_24h);
    IGP_PUT(7, f.ip_country_changes_7d); IGP_PUT(8, f.device_age_days); IGP_PUT(9, f.account_age_days);
    IGP_PUT(10, f.total_deposits); IGP_PUT(11, f.total_withdrawals); IGP_PUT(12, f.net_deposit);
    IGP_PUT(13, f.deposit_count); IGP_PUT(14, f.withdraw_count); IGP_PUT(15, f.time_since_last_tx);
    IGP_PUT(16, f.session_duration); IGP_PUT(17, f.avg_bet_size); IGP_PUT(18, f.win_rate);
    IGP_PUT(19, (flags & FR_VPN) ? 1.f : 0.f); IGP_PUT(20, (flags & FR_PROXY) ? 1.f : 0.f);
    IGP_PUT(21, (flags & FR_TOR) ? 1.f : 0.f); IGP_PUT(22, (flags & FR_DISPOSABLE) ? 1.f : 0.f);
    IGP_PUT(23, f.bonus_claim_count); IGP_PUT(24, f.bonus_wager_rate);
    IGP_PUT(25, (flags & FR_BONUS_ONLY) ? 1.f : 0.f); IGP_PUT(26, amount);
    IGP_PUT(27, tx_type == TX_DEPOSIT ? 1.f : 0.f); IGP_PUT(28, tx_type == TX_WITHDRAW ? 1.f : 0.f);
    IGP_PUT(29, tx_type == TX_BET ? 1.f : 0.f);
#undef IGP_PUT
    float x0 = r0, x1 = r1;
    if ((K1_MINMAX >> ql) & 1u) x0 = minmax_scale(r0, 0.f, k1_hi(ql));
    if ((K1_MINMAX >> (ql + 16)) & 1u) x1 = minmax_scale(r1, 0.f, k1_hi(ql + 16));
    // one divergent log1p pass for the quarter instead of two: lanes 3, 10, 11 transform their
    // x0; input 26 (x1 of lane 10) is moved to lane 12, transformed there and moved back
    static_assert(K1_LOG == ((1u << 3) | (1u << 10) | (1u << 11) | (1u << 26)), "log lanes moved");
    const bool lg0 = (K1_LOG >> ql) & 1u;
    const float in26 = dpp_t<DPP_SHR2>(r1);  // lane 12 <- lane 10's x1 input
    const float lin = lg0 ? r0 : in26;
    const float lout = (lg0 || ql == 12) ? log_transform(lin, id) : 0.f;
    const float lout26 = dpp_t<DPP_SHL2>(lout);  // lane 10 <- lane 12
    if (lg0) x0 = lout;
    if (ql == 10) x1 = lout26;
    // X row and FeatRec go out through LDS as whole words: written directly, the ext part (offset
    // 30 floats) straddled cache lines in 9 partial 4-B store instructions per wave and the
    // FeatRec left as 8 single-lane 16-B stores; staged, a wave writes its 4 rows in 2 x 16-B and
    // 1 x 8-B store instructions over contiguous memory
    float* const sx = s_xst[threadIdx.x >> 4];
    sx[ql] = x0;
    if (ql + 16 < 30) sx[ql + 16] = x1;
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      const int j = ql + 16 * u;
      if (j < ext_w) sx[30 + j] = extv[u];
    }
    if (ql == 0) *reinterpret_cast<FeatRec*>(s_fst[threadIdx.x >> 4]) = f;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int wst = 30 + min(ext_w, 112);
    if (((wst | (int)a.x_stride) & 3) == 0) {
      for (int c = ql; c < (wst >> 2); c += K1_QL)
        reinterpret_cast<float4*>(xr)[c] = reinterpret_cast<const float4*>(sx)[c];
    } else {
      for (int c = ql; c < wst; c += K1_QL) xr[c] = sx[c];
    }
    for (int j = ql + 112; j < ext_w; j += K1_QL) xr[30 + j] = has ? a.ext[(size_t)s * ext_w + j] : 0.f;
    K1_MARK(3);
    reinterpret_cast<uint2*>(a.feat + row)[ql] = s_fst[threadIdx.x >> 4][ql];
    if (a.fenc)
      write_fenc(a, row, ql, (rq.tx_type & FV_ENC_BIT) != 0, reinterpret_cast<const uint32_t*>(s_fst[threadIdx.x >> 4]),
                 s_enc[threadIdx.x >> 4]);

    // ---- score-then-update (engine.go:486-488)
    if (a.dbuf && has) {
      const DedupTab t = dedup_region(a.dbuf, a.dcap, a.dmax, dedup_ring_region(seq));
      h = (int)dh;
      if (dkey != s) {  // probe collision: walk the chain
        h = dedup_find(t, s);
        if (h >= 0) { dfirst = t.first[h]; dcount = t.count[h]; }
      }
      if (h >= 0) {
        if (dcount == 1) {
          apply_event_q(a.upd, cfg, rq, rt, wd, wi, ql, hour_word, s_lc);
        }
      }
    }
  }
  K1_MARK(4);
  if (trow) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    K1_MARK(5);
  }
#undef K1_MARK
}

__device__ __forceinline__ void globalize(UpdateArgs& u) {
  as_global(u.cfg); as_global(u.hdr); as_global(u.req); as_global(u.ring_ts); as_global(u.ring_amt);
  as_global(u.hll); as_global(u.rt); as_global(u.ev); as_global(u.dbuf); as_global(u.hll_lc);
}
__device__ __forceinline__ void globalize(AssembleArgs& a) {
  as_global(a.hdr); as_global(a.cfg); as_global(a.req); as_global(a.ring_ts); as_global(a.ring_amt);
  as_global(a.hll); as_global(a.rt); as_global(a.batch); as_global(a.ext); as_global(a.bl_keys);
  as_global(a.bl_exp); as_global(a.ip_keys); as_global(a.ip_flags); as_global(a.hll_lc); as_global(a.X);
  as_global(a.feat); as_global(a.fenc); as_global(a.fenc_route); as_global(a.dbuf); as_global(a.trace);
  globalize(a.upd);
}

__global__ void __launch_bounds__(256) feature_assemble_kernel(AssembleArgs) {
  AssembleArgs a = kernarg_vgpr<AssembleArgs>();
  globalize(a);
  feature_assemble_body(a);
}

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
  if (i < 4) t.ctr[i] = 0;
}

__global__ void dedup_insert_kernel(UpdateArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  // the batch clock's hour-of-day event-row word (sin/cos in double), once per batch for K1
  if (i == 0 && a.hdr) upd_region(a).ctr[1] = (int32_t)event_word(4, 0, 0, a.hdr->now, 0, false, false);
  if (i >= upd_n(a)) return;
  const ReqRec& r = a.req[i];
  const DedupTab t = upd_region(a);
  const bool mine = r.slot >= 0 && row_owned(r, *a.cfg);
  if (i < t.nmax) t.rows[i] = mine ? r.slot : -1;
  if (mine) dedup_insert(t, r.slot, i);
}

// Scorer head: register the batch's events in its dedup region (cleared two batches ahead by
// update_multi_kernel) and build, for every account, its row list (position = the count its
// row's add returned) and the list of multi-event accounts (added by the account's second
// row). One thread per row, 64-thread workgroups spread over the chip: the kernel is a chain
// of memory-side atomics (CAS, add, add), not work.
// With a.src (the scorer's copy stage) the batch comes straight from the pinned host slab: each
// thread reads its row through the fabric and writes the device copy K1 and the update read, the
// first thread the header - no H2D copy (an SDMA job and a launch per batch) ahead of it.
__global__ void __launch_bounds__(64) dedup_insert_list_kernel(UpdateArgs a) {
  // the wave's rows grouped by account first (a 128-entry LDS table): one global probe and one
  // count add per account and wave, not per row - under Zipf traffic the top account's rows
  // (~1 in 5) otherwise queue their CAS / add on one hash slot
  __shared__ int s_key[128], s_cnt[128], s_min[128], s_base[128], s_h[128];
  const int lane = threadIdx.x;
  const int i = blockIdx.x * 64 + lane;
  int2 r = make_int2(-1, 0);  // {slot, tx_type}
  int4 hv;
  if (a.xrecv) {
    // rows-region exchange: compact this owner's chunk of every sender's block (host memory)
    // here instead of a separate compact kernel and a device round trip of the rows. Lane p < xn
    // reads sender p's header record; a wave scan of the counts places every row.
    int cnt = 0;
    int64_t ts = 0;
    if (lane < a.xn) {
      const ReqRec* h = a.xrecv + (size_t)lane * a.xpstride;
      const int c = h->slot;
      cnt = c < 0 ? 0 : (c > a.xc ? a.xc : c);
      ts = cnt > 0 ? h->ts : 0;
    }
    const int4 h0 = *a.xhdr;
    int incl = cnt;  // inclusive prefix over the lanes (senders)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    const int excl = incl - cnt;
    const int total = __shfl(incl, 63, 64);
    const int64_t t = wave_max(ts);
    hv = make_int4(min(total, a.n_max), h0.y, t > 0 ? (int)(uint32_t)(uint64_t)t : h0.z,
                   t > 0 ? (int)(uint32_t)((uint64_t)t >> 32) : h0.w);
    if (i == 0) {
      *reinterpret_cast<int4*>(const_cast<BatchHdr*>(a.hdr)) = hv;
      a.route[a.n_max] = total > a.n_max ? total - a.n_max : 0;
    }
    int p = 0;  // the last sender whose rows start at or before row i (the whole wave: converged)
    for (int q = 1; q < a.xn; ++q)
      if (__builtin_amdgcn_readlane(excl, q) <= i && __builtin_amdgcn_readlane(cnt, q) > 0) p = q;
    const int j = i - __shfl(excl, p, 64);
    if (i < hv.x) {
      const uint4* sp = reinterpret_cast<const uint4*>(a.xrecv + (size_t)p * a.xpstride + 1 + j);
      uint4* dp = reinterpret_cast<uint4*>(const_cast<ReqRec*>(a.req + i));
      uint4 q0 = sp[0];
      const uint4 q1 = sp[1], q2 = sp[2];
      q0.y &= 0xffu | (uint32_t)FV_ENC_BIT;  // owner bits of tx_type: this GPU owns every row it receives
      dp[0] = q0;
      dp[1] = q1;
      dp[2] = q2;
      a.route[i] = p * a.xc + j;
      r = make_int2((int)q0.x, (int)q0.y);
    }
  } else {
    // the batch header {n, seq, now}: from the host slab (every lane the same 16 bytes: one
    // request per wave) or the device copy
    hv = *reinterpret_cast<const int4*>(a.src ? reinterpret_cast<const void*>(a.src)
                                              : reinterpret_cast<const void*>(a.hdr));
  }
  const int n = min(hv.x, a.n_max);  // as upd_n: the header's live count
  const int64_t now = (int64_t)(((uint64_t)(uint32_t)hv.w << 32) | (uint32_t)hv.z);
  const DedupTab t = dedup_region(a.dbuf, a.dcap, a.dmax, dedup_ring_region(hv.y));
  const bool live = i < n;
  if (a.xrecv) {
    // (rows, route and header written above)
  } else if (a.src) {
    if (i == 0) *reinterpret_cast<int4*>(const_cast<BatchHdr*>(a.hdr)) = hv;
    if (live) {
      const uint4* sp = reinterpret_cast<const uint4*>(a.src + sizeof(BatchHdr)) + 3 * (size_t)i;
      uint4* dp = reinterpret_cast<uint4*>(const_cast<ReqRec*>(a.req + i));
      const uint4 q0 = sp[0], q1 = sp[1], q2 = sp[2];
      dp[0] = q0;
      dp[1] = q1;
      dp[2] = q2;
      r = make_int2((int)q0.x, (int)q0.y);
    }
  } else if (live) {
    r = *reinterpret_cast<const int2*>(a.req + i);
  }
  // the batch clock's hour-of-day event-row word (sin/cos in double), once per batch for K1
  if (i == 0) t.ctr[1] = (int32_t)event_word(4, 0, 0, now, 0, false, false);
  s_key[lane] = s_key[64 + lane] = -1;
  s_cnt[lane] = s_cnt[64 + lane] = 0;
  s_min[lane] = s_min[64 + lane] = 0x7fffffff;
  const ScoreCfg& cfg = *a.cfg;
  const bool mine = r.x >= 0 && !(cfg.owner_filter && ((r.y >> 8) & 0xff) != cfg.my_rank);
  if (live && i < t.nmax) t.rows[i] = mine ? r.x : -1;  // compact account column for hot-account scans
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  int e = 0, lp = 0;
  if (mine) {  // at most 64 keys in 128 entries: the probe always ends
    e = (int)(mix32((uint32_t)r.x) & 127u);
    for (int q = 0; q < 128; ++q) {
      const int prev = atomicCAS(&s_key[e], -1, r.x);
      if (prev == -1 || prev == r.x) break;
      e = (e + 1) & 127;
    }
    lp = atomicAdd(&s_cnt[e], 1);
    atomicMin(&s_min[e], i);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  if (mine && lp == 0) {  // the account's first row in this wave probes the region for everyone
    uint32_t h = mix32((uint32_t)r.x) & (uint32_t)(t.cap - 1);
    for (int p = 0; p < t.cap; ++p) {
      const int prev = atomicCAS(&t.keys[h], -1, r.x);
      if (prev == -1 || prev == r.x) break;
      h = (h + 1) & (uint32_t)(t.cap - 1);
    }
    atomicMin(&t.first[h], s_min[e]);
    s_base[e] = atomicAdd(&t.count[h], s_cnt[e]);
    s_h[e] = (int)h;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  if (!mine) return;
  const int h = s_h[e];
  const int pos = s_base[e] + lp;  // list order is arbitrary: the apply sorts the rows
  if (pos < DEDUP_LIST) t.list[(size_t)h * DEDUP_LIST + pos] = i;
  if (pos == 1) {  // the account's second row registers it as a multi-event account
    const int m = atomicAdd(&t.ctr[0], 1);
    if (2 * m + 1 < t.nmax) *reinterpret_cast<int2*>(t.mlist + 2 * m) = make_int2(h, r.x);
  }
  if (pos == DEDUP_LIST) {  // ... and its (DEDUP_LIST + 1)-th as a hot account (update_segments_kernel)
    const int m = atomicAdd(&t.ctr[2], 1);
    if (m < t.hot_cap) *reinterpret_cast<int2*>(t.hot + 2 * m) = make_int2(h, r.x);
  }
}

__global__ void update_single_kernel(UpdateArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= upd_n(a)) return;
  const ReqRec& r = a.req[i];
  if (r.slot >= 0 && row_owned(r, *a.cfg)) update_event(a, upd_region(a), i, r.slot);
}

// lane `l` (wave-uniform) of a 64-bit value, via two v_readlane
__device__ __forceinline__ int64_t rdlane64(int64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// PFADD of up to 64 same-account events at once: the per-register winner writes the max,
// each event learns whether it raised its register (the GRU's new-device/new-ip feature)
// exactly as the sequential order would have.
// pre: the lane's register byte rg[hq & 255], loaded by the caller beside the other HLL's
template <bool LDSR>
__device__ __forceinline__ uint32_t hll_segment(const UpdateArgs& a, uint8_t* rg, uint32_t exp, uint64_t hq,
                                                int64_t ts, int lane, bool& changed, int pre) {
  const bool has = hq != 0;
  const uint64_t any = __ballot(has);
  if (!any) return exp;
  const int fl = __ffsll((long long)any) - 1;
  const int ll = 63 - __clzll((long long)any);
  const int64_t tfirst = rdlane64(ts, fl), tlast = rdlane64(ts, ll);
  const bool reset = tfirst >= (int64_t)exp;
  const int idx = has ? (int)(hq & 255u) : -1;
  const int rank = has ? hll_rank(hq) : 0;
  const int before = (has && !reset) ? pre : 0;
  if (reset) {
    reinterpret_cast<uint32_t*>(rg)[lane] = 0u;
    if constexpr (LDSR) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // one wave's LDS: in order
    else __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  }
  int pm = before;
  bool win = has;
  // one pass per distinct register index among the events (a few per account: its devices /
  // ips), not per event. Lanes of a group share idx; when they also share the rank (the same
  // hash repeated, the common case) the group's first lane is the only one that can raise the
  // register and the later ones see its rank; a group of different ranks (distinct hashes on
  // one register) walks its lanes. Wave-uniform lanes come through v_readlane.
  uint64_t rem = any;
  for (int ng = 0; rem && ng < 8; ++ng) {
    const int lead = __ffsll((long long)rem) - 1;
    const int v = __builtin_amdgcn_readlane(idx, lead), rl = __builtin_amdgcn_readlane(rank, lead);
    const bool in = has && idx == v;
    const uint64_t g = __ballot(in);
    rem &= ~g;
    if (__ballot(in && rank == rl) == g) {
      if (in && lane != lead) {
        pm = max(pm, rl);
        win = false;
      }
    } else {
      for (uint64_t q = g; q; q &= q - 1) {
        const int y = __ffsll((long long)q) - 1;
        const int ry = __builtin_amdgcn_readlane(rank, y);
        if (in && y != lane) {
          if (y < lane) pm = max(pm, ry);
          if (ry > rank || (ry == rank && y < lane)) win = false;
        }
      }
    }
  }
  // more than 8 distinct registers in the chunk: the rest lane by lane (groups leave whole, so
  // a remaining lane's group mates are all in `rem`)
  const bool left = has && ((rem >> lane) & 1ull);
  for (uint64_t q = rem; q; q &= q - 1) {
    const int y = __ffsll((long long)q) - 1;
    const int iy = __builtin_amdgcn_readlane(idx, y), ry = __builtin_amdgcn_readlane(rank, y);
    if (left && iy == idx && y != lane) {
      if (y < lane) pm = max(pm, ry);
      if (ry > rank || (ry == rank && y < lane)) win = false;
    }
  }
  changed = has && rank > pm;
  if (win && rank > before) rg[idx] = (uint8_t)rank;
  return (uint32_t)(tlast + a.cfg->hll_ttl);
}

// the estimate of 256 register bytes (the store's or a wave's LDS copy) by a whole wave: every
// quarter reads the file as K1's layout (lane ql: words ql + 16 i) and all lanes get the value
__device__ __forceinline__ int hll_count_wave(const uint8_t* rg, int lane, const int32_t* lc) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(rg);
  const int ql = lane & 15;
  const uint32_t q[4] = {w[ql], w[ql + 16], w[ql + 32], w[ql + 48]};
  return hll_count_q(q, lc);
}

// Apply c (1..64) events of account s, held in row order by lanes 0..c-1 (`j` = the lane's
// request row), to the account's AcctRT `r` (the same value in every lane, updated in place):
// in parallel when the events span less than the shortest TTL (then no key can expire
// mid-chunk: on the scorer path every event of a batch happens at the batch clock, span 0);
// otherwise lane 0 applies them one by one. The caller stores r. `regs`: the account's HLL
// registers in the store, or (LDSR) the wave's LDS copy that a hot account's chunks share.
// A hot account's chunk k0 of ctot events (the scan below): a tx-ring entry or GRU event row
// that a later event of the same batch overwrites (event k < ctot - ring size) is not written.
template <bool LDSR>
__device__ void apply_chunk(const UpdateArgs& a, int s, AcctRT& r, int j, int c, int lane, uint8_t* regs,
                            int k0 = 0, int ctot = 0) {
  const bool act = lane < c;
  ReqRec ev{};
  if (act) ev = a.req[j];
  // scorer path: every event happens at the batch clock, whose hour-of-day word the batch's
  // dedup insert already computed (region ctr[1])
  const int64_t hour_word = (a.hdr && a.ev) ? (int64_t)(uint32_t)upd_region(a).ctr[1] : -1;
  const int64_t ts = act ? event_ts(a, ev) : 0;
  const ScoreCfg& cfg = *a.cfg;
  const int min_ttl = min(min(cfg.session_ttl, cfg.sum_ttl), min(cfg.hll_ttl, cfg.last_tx_ttl));
  const int64_t ts0 = rdlane64(ts, 0);
  const int64_t tsl = rdlane64(ts, c - 1);
  const int64_t big = 0x3fffffffffffffffLL;
  // every event at one clock (the scorer path): span 0 without the two 64-bit wave reductions
  const bool one_clock = __ballot(act && ts != ts0) == 0ull;
  const int64_t tmx = one_clock ? ts0 : wave_max(act ? ts : -big);
  const int64_t tmn = one_clock ? ts0 : -wave_max(act ? -ts : -big);
  if (tmx - tmn >= (int64_t)min_ttl) {
    for (int x = 0; x < c; ++x) {
      const int jx = __builtin_amdgcn_readlane(j, x);
      if (lane == 0) apply_event(a, jx, r, regs);
    }
    // every lane continues with lane 0's state
    r.ring_head = __shfl(r.ring_head, 0, 64);
    r.ev_head = __shfl(r.ev_head, 0, 64);
    r.ev_count = __shfl(r.ev_count, 0, 64);
    r.sum_compat = __shfl(r.sum_compat, 0, 64);
    r.sum_exp = (uint32_t)__shfl((int)r.sum_exp, 0, 64);
    r.hll_dev_exp = (uint32_t)__shfl((int)r.hll_dev_exp, 0, 64);
    r.hll_ip_exp = (uint32_t)__shfl((int)r.hll_ip_exp, 0, 64);
    r.last_tx = (uint32_t)__shfl((int)r.last_tx, 0, 64);
    r.last_tx_exp = (uint32_t)__shfl((int)r.last_tx_exp, 0, 64);
    r.session_start = (uint32_t)__shfl((int)r.session_start, 0, 64);
    r.session_exp = (uint32_t)__shfl((int)r.session_exp, 0, 64);
    r.last_event_ts = (uint32_t)__shfl((int)r.last_event_ts, 0, 64);
    r.hll_dev_n = __shfl(r.hll_dev_n, 0, 64);
    r.hll_ip_n = __shfl(r.hll_ip_n, 0, 64);
    if constexpr (LDSR) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // lane 0's register writes
    return;
  }
  const int64_t amt = act ? ev.amount : 0;
  // tx ring: consecutive positions from the head
  if (act && k0 + lane >= ctot - a.ring_size) {
    const int pos = (r.ring_head + lane) % a.ring_size;
    a.ring_ts[(size_t)s * a.ring_size + pos] = (uint32_t)ts;
    a.ring_amt[(size_t)s * a.ring_size + pos] = amt;
  }
  // compat sum: only the first event can find the key expired (span < TTL)
  const long long tot = wave_sum((long long)amt);
  r.sum_compat = (ts0 >= (int64_t)r.sum_exp ? 0 : r.sum_compat) + tot;
  r.sum_exp = (uint32_t)(tsl + cfg.sum_ttl);
  // HyperLogLogs
  bool new_dev = false, new_ip = false;
  const uint64_t dq = act ? ev.dev_hash : 0, iq = act ? ev.ip_hash : 0;
  const int pd = dq ? (int)regs[dq & 255u] : 0;  // both registers in one memory round trip
  const int pi = iq ? (int)regs[256 + (iq & 255u)] : 0;
  r.hll_dev_exp = hll_segment<LDSR>(a, regs, r.hll_dev_exp, dq, ts, lane, new_dev, pd);
  r.hll_ip_exp = hll_segment<LDSR>(a, regs + 256, r.hll_ip_exp, iq, ts, lane, new_ip, pi);
  // the next chunk re-reads registers this one wrote (other lanes' stores)
  if constexpr (LDSR) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  else __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  // a raised register (or a reset, which raises one) refreshes the cached estimate
  if (__ballot(new_dev)) r.hll_dev_n = hll_count_wave(regs, lane, a.hll_lc);
  if (__ballot(new_ip)) r.hll_ip_n = hll_count_wave(regs + 256, lane, a.hll_lc);
  // last tx / session
  if (ts0 >= (int64_t)r.session_exp || r.session_start == 0) r.session_start = (uint32_t)ts0;
  r.session_exp = (uint32_t)(tsl + cfg.session_ttl);
  r.last_tx = (uint32_t)tsl;
  r.last_tx_exp = (uint32_t)(tsl + cfg.last_tx_ttl);
  // event ring: event x's predecessor is event x-1 (event 0's is the stored last event)
  const int64_t up = __shfl(ts, lane > 0 ? lane - 1 : 0, 64);
  const int64_t prev = lane == 0 ? (int64_t)r.last_event_ts : up;
  if (a.ev && act && k0 + lane >= ctot - a.ev_ring) {
    const int pos = (r.ev_head + lane) % a.ev_ring;
    write_event_row(a.ev + ((size_t)s * a.ev_ring + pos) * a.ev_dim, amt, ev.tx_type & 0xff, ts, prev, new_dev,
                    new_ip, hour_word);
  }
  if (a.ev) {
    r.ev_head = (r.ev_head + c) % a.ev_ring;
    r.ev_count = r.ev_count + c > a.ev_ring ? a.ev_ring : r.ev_count + c;
  }
  r.ring_head = (r.ring_head + c) % a.ring_size;
  r.last_event_ts = (uint32_t)tsl;
}

// account s has more events in the batch than its dedup list holds (a hot account: Zipf
// traffic gives the top account hundreds of rows in an 8192-row batch): scan the batch 64 rows
// per ballot, compact the account's rows (row order) into a 64-event chunk in registers and
// apply full chunks in parallel (apply_chunk); the chunk carries over between windows. The scan
// reads the insert's compact row -> account column (4 B per row instead of a 48-B request
// record), SCAN_W windows per memory round trip, and the account's HLL registers stay in the
// wave's LDS slice `lr` (128 words) for all its chunks: a chunk's register reads and writes are
// LDS operations, and the store's copy is written back once at the end.
constexpr int SCAN_W = 16;
__device__ void apply_scan_chunks(const UpdateArgs& a, const DedupTab& t, int s, AcctRT r, int lane, uint32_t* lr,
                                  int ctot) {
  const int n = min(upd_n(a), t.nmax);
  uint32_t* const g = reinterpret_cast<uint32_t*>(a.hll + (size_t)s * 512);
  lr[lane] = g[lane];
  lr[64 + lane] = g[64 + lane];
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  uint8_t* const regs = reinterpret_cast<uint8_t*>(lr);
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;  // lanes below this one
  int pj = 0, p = 0;  // pending chunk: lane k < p holds its k-th row
  int k0 = 0;         // the account's events applied so far
  for (int base0 = 0; base0 < n; base0 += 64 * SCAN_W) {
    // the insert's compact row -> account column (4 B per row; -1: not applied here)
    int kv[SCAN_W];
#pragma unroll
    for (int u = 0; u < SCAN_W; ++u) {
      const int i = base0 + 64 * u + lane;
      kv[u] = i < n ? t.rows[i] : -1;  // written by the batch's insert launch
    }
#pragma unroll
    for (int u = 0; u < SCAN_W; ++u) {
      const int i = base0 + 64 * u + lane;
      const bool m = kv[u] == s;
      const uint64_t b = __ballot(m);
      if (!b) continue;
      const int cw = __popcll(b);
      // the window's rows compacted to lanes 0..cw-1 (a push permute; other lanes fill behind)
      const int dst = m ? __popcll(b & lt) : cw + __popcll(~b & lt);
      const int wj = __builtin_amdgcn_ds_permute(dst * 4, i);
      // append to the pending chunk: lanes p..p+cw-1 take window rows 0..cw-1
      const int take = __shfl(wj, lane >= p ? lane - p : 0, 64);
      if (lane >= p && lane < p + cw) pj = take;
      if (p + cw < 64) {
        p += cw;
        continue;
      }
      apply_chunk<true>(a, s, r, pj, 64, lane, regs, k0, ctot);
      k0 += 64;
      const int over = p + cw - 64;  // window rows that did not fit: the next chunk's head
      const int rest = __shfl(wj, min(lane + 64 - p, 63), 64);
      if (lane < over) pj = rest;
      p = over;
    }
  }
  if (p > 0) apply_chunk<true>(a, s, r, pj, p, lane, regs, k0, ctot);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  g[lane] = lr[lane];
  g[64 + lane] = lr[64 + lane];
  if (lane == 0) store_rt(a.rt + s, r);
}

// the c (>= 2) events of account s (dedup hash slot h) in row order, by one wave holding the
// account's pre-batch AcctRT `r`; more than DEDUP_LIST events: the chunked batch scan.
__device__ void apply_segment_wave(const UpdateArgs& a, const DedupTab& t, int h, int c, int s, AcctRT r,
                                   int lane, uint32_t* lr) {
  if (c > DEDUP_LIST) {
    apply_scan_chunks(a, t, s, r, lane, lr, c);
    return;
  }
  // sort the (distinct) row indices: rank = #smaller, then push each to lane `rank`
  // sc1 load: the entries come from other waves of the same launch (feature_assemble hand-off)
  const int raw = __hip_atomic_load(&t.list[(size_t)h * DEDUP_LIST + lane], __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);  // all 64 lanes: no wait on c first
  const int key = lane < c ? raw : (0x7fffffc0 | lane);
  int rank = 0;
  for (int y = 0; y < c; ++y) rank += __builtin_amdgcn_readlane(key, y) < key;  // lanes >= c: sentinels
  const int j = __builtin_amdgcn_ds_permute(rank * 4, key);
  apply_chunk<false>(a, s, r, j, c, lane, a.hll + (size_t)s * 512);
  if (lane == 0) store_rt(a.rt + s, r);
}

// standalone ingestion: one wave per multi-event account listed by update_single
constexpr int UPD_MULTI_BLOCKS = 64;  // 256 waves loop over the list (any count, no big grid)
// dependent memory round trips per account: {list count, first pair} -> {count, AcctRT, row
// list} -> request rows -> both HLL registers -> stores (the pair carries the account slot, so
// count, AcctRT and the row list are loaded together)
// The multi-event accounts: wave w0 of `nwaves` loops over the region's list; thread `gt` of
// `nthreads` also clears the dedup region batch seq + DEDUP_AHEAD will insert into (scorer ring).
template <int WPB>
__device__ __forceinline__ void update_multi_body(const UpdateArgs& a, int w0, int nwaves, int gt, int nthreads,
                                                  uint32_t (*s_regs)[128]) {
  const int lane = threadIdx.x & 63;
  const DedupTab t = upd_region(a);
  const int npair = t.nmax >> 1;
  int2 hs = w0 < npair ? *reinterpret_cast<const int2*>(t.mlist + 2 * w0) : make_int2(-1, -1);  // speculative
  // a batch with no live rows (graph warm-up, an empty padded launch) applies nothing: the
  // region's list may still hold the previous user of the region (a scorer that took over
  // the store carries the batch sequence over)
  const int nm = upd_n(a) > 0 ? min(t.ctr[0], npair) : 0;
  for (int w = w0; w < nm; w += nwaves) {
    if (w != w0) hs = *reinterpret_cast<const int2*>(t.mlist + 2 * w);
    const int h = hs.x, s = hs.y;
    if (h < 0 || h >= t.cap || s < 0) continue;
    const int c = t.count[h];
    const AcctRT r = load_rt(a.rt + s);
    if (c < 2) continue;
    if (c > DEDUP_LIST && a.region < 0) continue;  // scorer path: the hot workgroups of update_segments_kernel apply it
    apply_segment_wave(a, t, h, c, s, r, lane, s_regs[(threadIdx.x >> 6) & (WPB - 1)]);
  }
  // scorer ring: clear the region of batch seq + DEDUP_AHEAD (= seq-1's, consumed by now) for
  // its insert; the copy of that batch waits for this batch's state stage
  if (a.region < 0) {
    const DedupTab nt = dedup_region(a.dbuf, a.dcap, a.dmax, dedup_ring_region(a.hdr->seq + DEDUP_AHEAD));
    const int4 m1 = make_int4(-1, -1, -1, -1), big = make_int4(0x7fffffff, 0x7fffffff, 0x7fffffff, 0x7fffffff);
    const int4 z = make_int4(0, 0, 0, 0);
    for (int e4 = gt; e4 < (nt.cap >> 2); e4 += nthreads) {
      reinterpret_cast<int4*>(nt.keys)[e4] = m1;
      reinterpret_cast<int4*>(nt.first)[e4] = big;
      reinterpret_cast<int4*>(nt.count)[e4] = z;
    }
    if (gt == 0) {
      nt.ctr[0] = 0;
      nt.ctr[2] = 0;
    }
  }
}

__global__ void __launch_bounds__(256) update_multi_kernel(UpdateArgs a) {
  __shared__ uint32_t s_regs[4][128];  // per wave: a multi-event account's HLL registers
  const int w0 = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  update_multi_body<4>(a, w0, UPD_MULTI_BLOCKS * 4, blockIdx.x * 256 + threadIdx.x, UPD_MULTI_BLOCKS * 256, s_regs);
}

// Hot accounts on the scorer path (more than DEDUP_LIST events in one batch: Zipf traffic gives
// the top account ~1 in 5 rows), one 512-thread workgroup per account instead of one wave that
// scans the batch and applies 64-event chunks one after another. Every event of
// a scoring batch happens at the batch clock, so the account's events split in two:
//   bulk  ranks 0 .. ctot-T-1 (row order): their effects commute except the tx-ring positions,
//         which are head + rank: ring entries (only the last ring_size events are kept), the
//         1 h sum, HLL registers as a per-register max (LDS atomicMax), and the scalar state
//         (last tx, session, heads) once for all of them. Their GRU event rows are overwritten by
//         the tail's (T >= ev_ring), so no per-event flags are needed.
//   tail  the last T events (T = ev_ring rounded up to 64): exact sequential semantics through
//         apply_chunk (new-device / new-ip flags against the registers after the bulk, GRU rows).
// The ranks come from one ordered pass over the batch's compact row -> account column: per 512-row
// block a ballot per wave and a 16-entry scan of the wave counts. Equal to the CPU engine's
// sequential apply byte for byte (tests/test_engine_gpu.py hot-account tests).
constexpr int HOT_THREADS = 512;
constexpr int HOT_BLOCKS = 64;
constexpr int HOT_TAIL_MAX = 192;

struct HotLds {
  uint32_t regs[128];  // the account's HLL registers: dev words 0..63, ip 64..127
  uint32_t pre[512];   // per register: max rank over the bulk events
  int tail[HOT_TAIL_MAX];
  int wcnt[HOT_THREADS / 64];
  long long wamt[HOT_THREADS / 64];
  int any[2];
};

// hot accounts w = hb, hb + nhb, ... of the region's hot list, one HOT_THREADS workgroup each
__device__ __forceinline__ void update_hot_body(const UpdateArgs& a, int hb, int nhb, HotLds& L) {
  uint32_t* const s_regs = L.regs;
  uint32_t* const s_pre = L.pre;
  int* const s_tail = L.tail;
  int* const s_wcnt = L.wcnt;
  long long* const s_wamt = L.wamt;
  int* const s_any = L.any;
  const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
  constexpr int NW = HOT_THREADS / 64;
  if (upd_n(a) <= 0) return;
  const DedupTab t = upd_region(a);
  const int n = min(upd_n(a), t.nmax);
  const int nh = min(t.ctr[2], t.hot_cap);
  const ScoreCfg& cfg = *a.cfg;
  const int64_t now = a.hdr->now;
  const int R = a.ring_size;
  const int T = a.ev ? min(((max(a.ev_ring, 1) + 63) / 64) * 64, HOT_TAIL_MAX) : 64;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int w = hb; w < nh; w += nhb) {
    const int2 hs = *reinterpret_cast<const int2*>(t.hot + 2 * w);
    const int h = hs.x, s = hs.y;
    if (h < 0 || h >= t.cap || s < 0) continue;
    const int ctot = t.count[h];
    if (ctot <= DEDUP_LIST) continue;
    const int Tn = min(T, ctot);
    const int Nb = ctot - Tn;  // bulk events
    AcctRT r = load_rt(a.rt + s);
    uint32_t* const g = reinterpret_cast<uint32_t*>(a.hll + (size_t)s * 512);
    if (tid < 128) s_regs[tid] = g[tid];
    if (tid < 512) s_pre[tid] = 0u;
    if (tid < 2) s_any[tid] = 0;
    __syncthreads();
    long long amt = 0;
    bool any_dev = false, any_ip = false;
    int k_base = 0;  // the account's events in the earlier row blocks
    for (int b0 = 0; b0 < n; b0 += HOT_THREADS) {
      const int i = b0 + tid;
      const bool m = i < n && t.rows[i] == s;
      const uint64_t bal = __ballot(m);
      if (lane == 0) s_wcnt[wv] = __popcll(bal);
      __syncthreads();
      int off = 0, blk = 0;
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        const int cq = s_wcnt[q];
        off += q < wv ? cq : 0;
        blk += cq;
      }
      __syncthreads();  // s_wcnt is rewritten by the next block
      if (m) {
        const int k = k_base + off + __popcll(bal & lt);  // the event's rank in row order
        if (k >= Nb) {
          s_tail[k - Nb] = i;
        } else {
          const ReqRec ev = a.req[i];
          amt += ev.amount;
          if (k >= ctot - R) {  // ring entries a later event of the batch overwrites are not written
            const int pos = (r.ring_head + k) % R;
            a.ring_ts[(size_t)s * R + pos] = (uint32_t)now;
            a.ring_amt[(size_t)s * R + pos] = ev.amount;
          }
          if (ev.dev_hash) {
            any_dev = true;
            atomicMax(&s_pre[ev.dev_hash & 255u], (uint32_t)hll_rank(ev.dev_hash));
          }
          if (ev.ip_hash) {
            any_ip = true;
            atomicMax(&s_pre[256 + (ev.ip_hash & 255u)], (uint32_t)hll_rank(ev.ip_hash));
          }
        }
      }
      k_base += blk;
    }
    amt = wave_sum(amt);
    const bool wd = __ballot(any_dev) != 0ull, wi = __ballot(any_ip) != 0ull;
    if (lane == 0) {
      s_wamt[wv] = amt;
      if (wd) atomicOr(&s_any[0], 1);
      if (wi) atomicOr(&s_any[1], 1);
    }
    __syncthreads();
    long long tot = 0;
#pragma unroll
    for (int q = 0; q < NW; ++q) tot += s_wamt[q];
    const bool ad = s_any[0] != 0, ai = s_any[1] != 0;
    // the bulk's registers: a key expired at the batch clock was reset by its first PFADD
    if (tid < 512) {
      const bool ip = tid >= 256;
      if (ip ? ai : ad) {
        uint8_t* const rb = reinterpret_cast<uint8_t*>(s_regs);
        const uint32_t exp = ip ? r.hll_ip_exp : r.hll_dev_exp;
        const uint32_t base = now >= (int64_t)exp ? 0u : (uint32_t)rb[tid];
        rb[tid] = (uint8_t)max(base, s_pre[tid]);
      }
    }
    __syncthreads();
    if (Nb > 0) {  // the bulk's scalar state, as its events applied one by one at `now`
      r.ring_head = (r.ring_head + Nb) % R;
      if (now >= (int64_t)r.sum_exp) r.sum_compat = 0;
      r.sum_compat += tot;
      r.sum_exp = (uint32_t)(now + cfg.sum_ttl);
      if (ad) r.hll_dev_exp = (uint32_t)(now + cfg.hll_ttl);
      if (ai) r.hll_ip_exp = (uint32_t)(now + cfg.hll_ttl);
      r.last_tx = (uint32_t)now;
      r.last_tx_exp = (uint32_t)(now + cfg.last_tx_ttl);
      if (now >= (int64_t)r.session_exp || r.session_start == 0) r.session_start = (uint32_t)now;
      r.session_exp = (uint32_t)(now + cfg.session_ttl);
      if (a.ev) {
        r.ev_head = (r.ev_head + Nb) % a.ev_ring;
        r.ev_count = r.ev_count + Nb > a.ev_ring ? a.ev_ring : r.ev_count + Nb;
      }
      r.last_event_ts = (uint32_t)now;
    }
    if (wv == 0) {  // the tail, exact, 64 events at a time
      // the bulk's raised registers: the cached estimates first (the tail refreshes them again
      // only if one of its own events raises a register)
      if (ad) r.hll_dev_n = hll_count_wave(reinterpret_cast<const uint8_t*>(s_regs), lane, a.hll_lc);
      if (ai) r.hll_ip_n = hll_count_wave(reinterpret_cast<const uint8_t*>(s_regs + 64), lane, a.hll_lc);
      for (int q = 0; q < Tn; q += 64) {
        const int c = min(64, Tn - q);
        const int pj = lane < c ? s_tail[q + lane] : 0;
        apply_chunk<true>(a, s, r, pj, c, lane, reinterpret_cast<uint8_t*>(s_regs), Nb + q, ctot);
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      g[lane] = s_regs[lane];
      g[64 + lane] = s_regs[64 + lane];
      if (lane == 0) store_rt(a.rt + s, r);
    }
    __syncthreads();  // the LDS is the next hot account's
  }
}

// The scorer path's whole post-K1 update in one launch (the hot and the other multi-event
// accounts are disjoint sets): workgroups [0, UPD_SEG_MULTI) run the multi-event list as 8 waves
// each (256 waves, as update_multi_kernel) and clear the next region; workgroups
// [UPD_SEG_MULTI, + HOT_BLOCKS) take the hot accounts. One dispatch instead of two back to back on
// the state stream (each paid its argument fetch, the dependent header / counter loads and the
// queue's inter-dispatch gap: ~7 us per batch, r5n timeline).
constexpr int UPD_SEG_MULTI = UPD_MULTI_BLOCKS / 2;
__global__ void __launch_bounds__(HOT_THREADS) update_segments_kernel(UpdateArgs a) {
  __shared__ union {
    HotLds hot;
    uint32_t regs[HOT_THREADS / 64][128];
  } L;
  const int b = (int)blockIdx.x;
  if (b < UPD_SEG_MULTI) {
    const int w0 = __builtin_amdgcn_readfirstlane(b * (HOT_THREADS / 64) + (int)(threadIdx.x >> 6));
    update_multi_body<HOT_THREADS / 64>(a, w0, UPD_SEG_MULTI * (HOT_THREADS / 64), b * HOT_THREADS + threadIdx.x,
                                        UPD_SEG_MULTI * HOT_THREADS, L.regs);
  } else {
    update_hot_body(a, b - UPD_SEG_MULTI, HOT_BLOCKS, L.hot);
  }
}

// ---------------------------------------------------------------------------------- launch
void launch_feature_assemble(const AssembleArgs& a, hipStream_t st) {
  if (a.n_rows <= 0) return;
  IGP_LAUNCH(feature_assemble_kernel, dim3((a.n_rows + 15) / 16), dim3(256), 0, st, a);
}

void launch_dedup_insert(const UpdateArgs& a, hipStream_t st) {
  if (a.n_max <= 0) return;
  if (!a.hdr || a.region >= 0 || (a.dcap & 3)) throw std::runtime_error("dedup_insert: scorer ring regions only");
  IGP_LAUNCH(dedup_insert_list_kernel, dim3((a.n_max + 63) / 64), dim3(64), 0, st, a);
}

void launch_update_segments(const UpdateArgs& a, hipStream_t st) {
  if (a.n_max <= 0) return;
  // scorer path: the hot accounts (> DEDUP_LIST events) one workgroup each, then one wave per
  // other multi-event account, 256 waves looping over the region's list
  if (a.region < 0) {
    IGP_LAUNCH(update_segments_kernel, dim3(UPD_SEG_MULTI + HOT_BLOCKS), dim3(HOT_THREADS), 0, st, a);
    return;
  }
  IGP_LAUNCH(update_multi_kernel, dim3(UPD_MULTI_BLOCKS), dim3(256), 0, st, a);
}

void launch_feature_update(const UpdateArgs& a, hipStream_t st) {
  if (a.n_max <= 0) return;
  IGP_LAUNCH(dedup_reset_kernel, dim3((a.dcap + 255) / 256), dim3(256), 0, st, a);
  const int g = (a.n_max + 255) / 256;
  IGP_LAUNCH(dedup_insert_kernel, dim3(g), dim3(256), 0, st, a);
  IGP_LAUNCH(update_single_kernel, dim3(g), dim3(256), 0, st, a);
  launch_update_segments(a, st);
}

}  // namespace igp

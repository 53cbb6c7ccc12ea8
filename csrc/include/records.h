// Fixed-layout records shared by the HIP kernels (device) and the C++ runtime (host).
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace igp {

// Transaction types (exact strings of risk.proto:41 / wallet tx types).
enum TxType : uint8_t { TX_DEPOSIT = 0, TX_WITHDRAW = 1, TX_BET = 2, TX_WIN = 3, TX_REFUND = 4,
                        TX_BONUS = 5, TX_UNKNOWN = 255 };

// FeatRec flag bits
enum : int32_t { FR_VPN = 1, FR_PROXY = 2, FR_TOR = 4, FR_DISPOSABLE = 8, FR_BONUS_ONLY = 16,
                 FR_BLACKLISTED = 32, FR_PARTIAL = 64, FR_NOT_OWNED = 128 };

// 128-byte per-request raw feature record, written by feature_assemble. Field order follows
// proto FeatureVector (risk.proto:197-235); int64 members are 8-byte aligned.
struct FeatRec {
  int32_t tx_count_1m;           // w0
  int32_t tx_count_5m;           // w1
  int32_t tx_count_1h;           // w2
  int32_t flags;                 // w3  FR_* bits
  int64_t tx_sum_1h;             // w4-5
  float tx_avg_1h;               // w6
  int32_t unique_devices_24h;    // w7
  int32_t unique_ips_24h;        // w8
  int32_t ip_country_changes_7d; // w9
  int32_t device_age_days;       // w10
  int32_t account_age_days;      // w11
  int64_t total_deposits;        // w12-13
  int64_t total_withdrawals;     // w14-15
  int64_t net_deposit;           // w16-17
  int32_t deposit_count;         // w18
  int32_t withdraw_count;        // w19
  int32_t time_since_last_tx;    // w20
  int32_t session_duration;      // w21
  float avg_bet_size;            // w22
  float win_rate;                // w23
  int32_t bonus_claim_count;     // w24
  float bonus_wager_rate;        // w25
  int32_t tx_type;               // w26 request echo
  int32_t slot;                  // w27 feature-store slot (-1 unknown account)
  int64_t amount;                // w28-29 request echo
  int32_t reserved0;             // w30
  int32_t reserved1;             // w31
};
static_assert(sizeof(FeatRec) == 128, "FeatRec must be 128 bytes");

// 8-byte packed scoring result (the D2H / all-gather payload):
//   w0 = score[0:8) | rule_score[8:16) | action[16:18) | ml_present[18] | reasons[20:32)
//   w1 = ml score float bits
struct ResultRec {
  uint32_t packed;
  float ml;
};
static_assert(sizeof(ResultRec) == 8, "ResultRec must be 8 bytes");

#define IGP_RES_SCORE(p) ((p) & 0xffu)
#define IGP_RES_RULE(p) (((p) >> 8) & 0xffu)
#define IGP_RES_ACTION(p) (((p) >> 16) & 0x3u)
#define IGP_RES_REASONS(p) ((p) >> 20)

}  // namespace igp

namespace igp {

// Per-account real-time scalars (the reference's Redis keys other than the tx ZSET/HLLs),
// 64 bytes. Times are unix seconds (uint32); a key is alive iff now < its expiry.
struct AcctRT {
  uint32_t hll_dev_exp;     // features:<id>:devices:24h TTL
  uint32_t hll_ip_exp;      // features:<id>:ips:24h TTL
  uint32_t last_tx;         // features:<id>:last_tx
  uint32_t last_tx_exp;
  uint32_t session_start;   // features:<id>:session_start
  uint32_t session_exp;
  uint32_t sum_exp;         // features:<id>:tx_sum:1h TTL (compat sum mode)
  uint32_t last_event_ts;   // previous event time (GRU dt feature)
  int64_t sum_compat;       // INCRBY running sum (compat mode)
  int32_t ring_head;        // next tx-ring write position
  int32_t ev_head;          // next event-ring write position
  int32_t ev_count;
  // HyperLogLog estimates of the two register files (before the TTL check), kept by every path
  // that changes a register (PFCOUNT on a cached cardinality, as Redis keeps it in the HLL header,
  // redis_store.go:80-81): feature assembly reads these 8 bytes instead of 512 register bytes
  int32_t hll_dev_n, hll_ip_n;
  // padding as a scalar, not an array: a kernel-local copy of a struct with an array member became
  // an LDS-promoted alloca indexed by the flat work-item id, i.e. one read of the dispatch packet
  // (host memory) per wave for the work-group size (K1, the update kernels)
  int32_t pad0;
};
static_assert(sizeof(AcctRT) == 64, "AcctRT must be 64 bytes");

// Warehouse batch features (engine.go:127-140), 80 bytes.
struct AcctBatch {
  int64_t total_deposits;
  int64_t total_withdrawals;
  int64_t total_bets;
  int64_t total_wins;
  int64_t account_created_at;
  int32_t deposit_count;
  int32_t withdraw_count;
  int32_t bet_count;
  int32_t win_count;
  float avg_bet_size;
  int32_t bonus_claim_count;
  float bonus_wager_complete;
  int32_t present;          // 0 = batch features unavailable (partial features, quirk Q10)
  int32_t pad0, pad1;
};
static_assert(sizeof(AcctBatch) == 80, "AcctBatch must be 80 bytes");

// Scoring configuration block kept in device memory: graphs read it on every replay, so
// UpdateThresholds never needs a graph re-capture (engine.go:196-228, 246-257).
struct ScoreCfg {
  int32_t block_threshold;
  int32_t review_threshold;
  int32_t max_tx_per_minute;
  int32_t new_account_days;
  int64_t large_deposit_amount;
  int32_t max_devices_per_day;
  int32_t max_ips_per_day;
  double ml_weight;
  double rule_weight;
  double ml_high_risk;
  double ml_error_score;
  int32_t w_high_velocity, w_new_account_large_tx, w_multiple_devices, w_ip_country_mismatch;
  int32_t w_vpn, w_rapid_deposit_withdraw, w_bonus_abuse, w_known_fraudster;
  int32_t model_kind;       // 0 none, 1 heuristic (mockPredict), 2 model output buffer
  int32_t ml_col;           // column of the model output holding P(fraud)
  int32_t ml_stride;        // row stride of the model output
  int32_t log_identity;     // 1 = reference stub log1p(x)=x (quirk Q1)
  int32_t sum_compat;       // 1 = INCRBY-with-TTL 1h sum (quirk Q8)
  int32_t session_ttl, last_tx_ttl, hll_ttl, sum_ttl;
  int32_t bl_mask;          // blacklist table capacity - 1
  int32_t bl_max_probe;
  int32_t ip_mask;          // ip-intel table capacity - 1
  int32_t ip_max_probe;
  int32_t ext_width;        // feature-vector columns beyond the 30 reference ones
  int32_t owner_filter;     // 1: rows whose owner (ReqRec.tx_type bits 8..15) != my_rank are skipped
  int32_t my_rank;
  int32_t pad0, pad1, pad2;
};
static_assert(sizeof(ScoreCfg) == 176, "ScoreCfg must be 176 bytes");
// feature_assemble reads ScoreCfg bytes 128..159 as two int4 (csrc/kernels/features.hip)
static_assert(offsetof(ScoreCfg, bl_mask) == 132 && offsetof(ScoreCfg, ip_max_probe) == 144 &&
                  offsetof(ScoreCfg, ext_width) == 148 && offsetof(ScoreCfg, my_rank) == 156,
              "ScoreCfg K1 block moved");

// One scoring request / transaction event as shipped host->device (48 bytes). A batch is a
// contiguous slab [BatchHdr | ReqRec x n]: one H2D copy per micro-batch.
struct ReqRec {
  int32_t slot;       // feature-store slot on this GPU (-1 = unknown account)
  int32_t tx_type;    // TxType in bits 0..7, owner rank in bits 8..15 (broadcast serving mode),
                      // bit 16 FV_ENC_BIT: the request wants response bytes (encoded features)
  int64_t amount;     // cents
  uint64_t dev_hash;  // XXH64 digests, 0 = absent
  uint64_t fp_hash;
  uint64_t ip_hash;
  int64_t ts;         // event time (unix s) used by feature_update
};
static_assert(sizeof(ReqRec) == 48, "ReqRec must be 48 bytes");

// ReqRec.tx_type bit 16: the device writes the row's risk.v1 FeatureVector body, encoded, as the
// row's 128-byte D2H feature image instead of the raw FeatRec (features.hip write_fenc). The
// image's byte 127 tells them apart: 0x80 | length for an encoded body (<= 126 bytes), 0 for a
// raw FeatRec (the top byte of its rule score).
constexpr int32_t FV_ENC_BIT = 1 << 16;
constexpr uint8_t FV_IMG_ENCODED = 0x80;

// Per-batch header in device memory (written by one H2D copy per batch, read by every
// kernel of the captured graph): the number of live rows and the scoring clock.
struct BatchHdr {
  int32_t n;
  int32_t seq;    // batch sequence number (dedup-table ping-pong parity)
  int64_t now;
};
static_assert(sizeof(BatchHdr) == 16, "BatchHdr must be 16 bytes (dedup_insert_list_kernel reads it as one int4)");

}  // namespace igp

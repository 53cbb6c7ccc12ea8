// Fixed-layout records shared by the HIP kernels (device) and the C++ runtime (host).
#pragma once
#include <stdint.h>

namespace igp {

// Transaction types (exact strings of risk.proto:41 / wallet tx types).
enum TxType : uint8_t { TX_DEPOSIT = 0, TX_WITHDRAW = 1, TX_BET = 2, TX_WIN = 3, TX_REFUND = 4,
                        TX_BONUS = 5, TX_UNKNOWN = 255 };

// FeatRec flag bits
enum : int32_t { FR_VPN = 1, FR_PROXY = 2, FR_TOR = 4, FR_DISPOSABLE = 8, FR_BONUS_ONLY = 16,
                 FR_BLACKLISTED = 32, FR_PARTIAL = 64 };

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

// risk.v1 wire codec: ScoreBatchRequest / ScoreTransactionRequest bytes -> columnar batch
// (identifiers hashed on the way in, strings never reach Python or the GPU), and packed
// device results -> ScoreBatchResponse / ScoreTransactionResponse bytes.
// Field numbers: /root/reference/proto/risk/v1/risk.proto:38-82, 197-235.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <string_view>
#include <vector>

#include "../include/records.h"

namespace igp::wire {

// Account ids stay views into copies of the request payloads the batch owns (one copy per
// parse call, no per-row allocation).
struct RequestBatch {
  std::vector<std::string_view> account_id;
  std::vector<uint64_t> account_hash;
  std::vector<int64_t> amount;
  std::vector<uint8_t> tx_type;
  std::vector<uint64_t> device_hash, fp_hash, ip_hash;
  std::vector<std::unique_ptr<std::string>> arena;
  size_t size() const { return amount.size(); }
  void clear();
  void reserve(size_t n);
  // copy a payload into the arena; returns the stable copy
  const std::string& own(const char* data, size_t n);
};

// One parsed transaction for the native serving core (engine/serving.py): the account id
// (a view into the caller's payload), its digest and the device request record with the
// slot still unresolved (-1) and ts 0.
struct TxRow {
  std::string_view account;
  uint64_t account_hash;
  ReqRec rec;
};

uint8_t tx_type_id(const char* s, size_t n);

// Append one ScoreTransactionRequest message body.
void parse_tx(const char* data, size_t n, RequestBatch& out);
// Append every transaction of a ScoreBatchRequest.
void parse_batch(const char* data, size_t n, RequestBatch& out);
// AoS forms (no copy of the payload: views stay valid while the payload does)
void parse_tx_row(const char* data, size_t n, TxRow& out);
void parse_batch_rows(const char* data, size_t n, std::vector<TxRow>& out);

extern const char* const kReasonCodes[12];

struct ResultView {
  const ResultRec* res;
  const FeatRec* feat;          // may be null (features omitted)
  const int64_t* response_ms;   // may be null (0)
  size_t n;
};
std::string serialize_tx_response(const ResultView& v, size_t i);
std::string serialize_batch_response(const ResultView& v);
std::string serialize_feature_vector(const FeatRec& f);

// Single-pass writers on raw memory (the serving core's response path). A
// ScoreTransactionResponse body is at most kMaxTxResponse bytes; a ScoreBatchResponse entry
// (tag + length + body) at most kMaxTxResponse + 8.
constexpr size_t kMaxTxResponse = 1024;
size_t write_tx_response(char* out, const ResultRec& r, const FeatRec* f, int64_t ms);
constexpr size_t kMaxBatchRowBytes = kMaxTxResponse + 8;
// ScoreBatchResponse of n rows written at dst (capacity n * kMaxBatchRowBytes); returns its size
size_t write_batch_response(char* dst, const ResultRec* r, const FeatRec* f, const int64_t* ms, int64_t ms_all,
                            size_t n);
// the same into this thread's grow-only scratch buffer (valid until its next call on the thread)
std::string_view batch_response_scratch(const ResultRec* r, const FeatRec* f, const int64_t* ms, int64_t ms_all,
                                        size_t n);
// ScoreBatchResponse of n rows appended to `out`
void append_batch_response(std::string& out, const ResultRec* r, const FeatRec* f, const int64_t* ms, int64_t ms_all,
                           size_t n);

}  // namespace igp::wire

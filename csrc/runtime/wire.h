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
// parse call, no per-row allocation); account_check is the AccountIndex check digest.
struct RequestBatch {
  std::vector<std::string_view> account_id;
  std::vector<uint64_t> account_hash;
  std::vector<uint32_t> account_check;
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

uint8_t tx_type_id(const char* s, size_t n);

// Append one ScoreTransactionRequest message body.
void parse_tx(const char* data, size_t n, RequestBatch& out);
// Append every transaction of a ScoreBatchRequest.
void parse_batch(const char* data, size_t n, RequestBatch& out);

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

}  // namespace igp::wire

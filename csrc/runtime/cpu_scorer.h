// Native CPU scoring path: the host twin of the GPU pipeline (K1 feature_assemble + K7/K8,
// the model through exec::Executor or the heuristic, K5 ensemble, K6 score-then-update).
//
// This is config 1's serving path (BASELINE: ScoreTransaction on CPU, 32-feature logistic,
// batch 1) and the degraded-mode fallback when a GPU shard is unhealthy. It keeps the same
// SoA account state as the device store (records.h: AcctRT / AcctBatch, tx ring, HLL
// registers, event ring) and produces byte-identical FeatRec / ResultRec records, so the
// wire serializer and every test treat both backends alike. Scoring reads all rows of a batch
// first and applies the batch's events afterwards in request order (the device semantics).
#pragma once
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../include/records.h"
#include "executor.h"

namespace igp {

class CpuScorer {
 public:
  CpuScorer(int64_t capacity, int ring_size, int event_ring, int event_dim, int ext_width);

  void set_cfg(const ScoreCfg& c);
  const ScoreCfg& cfg() const { return cfg_; }
  // blacklist / ip-intel open-addressing tables (same layout as the device copies)
  void set_tables(const uint64_t* bl_keys, const uint32_t* bl_exp, size_t bl_n, const uint64_t* ip_keys,
                  const uint32_t* ip_flags, size_t ip_n);
  // model: executor + input name + output name + column holding P(fraud); null -> cfg.model_kind
  void set_model(std::shared_ptr<exec::Executor> ex, std::string in_name, std::string out_name, int ml_col);

  void set_batch(const int32_t* slots, const AcctBatch* rows, size_t n);
  void set_ext(const int32_t* slots, const float* ext, size_t n, int width);
  void reset(const int32_t* slots, size_t n);
  // ordered feature update (IngestEvents); events carry their own ts
  void ingest(const ReqRec* ev, size_t n);
  // score a batch at `now`: res[n], feat[n] (nullable), then apply the batch's events when update
  void score(const ReqRec* req, size_t n, int64_t now, bool update, ResultRec* res, FeatRec* feat);
  // K1 for one account (GetFeatures): synthetic request, no update
  FeatRec features(int32_t slot, int64_t now);
  // event history, oldest first, right-aligned: out[event_ring * event_dim]
  void event_history(int32_t slot, float* out) const;

  int64_t capacity() const { return cap_; }
  int ring_size() const { return R_; }
  int event_ring() const { return ER_; }
  int event_dim() const { return ED_; }
  int ext_width() const { return EW_; }
  // raw state (snapshots)
  std::vector<uint32_t> ring_ts;
  std::vector<int64_t> ring_amt;
  std::vector<uint8_t> hll;
  std::vector<AcctRT> rt;
  std::vector<AcctBatch> batch;
  std::vector<float> ext;
  std::vector<uint16_t> ev;

 private:
  void assemble(const ReqRec& q, int64_t now, FeatRec& f, float* x) const;
  void apply(const ReqRec& q, int64_t now);
  bool blacklisted(uint64_t key, int64_t now) const;
  int ip_flags(uint64_t key) const;

  int64_t cap_;
  int R_, ER_, ED_, EW_;
  ScoreCfg cfg_{};
  std::vector<uint64_t> bl_keys_, ip_keys_;
  std::vector<uint32_t> bl_exp_, ip_flags_;
  std::shared_ptr<exec::Executor> ex_;
  std::string in_name_, out_name_;
  int ml_col_ = 0;
  mutable std::mutex mu_;
};

}  // namespace igp

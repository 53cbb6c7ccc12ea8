// CPU devices behind the serving core's function table (device_ops.h):
//
// * CpuDevice      one CPU shard (CpuScorer): the degraded / GPU-less serving path and the CPU
//                  twin of the single-GPU pipeline.
// * ShmXchgDevice  one rank of a CPU data-parallel group on one node: the owner-routed
//                  exchange of csrc/kernels/exchange.hip over /dev/shm instead of RCCL. Every
//                  rank posts its [world][C + 1] ReqRec owner chunks, scores the rows it owns,
//                  posts [world][C] result records (+ FeatRec) back, and gathers its own rows'
//                  results: the same wire format, the same step protocol, so the multi-process
//                  CPU tests exercise the exact serving-core paths the GPU ranks run.
#pragma once
#include <atomic>
#include <memory>
#include <string>
#include <vector>

#include "../include/device_ops.h"
#include "../include/records.h"
#include "../include/results_region.h"
#include "cpu_scorer.h"
#include "shm.h"

namespace igp {

class CpuDevice {
 public:
  CpuDevice(std::shared_ptr<CpuScorer> sc, int depth, int cap);
  const IgpDeviceOps* ops() const { return &ops_; }

 private:
  struct Slot {
    std::vector<ReqRec> rows;
    std::vector<ResultRec> res;
    std::vector<FeatRec> feat;
    bool wf = false;
  };
  static char* rows_fn(void* ctx, int32_t slot);
  static int32_t submit_fn(void* ctx, int32_t slot, int32_t n, int32_t seq, int64_t now, int32_t wf, char* err, int32_t errlen);
  static int32_t wait_fn(void* ctx, int32_t slot, int64_t timeout_us, char* err, int32_t errlen);
  static const void* results_fn(void* ctx, int32_t slot);
  static const void* features_fn(void* ctx, int32_t slot);
  std::shared_ptr<CpuScorer> sc_;
  std::vector<Slot> slots_;
  IgpDeviceOps ops_{};
};

class ShmXchgDevice {
 public:
  ShmXchgDevice(std::shared_ptr<CpuScorer> sc, const std::string& shm_name, int world, int rank, int depth, int C,
                bool create, double timeout_s);
  const IgpDeviceOps* ops() const { return &ops_; }
  int64_t rows_scored() const { return rows_scored_.load(); }
  // steps whose pipeline slot differed from step index % depth here, or from the slot a peer ran
  // the same step on (the serving core's exchange-mode slot contract, serve_core.cpp)
  int64_t slot_violations() const { return slot_violations_.load(); }
  int64_t steps() const { return k_; }
  // fault injection: once the file `path` exists this rank keeps posting its rows but never
  // publishes its results again (the peers' steps must fail within the deadline;
  // tests/test_failover.py)
  void debug_stall_results_when(const std::string& path) { stall_file_ = path; }
  void unlink_shared() { region_.unlink(); }

 private:
  static constexpr int kRing = 2;
  struct alignas(64) Counter {
    std::atomic<int64_t> posted;
    std::atomic<int64_t> scored;
    std::atomic<int32_t> slot;  // pipeline slot of the step last posted
    char pad[44];
  };
  struct Slot {
    std::vector<ReqRec> send;   // [world][C + 1]
    std::vector<char> recv;     // [world][C * W]
  };
  static char* rows_fn(void* ctx, int32_t slot);
  static int32_t submit_fn(void* ctx, int32_t slot, int32_t n, int32_t seq, int64_t now, int32_t wf, char* err, int32_t errlen);
  static int32_t wait_fn(void* ctx, int32_t slot, int64_t timeout_us, char* err, int32_t errlen);
  static const void* results_fn(void* ctx, int32_t slot);
  static const void* features_fn(void* ctx, int32_t slot);
  void step(int slot, int64_t now);
  void wait_all(std::atomic<int64_t> Counter::*field, int64_t target);
  ReqRec* send_area(int r, int q) const;
  char* res_area(int r, int q) const;

  std::shared_ptr<CpuScorer> sc_;
  Region region_;
  Counter* counters_ = nullptr;
  char* data_ = nullptr;
  int world_, rank_, C_;
  size_t W_, send_bytes_, res_bytes_;
  double timeout_s_;
  int64_t k_ = 0;  // steps done
  std::string stall_file_;
  bool stalled_ = false;
  OwnerGenerations owners_;
  std::vector<Slot> slots_;
  std::vector<ReqRec> compact_;
  std::vector<int32_t> route_;
  std::vector<ResultRec> res_;
  std::vector<FeatRec> feat_;
  std::atomic<int64_t> rows_scored_{0};
  std::atomic<int64_t> slot_violations_{0};
  IgpDeviceOps ops_{};
};

}  // namespace igp

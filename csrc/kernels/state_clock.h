// Read-your-writes for feature-store readers.
//
// Contract: a read of an account's feature state (GetFeatures / features_many, the event history,
// CheckBonusAbuse's K1 + GRU step, the Python abuse runner) that is ISSUED after a
// ScoreBatch / ScoreTransaction response was delivered sees that batch's store updates - its
// single-event applies in K1 and the multi-event segments after it (the model stage, whose
// completion delivers the response, waits for K1 only).
//
// Enforcement on the device, no host sync: the scoring driver (PipeDriver, or XchgDriver for the
// owner-routed exchange) publishes the event it records after each batch's whole state stage;
// a reader makes its own stream wait for the latest published event before its first read
// (skipped when the host already sees it complete). Events are reused per pipeline slot: if the
// slot's event was re-recorded for a newer batch meanwhile, the reader waits for that newer
// batch instead - a superset of the contract, never less.
//
// One clock per GPU shard, owned by the backend (engine/backends.py) and handed to every driver
// of that shard, so a scorer rebuilt after a failover keeps publishing into the clock its
// readers hold. The published events belong to the driver: a driver that goes away (hot reload,
// leave_exchange) retracts its events before destroying them, and readers hold the clock's lock
// while they query / wait on the event, so no reader can touch an event after its retract.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <mutex>
#include <stdexcept>
#include <string>

namespace igp {

class StateClock {
 public:
  // producer: `e` was just recorded on the stream that ran the batch's last state kernel
  void publish(hipEvent_t e) {
    last_.store(e, std::memory_order_release);
    published_.fetch_add(1, std::memory_order_relaxed);
  }
  // consumer: order `st` after the latest published state stage
  void wait(hipStream_t st) {
    std::lock_guard<std::mutex> g(mu_);
    hipEvent_t e = last_.load(std::memory_order_acquire);
    if (!e) return;
    const hipError_t q = hipEventQuery(e);
    if (q == hipSuccess) {
      skips_.fetch_add(1, std::memory_order_relaxed);
      return;
    }
    if (q != hipErrorNotReady) throw std::runtime_error(std::string("StateClock query: ") + hipGetErrorString(q));
    const hipError_t w = hipStreamWaitEvent(st, e, 0);
    if (w != hipSuccess) throw std::runtime_error(std::string("StateClock wait: ") + hipGetErrorString(w));
    waits_.fetch_add(1, std::memory_order_relaxed);
  }
  // a driver's destructor, before hipEventDestroy of its n events: the clock forgets them. A
  // batch issued by that driver has already finished or is ordered before the caller's teardown
  // sync, so readers lose nothing by skipping its wait.
  void retract(const hipEvent_t* ev, size_t n) {
    std::lock_guard<std::mutex> g(mu_);
    hipEvent_t cur = last_.load(std::memory_order_acquire);
    for (size_t i = 0; i < n && cur; ++i)
      if (ev[i] == cur) {
        last_.compare_exchange_strong(cur, nullptr, std::memory_order_acq_rel);
        retracts_.fetch_add(1, std::memory_order_relaxed);
        break;
      }
  }
  int64_t published() const { return published_.load(); }
  int64_t retracts() const { return retracts_.load(); }
  int64_t waits() const { return waits_.load(); }
  int64_t skips() const { return skips_.load(); }

 private:
  std::atomic<hipEvent_t> last_{nullptr};
  std::atomic<int64_t> published_{0}, waits_{0}, skips_{0}, retracts_{0};
  std::mutex mu_;  // readers' query / wait vs retract (publish is lock-free)
};

}  // namespace igp

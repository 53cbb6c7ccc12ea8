// Owner generations of the node-shared results region (owner-routed exchange, N > 1).
//
// Every owner writes the rows it scored for all senders into its block of a node-shared region
// and then publishes the step's generation in its flag line [slot][owner] (one 64-byte line
// each); a sender's step is complete once every owner's line reached the generation. Used by the
// GPU exchange driver (exchange.hip XchgDriver::wait_owners, after the slot's local event) and
// by the CPU exchange device (cpu_device.cpp ShmXchgDevice), so the CPU multi-process tests run
// the same completion protocol, dead-owner path included.
//
// A wait always has a finite deadline: an owner that stops publishing - a
// hung GPU or a stuck process, alive enough that nothing else notices - fails the step with an
// error that names it, and the serving core then fails the step's requests and triggers the
// group failover (risk_engine.py _group_failed) instead of spinning forever.
#pragma once
#include <sys/prctl.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>

namespace igp {

class OwnerGenerations {
 public:
  static constexpr int kLineWords = 8;  // int64 words per flag line

  OwnerGenerations() = default;
  // `what`: how a timeout names the ranks behind ("results region: owner(s)", "rows region: sender(s)")
  OwnerGenerations(int64_t* flags, int world, int rank, const char* what = "results region: owner(s)")
      : flags_(flags), world_(world), rank_(rank), what_(what) {}
  bool valid() const { return flags_ != nullptr; }
  int world() const { return world_; }

  int64_t* line(int slot, int owner) const { return flags_ + (size_t(slot) * world_ + owner) * kLineWords; }
  int64_t published(int slot, int owner) const { return __atomic_load_n(line(slot, owner), __ATOMIC_ACQUIRE); }
  // this rank's rows of the step are in the region (the caller ordered its writes before this)
  void publish(int slot, int64_t gen) const { __atomic_store_n(line(slot, rank_), gen, __ATOMIC_RELEASE); }

  // 0: every owner reached `gen`; 1: `timeout_us` (>= 0, finite) passed - `err` names the owners
  // still behind. Spins `spin_us`, then sleeps 20 us at a time.
  int wait(int slot, int64_t gen, int64_t timeout_us, int64_t spin_us, char* err, int errlen) const {
    const auto t0 = std::chrono::steady_clock::now();
    const auto t_end = t0 + std::chrono::microseconds(timeout_us < 0 ? 0 : timeout_us);
    const auto t_spin = t0 + std::chrono::microseconds(spin_us);
    for (;;) {
      bool all = true;
      for (int o = 0; o < world_ && all; ++o) all = published(slot, o) >= gen;
      if (all) return 0;
      const auto now = std::chrono::steady_clock::now();
      if (now >= t_end) {
        describe(slot, gen, timeout_us, err, errlen);
        return 1;
      }
      if (now >= t_spin) {
        thread_local bool slack = false;
        if (!slack) {
          prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
          slack = true;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
    }
  }

 private:
  void describe(int slot, int64_t gen, int64_t timeout_us, char* err, int errlen) const {
    if (!err || errlen <= 0) return;
    std::string owners;
    for (int o = 0; o < world_; ++o)
      if (published(slot, o) < gen) owners += (owners.empty() ? "" : ",") + std::to_string(o);
    char buf[256];
    std::snprintf(buf, sizeof buf,
                  "%s %s did not publish generation %lld of slot %d within %.1f ms", what_,
                  owners.empty() ? "?" : owners.c_str(), (long long)gen, slot, double(timeout_us) / 1e3);
    std::strncpy(err, buf, size_t(errlen) - 1);
    err[errlen - 1] = 0;
  }

  int64_t* flags_ = nullptr;
  int world_ = 0, rank_ = 0;
  const char* what_ = "results region: owner(s)";
};

}  // namespace igp

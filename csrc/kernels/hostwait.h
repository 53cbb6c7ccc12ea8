// Host-side waits of the device drivers (driver.hip, exchange.hip): a short spin, then sleeps.
//
// A pipeline step completes every ~60-150 us and the serving core's completion thread waits on
// every one of them. The drivers used to spin 4096 hipEventQuery calls (milliseconds) before the
// first sleep, so that thread kept a core busy for good and queried the HIP runtime's event path
// beside the stepper thread's launches. Now: spin for IGP_WAIT_SPIN_US (default 30 us), then
// sleep 20 us at a time with the thread's timer slack at 1 us (Linux otherwise stretches a
// 20-us sleep to ~70 us).
#pragma once
#include <hip/hip_runtime.h>
#include <sys/prctl.h>

#include <chrono>
#include <cstdlib>
#include <thread>

namespace igp {

inline int64_t wait_spin_us() {
  static const int64_t v = [] {
    const char* e = std::getenv("IGP_WAIT_SPIN_US");
    return e ? std::atoll(e) : int64_t(30);
  }();
  return v;
}

inline void wait_backoff(std::chrono::steady_clock::time_point t_spin_end) {
  if (std::chrono::steady_clock::now() < t_spin_end) return;
  thread_local bool slack = false;
  if (!slack) {
    prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
    slack = true;
  }
  std::this_thread::sleep_for(std::chrono::microseconds(20));
}

// true: the event completed; false: the deadline passed. Errors other than "not ready" go to
// `on_error` (which returns or throws).
template <class OnError>
inline bool poll_event_until(hipEvent_t e, std::chrono::steady_clock::time_point t_end, OnError on_error) {
  const auto t_spin = std::chrono::steady_clock::now() + std::chrono::microseconds(wait_spin_us());
  for (;;) {
    const hipError_t q = hipEventQuery(e);
    if (q == hipSuccess) return true;
    if (q != hipErrorNotReady) {
      on_error(q);
      return false;
    }
    if (std::chrono::steady_clock::now() >= t_end) return false;
    wait_backoff(t_spin);
  }
}

}  // namespace igp

// Batch watchdog: deadline waits on HIP events, plus a bounded stall kernel that the
// fault-injection tests use to make a real device batch overrun its deadline.
//
// hipEventSynchronize has no timeout, so wait_for polls the caller's own event with
// hipEventQuery (GIL released): a short spin, then a back-off of 20 us -> 1 ms sleeps. Every
// wait is independent: a hung batch delays only the callers waiting on THAT batch (an earlier
// design queued every request on one watcher thread blocked in hipEventSynchronize, so one
// overrun cascaded into false timeouts for later batches), and nothing keeps a raw event after
// wait_for returns, so the event's owner may go away at once (reference: the Go service bounds
// each score with a context deadline, services/risk/internal/scoring/engine.go:279-282).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <atomic>
#include <chrono>
#include <stdexcept>
#include <string>
#include <thread>

namespace py = pybind11;

namespace igp {
namespace {

class EventWatch {
 public:
  // true once the event completed; false when `timeout_ms` passed first
  bool wait_for(uintptr_t event, double timeout_ms) {
    hipEvent_t ev = reinterpret_cast<hipEvent_t>(event);
    hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return true;
    if (q != hipErrorNotReady) throw std::runtime_error(std::string("EventWatch: ") + hipGetErrorString(q));
    py::gil_scoped_release nogil;
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::duration<double, std::milli>(timeout_ms);
    int64_t sleep_us = 20;
    for (int spin = 0;; ++spin) {
      q = hipEventQuery(ev);
      if (q == hipSuccess) {
        completed_.fetch_add(1);
        return true;
      }
      if (q != hipErrorNotReady) {
        py::gil_scoped_acquire gil;
        throw std::runtime_error(std::string("EventWatch: batch failed: ") + hipGetErrorString(q));
      }
      const auto now = std::chrono::steady_clock::now();
      if (now >= t_end) {
        timeouts_.fetch_add(1);
        return false;
      }
      if (spin < 256) continue;
      const auto left = std::chrono::duration_cast<std::chrono::microseconds>(t_end - now).count();
      std::this_thread::sleep_for(std::chrono::microseconds(std::min<int64_t>(sleep_us, std::max<int64_t>(left, 1))));
      sleep_us = std::min<int64_t>(sleep_us * 2, 1000);
    }
  }

  // waits that gave up at their deadline / that saw their event complete
  int64_t timeouts() const { return timeouts_.load(); }
  int64_t completed() const { return completed_.load(); }

 private:
  std::atomic<int64_t> timeouts_{0}, completed_{0};
};

// One wave that sleeps until `ticks` of the 100 MHz constant clock have passed (bounded: the
// host caps the duration; no memory traffic).
__global__ void __launch_bounds__(64) stall_kernel(int64_t ticks) {
  const int64_t t0 = wall_clock64();
  for (int i = 0; i < (1 << 28); ++i) {
    if (wall_clock64() - t0 >= ticks) break;
    __builtin_amdgcn_s_sleep(64);
  }
}

void stall(uintptr_t stream, double us) {
  if (!(us >= 0 && us <= 10e6)) throw std::runtime_error("stall: 0..10 s");
  const int64_t ticks = (int64_t)(us * 100.0);  // wall_clock64: 100 MHz
  hipLaunchKernelGGL(stall_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), ticks);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("stall launch: ") + hipGetErrorString(e));
}

}  // namespace

void register_watch(py::module_& m) {
  py::class_<EventWatch>(m, "EventWatch")
      .def(py::init<>())
      .def("wait_for", &EventWatch::wait_for, py::arg("event"), py::arg("timeout_ms"))
      .def("timeouts", &EventWatch::timeouts)
      .def("completed", &EventWatch::completed);
  m.def("stall", &stall, py::arg("stream"), py::arg("us"),
        "Enqueue a one-wave kernel that sleeps for `us` microseconds on `stream` (fault injection).");
}

}  // namespace igp

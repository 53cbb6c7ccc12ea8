// Batch watchdog: deadline waits on HIP events without polling, plus a bounded stall kernel
// that the fault-injection tests use to make a real device batch overrun its deadline.
//
// hipEventSynchronize has no timeout, so one watcher thread per EventWatch blocks in it (GIL
// released, FIFO over the requests) and signals a condition variable; the caller sleeps on that
// variable until the event completes or its deadline passes. A request that overran keeps being
// waited on, so a late batch is still observed (engine/backends.py drains the quarantined slot).
// The watcher's state is shared with the thread: destroying an EventWatch whose watcher is stuck
// in a hung event detaches it instead of blocking (reference: the Go service bounds each score
// with a context deadline, services/risk/internal/scoring/engine.go:279-282).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

namespace py = pybind11;

namespace igp {
namespace {

struct WatchReq {
  hipEvent_t ev;
  bool done = false;
  hipError_t err = hipSuccess;
};

struct WatchState {
  std::mutex mu;
  std::condition_variable cv;       // new request / stop
  std::condition_variable done_cv;  // a request completed
  std::deque<std::shared_ptr<WatchReq>> q;
  bool stop = false;
  int64_t completed = 0;
};

void watch_loop(std::shared_ptr<WatchState> s) {
  std::unique_lock<std::mutex> lk(s->mu);
  for (;;) {
    s->cv.wait(lk, [&] { return s->stop || !s->q.empty(); });
    if (s->q.empty()) return;  // stop requested, nothing left to observe
    auto r = s->q.front();
    lk.unlock();
    const hipError_t err = hipEventSynchronize(r->ev);
    lk.lock();
    r->err = err;
    r->done = true;
    s->q.pop_front();
    ++s->completed;
    s->done_cv.notify_all();
    if (s->stop) return;
  }
}

class EventWatch {
 public:
  EventWatch() : s_(std::make_shared<WatchState>()) { std::thread(watch_loop, s_).detach(); }
  ~EventWatch() {
    {
      std::lock_guard<std::mutex> lk(s_->mu);
      s_->stop = true;
    }
    s_->cv.notify_all();
  }

  // true once the event completed; false when `timeout_ms` passed first (the watcher goes on
  // waiting for it: pending() counts such requests until they finish)
  bool wait_for(uintptr_t event, double timeout_ms) {
    hipEvent_t ev = reinterpret_cast<hipEvent_t>(event);
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return true;
    if (q != hipErrorNotReady) throw std::runtime_error(std::string("EventWatch: ") + hipGetErrorString(q));
    auto r = std::make_shared<WatchReq>();
    r->ev = ev;
    py::gil_scoped_release nogil;
    std::unique_lock<std::mutex> lk(s_->mu);
    s_->q.push_back(r);
    s_->cv.notify_all();
    const bool ok = s_->done_cv.wait_for(lk, std::chrono::duration<double, std::milli>(timeout_ms),
                                         [&] { return r->done; });
    if (ok && r->err != hipSuccess)
      throw std::runtime_error(std::string("EventWatch: batch failed: ") + hipGetErrorString(r->err));
    return ok;
  }

  int pending() {
    std::lock_guard<std::mutex> lk(s_->mu);
    return (int)s_->q.size();
  }
  int64_t completed() {
    std::lock_guard<std::mutex> lk(s_->mu);
    return s_->completed;
  }

 private:
  std::shared_ptr<WatchState> s_;
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
      .def("pending", &EventWatch::pending)
      .def("completed", &EventWatch::completed);
  m.def("stall", &stall, py::arg("stream"), py::arg("us"),
        "Enqueue a one-wave kernel that sleeps for `us` microseconds on `stream` (fault injection).");
}

}  // namespace igp

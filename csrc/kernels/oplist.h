// Recorded kernel launches: the native driver's alternative to hipGraph replay.
//
// On MI355X a one-kernel hipGraphLaunch costs ~7.6 us of queue time before its kernel starts,
// against ~0.75 us between two plain kernel launches on the same stream
// (tools/probe/queue_hop_probe.hip, profiles/NOTES.md). The scorer's three stages are two or
// three kernels each, so replaying them as graphs spent ~20 us of device time per batch on graph
// launches. In record mode the launch bindings (bindings.hip) store each launch as a closure
// over its frozen argument struct - the same freezing a graph capture does - and the driver
// issues the list with plain launches on the stage's stream.
//
// Stage-end events: the driver's cross-stream hand-offs need an event after each stage. A
// hipEventRecord enqueues a marker command of its own (~2-3 us of host API time each, four per
// batch). run_recording() instead arms a thread-local stop event that the stage's LAST kernel
// launch binds to its own dispatch (hipExtLaunchKernel's stopEvent): the event completes with
// that kernel and no marker is issued. Every kernel launch goes through IGP_LAUNCH so any
// launcher can end a stage; a copy issued after it disarms the binding and the driver falls
// back to hipEventRecord.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <functional>
#include <memory>
#include <vector>

namespace igp {

struct StopEvent {
  hipEvent_t ev = nullptr;  // armed: the next kernel launches bind it
  bool bound = false;       // the most recent command issued while armed carries it
};
StopEvent& stop_event();  // thread-local (bindings.hip)

struct OpList {
  std::vector<std::function<void(hipStream_t)>> ops;
  void run(hipStream_t st) const {
    for (const auto& f : ops) f(st);
  }
  // run, with `ev` bound to the completion of the last op's last kernel; false when the last
  // command was not a kernel launch (the caller then records ev itself)
  bool run_recording(hipStream_t st, hipEvent_t ev) const {
    if (ops.empty()) return false;
    for (size_t i = 0; i + 1 < ops.size(); ++i) ops[i](st);
    StopEvent& s = stop_event();
    s.ev = ev;
    s.bound = false;
    try {
      ops.back()(st);
    } catch (...) {
      s.ev = nullptr;
      throw;
    }
    const bool ok = s.bound;
    s.ev = nullptr;
    s.bound = false;
    return ok;
  }
};

// non-null while a body is being recorded on this thread (bindings.hip record_begin / _end)
OpList*& recording();

}  // namespace igp

// kernel launch used by every launcher: a plain launch, or with the armed stop event bound
#define IGP_LAUNCH(kern, grid, block, lds, st, ...)                                                  \
  do {                                                                                              \
    ::igp::StopEvent& igp_se_ = ::igp::stop_event();                                                \
    if (igp_se_.ev) {                                                                               \
      hipExtLaunchKernelGGL(kern, grid, block, lds, st, nullptr, igp_se_.ev, 0, __VA_ARGS__);       \
      igp_se_.bound = true;                                                                         \
    } else {                                                                                        \
      hipLaunchKernelGGL(kern, grid, block, lds, st, __VA_ARGS__);                                  \
    }                                                                                               \
  } while (0)

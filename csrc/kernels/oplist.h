// Recorded kernel launches: the native driver's alternative to hipGraph replay.
//
// On MI355X a one-kernel hipGraphLaunch costs ~7.6 us of queue time before its kernel starts,
// against ~0.75 us between two plain kernel launches on the same stream
// (tools/probe/queue_hop_probe.hip, profiles/NOTES.md). The scorer's three stages are two or
// three kernels each, so replaying them as graphs spent ~20 us of device time per batch on graph
// launches. In record mode the launch bindings (bindings.hip) store each launch as a closure
// over its frozen argument struct - the same freezing a graph capture does - and the driver
// issues the list with plain launches on the stage's stream.
#pragma once
#include <hip/hip_runtime.h>

#include <functional>
#include <memory>
#include <vector>

namespace igp {

struct OpList {
  std::vector<std::function<void(hipStream_t)>> ops;
  void run(hipStream_t st) const {
    for (const auto& f : ops) f(st);
  }
};

// non-null while a body is being recorded on this thread (bindings.hip record_begin / _end)
OpList*& recording();

}  // namespace igp

// A statistical CPU profiler for the host runtime (no perf / gdb in the images this runs in):
// setitimer(ITIMER_PROF) delivers SIGPROF to the thread that burned the CPU, the handler records
// the interrupted instruction pointer and the thread id into a lock-free ring. tools/host_profile.py
// symbolises the samples from /proc/self/maps and the shared objects' symbol tables. Async-signal
// safe: the handler only does an atomic increment and two stores.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace igp {
namespace sampler {

struct Sample {
  uint64_t pc;
  int32_t tid;
  int32_t pad;
};

// start sampling at `hz` samples per CPU-second of the process (ring of `capacity` samples)
void start(int hz, size_t capacity);
// stop, and return the samples taken (oldest first; the ring keeps the last `capacity`)
std::vector<Sample> stop();

}  // namespace sampler
}  // namespace igp

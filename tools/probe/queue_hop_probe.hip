// Cost of the pipeline's cross-queue hand-offs on MI355X (the scorer's copy -> state -> model
// event links): build with
//   hipcc --offload-arch=gfx950 -O2 -o tools/probe/queue_hop_probe tools/probe/queue_hop_probe.hip
// and run with GPU_MAX_HW_QUEUES=8 (every stream its own hardware queue). Each test enqueues the
// whole sequence behind a 40 ms blocker kernel (so the host's enqueue cost is hidden and only
// device-side time is measured) and times it with host wall clock around one final synchronize:
//   same   : N tiny kernels back to back on one stream
//   hop    : N kernels alternating between two streams, each waiting the other's last event
//   waited : N kernels on stream B, each behind a wait on an event that completed long ago
//   graphs : N one-kernel graph launches back to back on one stream
// The tiny kernel is one wave that spins ~2 us on the 100 MHz clock (bounded, no memory).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                           \
    }                                                                                         \
  } while (0)

__global__ void __launch_bounds__(64) tick(int64_t ticks) {
  const int64_t t0 = wall_clock64();
  for (int i = 0; i < (1 << 26); ++i) {  // bounded: at most a few seconds
    if (wall_clock64() - t0 >= ticks) break;
    __builtin_amdgcn_s_sleep(1);
  }
}

using clk = std::chrono::steady_clock;

static double run(const char* name, int n, hipStream_t a, hipStream_t b, int mode, hipGraphExec_t g) {
  hipEvent_t ea, eb, done;
  CK(hipEventCreateWithFlags(&ea, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&eb, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
  CK(hipDeviceSynchronize());
  const int64_t block_ticks = 4000000;  // 40 ms: the queue fills while this runs
  const auto t0 = clk::now();
  hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, a, block_ticks);
  if (mode == 2) {
    CK(hipEventRecord(eb, a));
    CK(hipStreamWaitEvent(b, eb, 0));  // B's steps also start behind the blocker
    CK(hipEventRecord(ea, b));         // ... and wait an event that is complete by then
    hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, b, 10);
  }
  for (int i = 0; i < n; ++i) {
    if (mode == 0) {
      hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, a, 200);
    } else if (mode == 1) {
      hipStream_t s = (i & 1) ? b : a;
      hipEvent_t wait_on = (i & 1) ? ea : eb, rec = (i & 1) ? eb : ea;
      if (i > 0) CK(hipStreamWaitEvent(s, wait_on, 0));
      hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, s, 200);
      CK(hipEventRecord(rec, s));
    } else if (mode == 2) {
      CK(hipStreamWaitEvent(b, ea, 0));
      hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, b, 200);
    } else {
      CK(hipGraphLaunch(g, a));
    }
  }
  const auto t_enq = clk::now();
  CK(hipDeviceSynchronize());
  const double us = std::chrono::duration<double, std::micro>(clk::now() - t0).count() - block_ticks / 100.0;
  const double host_us = std::chrono::duration<double, std::micro>(t_enq - t0).count();
  std::printf("%-8s n=%d  %.2f us per step on the device (host enqueue %.2f us per step%s)\n", name, n, us / n,
              host_us / n, host_us > block_ticks / 100.0 ? ", EXCEEDS the blocker: host-bound" : "");
  CK(hipEventDestroy(ea));
  CK(hipEventDestroy(eb));
  CK(hipEventDestroy(done));
  return us / n;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 400;
  if (n < 1 || n > 100000) return 2;
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  // one-kernel graph
  hipGraph_t graph;
  hipGraphExec_t exec;
  CK(hipStreamBeginCapture(a, hipStreamCaptureModeThreadLocal));
  hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, a, 200);
  CK(hipStreamEndCapture(a, &graph));
  CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  for (int rep = 0; rep < 2; ++rep) {  // first pass warms up
    run("same", n, a, b, 0, exec);
    run("hop", n, a, b, 1, exec);
    run("waited", n, a, b, 2, exec);
    run("graphs", n, a, b, 3, exec);
  }
  CK(hipGraphExecDestroy(exec));
  CK(hipGraphDestroy(graph));
  CK(hipStreamDestroy(a));
  CK(hipStreamDestroy(b));
  return 0;
}

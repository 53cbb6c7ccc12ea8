// Native gRPC (HTTP/2) server for risk.v1 (VERDICT r2 "high-rate unary ScoreTransaction": the
// Python grpc.aio server saturated near 9 k unary calls/s, its own per-call cost).
//
// HTTP/2 framing and HPACK come from libnghttp2 (the image ships the shared library, not its
// headers: the few entry points are declared in h2grpc.cpp and resolved with dlopen). Per
// worker thread: its own SO_REUSEPORT listener on the shared port (the kernel spreads the
// connections), one epoll loop, the nghttp2 sessions of its connections and an eventfd that
// completions wake it with. Per call:
//
//   ScoreTransaction  the request payload goes straight to ServeCore::submit_tx (C++ parse,
//                     AccountIndex, micro-batch FIFO); the core's finisher hands the response
//                     back through its sink to the owning worker - no Python, no GIL
//   ScoreBatch        a batch thread runs ServeCore::score_batch_view and posts the bytes
//   PredictLTV / GetPlayerSegment / CheckBonusAbuse
//                     straight to the rank's AcctRouter (acct_core.h: owner-routed, micro-batched
//                     on the owner's model device, response bytes written in C++) - no Python
//   anything else     a cold thread calls the Python handler table (bytes in, bytes out,
//                     grpc status + message on error) with the GIL
//
// A hot call the native path could not serve (a device error or deadline inside the serving
// core, not a malformed request) is retried once through the cold handler table with the path
// suffixed "#retry:<error>": the engine then marks the shard unhealthy and answers from its
// fallback, and the watcher (api/native_grpc.py) turns the hot flag off.
//
// Responses are standard gRPC: HEADERS (:status 200, application/grpc), one length-prefixed
// DATA message, trailers with grpc-status; errors are Trailers-Only.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "acct_core.h"
#include "serve_core.h"

namespace igp {

struct GrpcReply {
  int32_t status = 0;    // grpc status code (0 OK)
  std::string body;      // serialized response message (status 0)
  std::string message;   // grpc-message (status != 0)
};

class GrpcServer {
 public:
  using ColdFn = std::function<GrpcReply(const std::string& path, std::string body)>;
  GrpcServer(std::shared_ptr<ServeCore> core, ColdFn cold, int cold_threads, int batch_threads,
             std::shared_ptr<AcctRouter> router = nullptr);
  ~GrpcServer();
  // bind `workers` listeners on host:port (0: any free port); returns the bound port
  int start(const std::string& host, int port, int workers);
  void stop();
  // hot RPCs through the serving core (false: through the cold handler table, e.g. while the
  // engine serves from its degraded-shard fallback or with fault injection active)
  void set_hot(bool on) { hot_.store(on, std::memory_order_relaxed); }
  struct Stats {
    int64_t calls, hot_tx, hot_batch, cold, errors, connections, hot_acct, hot_failures;
  };
  // the message of the latest hot-path failure (empty: none yet)
  std::string last_failure() const;
  // limits of one HTTP/2 connection: concurrent streams, request bytes buffered over its streams
  static constexpr uint32_t kMaxStreams = 1024;
  static constexpr size_t kMaxConnBuffered = size_t(256) << 20;
  Stats stats() const;

  struct Worker;

 private:
  friend struct Worker;
  void post(int worker, uint64_t conn_id, int32_t stream_id, GrpcReply&& r);
  void cold_loop();
  void batch_loop();
  void note_failure(const std::string& msg);
  void route_done(std::vector<ServeCore::Done>&& outs);

  std::shared_ptr<ServeCore> core_;
  std::shared_ptr<AcctRouter> router_;
  // completion hand-off from the cores' finisher threads: a sink call holds the gate shared,
  // stop() takes it exclusively once, so no sink call runs into a stopped / destroyed server
  struct SinkGate {
    std::shared_mutex mu;
    GrpcServer* srv = nullptr;
  };
  std::shared_ptr<SinkGate> gate_;
  mutable std::mutex fail_mu_;
  std::string last_failure_;
  ColdFn cold_;
  std::vector<std::unique_ptr<Worker>> workers_;
  std::vector<std::thread> threads_;
  struct Job {
    int worker;
    uint64_t conn;
    int32_t stream;
    std::string path;
    std::string body;
  };
  std::mutex jmu_;
  std::condition_variable jcv_;
  std::deque<Job> cold_q_, batch_q_;
  bool jstop_ = false;
  int n_cold_, n_batch_;
  std::atomic<bool> hot_{true};
  std::atomic<bool> running_{false};
  mutable std::atomic<int64_t> calls_{0}, hot_tx_{0}, hot_batch_{0}, cold_n_{0}, errors_{0}, conns_{0};
  mutable std::atomic<int64_t> hot_acct_{0}, hot_fail_{0};
};

// open-loop unary gRPC load generator (tools/bench_e2e.py --client native)
struct LoadResult {
  std::vector<double> latency_ms;  // per answered call, from its scheduled send time
  std::vector<double> sched_ms;    // that call's scheduled send time, from the schedule start
  int64_t errors = 0, sent = 0;
  double seconds = 0;
  double elapsed = 0;  // schedule start -> last completion (>= seconds)
};
LoadResult grpc_load(const std::string& host, int port, const std::string& path, const std::vector<std::string>& payloads,
                     double rate, double seconds, int conns, int max_inflight);

}  // namespace igp

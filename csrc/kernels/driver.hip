// Native micro-batch driver for the three-stream scoring pipeline (engine/scorer.py).
//
// Per batch the scorer replays three captured hipGraphs on three streams linked by events:
//   copy   : wait model_ev[slot] (slot buffers free), wait state_ev[batch-2] (its K1 cleared this
//            batch's dedup region) -> graph(copy)  -> record copy_ev[slot]
//   state  : wait copy_ev[slot]  -> graph(state) -> record state_ev[slot]
//   model  : wait state_ev[slot] -> graph(model) -> record model_ev[slot]
// Issued from Python this costs ~110 us of host time per batch (stream contexts, torch event
// objects, replay bookkeeping) while the GPU needs ~60 us, so the host bounded throughput
// (rocprofv3 timeline: GPU 58 % busy). The driver issues the same sequence with raw HIP calls
// on the graphs' exec handles, writes the batch header and copies the packed request rows
// into the pinned slab itself, all with the GIL released. (An asynchronous issue thread and a
// one-stream serial mode were measured slower and removed in round 5: profiles/NOTES.md.)
#include "hostwait.h"
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <dlfcn.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../include/device_ops.h"
#include "../include/records.h"
#include "launch.h"
#include "oplist.h"
#include "roctx.h"
#include "state_clock.h"

namespace py = pybind11;

namespace igp {
namespace {

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("PipeDriver ") + what + ": " + hipGetErrorString(e));
}

void copy_err(char* err, int32_t errlen, const char* msg) {
  if (!err || errlen <= 0) return;
  std::strncpy(err, msg, size_t(errlen) - 1);
  err[errlen - 1] = 0;
}

// the serving core calls a device's function table from threads of its own: the first call
// on a thread makes the driver's device current there (streams / events / graphs of device d)
void bind_device(int d) {
  thread_local int cur = -1;
  if (cur != d) {
    hip_ok(hipSetDevice(d), "set device");
    cur = d;
  }
}

// event wait with a deadline (hipEventSynchronize has none): query with a short back-off
bool poll_event(hipEvent_t e, int64_t timeout_us) {
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::microseconds(timeout_us);
  return poll_event_until(e, t_end, [](hipError_t q) { hip_ok(q, "event query"); });
}

class PipeDriver {
 public:
  PipeDriver(uintptr_t cstream, uintptr_t sstream, uintptr_t mstream, int depth, py::list host_slabs)
      : cs_(reinterpret_cast<hipStream_t>(cstream)),
        ss_(reinterpret_cast<hipStream_t>(sstream)),
        ms_(reinterpret_cast<hipStream_t>(mstream)),
        depth_(depth) {
    if (depth < 1 || (int)host_slabs.size() != depth) throw std::runtime_error("PipeDriver: one host slab per slot");
    for (auto h : host_slabs) slabs_.push_back(reinterpret_cast<char*>(h.cast<uintptr_t>()));
    // the copy / state / post-state events only order work between this device's queues: no
    // system-scope fence (cache writeback + invalidate at the stage's end, which also slows the
    // kernels running beside it); the model event keeps it (the host reads results from pinned
    // memory after it).
    const unsigned dev_flags = hipEventDisableTiming | (unsigned)hipEventDisableSystemFence;
    hip_ok(hipGetDevice(&device_), "get device");  // the serving core's threads bind to it
    ev_.resize(3 * depth);
    for (size_t i = 0; i < ev_.size(); ++i)
      hip_ok(hipEventCreateWithFlags(&ev_[i], i % 3 == 2 ? hipEventDisableTiming : dev_flags), "event create");
    if (depth > DEDUP_AHEAD)  // batch q's dedup region was cleared by batch q - DEDUP_AHEAD's update
      throw std::runtime_error("PipeDriver: depth exceeds the dedup ring (DEDUP_AHEAD)");
    for (auto& e : pe_) hip_ok(hipEventCreateWithFlags(&e, dev_flags), "event create");
    pe_seq_.fill(-1);
    slot_seq_.assign(depth, -1);
    recorded_.assign(3 * depth, false);
    host_done_.assign(depth, 0);
    const char* xe = getenv("IGP_EXT_EVENTS");
    ext_events_ = !(xe && atoi(xe) == 0);
  }
  ~PipeDriver() {
    if (clock_) {  // the shard's clock may still hold one of these events
      clock_->retract(ev_.data(), ev_.size());
      clock_->retract(pe_.data(), pe_.size());
    }
    for (auto& e : ev_) (void)hipEventDestroy(e);
    for (auto& e : pe_) (void)hipEventDestroy(e);
  }

  // stage-end events bound to the stages' last kernels (oplist.h) instead of recorded markers
  void set_ext_events(bool on) { ext_events_ = on; }
  bool ext_events() const { return ext_events_; }

  // the slot's pinned result rows (ResultRec [bucket]) and FeatRec rows: what the native
  // serving core reads after wait (device_ops)
  void set_host_results(int slot, uintptr_t res, uintptr_t feat) {
    if (slot < 0 || slot >= depth_) throw std::runtime_error("PipeDriver: bad slot");
    if ((int)host_res_.size() != depth_) {
      host_res_.assign(depth_, nullptr);
      host_feat_.assign(depth_, nullptr);
    }
    host_res_[slot] = reinterpret_cast<char*>(res);
    host_feat_[slot] = reinterpret_cast<char*>(feat);
  }

  // C function table for the native serving core (csrc/include/device_ops.h): the core issues
  // this pipeline's batches from its own threads (no Python, no GIL)
  uintptr_t device_ops() {
    if ((int)host_res_.size() != depth_) throw std::runtime_error("PipeDriver: set_host_results first");
    if (graphs_.empty()) throw std::runtime_error("PipeDriver: no graphs / op lists");
    buckets_.clear();
    for (auto& kv : graphs_) {
      const int b = int(kv.first >> 8);
      if (std::find(buckets_.begin(), buckets_.end(), b) == buckets_.end()) buckets_.push_back(b);
    }
    std::sort(buckets_.begin(), buckets_.end());
    ops_.abi = IGP_DEVICE_OPS_ABI;
    ops_.depth = depth_;
    ops_.world = 1;
    ops_.exchange = 0;
    ops_.cap = buckets_.back();
    ops_.features_always = 0;
    ops_.ctx = this;
    ops_.rows = [](void* ctx, int32_t slot) -> char* {
      return static_cast<PipeDriver*>(ctx)->slabs_[slot] + sizeof(BatchHdr);
    };
    ops_.submit = [](void* ctx, int32_t slot, int32_t n, int32_t seq, int64_t now, int32_t wf, char* err,
                     int32_t errlen) -> int32_t {
      auto* d = static_cast<PipeDriver*>(ctx);
      try {
        bind_device(d->device_);
        int bucket = -1;
        for (int b : d->buckets_)
          if (b >= (n > 0 ? n : 1)) { bucket = b; break; }
        if (bucket < 0) throw std::runtime_error("batch exceeds the largest bucket");
        auto it = d->graphs_.find(key(bucket, slot));
        if (it == d->graphs_.end()) throw std::runtime_error("no graphs for this bucket / slot");
        d->issue(Cmd{slot, bucket, n, seq, now, 0, wf != 0, it->second});
      } catch (const std::exception& e) {
        copy_err(err, errlen, e.what());
        return -1;
      }
      return 0;
    };
    ops_.wait = [](void* ctx, int32_t slot, int64_t timeout_us, char* err, int32_t errlen) -> int32_t {
      auto* d = static_cast<PipeDriver*>(ctx);
      try {
        bind_device(d->device_);
        hipEvent_t e = d->ev_[3 * slot + 2];
        if (timeout_us < 0) {
          hip_ok(hipEventSynchronize(e), "sync model");
        } else if (!poll_event(e, timeout_us)) {
          return 1;
        }
        d->host_done_[slot] = 1;
      } catch (const std::exception& e) {
        copy_err(err, errlen, e.what());
        return -1;
      }
      return 0;
    };
    ops_.results = [](void* ctx, int32_t slot) -> const void* { return static_cast<PipeDriver*>(ctx)->host_res_[slot]; };
    ops_.features = [](void* ctx, int32_t slot) -> const void* {
      return static_cast<PipeDriver*>(ctx)->host_feat_[slot];
    };
    return reinterpret_cast<uintptr_t>(&ops_);
  }

  void set_graphs(int bucket, int slot, uintptr_t gc, uintptr_t gs, uintptr_t gm, uintptr_t gmf) {
    if (slot < 0 || slot >= depth_) throw std::runtime_error("PipeDriver: bad slot");
    Graphs& g = graphs_[key(bucket, slot)];
    g.c = reinterpret_cast<hipGraphExec_t>(gc);
    g.s = reinterpret_cast<hipGraphExec_t>(gs);
    g.m = reinterpret_cast<hipGraphExec_t>(gm);
    g.mf = reinterpret_cast<hipGraphExec_t>(gmf);
  }
  // direct-launch mode: the stages' recorded launches (oplist.h) replace the graph replays
  void set_ops(int bucket, int slot, std::shared_ptr<OpList> c, std::shared_ptr<OpList> s,
               std::shared_ptr<OpList> m, std::shared_ptr<OpList> mf) {
    if (slot < 0 || slot >= depth_) throw std::runtime_error("PipeDriver: bad slot");
    if (!c || !s || !m || !mf) throw std::runtime_error("PipeDriver: set_ops needs four op lists");
    Graphs& g = graphs_[key(bucket, slot)];
    g.oc = std::move(c);
    g.os = std::move(s);
    g.om = std::move(m);
    g.omf = std::move(mf);
  }
  // readers of the feature store order themselves after the last published state stage
  void set_state_clock(std::shared_ptr<StateClock> c) { clock_ = std::move(c); }
  // direct launch with a split state stage: `s` of set_ops holds K1 only, `su` the update
  void set_state_update(int bucket, int slot, std::shared_ptr<OpList> su) {
    if (slot < 0 || slot >= depth_) throw std::runtime_error("PipeDriver: bad slot");
    graphs_[key(bucket, slot)].osu = std::move(su);
  }

  // rows: pointer to n packed ReqRec (0: already in the slab); the batch is tracked by its slot
  // (wait(slot)). Slot reuse is ordered on the device (the copy waits for the slot's previous
  // model graph); the caller must not repack a slot's pinned slab before wait(slot) of its
  // previous batch returned.
  void submit(int slot, int bucket, int n, int seq, int64_t now, uintptr_t rows, bool with_features) {
    if (slot < 0 || slot >= depth_) throw std::runtime_error("PipeDriver: bad slot");
    auto it = graphs_.find(key(bucket, slot));
    if (it == graphs_.end()) throw std::runtime_error("PipeDriver: no graphs for this bucket/slot");
    const Cmd c{slot, bucket, n, seq, now, rows, with_features, it->second};
    py::gil_scoped_release nogil;
    issue(c);
  }

 private:
  struct Graphs {
    hipGraphExec_t c = nullptr, s = nullptr, m = nullptr, mf = nullptr;  // mf: + FeatRec rows to the host
    std::shared_ptr<OpList> oc, os, om, omf;  // direct-launch mode (set_ops)
    std::shared_ptr<OpList> osu;              // split state stage: the update after K1
  };
  static void stage(hipGraphExec_t g, const std::shared_ptr<OpList>& ops, hipStream_t st, const char* what) {
    if (ops) ops->run(st);
    else hip_ok(hipGraphLaunch(g, st), what);
  }
  // stage with its end event bound to its last kernel (oplist.h run_recording); false: the
  // caller records ev (graph replay, IGP_EXT_EVENTS=0, or a stage ending in a copy)
  bool stage_rec(hipGraphExec_t g, const std::shared_ptr<OpList>& ops, hipStream_t st, hipEvent_t ev,
                 const char* what) const {
    if (ops && ext_events_) return ops->run_recording(st, ev);
    stage(g, ops, st, what);
    return false;
  }
  struct Cmd {
    int slot, bucket, n, seq;
    int64_t now;
    uintptr_t rows;
    bool with_features;
    Graphs g;
  };

  void issue(const Cmd& cmd) {
    const int slot = cmd.slot, n = cmd.n, seq = cmd.seq;
    const int64_t now = cmd.now;
    const uintptr_t rows = cmd.rows;
    const bool with_features = cmd.with_features;
    const Graphs g = cmd.g;
    Range range("igp.submit");
    const auto t0 = clk::now();
    char* slab = slabs_[slot];
    if (rows) std::memcpy(slab + sizeof(BatchHdr), reinterpret_cast<const void*>(rows), (size_t)n * sizeof(ReqRec));
    const auto t1 = clk::now();
    BatchHdr* h = reinterpret_cast<BatchHdr*>(slab);
    h->n = n;
    h->seq = seq;
    h->now = now;
    hipEvent_t ce = ev_[3 * slot], se = ev_[3 * slot + 1], me = ev_[3 * slot + 2];
    const int prev_seq = slot_seq_[slot];
    hipEvent_t pe = pe_[ring(seq)];
    pe_seq_[ring(seq)] = seq;
    slot_seq_[slot] = seq;
    // the slot's previous batch: skipped when the host already saw it complete (wait(slot))
    if (recorded_[3 * slot + 2] && !host_done_[slot]) hip_ok(hipStreamWaitEvent(cs_, me, 0), "wait model");
    host_done_[slot] = 0;
    // the slot's previous batch's split update stage (state stream, after K1) also reads the
    // slot's device header and rows: the model event above does not cover it (the model only
    // waited for K1). An event query first: no queue wait when it already finished.
    if (hipEvent_t e = post_event(prev_seq); e && hipEventQuery(e) != hipSuccess)
      hip_ok(hipStreamWaitEvent(cs_, e, 0), "wait slot update");
    // the state stage of batch seq - DEDUP_AHEAD cleared this batch's dedup region (the post
    // events are kept per batch in a ring of DEDUP_RING, so this is exact at any depth <= AHEAD)
    if (hipEvent_t e = post_event(seq - DEDUP_AHEAD); e && hipEventQuery(e) != hipSuccess)
      hip_ok(hipStreamWaitEvent(cs_, e, 0), "wait state-ahead");
    const auto t2 = clk::now();
    const bool cb = stage_rec(g.c, g.oc, cs_, ce, "copy graph");
    const auto t3 = clk::now();
    if (!cb) hip_ok(hipEventRecord(ce, cs_), "record copy");
    hip_ok(hipStreamWaitEvent(ss_, ce, 0), "wait copy");
    const auto t4 = clk::now();
    const bool sb = stage_rec(g.s, g.os, ss_, se, "state graph");
    const auto t5 = clk::now();
    if (!sb) hip_ok(hipEventRecord(se, ss_), "record state");
    hip_ok(hipStreamWaitEvent(ms_, se, 0), "wait state");
    // split state stage (direct launch): the model waited for K1 only; the multi-event update
    // (which also clears the dedup region of batch seq+3) follows on the state stream and its
    // own event gates that region's reuse
    const bool pb = g.osu && ext_events_ && g.osu->run_recording(ss_, pe);
    if (g.osu && !ext_events_) g.osu->run(ss_);
    if (!pb) hip_ok(hipEventRecord(pe, ss_), "record post");
    if (clock_) clock_->publish(pe);  // K1 + the multi-event update of this batch
    const auto t6 = clk::now();
    const bool mb = stage_rec(with_features ? g.mf : g.m, with_features ? g.omf : g.om, ms_, me, "model graph");
    const auto t7 = clk::now();
    if (!mb) hip_ok(hipEventRecord(me, ms_), "record model");
    const auto t8 = clk::now();
    auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    st_[0] += us(t0, t1);                          // row copy
    st_[1] += us(t1, t2) + us(t3, t4) + us(t5, t6) + us(t7, t8);  // event waits / records
    st_[2] += us(t2, t3);                          // copy graph launch
    st_[3] += us(t4, t5);                          // state graph launch
    st_[4] += us(t6, t7);                          // model graph launch
    st_[5] += 1;
    recorded_[3 * slot] = recorded_[3 * slot + 1] = recorded_[3 * slot + 2] = true;
  }
  static int ring(int seq) { return (int)((unsigned)seq % DEDUP_RING); }
  // the post-state event of batch `seq` if this driver issued it (and the ring still holds it)
  hipEvent_t post_event(int seq) const {
    if (seq < 0) return nullptr;
    return pe_seq_[ring(seq)] == seq ? pe_[ring(seq)] : nullptr;
  }

 public:
  void wait(int slot) {
    if (slot < 0 || slot >= depth_) throw std::runtime_error("PipeDriver: bad slot");
    py::gil_scoped_release nogil;
    Range range("igp.wait");
    const auto t0 = clk::now();
    hip_ok(hipEventSynchronize(ev_[3 * slot + 2]), "sync model");
    host_done_[slot] = 1;
    st_[6] += std::chrono::duration<double, std::micro>(clk::now() - t0).count();
  }

  // host time per submit (us): rows copy, event ops, copy / state / model graph launch, and
  // the total blocked in wait(); reset after reading
  py::dict stats() {
    py::dict d;
    const double n = st_[5] > 0 ? st_[5] : 1;
    d["submits"] = st_[5];
    d["rows_copy_us"] = st_[0] / n;
    d["event_ops_us"] = st_[1] / n;
    d["copy_launch_us"] = st_[2] / n;
    d["state_launch_us"] = st_[3] / n;
    d["model_launch_us"] = st_[4] / n;
    d["wait_us"] = st_[6] / n;
    for (double& v : st_) v = 0;
    return d;
  }

  bool query(int slot) {
    return hipEventQuery(ev_[3 * slot + 2]) == hipSuccess;
  }

  // the slot's model-stream event (completes with its batch)
  uintptr_t model_event(int slot) {
    return reinterpret_cast<uintptr_t>(ev_[3 * slot + 2]);
  }

 private:
  using clk = std::chrono::steady_clock;
  double st_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  static int64_t key(int bucket, int slot) { return ((int64_t)bucket << 8) | slot; }
  hipStream_t cs_, ss_, ms_;
  int depth_;
  std::vector<char*> slabs_;
  std::vector<hipEvent_t> ev_;
  // per batch (ring of DEDUP_RING by seq): the state stream's work of the batch is complete
  std::array<hipEvent_t, DEDUP_RING> pe_{};
  std::array<int, DEDUP_RING> pe_seq_{};  // the batch each ring event was last recorded for
  std::vector<int> slot_seq_;             // the slot's last batch
  std::vector<bool> recorded_;
  std::vector<uint8_t> host_done_;  // wait(slot) returned since the slot's last submit (bytes: set by waiter threads)
  std::shared_ptr<StateClock> clock_;
  std::unordered_map<int64_t, Graphs> graphs_;
  bool ext_events_ = true;
  // native serving core interface
  std::vector<char*> host_res_, host_feat_;
  std::vector<int> buckets_;
  IgpDeviceOps ops_{};
  int device_ = 0;
};

}  // namespace

void register_driver(py::module_& m) {
  py::class_<StateClock, std::shared_ptr<StateClock>>(m, "StateClock")
      .def(py::init<>())
      .def("wait", [](StateClock& c, uintptr_t stream) { c.wait(reinterpret_cast<hipStream_t>(stream)); },
           py::arg("stream"))
      .def_property_readonly("published", &StateClock::published)
      .def_property_readonly("waits", &StateClock::waits)
      .def_property_readonly("skips", &StateClock::skips)
      .def_property_readonly("retracts", &StateClock::retracts);
  py::class_<PipeDriver>(m, "PipeDriver")
      .def("set_state_clock", &PipeDriver::set_state_clock)
      .def(py::init<uintptr_t, uintptr_t, uintptr_t, int, py::list>())
      .def("set_graphs", &PipeDriver::set_graphs)
      .def("set_host_results", &PipeDriver::set_host_results)
      .def("device_ops", &PipeDriver::device_ops)
      .def("set_ops", &PipeDriver::set_ops)
      .def("set_state_update", &PipeDriver::set_state_update)
      .def("set_ext_events", &PipeDriver::set_ext_events)
      .def_property_readonly("ext_events", &PipeDriver::ext_events)
      .def("submit", &PipeDriver::submit)
      .def("wait", &PipeDriver::wait)
      .def("query", &PipeDriver::query)
      .def("model_event", &PipeDriver::model_event)
      .def("stats", &PipeDriver::stats);
}

}  // namespace igp

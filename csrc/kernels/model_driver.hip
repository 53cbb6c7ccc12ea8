// Native driver of the per-account model steps behind the account-RPC core (model_ops.h;
// host side csrc/runtime/acct_core.cpp): PredictLTV / GetPlayerSegment on the LTV chain and
// CheckBonusAbuse on the abuse step, issued from the core's own threads without Python.
//
// Per pipeline slot one pinned host slab, laid out
//     [BatchHdr 16 B | int32 slots [cap] | ReqRec [cap] (abuse only)]
// the core writes the slots, submit() writes the header (live rows, clock) - and for the abuse
// step one synthetic ReqRec per row (slot, TX_UNKNOWN, the clock: K1 then computes the account's
// live feature row without updating the store) - and issues the slot's recorded launches
// (oplist.h) or its captured graph for the smallest bucket >= n on the driver's stream:
//   LTV    one fused kernel (mlp_fused.hip): gathers the profile / ext rows of the slots it
//          reads from the pinned slab, runs the MLP 4x512 on MFMA and K9 in the epilogue, and
//          stores each row's 6 outputs straight into the slot's pinned output rows
//   abuse  H2D of the live rows -> K1 (features.hip, FeatRec images stored into pinned host
//          rows) -> K4 GRU over the HBM event rings (gru.hip / gru_ws.hip) -> score D2H
// Completion: one event per slot, polled by the core's completion thread with the deadline.
// Streams: one per slot (or one shared): the account-RPC micro-batches are small (a few hundred
// rows fill a few dozen CUs), so consecutive slots' steps run side by side on the chip instead of
// queueing behind each other on one stream.
#include "hostwait.h"
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../include/model_ops.h"
#include "../include/records.h"
#include "oplist.h"
#include "state_clock.h"

namespace py = pybind11;

namespace igp {
namespace {

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("ModelDriver ") + what + ": " + hipGetErrorString(e));
}

void copy_err(char* err, int32_t errlen, const char* msg) {
  if (!err || errlen <= 0) return;
  std::strncpy(err, msg, size_t(errlen) - 1);
  err[errlen - 1] = 0;
}

void bind_device(int d) {
  thread_local int cur = -1;
  if (cur != d) {
    hip_ok(hipSetDevice(d), "set device");
    cur = d;
  }
}

class ModelDriver {
 public:
  ModelDriver(py::list streams, int kind, int depth, int cap, int has_model, int rank, py::list slabs, py::list out0,
              py::list out1)
      : depth_(depth), cap_(cap), rank_(rank) {
    for (auto s : streams) st_.push_back(reinterpret_cast<hipStream_t>(s.cast<uintptr_t>()));
    if (st_.empty() || (st_.size() != 1 && (int)st_.size() != depth)) throw std::runtime_error("ModelDriver: one stream or one per slot");
    if (kind != IGP_MODEL_LTV && kind != IGP_MODEL_ABUSE) throw std::runtime_error("ModelDriver: kind");
    if (depth < 1 || cap < 1 || (int)slabs.size() != depth || (int)out0.size() != depth)
      throw std::runtime_error("ModelDriver: one slab / output per slot");
    if (kind == IGP_MODEL_ABUSE && (int)out1.size() != depth) throw std::runtime_error("ModelDriver: abuse needs out1");
    for (int s = 0; s < depth; ++s) {
      slabs_.push_back(reinterpret_cast<char*>(slabs[s].cast<uintptr_t>()));
      o0_.push_back(reinterpret_cast<void*>(out0[s].cast<uintptr_t>()));
      o1_.push_back(kind == IGP_MODEL_ABUSE ? reinterpret_cast<void*>(out1[s].cast<uintptr_t>()) : nullptr);
    }
    hip_ok(hipGetDevice(&device_), "get device");
    last_n_.assign(depth, 0);
    last_key_.assign(depth, -1);
    ev_.resize(depth);
    for (auto& e : ev_) hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event create");
    ops_.abi = IGP_MODEL_OPS_ABI;
    ops_.kind = kind;
    ops_.depth = depth;
    ops_.cap = cap;
    ops_.has_model = has_model;
    ops_.ctx = this;
    ops_.slots = [](void* ctx, int32_t slot) -> int32_t* {
      return reinterpret_cast<int32_t*>(static_cast<ModelDriver*>(ctx)->slabs_[slot] + sizeof(BatchHdr));
    };
    ops_.submit = [](void* ctx, int32_t slot, int32_t n, int64_t now, char* err, int32_t errlen) -> int32_t {
      auto* d = static_cast<ModelDriver*>(ctx);
      try {
        d->submit(slot, n, now);
      } catch (const std::exception& e) {
        copy_err(err, errlen, e.what());
        return -1;
      }
      return 0;
    };
    ops_.wait = [](void* ctx, int32_t slot, int64_t timeout_us, char* err, int32_t errlen) -> int32_t {
      auto* d = static_cast<ModelDriver*>(ctx);
      try {
        bind_device(d->device_);
        hipEvent_t e = d->ev_[slot];
        if (timeout_us < 0) {
          hip_ok(hipEventSynchronize(e), "sync");
        } else {
          const auto t_end = std::chrono::steady_clock::now() + std::chrono::microseconds(timeout_us);
          if (!poll_event_until(e, t_end, [](hipError_t q) { hip_ok(q, "event query"); })) return 1;
        }
        d->check_fallback(slot);
      } catch (const std::exception& e) {
        copy_err(err, errlen, e.what());
        return -1;
      }
      return 0;
    };
    ops_.out0 = [](void* ctx, int32_t slot) -> const void* { return static_cast<ModelDriver*>(ctx)->o0_[slot]; };
    ops_.out1 = [](void* ctx, int32_t slot) -> const void* { return static_cast<ModelDriver*>(ctx)->o1_[slot]; };
  }
  ~ModelDriver() {
    for (auto& e : ev_) (void)hipEventDestroy(e);
  }

  void set_ops(int bucket, int slot, std::shared_ptr<OpList> ops) {
    check(bucket, slot);
    steps_[key(bucket, slot)].ops = std::move(ops);
  }
  void set_graph(int bucket, int slot, uintptr_t exec) {
    check(bucket, slot);
    steps_[key(bucket, slot)].graph = reinterpret_cast<hipGraphExec_t>(exec);
  }
  // the same step without the weight-stationary GRU clusters (gru_wsx.hip): a cluster that
  // could not become co-resident gives up after a bounded wait and leaves NaN scores; wait()
  // then re-runs the slot's step on this body and every later step uses it
  void set_alt_graph(int bucket, int slot, uintptr_t exec) {
    check(bucket, slot);
    steps_[key(bucket, slot)].alt = reinterpret_cast<hipGraphExec_t>(exec);
  }
  bool fell_back() const { return fallback_.load(); }
  // small buckets (the weight-stationary GRU clusters, up to half the chip per launch) all run
  // on one extra stream, one launch at a time; larger ones on the slot's own stream
  void set_small_stream(uintptr_t stream, int max_rows) {
    small_st_ = reinterpret_cast<hipStream_t>(stream);
    shared_max_ = max_rows;
  }
  int64_t fallbacks() const { return fallbacks_; }
  uintptr_t model_ops() {
    has_alt_ = false;
    for (auto& kv : steps_) has_alt_ = has_alt_ || kv.second.alt != nullptr;
    buckets_.clear();
    for (auto& kv : steps_) {
      const int b = int(kv.first >> 8);
      if (std::find(buckets_.begin(), buckets_.end(), b) == buckets_.end()) buckets_.push_back(b);
    }
    std::sort(buckets_.begin(), buckets_.end());
    if (buckets_.empty() || buckets_.back() != cap_) throw std::runtime_error("ModelDriver: the largest bucket must be cap");
    for (int b : buckets_)
      for (int s = 0; s < depth_; ++s)
        if (!steps_.count(key(b, s))) throw std::runtime_error("ModelDriver: a bucket lacks a slot's step");
    return reinterpret_cast<uintptr_t>(&ops_);
  }
  int64_t submits() const { return submits_; }
  void set_state_clock(std::shared_ptr<StateClock> c) { clock_ = std::move(c); }

 private:
  struct StepBody {
    std::shared_ptr<OpList> ops;
    hipGraphExec_t graph = nullptr;
    hipGraphExec_t alt = nullptr;
  };
  // completion of an abuse step: NaN scores mean a cluster launch gave up - switch to the
  // alternative bodies and recompute this slot's rows (the step only reads the store)
  void check_fallback(int slot) {
    if (ops_.kind != IGP_MODEL_ABUSE || !has_alt_) return;
    const int n = last_n_[slot];
    const float* o = static_cast<const float*>(o0_[slot]);
    bool nan = false;
    for (int i = 0; i < n && !nan; ++i) nan = o[i] != o[i];
    if (!nan) return;
    fallback_.store(true);
    auto it = steps_.find(last_key_[slot]);
    if (it == steps_.end() || !it->second.alt) throw std::runtime_error("abuse step gave up and has no fallback body");
    hipStream_t st = stream_for(int(last_key_[slot] >> 8), slot);
    hip_ok(hipGraphLaunch(it->second.alt, st), "fallback graph launch");
    hip_ok(hipEventRecord(ev_[slot], st), "record");
    hip_ok(hipEventSynchronize(ev_[slot]), "sync fallback");
    ++fallbacks_;
  }
  static int64_t key(int bucket, int slot) { return (int64_t(bucket) << 8) | slot; }
  void check(int bucket, int slot) const {
    if (slot < 0 || slot >= depth_ || bucket < 1 || bucket > cap_) throw std::runtime_error("ModelDriver: bucket / slot");
  }

  void submit(int slot, int n, int64_t now) {
    bind_device(device_);
    int bucket = -1;
    for (int b : buckets_)
      if (b >= std::max(n, 1)) {
        bucket = b;
        break;
      }
    if (bucket < 0) throw std::runtime_error("batch exceeds the largest bucket");
    auto it = steps_.find(key(bucket, slot));
    if (it == steps_.end()) throw std::runtime_error("no step for this bucket / slot");
    char* slab = slabs_[slot];
    BatchHdr* h = reinterpret_cast<BatchHdr*>(slab);
    h->n = n;
    h->seq = ++seq_;
    h->now = now;
    if (ops_.kind == IGP_MODEL_ABUSE) {
      // one synthetic request per row: K1 reads the account's state at `now`, no update
      const int32_t* sl = reinterpret_cast<const int32_t*>(slab + sizeof(BatchHdr));
      ReqRec* rq = reinterpret_cast<ReqRec*>(slab + sizeof(BatchHdr) + sizeof(int32_t) * size_t(cap_));
      for (int i = 0; i < n; ++i) {
        ReqRec& r = rq[i];
        std::memset(&r, 0, sizeof r);
        r.slot = sl[i];
        r.tx_type = int32_t(TX_UNKNOWN) | (rank_ << 8);
        r.ts = now;
      }
    }
    const StepBody& b = it->second;
    hipStream_t st = stream_for(bucket, slot);
    last_n_[slot] = n;
    last_key_[slot] = key(bucket, slot);
    // the abuse step reads the feature store (K1 rule signals, the GRU event rings): it sees every
    // scoring batch issued before this call (state_clock.h), without a host sync
    if (ops_.kind == IGP_MODEL_ABUSE && clock_) clock_->wait(st);
    if (b.alt && fallback_.load()) {
      hip_ok(hipGraphLaunch(b.alt, st), "graph launch");
      hip_ok(hipEventRecord(ev_[slot], st), "record");
    } else if (b.ops) {
      if (!b.ops->run_recording(st, ev_[slot])) hip_ok(hipEventRecord(ev_[slot], st), "record");
    } else {
      hip_ok(hipGraphLaunch(b.graph, st), "graph launch");
      hip_ok(hipEventRecord(ev_[slot], st), "record");
    }
    ++submits_;
  }

  std::vector<hipStream_t> st_;
  int depth_, cap_, rank_;
  int device_ = 0;
  int32_t seq_ = 0;
  int64_t submits_ = 0;
  std::vector<char*> slabs_;
  std::vector<void*> o0_, o1_;
  std::vector<hipEvent_t> ev_;
  std::map<int64_t, StepBody> steps_;
  std::vector<int> buckets_;
  std::vector<int> last_n_;
  std::vector<int64_t> last_key_;
  bool has_alt_ = false;
  int shared_max_ = 0;  // buckets up to this many rows run on small_st_
  hipStream_t small_st_ = nullptr;
  hipStream_t stream_for(int bucket, int slot) const {
    if (small_st_ && bucket <= shared_max_) return small_st_;
    return st_[st_.size() == 1 ? 0 : slot];
  }
  std::atomic<bool> fallback_{false};
  int64_t fallbacks_ = 0;
  IgpModelOps ops_{};
  std::shared_ptr<StateClock> clock_;
};

}  // namespace

void register_model_driver(py::module_& m) {
  m.attr("MODEL_LTV") = int(IGP_MODEL_LTV);
  m.attr("MODEL_ABUSE") = int(IGP_MODEL_ABUSE);
  py::class_<ModelDriver, std::shared_ptr<ModelDriver>>(m, "ModelDriver")
      .def(py::init<py::list, int, int, int, int, int, py::list, py::list, py::list>(), py::arg("streams"),
           py::arg("kind"), py::arg("depth"), py::arg("cap"), py::arg("has_model"), py::arg("rank"), py::arg("slabs"),
           py::arg("out0"), py::arg("out1"))
      .def("set_ops", &ModelDriver::set_ops)
      .def("set_graph", &ModelDriver::set_graph)
      .def("set_alt_graph", &ModelDriver::set_alt_graph)
      .def("set_small_stream", &ModelDriver::set_small_stream)
      .def_property_readonly("fell_back", &ModelDriver::fell_back)
      .def_property_readonly("fallbacks", [](const ModelDriver& d) { return d.fallbacks(); })
      .def("model_ops", &ModelDriver::model_ops)
      .def("set_state_clock", &ModelDriver::set_state_clock)
      .def_property_readonly("submits", &ModelDriver::submits);
}

}  // namespace igp

// Owner-routed data-parallel exchange (VERDICT r1 "make DP serving actually
// data-parallel"): every rank that ingests requests routes each row to the GPU that owns its
// account, every GPU scores ONLY the rows it owns, and the packed results travel back to the
// ingress rank. Two RCCL all-to-alls per micro-batch, both device-resident:
//
//   ingress host : rows sorted by owner into N chunks of (1 + C) ReqRec; record 0 of chunk o
//                  carries the row count in its `slot` field            (one pinned H2D copy)
//   xs stream    : ncclAllToAll(xsend -> xrecv), (C+1)*48 B per peer
//   copy stream  : exchange_compact: the received chunks -> contiguous scorer rows, BatchHdr.n
//                  = total rows, route[i] = (peer, index) of compact row i; then dedup insert
//   state/model  : the unchanged K1 / update / trees / head / ensemble graphs over n rows
//   model stream : exchange_scatter: ResultRec (+FeatRec) of row i -> rsend[peer][index]
//   ys stream    : ncclAllToAll(rsend -> rrecv), C*W B per peer; rrecv -> pinned host
//
// No host synchronisation and no count read-back in the loop: counts ride in the chunk
// header record, the compact kernel computes the prefix on device, and kernels read the live
// row count from BatchHdr. The chunk capacity C is fixed per captured graph (a batch bucket).
//
// RCCL is the copy torch already loaded (torch/lib/librccl.so.1), resolved with dlopen, so the
// process holds one RCCL whether or not torch.distributed uses it; our communicators are our
// own (ncclCommInitRank over a unique id that Python broadcasts once).
#include "hostwait.h"
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <dlfcn.h>

#include <chrono>
#include <algorithm>
#include <thread>
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
#include "../include/results_region.h"

namespace py = pybind11;

namespace igp {

constexpr int XCHG_MAX_WORLD = 64;

// ------------------------------------------------------------------------------- kernels
struct XchgCompactArgs {
  const ReqRec* recv;  // sender p's chunk at recv + p * pstride: header record (slot = row count) + C rows
  ReqRec* rows;        // scorer slab rows [cap]
  BatchHdr* hdr;       // n written here (seq / now came with the batch header copy)
  int32_t* route;      // [cap + 1]: route[i] = peer * C + index; route[cap] = rows over cap
  int32_t N, C, cap;
  int64_t pstride;     // records between two senders' chunks: C + 1 (all-to-all receive buffer) or
                       // world * (C + 1) (the node-shared rows region: [sender][owner][C + 1])
  const int4* hdr_src; // nullable: the batch header {n, seq, now} in the pinned slab, copied first
};

__global__ __launch_bounds__(256) void exchange_compact_kernel(XchgCompactArgs a) {
  __shared__ int cnt[XCHG_MAX_WORLD];
  __shared__ int pre[XCHG_MAX_WORLD + 1];
  __shared__ int64_t tsp[XCHG_MAX_WORLD];
  if (threadIdx.x < (unsigned)a.N) {
    const ReqRec* h = a.recv + (size_t)threadIdx.x * a.pstride;
    const int c = h->slot;
    cnt[threadIdx.x] = c < 0 ? 0 : (c > a.C ? a.C : c);
    tsp[threadIdx.x] = h->ts;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    int64_t t = 0;
    for (int p = 0; p < a.N; ++p) {
      pre[p] = s;
      s += cnt[p];
      // senders of the serving core stamp their step clock into the chunk header: the step is
      // scored at the latest clock among the senders that sent rows (0: keep the batch header's)
      if (cnt[p] > 0 && tsp[p] > t) t = tsp[p];
    }
    pre[a.N] = s;
    if (blockIdx.x == 0) {
      if (a.hdr_src) *reinterpret_cast<int4*>(a.hdr) = *a.hdr_src;
      a.hdr->n = s < a.cap ? s : a.cap;
      if (t > 0) a.hdr->now = t;
      a.route[a.cap] = s > a.cap ? s - a.cap : 0;
    }
  }
  __syncthreads();
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int p = t / a.C;
  const int j = t - p * a.C;
  if (p >= a.N || j >= cnt[p]) return;
  const int dst = pre[p] + j;
  if (dst >= a.cap) return;
  const int4* src = reinterpret_cast<const int4*>(a.recv + (size_t)p * a.pstride + 1 + j);
  int4* out = reinterpret_cast<int4*>(a.rows + dst);
  int4 q0 = src[0];
  const int4 q1 = src[1], q2 = src[2];
  q0.y &= 0xff | FV_ENC_BIT;  // owner bits of tx_type: this GPU owns every row it receives
  out[0] = q0;
  out[1] = q1;
  out[2] = q2;
  a.route[dst] = p * a.C + j;
}

// Before the row all-to-all: zero the chunk-header row counts of the receive buffer. After an
// abort (a peer died inside the collective, ncclCommAbort) the kernels queued behind the
// all-to-all still run; with the counts cleared they compact zero rows instead of replaying a
// stale chunk of an older batch into the feature store.
// also copies the batch header {n, seq, now} from the pinned host slab to the device slab
// (nullable): one thread of a kernel that runs anyway instead of a 16-byte copy job per step
__global__ __launch_bounds__(64) void exchange_clear_kernel(ReqRec* recv, int32_t N, int32_t C, const int4* hdr_src,
                                                            int4* hdr_dst) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < N) recv[(size_t)p * (C + 1)].slot = 0;
  if (p == 0 && hdr_src) *hdr_dst = *hdr_src;
}

struct XchgScatterArgs {
  const BatchHdr* hdr;
  const int32_t* route;
  const ResultRec* res;  // [cap]
  const FeatRec* feat;   // [cap] feature images (raw or encoded, features.hip write_fenc; nullable: results only)
  uint8_t* send;         // [N][C * W]: C ResultRec, then (features) C FeatRec per peer
  int32_t C, cap;
};

__global__ __launch_bounds__(256) void exchange_scatter_kernel(XchgScatterArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.cap || i >= a.hdr->n) return;
  const int d = a.route[i];
  const int p = d / a.C, j = d - p * a.C;
  const size_t W = a.feat ? sizeof(ResultRec) + sizeof(FeatRec) : sizeof(ResultRec);
  uint8_t* base = a.send + (size_t)p * a.C * W;
  *reinterpret_cast<int2*>(base + (size_t)j * sizeof(ResultRec)) = *reinterpret_cast<const int2*>(a.res + i);
  if (a.feat) {
    const int4* s = reinterpret_cast<const int4*>(a.feat + i);
    int4* o = reinterpret_cast<int4*>(base + (size_t)a.C * sizeof(ResultRec) + (size_t)j * sizeof(FeatRec));
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = s[k];
  }
}

namespace {

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("exchange ") + what + ": " + hipGetErrorString(e));
}

// the serving core calls the driver's function table from threads of its own: the first call
// on a thread makes the driver's device current there
void bind_device(int d) {
  thread_local int cur = -1;
  if (cur != d) {
    hip_ok(hipSetDevice(d), "set device");
    cur = d;
  }
}

// ------------------------------------------------------------------------------- RCCL (dlopen)
struct Uid {
  char b[128];
};
struct Rccl {
  int (*get_unique_id)(Uid*) = nullptr;
  int (*comm_init_rank)(void**, int, Uid, int) = nullptr;
  int (*all_to_all)(const void*, void*, size_t, int, void*, hipStream_t) = nullptr;
  int (*comm_destroy)(void*) = nullptr;
  int (*comm_abort)(void*) = nullptr;
  int (*async_error)(void*, int*) = nullptr;
  const char* (*err)(int) = nullptr;
};
constexpr int kUint8 = 1;  // ncclUint8

const Rccl& rccl(const std::string& path) {
  static Rccl r;
  static bool loaded = false;
  if (loaded) return r;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // torch's copy, already mapped
  if (!h && !path.empty()) h = dlopen(path.c_str(), RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) throw std::runtime_error(std::string("exchange: cannot load RCCL: ") + dlerror());
  auto sym = [&](const char* s) {
    void* f = dlsym(h, s);
    if (!f) throw std::runtime_error(std::string("exchange: RCCL lacks ") + s);
    return f;
  };
  r.get_unique_id = reinterpret_cast<int (*)(Uid*)>(sym("ncclGetUniqueId"));
  r.comm_init_rank = reinterpret_cast<int (*)(void**, int, Uid, int)>(sym("ncclCommInitRank"));
  r.all_to_all = reinterpret_cast<int (*)(const void*, void*, size_t, int, void*, hipStream_t)>(sym("ncclAllToAll"));
  r.comm_destroy = reinterpret_cast<int (*)(void*)>(sym("ncclCommDestroy"));
  r.comm_abort = reinterpret_cast<int (*)(void*)>(sym("ncclCommAbort"));
  r.async_error = reinterpret_cast<int (*)(void*, int*)>(sym("ncclCommGetAsyncError"));
  r.err = reinterpret_cast<const char* (*)(int)>(sym("ncclGetErrorString"));
  loaded = true;
  return r;
}

void nccl_ok(const Rccl& r, int e, const char* what) {
  if (e != 0) throw std::runtime_error(std::string("RCCL ") + what + ": " + r.err(e));
}

class RcclComm {
 public:
  RcclComm(const std::string& lib, int rank, int world, py::bytes uid) : r_(rccl(lib)), rank_(rank), world_(world) {
    std::string s = uid;
    if (s.size() != sizeof(Uid)) throw std::runtime_error("RcclComm: unique id must be 128 bytes");
    if (world < 1 || world > XCHG_MAX_WORLD || rank < 0 || rank >= world) throw std::runtime_error("RcclComm: rank/world");
    Uid id;
    std::memcpy(id.b, s.data(), sizeof(Uid));
    int e;
    {
      py::gil_scoped_release nogil;  // blocks until every rank joined
      e = r_.comm_init_rank(&comm_, world, id, rank);
    }
    nccl_ok(r_, e, "ncclCommInitRank");
  }
  // communicators live until destroy() or process exit: destroying one from a static
  // destructor after the HIP runtime began tearing down faults (seen under rocprofv3)
  ~RcclComm() = default;
  // the owner drained the streams and destroyed every graph that captured this communicator's
  // collectives first (engine/dp.py DpGpuScorer.close): RCCL waits for those graph references
  void destroy() {
    if (!comm_) return;
    void* c = comm_;
    comm_ = nullptr;
    py::gil_scoped_release nogil;
    (void)r_.comm_destroy(c);
  }
  bool alive() const { return comm_ != nullptr; }
  uintptr_t ptr() const { return reinterpret_cast<uintptr_t>(comm_); }
  int rank() const { return rank_; }
  int world() const { return world_; }
  void all_to_all(uintptr_t send, uintptr_t recv, size_t bytes_per_peer, uintptr_t stream) {
    nccl_ok(r_, r_.all_to_all(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), bytes_per_peer,
                              kUint8, comm_, reinterpret_cast<hipStream_t>(stream)),
            "ncclAllToAll");
  }
  // 0 = healthy; otherwise the ncclResult_t of an asynchronous failure (a peer died)
  int async_error() const {
    int e = 0;
    if (!comm_) return 0;
    (void)r_.async_error(comm_, &e);
    return e;
  }
  // tear down after a failure: in-flight collectives are cancelled (failover path)
  void abort() {
    if (comm_) (void)r_.comm_abort(comm_);
    comm_ = nullptr;
  }

 private:
  const Rccl& r_;
  void* comm_ = nullptr;
  int rank_, world_;
};

// ------------------------------------------------------------------------------- driver
// Per micro-batch (slot s, chunk capacity C), one pipeline stage per stream so no stream ever
// blocks on a later stage of its own batch (rocprofv3: with send and post both on the copy
// stream, the copy stream sat behind the row all-to-all of every batch and the pipeline
// serialised at ~190 us per batch):
//   xs: wait done[s] (the slot's previous batch fully returned) -> graph send (H2D chunks +
//       header) -> ncclAllToAll(rows) -> ev x
//   cs: wait x, wait state[-2] (its K1 cleared this batch's dedup region) -> graph post
//       (compact + dedup insert) -> ev post
//   ss: wait post -> graph state (K1 + multi-event update) -> ev state
//   ms: wait state -> graph model (trees / head / ensemble / scatter) -> ev model
//   ys: wait model -> ncclAllToAll(results) -> D2H rrecv -> pinned -> ev done[s]
// xs / ys run on CUs reserved for communication (engine/dp.py IGP_XCHG_COMM_CUS).
class XchgDriver {
 public:
  // cx / cy: the row and result communicators; both null for the node-shared rows + results
  // regions (set_rows_shm + set_results_shm: no collective on the hot path)
  XchgDriver(uintptr_t cs, uintptr_t ss, uintptr_t ms, uintptr_t xs, uintptr_t ys, int depth, int world,
             const RcclComm* cx, const RcclComm* cy)
      : cs_(S(cs)), ss_(S(ss)), ms_(S(ms)), xs_(S(xs)), ys_(S(ys)), depth_(depth), world_(world),
        cx_(cx ? cx->ptr() : 0), cy_(cy ? cy->ptr() : 0), r_(cx ? &rccl("") : nullptr) {
    if (!cx != !cy) throw std::runtime_error("XchgDriver: both communicators or neither");
    if (cx && (cx->world() != world || cy->world() != world)) throw std::runtime_error("XchgDriver: communicator world");
    if (depth < 1 || depth > DEDUP_AHEAD)  // the copy of batch q relies on batch q - depth's state stage
      throw std::runtime_error("XchgDriver: depth exceeds the dedup ring (DEDUP_AHEAD)");
    hip_ok(hipGetDevice(&device_), "get device");  // the serving core's threads bind to it
    ev_.resize(6 * depth);
    // the hop / post / state / model events only order work between this device's queues: no
    // system-scope fence at the stage's end (as PipeDriver, driver.hip); the done event keeps it
    // (the host reads the results from pinned memory after it)
    const unsigned dev_flags = hipEventDisableTiming | (unsigned)hipEventDisableSystemFence;
    for (size_t i = 0; i < ev_.size(); ++i)
      hip_ok(hipEventCreateWithFlags(&ev_[i], i % 6 == 5 ? hipEventDisableTiming : dev_flags), "event create");
    done_recorded_.assign(depth, false);
    gen_.assign(size_t(depth), 0);
    slots_.resize(depth);
  }
  ~XchgDriver() {
    if (clock_) clock_->retract(ev_.data(), ev_.size());  // before the events go
    for (auto& e : ev_) (void)hipEventDestroy(e);
  }

  void set_slot(int slot, uintptr_t host_hdr, uintptr_t host_x, uintptr_t host_rr, uintptr_t xsend, uintptr_t xrecv,
                uintptr_t rsend, uintptr_t rrecv, size_t host_x_bytes, size_t host_rr_bytes) {
    check_slot(slot);
    slots_[slot] = {reinterpret_cast<char*>(host_hdr), reinterpret_cast<char*>(host_x), reinterpret_cast<char*>(host_rr),
                    reinterpret_cast<void*>(xsend), reinterpret_cast<void*>(xrecv), reinterpret_cast<void*>(rsend),
                    reinterpret_cast<void*>(rrecv), host_x_bytes, host_rr_bytes};
  }

  // captured: the send graph also holds the row all-to-all + compact / dedup insert, the model
  // graphs the result all-to-all + D2H (post is then unused)
  void set_captured(bool c) { captured_ = c; }
  void set_graphs(int C, int slot, uintptr_t send, uintptr_t post, uintptr_t state, uintptr_t model, uintptr_t model_f) {
    check_slot(slot);
    Graphs& g = graphs_[key(C, slot)];
    g.send = G(send);
    g.post = G(post);
    g.state = G(state);
    g.model = G(model);
    g.model_f = G(model_f);
  }

  // captured mode: the collective-free stages as recorded launches (oplist.h) instead of graph
  // replays - the state stage (K1 + update), and with node-shared results the model stages too
  // (model_f / model null: those stay graphs). A hipGraphLaunch costs ~20 us of host time even
  // for a two-kernel graph (rocprofv3 HIP API trace, profiles/NOTES.md round 5), and the serving
  // core issues every step from one thread.
  void set_stage_ops(int C, int slot, std::shared_ptr<OpList> state, std::shared_ptr<OpList> model,
                     std::shared_ptr<OpList> model_f) {
    check_slot(slot);
    if (!state || !model != !model_f) throw std::runtime_error("XchgDriver: set_stage_ops lists");
    Graphs& g = graphs_[key(C, slot)];
    g.ostate = std::move(state);
    g.omodel = std::move(model);
    g.omodel_f = std::move(model_f);
  }

  // src: nbytes of prebuilt chunks ([N][C+1] ReqRec) copied into the slot's pinned buffer
  // (0: already there). The caller must not refill a slot before wait(slot) of its last batch.
  void submit(int slot, int C, int seq, int64_t now, uintptr_t src, size_t nbytes, bool with_features) {
    check_slot(slot);
    py::gil_scoped_release nogil;
    submit_impl(slot, C, seq, now, src, nbytes, with_features);
  }

  // C function table for the native serving core (csrc/include/device_ops.h) with chunk
  // capacity C: every step returns FeatRec rows too, so the result all-to-all has one size on
  // every rank whatever the callers of each rank asked for
  uintptr_t device_ops(int C) {
    bool have = false;
    for (auto& kv : graphs_) have |= int(kv.first >> 8) == C;
    if (!have) throw std::runtime_error("XchgDriver: no graphs for this chunk capacity");
    ops_C_ = C;
    ops_.abi = IGP_DEVICE_OPS_ABI;
    ops_.depth = depth_;
    ops_.world = world_;
    ops_.exchange = 1;
    ops_.cap = C;
    ops_.features_always = 1;
    ops_.ctx = this;
    ops_.rows = [](void* ctx, int32_t slot) -> char* { return static_cast<XchgDriver*>(ctx)->slots_[slot].host_x; };
    ops_.submit = [](void* ctx, int32_t slot, int32_t, int32_t seq, int64_t now, int32_t, char* err,
                     int32_t errlen) -> int32_t {
      auto* d = static_cast<XchgDriver*>(ctx);
      try {
        bind_device(d->device_);
        d->submit_impl(slot, d->ops_C_, seq, now, 0, 0, true);
      } catch (const std::exception& e) {
        if (err && errlen > 0) {
          std::strncpy(err, e.what(), size_t(errlen) - 1);
          err[errlen - 1] = 0;
        }
        return -1;
      }
      return 0;
    };
    ops_.wait = [](void* ctx, int32_t slot, int64_t timeout_us, char* err, int32_t errlen) -> int32_t {
      auto* d = static_cast<XchgDriver*>(ctx);
      try {
        bind_device(d->device_);
      } catch (const std::exception& ex) {
        if (err && errlen > 0) {
          std::strncpy(err, ex.what(), size_t(errlen) - 1);
          err[errlen - 1] = 0;
        }
        return -1;
      }
      hipEvent_t e = d->E(slot, 5);
      const auto t_start = std::chrono::steady_clock::now();
      auto owners = [&]() -> int32_t {
        if (!d->rshm_) return 0;
        int64_t left = -1;
        if (timeout_us >= 0)
          left = std::max<int64_t>(0, timeout_us - std::chrono::duration_cast<std::chrono::microseconds>(
                                                       std::chrono::steady_clock::now() - t_start).count());
        return d->wait_owners(slot, left, err, errlen);
      };
      if (timeout_us < 0) {
        const hipError_t r = hipEventSynchronize(e);
        if (r == hipSuccess) return owners();
        if (err && errlen > 0) {
          std::strncpy(err, hipGetErrorString(r), size_t(errlen) - 1);
          err[errlen - 1] = 0;
        }
        return -1;
      }
      const auto t_end = std::chrono::steady_clock::now() + std::chrono::microseconds(timeout_us);
      bool failed = false;
      const bool done = poll_event_until(e, t_end, [&](hipError_t q) {
        failed = true;
        if (err && errlen > 0) {
          std::strncpy(err, hipGetErrorString(q), size_t(errlen) - 1);
          err[errlen - 1] = 0;
        }
      });
      if (done) return owners();
      return failed ? -1 : 1;
    };
    ops_.results = [](void* ctx, int32_t slot) -> const void* {
      auto* d = static_cast<XchgDriver*>(ctx);
      if (d->rshm_) return d->rshm_ + size_t(slot) * d->rshm_slot_stride_ + size_t(d->rank_) * d->ops_C_ * kResFeatW;
      return d->slots_[slot].host_rr;
    };
    ops_.features = [](void*, int32_t) -> const void* { return nullptr; };
    ops_.res_owner_stride = rshm_ ? int64_t(rshm_owner_stride_) : 0;
    return reinterpret_cast<uintptr_t>(&ops_);
  }

  // Per-GPU D2H result path (instead of the result all-to-all): every owner's scatter kernel
  // writes its scored rows for ALL senders ([sender][C][W]) straight into its block of a
  // node-shared pinned host region [slot][owner][sender][C][W] (no copy job); a sender reads its
  // chunk of every owner's block. Completion is two-level: the slot's local event (this rank's
  // model stage, scatter included, finished), then one release-published generation per
  // (slot, owner) in the region's flag lines, polled until every owner reached the step. Reuse
  // of a block is ordered by the next step's row all-to-all (no owner can write step k + depth
  // before every sender issued it, i.e. finished reading step k).
  void set_results_shm(uintptr_t base, size_t slot_stride, size_t owner_stride, uintptr_t flags, int rank) {
    if (!base || !flags || rank < 0 || rank >= world_) throw std::runtime_error("XchgDriver: results region");
    rshm_ = reinterpret_cast<char*>(base);
    rshm_slot_stride_ = slot_stride;
    rshm_owner_stride_ = owner_stride;
    owners_ = OwnerGenerations(reinterpret_cast<int64_t*>(flags), world_, rank);
    rank_ = rank;
    // a driver replacing another on the same region (model hot reload, every rank paused at the
    // same step): continue from the generation this owner published last
    for (int s = 0; s < depth_; ++s) gen_[size_t(s)] = owners_.published(s, rank_);
  }
  // the longest a step waits for the other owners when its caller gives no deadline (the serving
  // core's drain of a step that already overran its own): the engine sets it from the serving
  // deadline (engine/dp.py), so a dead or hung owner fails the step instead of hanging it
  void set_owner_deadline_us(int64_t us) {
    if (us <= 0) throw std::runtime_error("XchgDriver: the owner deadline must be finite and positive");
    owner_deadline_us_ = us;
  }
  int64_t owner_deadline_us() const { return owner_deadline_us_; }

  // Node-shared rows region (no row all-to-all): [slot][sender][owner][C + 1] ReqRec in page-
  // locked /dev/shm plus one generation line per (slot, sender). A sender packs its chunks for
  // every owner straight into its block (the serving core through device_ops().rows, or
  // submit()'s copy) and publishes the step's generation; an owner waits on the host until
  // every sender of the step published (finite deadline, results_region.h), then its copy
  // stage compacts its chunk of every sender's block straight from host memory (zero copy,
  // one kernel) and inserts the batch into the dedup region - three recorded stages per step,
  // no collective. A block is reused (step k + depth) only after the sender's wait(slot) of
  // step k saw every owner's results, i.e. after every owner's copy stage of step k finished.
  void set_rows_shm(uintptr_t base, size_t slot_stride, size_t sender_stride, uintptr_t flags) {
    if (!rshm_) throw std::runtime_error("XchgDriver: the rows region needs the results region (set_results_shm first)");
    if (!base || !flags || sender_stride == 0 || slot_stride < size_t(world_) * sender_stride)
      throw std::runtime_error("XchgDriver: rows region");
    rows_ = reinterpret_cast<char*>(base);
    senders_ = OwnerGenerations(reinterpret_cast<int64_t*>(flags), world_, rank_, "rows region: sender(s)");
    for (int s = 0; s < depth_; ++s) {
      slots_[size_t(s)].host_x = rows_ + size_t(s) * slot_stride + size_t(rank_) * sender_stride;
      slots_[size_t(s)].host_x_bytes = sender_stride;
    }
  }
  // the copy stage of the rows-region mode (compact from the region + dedup insert)
  void set_copy_ops(int C, int slot, std::shared_ptr<OpList> copy) {
    check_slot(slot);
    if (!copy) throw std::runtime_error("XchgDriver: set_copy_ops list");
    graphs_[key(C, slot)].ocopy = std::move(copy);
  }

  // d2h mode, inside wait(slot): publish this owner's generation, then wait for every owner's.
  // 1 = an owner missed the deadline (err names it); timeout_us < 0: the owner deadline.
  int32_t wait_owners(int slot, int64_t timeout_us, char* err, int32_t errlen) {
    const int64_t g = gen_[size_t(slot)];
    owners_.publish(slot, g);
    // every step's results wait is a host barrier on the slowest owner: its time is accounted
    // (mean and worst per stats() window) next to the senders' rows wait
    const auto t0 = clk::now();
    const int32_t rc = owners_.wait(slot, g, timeout_us >= 0 ? timeout_us : owner_deadline_us_, wait_spin_us(), err, errlen);
    const double dt = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
    st_[5] += dt;
    st_[6] = std::max(st_[6], dt);
    return rc;
  }

  void submit_impl(int slot, int C, int seq, int64_t now, uintptr_t src, size_t nbytes, bool with_features) {
    auto it = graphs_.find(key(C, slot));
    ++gen_[size_t(slot)];  // every rank submits the same steps on the same slots: the same generations
    if (it == graphs_.end()) throw std::runtime_error("XchgDriver: no graphs for this chunk capacity / slot");
    const Graphs g = it->second;
    const Slot& sl = slots_[slot];
    const size_t xbytes = (size_t)(C + 1) * sizeof(ReqRec);
    const size_t W = with_features ? sizeof(ResultRec) + sizeof(FeatRec) : sizeof(ResultRec);
    const size_t rbytes = (size_t)C * W;
    if (nbytes > sl.host_x_bytes || (size_t)world_ * xbytes > sl.host_x_bytes) throw std::runtime_error("XchgDriver: chunks exceed the slot buffer");
    if ((size_t)world_ * rbytes > sl.host_rr_bytes) throw std::runtime_error("XchgDriver: results exceed the slot buffer");
    if (with_features && !g.model_f && !g.omodel_f) throw std::runtime_error("XchgDriver: no feature graph");
    Range range("igp.xsubmit");
    const auto t0 = clk::now();
    if (src) std::memcpy(sl.host_x, reinterpret_cast<const void*>(src), nbytes);
    BatchHdr* h = reinterpret_cast<BatchHdr*>(sl.host_hdr);
    h->n = 0;  // written on device by exchange_compact
    h->seq = seq;
    h->now = now;
    const auto t1 = clk::now();
    hipEvent_t e_send = E(slot, 0), e_x = E(slot, 1), e_post = E(slot, 2), e_state = E(slot, 3), e_model = E(slot, 4),
               e_done = E(slot, 5);
    if (rows_) {
      if (!g.ocopy || !(g.ostate || g.state) || !((with_features ? g.omodel_f : g.omodel) || (with_features ? g.model_f : g.model)))
        throw std::runtime_error("XchgDriver: rows-region mode lacks a stage body");
      // this sender's chunks are in its block: publish, then wait for every sender of the step
      senders_.publish(slot, gen_[size_t(slot)]);
      char err[256] = {0};
      if (senders_.wait(slot, gen_[size_t(slot)], owner_deadline_us_, wait_spin_us(), err, sizeof err) != 0)
        throw std::runtime_error(err);
      const auto t2 = clk::now();
      // the slot's previous batch (q - depth) finished: its device rows / route / dedup region are free
      if (done_recorded_[slot]) hip_ok(hipStreamWaitEvent(cs_, e_done, 0), "wait done");
      if (!g.ocopy->run_recording(cs_, e_post)) hip_ok(hipEventRecord(e_post, cs_), "record post");
      hip_ok(hipStreamWaitEvent(ss_, e_post, 0), "wait post");
      if (g.ostate) {
        if (!g.ostate->run_recording(ss_, e_state)) hip_ok(hipEventRecord(e_state, ss_), "record state");
      } else {
        hip_ok(hipGraphLaunch(g.state, ss_), "state graph");
        hip_ok(hipEventRecord(e_state, ss_), "record state");
      }
      if (clock_) clock_->publish(e_state);
      hip_ok(hipStreamWaitEvent(ms_, e_state, 0), "wait state");
      const std::shared_ptr<OpList>& om = with_features ? g.omodel_f : g.omodel;
      if (om) {
        if (!om->run_recording(ms_, e_done)) hip_ok(hipEventRecord(e_done, ms_), "record done");
      } else {
        hip_ok(hipGraphLaunch(with_features ? g.model_f : g.model, ms_), "model graph");
        hip_ok(hipEventRecord(e_done, ms_), "record done");
      }
      auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
      st_[0] += us(t0, t1);
      st_[1] += us(t2, clk::now());
      const double sw = us(t1, t2);  // the wait for the other senders' rows (host)
      st_[2] += sw;
      st_[7] = std::max(st_[7], sw);
      st_[3] += 1;
      done_recorded_[slot] = true;
      return;
    }
    (void)e_send;
    // a hop between two streams costs an event record + wait; when the exchange runs its
    // collectives on the copy / model streams themselves (IGP_XCHG_STREAMS=3) there is none
    auto hop = [&](hipStream_t from, hipStream_t to, hipEvent_t e, const char* what) {
      if (from == to) return;
      hip_ok(hipEventRecord(e, from), what);
      hip_ok(hipStreamWaitEvent(to, e, 0), what);
    };
    if (captured_) {
      // the collectives and the D2H copy are nodes of the graphs (RCCL stream capture): three
      // launches per batch, the same shape as the single-GPU pipeline
      // the slot's previous batch (q - depth) finished: its buffers are free, and its state
      // stage - with every earlier one, the state stream runs in order - cleared this batch's
      // dedup region (cleared by batch q - DEDUP_AHEAD, and depth <= DEDUP_AHEAD)
      if (done_recorded_[slot]) hip_ok(hipStreamWaitEvent(cs_, e_done, 0), "wait done");
      hip_ok(hipGraphLaunch(g.send, cs_), "send+post graph");
      hip_ok(hipEventRecord(e_post, cs_), "record post");
      hip_ok(hipStreamWaitEvent(ss_, e_post, 0), "wait post");
      // recorded stages bind their end event to their last kernel (no marker command)
      if (g.ostate) {
        if (!g.ostate->run_recording(ss_, e_state)) hip_ok(hipEventRecord(e_state, ss_), "record state");
      } else {
        hip_ok(hipGraphLaunch(g.state, ss_), "state graph");
        hip_ok(hipEventRecord(e_state, ss_), "record state");
      }
      if (clock_) clock_->publish(e_state);  // K1 + multi-event update: readers order after it
      hip_ok(hipStreamWaitEvent(ms_, e_state, 0), "wait state");
      const std::shared_ptr<OpList>& om = with_features ? g.omodel_f : g.omodel;
      if (om) {
        if (!om->run_recording(ms_, e_done)) hip_ok(hipEventRecord(e_done, ms_), "record done");
      } else {
        hip_ok(hipGraphLaunch(with_features ? g.model_f : g.model, ms_), "model+results graph");
        hip_ok(hipEventRecord(e_done, ms_), "record done");
      }
      st_[0] += std::chrono::duration<double, std::micro>(t1 - t0).count();
      st_[1] += std::chrono::duration<double, std::micro>(clk::now() - t1).count();
      st_[3] += 1;
      done_recorded_[slot] = true;
      return;
    }
    if (done_recorded_[slot]) hip_ok(hipStreamWaitEvent(xs_, e_done, 0), "wait done");
    hip_ok(hipGraphLaunch(g.send, xs_), "send graph");
    const auto t2 = clk::now();
    if (!r_) throw std::runtime_error("XchgDriver: no communicators for the row all-to-all");
    nccl_ok(*r_, r_->all_to_all(sl.xsend, sl.xrecv, xbytes, kUint8, reinterpret_cast<void*>(cx_), xs_), "all_to_all rows");
    const auto t3 = clk::now();
    hop(xs_, cs_, e_x, "x -> copy");
    hip_ok(hipGraphLaunch(g.post, cs_), "post graph");
    hip_ok(hipEventRecord(e_post, cs_), "record post");
    hip_ok(hipStreamWaitEvent(ss_, e_post, 0), "wait post");
    hip_ok(hipGraphLaunch(g.state, ss_), "state graph");
    hip_ok(hipEventRecord(e_state, ss_), "record state");
    if (clock_) clock_->publish(e_state);
    hip_ok(hipStreamWaitEvent(ms_, e_state, 0), "wait state");
    hip_ok(hipGraphLaunch(with_features ? g.model_f : g.model, ms_), "model graph");
    if (rshm_) {  // node-shared results: the model stage's scatter wrote them into the region
      hip_ok(hipEventRecord(e_done, ms_), "record done");
      auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
      st_[0] += us(t0, t1);
      st_[1] += us(t1, t2) + us(t3, clk::now());
      st_[2] += us(t2, t3);
      st_[3] += 1;
      done_recorded_[slot] = true;
      return;
    }
    hop(ms_, ys_, e_model, "model -> y");
    const auto t4 = clk::now();
    nccl_ok(*r_, r_->all_to_all(sl.rsend, sl.rrecv, rbytes, kUint8, reinterpret_cast<void*>(cy_), ys_), "all_to_all results");
    const auto t5 = clk::now();
    hip_ok(hipMemcpyAsync(sl.host_rr, sl.rrecv, (size_t)world_ * rbytes, hipMemcpyDeviceToHost, ys_), "results D2H");
    hip_ok(hipEventRecord(e_done, ys_), "record done");
    const auto t6 = clk::now();
    auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    st_[0] += us(t0, t1);
    st_[1] += us(t1, t2) + us(t3, t4) + us(t5, t6);
    st_[2] += us(t2, t3) + us(t4, t5);
    st_[3] += 1;
    done_recorded_[slot] = true;
  }

  void wait(int slot) {
    check_slot(slot);
    py::gil_scoped_release nogil;
    Range range("igp.xwait");
    const auto t0 = clk::now();
    hip_ok(hipEventSynchronize(E(slot, 5)), "sync done");
    st_[4] += std::chrono::duration<double, std::micro>(clk::now() - t0).count();
  }
  bool query(int slot) {
    check_slot(slot);
    return hipEventQuery(E(slot, 5)) == hipSuccess;
  }
  // last submitted batch's state-stream event (snapshot ordering)
  uintptr_t state_event(int slot) const { return reinterpret_cast<uintptr_t>(ev_[6 * slot + 3]); }
  void set_state_clock(std::shared_ptr<StateClock> c) { clock_ = std::move(c); }
  // the slot's completion event (the watchdog's deadline wait, watch.hip)
  uintptr_t done_event(int slot) const { return reinterpret_cast<uintptr_t>(E(slot, 5)); }

  py::dict stats() {
    py::dict d;
    const double n = st_[3] > 0 ? st_[3] : 1;
    d["submits"] = st_[3];
    d["rows_copy_us"] = st_[0] / n;
    d["launch_event_ops_us"] = st_[1] / n;
    d[rows_ ? "sender_wait_us" : "rccl_issue_us"] = st_[2] / n;
    d["wait_us"] = st_[4] / n;
    d["owner_wait_us"] = st_[5] / n;       // results region: wait for every owner's generation
    d["owner_wait_max_us"] = st_[6];
    d["sender_wait_max_us"] = st_[7];
    for (double& v : st_) v = 0;
    return d;
  }

 private:
  using clk = std::chrono::steady_clock;
  struct Graphs {
    hipGraphExec_t send = nullptr, post = nullptr, state = nullptr, model = nullptr, model_f = nullptr;
    std::shared_ptr<OpList> ostate, omodel, omodel_f;  // set_stage_ops (captured mode)
    std::shared_ptr<OpList> ocopy;                     // set_copy_ops (rows-region mode)
  };
  struct Slot {
    char* host_hdr;
    char* host_x;
    char* host_rr;
    void* xsend;
    void* xrecv;
    void* rsend;
    void* rrecv;
    size_t host_x_bytes, host_rr_bytes;
  };
  static hipStream_t S(uintptr_t p) { return reinterpret_cast<hipStream_t>(p); }
  static hipGraphExec_t G(uintptr_t p) { return reinterpret_cast<hipGraphExec_t>(p); }
  static int64_t key(int C, int slot) { return ((int64_t)C << 8) | slot; }
  hipEvent_t E(int slot, int k) const { return ev_[6 * slot + k]; }
  void check_slot(int s) const {
    if (s < 0 || s >= depth_) throw std::runtime_error("XchgDriver: bad slot");
  }
  hipStream_t cs_, ss_, ms_, xs_, ys_;
  std::shared_ptr<StateClock> clock_;
  int depth_, world_;
  uintptr_t cx_, cy_;
  const Rccl* r_;
  std::vector<hipEvent_t> ev_;
  std::vector<bool> done_recorded_;
  std::vector<Slot> slots_;
  std::unordered_map<int64_t, Graphs> graphs_;
  double st_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  bool captured_ = false;
  IgpDeviceOps ops_{};
  int ops_C_ = 0;
  int device_ = 0;
  static constexpr size_t kResFeatW = sizeof(ResultRec) + sizeof(FeatRec);
  // per-GPU D2H result path (set_results_shm)
  char* rshm_ = nullptr;
  size_t rshm_slot_stride_ = 0, rshm_owner_stride_ = 0;
  OwnerGenerations owners_;
  OwnerGenerations senders_;  // rows-region mode: the generation lines of the senders
  char* rows_ = nullptr;
  int64_t owner_deadline_us_ = 10000000;  // set_owner_deadline_us (engine: from the serving deadline)
  int rank_ = 0;
  std::vector<int64_t> gen_;
};

template <class T>
T P(uintptr_t p) {
  return reinterpret_cast<T>(p);
}

}  // namespace

void register_exchange(py::module_& m) {
  m.attr("XCHG_MAX_WORLD") = XCHG_MAX_WORLD;
  m.def("rccl_unique_id", [](const std::string& lib) {
    const Rccl& r = rccl(lib);
    Uid id;
    nccl_ok(r, r.get_unique_id(&id), "ncclGetUniqueId");
    return py::bytes(id.b, sizeof(id.b));
  });
  py::class_<RcclComm>(m, "RcclComm")
      .def(py::init<const std::string&, int, int, py::bytes>())
      .def("ptr", &RcclComm::ptr)
      .def("rank", &RcclComm::rank)
      .def("world", &RcclComm::world)
      .def("all_to_all", &RcclComm::all_to_all)
      .def("async_error", &RcclComm::async_error)
      .def("destroy", &RcclComm::destroy)
      .def_property_readonly("alive", &RcclComm::alive)
      .def("abort", &RcclComm::abort);
  py::class_<XchgDriver>(m, "XchgDriver")
      .def(py::init<uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int, int, const RcclComm*, const RcclComm*>(),
           py::keep_alive<1, 9>(), py::keep_alive<1, 10>())
      .def("set_rows_shm", &XchgDriver::set_rows_shm)
      .def("set_copy_ops", &XchgDriver::set_copy_ops)
      .def("set_slot", &XchgDriver::set_slot)
      .def("set_graphs", &XchgDriver::set_graphs)
      .def("set_captured", &XchgDriver::set_captured)
      .def("set_stage_ops", &XchgDriver::set_stage_ops, py::arg("C"), py::arg("slot"), py::arg("state"),
           py::arg("model") = nullptr, py::arg("model_f") = nullptr)
      .def("set_results_shm", &XchgDriver::set_results_shm)
      .def("set_owner_deadline_us", &XchgDriver::set_owner_deadline_us)
      .def_property_readonly("owner_deadline_us", &XchgDriver::owner_deadline_us)
      .def("submit", &XchgDriver::submit)
      .def("device_ops", &XchgDriver::device_ops)
      .def("wait", &XchgDriver::wait)
      .def("query", &XchgDriver::query)
      .def("state_event", &XchgDriver::state_event)
      .def("set_state_clock", &XchgDriver::set_state_clock)
      .def("done_event", &XchgDriver::done_event)
      .def("stats", &XchgDriver::stats);
  // page-lock a host range (the node-shared result region of the D2H result path) so device
  // copies into it are asynchronous DMA and capturable
  m.def("host_register", [](uintptr_t p, size_t n) {
    const hipError_t e = hipHostRegister(reinterpret_cast<void*>(p), n, hipHostRegisterDefault);
    if (e != hipSuccess) throw std::runtime_error(std::string("hipHostRegister: ") + hipGetErrorString(e));
  });
  m.def("host_unregister", [](uintptr_t p) { (void)hipHostUnregister(reinterpret_cast<void*>(p)); });
  // kernel launches (captured into the exchange graphs from Python)
  m.def("exchange_compact", [](uintptr_t recv, uintptr_t rows, uintptr_t hdr, uintptr_t route, int N, int C, int cap,
                               uintptr_t stream, int64_t pstride, uintptr_t hdr_src) {
    if (N < 1 || N > XCHG_MAX_WORLD || C < 1 || cap < 1) throw std::runtime_error("exchange_compact: bad sizes");
    if (pstride == 0) pstride = C + 1;
    if (pstride < C + 1) throw std::runtime_error("exchange_compact: sender stride below the chunk size");
    XchgCompactArgs a{P<const ReqRec*>(recv), P<ReqRec*>(rows), P<BatchHdr*>(hdr), P<int32_t*>(route), N, C, cap,
                      pstride, P<const int4*>(hdr_src)};
    const int threads = N * C;
    auto f = [a, threads](hipStream_t st) {
      IGP_LAUNCH(exchange_compact_kernel, dim3((threads + 255) / 256), dim3(256), 0, st, a);
    };
    if (OpList* r = recording()) {
      r->ops.emplace_back(f);
      return;
    }
    f(P<hipStream_t>(stream));
    hip_ok(hipGetLastError(), "exchange_compact");
  }, py::arg("recv"), py::arg("rows"), py::arg("hdr"), py::arg("route"), py::arg("N"), py::arg("C"), py::arg("cap"),
        py::arg("stream"), py::arg("pstride") = 0, py::arg("hdr_src") = 0);
  m.def("exchange_clear", [](uintptr_t recv, int N, int C, uintptr_t stream, uintptr_t hdr_src, uintptr_t hdr_dst) {
    if (N < 1 || N > XCHG_MAX_WORLD || C < 1) throw std::runtime_error("exchange_clear: bad sizes");
    if (!hdr_src != !hdr_dst) throw std::runtime_error("exchange_clear: header source and destination together");
    ReqRec* r = P<ReqRec*>(recv);
    const int4* hs = P<const int4*>(hdr_src);
    int4* hd = P<int4*>(hdr_dst);
    auto f = [r, N, C, hs, hd](hipStream_t st) {
      IGP_LAUNCH(exchange_clear_kernel, dim3(1), dim3(64), 0, st, r, N, C, hs, hd);
    };
    if (OpList* rec = recording()) {
      rec->ops.emplace_back(f);
      return;
    }
    f(P<hipStream_t>(stream));
    hip_ok(hipGetLastError(), "exchange_clear");
  }, py::arg("recv"), py::arg("N"), py::arg("C"), py::arg("stream"), py::arg("hdr_src") = 0, py::arg("hdr_dst") = 0);
  m.def("exchange_scatter", [](uintptr_t hdr, uintptr_t route, uintptr_t res, uintptr_t feat, uintptr_t send, int C,
                               int cap, uintptr_t stream) {
    if (C < 1 || cap < 1) throw std::runtime_error("exchange_scatter: bad sizes");
    XchgScatterArgs a{P<const BatchHdr*>(hdr), P<const int32_t*>(route), P<const ResultRec*>(res),
                      P<const FeatRec*>(feat), P<uint8_t*>(send), C, cap};
    auto f = [a, cap](hipStream_t st) {
      IGP_LAUNCH(exchange_scatter_kernel, dim3((cap + 255) / 256), dim3(256), 0, st, a);
    };
    if (OpList* r = recording()) {
      r->ops.emplace_back(f);
      return;
    }
    f(P<hipStream_t>(stream));
    hip_ok(hipGetLastError(), "exchange_scatter");
  });
}

}  // namespace igp

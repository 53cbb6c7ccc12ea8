#include "cpu_device.h"

#include <unistd.h>

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace igp {
namespace {

void set_err(char* err, int32_t errlen, const char* msg) {
  if (!err || errlen <= 0) return;
  std::strncpy(err, msg, size_t(errlen) - 1);
  err[errlen - 1] = 0;
}

}  // namespace

// ============================================================================ CpuDevice
CpuDevice::CpuDevice(std::shared_ptr<CpuScorer> sc, int depth, int cap) : sc_(std::move(sc)) {
  if (!sc_ || depth < 1 || cap < 1) throw std::runtime_error("CpuDevice: scorer / depth / capacity");
  slots_.resize(depth);
  for (auto& s : slots_) {
    s.rows.resize(cap);
    s.res.resize(cap);
    s.feat.resize(cap);
  }
  ops_.abi = IGP_DEVICE_OPS_ABI;
  ops_.depth = depth;
  ops_.world = 1;
  ops_.exchange = 0;
  ops_.cap = cap;
  ops_.features_always = 0;
  ops_.ctx = this;
  ops_.rows = &rows_fn;
  ops_.submit = &submit_fn;
  ops_.wait = &wait_fn;
  ops_.results = &results_fn;
  ops_.features = &features_fn;
}

char* CpuDevice::rows_fn(void* ctx, int32_t slot) {
  return reinterpret_cast<char*>(static_cast<CpuDevice*>(ctx)->slots_[slot].rows.data());
}

int32_t CpuDevice::submit_fn(void* ctx, int32_t slot, int32_t n, int32_t, int64_t now, int32_t wf, char* err,
                             int32_t errlen) {
  auto* d = static_cast<CpuDevice*>(ctx);
  Slot& s = d->slots_[slot];
  try {
    s.wf = wf != 0;
    d->sc_->score(s.rows.data(), size_t(n), now, true, s.res.data(), s.wf ? s.feat.data() : nullptr);
  } catch (const std::exception& e) {
    set_err(err, errlen, e.what());
    return -1;
  }
  return 0;
}

int32_t CpuDevice::wait_fn(void*, int32_t, int64_t, char*, int32_t) { return 0; }  // scored in submit

const void* CpuDevice::results_fn(void* ctx, int32_t slot) {
  return static_cast<CpuDevice*>(ctx)->slots_[slot].res.data();
}

const void* CpuDevice::features_fn(void* ctx, int32_t slot) {
  const Slot& s = static_cast<CpuDevice*>(ctx)->slots_[slot];
  return s.wf ? s.feat.data() : nullptr;
}

// ============================================================================ ShmXchgDevice
// shm layout: [world] Counter | [kRing][world] owner generation lines (results_region.h) |
// per rank r, ring q: send [world][C + 1] ReqRec | per rank r, ring q: results [world][C * W]
// (C ResultRec, then C FeatRec per destination rank). A step completes as on the GPU exchange's
// node-shared results region: each owner publishes the step's generation after writing its rows,
// and every rank waits for all owners with a finite deadline (OwnerGenerations).
ShmXchgDevice::ShmXchgDevice(std::shared_ptr<CpuScorer> sc, const std::string& shm_name, int world, int rank, int depth,
                             int C, bool create, double timeout_s)
    : sc_(std::move(sc)), world_(world), rank_(rank), C_(C), timeout_s_(timeout_s) {
  if (!sc_ || world < 1 || rank < 0 || rank >= world || depth < 1 || C < 1)
    throw std::runtime_error("ShmXchgDevice: bad arguments");
  W_ = sizeof(ResultRec) + sizeof(FeatRec);
  send_bytes_ = size_t(world) * size_t(C + 1) * sizeof(ReqRec);
  res_bytes_ = size_t(world) * size_t(C) * W_;
  const size_t flag_bytes = sizeof(int64_t) * OwnerGenerations::kLineWords * kRing * size_t(world);
  const size_t bytes = sizeof(Counter) * size_t(world) + flag_bytes + size_t(world) * kRing * (send_bytes_ + res_bytes_);
  region_ = Region::shared(shm_name, bytes, create);
  counters_ = reinterpret_cast<Counter*>(region_.base());
  char* flags = reinterpret_cast<char*>(region_.base()) + sizeof(Counter) * size_t(world);
  owners_ = OwnerGenerations(reinterpret_cast<int64_t*>(flags), world, rank);
  data_ = flags + flag_bytes;
  slots_.resize(depth);
  for (auto& s : slots_) {
    s.send.resize(size_t(world) * size_t(C + 1));
    s.recv.resize(res_bytes_);
  }
  compact_.resize(size_t(world) * size_t(C));
  route_.resize(size_t(world) * size_t(C));
  res_.resize(size_t(world) * size_t(C));
  feat_.resize(size_t(world) * size_t(C));
  ops_.abi = IGP_DEVICE_OPS_ABI;
  ops_.depth = depth;
  ops_.world = world;
  ops_.exchange = 1;
  ops_.cap = C;
  ops_.features_always = 1;
  ops_.ctx = this;
  ops_.rows = &rows_fn;
  ops_.submit = &submit_fn;
  ops_.wait = &wait_fn;
  ops_.results = &results_fn;
  ops_.features = &features_fn;
}

ReqRec* ShmXchgDevice::send_area(int r, int q) const {
  return reinterpret_cast<ReqRec*>(data_ + (size_t(r) * kRing + size_t(q)) * send_bytes_);
}

char* ShmXchgDevice::res_area(int r, int q) const {
  return data_ + size_t(world_) * kRing * send_bytes_ + (size_t(r) * kRing + size_t(q)) * res_bytes_;
}

void ShmXchgDevice::wait_all(std::atomic<int64_t> Counter::*field, int64_t target) {
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s_);
  for (int spin = 0;; ++spin) {
    bool all = true;
    for (int r = 0; r < world_ && all; ++r) all = (counters_[r].*field).load(std::memory_order_acquire) >= target;
    if (all) return;
    if (spin < 2000) {
      std::this_thread::yield();
    } else {
      if (std::chrono::steady_clock::now() > t_end) throw std::runtime_error("ShmXchgDevice: a peer missed the step");
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
}

void ShmXchgDevice::step(int slot, int64_t now) {
  Slot& s = slots_[slot];
  const int q = int(k_ % kRing);
  const size_t stride = size_t(C_) + 1;
  // 1. post my owner chunks (and the slot this step runs on: every rank must use the same one)
  if (slot != int(k_ % int64_t(slots_.size()))) slot_violations_.fetch_add(1);
  std::memcpy(send_area(rank_, q), s.send.data(), send_bytes_);
  counters_[rank_].slot.store(slot, std::memory_order_relaxed);
  counters_[rank_].posted.store(k_ + 1, std::memory_order_release);
  wait_all(&Counter::posted, k_ + 1);
  for (int p = 0; p < world_; ++p)  // a peer cannot post step k + 2 before this rank scored k + 1
    if (counters_[p].slot.load(std::memory_order_relaxed) != slot) slot_violations_.fetch_add(1);
  // 2. compact the rows every sender routed to me (sender order, then row order)
  size_t n = 0;
  int64_t t = 0;  // the step's clock: the latest clock of the senders that sent rows
  for (int p = 0; p < world_; ++p) {
    const ReqRec* chunk = send_area(p, q) + size_t(rank_) * stride;
    int c = chunk[0].slot;
    c = c < 0 ? 0 : (c > C_ ? C_ : c);
    if (c > 0 && chunk[0].ts > t) t = chunk[0].ts;
    for (int j = 0; j < c; ++j) {
      compact_[n] = chunk[1 + j];
      compact_[n].tx_type &= 0xff;
      route_[n] = p * C_ + j;
      ++n;
    }
  }
  // 3. score my rows (score-then-update of my shard)
  if (n) sc_->score(compact_.data(), n, t > 0 ? t : now, true, res_.data(), feat_.data());
  rows_scored_.fetch_add(int64_t(n));
  // 4. results back: [destination p][C] ResultRec, then [C] FeatRec
  char* out = res_area(rank_, q);
  for (size_t i = 0; i < n; ++i) {
    const int p = route_[i] / C_, j = route_[i] % C_;
    char* base = out + size_t(p) * size_t(C_) * W_;
    std::memcpy(base + size_t(j) * sizeof(ResultRec), &res_[i], sizeof(ResultRec));
    std::memcpy(base + size_t(C_) * sizeof(ResultRec) + size_t(j) * sizeof(FeatRec), &feat_[i], sizeof(FeatRec));
  }
  // fault injection (FAULT_INJECT=xchg_stall_results): an owner that keeps stepping but never
  // publishes its results - a hung device, alive enough that the posts keep coming
  if (!stall_file_.empty() && !stalled_) stalled_ = ::access(stall_file_.c_str(), F_OK) == 0;
  if (!stalled_) owners_.publish(q, k_ + 1);
  char err[256] = {0};
  if (owners_.wait(q, k_ + 1, int64_t(timeout_s_ * 1e6), 30, err, sizeof err) != 0)
    throw std::runtime_error(std::string("ShmXchgDevice: ") + err);
  // 5. gather my rows' results from every owner
  for (int p = 0; p < world_; ++p)
    std::memcpy(s.recv.data() + size_t(p) * size_t(C_) * W_, res_area(p, q) + size_t(rank_) * size_t(C_) * W_,
                size_t(C_) * W_);
  ++k_;
}

char* ShmXchgDevice::rows_fn(void* ctx, int32_t slot) {
  return reinterpret_cast<char*>(static_cast<ShmXchgDevice*>(ctx)->slots_[slot].send.data());
}

int32_t ShmXchgDevice::submit_fn(void* ctx, int32_t slot, int32_t, int32_t, int64_t now, int32_t, char* err,
                                 int32_t errlen) {
  try {
    static_cast<ShmXchgDevice*>(ctx)->step(slot, now);
  } catch (const std::exception& e) {
    set_err(err, errlen, e.what());
    return -1;
  }
  return 0;
}

int32_t ShmXchgDevice::wait_fn(void*, int32_t, int64_t, char*, int32_t) { return 0; }  // synchronous step

const void* ShmXchgDevice::results_fn(void* ctx, int32_t slot) {
  return static_cast<ShmXchgDevice*>(ctx)->slots_[slot].recv.data();
}

const void* ShmXchgDevice::features_fn(void*, int32_t) { return nullptr; }

}  // namespace igp

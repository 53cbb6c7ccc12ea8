#include "serve_core.h"
#include "thread_name.h"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <ctime>
#include <stdexcept>

namespace igp {

// ============================================================================ StepClock
StepClock::StepClock(const std::string& shm_name, int world, int rank, bool create) : world_(world), rank_(rank) {
  if (world < 1 || rank < 0 || rank >= world) throw std::runtime_error("StepClock: rank / world");
  region_ = Region::shared(shm_name, sizeof(Slot) * size_t(world), create);
  slots_ = reinterpret_cast<Slot*>(region_.base());
}

StepClock::StepClock(int world) : world_(world) {
  if (world < 1) throw std::runtime_error("StepClock: world");
  region_ = Region::anon(sizeof(Slot) * size_t(world));
  slots_ = reinterpret_cast<Slot*>(region_.base());
}

void StepClock::post(int64_t issued) { slots_[rank_].issued.store(issued, std::memory_order_release); }
int64_t StepClock::issued(int r) const { return slots_[r].issued.load(std::memory_order_acquire); }
int64_t StepClock::max_issued() const {
  int64_t m = 0;
  for (int r = 0; r < world_; ++r) m = std::max(m, issued(r));
  return m;
}
void StepClock::hold(int64_t gen) { slots_[rank_].hold.store(gen, std::memory_order_release); }
int64_t StepClock::hold_of(int r) const { return slots_[r].hold.load(std::memory_order_acquire); }
bool StepClock::all_hold(int64_t gen) const {
  for (int r = 0; r < world_; ++r)
    if (hold_of(r) < gen) return false;
  return true;
}

// ============================================================================ items
struct ServeCore::Item {
  int kind = 0;                 // 0: a caller thread waits (batch / rows); 1: unary (finisher pool)
  size_t n = 0;
  std::vector<ReqRec> rows;     // exchange: sorted by owner
  std::vector<int32_t> perm;    // exchange: sorted position -> request row (empty: identity)
  std::vector<int32_t> ostart;  // exchange: [world + 1] owner ranges of `rows`
  std::vector<int32_t> ocur;    // next untaken row per owner (direct: [1])
  int64_t remaining = 0;        // rows not yet in a step (q_mu_)
  int64_t taken = 0;            // rows handed to steps (q_mu_)
  int64_t aborted_rows = 0;     // rows that never reached a step (abort; m)
  int64_t now = 0;
  bool wf = false;
  ResultRec* res = nullptr;     // outputs in request order
  FeatRec* feat = nullptr;
  ResultRec res1{};             // unary storage
  FeatRec feat1{};
  uint64_t tag = 0;
  int64_t t0 = 0, t_enq = 0;
  int64_t t_issue = 0;          // the first step holding rows of this item was formed (q_mu_)
  int32_t seq_first = 0, seq_last = 0;  // batch sequence numbers of its first / last step (q_mu_)
  // completion hand-off (m)
  std::mutex m;
  std::condition_variable cv;
  std::vector<std::pair<Step*, Seg>> ready;
  bool failed = false;
  std::string err;
};

int64_t ServeCore::now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

namespace {
int64_t wall_s() { return int64_t(std::time(nullptr)); }
constexpr size_t kResBytes = sizeof(ResultRec), kFeatBytes = sizeof(FeatRec);
}  // namespace

// ============================================================================ ServeCore
ServeCore::ServeCore(std::vector<std::shared_ptr<AccountIndex>> indexes, const IgpDeviceOps* dev, int rank,
                     std::shared_ptr<StepClock> clock, Options opt)
    : idx_(std::move(indexes)), dev_(dev), rank_(rank), clock_(std::move(clock)), opt_(opt) {
  if (!dev_ || dev_->abi != IGP_DEVICE_OPS_ABI) throw std::runtime_error("ServeCore: device function table ABI mismatch");
  world_ = dev_->world;
  exchange_ = dev_->exchange != 0;
  cap_ = dev_->cap;
  depth_ = dev_->depth;
  if ((int)idx_.size() != world_) throw std::runtime_error("ServeCore: one account index per owner expected");
  if (cap_ < 1 || depth_ < 1) throw std::runtime_error("ServeCore: device capacity / depth");
  if (exchange_ && !clock_) throw std::runtime_error("ServeCore: the exchange needs a StepClock");
  if (exchange_ && clock_->world() != world_) throw std::runtime_error("ServeCore: StepClock world");
  if (!exchange_ && world_ != 1) throw std::runtime_error("ServeCore: a direct device serves one owner");
  for (auto& a : dec_) a.store(0);
  for (auto& a : act_) a.store(0);
  steps_.resize(depth_);
  for (int s = 0; s < depth_; ++s) {
    steps_[s] = std::make_unique<Step>();
    free_slots_.push_back(depth_ - 1 - s);
  }
  if (clock_) issued_.store(clock_->issued(rank_));
  seq_ = opt_.seq0;
  threads_.emplace_back([this] {
    name_thread("core-step");
    stepper_loop();
  });
  threads_.emplace_back([this] {
    name_thread("core-done");
    completion_loop();
  });
  for (int i = 0; i < std::max(1, opt_.finishers); ++i)
    threads_.emplace_back([this] {
      name_thread("core-fin");
      finisher_loop();
    });
  threads_.emplace_back([this] {
    name_thread("core-link");
    link_loop();
  });
}

ServeCore::~ServeCore() {
  try {
    stop();
  } catch (...) {
  }
}

// ---------------------------------------------------------------------------- ingress
void ServeCore::resolve_rows(std::vector<wire::TxRow>& rows, Item* it) {
  const size_t n = rows.size();
  // rows of a request that is answered with response bytes: GPU devices return each row's
  // FeatureVector already encoded (records.h FV_ENC_BIT; CPU devices ignore the bit)
  const int32_t enc = it->wf ? FV_ENC_BIT : 0;
  it->n = n;
  it->rows.resize(n);
  thread_local std::vector<std::string_view> ids;
  thread_local std::vector<uint64_t> hs;
  thread_local std::vector<int32_t> slots;
  ids.resize(n);
  hs.resize(n);
  slots.resize(n);
  if (world_ == 1) {
    for (size_t k = 0; k < n; ++k) {
      ids[k] = rows[k].account;
      hs[k] = rows[k].account_hash;
    }
    idx_[0]->lookup_views(ids.data(), hs.data(), n, true, slots.data(), nullptr);
    for (size_t k = 0; k < n; ++k) {
      it->rows[k] = rows[k].rec;
      it->rows[k].slot = slots[k];
      it->rows[k].tx_type |= enc;
    }
    it->ocur.assign(1, 0);
    it->ostart = {0, int32_t(n)};  // one owner (a world-1 exchange reads the owner ranges too)
  } else {
    // counting sort by owner (owner = digest % world, the registry's routing)
    it->ostart.assign(world_ + 1, 0);
    thread_local std::vector<int32_t> own;
    own.resize(n);
    for (size_t k = 0; k < n; ++k) {
      own[k] = int32_t(rows[k].account_hash % uint64_t(world_));
      ++it->ostart[own[k] + 1];
    }
    for (int o = 0; o < world_; ++o) it->ostart[o + 1] += it->ostart[o];
    it->ocur.assign(it->ostart.begin(), it->ostart.end() - 1);
    std::vector<int32_t> fill(it->ostart.begin(), it->ostart.end() - 1);
    it->perm.resize(n);
    for (size_t k = 0; k < n; ++k) {
      const int32_t pos = fill[own[k]]++;
      it->perm[pos] = int32_t(k);
      ids[pos] = rows[k].account;
      hs[pos] = rows[k].account_hash;
    }
    for (int o = 0; o < world_; ++o) {
      const int32_t b = it->ostart[o], e = it->ostart[o + 1];
      if (e > b) idx_[o]->lookup_views(ids.data() + b, hs.data() + b, size_t(e - b), true, slots.data() + b, nullptr);
    }
    for (size_t pos = 0; pos < n; ++pos) {
      it->rows[pos] = rows[it->perm[pos]].rec;
      it->rows[pos].slot = slots[pos];
      it->rows[pos].tx_type |= enc;
    }
  }
  bool link_room = false;
  if (links_ && n) {  // bounded: links are best-effort under overload (no copy for a full queue)
    std::lock_guard<std::mutex> g(l_mu_);
    link_room = lq_.size() < kLinkQueue;
  }
  if (link_room) {  // (device, account) co-occurrences, off the scoring path
    std::vector<uint64_t> d(n);
    std::vector<int64_t> a(n);
    for (size_t pos = 0; pos < n; ++pos) {
      const int32_t o = world_ == 1 ? 0 : int32_t(rows[it->perm[pos]].account_hash % uint64_t(world_));
      d[pos] = it->rows[pos].dev_hash;
      a[pos] = it->rows[pos].slot >= 0 ? ((int64_t(o) << 32) | it->rows[pos].slot) : -1;
    }
    std::lock_guard<std::mutex> g(l_mu_);
    if (lq_.size() < kLinkQueue) {
      links_->note_queued();  // (a reader of linked accounts waits for the inserts queued before it)
      lq_.emplace_back(std::move(d), std::move(a));
      l_cv_.notify_one();
    }
  }
}

void ServeCore::enqueue(Item* it) {
  it->remaining = int64_t(it->n);
  it->t_enq = now_ns();
  {
    std::lock_guard<std::mutex> lk(q_mu_);
    if (stopping_ || stopped_) throw std::runtime_error("ServeCore: stopped");
    queue_.push_back(it);
    queued_rows_ += int64_t(it->n);
  }
  q_cv_.notify_all();
}

void ServeCore::wait_item(Item* it) {
  size_t done = 0;
  std::unique_lock<std::mutex> l(it->m);
  while (done + size_t(it->aborted_rows) < it->n) {
    it->cv.wait(l, [&] { return !it->ready.empty() || done + size_t(it->aborted_rows) >= it->n; });
    std::vector<std::pair<Step*, Seg>> batch;
    batch.swap(it->ready);
    l.unlock();
    const int64_t t = now_ns();
    for (auto& [st, seg] : batch) {
      if (st->failed) {
        it->failed = true;
        if (it->err.empty()) it->err = st->err;
      } else {
        finish_seg(*st, seg);
      }
      done += size_t(seg.count);
      release_step_ref(st);
    }
    a_copy_.fetch_add(now_ns() - t, std::memory_order_relaxed);
    l.lock();
  }
}

std::string ServeCore::score_batch(const char* data, size_t n, int64_t now, int64_t t0_ns) {
  const std::string_view v = score_batch_view(data, n, now, t0_ns);
  return std::string(v.data(), v.size());
}

std::string_view ServeCore::score_batch_view(const char* data, size_t n, int64_t now, int64_t t0_ns) {
  const int64_t t0 = t0_ns > 0 ? t0_ns : now_ns();
  thread_local std::vector<wire::TxRow> rows;
  rows.clear();
  const int64_t ta = now_ns();
  wire::parse_batch_rows(data, n, rows);
  const int64_t tb = now_ns();
  if (rows.empty()) return {};
  Item it;
  // the item's packed rows reuse this thread's buffer: a fresh 512 KB vector per 8192-row
  // request was an mmap'd allocation, zero-filled and page-faulted every time (~8 % of the
  // ingress threads' samples; same-box A/B 4 runs each: 121.7 vs 114.8 M scores/s, p99 1.47 vs
  // 1.79 ms, profiles/r5/host); the item is done with its rows when wait_item returns
  thread_local std::vector<ReqRec> rows_buf;
  it.rows.swap(rows_buf);
  struct GiveBack {
    std::vector<ReqRec>& buf;
    Item& item;
    ~GiveBack() { buf.swap(item.rows); }
  } give_back{rows_buf, it};
  it.kind = 0;
  it.now = now >= 0 ? now : wall_s();
  it.wf = opt_.features;
  resolve_rows(rows, &it);
  const int64_t tc = now_ns();
  thread_local std::vector<ResultRec> res;
  thread_local std::vector<FeatRec> feat;
  res.resize(it.n);
  if (it.wf) feat.resize(it.n);
  it.res = res.data();
  it.feat = it.wf ? feat.data() : nullptr;
  enqueue(&it);
  const int64_t tq = it.t_enq;
  wait_item(&it);
  if (it.failed) throw std::runtime_error("ServeCore: batch failed: " + it.err);
  const int64_t td = now_ns();
  const std::string_view out = wire::batch_response_scratch(it.res, it.feat, nullptr, (td - t0) / 1000000, it.n);
  const int64_t te = now_ns();
  // this call's stage times (last_timings(): per-request tails, not only sums)
  CallTimings& ct = last_timings_tl();
  ct = CallTimings{tb - ta, tc - tb, it.t_issue - tq, td - it.t_issue, te - td, te - t0, int64_t(it.n), it.seq_first,
                   it.seq_last};
  a_parse_.fetch_add(tb - ta, std::memory_order_relaxed);
  a_resolve_.fetch_add(tc - tb, std::memory_order_relaxed);
  a_serialize_.fetch_add(te - td, std::memory_order_relaxed);
  a_items_.fetch_add(1, std::memory_order_relaxed);
  a_rows_.fetch_add(int64_t(it.n), std::memory_order_relaxed);
  return out;
}

void ServeCore::score_rows(const ReqRec* rows, const int32_t* owners, size_t n, int64_t now, bool want_features,
                           ResultRec* res, FeatRec* feat) {
  if (n == 0) return;
  Item it;
  it.kind = 0;
  it.n = n;
  it.now = now >= 0 ? now : wall_s();
  it.wf = want_features && feat != nullptr;
  it.res = res;
  it.feat = it.wf ? feat : nullptr;
  if (world_ == 1) {
    it.rows.assign(rows, rows + n);
    it.ocur.assign(1, 0);
    it.ostart = {0, int32_t(n)};
  } else {
    if (!owners) throw std::runtime_error("ServeCore.score_rows: owners required when world > 1");
    it.ostart.assign(world_ + 1, 0);
    for (size_t k = 0; k < n; ++k) {
      if (owners[k] < 0 || owners[k] >= world_) throw std::runtime_error("ServeCore.score_rows: owner out of range");
      ++it.ostart[owners[k] + 1];
    }
    for (int o = 0; o < world_; ++o) it.ostart[o + 1] += it.ostart[o];
    it.ocur.assign(it.ostart.begin(), it.ostart.end() - 1);
    std::vector<int32_t> fill(it.ocur);
    it.perm.resize(n);
    it.rows.resize(n);
    for (size_t k = 0; k < n; ++k) {
      const int32_t pos = fill[owners[k]]++;
      it.perm[pos] = int32_t(k);
      it.rows[pos] = rows[k];
    }
  }
  enqueue(&it);
  wait_item(&it);
  if (it.failed) throw std::runtime_error("ServeCore: batch failed: " + it.err);
}

void ServeCore::submit_tx(const char* data, size_t n, uint64_t tag, int64_t now, int64_t t0_ns) {
  auto* it = new Item();
  it->kind = 1;
  it->tag = tag;
  it->t0 = t0_ns > 0 ? t0_ns : now_ns();
  it->now = now >= 0 ? now : wall_s();
  it->wf = opt_.features;
  it->res = &it->res1;
  it->feat = it->wf ? &it->feat1 : nullptr;
  try {
    std::vector<wire::TxRow> rows(1);
    wire::parse_tx_row(data, n, rows[0]);
    resolve_rows(rows, it);
    enqueue(it);
  } catch (const std::exception& e) {
    std::vector<Done> d;
    d.push_back(Done{tag, std::string(), e.what()});
    delete it;
    deliver(std::move(d));
  }
}

void ServeCore::submit_tx_many(const TxCall* calls, size_t n, int64_t now) {
  if (n == 0) return;
  thread_local std::vector<wire::TxRow> rows;
  thread_local std::vector<Item*> items;
  thread_local std::vector<std::string_view> ids;
  thread_local std::vector<uint64_t> hs;
  thread_local std::vector<int32_t> slots;
  thread_local std::vector<uint8_t> ok;
  rows.resize(n);
  items.assign(n, nullptr);
  ok.assign(n, 0);
  std::vector<Done> bad;
  const int64_t wnow = now >= 0 ? now : wall_s();
  const int32_t enc = opt_.features ? FV_ENC_BIT : 0;
  for (size_t k = 0; k < n; ++k) {
    try {
      wire::parse_tx_row(calls[k].data, calls[k].n, rows[k]);
      ok[k] = 1;
    } catch (const std::exception& e) {
      bad.push_back(Done{calls[k].tag, std::string(), e.what()});
    }
  }
  if (world_ == 1) {  // one batched lookup for the account ids of every call
    ids.resize(n);
    hs.resize(n);
    slots.assign(n, -1);
    size_t m = 0;
    for (size_t k = 0; k < n; ++k)
      if (ok[k]) {
        ids[m] = rows[k].account;
        hs[m] = rows[k].account_hash;
        ++m;
      }
    idx_[0]->lookup_views(ids.data(), hs.data(), m, true, slots.data(), nullptr);
    m = 0;
    for (size_t k = 0; k < n; ++k) {
      if (!ok[k]) continue;
      auto* it = new Item();
      it->kind = 1;
      it->tag = calls[k].tag;
      it->t0 = calls[k].t0_ns > 0 ? calls[k].t0_ns : now_ns();
      it->now = wnow;
      it->wf = opt_.features;
      it->res = &it->res1;
      it->feat = it->wf ? &it->feat1 : nullptr;
      it->n = 1;
      it->rows.resize(1);
      it->rows[0] = rows[k].rec;
      it->rows[0].slot = slots[m++];
      it->rows[0].tx_type |= enc;
      it->ocur.assign(1, 0);
      it->ostart = {0, 1};
      items[k] = it;
    }
    if (links_ && m) {  // (device, account) co-occurrences of every call: ONE link job for the batch
      std::vector<uint64_t> d;
      std::vector<int64_t> acc;
      d.reserve(m);
      acc.reserve(m);
      for (Item* it : items)
        if (it) {
          d.push_back(it->rows[0].dev_hash);
          acc.push_back(it->rows[0].slot >= 0 ? int64_t(it->rows[0].slot) : -1);
        }
      std::lock_guard<std::mutex> g(l_mu_);
      if (lq_.size() < kLinkQueue) {  // bounded: links are best-effort under overload (as resolve_rows)
        links_->note_queued();
        lq_.emplace_back(std::move(d), std::move(acc));
        l_cv_.notify_one();
      }
    }
  } else {  // owner routing per call (resolve_rows sorts one call's row by owner)
    for (size_t k = 0; k < n; ++k) {
      if (!ok[k]) continue;
      auto* it = new Item();
      it->kind = 1;
      it->tag = calls[k].tag;
      it->t0 = calls[k].t0_ns > 0 ? calls[k].t0_ns : now_ns();
      it->now = wnow;
      it->wf = opt_.features;
      it->res = &it->res1;
      it->feat = it->wf ? &it->feat1 : nullptr;
      std::vector<wire::TxRow> one(1, rows[k]);
      resolve_rows(one, it);
      items[k] = it;
    }
  }
  const int64_t t_enq = now_ns();
  bool stopped = false;
  {
    std::lock_guard<std::mutex> lk(q_mu_);
    stopped = stopping_ || stopped_;
    if (!stopped) {
      for (Item* it : items)
        if (it) {
          it->remaining = int64_t(it->n);
          it->t_enq = t_enq;
          uqueue_.push_back(it);
          queued_rows_ += int64_t(it->n);
        }
      last_unary_ns_ = t_enq;
    }
  }
  if (stopped) {
    for (size_t k = 0; k < n; ++k)
      if (items[k]) {
        bad.push_back(Done{items[k]->tag, std::string(), "ServeCore: stopped"});
        delete items[k];
      }
  } else {
    q_cv_.notify_all();
  }
  if (!bad.empty()) deliver(std::move(bad));
}

void ServeCore::deliver(std::vector<Done>&& outs) {
  Sink sink;
  {
    std::lock_guard<std::mutex> g(out_mu_);
    sink = sink_;
    if (!sink) {
      for (auto& d : outs) outq_.push_back(std::move(d));
      outs.clear();
    } else {
      // tags of the native server go to its sink, the others to poll()
      size_t k = 0;
      for (size_t i = 0; i < outs.size(); ++i) {
        if (outs[i].tag & kSinkTag) {
          if (k != i) outs[k] = std::move(outs[i]);  // (a self-move would empty the strings)
          ++k;
        } else {
          outq_.push_back(std::move(outs[i]));
        }
      }
      outs.resize(k);
    }
  }
  out_cv_.notify_all();
  if (sink && !outs.empty()) sink(std::move(outs));
}

size_t ServeCore::poll(std::vector<Done>& out, size_t max, int64_t timeout_us) {
  std::unique_lock<std::mutex> l(out_mu_);
  if (outq_.empty() && timeout_us != 0) {
    if (timeout_us < 0) out_cv_.wait(l, [&] { return !outq_.empty(); });
    else out_cv_.wait_for(l, std::chrono::microseconds(timeout_us), [&] { return !outq_.empty(); });
  }
  size_t k = 0;
  while (!outq_.empty() && k < max) {
    out.push_back(std::move(outq_.front()));
    outq_.pop_front();
    ++k;
  }
  return k;
}

int ServeCore::pending_items() {
  std::lock_guard<std::mutex> lk(q_mu_);
  return int(queue_.size() + uqueue_.size());
}

// ---------------------------------------------------------------------------- stepper
// Takes rows from the FIFO into the next free slot and launches it. Called with q_mu_ held
// (released around the copy into the pinned buffer and the device calls).
// The pipeline slot the next step runs on, or -1 when it is busy. Exchange mode: slot =
// step index % depth on EVERY rank (steps are issued in the same sequence everywhere), so a step
// uses the same slot index on all ranks - the per-GPU D2H result path indexes its node-shared
// region and generation flags by slot (with a free-slot stack, ranks released steps in
// different orders and could run one step on different slots). Direct mode: any free slot.
int ServeCore::next_slot_locked() const {
  if (!exchange_) {
    if (free_slots_.empty()) return -1;
    if (opt_.unary_depth > 0 && inflight_ >= opt_.unary_depth && now_ns() - last_unary_ns_ < kUnaryWindowNs) return -1;
    return free_slots_.back();
  }
  const int s = int(issued_.load() % int64_t(depth_));
  return std::find(free_slots_.begin(), free_slots_.end(), s) != free_slots_.end() ? s : -1;
}

bool ServeCore::issue_step(std::unique_lock<std::mutex>& lk, bool allow_empty) {
  const int slot = next_slot_locked();
  if (slot < 0) return false;
  Step* st = steps_[slot].get();
  st->slot = slot;
  st->segs.clear();
  st->failed = false;
  st->err.clear();
  st->wf = false;
  int64_t now = 0;
  int n = 0;
  thread_local std::vector<int32_t> fill;
  if (!exchange_) {
    for (std::deque<Item*>* q : {&uqueue_, &queue_}) {  // unary calls first
      while (!q->empty() && n < cap_) {
        Item* it = q->front();
        const int take = int(std::min<int64_t>(it->remaining, cap_ - n));
        st->segs.push_back(Seg{it, 0, it->ocur[0], n, take});
        it->ocur[0] += take;
        it->remaining -= take;
        it->taken += take;
        if (!it->t_issue) it->t_issue = now_ns();
        n += take;
        now = std::max(now, it->now);
        st->wf |= it->wf;
        if (it->remaining == 0) q->pop_front();
      }
    }
  } else {
    fill.assign(world_, 0);
    int full = 0;
    for (std::deque<Item*>* q : {&uqueue_, &queue_}) {  // unary calls first
      for (auto qi = q->begin(); qi != q->end() && full < world_;) {
        Item* it = *qi;
        bool took = false;
        for (int o = 0; o < world_; ++o) {
          const int avail = it->ostart[o + 1] - it->ocur[o];
          if (avail <= 0 || fill[o] >= cap_) continue;
          const int take = std::min(avail, cap_ - fill[o]);
          st->segs.push_back(Seg{it, o, it->ocur[o], fill[o], take});
          it->ocur[o] += take;
          it->remaining -= take;
          it->taken += take;
          if (!it->t_issue) it->t_issue = now_ns();
          fill[o] += take;
          n += take;
          if (fill[o] == cap_) ++full;
          took = true;
        }
        if (took) {
          now = std::max(now, it->now);
          st->wf |= it->wf;
        }
        qi = it->remaining == 0 ? q->erase(qi) : qi + 1;
      }
    }
  }
  if (n == 0 && !allow_empty) return false;
  free_slots_.erase(std::find(free_slots_.begin(), free_slots_.end(), slot));
  queued_rows_ -= n;
  ++inflight_;
  st->n = n;
  st->refs.store(int(st->segs.size()) + 1);  // + the completion thread's own reference
  if (dev_->features_always) st->wf = true;
  if (now == 0) now = wall_s();
  const int32_t seq = ++seq_;
  st->seq = seq;
  for (const Seg& sg : st->segs) {  // the steps an item's rows ride in (the ordering contract, dp.py)
    if (!sg.item->seq_first) sg.item->seq_first = seq;
    sg.item->seq_last = seq;
  }
  lk.unlock();
  // pack the rows into the slot's pinned buffer (outside the queue lock)
  const int64_t t0 = now_ns();
  char* buf = dev_->rows(dev_->ctx, slot);
  if (!exchange_) {
    for (const Seg& s : st->segs)
      std::memcpy(buf + size_t(s.dev_pos) * sizeof(ReqRec), s.item->rows.data() + s.item_pos,
                  size_t(s.count) * sizeof(ReqRec));
  } else {
    ReqRec* chunks = reinterpret_cast<ReqRec*>(buf);
    const size_t stride = size_t(cap_) + 1;
    for (int o = 0; o < world_; ++o) {
      ReqRec& h = chunks[size_t(o) * stride];
      std::memset(&h, 0, sizeof h);
      h.slot = fill[o];  // row count of owner o's chunk
      h.ts = now;        // this sender's clock: the owner scores the step at its senders' latest
    }
    for (const Seg& s : st->segs)
      std::memcpy(chunks + size_t(s.owner) * stride + 1 + s.dev_pos, s.item->rows.data() + s.item_pos,
                  size_t(s.count) * sizeof(ReqRec));
  }
  const int64_t t1 = now_ns();
  // the step is announced before the launch: an exchange device may block inside submit until
  // every peer reached this step, and an idle peer only issues it once it sees us ahead
  const int64_t issued = issued_.fetch_add(1) + 1;
  if (clock_) clock_->post(issued);
  char err[256] = {0};
  const int rc = dev_->submit(dev_->ctx, slot, n, seq, now, st->wf ? 1 : 0, err, sizeof err);
  const int64_t t2 = now_ns();
  st->t_submit = t2;
  if (rc != 0) {
    st->failed = true;
    st->err = err[0] ? err : "device submit failed";
  }
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.pack_ns += t1 - t0;
    st_.submit_ns += t2 - t1;
    st_.steps += 1;
    if (n == 0) st_.empty_steps += 1;
    st_.max_step_rows = std::max<int64_t>(st_.max_step_rows, n);
    for (const Seg& s : st->segs) {
      if (s.item->kind == 1) st_.unary += 1;
    }
  }
  {
    std::lock_guard<std::mutex> g(c_mu_);
    done_fifo_.push_back(st);
  }
  c_cv_.notify_one();
  lk.lock();
  return true;
}

void ServeCore::note_wait(int64_t ServeStats::*field, int64_t ns) {
  std::lock_guard<std::mutex> g(st_mu_);
  st_.*field += ns;
}

void ServeCore::stepper_loop() {
  std::unique_lock<std::mutex> lk(q_mu_);
  const int64_t max_wait = int64_t(opt_.max_wait_us) * 1000;
  const int64_t full_rows = exchange_ ? int64_t(cap_) * world_ * 7 / 8 : int64_t(cap_);
  int64_t hold_since = 0;
  for (;;) {
    if (aborting_) {  // failover: no convergence with peers that may be dead
      stopped_ = true;
      idle_cv_.notify_all();
      return;
    }
    const bool peer_ahead = exchange_ && clock_->max_issued() > issued_.load();
    // pause / stop: converge on a generation (exchange: every rank at the same step count)
    const bool draining = stopping_ && queue_.empty() && uqueue_.empty();
    if (pause_req_ || draining) {
      const int64_t gen = hold_gen_;
      if (!held_) {
        if (clock_) clock_->hold(gen);
        held_ = true;
        hold_since = now_ns();
      }
      if (peer_ahead) {
        if (next_slot_locked() >= 0) {
          issue_step(lk, true);
          continue;
        }
      } else if (!exchange_ || (clock_->all_hold(gen) && clock_->max_issued() == issued_.load())) {
        if (inflight_ == 0) {
          if (draining) {
            stopped_ = true;
            idle_cv_.notify_all();
            return;
          }
          paused_ = true;
          idle_cv_.notify_all();
          q_cv_.wait(lk, [&] { return !pause_req_ || stopping_; });
          paused_ = false;
          held_ = false;
          continue;
        }
      } else if (stopping_ && now_ns() - hold_since > opt_.stop_timeout_us * 1000) {
        stopped_ = true;  // a peer never converged (died): give up
        idle_cv_.notify_all();
        return;
      }
      q_cv_.wait_for(lk, std::chrono::microseconds(exchange_ ? 50 : 1000));
      continue;
    }
    const bool slot = next_slot_locked() >= 0;
    if (slot && (queued_rows_ > 0 || peer_ahead)) {
      const int64_t t_front = std::min(queue_.empty() ? INT64_MAX : queue_.front()->t_enq,
                                       uqueue_.empty() ? INT64_MAX : uqueue_.front()->t_enq);
      const int64_t age = t_front == INT64_MAX ? 0 : now_ns() - t_front;
      if (peer_ahead || inflight_ == 0 || queued_rows_ >= full_rows || age >= max_wait) {
        issue_step(lk, peer_ahead);
        continue;
      }
      const int64_t w0 = now_ns();
      q_cv_.wait_for(lk, std::chrono::nanoseconds(std::max<int64_t>(max_wait - age, 1000)));
      note_wait(&ServeStats::rows_wait_ns, now_ns() - w0);
      continue;
    }
    // nothing to issue: sleep until new work / a free slot; exchange ranks also watch the peers
    const bool blocked = !slot && queued_rows_ > 0;
    const int64_t w0 = blocked ? now_ns() : 0;
    if (exchange_) q_cv_.wait_for(lk, std::chrono::microseconds(50));
    else q_cv_.wait_for(lk, std::chrono::milliseconds(100));
    if (blocked) {
      note_wait(&ServeStats::slot_wait_ns, now_ns() - w0);
      note_wait(&ServeStats::slot_waits, 1);
      note_wait(&ServeStats::slot_wait_inflight, inflight_);
    }
  }
}

// ---------------------------------------------------------------------------- completion
void ServeCore::completion_loop() {
  for (;;) {
    Step* st;
    {
      std::unique_lock<std::mutex> l(c_mu_);
      c_cv_.wait(l, [&] { return c_stop_ || !done_fifo_.empty(); });
      if (done_fifo_.empty()) return;
      st = done_fifo_.front();
      done_fifo_.pop_front();
    }
    bool late = false;  // overran its deadline: answered as failed, slot kept until it drains
    if (!st->failed) {
      char err[256] = {0};
      const int rc = dev_->wait(dev_->ctx, st->slot, opt_.timeout_us, err, sizeof err);
      if (rc != 0) {
        st->failed = true;
        late = rc == 1;
        st->err = rc == 1 ? "device step exceeded its deadline" : (err[0] ? err : "device wait failed");
        std::lock_guard<std::mutex> g(st_mu_);
        st_.wait_errors += 1;
      }
    }
    const int64_t t = now_ns();
    st->t_done = t;
    {
      std::lock_guard<std::mutex> g(st_mu_);
      st_.device_ns += t - st->t_submit;
    }
    std::vector<Seg> unary;
    for (const Seg& s : st->segs) {
      if (s.item->kind == 1) {
        unary.push_back(s);
        continue;
      }
      // notify under the item's lock: a waiter whose rows are now complete returns (and a
      // batch item on its stack goes away) only after this lock is released
      std::lock_guard<std::mutex> g(s.item->m);
      s.item->ready.emplace_back(st, s);
      s.item->cv.notify_one();
    }
    if (!unary.empty()) {
      const size_t nf = size_t(std::max(1, opt_.finishers));
      const size_t per = std::max<size_t>(64, (unary.size() + nf - 1) / nf);
      std::lock_guard<std::mutex> g(f_mu_);
      for (size_t b = 0; b < unary.size(); b += per) {
        FTask task{st, std::vector<Seg>(unary.begin() + b, unary.begin() + std::min(unary.size(), b + per))};
        ftasks_.push_back(std::move(task));
      }
      f_cv_.notify_all();
    }
    if (late) {
      // the device may still read the slot's pinned rows and write its results: the slot
      // stays out of service until the late step really finished (watchdog quarantine)
      late_.fetch_add(1);
      char err[256] = {0};
      (void)dev_->wait(dev_->ctx, st->slot, -1, err, sizeof err);
      late_.fetch_sub(1);
    }
    release_step_ref(st);  // the completion thread's own reference
  }
}

void ServeCore::finish_seg(const Step& st, const Seg& s) {
  Item* it = s.item;
  const char* base = static_cast<const char*>(dev_->results(dev_->ctx, st.slot));
  if (!exchange_) {
    const ResultRec* r = reinterpret_cast<const ResultRec*>(base) + s.dev_pos;
    std::memcpy(it->res + s.item_pos, r, size_t(s.count) * kResBytes);
    if (it->feat) {
      const FeatRec* f = static_cast<const FeatRec*>(dev_->features(dev_->ctx, st.slot));
      if (f) std::memcpy(it->feat + s.item_pos, f + s.dev_pos, size_t(s.count) * kFeatBytes);
    }
    record_decisions(r, s.count);
    audit_seg(r, it->rows.data() + s.item_pos, 0, s.count);
    return;
  }
  const size_t W = kResBytes + (st.wf ? kFeatBytes : 0);
  const size_t ostride = dev_->res_owner_stride > 0 ? size_t(dev_->res_owner_stride) : size_t(cap_) * W;
  const char* chunk = base + size_t(s.owner) * ostride;
  const ResultRec* r = reinterpret_cast<const ResultRec*>(chunk) + s.dev_pos;
  const FeatRec* f = st.wf ? reinterpret_cast<const FeatRec*>(chunk + size_t(cap_) * kResBytes) + s.dev_pos : nullptr;
  const int32_t* perm = it->perm.empty() ? nullptr : it->perm.data() + s.item_pos;
  for (int i = 0; i < s.count; ++i) {
    const int32_t dst = perm ? perm[i] : s.item_pos + i;
    it->res[dst] = r[i];
    if (it->feat && f) it->feat[dst] = f[i];
  }
  record_decisions(r, s.count);
  audit_seg(r, it->rows.data() + s.item_pos, s.owner, s.count);
}

void ServeCore::audit_seg(const ResultRec* r, const ReqRec* rows, int owner, int n) {
  AuditRing* a = audit_.get();
  if (!a || n <= 0) return;
  const int64_t t_ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                           std::chrono::system_clock::now().time_since_epoch()).count();
  a->append(r, &rows[0].slot, sizeof(ReqRec) / sizeof(int32_t), owner, size_t(n), t_ms, model_ver_.load());
}

// decision counters of /metrics (obs/metrics.py): score deciles, actions, ML high-risk and
// blacklist bits of the packed result word; one atomic add per counter per segment
void ServeCore::record_decisions(const ResultRec* r, int n) {
  int64_t dec[11] = {0}, act[4] = {0}, hi = 0, bl = 0;
  for (int i = 0; i < n; ++i) {
    const uint32_t p = r[i].packed;
    ++dec[std::min<uint32_t>(IGP_RES_SCORE(p) / 10, 10)];
    ++act[IGP_RES_ACTION(p)];
    hi += (p >> 28) & 1;
    bl += (p >> 27) & 1;
  }
  for (int k = 0; k < 11; ++k)
    if (dec[k]) dec_[k].fetch_add(dec[k], std::memory_order_relaxed);
  for (int k = 0; k < 4; ++k)
    if (act[k]) act_[k].fetch_add(act[k], std::memory_order_relaxed);
  if (hi) hi_.fetch_add(hi, std::memory_order_relaxed);
  if (bl) bl_.fetch_add(bl, std::memory_order_relaxed);
  scored_.fetch_add(n, std::memory_order_relaxed);
}

void ServeCore::release_step_ref(Step* st) {
  if (st->refs.fetch_sub(1) != 1) return;
  if (st->t_done) {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.release_ns += now_ns() - st->t_done;
  }
  st->t_done = 0;
  {
    std::lock_guard<std::mutex> lk(q_mu_);
    free_slots_.push_back(st->slot);
    --inflight_;
  }
  q_cv_.notify_all();
  idle_cv_.notify_all();
}

void ServeCore::finisher_loop() {
  for (;;) {
    FTask task;
    {
      std::unique_lock<std::mutex> l(f_mu_);
      f_cv_.wait(l, [&] { return f_stop_ || !ftasks_.empty(); });
      if (ftasks_.empty()) return;
      task = std::move(ftasks_.front());
      ftasks_.pop_front();
    }
    std::vector<Done> outs;
    outs.reserve(task.segs.size());
    const int64_t t = now_ns();
    for (const Seg& s : task.segs) {
      Item* it = s.item;
      Done d{it->tag, std::string(), std::string()};
      if (task.step->failed) {
        d.err = task.step->err;
      } else {
        finish_seg(*task.step, s);
        char body[wire::kMaxTxResponse];
        const size_t len = wire::write_tx_response(body, it->res1, it->feat, (t - it->t0) / 1000000);
        d.bytes.assign(body, len);
      }
      outs.push_back(std::move(d));
      delete it;
      release_step_ref(task.step);
    }
    a_serialize_.fetch_add(now_ns() - t, std::memory_order_relaxed);
    a_items_.fetch_add(int64_t(outs.size()), std::memory_order_relaxed);
    a_rows_.fetch_add(int64_t(outs.size()), std::memory_order_relaxed);
    deliver(std::move(outs));
  }
}

void ServeCore::link_loop() {
  for (;;) {
    std::pair<std::vector<uint64_t>, std::vector<int64_t>> job;
    {
      std::unique_lock<std::mutex> l(l_mu_);
      l_cv_.wait(l, [&] { return l_stop_ || !lq_.empty(); });
      if (lq_.empty()) return;
      job = std::move(lq_.front());
      lq_.pop_front();
    }
    if (links_) {
      links_->add(job.first.data(), job.second.data(), job.first.size());
      links_->note_done();
    }
  }
}

// ---------------------------------------------------------------------------- control
void ServeCore::pause() {
  std::unique_lock<std::mutex> lk(q_mu_);
  if (stopped_) throw std::runtime_error("ServeCore: stopped");
  if (paused_ || pause_req_) throw std::runtime_error("ServeCore: already paused");
  pause_req_ = true;
  hold_gen_ = ++gen_;
  q_cv_.notify_all();
  idle_cv_.wait(lk, [&] { return paused_ || stopped_; });
}

void ServeCore::resume() {
  {
    std::lock_guard<std::mutex> lk(q_mu_);
    pause_req_ = false;
  }
  q_cv_.notify_all();
}

void ServeCore::set_device(const IgpDeviceOps* dev) {
  std::lock_guard<std::mutex> lk(q_mu_);
  if (!paused_) throw std::runtime_error("ServeCore.set_device: pause() first");
  if (!dev || dev->abi != IGP_DEVICE_OPS_ABI) throw std::runtime_error("ServeCore.set_device: ABI mismatch");
  if (dev->world != world_ || (dev->exchange != 0) != exchange_)
    throw std::runtime_error("ServeCore.set_device: the new device must have the same world / mode");
  dev_ = dev;
  cap_ = dev->cap;
  depth_ = dev->depth;
  steps_.clear();
  free_slots_.clear();
  steps_.resize(depth_);
  for (int s = 0; s < depth_; ++s) {
    steps_[s] = std::make_unique<Step>();
    free_slots_.push_back(depth_ - 1 - s);
  }
}

void ServeCore::abort() {
  std::deque<Item*> dropped;
  {
    std::unique_lock<std::mutex> lk(q_mu_);
    if (threads_.empty()) return;
    aborting_ = true;
    stopping_ = true;
    dropped.swap(queue_);
    dropped.insert(dropped.end(), uqueue_.begin(), uqueue_.end());
    uqueue_.clear();
    queued_rows_ = 0;
  }
  q_cv_.notify_all();
  // queued items never reach a step: fail them now (rows already in steps fail or finish with
  // their steps). Unary failures go through deliver(): sink-tagged calls (the native gRPC
  // server) reach their connection instead of the poll() queue nobody drains
  std::vector<Done> unary;
  for (Item* it : dropped) {
    if (it->kind == 1) {
      unary.push_back(Done{it->tag, std::string(), "ServeCore: aborted"});
      delete it;
      continue;
    }
    std::lock_guard<std::mutex> g(it->m);
    it->failed = true;
    it->err = "ServeCore: aborted";
    it->aborted_rows = int64_t(it->n) - it->taken;
    it->cv.notify_one();
  }
  deliver(std::move(unary));
  stop();
}

void ServeCore::stop() {
  {
    std::unique_lock<std::mutex> lk(q_mu_);
    if (threads_.empty()) return;
    if (!stopping_) {
      stopping_ = true;
      pause_req_ = false;
      held_ = false;
      hold_gen_ = ++gen_;
    }
  }
  q_cv_.notify_all();
  threads_[0].join();  // stepper: drained the queue, converged, every step completed
  {
    std::lock_guard<std::mutex> g(c_mu_);
    c_stop_ = true;
  }
  c_cv_.notify_all();
  threads_[1].join();
  {
    std::lock_guard<std::mutex> g(f_mu_);
    f_stop_ = true;
  }
  f_cv_.notify_all();
  {
    std::lock_guard<std::mutex> g(l_mu_);
    l_stop_ = true;
  }
  l_cv_.notify_all();
  for (size_t i = 2; i < threads_.size(); ++i) threads_[i].join();
  threads_.clear();
}

ServeStats ServeCore::stats(bool reset) {
  ServeStats s;
  {
    std::lock_guard<std::mutex> g(st_mu_);
    s = st_;
    if (reset) st_ = ServeStats();
  }
  auto take = [&](std::atomic<int64_t>& a) { return reset ? a.exchange(0) : a.load(); };
  s.parse_ns = take(a_parse_);
  s.resolve_ns = take(a_resolve_);
  s.serialize_ns = take(a_serialize_);
  s.copy_ns = take(a_copy_);
  s.items = take(a_items_);
  s.rows = take(a_rows_);
  for (int k = 0; k < 4; ++k) s.actions[k] = act_[k].load();
  for (int k = 0; k < 11; ++k) s.deciles[k] = dec_[k].load();
  s.ml_high = hi_.load();
  s.blacklisted = bl_.load();
  s.scored = scored_.load();
  return s;
}

}  // namespace igp

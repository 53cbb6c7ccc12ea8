#include "acct_core.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <ctime>
#include <stdexcept>

#include "pb.h"
#include "xxh64.h"
#include "thread_name.h"

namespace igp {

namespace {

int64_t mono_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void wall_now(int64_t& sec, int32_t& nanos) {
  const int64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(
                         std::chrono::system_clock::now().time_since_epoch()).count();
  sec = ns / 1000000000;
  nanos = int32_t(ns % 1000000000);
}

constexpr int kInvalidArgument = 3, kInternal = 13, kUnavailable = 14;

}  // namespace

// ============================================================================ wire
namespace acctwire {

const char* const kNbaCodes[13] = {
    "NO_ACTION", "SEND_WINBACK_BONUS", "SEND_ENGAGEMENT_EMAIL", "VIP_MANAGER_CALL", "EXCLUSIVE_EVENT_INVITE",
    "ASSIGN_VIP_MANAGER", "RETENTION_BONUS", "LOYALTY_REWARD", "SUGGEST_BONUS", "RECOMMEND_NEW_GAMES",
    "STANDARD_PROMOTION", "ONBOARDING_GUIDE", "SMALL_DEPOSIT_BONUS"};  // golden/ltv.py NBA_CODES

namespace {
// golden/ltv.py SEGMENT_PLAYBOOK: NBA ids of each segment's generic actions (index = segment)
const int kPlaybook[6][2] = {{-1, -1}, {4, 3}, {7, 6}, {10, 8}, {12, 11}, {1, 2}};
const char* const kSignals[8] = {"BONUS_ONLY_PLAYER", "LOW_WAGER_COMPLETION", "MULTIPLE_DEVICES", "MULTIPLE_IPS",
                                 "VPN_PROXY_TOR",     "HIGH_VELOCITY",        "SHARED_DEVICE",    "SEQUENCE_MODEL"};

int nba_of(float v) {
  const int k = int(v);
  return k >= 0 && k < 13 ? k : 0;
}
}  // namespace

void parse_request(const char* data, size_t n, std::string_view& account, std::string_view& bonus) {
  pb::Reader r(data, n);
  uint32_t f, w;
  account = {};
  bonus = {};
  while (r.tag(f, w)) {
    if (f == 1 && w == pb::LEN) account = r.bytes();
    else if (f == 2 && w == pb::LEN) bonus = r.bytes();
    else r.skip(w);
  }
}

// PredictLTVResponse (risk.proto:95-108); Python twin: api/grpc_server.py RiskServicer.ltv_response
void write_ltv(std::string& out, std::string_view account, const float* row, int64_t sec, int32_t nanos) {
  pb::Writer w;
  w.buf.reserve(96 + account.size());
  w.str(1, account);
  w.f32(2, row[0]);
  w.i32(3, int32_t(row[4]));
  w.f32(4, row[1]);
  w.i32(5, int32_t(double(row[2])));  // int(float): truncation
  w.f32(6, row[3]);
  w.str(7, kNbaCodes[nba_of(row[5])]);
  // Timestamp sub-message sized first and written in place (no second buffer per answer)
  pb::Sizer ts;
  ts.i64(1, sec);
  ts.i32(2, nanos);
  w.msg_header(8, ts.n);
  w.i64(1, sec);
  w.i32(2, nanos);
  out = std::move(w.buf);
}

// GetPlayerSegmentResponse (risk.proto:110-120): recommended_actions = the NBA, then the
// segment's playbook without repeats (engine/ltv.py recommended_from)
void write_segment(std::string& out, std::string_view account, const float* row) {
  pb::Writer w;
  w.buf.reserve(96 + account.size());
  const int seg = int(row[4]);
  w.str(1, account);
  w.i32(2, seg);
  w.f32(3, row[0]);
  w.f32(4, row[1]);
  const int nba = nba_of(row[5]);
  w.str_always(5, kNbaCodes[nba]);
  if (seg >= 0 && seg < 6)
    for (int k = 0; k < 2; ++k) {
      const int a = kPlaybook[seg][k];
      if (a >= 0 && a != nba) w.str_always(5, kNbaCodes[a]);
    }
  out = std::move(w.buf);
}

// CheckBonusAbuseResponse (risk.proto:135-145)
void write_abuse(std::string& out, bool is_abuser, float score, const std::vector<std::string_view>& signals,
                 const std::vector<std::string_view>& linked) {
  pb::Writer w;
  w.boolean(1, is_abuser);
  w.f32(2, score);
  for (auto s : signals) w.str_always(3, s);
  for (auto s : linked) w.str_always(4, s);
  out = std::move(w.buf);
}

}  // namespace acctwire

// ============================================================================ AcctCore
AcctCore::AcctCore(AcctRouter* router, const IgpModelOps* dev, Options opt) : router_(router), dev_(dev), opt_(opt) {
  if (!dev_ || dev_->abi != IGP_MODEL_OPS_ABI) throw std::runtime_error("AcctCore: model device ABI mismatch");
  kind_ = dev_->kind;
  if (kind_ != IGP_MODEL_LTV && kind_ != IGP_MODEL_ABUSE) throw std::runtime_error("AcctCore: unknown model kind");
  cap_ = dev_->cap;
  depth_ = dev_->depth;
  if (cap_ < 1 || depth_ < 1) throw std::runtime_error("AcctCore: device capacity / depth");
  steps_.resize(depth_);
  for (int s = 0; s < depth_; ++s) {
    steps_[s] = std::make_unique<Step>();
    free_slots_.push_back(depth_ - 1 - s);
  }
  const std::string k = kind_ == IGP_MODEL_LTV ? "ltv" : "abuse";
  threads_.emplace_back([this, k] {
    name_thread("acct-" + k + "-step");
    stepper_loop();
  });
  threads_.emplace_back([this, k] {
    name_thread("acct-" + k + "-done");
    completion_loop();
  });
  for (int i = 0; i < std::max(1, opt_.finishers); ++i)
    threads_.emplace_back([this, k] {
      name_thread("acct-" + k + "-fin");
      finisher_loop();
    });
}

AcctCore::~AcctCore() {
  try {
    stop();
  } catch (...) {
  }
}

void AcctCore::submit(uint8_t rpc, int32_t slot, std::string_view account, uint64_t tag, int origin, int64_t now,
                      int64_t t0_ns, uint64_t link_ticket) {
  Item it{rpc, int16_t(origin), slot, tag, now, t0_ns, mono_ns(), link_ticket, std::string(account)};
  bool wake;
  {
    std::lock_guard<std::mutex> lk(q_mu_);
    if (stopping_ || stopped_) throw std::runtime_error(std::string(kColdPrefix) + "AcctCore: stopped");
    // the stepper needs a wake-up only when this call changes what it waits for: the first call
    // into an empty queue (it sleeps until work arrives) or the one that fills a step; otherwise
    // it wakes on its own at the queue head's max_wait deadline or when a slot frees (release).
    // A notify per call cost a futex wake per call on the submitting thread (cfg5 bench: one
    // submitter at ~1.2 us per call, the device steps a third full)
    wake = queue_.empty() || queue_.size() + 1 >= size_t(cap_);
    queue_.push_back(std::move(it));
  }
  if (wake) q_cv_.notify_all();
}

void AcctCore::submit_many(const Call* calls, size_t n) {
  if (!n) return;
  const int64_t t_enq = mono_ns();
  std::vector<Item> items;
  items.reserve(n);
  for (size_t k = 0; k < n; ++k) {
    const Call& c = calls[k];
    items.push_back(Item{c.rpc, int16_t(-1), c.slot, c.tag, c.now, c.t0, t_enq, c.ticket, std::string(c.account)});
  }
  bool wake;
  {
    std::lock_guard<std::mutex> lk(q_mu_);
    if (stopping_ || stopped_) throw std::runtime_error(std::string(kColdPrefix) + "AcctCore: stopped");
    const size_t q0 = queue_.size();
    wake = q0 == 0 || (q0 < size_t(cap_) && q0 + n >= size_t(cap_));  // as submit()
    for (auto& it : items) queue_.push_back(std::move(it));
  }
  if (wake) q_cv_.notify_all();
}

bool AcctCore::issue(std::unique_lock<std::mutex>& lk) {
  const int slot = free_slots_.back();
  free_slots_.pop_back();
  Step* st = steps_[size_t(slot)].get();
  st->slot = slot;
  st->items.clear();
  st->failed = false;
  st->err.clear();
  const size_t n = std::min(queue_.size(), size_t(cap_));
  const int why = queue_.size() >= size_t(cap_) ? 0 : inflight_ == 0 ? 1 : 2;
  const int64_t t_free = st->t_release;
  int64_t now = 0;
  const bool whole = queue_.head == 0 && n == queue_.v.size();
  if (whole) {
    st->items.swap(queue_.v);  // the step's old (cleared) vector becomes the queue's storage
  } else {
    st->items.reserve(n);
    for (size_t k = 0; k < n; ++k) {
      st->items.push_back(std::move(queue_.front()));
      queue_.pop_front();
    }
  }
  ++inflight_;
  const IgpModelOps* dev = dev_;
  lk.unlock();
  for (const Item& it : st->items) now = std::max(now, it.now);
  int32_t* sl = dev->slots(dev->ctx, slot);
  for (size_t k = 0; k < n; ++k) sl[k] = st->items[k].slot;
  char err[256] = {0};
  const int64_t t1 = mono_ns();
  const int rc = dev->submit(dev->ctx, slot, int32_t(n), now, err, sizeof err);
  st->t_submit = mono_ns();
  if (rc != 0) {
    st->failed = true;
    st->err = err[0] ? err : "model device submit failed";
  }
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.steps += 1;
    st_.rows += int64_t(n);
    st_.max_step_rows = std::max<int64_t>(st_.max_step_rows, int64_t(n));
    st_.submit_ns += st->t_submit - t1;
    if (t_free > 0) st_.free_ns += t1 - t_free;
    (why == 0 ? st_.full_steps : why == 1 ? st_.idle_steps : st_.aged_steps) += 1;
    for (const Item& it : st->items) st_.queue_ns += t1 - it.t_enq;
  }
  {
    std::lock_guard<std::mutex> g(c_mu_);
    done_fifo_.push_back(st);
  }
  c_cv_.notify_one();
  lk.lock();
  return true;
}

void AcctCore::stepper_loop() {
  std::unique_lock<std::mutex> lk(q_mu_);
  const int64_t max_wait = int64_t(opt_.max_wait_us) * 1000;
  for (;;) {
    if (stopping_ && queue_.empty()) {
      idle_cv_.wait(lk, [&] { return inflight_ == 0; });
      stopped_ = true;
      idle_cv_.notify_all();
      return;
    }
    if (hold_) {  // set_device: no new steps until the swap is done
      idle_cv_.notify_all();
      q_cv_.wait(lk, [&] { return !hold_ || stopping_; });
      continue;
    }
    if (!queue_.empty() && !free_slots_.empty()) {
      const int64_t age = mono_ns() - queue_.front().t_enq;
      if (inflight_ == 0 || queue_.size() >= size_t(cap_) || age >= max_wait || stopping_) {
        issue(lk);
        continue;
      }
      q_cv_.wait_for(lk, std::chrono::nanoseconds(std::max<int64_t>(max_wait - age, 1000)));
      continue;
    }
    q_cv_.wait_for(lk, std::chrono::milliseconds(100));
  }
}

void AcctCore::completion_loop() {
  for (;;) {
    Step* st;
    {
      std::unique_lock<std::mutex> l(c_mu_);
      c_cv_.wait(l, [&] { return c_stop_ || !done_fifo_.empty(); });
      if (done_fifo_.empty()) return;
      st = done_fifo_.front();
      done_fifo_.pop_front();
    }
    const IgpModelOps* dev = dev_;
    bool late = false;
    if (!st->failed) {
      char err[256] = {0};
      const int rc = dev->wait(dev->ctx, st->slot, opt_.timeout_us, err, sizeof err);
      if (rc != 0) {
        st->failed = true;
        late = rc == 1;
        st->err = rc == 1 ? "model step exceeded its deadline" : (err[0] ? err : "model device wait failed");
        std::lock_guard<std::mutex> g(st_mu_);
        st_.wait_errors += 1;
      }
    }
    st->t_done = mono_ns();
    {
      std::lock_guard<std::mutex> g(st_mu_);
      st_.device_ns += st->t_done - st->t_submit;
    }
    // the calls and a copy of the outputs leave the slot; answers are written from the copy
    Batch* bt = nullptr;
    {
      std::lock_guard<std::mutex> g(f_mu_);
      if (!batch_pool_.empty()) {
        bt = batch_pool_.back().release();
        batch_pool_.pop_back();
      }
    }
    if (!bt) bt = new Batch();
    bt->items.swap(st->items);
    st->items.clear();
    bt->failed = st->failed;
    bt->err = st->err;
    bt->has_model = dev->has_model != 0;
    const size_t n = bt->items.size();
    const size_t s0 = kind_ == IGP_MODEL_LTV ? 6 * sizeof(float) : sizeof(float);
    const size_t s1 = kind_ == IGP_MODEL_ABUSE ? sizeof(FeatRec) : 0;
    if (!bt->failed) {
      bt->o0.resize(n * s0);
      if (n) std::memcpy(bt->o0.data(), dev->out0(dev->ctx, st->slot), n * s0);
      bt->o1.resize(n * s1);
      if (n && s1) std::memcpy(bt->o1.data(), dev->out1(dev->ctx, st->slot), n * s1);
    }
    if (late) {  // the device may still write the slot's outputs: keep it until it drained
      char err[256] = {0};
      (void)dev->wait(dev->ctx, st->slot, -1, err, sizeof err);
    }
    release(st);
    const size_t nf = size_t(std::max(1, opt_.finishers));
    const size_t per = std::max<size_t>(32, (n + nf - 1) / nf);
    {
      std::lock_guard<std::mutex> g(f_mu_);
      bt->refs.store(int((n + per - 1) / per));
      if (n == 0) {
        batch_pool_.emplace_back(bt);
      } else {
        for (size_t b = 0; b < n; b += per) ftasks_.push_back(FTask{bt, b, std::min(n, b + per)});
      }
    }
    f_cv_.notify_all();
  }
}

void AcctCore::recycle(Batch* bt) {
  if (bt->refs.fetch_sub(1) != 1) return;
  bt->items.clear();
  std::lock_guard<std::mutex> g(f_mu_);
  batch_pool_.emplace_back(bt);
}

void AcctCore::release(Step* st) {
  const int64_t t = mono_ns();
  {
    std::lock_guard<std::mutex> g(st_mu_);
    if (st->t_done > 0) st_.turn_ns += t - st->t_done;
  }
  st->t_release = t;
  {
    std::lock_guard<std::mutex> lk(q_mu_);
    free_slots_.push_back(st->slot);
    --inflight_;
  }
  q_cv_.notify_all();
  idle_cv_.notify_all();
}

void AcctCore::finish(Batch& st, size_t b, size_t e) {
  using Done = ServeCore::Done;
  std::vector<Done> local;
  local.reserve(e - b);
  std::vector<std::pair<int, Done>> remote;
  const void* o0 = st.failed ? nullptr : st.o0.data();
  const void* o1 = st.failed ? nullptr : st.o1.data();
  int64_t sec = 0;
  int32_t nanos = 0;
  wall_now(sec, nanos);
  AbuseParams ap;
  if (kind_ == IGP_MODEL_ABUSE) ap = router_->abuse();
  std::vector<std::string_view> sig, linked;
  // the linked accounts of the whole range under one lock acquisition, after one wait for the
  // link inserts queued before the range's latest local call (a per-call lock and wait starved
  // the finishers behind the ScoreBatch link inserts: 27 k of 100 k calls/s answered in the
  // mixed-traffic run, profiles/r6/c)
  std::vector<std::vector<int64_t>> lk;
  LinkIndex* li = kind_ == IGP_MODEL_ABUSE && !st.failed ? router_->links() : nullptr;
  if (li) {
    uint64_t ticket = 0;
    bool any_local = false;
    std::vector<int64_t> accts;
    accts.reserve(e - b);
    for (size_t i = b; i < e; ++i) {
      const Item& it = st.items[i];
      if (it.origin < 0) {
        ticket = std::max(ticket, it.ticket);
        any_local = true;
      }
      accts.push_back((int64_t(router_->rank()) << 32) | uint32_t(it.slot));
    }
    if (any_local) li->wait_done(ticket, ap.link_wait_us);
    li->linked_many(accts.data(), accts.size(), size_t(ap.linked_limit), lk);
  }
  for (size_t i = b; i < e; ++i) {
    const Item& it = st.items[i];
    Done d{it.tag, std::string(), std::string()};
    if (st.failed) {
      d.err = st.err;
    } else if (kind_ == IGP_MODEL_LTV) {
      const float* row = static_cast<const float*>(o0) + i * 6;
      if (it.rpc == RPC_SEGMENT) acctwire::write_segment(d.bytes, it.account, row);
      else acctwire::write_ltv(d.bytes, it.account, row, sec, nanos);
    } else {
      // engine/abuse.py AbuseService.check: rule signals of the live feature row, the linked
      // accounts, the sequence model; score = min(1, sum of signal weights), max with the model
      const FeatRec& f = static_cast<const FeatRec*>(o1)[i];
      sig.clear();
      linked.clear();
      double score = 0.0;
      auto fire = [&](int k) {
        sig.push_back(acctwire::kSignals[k]);
        score += ap.w[k];
      };
      if (f.flags & FR_BONUS_ONLY) fire(0);
      if (f.bonus_claim_count > 0 && double(f.bonus_wager_rate) < 0.3) fire(1);
      if (f.unique_devices_24h > ap.max_devices_per_day) fire(2);
      if (f.unique_ips_24h > ap.max_ips_per_day) fire(3);
      if (f.flags & (FR_VPN | FR_PROXY | FR_TOR)) fire(4);
      if (f.tx_count_1m > ap.max_tx_per_minute) fire(5);
      if (li) {  // the device / account co-occurrences of every request ingested before this one
        for (int64_t k : lk[i - b]) {
          const int o = int(k >> 32);
          if (o < 0 || o >= router_->world()) continue;
          const std::string_view id = router_->index(o).id_view(int32_t(k & 0xffffffff));
          if (!id.empty()) linked.push_back(id);
        }
      }
      if (!linked.empty()) fire(6);
      score = std::min(1.0, score);
      if (st.has_model) {
        const double ms = double(static_cast<const float*>(o0)[i]);
        if (ms >= ap.threshold) sig.push_back(acctwire::kSignals[7]);
        score = std::max(score, ms);
      }
      acctwire::write_abuse(d.bytes, score >= ap.threshold, float(score), sig, linked);
    }
    if (it.origin < 0) local.push_back(std::move(d));
    else remote.emplace_back(int(it.origin), std::move(d));
  }
  if (!local.empty()) router_->deliver(-1, std::move(local));
  for (auto& [o, d] : remote) {
    std::vector<Done> one;
    one.push_back(std::move(d));
    router_->deliver(o, std::move(one));
  }
}

void AcctCore::finisher_loop() {
  for (;;) {
    FTask t;
    {
      std::unique_lock<std::mutex> l(f_mu_);
      f_cv_.wait(l, [&] { return f_stop_ || !ftasks_.empty(); });
      if (ftasks_.empty()) return;
      t = ftasks_.front();
      ftasks_.pop_front();
    }
    const int64_t t0 = mono_ns();
    finish(*t.bt, t.b, t.e);
    {
      std::lock_guard<std::mutex> g(st_mu_);
      st_.finish_ns += mono_ns() - t0;
      st_.items += int64_t(t.e - t.b);
    }
    recycle(t.bt);
  }
}

void AcctCore::set_device(const IgpModelOps* dev) {
  if (!dev || dev->abi != IGP_MODEL_OPS_ABI || dev->kind != kind_)
    throw std::runtime_error("AcctCore.set_device: ABI / kind mismatch");
  std::unique_lock<std::mutex> lk(q_mu_);
  hold_ = true;
  q_cv_.notify_all();
  idle_cv_.wait(lk, [&] { return inflight_ == 0 || stopped_; });
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
  hold_ = false;
  lk.unlock();
  q_cv_.notify_all();
}

void AcctCore::pause() {
  std::unique_lock<std::mutex> lk(q_mu_);
  hold_ = true;
  q_cv_.notify_all();
  idle_cv_.wait(lk, [&] { return inflight_ == 0 || stopped_; });
}

void AcctCore::resume() {
  {
    std::lock_guard<std::mutex> lk(q_mu_);
    hold_ = false;
  }
  q_cv_.notify_all();
}

void AcctCore::stop() {
  {
    std::lock_guard<std::mutex> lk(q_mu_);
    if (threads_.empty()) return;
    stopping_ = true;
    hold_ = false;
  }
  q_cv_.notify_all();
  threads_[0].join();  // stepper: issued the rest of the queue, every step finished
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
  for (size_t i = 2; i < threads_.size(); ++i) threads_[i].join();
  threads_.clear();
}

AcctStats AcctCore::stats(bool reset) {
  std::lock_guard<std::mutex> g(st_mu_);
  AcctStats s = st_;
  if (reset) st_ = AcctStats();
  return s;
}

// ============================================================================ AcctMailbox
namespace {
constexpr uint64_t kMailboxMagic = 0x49475041434d4231ULL;  // "IGPACMB1"
struct MbHdr {
  uint64_t magic;
  int32_t world, req_cap, rep_cap, ready;
  char pad[40];
};
}  // namespace

AcctMailbox::AcctMailbox(const std::string& shm_name, int world, int rank, int req_cap, int rep_cap, bool create)
    : world_(world), rank_(rank), req_cap_(req_cap), rep_cap_(rep_cap) {
  if (world < 2 || rank < 0 || rank >= world || req_cap < 2 || rep_cap < 2)
    throw std::runtime_error("AcctMailbox: world / rank / ring sizes");
  req_ring_bytes_ = sizeof(RingHdr) + sizeof(ReqMsg) * size_t(req_cap);
  rep_ring_bytes_ = sizeof(RingHdr) + sizeof(RepMsg) * size_t(rep_cap);
  const size_t pairs = size_t(world) * size_t(world);
  rep_off_ = 64 + pairs * req_ring_bytes_;
  const size_t bytes = rep_off_ + pairs * rep_ring_bytes_;
  region_ = Region::shared(shm_name, bytes, create);
  base_ = static_cast<char*>(region_.base());
  auto* h = reinterpret_cast<MbHdr*>(base_);
  if (create) {
    h->world = world;
    h->req_cap = req_cap;
    h->rep_cap = rep_cap;
    h->magic = kMailboxMagic;  // the ring counters are zero (a fresh sparse file)
  } else if (h->magic != kMailboxMagic || h->world != world || h->req_cap != req_cap || h->rep_cap != rep_cap) {
    throw std::runtime_error("AcctMailbox: " + shm_name + " has another layout");
  }
  for (int i = 0; i < world; ++i) {
    req_mu_.push_back(std::make_unique<std::mutex>());
    rep_mu_.push_back(std::make_unique<std::mutex>());
  }
}

AcctMailbox::RingHdr* AcctMailbox::req_hdr(int s, int o) const {
  return reinterpret_cast<RingHdr*>(base_ + 64 + size_t(s * world_ + o) * req_ring_bytes_);
}
AcctMailbox::ReqMsg* AcctMailbox::req_msgs(int s, int o) const {
  return reinterpret_cast<ReqMsg*>(reinterpret_cast<char*>(req_hdr(s, o)) + sizeof(RingHdr));
}
AcctMailbox::RingHdr* AcctMailbox::rep_hdr(int o, int s) const {
  return reinterpret_cast<RingHdr*>(base_ + rep_off_ + size_t(o * world_ + s) * rep_ring_bytes_);
}
AcctMailbox::RepMsg* AcctMailbox::rep_msgs(int o, int s) const {
  return reinterpret_cast<RepMsg*>(reinterpret_cast<char*>(rep_hdr(o, s)) + sizeof(RingHdr));
}

namespace {
// wait for a free ring entry (the consumer is another process's poller: spin, then yield)
template <class H>
bool reserve(H* h, uint64_t cap, uint64_t& head, int64_t timeout_us) {
  head = h->head.v.load(std::memory_order_relaxed);
  if (head - h->tail.v.load(std::memory_order_acquire) < cap) return true;
  const int64_t t_end = mono_ns() + timeout_us * 1000;
  for (int spin = 0;; ++spin) {
    if (head - h->tail.v.load(std::memory_order_acquire) < cap) return true;
    if (mono_ns() > t_end) return false;
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}
}  // namespace

bool AcctMailbox::send_req(int owner, const ReqMsg& m, int64_t timeout_us) {
  std::lock_guard<std::mutex> g(*req_mu_[size_t(owner)]);
  RingHdr* h = req_hdr(rank_, owner);
  uint64_t head;
  if (!reserve(h, uint64_t(req_cap_), head, timeout_us)) return false;
  req_msgs(rank_, owner)[head % uint64_t(req_cap_)] = m;
  h->head.v.store(head + 1, std::memory_order_release);
  return true;
}

bool AcctMailbox::send_rep(int sender, uint64_t tag, int32_t status, std::string_view data, int64_t timeout_us) {
  std::lock_guard<std::mutex> g(*rep_mu_[size_t(sender)]);
  RingHdr* h = rep_hdr(rank_, sender);
  uint64_t head;
  if (!reserve(h, uint64_t(rep_cap_), head, timeout_us)) return false;
  RepMsg& m = rep_msgs(rank_, sender)[head % uint64_t(rep_cap_)];
  m.tag = tag;
  m.status = status;
  if (data.size() > kRepData) {
    // never a truncated answer marked OK (e.g. CheckBonusAbuse with 16 long linked ids): the
    // ingress serves the call through its cold path instead
    oversize_.fetch_add(1, std::memory_order_relaxed);
    const std::string msg = std::string(kColdPrefix) + "reply of " + std::to_string(data.size()) +
                            " bytes exceeds the mailbox record";
    m.status = status ? status : kInternal;
    m.len = int32_t(std::min(msg.size(), kRepData));
    std::memcpy(m.data, msg.data(), size_t(m.len));
  } else {
    m.len = int32_t(data.size());
    std::memcpy(m.data, data.data(), size_t(m.len));
  }
  h->head.v.store(head + 1, std::memory_order_release);
  return true;
}

size_t AcctMailbox::poll_req(const std::function<void(int, const ReqMsg&)>& fn) {
  size_t k = 0;
  for (int s = 0; s < world_; ++s) {
    if (s == rank_) continue;
    RingHdr* h = req_hdr(s, rank_);
    uint64_t t = h->tail.v.load(std::memory_order_relaxed);
    const uint64_t hd = h->head.v.load(std::memory_order_acquire);
    for (; t < hd; ++t, ++k) {
      fn(s, req_msgs(s, rank_)[t % uint64_t(req_cap_)]);
      h->tail.v.store(t + 1, std::memory_order_release);
    }
  }
  return k;
}

size_t AcctMailbox::poll_rep(const std::function<void(int, const RepMsg&)>& fn) {
  size_t k = 0;
  for (int o = 0; o < world_; ++o) {
    if (o == rank_) continue;
    RingHdr* h = rep_hdr(o, rank_);
    uint64_t t = h->tail.v.load(std::memory_order_relaxed);
    const uint64_t hd = h->head.v.load(std::memory_order_acquire);
    for (; t < hd; ++t, ++k) {
      fn(o, rep_msgs(o, rank_)[t % uint64_t(rep_cap_)]);
      h->tail.v.store(t + 1, std::memory_order_release);
    }
  }
  return k;
}

// ============================================================================ AcctRouter
AcctRouter::AcctRouter(std::vector<std::shared_ptr<AccountIndex>> indexes, int rank, const std::string& mailbox,
                       bool create, int req_cap, int rep_cap)
    : idx_(std::move(indexes)), world_(int(idx_.size())), rank_(rank) {
  if (world_ < 1 || rank_ < 0 || rank_ >= world_) throw std::runtime_error("AcctRouter: indexes / rank");
  for (auto& i : idx_)
    if (!i) throw std::runtime_error("AcctRouter: null account index");
  if (world_ > 1) {
    if (mailbox.empty()) throw std::runtime_error("AcctRouter: world > 1 needs a mailbox name");
    mb_ = std::make_unique<AcctMailbox>(mailbox, world_, rank_, req_cap, rep_cap, create);
    mb_thread_ = std::thread([this] {
      name_thread("acct-mailbox");
      mailbox_loop();
    });
  }
}

AcctRouter::~AcctRouter() {
  try {
    stop();
  } catch (...) {
  }
}

void AcctRouter::attach(const IgpModelOps* dev, AcctCore::Options opt) {
  if (!dev || dev->abi != IGP_MODEL_OPS_ABI) throw std::runtime_error("AcctRouter.attach: ABI mismatch");
  auto c = std::make_shared<AcctCore>(this, dev, opt);
  std::lock_guard<std::mutex> g(p_mu_);
  (dev->kind == IGP_MODEL_LTV ? ltv_ : abuse_) = std::move(c);
}

void AcctRouter::set_device(int kind, const IgpModelOps* dev) {
  AcctCore* c = kind == IGP_MODEL_LTV ? ltv_.get() : abuse_.get();
  if (!c) throw std::runtime_error("AcctRouter.set_device: no core of that kind");
  c->set_device(dev);
}

void AcctRouter::pause() {
  for (AcctCore* c : {ltv_.get(), abuse_.get()})
    if (c) c->pause();
}

void AcctRouter::resume() {
  for (AcctCore* c : {ltv_.get(), abuse_.get()})
    if (c) c->resume();
}

void AcctRouter::set_abuse(const AbuseParams& p) {
  std::lock_guard<std::mutex> g(p_mu_);
  abuse_params_ = p;
}

AbuseParams AcctRouter::abuse() const {
  std::lock_guard<std::mutex> g(p_mu_);
  return abuse_params_;
}

AcctCore* AcctRouter::core_for(uint8_t rpc) const {
  return rpc == RPC_ABUSE ? abuse_.get() : ltv_.get();
}

bool AcctRouter::serves(uint8_t rpc) const { return core_for(rpc) != nullptr; }

void AcctRouter::set_sink(Sink s) {
  std::lock_guard<std::mutex> g(out_mu_);
  sink_ = std::move(s);
}

AcctRouter::Sink AcctRouter::sink() const {
  std::lock_guard<std::mutex> g(out_mu_);
  return sink_;
}

void AcctRouter::deliver(int origin, std::vector<Done>&& outs) {
  if (origin >= 0) {  // answers to another rank's ingress: its reply ring
    for (auto& d : outs) {
      const bool ok = d.err.empty();
      if (!mb_->send_rep(origin, d.tag, ok ? 0 : kInternal, ok ? std::string_view(d.bytes) : std::string_view(d.err),
                         2000000)) {
        // the ingress rank stopped draining (dead): its caller times out there
      }
    }
    return;
  }
  Sink sink;
  {
    std::lock_guard<std::mutex> g(out_mu_);
    sink = sink_;
    size_t k = 0;
    for (size_t i = 0; i < outs.size(); ++i) {
      if (sink && (outs[i].tag & kSinkTag)) {
        if (k != i) outs[k] = std::move(outs[i]);
        ++k;
      } else {
        outq_.push_back(std::move(outs[i]));
      }
    }
    outs.resize(k);
  }
  out_cv_.notify_all();
  if (sink && !outs.empty()) sink(std::move(outs));
}

void AcctRouter::answer_now(int origin, uint64_t tag, std::string bytes, std::string err) {
  std::vector<Done> d;
  d.push_back(Done{tag, std::move(bytes), std::move(err)});
  deliver(origin, std::move(d));
}

size_t AcctRouter::poll(std::vector<Done>& out, size_t max, int64_t timeout_us) {
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

void AcctRouter::local(uint8_t rpc, int32_t slot, std::string_view account, uint64_t tag, int origin, int64_t now,
                       int64_t t0, uint64_t ticket) {
  AcctCore* c = core_for(rpc);
  if (!c) {
    answer_now(origin, tag, std::string(), std::string(kColdPrefix) + "no native model core for this RPC on rank " +
                                               std::to_string(rank_));
    return;
  }
  if (rpc == RPC_ABUSE && slot < 0) {
    // unknown account: no state to check (engine/abuse.py): is_abuser false, score 0, no signals
    answer_now(origin, tag, std::string(), std::string());
    return;
  }
  c->submit(rpc, slot, account, tag, origin, now, t0, ticket);
}

void AcctRouter::submit(uint8_t rpc, const char* data, size_t n, uint64_t tag, int64_t t0_ns, int64_t now) {
  std::string_view account, bonus;
  try {
    acctwire::parse_request(data, n, account, bonus);
  } catch (const std::exception& e) {
    answer_now(-1, tag, std::string(), std::string("pb: ") + e.what());
    return;
  }
  if (account.empty()) {
    answer_now(-1, tag, std::string(), "invalid: account_id is required");
    return;
  }
  if (now < 0) now = int64_t(std::time(nullptr));
  const uint64_t h = id_hash(account, SEED_ACCOUNT);
  const int owner = int(h % uint64_t(world_));
  const int32_t slot = idx_[size_t(owner)]->find(account, h);
  const uint64_t ticket = links_ ? links_->ticket() : 0;
  try {
    if (owner == rank_) {
      local(rpc, slot, account, tag, -1, now, t0_ns, ticket);
      return;
    }
    if (account.size() > size_t(AcctMailbox::kIdMax)) {
      answer_now(-1, tag, std::string(), "invalid: account_id too long for cross-rank routing");
      return;
    }
    AcctMailbox::ReqMsg m{};
    m.tag = tag;
    m.now = now;
    m.t0 = t0_ns;
    m.ticket = 0;
    m.slot = slot;
    m.rpc = rpc;
    m.idlen = uint8_t(account.size());
    std::memcpy(m.id, account.data(), account.size());
    {
      std::lock_guard<std::mutex> g(r_mu_);
      remote_[tag] = {mono_ns() + remote_timeout_us * 1000, owner};
    }
    remote_out_.fetch_add(1, std::memory_order_relaxed);
    if (!mb_->send_req(owner, m, 1000000)) {
      {
        std::lock_guard<std::mutex> g(r_mu_);
        remote_.erase(tag);
      }
      answer_now(-1, tag, std::string(), "owner rank " + std::to_string(owner) + " is not draining its mailbox");
    }
  } catch (const std::exception& e) {
    answer_now(-1, tag, std::string(), e.what());
  }
}

void AcctRouter::submit_many(uint8_t rpc, const std::string_view* data, const uint64_t* tags, const int64_t* t0_ns,
                             size_t n, int64_t now) {
  if (now < 0) now = int64_t(std::time(nullptr));
  AcctCore* c = core_for(rpc);
  if (!c) {  // no local core: answered per call by submit()
    for (size_t k = 0; k < n; ++k) submit(rpc, data[k].data(), data[k].size(), tags[k], t0_ns[k], now);
    return;
  }
  const uint64_t ticket = links_ ? links_->ticket() : 0;
  // parse every call, then resolve this rank's accounts in one batched index lookup (probe lines
  // prefetched for the whole range: one overlapped round of cache misses, not one per call)
  thread_local std::vector<std::string_view> acc;
  thread_local std::vector<uint64_t> hs;
  thread_local std::vector<uint8_t> mine;
  thread_local std::vector<int32_t> slots;
  acc.assign(n, std::string_view());
  hs.assign(n, 0);
  mine.assign(n, 0);
  slots.assign(n, -1);
  size_t n_mine = 0;
  for (size_t k = 0; k < n; ++k) {
    std::string_view account, bonus;
    try {
      acctwire::parse_request(data[k].data(), data[k].size(), account, bonus);
    } catch (const std::exception& e) {
      answer_now(-1, tags[k], std::string(), std::string("pb: ") + e.what());
      continue;
    }
    if (account.empty()) {
      answer_now(-1, tags[k], std::string(), "invalid: account_id is required");
      continue;
    }
    const uint64_t h = id_hash(account, SEED_ACCOUNT);
    const int owner = int(h % uint64_t(world_));
    if (owner != rank_) {  // another rank's account: the mailbox path of submit()
      submit(rpc, data[k].data(), data[k].size(), tags[k], t0_ns[k], now);
      continue;
    }
    acc[k] = account;
    hs[k] = h;
    mine[k] = 1;
    ++n_mine;
  }
  if (n_mine) idx_[size_t(rank_)]->lookup_views(acc.data(), hs.data(), n, false, slots.data(), nullptr, mine.data());
  std::vector<AcctCore::Call> calls;
  calls.reserve(n_mine);
  for (size_t k = 0; k < n; ++k) {
    if (!mine[k]) continue;
    const int32_t slot = slots[k];
    if (rpc == RPC_ABUSE && slot < 0) {  // as local(): an unknown account has nothing to check
      answer_now(-1, tags[k], std::string(), std::string());
      continue;
    }
    calls.push_back(AcctCore::Call{rpc, slot, acc[k], tags[k], now, t0_ns[k], ticket});
  }
  try {
    c->submit_many(calls.data(), calls.size());
  } catch (const std::exception& e) {
    for (const auto& cl : calls) answer_now(-1, cl.tag, std::string(), e.what());
  }
}

void AcctRouter::mailbox_loop() {
  int idle = 0;
  int64_t next_sweep = mono_ns() + 100000000;
  std::vector<Done> batch;
  while (!stop_.load(std::memory_order_acquire)) {
    size_t k = mb_->poll_req([&](int sender, const AcctMailbox::ReqMsg& m) {
      const std::string_view id(m.id, m.idlen);
      try {
        local(m.rpc, m.slot, id, m.tag, sender, m.now, m.t0, 0);
      } catch (const std::exception& e) {
        mb_->send_rep(sender, m.tag, kUnavailable, e.what(), 100000);
      }
    });
    batch.clear();
    k += mb_->poll_rep([&](int, const AcctMailbox::RepMsg& m) {
      {
        std::lock_guard<std::mutex> g(r_mu_);
        if (remote_.erase(m.tag) == 0) return;  // expired meanwhile: already answered
      }
      Done d{m.tag, std::string(), std::string()};
      if (m.status == 0) d.bytes.assign(m.data, size_t(m.len));
      else d.err.assign(m.data, size_t(m.len));
      batch.push_back(std::move(d));
    });
    if (!batch.empty()) deliver(-1, std::move(batch));
    const int64_t t = mono_ns();
    if (t > next_sweep) {  // calls whose owner never answered (a dead rank)
      next_sweep = t + 100000000;
      std::vector<Done> exp;
      {
        std::lock_guard<std::mutex> g(r_mu_);
        for (auto it = remote_.begin(); it != remote_.end();) {
          if (it->second.first < t) {
            exp.push_back(Done{it->first, std::string(),
                               "owner rank " + std::to_string(it->second.second) + " did not answer in time"});
            it = remote_.erase(it);
          } else {
            ++it;
          }
        }
      }
      if (!exp.empty()) {
        expired_.fetch_add(int64_t(exp.size()), std::memory_order_relaxed);
        deliver(-1, std::move(exp));
      }
    }
    if (k) {
      idle = 0;
    } else if (++idle > 200) {
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    } else if (idle > 20) {
      std::this_thread::yield();
    }
  }
}

void AcctRouter::stop() {
  if (ltv_) ltv_->stop();
  if (abuse_) abuse_->stop();
  if (!stop_.exchange(true) && mb_thread_.joinable()) mb_thread_.join();
}

AcctStats AcctRouter::stats(int kind, bool reset) {
  AcctCore* c = kind == IGP_MODEL_LTV ? ltv_.get() : abuse_.get();
  return c ? c->stats(reset) : AcctStats();
}

}  // namespace igp

// Native account-RPC serving: PredictLTV, GetPlayerSegment and CheckBonusAbuse from request
// bytes to response bytes, GIL-free, owner-routed on every rank (VERDICT r3 "cold RPCs at
// serving rate"; reference: proto/risk/v1/risk.proto:16-20, the callers
// services/bonus/internal/service/bonus_engine.go:269 and prediction/ltv.go:113-151, 385-398).
//
//   ingress (HTTP/2 worker threads, Python tests / bench)
//     request bytes -> account_id (+ bonus_id) -> XXH64 digest -> owner = digest % world
//     owner == this rank: AccountIndex slot (the node-shared table) -> the model core's FIFO
//     owner != this rank: one 128-byte record into the (this rank -> owner) request ring of the
//                         node-shared mailbox (/dev/shm); the owner answers with the response
//                         bytes through its (owner -> this rank) reply ring
//   AcctCore (one per local model device: the LTV chain, the abuse step)
//     stepper     micro-batches the FIFO (up to the device capacity, or max_wait_us) into the
//                 slot's int32 slot array and launches it through the device table (model_ops.h)
//     completion  waits for slots in submit order, hands the rows to the finishers
//     finishers   write the response bytes: PredictLTVResponse / GetPlayerSegmentResponse from
//                 the K9 row; CheckBonusAbuseResponse from the FeatRec rule signals, the GRU
//                 score and the device <-> account link index (linked_accounts)
//   delivery: local calls -> the sink (native gRPC server) or the poll() queue; remote calls ->
//             the mailbox reply ring of the rank that ingested them
//
// Requests for accounts of other ranks never touch the GPU of the ingress rank, and no
// collective runs per request: a request is 128 bytes of /dev/shm, the answer < 2 KiB. Every
// rank serves all three RPCs at its own rate; the owner's device batches the rows of every
// ingress rank together.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../include/model_ops.h"
#include "../include/records.h"
#include "account_index.h"
#include "link_index.h"
#include "serve_core.h"
#include "shm.h"

namespace igp {

enum AcctRpc : uint8_t { RPC_LTV = 1, RPC_SEGMENT = 2, RPC_ABUSE = 3 };

// CheckBonusAbuse signal rules (engine/abuse.py SIGNAL_WEIGHTS / rule_signal_columns): weights in
// the order BONUS_ONLY_PLAYER, LOW_WAGER_COMPLETION, MULTIPLE_DEVICES, MULTIPLE_IPS,
// VPN_PROXY_TOR, HIGH_VELOCITY, SHARED_DEVICE
struct AbuseParams {
  int32_t max_devices_per_day = 3, max_ips_per_day = 5, max_tx_per_minute = 10;
  double threshold = 0.7;
  double w[7] = {0.35, 0.2, 0.15, 0.1, 0.1, 0.1, 0.25};
  int32_t linked_limit = 16;
  // wait at most this long for link inserts queued before the request (AbuseConfig.link_wait_us).
  // The serving core keeps at most kLinkQueue batch inserts queued (~1 ms each) and drops the
  // rest under overload, so links are best-effort there anyway; a long wait only adds latency:
  // 2 ms put ~0.4-1.3 ms of link waiting on every CheckBonusAbuse micro-batch under ScoreBatch
  // load (tools/bench_mixed.py abuse_finish_us_per_step, profiles/r6/j)
  int64_t link_wait_us = 200;
};

namespace acctwire {
// account_id (field 1) and bonus_id (field 2, CheckBonusAbuseRequest) of a request body
void parse_request(const char* data, size_t n, std::string_view& account, std::string_view& bonus);
extern const char* const kNbaCodes[13];
void write_ltv(std::string& out, std::string_view account, const float* row, int64_t sec, int32_t nanos);
void write_segment(std::string& out, std::string_view account, const float* row);
void write_abuse(std::string& out, bool is_abuser, float score, const std::vector<std::string_view>& signals,
                 const std::vector<std::string_view>& linked);
}  // namespace acctwire

struct AcctStats {
  int64_t items = 0, steps = 0, rows = 0, device_ns = 0, queue_ns = 0, finish_ns = 0, wait_errors = 0;
  int64_t max_step_rows = 0, remote_in = 0, unknown = 0;
  // slot cycle: time in dev->submit, device done -> slot released (answers written), slot free ->
  // next step issued on it; steps issued full / on an idle device / when the queue head aged out
  int64_t submit_ns = 0, turn_ns = 0, free_ns = 0, full_steps = 0, idle_steps = 0, aged_steps = 0;
};

class AcctRouter;

// One model device of this rank's shard and its micro-batching pipeline.
class AcctCore {
 public:
  struct Options {
    int max_wait_us = 200;
    int64_t timeout_us = -1;  // device wait deadline per step (-1: none)
    int finishers = 2;
  };
  AcctCore(AcctRouter* router, const IgpModelOps* dev, Options opt);
  ~AcctCore();
  AcctCore(const AcctCore&) = delete;
  AcctCore& operator=(const AcctCore&) = delete;

  // origin: -1 local call (tag back through the router's sink / poll queue), else the ingress rank
  void submit(uint8_t rpc, int32_t slot, std::string_view account, uint64_t tag, int origin, int64_t now,
              int64_t t0_ns, uint64_t link_ticket);
  // several local calls under one queue-lock acquisition (AcctRouter::submit_many)
  struct Call {
    uint8_t rpc;
    int32_t slot;
    std::string_view account;
    uint64_t tag;
    int64_t now, t0;
    uint64_t ticket;
  };
  void submit_many(const Call* calls, size_t n);
  void stop();
  // swap the device function table (hot model reload): blocks new steps, drains, swaps
  void set_device(const IgpModelOps* dev);
  // no new device steps until resume(); returns once every step in flight finished (a device's
  // shared state - its config block - can then be rewritten without a step reading it)
  void pause();
  void resume();
  int kind() const { return kind_; }
  AcctStats stats(bool reset);

 private:
  struct Item {
    uint8_t rpc;
    int16_t origin;
    int32_t slot;
    uint64_t tag;
    int64_t now, t0, t_enq;
    uint64_t ticket;
    std::string account;
  };
  struct Step {
    int slot = 0;
    std::vector<Item> items;
    int64_t t_submit = 0, t_done = 0, t_release = 0;
    bool failed = false;
    std::string err;
  };
  // a completed step's calls and a copy of its outputs: the device slot is released as soon as
  // the outputs are copied out of its host buffers, and the finishers write the answers from here
  // (answer writing no longer holds the slot: cfg4 spent 364 us per step between the device
  // finishing and the slot freeing, profiles/r6/s)
  struct Batch {
    std::vector<Item> items;
    std::vector<char> o0, o1;
    bool failed = false, has_model = false;
    std::string err;
    std::atomic<int> refs{0};
  };
  void stepper_loop();
  void completion_loop();
  void finisher_loop();
  bool issue(std::unique_lock<std::mutex>& lk);
  void finish(Batch& bt, size_t b, size_t e);
  void release(Step* st);
  void recycle(Batch* bt);

  AcctRouter* router_;
  const IgpModelOps* dev_;
  int kind_, cap_, depth_;
  Options opt_;

  std::mutex q_mu_;
  std::condition_variable q_cv_, idle_cv_;
  // FIFO of queued calls: a vector with a head index. A step that takes the whole queue swaps
  // the storage with its item vector (O(1) under the queue lock, which the submitting threads
  // also take); a partial take moves items and compacts once the consumed head passes half
  struct ItemQueue {
    std::vector<Item> v;
    size_t head = 0;
    bool empty() const { return head == v.size(); }
    size_t size() const { return v.size() - head; }
    Item& front() { return v[head]; }
    void push_back(Item&& it) { v.push_back(std::move(it)); }
    void pop_front() {
      if (++head == v.size()) {
        v.clear();
        head = 0;
      } else if (head >= 4096 && 2 * head >= v.size()) {
        v.erase(v.begin(), v.begin() + std::ptrdiff_t(head));
        head = 0;
      }
    }
  };
  ItemQueue queue_;
  std::vector<int> free_slots_;
  std::vector<std::unique_ptr<Step>> steps_;
  int inflight_ = 0;
  bool stopping_ = false, stopped_ = false, hold_ = false;

  std::mutex c_mu_;
  std::condition_variable c_cv_;
  std::deque<Step*> done_fifo_;
  bool c_stop_ = false;

  struct FTask {
    Batch* bt;
    size_t b, e;
  };
  std::mutex f_mu_;
  std::condition_variable f_cv_;
  std::deque<FTask> ftasks_;
  std::vector<std::unique_ptr<Batch>> batch_pool_;  // under f_mu_
  bool f_stop_ = false;

  std::mutex st_mu_;
  AcctStats st_;
  std::vector<std::thread> threads_;
};

// Node-shared request / reply rings between the ranks of one node (/dev/shm). Ring (s, o)
// carries requests from ingress rank s to owner o; ring (o, s) of the reply half carries the
// answers back. Single consumer per ring (the router thread of the receiving rank); producers
// of one process serialise on a process-local mutex per ring.
class AcctMailbox {
 public:
  static constexpr int kIdMax = 88;
  struct ReqMsg {
    uint64_t tag;
    int64_t now, t0;
    uint64_t ticket;
    int32_t slot;
    uint8_t rpc, idlen;
    uint8_t pad[2];
    char id[kIdMax];
  };
  static_assert(sizeof(ReqMsg) == 128, "ReqMsg must be 128 bytes");
  static constexpr size_t kRepData = 2032;
  struct RepMsg {
    uint64_t tag;
    int32_t status;  // grpc status (0: data = response bytes, else the message)
    int32_t len;
    char data[kRepData];
  };
  static_assert(sizeof(RepMsg) == 2048, "RepMsg must be 2048 bytes");

  AcctMailbox(const std::string& shm_name, int world, int rank, int req_cap, int rep_cap, bool create);
  // blocking up to `timeout_us` for ring space; false: the ring stayed full
  bool send_req(int owner, const ReqMsg& m, int64_t timeout_us);
  bool send_rep(int sender, uint64_t tag, int32_t status, std::string_view data, int64_t timeout_us);
  // drain inbound rings; returns the number of messages handled
  size_t poll_req(const std::function<void(int sender, const ReqMsg&)>& fn);
  size_t poll_rep(const std::function<void(int owner, const RepMsg&)>& fn);
  void unlink_shared() { region_.unlink(); }
  int world() const { return world_; }
  int64_t oversize() const { return oversize_.load(); }  // replies too long for a record (sent as cold)

 private:
  struct alignas(64) Ctr {
    std::atomic<uint64_t> v;
    char pad[56];
  };
  struct RingHdr {
    Ctr head, tail;
  };
  RingHdr* req_hdr(int s, int o) const;
  ReqMsg* req_msgs(int s, int o) const;
  RingHdr* rep_hdr(int o, int s) const;
  RepMsg* rep_msgs(int o, int s) const;

  Region region_;
  char* base_ = nullptr;
  int world_, rank_, req_cap_, rep_cap_;
  size_t req_ring_bytes_, rep_ring_bytes_, rep_off_;
  std::vector<std::unique_ptr<std::mutex>> req_mu_, rep_mu_;
  std::atomic<int64_t> oversize_{0};
};

// This rank's entry point for the three RPCs: parse, route (local core or mailbox), deliver.
class AcctRouter {
 public:
  using Done = ServeCore::Done;
  using Sink = ServeCore::Sink;
  static constexpr uint64_t kSinkTag = ServeCore::kSinkTag;

  // indexes: one per owner (the node-shared registry when world > 1); mailbox: /dev/shm name
  // of the node's mailbox (world > 1; every rank passes the same name, rank 0 creates it)
  AcctRouter(std::vector<std::shared_ptr<AccountIndex>> indexes, int rank, const std::string& mailbox,
             bool create, int req_cap = 4096, int rep_cap = 1024);
  ~AcctRouter();

  // the local model devices (kind from the table): LTV serves PredictLTV + GetPlayerSegment
  void attach(const IgpModelOps* dev, AcctCore::Options opt);
  void set_device(int kind, const IgpModelOps* dev);
  void pause();   // every local core (AcctCore::pause)
  void resume();
  void set_links(std::shared_ptr<LinkIndex> l) { links_ = std::move(l); }
  void set_abuse(const AbuseParams& p);
  AbuseParams abuse() const;
  bool serves(uint8_t rpc) const;

  // one unary call (request body without the gRPC prefix); the answer comes back with `tag`
  // through the sink (tags with kSinkTag) or poll()
  // now: the clock the account's features are read at (unix s; < 0: the wall clock)
  void submit(uint8_t rpc, const char* data, size_t n, uint64_t tag, int64_t t0_ns, int64_t now = -1);
  // n calls of one RPC (a submitter's batch): each parsed and routed as submit(), the local ones
  // queued on their core under one lock acquisition instead of one per call
  void submit_many(uint8_t rpc, const std::string_view* data, const uint64_t* tags, const int64_t* t0_ns, size_t n,
                   int64_t now = -1);
  void set_sink(Sink s);
  Sink sink() const;
  size_t poll(std::vector<Done>& out, size_t max, int64_t timeout_us);

  void stop();
  void unlink_shared() {
    if (mb_) mb_->unlink_shared();
  }
  int world() const { return world_; }
  int rank() const { return rank_; }
  AcctStats stats(int kind, bool reset);
  int64_t remote_out() const { return remote_out_.load(); }
  int64_t remote_expired() const { return expired_.load(); }
  int64_t reply_oversize() const { return mb_ ? mb_->oversize() : 0; }

  // used by the cores
  void deliver(int origin, std::vector<Done>&& outs);
  AccountIndex& index(int owner) { return *idx_[size_t(owner)]; }
  LinkIndex* links() const { return links_.get(); }
  int64_t remote_timeout_us = 10000000;  // a forwarded call unanswered this long fails (dead owner)

 private:
  void local(uint8_t rpc, int32_t slot, std::string_view account, uint64_t tag, int origin, int64_t now, int64_t t0,
             uint64_t ticket);
  void answer_now(int origin, uint64_t tag, std::string bytes, std::string err);
  void mailbox_loop();
  AcctCore* core_for(uint8_t rpc) const;

  std::vector<std::shared_ptr<AccountIndex>> idx_;
  int world_, rank_;
  std::unique_ptr<AcctMailbox> mb_;
  std::shared_ptr<AcctCore> ltv_, abuse_;
  std::shared_ptr<LinkIndex> links_;
  mutable std::mutex p_mu_;
  AbuseParams abuse_params_;

  mutable std::mutex out_mu_;
  std::condition_variable out_cv_;
  std::deque<Done> outq_;
  Sink sink_;

  // forwarded calls awaiting their owner's reply: tag -> (deadline, owner)
  std::mutex r_mu_;
  std::unordered_map<uint64_t, std::pair<int64_t, int>> remote_;
  std::atomic<int64_t> remote_out_{0}, expired_{0};
  std::atomic<bool> stop_{false};
  std::thread mb_thread_;
};

}  // namespace igp

// Device <-> account co-occurrence index for multi-account detection (CheckBonusAbuse's
// linked_accounts, risk.proto:135-145; the reference declares the field but never fills it).
//
// Every scored request contributes (device digest, account key) where the account key is
// (owner << 32 | slot). Two bounded tables, device -> recent accounts and account -> recent
// devices, each a set-associative array (4-way buckets, one bucket per hash; a full bucket
// evicts its least recently touched key) whose entries hold the `per_key` most recent values
// (move-to-front on repeat). Memory is fixed at construction, an insert touches one or two
// cache lines per table, and the batch insert prefetches the buckets of upcoming rows: it is
// on the scoring hot path (every ScoreBatch / micro-batch), ~8192 rows per call.
//
// The tables live in a memory region: process-private, or node-shared (/dev/shm) so that every
// rank of a one-process-per-GPU group records the traffic it ingests into ONE index and every
// rank's CheckBonusAbuse sees the links of all of them (a device shared by accounts that reached
// different ingress ranks). A spin lock in the region serialises writers and readers across the
// processes (a batch insert holds it ~1 ms per 8192 rows; readers are single lookups). The lock
// word holds its owner's pid: a waiter that finds the owner process gone (SIGKILL, abort while
// inside a critical section) takes the lock over instead of spinning forever, and readers wait
// a bounded time (kReadWaitUs) and then answer "no links"; such answers are counted
// (read_timeouts, exported as a metric) so abuse-score drift from lock timeouts is visible.
#pragma once
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include <signal.h>
#include <unistd.h>

#include "shm.h"

namespace igp {

class LinkIndex {
 public:
  static constexpr int kMaxPerKey = 16;
  static constexpr int64_t kReadWaitUs = 50000;  // a reader gives up (no links) after this long

  explicit LinkIndex(int per_key = 8, int64_t buckets = int64_t(1) << 18) { init(per_key, buckets, "", false); }
  // node-shared index in /dev/shm/<name> (create: this process sizes it; the others map it)
  LinkIndex(int per_key, int64_t buckets, const std::string& shm_name, bool create) {
    init(per_key, buckets, shm_name, create);
  }

  // the lock is taken per chunk of kAddChunk rows, not for the whole batch: a reader
  // (CheckBonusAbuse) then waits at most one chunk (~30 us) behind an 8192-row ScoreBatch insert
  // instead of the whole ~1 ms of it (mixed-traffic run, profiles/r6/c)
  static constexpr size_t kAddChunk = 256;
  void add(const uint64_t* dev, const int64_t* acct, size_t n) {
    constexpr size_t kAhead = 8;
    for (size_t c0 = 0; c0 < n; c0 += kAddChunk) {
      const size_t c1 = std::min(n, c0 + kAddChunk);
      {
        Guard g(hdr_->lock, -1);
        for (size_t i = c0; i < c1; ++i) {
          if (i + kAhead < c1) {
            dev_.prefetch(dev[i + kAhead]);
            acct_.prefetch(akey(acct[i + kAhead]));
          }
          if (dev[i] == 0 || acct[i] < 0) continue;
          const uint32_t now = ++hdr_->clock;
          push(dev_.touch(dev[i], now, hdr_->dev_used), acct[i]);
          push(acct_.touch(akey(acct[i]), now, hdr_->acct_used), int64_t(dev[i]));
        }
      }
      // hand the lock to a waiting reader between chunks: the spin lock is not fair, and an
      // inserter that re-took it at once kept CheckBonusAbuse's lookups out for the whole
      // 8192-row batch (~0.6 ms of every abuse micro-batch's finish under ScoreBatch load,
      // profiles/r6/o). Bounded: a reader that never takes it costs at most ~20 us per chunk.
      if (c1 < n && hdr_->readers.load(std::memory_order_acquire) > 0) {
        const auto t_end = std::chrono::steady_clock::now() + std::chrono::microseconds(20);
        while (hdr_->readers.load(std::memory_order_acquire) > 0 && std::chrono::steady_clock::now() < t_end)
          std::this_thread::yield();
      }
    }
  }

  // accounts sharing at least one device with `acct` (excluding itself), most recent first
  std::vector<int64_t> linked(int64_t acct, size_t limit) const {
    Guard g(hdr_->lock, kReadWaitUs, &hdr_->readers);
    std::vector<int64_t> out;
    if (!g.held) {
      read_timeouts_.fetch_add(1, std::memory_order_relaxed);
      return out;
    }
    linked_locked(acct, limit, out);
    return out;
  }
  // linked() of n accounts under one lock acquisition (a micro-batch of CheckBonusAbuse calls)
  void linked_many(const int64_t* acct, size_t n, size_t limit, std::vector<std::vector<int64_t>>& out) const {
    out.assign(n, {});
    if (!n) return;
    Guard g(hdr_->lock, kReadWaitUs, &hdr_->readers);
    if (!g.held) {
      read_timeouts_.fetch_add(int64_t(n), std::memory_order_relaxed);
      return;
    }
    for (size_t i = 0; i < n; ++i) linked_locked(acct[i], limit, out[i]);
  }

  std::vector<int64_t> devices_of(int64_t acct) const {
    Guard g(hdr_->lock, kReadWaitUs, &hdr_->readers);
    if (!g.held) read_timeouts_.fetch_add(1, std::memory_order_relaxed);
    CEntry a;
    return g.held && acct_.find(akey(acct), a) ? std::vector<int64_t>(a.v, a.v + a.n) : std::vector<int64_t>{};
  }

  size_t n_devices() const {
    Guard g(hdr_->lock, kReadWaitUs, &hdr_->readers);
    return size_t(hdr_->dev_used);
  }
  // tests: take the lock and keep it (a process that dies inside a critical section)
  void debug_acquire_and_leak() { Guard(hdr_->lock, -1).leak(); }
  int64_t takeovers() const { return takeovers_.load(); }
  // lookups answered "no links" because the lock was not free within kReadWaitUs
  int64_t read_timeouts() const { return read_timeouts_.load(); }
  bool shared() const { return region_.shared_mapping(); }
  void unlink_shared() { region_.unlink(); }

  // insert tickets (process-local): a producer that queues an insert for later (the serving
  // core's link thread) takes a ticket; a reader that must see every insert queued before it
  // (CheckBonusAbuse's linked_accounts) waits until the tickets handed out before its own were
  // completed
  uint64_t ticket() const { return enq_.load(std::memory_order_acquire); }
  void note_queued() { enq_.fetch_add(1, std::memory_order_acq_rel); }
  void note_done() { done_.fetch_add(1, std::memory_order_acq_rel); }
  bool wait_done(uint64_t ticket, int64_t timeout_us) const {
    if (done_.load(std::memory_order_acquire) >= ticket) return true;
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::microseconds(timeout_us);
    while (done_.load(std::memory_order_acquire) < ticket) {
      if (std::chrono::steady_clock::now() >= t_end) return false;
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    return true;
  }

 private:
  static constexpr uint64_t kMagic = 0x49475031494e4b31ULL;  // "IGP1INK1"
  struct alignas(64) Hdr {
    uint64_t magic;
    int64_t buckets;
    int32_t per_key;
    std::atomic<uint32_t> lock;
    uint32_t clock;
    std::atomic<int32_t> readers;  // readers waiting for the lock (the inserter yields to them)
    uint64_t dev_used, acct_used;
    char pad[16];
  };
  static_assert(sizeof(Hdr) == 64, "LinkIndex header must be one line");
  // cross-process spin lock (the region's word = the owner's pid, 0: free); short critical
  // sections. timeout_us < 0: wait until acquired. A waiter checks every ~1 ms whether the owner
  // process still exists and takes the word over (CAS owner -> self) when it does not.
  static std::atomic<int64_t> takeovers_;
  static std::atomic<int64_t> read_timeouts_;
  struct Guard {
    std::atomic<uint32_t>& l;
    bool held = false;
    Guard(std::atomic<uint32_t>& x, int64_t timeout_us, std::atomic<int32_t>* waiting = nullptr) : l(x) {
      uint32_t z0 = 0;
      if (l.compare_exchange_strong(z0, uint32_t(::getpid()), std::memory_order_acquire, std::memory_order_relaxed)) {
        held = true;
        return;
      }
      if (waiting) waiting->fetch_add(1, std::memory_order_acq_rel);
      acquire(timeout_us);
      if (waiting) waiting->fetch_sub(1, std::memory_order_acq_rel);
    }
    void acquire(int64_t timeout_us) {
      const uint32_t me = uint32_t(::getpid());
      const auto t0 = std::chrono::steady_clock::now();
      auto next_check = t0 + std::chrono::milliseconds(1);
      for (int spin = 0;; ++spin) {
        uint32_t z = 0;
        if (l.compare_exchange_weak(z, me, std::memory_order_acquire, std::memory_order_relaxed)) {
          held = true;
          return;
        }
        // writers back off to sleeps; a reader keeps yielding (the inserter holds the lock for
        // one chunk at a time and hands it over when readers wait: a sleeping reader would
        // oversleep that window by the timer slack)
        if (spin > 256 && timeout_us < 0) std::this_thread::sleep_for(std::chrono::microseconds(5));
        else if (spin > 32) std::this_thread::yield();
        if (spin > 32) {
          const auto t = std::chrono::steady_clock::now();
          if (t >= next_check) {
            next_check = t + std::chrono::milliseconds(1);
            uint32_t owner = l.load(std::memory_order_relaxed);
            if (owner != 0 && owner != me && ::kill(pid_t(owner), 0) != 0 && errno == ESRCH &&
                l.compare_exchange_strong(owner, me, std::memory_order_acquire, std::memory_order_relaxed)) {
              takeovers_.fetch_add(1, std::memory_order_relaxed);
              held = true;
              return;
            }
          }
          if (timeout_us >= 0 && t - t0 >= std::chrono::microseconds(timeout_us)) return;
        }
      }
    }
    void leak() { held = false; }
    ~Guard() {
      if (held) l.store(0, std::memory_order_release);
    }
  };

  // table keys are never 0 (empty): device digests are non-zero, account keys are stored + 1
  static uint64_t akey(int64_t acct) { return uint64_t(acct) + 1; }
  // bucket = 4 key slots in one 64-byte line; the value lists live in a parallel array and are
  // touched only for the matching (or evicted) slot
  struct Key {
    uint64_t key;    // 0 = empty
    uint32_t stamp;  // last touch (eviction order within the bucket)
    int32_t n;       // values held
  };
  struct alignas(64) Bucket {
    Key k[4];
  };
  struct Entry {
    Key* kk;
    int64_t* v;  // oldest first
    int32_t& n() { return kk->n; }
  };
  struct CEntry {
    const Key* kk;
    const int64_t* v;
    int32_t n;
  };
  struct Table {
    Bucket* b = nullptr;
    int64_t* vals = nullptr;  // [buckets * 4][kMaxPerKey]
    uint64_t mask = 0;
    static size_t bytes(int64_t buckets) {
      return sizeof(Bucket) * size_t(buckets) + sizeof(int64_t) * size_t(buckets) * 4 * kMaxPerKey;
    }
    void map(char* base, int64_t buckets) {
      b = reinterpret_cast<Bucket*>(base);
      vals = reinterpret_cast<int64_t*>(base + sizeof(Bucket) * size_t(buckets));
      mask = uint64_t(buckets - 1);
    }
    static uint64_t mix(uint64_t k) {
      k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33;
      return k;
    }
    void prefetch(uint64_t key) const { __builtin_prefetch(&b[mix(key) & mask]); }
    bool find(uint64_t key, CEntry& out) const {
      if (key == 0) return false;
      const size_t bi = mix(key) & mask;
      for (int w = 0; w < 4; ++w)
        if (b[bi].k[w].key == key) {
          out = CEntry{&b[bi].k[w], &vals[(bi * 4 + w) * kMaxPerKey], b[bi].k[w].n};
          return true;
        }
      return false;
    }
    Entry touch(uint64_t key, uint32_t now, uint64_t& used) {
      const size_t bi = mix(key) & mask;
      Key* k = b[bi].k;
      int victim = 0;
      for (int w = 0; w < 4; ++w) {
        if (k[w].key == key) {
          k[w].stamp = now;
          return Entry{k + w, &vals[(bi * 4 + w) * kMaxPerKey]};
        }
        if (k[w].key == 0) { victim = w; break; }
        if (k[w].stamp < k[victim].stamp) victim = w;
      }
      if (k[victim].key == 0) ++used;
      k[victim] = Key{key, now, 0};
      return Entry{k + victim, &vals[(bi * 4 + victim) * kMaxPerKey]};
    }
  };

  void init(int per_key, int64_t buckets, const std::string& shm_name, bool create) {
    int64_t nb = 1;
    while (nb < buckets) nb <<= 1;
    const size_t tb = Table::bytes(nb);
    const size_t total = sizeof(Hdr) + 2 * tb;
    const bool fresh = shm_name.empty() || create;
    region_ = shm_name.empty() ? Region::anon(total) : Region::shared(shm_name, total, create);
    char* base = static_cast<char*>(region_.base());
    hdr_ = reinterpret_cast<Hdr*>(base);
    if (fresh) {  // zero pages (anonymous / a fresh sparse file): empty tables
      hdr_->buckets = nb;
      hdr_->per_key = std::max(1, std::min(per_key, kMaxPerKey));
      hdr_->magic = kMagic;
    } else if (hdr_->magic != kMagic || hdr_->buckets != nb) {
      throw std::runtime_error("LinkIndex: " + shm_name + " has another layout");
    }
    per_key_ = hdr_->per_key;
    dev_.map(base + sizeof(Hdr), nb);
    acct_.map(base + sizeof(Hdr) + tb, nb);
  }

  void linked_locked(int64_t acct, size_t limit, std::vector<int64_t>& out) const {
    CEntry a;
    if (!acct_.find(akey(acct), a)) return;
    for (int d = a.n - 1; d >= 0; --d) {
      CEntry e;
      if (!dev_.find(uint64_t(a.v[d]), e)) continue;
      for (int k = e.n - 1; k >= 0; --k) {
        const int64_t x = e.v[k];
        if (x == acct || std::find(out.begin(), out.end(), x) != out.end()) continue;
        out.push_back(x);
        if (out.size() >= limit) return;
      }
    }
  }

  void push(Entry en, int64_t x) {
    int32_t& n = en.n();
    for (int k = 0; k < n; ++k)
      if (en.v[k] == x) {  // move to the most recent position
        std::memmove(en.v + k, en.v + k + 1, sizeof(int64_t) * size_t(n - k - 1));
        en.v[n - 1] = x;
        return;
      }
    if (n >= per_key_) {
      std::memmove(en.v, en.v + 1, sizeof(int64_t) * size_t(n - 1));
      en.v[n - 1] = x;
      return;
    }
    en.v[n++] = x;
  }

  Region region_;
  Hdr* hdr_ = nullptr;
  int per_key_ = 8;
  Table dev_, acct_;
  std::atomic<uint64_t> enq_{0}, done_{0};
};

inline std::atomic<int64_t> LinkIndex::takeovers_{0};
inline std::atomic<int64_t> LinkIndex::read_timeouts_{0};

}  // namespace igp

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
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

namespace igp {

class LinkIndex {
 public:
  static constexpr int kMaxPerKey = 16;

  explicit LinkIndex(int per_key = 8, int64_t buckets = int64_t(1) << 18)
      : per_key_(std::max(1, std::min(per_key, kMaxPerKey))) {
    int64_t b = 1;
    while (b < buckets) b <<= 1;
    dev_.init(b);
    acct_.init(b);
  }

  void add(const uint64_t* dev, const int64_t* acct, size_t n) {
    constexpr size_t kAhead = 8;
    std::lock_guard<std::mutex> g(mu_);
    for (size_t i = 0; i < n; ++i) {
      if (i + kAhead < n) {
        dev_.prefetch(dev[i + kAhead]);
        acct_.prefetch(akey(acct[i + kAhead]));
      }
      if (dev[i] == 0 || acct[i] < 0) continue;
      ++clock_;
      push(dev_.touch(dev[i], clock_), acct[i]);
      push(acct_.touch(akey(acct[i]), clock_), int64_t(dev[i]));
    }
  }

  // accounts sharing at least one device with `acct` (excluding itself), most recent first
  std::vector<int64_t> linked(int64_t acct, size_t limit) const {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<int64_t> out;
    CEntry a;
    if (!acct_.find(akey(acct), a)) return out;
    for (int d = a.n - 1; d >= 0; --d) {
      CEntry e;
      if (!dev_.find(uint64_t(a.v[d]), e)) continue;
      for (int k = e.n - 1; k >= 0; --k) {
        const int64_t x = e.v[k];
        if (x == acct || std::find(out.begin(), out.end(), x) != out.end()) continue;
        out.push_back(x);
        if (out.size() >= limit) return out;
      }
    }
    return out;
  }

  std::vector<int64_t> devices_of(int64_t acct) const {
    std::lock_guard<std::mutex> g(mu_);
    CEntry a;
    return acct_.find(akey(acct), a) ? std::vector<int64_t>(a.v, a.v + a.n) : std::vector<int64_t>{};
  }

  size_t n_devices() const {
    std::lock_guard<std::mutex> g(mu_);
    return dev_.used;
  }

 private:
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
    std::vector<Bucket> b;
    std::vector<int64_t> vals;  // [buckets * 4][kMaxPerKey]
    uint64_t mask = 0;
    size_t used = 0;
    void init(int64_t buckets) {
      b.assign(size_t(buckets), Bucket{});
      vals.assign(size_t(buckets) * 4 * kMaxPerKey, 0);
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
    Entry touch(uint64_t key, uint32_t now) {
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
  int per_key_;
  uint32_t clock_ = 0;
  Table dev_, acct_;
  mutable std::mutex mu_;
};

}  // namespace igp

// Device <-> account co-occurrence index for multi-account detection (CheckBonusAbuse's
// linked_accounts, risk.proto:135-145; the reference declares the field but never fills it).
//
// Every scored request contributes (device digest, account key) where the account key is
// (owner << 32 | slot). Both directions are bounded (most recent `per_key` entries, LRU by
// overwrite) so an abusive device shared by millions of rows cannot grow the index without
// bound. Thread-safe; the batch insert takes one lock per batch.
#pragma once
#include <cstdint>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace igp {

class LinkIndex {
 public:
  explicit LinkIndex(int per_key = 32) : per_key_(per_key < 1 ? 1 : per_key) {}

  void add(const uint64_t* dev, const int64_t* acct, size_t n) {
    std::lock_guard<std::mutex> g(mu_);
    for (size_t i = 0; i < n; ++i) {
      if (dev[i] == 0 || acct[i] < 0) continue;
      push(by_dev_[dev[i]], acct[i]);
      push(by_acct_[acct[i]], int64_t(dev[i]));
    }
  }

  // accounts sharing at least one device with `acct` (excluding itself), most recent first
  std::vector<int64_t> linked(int64_t acct, size_t limit) const {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<int64_t> out;
    auto it = by_acct_.find(acct);
    if (it == by_acct_.end()) return out;
    for (auto d = it->second.rbegin(); d != it->second.rend(); ++d) {
      auto jt = by_dev_.find(uint64_t(*d));
      if (jt == by_dev_.end()) continue;
      for (auto a = jt->second.rbegin(); a != jt->second.rend(); ++a) {
        if (*a == acct) continue;
        bool seen = false;
        for (int64_t x : out) seen |= (x == *a);
        if (!seen) out.push_back(*a);
        if (out.size() >= limit) return out;
      }
    }
    return out;
  }

  std::vector<int64_t> devices_of(int64_t acct) const {
    std::lock_guard<std::mutex> g(mu_);
    auto it = by_acct_.find(acct);
    return it == by_acct_.end() ? std::vector<int64_t>{} : it->second;
  }

  size_t n_devices() const {
    std::lock_guard<std::mutex> g(mu_);
    return by_dev_.size();
  }

 private:
  void push(std::vector<int64_t>& v, int64_t x) {
    for (size_t k = 0; k < v.size(); ++k)
      if (v[k] == x) {  // move to most-recent position
        v.erase(v.begin() + k);
        break;
      }
    if ((int)v.size() >= per_key_) v.erase(v.begin());
    v.push_back(x);
  }
  int per_key_;
  std::unordered_map<uint64_t, std::vector<int64_t>> by_dev_;
  std::unordered_map<int64_t, std::vector<int64_t>> by_acct_;
  mutable std::mutex mu_;
};

}  // namespace igp

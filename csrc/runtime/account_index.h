// Account-id -> feature-store slot map (one per GPU shard).
//
// Replaces the per-account Redis key namespace ``features:<uuid>:*`` of
// services/risk/internal/features/redis_store.go:25-35. Open addressing on the XXH64
// digest with the full id kept for verification (digest collisions resolve by probing),
// so ids of any length/format work. Thread-safe (readers share, inserts exclusive).
#pragma once
#include <algorithm>
#include <cstdint>
#include <shared_mutex>
#include <string>
#include <string_view>
#include <vector>

namespace igp {

class AccountIndex {
 public:
  explicit AccountIndex(int64_t capacity);
  // slot of id, or -1
  int32_t find(std::string_view id, uint64_t h) const;
  // slot of id, inserting a fresh slot if absent; -1 if the index is full
  int32_t find_or_insert(std::string_view id, uint64_t h, bool* inserted = nullptr);
  void lookup(const std::vector<std::string>& ids, const std::vector<uint64_t>& hashes,
              bool insert, int32_t* slots, uint8_t* fresh);
  int64_t size() const { return n_; }
  int64_t capacity() const { return cap_; }
  std::string id_of(int32_t slot) const;

 private:
  int64_t probe(std::string_view id, uint64_t h, bool& found) const;
  int64_t cap_;
  int64_t mask_;
  int64_t n_ = 0;
  std::vector<uint64_t> keys_;   // 0 = empty (digest 0 is never stored: ids are non-empty)
  std::vector<int32_t> slot_;
  std::vector<std::string> ids_; // by slot
  mutable std::shared_mutex mu_;
};

}  // namespace igp

// Account-id -> feature-store slot map (one per GPU shard).
//
// Replaces the per-account Redis key namespace ``features:<uuid>:*`` of
// services/risk/internal/features/redis_store.go:25-35. Open addressing over 16-byte entries
// {XXH64 digest, 32-bit check digest (a second, independently seeded XXH64), slot}: one
// cache line holds four entries and a lookup touches one line, with no pointer chase to the
// stored id string (96 bits identify an id; a false match needs ~2^48 ids). The batch path
// prefetches every probe line of the batch before probing (memory-level parallelism over
// ~8192 random lookups) and takes the lock once per batch. Full ids are kept by slot for the
// reverse map (id_of: linked accounts, snapshots).
#pragma once
#include <algorithm>
#include <cstdint>
#include <shared_mutex>
#include <string>
#include <string_view>
#include <vector>

#include "xxh64.h"

namespace igp {

constexpr uint64_t SEED_ACCOUNT_CHECK = 0x41434b32;  // "ACK2"

inline uint32_t id_check(std::string_view s) { return uint32_t(xxh64(s.data(), s.size(), SEED_ACCOUNT_CHECK) >> 32); }

class AccountIndex {
 public:
  explicit AccountIndex(int64_t capacity);
  // slot of id, or -1
  int32_t find(std::string_view id, uint64_t h) const;
  // slot of id, inserting a fresh slot if absent; -1 if the index is full
  int32_t find_or_insert(std::string_view id, uint64_t h, bool* inserted = nullptr);
  void lookup(const std::vector<std::string>& ids, const std::vector<uint64_t>& hashes,
              bool insert, int32_t* slots, uint8_t* fresh);
  // batch path: ids[k] with precomputed digests; rows with sel[k] == 0 are skipped (slot -1)
  void lookup_views(const std::string_view* ids, const uint64_t* h, const uint32_t* check, size_t n, bool insert,
                    int32_t* slots, uint8_t* fresh, const uint8_t* sel = nullptr);
  int64_t size() const { return n_; }
  int64_t capacity() const { return cap_; }
  std::string id_of(int32_t slot) const;

 private:
  struct Entry {
    uint64_t h;      // 0 = empty (digest 0 is never stored: ids are non-empty)
    uint32_t check;
    int32_t slot;
  };
  static_assert(sizeof(Entry) == 16, "AccountIndex entry must be 16 bytes");
  int64_t probe(uint64_t h, uint32_t check, bool& found) const;
  int32_t insert_at(int64_t i, std::string_view id, uint64_t h, uint32_t check);
  int64_t cap_;
  int64_t mask_;
  int64_t n_ = 0;
  std::vector<Entry> tab_;
  std::vector<std::string> ids_; // by slot
  mutable std::shared_mutex mu_;
};

}  // namespace igp

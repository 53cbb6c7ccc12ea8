// Account-id -> feature-store slot map (one per owner shard).
//
// Replaces the per-account Redis key namespace ``features:<uuid>:*`` of
// services/risk/internal/features/redis_store.go:25-35.
//
// Lock-free open addressing over 32-byte entries {XXH64 digest, state, id offset, inline key};
// the id bytes live in an append-only arena, so identity is the exact id string (a digest match
// is always confirmed against the id: two ids that collide on 64 bits get two slots, and the
// collision is counted). The inline key makes that confirmation free for the common ids: a
// canonical UUID string (36 chars, lower-case hex) is stored as its 16 binary bytes and a short
// id (<= 15 bytes) verbatim, both exact encodings of the string, so a lookup costs ONE cache
// miss (the entry) instead of two (entry + arena); longer ids keep a 16-byte prefix for a
// fast reject and are confirmed against the arena (uniform traffic over 1 M
// accounts made the second miss the resolve cost). Inserts claim an empty entry with one 64-bit CAS, take the
// next slot with a fetch_add, write the id, then publish the slot with a release store;
// readers that meet a claimed-but-unpublished entry spin until it is published.
//
// The table can live in a node-shared /dev/shm region: every rank of a one-process-per-GPU
// group then resolves ids through the same table, so an account gets ONE slot on its owner
// no matter which rank's ingress saw it first (multi-ingress serving, engine/serving.py).
// The batch path prefetches every probe line, then every candidate's id bytes, before it
// compares (memory-level parallelism over ~8192 random lookups per batch).
#pragma once
#include <atomic>
#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

#include "shm.h"
#include "xxh64.h"

namespace igp {

class AccountIndex {
 public:
  // process-private index
  explicit AccountIndex(int64_t capacity);
  // node-shared index in /dev/shm/<name> (create: this process sizes and initialises it)
  AccountIndex(int64_t capacity, const std::string& shm_name, bool create);

  // slot of id, or -1
  int32_t find(std::string_view id, uint64_t h) const;
  // slot of id, inserting a fresh slot if absent; -1 if the index is full
  int32_t find_or_insert(std::string_view id, uint64_t h, bool* inserted = nullptr);
  void lookup(const std::vector<std::string>& ids, const std::vector<uint64_t>& hashes, bool insert, int32_t* slots,
              uint8_t* fresh);
  // batch path: ids[k] with precomputed digests; rows with sel[k] == 0 are skipped (slot -1)
  void lookup_views(const std::string_view* ids, const uint64_t* h, size_t n, bool insert, int32_t* slots,
                    uint8_t* fresh, const uint8_t* sel = nullptr);
  int64_t size() const;
  int64_t capacity() const { return hdr_->cap; }
  int64_t collisions() const { return hdr_->collisions.load(std::memory_order_relaxed); }
  std::string id_of(int32_t slot) const;
  // the id bytes in the arena (no copy); empty for an out-of-range slot
  std::string_view id_view(int32_t slot) const;
  bool shared() const { return region_.shared_mapping(); }
  void unlink_shared() { region_.unlink(); }

  static size_t region_bytes(int64_t capacity);

 private:
  struct Hdr {
    uint64_t magic;
    int64_t cap;
    int64_t tsize;        // power of two, >= 2 * cap
    int64_t arena_bytes;
    std::atomic<int64_t> n;           // slots handed out (may pass cap by the racing inserts that lost)
    std::atomic<int64_t> arena_used;  // bytes
    std::atomic<int64_t> collisions;  // distinct ids sharing a 64-bit digest
    std::atomic<int32_t> ready;
    int32_t pad[5];
  };
  struct Entry {
    std::atomic<uint64_t> h;      // 0 = empty
    std::atomic<int32_t> state;   // 0 = claimed, not yet published; s + 1 = slot s; -1 = dead (index full)
    uint32_t off8;                // id offset in the arena, 8-byte units | kExact | kUuid
    uint8_t key[16];              // inline key (written before the publish)
  };
  static_assert(sizeof(Entry) == 32, "AccountIndex entry must be 32 bytes");
  static constexpr uint32_t kExact = 1u << 31, kUuid = 1u << 30, kOffMask = (1u << 30) - 1;
 public:
  // the inline key of an id: returns kExact [| kUuid] when the key IS the id (exact encoding)
  static uint32_t encode_key(std::string_view id, uint8_t key[16], bool scalar = false);
 private:
  bool key_equal(const Entry& e, std::string_view id, uint32_t form, const uint8_t* key) const;

  void layout(void* base);
  void init_fresh(int64_t capacity);
  int32_t published(const Entry& e) const;  // spins on a claimed entry; slot or -1 (dead / stuck)
  bool id_equal(uint32_t off8, std::string_view id) const;
  int32_t find_from(int64_t i, std::string_view id, uint64_t h) const;
  int32_t insert(std::string_view id, uint64_t h, bool* inserted);

  Region region_;
  Hdr* hdr_ = nullptr;
  Entry* tab_ = nullptr;
  uint32_t* slot_off_ = nullptr;  // slot -> id offset (8-byte units)
  char* arena_ = nullptr;
  int64_t mask_ = 0;
};

}  // namespace igp

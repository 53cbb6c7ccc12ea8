#include "account_index.h"

#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace igp {
namespace {

constexpr uint64_t kMagic = 0x3258444954434341ull;  // "ACCTIDX2" (32-byte entries with inline keys)
constexpr int64_t kArenaPerAccount = 64;            // bytes reserved per slot (4-byte length + id, 8-aligned)

int64_t table_size(int64_t capacity) {
  int64_t t = 16;
  while (t < capacity * 2) t <<= 1;  // load factor <= 0.5
  return t;
}

inline void cpu_relax() { __builtin_ia32_pause(); }

}  // namespace

size_t AccountIndex::region_bytes(int64_t capacity) {
  const int64_t t = table_size(capacity);
  return sizeof(Hdr) + size_t(t) * sizeof(Entry) + size_t(capacity) * sizeof(uint32_t) + 64 +
         size_t(capacity) * kArenaPerAccount;
}

void AccountIndex::layout(void* base) {
  hdr_ = reinterpret_cast<Hdr*>(base);
  tab_ = reinterpret_cast<Entry*>(reinterpret_cast<char*>(base) + sizeof(Hdr));
  slot_off_ = reinterpret_cast<uint32_t*>(tab_ + hdr_->tsize);
  const uintptr_t a = reinterpret_cast<uintptr_t>(slot_off_ + hdr_->cap);
  arena_ = reinterpret_cast<char*>((a + 63) & ~uintptr_t(63));
  mask_ = hdr_->tsize - 1;
}

void AccountIndex::init_fresh(int64_t capacity) {
  // the mapping is zero-filled: every entry is empty (h = 0) already
  Hdr* h = reinterpret_cast<Hdr*>(region_.base());
  h->magic = kMagic;
  h->cap = capacity;
  h->tsize = table_size(capacity);
  h->arena_bytes = capacity * kArenaPerAccount;
  h->n.store(0);
  h->arena_used.store(8);  // offset 0 is never a valid id
  h->collisions.store(0);
  layout(h);
  h->ready.store(1, std::memory_order_release);
}

AccountIndex::AccountIndex(int64_t capacity) {
  if (capacity <= 0) throw std::runtime_error("AccountIndex: capacity must be > 0");
  region_ = Region::anon(region_bytes(capacity));
  init_fresh(capacity);
}

AccountIndex::AccountIndex(int64_t capacity, const std::string& shm_name, bool create) {
  if (capacity <= 0) throw std::runtime_error("AccountIndex: capacity must be > 0");
  const size_t bytes = region_bytes(capacity);
  region_ = Region::shared(shm_name, bytes, create);
  if (create) {
    init_fresh(capacity);
    return;
  }
  Hdr* h = reinterpret_cast<Hdr*>(region_.base());
  for (int i = 0; h->ready.load(std::memory_order_acquire) != 1; ++i) {
    if (i > 20000) throw std::runtime_error("AccountIndex: shared index " + shm_name + " never became ready");
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
  if (h->magic != kMagic || h->cap != capacity) throw std::runtime_error("AccountIndex: shared index layout mismatch");
  layout(h);
}

int64_t AccountIndex::size() const { return std::min(hdr_->n.load(std::memory_order_acquire), hdr_->cap); }

int32_t AccountIndex::published(const Entry& e) const {
  int32_t st = e.state.load(std::memory_order_acquire);
  for (int spin = 0; st == 0; ++spin) {
    // an insert is between its claim and its publish (a few hundred ns); a process that died
    // there leaves the entry claimed for good: give up after ~50 ms (the row scores as an
    // unknown account, partial features)
    if (spin > (1 << 16)) {
      if (spin > (1 << 16) + 500) return -1;
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    } else {
      cpu_relax();
    }
    st = e.state.load(std::memory_order_acquire);
  }
  return st > 0 ? st - 1 : -1;
}

namespace {
// char -> hex digit value; 0x10 marks a char that is not a lower-case hex digit (upper case is not
// the canonical UUID form: such ids take the non-UUID encoding)
struct HexTable {
  uint8_t v[256];
  constexpr HexTable() : v() {
    for (int i = 0; i < 256; ++i) v[i] = 0x10;
    for (int i = 0; i < 10; ++i) v['0' + i] = uint8_t(i);
    for (int i = 0; i < 6; ++i) v['a' + i] = uint8_t(10 + i);
  }
};
constexpr HexTable kHex;
// byte k of a canonical UUID = hex pair at these string positions (hyphens at 8, 13, 18, 23)
constexpr uint8_t kPos[16] = {0, 2, 4, 6, 9, 11, 14, 16, 19, 21, 24, 26, 28, 30, 32, 34};
}  // namespace

// The 32 hex digits of a canonical lower-case UUID -> 16 key bytes, SSSE3: three unaligned loads,
// byte shuffles that drop the hyphens, a range check and a nibble pack (the table loop above was
// ~13 % of the ingress threads' samples; resolve 42 -> 35 ns/row, serving throughput unchanged:
// not ingress-bound, profiles/r5/host/keys). false: not 32 lower-case hex digits.
__attribute__((target("ssse3"))) static bool uuid_hex_simd(const unsigned char* c, uint8_t key[16]) {
  const __m128i v0 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(c));       // chars 0..15
  const __m128i v1 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(c + 16));  // chars 16..31
  const __m128i v2 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(c + 20));  // chars 20..35
  const char z = char(0x80);
  // key bytes 0..7 <- chars 0-7, 9-12, 14-17; key bytes 8..15 <- chars 19-22, 24-35
  const __m128i a = _mm_or_si128(
      _mm_shuffle_epi8(v0, _mm_setr_epi8(0, 1, 2, 3, 4, 5, 6, 7, 9, 10, 11, 12, 14, 15, z, z)),
      _mm_shuffle_epi8(v1, _mm_setr_epi8(z, z, z, z, z, z, z, z, z, z, z, z, z, z, 0, 1)));
  const __m128i b = _mm_or_si128(
      _mm_shuffle_epi8(v1, _mm_setr_epi8(3, 4, 5, 6, 8, 9, 10, 11, 12, 13, 14, 15, z, z, z, z)),
      _mm_shuffle_epi8(v2, _mm_setr_epi8(z, z, z, z, z, z, z, z, z, z, z, z, 12, 13, 14, 15)));
  auto nibbles = [](__m128i v, __m128i& ok) {
    const __m128i d = _mm_sub_epi8(v, _mm_set1_epi8('0'));
    const __m128i h = _mm_sub_epi8(v, _mm_set1_epi8('a'));
    const __m128i is_d = _mm_cmpeq_epi8(_mm_min_epu8(d, _mm_set1_epi8(9)), d);  // d <= 9 unsigned
    const __m128i is_h = _mm_cmpeq_epi8(_mm_min_epu8(h, _mm_set1_epi8(5)), h);  // h <= 5 unsigned
    ok = _mm_and_si128(ok, _mm_or_si128(is_d, is_h));
    return _mm_or_si128(_mm_and_si128(is_d, d), _mm_and_si128(is_h, _mm_add_epi8(h, _mm_set1_epi8(10))));
  };
  __m128i ok = _mm_set1_epi8(char(0xff));
  const __m128i na = nibbles(a, ok), nb = nibbles(b, ok);
  if (_mm_movemask_epi8(ok) != 0xffff) return false;
  const __m128i w = _mm_set1_epi16(0x0110);  // even char x 16 + odd char
  const __m128i packed = _mm_packus_epi16(_mm_maddubs_epi16(na, w), _mm_maddubs_epi16(nb, w));
  _mm_storeu_si128(reinterpret_cast<__m128i*>(key), packed);
  return true;
}

// the scalar decode (table lookups): the reference the SIMD path is tested against
static bool uuid_hex_scalar(const unsigned char* c, uint8_t key[16]) {
  uint32_t bad = 0;
  for (int k = 0; k < 16; ++k) {
    const uint32_t hi = kHex.v[c[kPos[k]]], lo = kHex.v[c[kPos[k] + 1]];
    bad |= hi | lo;
    key[k] = uint8_t(hi << 4 | lo);
  }
  return !(bad & 0x10);
}

uint32_t AccountIndex::encode_key(std::string_view id, uint8_t key[16], bool scalar) {
  const unsigned char* c = reinterpret_cast<const unsigned char*>(id.data());
  if (id.size() == 36 && c[8] == '-' && c[13] == '-' && c[18] == '-' && c[23] == '-') {
    if (scalar ? uuid_hex_scalar(c, key) : uuid_hex_simd(c, key)) return kExact | kUuid;
  }
  std::memset(key, 0, 16);
  if (id.size() <= 15) {
    key[0] = uint8_t(id.size());
    std::memcpy(key + 1, id.data(), id.size());
    return kExact;
  }
  std::memcpy(key, id.data(), 16);  // prefix of a long id: a fast reject before the arena compare
  return 0;
}

bool AccountIndex::key_equal(const Entry& e, std::string_view id, uint32_t form, const uint8_t* key) const {
  if ((e.off8 & (kExact | kUuid)) != form) return false;  // the encoding form is a function of the id
  if (std::memcmp(e.key, key, 16) != 0) return false;
  return (form & kExact) || id_equal(e.off8 & kOffMask, id);
}

bool AccountIndex::id_equal(uint32_t off8, std::string_view id) const {
  const char* p = arena_ + size_t(off8) * 8;
  uint32_t len;
  std::memcpy(&len, p, 4);
  return len == id.size() && std::memcmp(p + 4, id.data(), id.size()) == 0;
}

int32_t AccountIndex::find_from(int64_t i, std::string_view id, uint64_t h) const {
  uint8_t key[16];
  const uint32_t form = encode_key(id, key);
  for (int64_t probes = 0; probes <= mask_; ++probes, i = (i + 1) & mask_) {
    const Entry& e = tab_[size_t(i)];
    const uint64_t hv = e.h.load(std::memory_order_acquire);
    if (hv == 0) return -1;
    if (hv != h) continue;
    const int32_t s = published(e);
    if (s >= 0 && key_equal(e, id, form, key)) return s;
  }
  return -1;
}

int32_t AccountIndex::find(std::string_view id, uint64_t h) const {
  if (h == 0) return -1;
  return find_from(int64_t(h & uint64_t(mask_)), id, h);
}

int32_t AccountIndex::insert(std::string_view id, uint64_t h, bool* inserted) {
  if (inserted) *inserted = false;
  if (h == 0) return -1;
  uint8_t key[16];
  const uint32_t form = encode_key(id, key);
  int64_t i = int64_t(h & uint64_t(mask_));
  for (int64_t probes = 0; probes <= mask_; ++probes, i = (i + 1) & mask_) {
    Entry& e = tab_[size_t(i)];
    uint64_t hv = e.h.load(std::memory_order_acquire);
    if (hv == 0) {
      if (hdr_->n.load(std::memory_order_relaxed) >= hdr_->cap) return -1;  // full: claim nothing
      if (e.h.compare_exchange_strong(hv, h, std::memory_order_acq_rel)) {
        const int64_t s = hdr_->n.fetch_add(1, std::memory_order_acq_rel);
        if (s >= hdr_->cap) {  // lost the race for the last slot
          e.state.store(-1, std::memory_order_release);
          return -1;
        }
        const int64_t need = (4 + int64_t(id.size()) + 7) & ~int64_t(7);
        const int64_t off = hdr_->arena_used.fetch_add(need, std::memory_order_relaxed);
        if (off + need > hdr_->arena_bytes) {  // ids far longer than a UUID filled the arena
          e.state.store(-1, std::memory_order_release);
          return -1;
        }
        char* p = arena_ + off;
        const uint32_t len = uint32_t(id.size());
        std::memcpy(p, &len, 4);
        std::memcpy(p + 4, id.data(), id.size());
        if (off / 8 > int64_t(kOffMask)) {
          e.state.store(-1, std::memory_order_release);
          return -1;
        }
        std::memcpy(e.key, key, 16);
        e.off8 = uint32_t(off / 8) | form;
        slot_off_[s] = uint32_t(off / 8);
        e.state.store(int32_t(s + 1), std::memory_order_release);
        if (inserted) *inserted = true;
        return int32_t(s);
      }
      // another inserter claimed this entry first: hv now holds its digest
    }
    if (hv != h) continue;
    const int32_t s = published(e);
    if (s >= 0) {
      if (key_equal(e, id, form, key)) return s;
      hdr_->collisions.fetch_add(1, std::memory_order_relaxed);
    }
  }
  return -1;
}

int32_t AccountIndex::find_or_insert(std::string_view id, uint64_t h, bool* inserted) {
  const int32_t s = find(id, h);
  if (s >= 0) {
    if (inserted) *inserted = false;
    return s;
  }
  return insert(id, h, inserted);
}

void AccountIndex::lookup(const std::vector<std::string>& ids, const std::vector<uint64_t>& hashes, bool insert_,
                          int32_t* slots, uint8_t* fresh) {
  std::vector<std::string_view> v(ids.begin(), ids.end());
  lookup_views(v.data(), hashes.data(), ids.size(), insert_, slots, fresh);
}

void AccountIndex::lookup_views(const std::string_view* ids, const uint64_t* h, size_t n, bool insert_, int32_t* slots,
                                uint8_t* fresh, const uint8_t* sel) {
  constexpr size_t kAhead = 16;  // probe lines in flight (32: same, 64: slower; profiles/r5/host)
  // pass 1: probe every row (prefetched); an exact inline key settles the row on the spot (one
  // miss per row); long ids remember their candidate and prefetch its arena bytes
  std::vector<int64_t> cand;
  std::vector<uint32_t> later;
  const Entry* t = tab_;
  for (size_t k = 0; k < std::min(n, kAhead); ++k) __builtin_prefetch(t + (h[k] & uint64_t(mask_)));
  uint8_t key[16];
  for (size_t k = 0; k < n; ++k) {
    if (k + kAhead < n) __builtin_prefetch(t + (h[k + kAhead] & uint64_t(mask_)));
    if (fresh) fresh[k] = 0;
    slots[k] = -1;
    if (h[k] == 0 || (sel && !sel[k])) continue;
    const uint32_t form = encode_key(ids[k], key);
    int64_t i = int64_t(h[k] & uint64_t(mask_));
    bool settled = false, deferred = false;
    for (int64_t probes = 0; probes <= mask_; ++probes, i = (i + 1) & mask_) {
      const Entry& e = t[size_t(i)];
      const uint64_t hv = e.h.load(std::memory_order_acquire);
      if (hv == 0) break;
      if (hv != h[k]) continue;
      if (!(form & kExact)) {  // confirm against the arena in pass 2
        if (e.state.load(std::memory_order_acquire) > 0) __builtin_prefetch(arena_ + size_t(e.off8 & kOffMask) * 8);
        if (cand.empty()) cand.assign(n, -1);
        cand[k] = i;
        later.push_back(uint32_t(k));
        deferred = true;
        break;
      }
      const int32_t s = published(e);
      if (s >= 0 && key_equal(e, ids[k], form, key)) {
        slots[k] = s;
        settled = true;
        break;
      }
    }
    if (!settled && !deferred && insert_) later.push_back(uint32_t(k));
  }
  // pass 2: long ids against the stored bytes (lines already in flight), then inserts in row
  // order (a batch's new accounts get slots in arrival order)
  std::vector<uint32_t> miss;
  for (uint32_t k : later) {
    if (!cand.empty() && cand[k] >= 0) {
      const int32_t s2 = find_from(cand[k], ids[k], h[k]);
      if (s2 >= 0) {
        slots[k] = s2;
        continue;
      }
    }
    if (insert_) miss.push_back(k);
  }
  for (uint32_t k : miss) {
    bool ins = false;
    slots[k] = insert(ids[k], h[k], &ins);
    if (fresh) fresh[k] = ins;
  }
}

std::string AccountIndex::id_of(int32_t slot) const {
  if (slot < 0 || slot >= size()) throw std::runtime_error("AccountIndex: bad slot");
  const char* p = arena_ + size_t(slot_off_[slot]) * 8;
  uint32_t len;
  std::memcpy(&len, p, 4);
  return std::string(p + 4, len);
}

std::string_view AccountIndex::id_view(int32_t slot) const {
  if (slot < 0 || slot >= size()) return {};
  const char* p = arena_ + size_t(slot_off_[slot]) * 8;
  uint32_t len;
  std::memcpy(&len, p, 4);
  return std::string_view(p + 4, len);
}

}  // namespace igp

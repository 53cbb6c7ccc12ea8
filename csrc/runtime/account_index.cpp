#include "account_index.h"

#include <mutex>
#include <stdexcept>

namespace igp {

AccountIndex::AccountIndex(int64_t capacity) {
  if (capacity <= 0) throw std::runtime_error("AccountIndex: capacity must be > 0");
  int64_t t = 16;
  while (t < capacity * 2) t <<= 1;  // load factor <= 0.5
  cap_ = capacity;
  mask_ = t - 1;
  tab_.assign(size_t(t), Entry{0, 0, -1});
  ids_.reserve(size_t(std::min<int64_t>(capacity, 1 << 20)));
}

int64_t AccountIndex::probe(uint64_t h, uint32_t check, bool& found) const {
  int64_t i = int64_t(h & uint64_t(mask_));
  for (;;) {
    const Entry& e = tab_[size_t(i)];
    if (e.h == 0) { found = false; return i; }
    if (e.h == h && e.check == check) { found = true; return i; }
    i = (i + 1) & mask_;
  }
}

int32_t AccountIndex::insert_at(int64_t i, std::string_view id, uint64_t h, uint32_t check) {
  if (n_ >= cap_) return -1;
  tab_[size_t(i)] = Entry{h, check, int32_t(n_)};
  ids_.emplace_back(id);
  return int32_t(n_++);
}

int32_t AccountIndex::find(std::string_view id, uint64_t h) const {
  if (h == 0) return -1;
  const uint32_t c = id_check(id);
  std::shared_lock<std::shared_mutex> lk(mu_);
  bool found;
  int64_t i = probe(h, c, found);
  return found ? tab_[size_t(i)].slot : -1;
}

int32_t AccountIndex::find_or_insert(std::string_view id, uint64_t h, bool* inserted) {
  if (inserted) *inserted = false;
  if (h == 0) return -1;
  const uint32_t c = id_check(id);
  {
    std::shared_lock<std::shared_mutex> lk(mu_);
    bool found;
    int64_t i = probe(h, c, found);
    if (found) return tab_[size_t(i)].slot;
  }
  std::unique_lock<std::shared_mutex> lk(mu_);
  bool found;
  int64_t i = probe(h, c, found);
  if (found) return tab_[size_t(i)].slot;
  const int32_t s = insert_at(i, id, h, c);
  if (inserted) *inserted = s >= 0;
  return s;
}

void AccountIndex::lookup(const std::vector<std::string>& ids, const std::vector<uint64_t>& hashes,
                          bool insert, int32_t* slots, uint8_t* fresh) {
  std::vector<std::string_view> v(ids.begin(), ids.end());
  std::vector<uint32_t> c(ids.size());
  for (size_t k = 0; k < ids.size(); ++k) c[k] = id_check(ids[k]);
  lookup_views(v.data(), hashes.data(), c.data(), ids.size(), insert, slots, fresh);
}

void AccountIndex::lookup_views(const std::string_view* ids, const uint64_t* h, const uint32_t* check, size_t n,
                                bool insert, int32_t* slots, uint8_t* fresh, const uint8_t* sel) {
  constexpr size_t kAhead = 16;  // probe lines in flight
  std::vector<uint32_t> miss;
  {
    std::shared_lock<std::shared_mutex> lk(mu_);
    const Entry* t = tab_.data();
    for (size_t k = 0; k < std::min(n, kAhead); ++k) __builtin_prefetch(t + (h[k] & uint64_t(mask_)));
    for (size_t k = 0; k < n; ++k) {
      if (k + kAhead < n) __builtin_prefetch(t + (h[k + kAhead] & uint64_t(mask_)));
      if (fresh) fresh[k] = 0;
      if (h[k] == 0 || (sel && !sel[k])) { slots[k] = -1; continue; }
      bool found;
      const int64_t i = probe(h[k], check[k], found);
      if (found) {
        slots[k] = t[size_t(i)].slot;
      } else {
        slots[k] = -1;
        if (insert) miss.push_back(uint32_t(k));
      }
    }
  }
  if (miss.empty()) return;
  std::unique_lock<std::shared_mutex> lk(mu_);
  for (uint32_t k : miss) {  // in row order: a batch's new accounts get slots in arrival order
    bool found;
    const int64_t i = probe(h[k], check[k], found);
    if (found) {
      slots[k] = tab_[size_t(i)].slot;  // inserted earlier in this batch (or by another thread)
      continue;
    }
    slots[k] = insert_at(i, ids[k], h[k], check[k]);
    if (fresh) fresh[k] = slots[k] >= 0;
  }
}

std::string AccountIndex::id_of(int32_t slot) const {
  std::shared_lock<std::shared_mutex> lk(mu_);
  if (slot < 0 || slot >= n_) throw std::runtime_error("AccountIndex: bad slot");
  return ids_[size_t(slot)];
}

}  // namespace igp

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
  keys_.assign(size_t(t), 0);
  slot_.assign(size_t(t), -1);
  ids_.reserve(size_t(std::min<int64_t>(capacity, 1 << 20)));
}

int64_t AccountIndex::probe(std::string_view id, uint64_t h, bool& found) const {
  int64_t i = int64_t(h & uint64_t(mask_));
  for (;;) {
    uint64_t k = keys_[size_t(i)];
    if (k == 0) { found = false; return i; }
    if (k == h && ids_[size_t(slot_[size_t(i)])] == id) { found = true; return i; }
    i = (i + 1) & mask_;
  }
}

int32_t AccountIndex::find(std::string_view id, uint64_t h) const {
  if (h == 0) return -1;
  std::shared_lock<std::shared_mutex> lk(mu_);
  bool found;
  int64_t i = probe(id, h, found);
  return found ? slot_[size_t(i)] : -1;
}

int32_t AccountIndex::find_or_insert(std::string_view id, uint64_t h, bool* inserted) {
  if (inserted) *inserted = false;
  if (h == 0) return -1;
  {
    std::shared_lock<std::shared_mutex> lk(mu_);
    bool found;
    int64_t i = probe(id, h, found);
    if (found) return slot_[size_t(i)];
  }
  std::unique_lock<std::shared_mutex> lk(mu_);
  bool found;
  int64_t i = probe(id, h, found);
  if (found) return slot_[size_t(i)];
  if (n_ >= cap_) return -1;
  keys_[size_t(i)] = h;
  slot_[size_t(i)] = int32_t(n_);
  ids_.emplace_back(id);
  if (inserted) *inserted = true;
  return int32_t(n_++);
}

void AccountIndex::lookup(const std::vector<std::string>& ids, const std::vector<uint64_t>& hashes,
                          bool insert, int32_t* slots, uint8_t* fresh) {
  for (size_t k = 0; k < ids.size(); ++k) {
    bool ins = false;
    slots[k] = insert ? find_or_insert(ids[k], hashes[k], &ins) : find(ids[k], hashes[k]);
    if (fresh) fresh[k] = ins;
  }
}

std::string AccountIndex::id_of(int32_t slot) const {
  std::shared_lock<std::shared_mutex> lk(mu_);
  if (slot < 0 || slot >= n_) throw std::runtime_error("AccountIndex: bad slot");
  return ids_[size_t(slot)];
}

}  // namespace igp

#include "audit.h"

#include <dlfcn.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string_view>
#include <unordered_map>

#include "wire.h"
#include "xxh64.h"

namespace igp {

// ---------------------------------------------------------------------------- libsqlite3 (dlopen)
namespace {

struct Sqlite {
  int (*open_v2)(const char*, void**, int, const char*) = nullptr;
  int (*close)(void*) = nullptr;
  int (*exec)(void*, const char*, void*, void*, char**) = nullptr;
  int (*prepare_v2)(void*, const char*, int, void**, const char**) = nullptr;
  int (*bind_text)(void*, int, const char*, int, void (*)(void*)) = nullptr;
  int (*bind_int64)(void*, int, long long) = nullptr;
  int (*bind_double)(void*, int, double) = nullptr;
  int (*step)(void*) = nullptr;
  int (*reset)(void*) = nullptr;
  int (*finalize)(void*) = nullptr;
  const char* (*errmsg)(void*) = nullptr;
  void (*free_)(void*) = nullptr;
};
constexpr int kOpenRW = 0x2, kOpenCreate = 0x4, kRow = 100, kDone = 101, kOk = 0;

const Sqlite& sqlite() {
  static Sqlite s;
  static bool loaded = false;
  static std::mutex mu;
  std::lock_guard<std::mutex> g(mu);
  if (loaded) return s;
  void* h = dlopen("libsqlite3.so.0", RTLD_NOW | RTLD_LOCAL);
  if (!h) throw std::runtime_error(std::string("audit: cannot load libsqlite3: ") + dlerror());
  auto sym = [&](const char* n) {
    void* f = dlsym(h, n);
    if (!f) throw std::runtime_error(std::string("audit: libsqlite3 lacks ") + n);
    return f;
  };
  s.open_v2 = reinterpret_cast<decltype(s.open_v2)>(sym("sqlite3_open_v2"));
  s.close = reinterpret_cast<decltype(s.close)>(sym("sqlite3_close"));
  s.exec = reinterpret_cast<decltype(s.exec)>(sym("sqlite3_exec"));
  s.prepare_v2 = reinterpret_cast<decltype(s.prepare_v2)>(sym("sqlite3_prepare_v2"));
  s.bind_text = reinterpret_cast<decltype(s.bind_text)>(sym("sqlite3_bind_text"));
  s.bind_int64 = reinterpret_cast<decltype(s.bind_int64)>(sym("sqlite3_bind_int64"));
  s.bind_double = reinterpret_cast<decltype(s.bind_double)>(sym("sqlite3_bind_double"));
  s.step = reinterpret_cast<decltype(s.step)>(sym("sqlite3_step"));
  s.reset = reinterpret_cast<decltype(s.reset)>(sym("sqlite3_reset"));
  s.finalize = reinterpret_cast<decltype(s.finalize)>(sym("sqlite3_finalize"));
  s.errmsg = reinterpret_cast<decltype(s.errmsg)>(sym("sqlite3_errmsg"));
  s.free_ = reinterpret_cast<decltype(s.free_)>(sym("sqlite3_free"));
  loaded = true;
  return s;
}

const char* kActions[4] = {"unspecified", "approve", "review", "block"};

// '["HIGH_VELOCITY", "ML_HIGH_RISK"]' for a 12-bit reason mask (json.dumps of the names in
// rule order, as the Python audit path writes them); built once per mask
struct ReasonJson {
  std::vector<std::string> s;
  ReasonJson() : s(4096) {
    for (uint32_t mask = 0; mask < 4096; ++mask) {
      std::string j = "[";
      bool first = true;
      for (int b = 0; b < 12; ++b) {
        if (!(mask >> b & 1u)) continue;
        if (!first) j += ", ";
        j += '"';
        j += wire::kReasonCodes[b];
        j += '"';
        first = false;
      }
      s[mask] = j + "]";
    }
  }
};
const std::string& reasons_json(uint32_t mask) {
  static const ReasonJson table;
  return table.s[mask & 4095u];
}

// one risk_scores writer: open, schema, BEGIN, prepared INSERT per row, COMMIT; any failure
// throws, and the destructor rolls an open transaction back (the caller decides what happens
// to its rows)
class Db {
 public:
  Db(const std::string& path, const std::string& schema_sql) : q_(sqlite()) {
    if (q_.open_v2(path.c_str(), &db_, kOpenRW | kOpenCreate, nullptr) != kOk) fail("open");
    // a 256 MiB page cache keeps the account/time index resident during a bulk insert
    exec("PRAGMA busy_timeout=5000; PRAGMA journal_mode=WAL; PRAGMA synchronous=NORMAL; "
         "PRAGMA cache_size=-262144; PRAGMA temp_store=MEMORY;");
    if (!schema_sql.empty()) exec(schema_sql.c_str());
  }
  ~Db() {
    if (ins_) q_.finalize(ins_);
    if (open_tx_) {
      char* m = nullptr;
      q_.exec(db_, "ROLLBACK", nullptr, nullptr, &m);
      if (m) q_.free_(m);
    }
    if (db_) q_.close(db_);
  }
  Db(const Db&) = delete;
  Db& operator=(const Db&) = delete;

  void begin() {
    exec("BEGIN IMMEDIATE");
    open_tx_ = true;
    if (q_.prepare_v2(db_,
                      "INSERT INTO risk_scores(account_id, score, rule_score, ml_score, action, reason_codes, "
                      "model_version, created_at) VALUES (?,?,?,?,?,?,?,?)",
                      -1, &ins_, nullptr) != kOk)
      fail("prepare");
  }
  void row(std::string_view id, uint32_t p, float ml, uint16_t ver, int64_t t_ms) {
    char v[8];
    const int vn = std::snprintf(v, sizeof v, "%u", unsigned(ver));
    const std::string& rj = reasons_json(IGP_RES_REASONS(p));
    q_.bind_text(ins_, 1, id.data() ? id.data() : "", int(id.size()), nullptr);
    q_.bind_int64(ins_, 2, IGP_RES_SCORE(p));
    q_.bind_int64(ins_, 3, IGP_RES_RULE(p));
    q_.bind_double(ins_, 4, std::isnan(ml) ? 0.0 : double(ml));  // SQLite stores NaN as NULL
    q_.bind_text(ins_, 5, kActions[IGP_RES_ACTION(p)], -1, nullptr);
    q_.bind_text(ins_, 6, rj.data(), int(rj.size()), nullptr);
    q_.bind_text(ins_, 7, v, vn, nullptr);
    q_.bind_double(ins_, 8, double(t_ms) / 1000.0);
    if (q_.step(ins_) != kDone) fail("insert");
    q_.reset(ins_);
  }
  // true when `name` is already in audit_segments
  bool segment_loaded(const std::string& name) {
    void* st = nullptr;
    if (q_.prepare_v2(db_, "SELECT 1 FROM audit_segments WHERE name=?", -1, &st, nullptr) != kOk) fail("prepare");
    q_.bind_text(st, 1, name.data(), int(name.size()), nullptr);
    const int rc = q_.step(st);
    q_.finalize(st);
    if (rc != kRow && rc != kDone) fail("select");
    return rc == kRow;
  }
  void mark_segment(const std::string& name, int64_t rows) {
    void* st = nullptr;
    if (q_.prepare_v2(db_, "INSERT INTO audit_segments(name, rows, loaded_at) VALUES (?,?,strftime('%s','now'))",
                      -1, &st, nullptr) != kOk)
      fail("prepare");
    q_.bind_text(st, 1, name.data(), int(name.size()), nullptr);
    q_.bind_int64(st, 2, rows);
    const int rc = q_.step(st);
    q_.finalize(st);
    if (rc != kDone) fail("insert segment");
  }
  void commit() {
    if (ins_) {
      q_.finalize(ins_);
      ins_ = nullptr;
    }
    exec("COMMIT");
    open_tx_ = false;
  }
  void exec(const char* sql) {
    char* msg = nullptr;
    if (q_.exec(db_, sql, nullptr, nullptr, &msg) != kOk) {
      std::string e = std::string("audit: ") + (msg ? msg : "exec failed");
      if (msg) q_.free_(msg);
      throw std::runtime_error(e);
    }
  }

 private:
  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("audit: ") + what + ": " + (db_ ? q_.errmsg(db_) : "open failed"));
  }
  const Sqlite& q_;
  void* db_ = nullptr;
  void* ins_ = nullptr;
  bool open_tx_ = false;
};

std::string_view id_for(const AuditRec& r, const std::vector<std::shared_ptr<AccountIndex>>& indexes) {
  if (r.slot < 0 || r.owner < 0 || size_t(r.owner) >= indexes.size() || !indexes[size_t(r.owner)]) return {};
  return indexes[size_t(r.owner)]->id_view(r.slot);
}

void write_all(int fd, const void* p, size_t n, const std::string& path) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    const ssize_t w = ::write(fd, c, n);
    if (w < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error("audit: write " + path + ": " + std::strerror(errno));
    }
    c += w;
    n -= size_t(w);
  }
}

}  // namespace

// ---------------------------------------------------------------------------- ring
AuditRing::AuditRing(int64_t capacity) {
  if (capacity < 1) throw std::runtime_error("AuditRing: capacity");
  buf_.resize(size_t(capacity));
}

void AuditRing::append(const ResultRec* res, const int32_t* slots, size_t stride_slots, int owner, size_t n,
                       int64_t t_ms, uint16_t model_version) {
  if (n == 0) return;
  std::lock_guard<std::mutex> g(mu_);
  const int64_t cap = int64_t(buf_.size());
  for (size_t i = 0; i < n; ++i) {
    AuditRec& r = buf_[size_t(head_ % cap)];
    r.t_ms = t_ms;
    r.slot = slots[i * stride_slots];
    r.owner = int16_t(owner);
    r.model_version = model_version;
    r.packed = res[i].packed;
    r.ml = res[i].ml;
    ++head_;
  }
  appended_ += int64_t(n);
  if (head_ - tail_ > cap) {  // overwrote the oldest rows before a flush drained them
    evicted_ += head_ - tail_ - cap;
    tail_ = head_ - cap;
  }
}

int64_t AuditRing::pending() const {
  std::lock_guard<std::mutex> g(mu_);
  return head_ - tail_;
}
int64_t AuditRing::evicted() const {
  std::lock_guard<std::mutex> g(mu_);
  return evicted_;
}
int64_t AuditRing::appended() const {
  std::lock_guard<std::mutex> g(mu_);
  return appended_;
}

std::vector<AuditRec> AuditRing::peek(int64_t max) const {
  std::lock_guard<std::mutex> g(mu_);
  const int64_t cap = int64_t(buf_.size()), n = std::min(max, head_ - tail_);
  std::vector<AuditRec> out(size_t(std::max<int64_t>(n, 0)));
  for (int64_t i = 0; i < n; ++i) out[size_t(i)] = buf_[size_t((tail_ + i) % cap)];
  return out;
}

// the live rows out of the ring (appends continue into it meanwhile)
std::vector<AuditRec> AuditRing::take(int64_t* t0) {
  std::lock_guard<std::mutex> g(mu_);
  const int64_t cap = int64_t(buf_.size());
  *t0 = tail_;
  std::vector<AuditRec> rows(size_t(head_ - tail_));
  const int64_t a = tail_ % cap, n = head_ - tail_, first = std::min(n, cap - a);
  if (n) {
    std::memcpy(rows.data(), buf_.data() + a, size_t(first) * sizeof(AuditRec));
    if (first < n) std::memcpy(rows.data() + first, buf_.data(), size_t(n - first) * sizeof(AuditRec));
  }
  tail_ = head_;
  return rows;
}

// a failed drain: the rows go back in front of the ring unless newer rows already overwrote
// their places (then they count as evicted)
void AuditRing::put_back(int64_t t0, size_t n) {
  std::lock_guard<std::mutex> g(mu_);
  if (head_ - t0 <= int64_t(buf_.size())) {
    tail_ = t0;
  } else {
    evicted_ += int64_t(n);
  }
}

int64_t AuditRing::flush_sqlite(const std::string& path, const std::string& schema_sql,
                                const std::vector<std::shared_ptr<AccountIndex>>& indexes) {
  int64_t t0;
  std::vector<AuditRec> rows = take(&t0);
  if (rows.empty()) return 0;
  try {
    Db db(path, schema_sql);
    db.begin();
    for (const AuditRec& r : rows) db.row(id_for(r, indexes), r.packed, r.ml, r.model_version, r.t_ms);
    db.commit();
  } catch (...) {
    put_back(t0, rows.size());
    throw;
  }
  return int64_t(rows.size());
}

std::pair<std::string, int64_t> AuditRing::flush_segment(const std::string& dir, const std::string& tag,
                                                         const std::vector<std::shared_ptr<AccountIndex>>& indexes) {
  int64_t t0;
  std::vector<AuditRec> rows = take(&t0);
  if (rows.empty()) return {"", 0};
  const size_t n = rows.size();
  std::string path;
  try {
    // dictionary-encode the account ids: (owner, slot) -> position in the segment's id table
    std::vector<uint32_t> ref(n);
    std::vector<uint32_t> off{0};
    std::string chars;
    std::unordered_map<uint64_t, uint32_t> dict;
    dict.reserve(std::min<size_t>(n, size_t(1) << 22));
    int64_t tmin = rows[0].t_ms, tmax = rows[0].t_ms;
    for (size_t i = 0; i < n; ++i) {
      const AuditRec& r = rows[i];
      tmin = std::min(tmin, r.t_ms);
      tmax = std::max(tmax, r.t_ms);
      const uint64_t key = r.slot < 0 ? ~uint64_t(0) : (uint64_t(uint16_t(r.owner)) << 32) | uint32_t(r.slot);
      auto it = dict.find(key);
      if (it == dict.end()) {
        const std::string_view id = r.slot < 0 ? std::string_view() : id_for(r, indexes);
        chars.append(id.data() ? id.data() : "", id.size());
        it = dict.emplace(key, uint32_t(off.size() - 1)).first;
        off.push_back(uint32_t(chars.size()));
      }
      ref[i] = it->second;
    }
    // body in one buffer (hashed), the header in front of it
    const size_t ids_bytes = off.size() * 4 + chars.size(), pad = (8 - ids_bytes % 8) % 8;
    std::string body(ids_bytes + pad + n * 22, '\0');
    char* b = body.data();
    std::memcpy(b, off.data(), off.size() * 4);
    std::memcpy(b + off.size() * 4, chars.data(), chars.size());
    char* col = b + ids_bytes + pad;
    int64_t* t = reinterpret_cast<int64_t*>(col);
    std::memcpy(col + n * 8, ref.data(), n * 4);
    uint32_t* packed = reinterpret_cast<uint32_t*>(col + n * 12);
    float* ml = reinterpret_cast<float*>(col + n * 16);
    uint16_t* ver = reinterpret_cast<uint16_t*>(col + n * 20);
    for (size_t i = 0; i < n; ++i) {
      t[i] = rows[i].t_ms;
      packed[i] = rows[i].packed;
      ml[i] = rows[i].ml;
      ver[i] = rows[i].model_version;
    }
    AuditSegHdr h{};
    std::memcpy(h.magic, "IGPAUDS1", 8);
    h.format = 1;
    h.rows = int64_t(n);
    h.n_ids = int64_t(off.size() - 1);
    h.id_bytes = int64_t(chars.size());
    h.t_min = tmin;
    h.t_max = tmax;
    h.body_hash = xxh64(body.data(), body.size(), 0);
    uint64_t seq;
    {
      std::lock_guard<std::mutex> g(mu_);
      seq = uint64_t(seg_seq_++);
    }
    char name[192];
    std::snprintf(name, sizeof name, "audit-%013lld-%s-%06llu.seg", static_cast<long long>(tmin), tag.c_str(),
                  static_cast<unsigned long long>(seq));
    path = dir + "/" + name;
    const std::string tmp = dir + "/.tmp-" + name;
    ::mkdir(dir.c_str(), 0755);
    const int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0) throw std::runtime_error("audit: create " + tmp + ": " + std::strerror(errno));
    try {
      write_all(fd, &h, sizeof h, tmp);
      write_all(fd, body.data(), body.size(), tmp);
      if (::fdatasync(fd) != 0) throw std::runtime_error("audit: fdatasync " + tmp + ": " + std::strerror(errno));
    } catch (...) {
      ::close(fd);
      ::unlink(tmp.c_str());
      throw;
    }
    ::close(fd);
    if (::rename(tmp.c_str(), path.c_str()) != 0) {
      const std::string e = std::strerror(errno);
      ::unlink(tmp.c_str());
      throw std::runtime_error("audit: rename " + path + ": " + e);
    }
    const int dfd = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
    if (dfd >= 0) {
      ::fsync(dfd);
      ::close(dfd);
    }
  } catch (...) {
    put_back(t0, n);
    throw;
  }
  return {path, int64_t(n)};
}

// ---------------------------------------------------------------------------- segment loader
int64_t audit_load_segment(const std::string& seg_path, const std::string& db_path, const std::string& schema_sql) {
  const int fd = ::open(seg_path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) throw std::runtime_error("audit: open " + seg_path + ": " + std::strerror(errno));
  struct stat sb {};
  ::fstat(fd, &sb);
  std::string buf(size_t(sb.st_size), '\0');
  size_t got = 0;
  while (got < buf.size()) {
    const ssize_t r = ::read(fd, buf.data() + got, buf.size() - got);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) break;
    got += size_t(r);
  }
  ::close(fd);
  AuditSegHdr h{};
  if (got != buf.size() || buf.size() < sizeof h) throw std::runtime_error("audit: short segment " + seg_path);
  std::memcpy(&h, buf.data(), sizeof h);
  if (std::memcmp(h.magic, "IGPAUDS1", 8) != 0 || h.format != 1 || h.rows < 0 || h.n_ids < 0 || h.id_bytes < 0)
    throw std::runtime_error("audit: not an audit segment: " + seg_path);
  const size_t n = size_t(h.rows), ids_bytes = size_t(h.n_ids + 1) * 4 + size_t(h.id_bytes);
  const size_t pad = (8 - ids_bytes % 8) % 8, body = ids_bytes + pad + n * 22;
  if (buf.size() != sizeof h + body) throw std::runtime_error("audit: segment size mismatch: " + seg_path);
  const char* b = buf.data() + sizeof h;
  if (xxh64(b, body, 0) != h.body_hash) throw std::runtime_error("audit: segment checksum mismatch: " + seg_path);
  std::vector<uint32_t> off(size_t(h.n_ids + 1));
  std::memcpy(off.data(), b, off.size() * 4);
  const char* chars = b + off.size() * 4;
  for (int64_t k = 0; k < h.n_ids; ++k)
    if (off[size_t(k)] > off[size_t(k) + 1] || off[size_t(k) + 1] > uint64_t(h.id_bytes))
      throw std::runtime_error("audit: corrupt id table: " + seg_path);
  const char* col = b + ids_bytes + pad;
  auto at = [&](size_t byte_off, size_t i, auto* out) { std::memcpy(out, col + byte_off + i * sizeof(*out), sizeof(*out)); };
  const std::string name = seg_path.substr(seg_path.find_last_of('/') + 1);
  Db db(db_path, schema_sql);
  db.exec("CREATE TABLE IF NOT EXISTS audit_segments (name TEXT PRIMARY KEY, rows INTEGER NOT NULL, "
          "loaded_at REAL NOT NULL)");
  db.begin();
  int64_t inserted = 0;
  if (!db.segment_loaded(name)) {
    for (size_t i = 0; i < n; ++i) {
      int64_t t;
      uint32_t k, p;
      float ml;
      uint16_t ver;
      at(0, i, &t);
      at(n * 8, i, &k);
      at(n * 12, i, &p);
      at(n * 16, i, &ml);
      at(n * 20, i, &ver);
      if (int64_t(k) >= h.n_ids) throw std::runtime_error("audit: corrupt id reference: " + seg_path);
      db.row(std::string_view(chars + off[k], off[k + 1] - off[k]), p, ml, ver, t);
    }
    db.mark_segment(name, int64_t(n));
    inserted = int64_t(n);
  }
  db.commit();
  ::unlink(seg_path.c_str());
  return inserted;
}

}  // namespace igp

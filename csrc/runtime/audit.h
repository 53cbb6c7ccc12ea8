// risk_scores audit at serving rate (VERDICT r2 "audit of every score"): a columnar ring of
// 24-byte records written by the serving core as it hands results back, drained two ways:
//
//  * flush_sqlite: straight into risk_scores of a SQLite file (libsqlite3 through dlopen: the
//    image has the library, not its headers), one prepared INSERT inside one transaction;
//  * flush_segment: a durable columnar segment file (dictionary-encoded account ids, one write
//    per column, fsync + atomic rename) at GB/s, which load_segment later ingests into SQLite
//    exactly once (the segment name is committed in audit_segments in the same transaction).
//
// SQLite ingests a few hundred thousand rows per second per file (one B-tree insert per row
// plus the account index), far below an 8 M scores/s serving rate; the segment tier is what
// keeps the ring from evicting under load, the loader catches SQLite up behind it.
// Account ids are resolved at flush time from the (node-shared) account index; reason-code
// JSON strings are built once per distinct reason mask. Reference: deploy/init-db.sql:122-138
// declares the table, nothing writes it.
#pragma once
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../include/records.h"
#include "account_index.h"

namespace igp {

struct AuditRec {
  int64_t t_ms;       // wall clock when the result was handed back (unix ms)
  int32_t slot;       // feature-store slot on its owner (-1: unknown account)
  int16_t owner;
  uint16_t model_version;
  uint32_t packed;    // ResultRec word 0 (score, rule score, action, reasons)
  float ml;
};
static_assert(sizeof(AuditRec) == 24, "AuditRec must be 24 bytes");

// header of a segment file; the body follows it:
//   uint32 id_off[n_ids + 1]; char ids[id_bytes]; (pad to 8)
//   int64 t_ms[rows]; uint32 id_ref[rows]; uint32 packed[rows]; float ml[rows]; uint16 version[rows]
struct AuditSegHdr {
  char magic[8];      // "IGPAUDS1"
  uint32_t format;    // 1
  uint32_t flags;
  int64_t rows, n_ids, id_bytes, t_min, t_max;
  uint64_t body_hash; // xxh64 of the body
};

class AuditRing {
 public:
  explicit AuditRing(int64_t capacity);
  // one segment of results (rows of one owner); thread-safe
  void append(const ResultRec* res, const int32_t* slots, size_t stride_slots, int owner, size_t n, int64_t t_ms,
              uint16_t model_version);
  int64_t pending() const;
  int64_t capacity() const { return int64_t(buf_.size()); }
  int64_t evicted() const;
  int64_t appended() const;
  // drain into risk_scores of the SQLite file at `path` (schema_sql runs first); rows of a
  // failed write go back into the ring. Returns the rows written.
  int64_t flush_sqlite(const std::string& path, const std::string& schema_sql,
                       const std::vector<std::shared_ptr<AccountIndex>>& indexes);
  // drain into a new segment file under `dir` (named so that lexical order = flush order;
  // `tag` tells writers sharing the directory apart). Returns (path, rows); ("", 0) when empty.
  std::pair<std::string, int64_t> flush_segment(const std::string& dir, const std::string& tag,
                                                const std::vector<std::shared_ptr<AccountIndex>>& indexes);
  // the next `max` rows (tests / exporters); does not consume
  std::vector<AuditRec> peek(int64_t max) const;

 private:
  std::vector<AuditRec> take(int64_t* t0);
  void put_back(int64_t t0, size_t n);

  mutable std::mutex mu_;
  std::vector<AuditRec> buf_;
  int64_t head_ = 0, tail_ = 0;  // monotonic; live rows [tail_, head_)
  int64_t evicted_ = 0, appended_ = 0;
  int64_t seg_seq_ = 0;
};

// ingest one segment file into risk_scores of `db_path` exactly once (its name goes into
// audit_segments in the same transaction; an already-loaded segment is skipped), then delete
// the file. Returns the rows inserted (0 for a skipped segment).
int64_t audit_load_segment(const std::string& seg_path, const std::string& db_path, const std::string& schema_sql);

}  // namespace igp

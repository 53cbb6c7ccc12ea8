"""Score / LTV audit log: the ``risk_scores`` and ``ltv_predictions`` tables of
deploy/schema.sql (reference: deploy/init-db.sql:122-155, declared and never written).

Rows are buffered per scored batch (one ring entry per batch, not per request: the hot path
pays one deque append) and drained into SQLite by :meth:`AuditLog.flush`. Each entry carries
the model version that produced it, captured when the batch was scored, so a model reload
between scoring and flushing cannot re-label old decisions.

Durability rules:
* appenders and the flusher share one lock; a flush swaps the rings out under it, so rows
  appended while the SQLite write runs land in the fresh rings and are never lost;
* a failed write (locked DB, full disk, missing table) puts the drained entries back in
  front of the rings and re-raises;
* the schema script (all ``CREATE ... IF NOT EXISTS``) runs on every flush;
* the rings are bounded by row count; entries evicted before a flush are counted
  (``evicted_rows``, exported as a Prometheus counter by the engine).

Rows the native serving core hands back are not recorded here but in its own columnar ring
(csrc/runtime/audit.cpp: 24 bytes per row appended by the core's completion thread);
:meth:`attach_native` joins that ring to this log, so ``pending`` / ``flush`` /
``evicted_rows`` cover both. The Python rings keep the rows of the paths the core does not
serve (the degraded-shard fallback, golden shards) and the LTV answers.

The native ring drains one of two ways (``server.audit_mode``):

* ``sqlite``: straight into risk_scores, one prepared INSERT per row in one transaction
  (account ids resolved from the account index at flush time);
* ``segments``: into a durable columnar segment file under ``<audit_db>.segments/``
  (dictionary-encoded ids, fsync + atomic rename: ~5 M rows/s), which a background loader
  thread ingests into risk_scores exactly once (segment names are committed in
  ``audit_segments`` with the rows). SQLite takes ~0.15-0.4 M rows/s per file with the account
  index, so at serving rate (millions of scores/s) this is the mode that keeps the ring from
  evicting; the table catches up behind the segments;
* ``auto`` (default): ``sqlite`` for a small backlog, ``segments`` once the ring holds more than
  ``audit_direct_max`` rows or segments are still waiting (rows reach the table in order).
"""
from __future__ import annotations

import collections
import json
import os
import sqlite3
import threading
import time
from typing import Optional

import numpy as np

from ..config import ACTION_NAMES, REASON_CODES

SCHEMA = os.path.join(os.path.dirname(__file__), "..", "..", "deploy", "schema.sql")


class AuditLog:
    def __init__(self, enabled: bool, max_rows: int = 1_000_000, mode: str = "auto", direct_max: int = 262144,
                 tag: str = ""):
        if mode not in ("auto", "sqlite", "segments"):
            raise ValueError(f"audit mode must be auto|sqlite|segments, got {mode!r}")
        self.enabled = bool(enabled)
        self.max_rows = int(max_rows)
        self.mode = mode
        self.direct_max = int(direct_max)
        self.tag = tag or f"p{os.getpid()}"
        self._loader: Optional[threading.Thread] = None
        self._loader_wake = threading.Event()
        self._loader_stop = False
        self.loader_paused = False   # tests / maintenance: segments accumulate, nothing is loaded
        self._loader_db: Optional[str] = None
        self.segments_loaded = 0     # rows the background loader put into risk_scores
        self.loader_error: Optional[str] = None
        self._lock = threading.Lock()
        self._scores: collections.deque = collections.deque()   # (ts, ids, res[n,2] u32, model_version)
        self._ltv: collections.deque = collections.deque()      # (ts, LtvResult, model_version)
        self._n_scores = 0
        self._evicted = 0
        self._native = None         # csrc AuditRing of the serving core
        self._native_indexes = []   # AccountIndex per owner (slot -> account id at flush)

    def attach_native(self, ring, indexes) -> None:
        self._native = ring
        self._native_indexes = list(indexes)

    @property
    def native(self):
        return self._native

    @property
    def evicted_rows(self) -> int:
        return self._evicted + (int(self._native.evicted) if self._native is not None else 0)

    # ------------------------------------------------------------------ appenders
    def record_scores(self, ids, res: np.ndarray, model_version) -> None:
        if not self.enabled or len(res) == 0:
            return
        entry = (time.time(), list(ids), np.array(res, np.uint32, copy=True), str(model_version))
        with self._lock:
            self._scores.append(entry)
            self._n_scores += len(entry[1])
            while self._n_scores > self.max_rows and len(self._scores) > 1:
                old = self._scores.popleft()
                self._n_scores -= len(old[1])
                self._evicted += len(old[1])

    def record_ltv(self, results, model_version) -> None:
        if not self.enabled:
            return
        ts = time.time()
        with self._lock:
            for r in results:
                if r.found:
                    self._ltv.append((ts, r, None if model_version is None else str(model_version)))
            while len(self._ltv) > self.max_rows:
                self._ltv.popleft()
                self._evicted += 1

    def pending(self) -> int:
        with self._lock:
            n = self._n_scores + len(self._ltv)
        return n + (int(self._native.pending()) if self._native is not None else 0)

    # ------------------------------------------------------------------ drain
    def flush(self, path: str) -> int:
        """Write every buffered row to the SQLite database at ``path``; returns the row count."""
        n_native = 0
        ring = self._native
        if ring is not None and ring.pending():
            seg_dir = self.segment_dir(path)
            segs = self.mode == "segments" or (self.mode == "auto" and (
                ring.pending() > self.direct_max or bool(_segments(seg_dir))))
            try:  # GIL released; rows of a failed write go back into the native ring
                if segs:
                    _, n_native = ring.flush_segment(seg_dir, self.tag, self._native_indexes)
                    self._kick_loader(path)
                else:
                    n_native = int(ring.flush_sqlite(path, _schema(), self._native_indexes))
            except RuntimeError as e:
                raise sqlite3.OperationalError(str(e)) from e
        with self._lock:
            scores, self._scores = self._scores, collections.deque()
            ltv, self._ltv = self._ltv, collections.deque()
            n_scores, self._n_scores = self._n_scores, 0
        try:
            n = self._write(path, scores, ltv)
        except BaseException:
            with self._lock:  # put the rows back in front (oldest first), then re-raise
                self._scores.extendleft(reversed(scores))
                self._ltv.extendleft(reversed(ltv))
                self._n_scores += n_scores
            raise
        return n + n_native

    # ------------------------------------------------------------------ segment loader
    @staticmethod
    def segment_dir(path: str) -> str:
        return path + ".segments"

    def _kick_loader(self, path: str) -> None:
        with self._lock:
            self._loader_db = path
            if self._loader is None or not self._loader.is_alive():
                self._loader_stop = False
                self._loader = threading.Thread(target=self._load_loop, name="audit-loader", daemon=True)
                self._loader.start()
        self._loader_wake.set()

    def resume_loading(self, path: str) -> None:
        """Start loading segments an earlier process left under ``path``'s segment directory."""
        if _segments(self.segment_dir(path)):
            self._kick_loader(path)

    def _load_loop(self) -> None:
        from ..native import native
        N = native()
        while not self._loader_stop:
            self._loader_wake.wait(1.0)
            self._loader_wake.clear()
            path = self._loader_db
            if self.loader_paused:
                continue
            for seg in _segments(self.segment_dir(path)):
                if self._loader_stop or self.loader_paused:
                    break
                try:
                    n = int(N.audit_load_segment(seg, path, _schema()))
                    with self._lock:
                        self.segments_loaded += n
                    self.loader_error = None
                except RuntimeError as e:
                    if not os.path.exists(seg):  # another process's loader took it
                        continue
                    self.loader_error = str(e)   # locked / full disk: retried on the next pass
                    time.sleep(0.5)
                    break

    def wait_loaded(self, path: str, timeout_s: float = 60.0) -> bool:
        """Block until no segment of ``path`` waits for the loader (tests / shutdown)."""
        t_end = time.time() + timeout_s
        self._kick_loader(path)
        while _segments(self.segment_dir(path)):
            if time.time() > t_end:
                return False
            self._loader_wake.set()
            time.sleep(0.02)
        return True

    def segments_waiting(self, path: str) -> int:
        return len(_segments(self.segment_dir(path)))

    def close(self) -> None:
        self._loader_stop = True
        self._loader_wake.set()
        if self._loader is not None:
            self._loader.join(30)

    @staticmethod
    def _write(path: str, scores, ltv) -> int:
        from ..golden.ltv import SEGMENTS
        out = []
        for ts, ids, res, ver in scores:
            p = res[:, 0]
            ml = res[:, 1].view(np.float32)
            for aid, pw, m in zip(ids, p.tolist(), ml.tolist()):
                reasons = [REASON_CODES[b] for b in range(len(REASON_CODES)) if (pw >> 20) >> b & 1]
                out.append((aid, pw & 0xFF, (pw >> 8) & 0xFF, m, ACTION_NAMES.get((pw >> 16) & 3, "unspecified"),
                            json.dumps(reasons), ver, ts))
        lrows = [(r.account_id, float(r.predicted_ltv), SEGMENTS[int(r.segment)], float(r.churn_risk),
                  int(r.survival_days), float(r.confidence), r.next_best_action, ver, ts) for ts, r, ver in ltv]
        db = sqlite3.connect(path, timeout=5.0)
        try:
            db.executescript(_schema())
            db.executemany("INSERT INTO risk_scores(account_id, score, rule_score, ml_score, action, reason_codes,"
                           " model_version, created_at) VALUES (?,?,?,?,?,?,?,?)", out)
            db.executemany("INSERT INTO ltv_predictions(account_id, predicted_ltv, segment, churn_risk, survival_days,"
                           " confidence, next_best_action, model_version, created_at) VALUES (?,?,?,?,?,?,?,?,?)",
                           lrows)
            db.commit()
        finally:
            db.close()
        return len(out) + len(lrows)


def _segments(seg_dir: str):
    """Finished segment files of a directory, oldest first (names sort by first row time)."""
    try:
        names = os.listdir(seg_dir)
    except OSError:
        return []
    return [os.path.join(seg_dir, n) for n in sorted(names) if n.startswith("audit-") and n.endswith(".seg")]


_SCHEMA_TEXT: Optional[str] = None


def _schema() -> str:
    global _SCHEMA_TEXT
    if _SCHEMA_TEXT is None:
        with open(SCHEMA) as f:
            _SCHEMA_TEXT = f.read()
    return _SCHEMA_TEXT


def flush_if_configured(engine, log=None) -> Optional[int]:
    """Serve-loop helper: drain the engine's audit rings when ``server.audit_db`` is set."""
    path = engine.cfg.server.audit_db
    if not path:
        return None
    try:
        return engine.flush_audit(path)
    except Exception as e:  # rows stay buffered; next tick retries
        if log is not None:
            log.error("audit flush failed", extra={"fields": dict(error=str(e), db=path)})
        return None

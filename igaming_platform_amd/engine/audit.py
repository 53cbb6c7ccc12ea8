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
    def __init__(self, enabled: bool, max_rows: int = 1_000_000):
        self.enabled = bool(enabled)
        self.max_rows = int(max_rows)
        self._lock = threading.Lock()
        self._scores: collections.deque = collections.deque()   # (ts, ids, res[n,2] u32, model_version)
        self._ltv: collections.deque = collections.deque()      # (ts, LtvResult, model_version)
        self._n_scores = 0
        self.evicted_rows = 0

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
                self.evicted_rows += len(old[1])

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
                self.evicted_rows += 1

    def pending(self) -> int:
        with self._lock:
            return self._n_scores + len(self._ltv)

    # ------------------------------------------------------------------ drain
    def flush(self, path: str) -> int:
        """Write every buffered row to the SQLite database at ``path``; returns the row count."""
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
        return n

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
            with open(SCHEMA) as f:
                db.executescript(f.read())
            db.executemany("INSERT INTO risk_scores(account_id, score, rule_score, ml_score, action, reason_codes,"
                           " model_version, created_at) VALUES (?,?,?,?,?,?,?,?)", out)
            db.executemany("INSERT INTO ltv_predictions(account_id, predicted_ltv, segment, churn_risk, survival_days,"
                           " confidence, next_best_action, model_version, created_at) VALUES (?,?,?,?,?,?,?,?,?)",
                           lrows)
            db.commit()
        finally:
            db.close()
        return len(out) + len(lrows)


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

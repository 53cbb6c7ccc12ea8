"""risk_scores audit at serving rate: the serving core's native columnar
ring (csrc/runtime/audit.cpp), its direct SQLite writer, the durable segment tier and the
exactly-once segment loader. Reference: deploy/init-db.sql:122-138 declares risk_scores,
nothing in the reference writes it."""
import os
import shutil
import sqlite3
import threading
import time

import numpy as np
import pytest

from igaming_platform_amd.config import Config
from igaming_platform_amd.engine.audit import SCHEMA
from igaming_platform_amd.engine.risk_engine import RiskEngine
from igaming_platform_amd.native import native


def _txs(n, rng):
    return [dict(account_id=f"acct-{int(rng.integers(0, 40))}", transaction_type=["deposit", "withdraw", "bet", "win"][i % 4],
                 amount=int(rng.integers(100, 500000)), ip_address=f"10.0.{i % 7}.{i % 13}", device_id=f"dev-{i % 11}")
            for i in range(n)]


def _index(n):
    N = native()
    idx = N.AccountIndex(1 << 20)
    slots, _ = idx.lookup([f"acct-{i:07d}" for i in range(n)], True)
    return idx, np.asarray(slots, np.int32)


def _res(rng, b):
    res = rng.integers(0, 1 << 31, (b, 2)).astype(np.uint32)
    res[:, 1] = rng.random(b, dtype=np.float32).view(np.uint32)
    return res


def test_core_rows_go_to_the_native_ring(tmp_path):
    """The single-shard engine's serving core appends every row it hands back to its native
    ring (no Python record), stamped with the model version in force."""
    cfg = Config()
    cfg.server.audit_db = str(tmp_path / "a.db")
    eng = RiskEngine(cfg, backend="cpu", capacity=64)
    try:
        ring = eng.auditlog.native
        assert ring is not None
        eng.score(_txs(5, np.random.default_rng(0)))
        out = eng.score_batch_bytes(_batch_bytes(eng, 12))
        assert out and ring.appended == 17 and ring.pending() == 17 and eng.auditlog.pending() == 17
        cols = ring.peek(100)
        assert set(cols["model_version"].tolist()) == {1} and (cols["slot"] >= 0).all()
        assert eng.flush_audit(cfg.server.audit_db) == 17 and eng.auditlog.pending() == 0
    finally:
        eng.close()


def _batch_bytes(eng, n):
    from igaming_platform_amd.proto import risk_v1 as P
    txs = [P.ScoreTransactionRequest.FromString(eng._tx_bytes(t)) for t in _txs(n, np.random.default_rng(4))]
    return P.ScoreBatchRequest(transactions=txs).SerializeToString()


def test_segment_mode_lands_every_row_once(tmp_path):
    """segments mode: flush writes a durable segment, the background loader ingests it into
    risk_scores; the rows equal the responses, and a segment seen again (a crash between the
    commit and the unlink) is skipped."""
    from igaming_platform_amd.proto import risk_v1 as P
    cfg = Config()
    db = str(tmp_path / "s.db")
    cfg.server.audit_db = db
    cfg.server.audit_mode = "segments"
    eng = RiskEngine(cfg, backend="cpu", capacity=64)
    try:
        txs = _txs(40, np.random.default_rng(9))
        out = eng.score_tx_many_bytes([eng._tx_bytes(t) for t in txs], [0.0] * len(txs))
        resp = [P.ScoreTransactionResponse.FromString(b) for b in out]
        seg_dir = eng.auditlog.segment_dir(db)
        eng.auditlog.loader_paused = True  # keep a copy of the segment first
        assert eng.flush_audit(db) == 40
        segs = sorted(os.listdir(seg_dir))
        assert len(segs) == 1 and segs[0].startswith("audit-") and segs[0].endswith(".seg")
        keep = str(tmp_path / "copy.seg")
        shutil.copy(os.path.join(seg_dir, segs[0]), keep)
        eng.auditlog.loader_paused = False
        assert eng.auditlog.wait_loaded(db, 30)
        con = sqlite3.connect(db)
        rows = con.execute("SELECT account_id, score, rule_score, model_version FROM risk_scores ORDER BY id").fetchall()
        assert [(r[0], r[1], r[2]) for r in rows] == [(t["account_id"], x.score, x.rule_score) for t, x in zip(txs, resp)]
        assert {r[3] for r in rows} == {"1"}
        assert con.execute("SELECT rows FROM audit_segments").fetchall() == [(40,)]
        # the same segment again: exactly once
        shutil.copy(keep, os.path.join(seg_dir, segs[0]))
        assert native().audit_load_segment(os.path.join(seg_dir, segs[0]), db, open(SCHEMA).read()) == 0
        assert con.execute("SELECT COUNT(*) FROM risk_scores").fetchone()[0] == 40
        assert not os.path.exists(os.path.join(seg_dir, segs[0]))
    finally:
        eng.close()


def test_auto_mode_switches_to_segments_for_a_backlog(tmp_path):
    cfg = Config()
    db = str(tmp_path / "auto.db")
    cfg.server.audit_db = db
    cfg.server.audit_direct_max = 8
    eng = RiskEngine(cfg, backend="cpu", capacity=64)
    try:
        eng.score(_txs(5, np.random.default_rng(1)))
        assert eng.flush_audit(db) == 5 and eng.auditlog.segments_waiting(db) == 0  # direct
        eng.score(_txs(20, np.random.default_rng(2)))
        eng.auditlog.loader_paused = True
        assert eng.flush_audit(db) == 20 and eng.auditlog.segments_waiting(db) == 1  # backlog -> segment
        eng.score(_txs(3, np.random.default_rng(3)))
        assert eng.flush_audit(db) == 3 and eng.auditlog.segments_waiting(db) == 2  # keeps order
        eng.auditlog.loader_paused = False
        assert eng.auditlog.wait_loaded(db, 30)
        assert sqlite3.connect(db).execute("SELECT COUNT(*) FROM risk_scores").fetchone()[0] == 28
    finally:
        eng.close()


def test_corrupt_segment_is_refused(tmp_path):
    N = native()
    idx, slots = _index(100)
    ring = N.AuditRing(1024)
    rng = np.random.default_rng(0)
    ring.append(_res(rng, 50), slots[:50], 0, int(time.time() * 1000), 3)
    path, n = ring.flush_segment(str(tmp_path / "segs"), "t", [idx])
    assert n == 50
    raw = bytearray(open(path, "rb").read())
    raw[-7] ^= 0x40
    open(path, "wb").write(bytes(raw))
    with pytest.raises(RuntimeError, match="checksum"):
        N.audit_load_segment(path, str(tmp_path / "c.db"), open(SCHEMA).read())
    assert os.path.exists(path)  # left for inspection, not half-loaded


def test_failed_direct_flush_puts_rows_back(tmp_path):
    N = native()
    idx, slots = _index(64)
    ring = N.AuditRing(4096)
    ring.append(_res(np.random.default_rng(1), 64), slots, 0, int(time.time() * 1000), 1)
    with pytest.raises(RuntimeError):
        ring.flush_sqlite(str(tmp_path / "missing" / "x.db"), open(SCHEMA).read(), [idx])
    assert ring.pending() == 64
    assert ring.flush_sqlite(str(tmp_path / "ok.db"), open(SCHEMA).read(), [idx]) == 64
    got = sqlite3.connect(str(tmp_path / "ok.db")).execute("SELECT account_id FROM risk_scores ORDER BY id").fetchall()
    assert [g[0] for g in got] == [f"acct-{i:07d}" for i in range(64)]


def test_ring_keeps_up_at_8m_scores_per_s_and_flushes_10m_rows_under_5s(tmp_path):
    """VERDICT r2 item 7 'done when': 8 M scores/s sustained for 2 s with a flusher running
    evicts nothing, and a 10 M-row backlog drains (segment tier) in under 5 s."""
    N = native()
    idx, slots = _index(1 << 20)
    rng = np.random.default_rng(7)
    B = 4096
    res = _res(rng, B)
    picks = [np.ascontiguousarray(slots[rng.integers(0, len(slots), B)]) for _ in range(64)]
    ring = N.AuditRing(1 << 24)
    seg_dir = str(tmp_path / "segs")
    stop = threading.Event()
    flushed = []

    def flusher():
        while not stop.wait(0.5):
            flushed.append(ring.flush_segment(seg_dir, "rate", [idx])[1])
    th = threading.Thread(target=flusher)
    th.start()
    rate, secs = 8_000_000, 2.0
    t0 = time.perf_counter()
    sent = 0
    while sent < rate * secs:  # paced: at most `rate` rows per second
        ahead = sent / rate - (time.perf_counter() - t0)
        if ahead > 0:
            time.sleep(ahead)
        ring.append(res, picks[(sent // B) % 64], 0, int(time.time() * 1000), 1)
        sent += B
    wall = time.perf_counter() - t0
    stop.set()
    th.join()
    assert ring.evicted == 0, ring.evicted
    assert sent / wall > 0.9 * rate, f"appender reached only {sent / wall / 1e6:.2f} M rows/s"
    assert sum(flushed) + ring.pending() == sent
    shutil.rmtree(seg_dir)
    # a 10 M-row backlog
    ring2 = N.AuditRing(1 << 24)
    for k in range(10_000_000 // B + 1):
        ring2.append(res, picks[k % 64], 0, int(time.time() * 1000), 1)
    n_rows = ring2.pending()
    t0 = time.perf_counter()
    path, n = ring2.flush_segment(seg_dir, "bulk", [idx])
    dt = time.perf_counter() - t0
    assert n == n_rows >= 10_000_000 and ring2.pending() == 0
    assert dt < 5.0, f"10M-row flush took {dt:.2f} s"
    assert os.path.getsize(path) < 26 * n_rows  # columnar + dictionary ids: ~24 B/row

"""Engine (CPU backend) against the golden model, plus thresholds, blacklist, sharding,
snapshots, degradation and the LTV / abuse services."""
import numpy as np
import pytest

from igaming_platform_amd.config import Config, TX_TYPE_ID
from igaming_platform_amd.engine.risk_engine import RiskEngine
from igaming_platform_amd.golden import ltv as GL, scoring as GS
from igaming_platform_amd.golden.features import BatchFeatures, GoldenFeatureStore, TxEvent, model_input
from igaming_platform_amd.layouts import ACCTBATCH
from igaming_platform_amd.utils.faults import Faults
from igaming_platform_amd.utils.hashing import SEED_DEVICE, SEED_FINGERPRINT, SEED_IP, id_hash

NOW = 1_760_000_000


def _txs(n, rng, n_acc=30):
    types = ["deposit", "withdraw", "bet", "win"]
    out = []
    for i in range(n):
        a = int(rng.integers(0, n_acc))
        out.append(dict(account_id=f"acc-{a}", amount=int(rng.choice([500, 5000, 150000, 2_000_000])),
                        transaction_type=types[int(rng.integers(0, 4))],
                        device_id=f"dev-{a}-{int(rng.integers(0, 5))}", ip_address=f"10.1.{a}.{int(rng.integers(0, 7))}",
                        fingerprint=f"fp-{a}"))
    return out


def _batch_rows(n_acc, rng):
    rows = np.zeros(n_acc, ACCTBATCH)
    rows["present"] = 1
    rows["total_deposits"] = rng.integers(0, 10**6, n_acc)
    rows["total_withdrawals"] = rng.integers(0, 10**6, n_acc)
    rows["deposit_count"] = rng.integers(0, 5, n_acc)
    rows["bet_count"] = rng.integers(0, 50, n_acc)
    rows["win_count"] = rows["bet_count"] // 3
    rows["bonus_claim_count"] = rng.integers(0, 6, n_acc)
    rows["account_created_at"] = NOW - rng.integers(0, 60, n_acc) * 86400
    rows["avg_bet_size"] = 12.5
    return rows


class Golden:
    """Sequential golden re-implementation of the batch semantics (score all, then update)."""

    def __init__(self, cfg):
        self.cfg = cfg
        self.st = GoldenFeatureStore(cfg.features)

    def load(self, ids, rows):
        for i, r in zip(ids, rows):
            self.st.set_batch(i, BatchFeatures(
                total_deposits=int(r["total_deposits"]), total_withdrawals=int(r["total_withdrawals"]),
                deposit_count=int(r["deposit_count"]), withdraw_count=0, bet_count=int(r["bet_count"]),
                win_count=int(r["win_count"]), avg_bet_size=float(r["avg_bet_size"]),
                account_created_at=int(r["account_created_at"]), bonus_claim_count=int(r["bonus_claim_count"])))

    def score(self, txs, now, blacklist=()):
        self.st.blacklist = {h: 0 for h in blacklist}
        out = []
        for t in txs:
            ip = id_hash(t.get("ip_address", ""), SEED_IP)
            f = self.st.raw_features(t["account_id"], now, ip_hash=ip)
            bl = self.st.blacklisted([id_hash(t.get("device_id", ""), SEED_DEVICE),
                                      id_hash(t.get("fingerprint", ""), SEED_FINGERPRINT), ip], now)
            tx = TX_TYPE_ID.get(t["transaction_type"], 255)
            rule, reasons = GS.apply_rules(self.cfg.scoring, f, t["amount"], tx, bl)
            x = model_input(f, t["amount"], tx, self.cfg.features.log_transform, self.cfg.features.width)
            out.append(GS.ensemble(self.cfg.scoring, rule, reasons, GS.heuristic_predict(x)))
        for t in txs:
            self.st.apply(TxEvent(t["account_id"], t["amount"], TX_TYPE_ID.get(t["transaction_type"], 255),
                                  id_hash(t.get("device_id", ""), SEED_DEVICE), id_hash(t.get("ip_address", ""), SEED_IP),
                                  now))
        return out


@pytest.mark.parametrize("shards", [1, 3])
def test_engine_matches_golden_over_batches(shards):
    cfg = Config()
    rng = np.random.default_rng(7)
    eng = RiskEngine(cfg, backend="cpu", capacity=200, shards=shards)
    gold = Golden(cfg)
    ids = [f"acc-{i}" for i in range(30)]
    rows = _batch_rows(30, rng)
    eng.load_batch_features(ids, rows)
    gold.load(ids, rows)
    eng.add_to_blacklist("device", "dev-3-1", "chargeback", "test")
    bl = [id_hash("dev-3-1", SEED_DEVICE)]
    for step in range(6):
        txs = _txs(40, rng)
        now = NOW + step * 20
        got = eng.score(txs, now=now)
        exp = gold.score(txs, now, bl)
        for g, (s, a, reasons, ml) in zip(got, exp):
            assert (g["score"], g["action"], g["reason_codes"]) == (s, a, reasons)
            assert g["ml_score"] == pytest.approx(ml, abs=1e-6)


def test_thresholds_update_changes_actions():
    eng = RiskEngine(Config(), backend="cpu", capacity=50)
    tx = dict(account_id="x", amount=2_000_000, transaction_type="deposit")
    assert eng.score([tx], now=NOW)[0]["score"] == 24
    assert eng.get_thresholds() == (80, 50)
    eng.update_thresholds(20, 10)
    r = eng.score([tx], now=NOW)[0]
    assert r["action"] == 3 and eng.get_thresholds() == (20, 10)
    with pytest.raises(ValueError):
        eng.update_thresholds(101, 10)


def test_blacklist_types_and_expiry():
    eng = RiskEngine(Config(), backend="cpu", capacity=50)
    eng.add_to_blacklist("ip", "6.6.6.6", "botnet", "ops", expires_at=NOW + 100)
    eng.add_to_blacklist("email", "x@evil.test", "fraud", "ops")
    assert [m.type for m in eng.check_blacklist(ip="6.6.6.6", now=NOW)] == ["ip"]
    assert eng.check_blacklist(ip="6.6.6.6", now=NOW + 101) == []
    assert eng.check_blacklist(email="x@evil.test", now=NOW)[0].reason == "fraud"
    r = eng.score([dict(account_id="a", amount=1, transaction_type="bet", ip_address="6.6.6.6")], now=NOW)[0]
    assert "KNOWN_FRAUDSTER" in r["reason_codes"]
    r = eng.score([dict(account_id="a", amount=1, transaction_type="bet", ip_address="6.6.6.6")], now=NOW + 200)[0]
    assert "KNOWN_FRAUDSTER" not in r["reason_codes"]
    with pytest.raises(ValueError):
        eng.add_to_blacklist("phone", "1", "", "")


def test_ingest_then_features_and_velocity_rule():
    eng = RiskEngine(Config(), backend="cpu", capacity=50)
    eng.ingest_events([dict(account_id="v", amount=100, transaction_type="bet", ts=NOW - i) for i in range(12)])
    f = eng.get_features("v", now=NOW)
    assert f["tx_count_1m"] == 12 and f["tx_sum_1h"] == 1200
    r = eng.score([dict(account_id="v", amount=100, transaction_type="bet")], now=NOW)[0]
    assert r["reason_codes"][0] == "HIGH_VELOCITY"
    assert eng.get_features("nobody", now=NOW)["flags"] & 64


def test_snapshot_restore_round_trip(tmp_path):
    cfg = Config()
    a = RiskEngine(cfg, backend="cpu", capacity=50, shards=2)
    txs = _txs(30, np.random.default_rng(2), n_acc=10)
    a.score(txs, now=NOW)
    a.snapshot(str(tmp_path))
    b = RiskEngine(cfg, backend="cpu", capacity=50, shards=2)
    assert b.restore(str(tmp_path)) == sum(a.registry.size(o) for o in range(2))
    for i in range(10):
        fa, fb = a.get_features(f"acc-{i}", now=NOW + 5), b.get_features(f"acc-{i}", now=NOW + 5)
        assert fa.tobytes() == fb.tobytes()


def test_shard_failure_degrades_to_fallback():
    faults = Faults("")
    eng = RiskEngine(Config(), backend="cpu", capacity=50, shards=2, faults=faults)
    txs = [dict(account_id=f"acc-{i}", amount=100, transaction_type="bet") for i in range(20)]
    eng.score(txs, now=NOW)
    faults.set("backend_error", shard=1)
    r = eng.score(txs, now=NOW)
    assert len(r) == 20 and eng.healthy == [True, False] and eng.ready()
    _, owners = eng.registry.resolve_ids([t["account_id"] for t in txs])
    for x, o in zip(r, owners):
        if o == 1:  # degraded rows: partial features (engine.go:267-270)
            assert x["features"]["flags"] & 64
    faults.clear()
    eng.recover()
    assert eng.healthy == [True, True]


def test_ltv_and_segment_cpu():
    eng = RiskEngine(Config(), backend="cpu", capacity=50)
    vip = GL.PlayerFeatures(days_since_registration=400, days_since_last_bet=1, days_since_last_deposit=2,
                            sessions_per_week=6, deposit_frequency=5, net_revenue=20000, bet_count=500)
    eng.set_players(["vip"], [vip])
    r = eng.predict_ltv("vip")
    p = GL.predict(GL.PlayerFeatures.from_row(np.float32(vip.row())))
    assert r.segment == GL.SEG_VIP == p.segment and r.found
    assert r.predicted_ltv == pytest.approx(p.predicted_ltv, rel=1e-6)
    assert r.recommended_actions()[0] == p.next_best_action
    assert not eng.predict_ltv("unknown").found


def test_ltv_predictions_audit(tmp_path):
    """Answered PredictLTV calls land in ltv_predictions (init-db.sql:141-155, declared and never
    written by the reference) with the values returned; unknown players are not logged."""
    import sqlite3
    cfg = Config()
    cfg.server.audit_db = str(tmp_path / "audit.db")
    eng = RiskEngine(cfg, backend="cpu", capacity=50)
    vip = GL.PlayerFeatures(days_since_registration=400, days_since_last_bet=1, days_since_last_deposit=2,
                            sessions_per_week=6, deposit_frequency=5, net_revenue=20000, bet_count=500)
    low = GL.PlayerFeatures(days_since_registration=30, days_since_last_bet=40, days_since_last_deposit=50,
                            sessions_per_week=0.2, deposit_frequency=0.1, net_revenue=15, bet_count=3)
    eng.set_players(["vip", "low"], [vip, low])
    got = eng.predict_ltv_batch(["vip", "low", "nobody"])
    path = str(tmp_path / "audit.db")
    assert eng.flush_audit(path) == 2 and eng.auditlog.pending() == 0
    rows = sqlite3.connect(path).execute(
        "SELECT account_id, predicted_ltv, segment, churn_risk, survival_days, next_best_action, model_version "
        "FROM ltv_predictions ORDER BY id").fetchall()
    assert [r[0] for r in rows] == ["vip", "low"]
    for r, g in zip(rows, got):
        assert r[1] == pytest.approx(g.predicted_ltv, rel=1e-6) and r[2] == GL.SEGMENTS[g.segment]
        assert r[3] == pytest.approx(g.churn_risk, rel=1e-6) and r[4] == g.survival_days and r[5] == g.next_best_action
        assert r[6] == "rules"  # the LTV model's own version, not the fraud model's


def test_ltv_model_cpu_matches_executor():
    from igaming_platform_amd.engine.ltv import ltv_model_input
    from igaming_platform_amd.native import native
    from igaming_platform_amd.onnx import builders
    m = builders.build("ltv_mlp", n_features=64, width=64, layers=2).SerializeToString()
    eng = RiskEngine(Config(), backend="cpu", capacity=50, ltv_model=m)
    f = GL.PlayerFeatures(days_since_registration=200, net_revenue=300, days_since_last_bet=10)
    eng.set_players(["p"], [f])
    X = ltv_model_input(np.float32([f.row()]), None, 64)
    ml = native().Executor(native().OnnxModel.from_bytes(m)).run({"input": X})["output"][0, 0]
    r = eng.predict_ltv("p")
    assert r.predicted_ltv == pytest.approx(GL.predict(f, float(ml)).predicted_ltv, rel=1e-5)


def test_bonus_abuse_signals_and_links():
    eng = RiskEngine(Config(), backend="cpu", capacity=50)
    rows = np.zeros(1, ACCTBATCH)
    rows["present"], rows["bonus_claim_count"], rows["total_deposits"] = 1, 5, 100
    eng.load_batch_features(["abuser"], rows)
    eng.score([dict(account_id="abuser", amount=1, transaction_type="bet", device_id="shared"),
               dict(account_id="alt1", amount=1, transaction_type="bet", device_id="shared")], now=NOW)
    r = eng.check_bonus_abuse("abuser", "welcome", now=NOW)
    assert "BONUS_ONLY_PLAYER" in r.signals and "LOW_WAGER_COMPLETION" in r.signals
    assert "SHARED_DEVICE" in r.signals and r.linked_accounts == ["alt1"]
    assert r.is_abuser and r.abuse_score == pytest.approx(0.8)
    clean = eng.check_bonus_abuse("nobody", now=NOW)
    assert not clean.is_abuser and clean.signals == []


def test_bonus_abuse_gru_model_cpu():
    from igaming_platform_amd.onnx import builders
    m = builders.build("gru", seq=100, hidden=64, layers=2).SerializeToString()
    eng = RiskEngine(Config(), backend="cpu", capacity=50, abuse_model=m)
    eng.ingest_events([dict(account_id="g", amount=100 * i, transaction_type="deposit", ts=NOW - 100 + i)
                       for i in range(30)])
    r = eng.check_bonus_abuse("g", now=NOW)
    assert r.model_score is not None and 0.0 < r.model_score < 1.0


def test_explain_text():
    eng = RiskEngine(Config(), backend="cpu", capacity=50)
    txt = eng.explain(dict(account_id="e", amount=500000, transaction_type="deposit"), now=NOW)
    assert "Fraud Score Analysis" in txt and "NEW_ACCOUNT_LARGE_TX (+30)" in txt


def test_onnx_fraud_model_cpu():
    from igaming_platform_amd.onnx import builders
    cfg = Config()
    cfg.features.width = 32
    m = builders.build("logistic", n_features=32).SerializeToString()
    eng = RiskEngine(cfg, backend="cpu", capacity=50, fraud_model=m)
    r = eng.score([dict(account_id="m", amount=1000, transaction_type="deposit")], now=NOW)[0]
    assert 0.0 < r["ml_score"] < 1.0 and eng.model_kind == "onnx"


@pytest.mark.parametrize("log_mode,sum_mode,width", [("log1p", "sliding", 30), ("identity", "compat", 30),
                                                     ("log1p", "sliding", 48)])
def test_native_cpu_backend_equals_golden_backend(log_mode, sum_mode, width):
    """The C++ CpuScorer (serving path) against the pure-Python golden backend (the spec)."""
    cfg = Config()
    cfg.features.log_transform, cfg.features.sum_mode, cfg.features.width = log_mode, sum_mode, width
    rng = np.random.default_rng(11)
    engines = [RiskEngine(cfg, backend=b, capacity=200) for b in ("cpu", "golden")]
    ids = [f"acc-{i}" for i in range(30)]
    rows = _batch_rows(30, rng)
    ext = rng.standard_normal((30, width - 30)).astype(np.float32)
    for e in engines:
        e.load_batch_features(ids, rows)
        if width > 30:
            e.load_ext_features(ids, ext)
        e.add_to_blacklist("fingerprint", "fp-7", "x", "t", expires_at=NOW + 30)
        e.set_ip_intel("10.1.4.3", proxy=True)
        e.ingest_events([dict(account_id=f"acc-{i % 30}", amount=100 + i, transaction_type="deposit",
                              device_id=f"d{i % 4}", ts=NOW - 4000 + 37 * i) for i in range(120)])
    for step in range(5):
        txs = _txs(50, rng)
        a, b = (e.score(txs, now=NOW + 17 * step) for e in engines)
        for x, y in zip(a, b):
            assert (x["score"], x["action"], x["reason_codes"], x["rule_score"]) == \
                   (y["score"], y["action"], y["reason_codes"], y["rule_score"])
            assert x["ml_score"] == pytest.approx(y["ml_score"], abs=1e-7)
            assert x["features"].tobytes() == y["features"].tobytes()
    for i in range(30):
        assert engines[0].get_features(f"acc-{i}", NOW + 99).tobytes() == \
               engines[1].get_features(f"acc-{i}", NOW + 99).tobytes()


@pytest.mark.parametrize("backend", ["cpu", "golden"])
def test_model_hot_reload_keeps_state(backend):
    """reload_model swaps the fraud model between batches: the scores after the swap equal an
    engine that ran the new model from the start (feature updates do not depend on the model);
    the version counts up; a width mismatch is refused."""
    from igaming_platform_amd.onnx import builders
    m = builders.build("logistic", n_features=30).SerializeToString()
    a = RiskEngine(Config(), backend=backend, capacity=80)
    b = RiskEngine(Config(), backend=backend, capacity=80, fraud_model=m)
    rng = np.random.default_rng(5)
    t1, t2 = _txs(120, rng), _txs(120, rng)
    a.score(t1, now=NOW)
    b.score(t1, now=NOW)
    assert a.model_kind == "heuristic" and a.model_version == 1
    assert a.reload_model(m) == 2 and a.model_kind == "onnx"
    ra, rb = a.score(t2, now=NOW + 30), b.score(t2, now=NOW + 30)
    assert [(x["score"], x["action"], x["ml_score"]) for x in ra] == [(x["score"], x["action"], x["ml_score"]) for x in rb]
    with pytest.raises(ValueError):
        a.reload_model(builders.build("logistic", n_features=32).SerializeToString())
    assert a.reload_model(None) == 3 and a.model_kind == "heuristic"


def test_http_reload_model_endpoint():
    import json
    import urllib.request
    from igaming_platform_amd.api.http_server import HttpServer
    from igaming_platform_amd.onnx import builders
    eng = RiskEngine(Config(), backend="cpu", capacity=20)
    srv = HttpServer(eng).start()
    try:
        body = builders.build("logistic", n_features=30).SerializeToString()
        req = urllib.request.Request(f"http://127.0.0.1:{srv.port}/admin/reload_model", data=body, method="POST")
        with urllib.request.urlopen(req, timeout=30) as r:
            assert json.loads(r.read()) == {"model_version": 2, "model_kind": "onnx"}
    finally:
        srv.stop()


def test_audit_ring_drains_into_risk_scores(tmp_path):
    """Every scored request lands in the risk_scores audit table (init-db.sql:122-138, declared and
    never written by the reference): same score / rule score / action / reasons as the response,
    via the engine call and via POST /admin/flush_audit."""
    import json
    import sqlite3
    import urllib.request
    from igaming_platform_amd.api.http_server import HttpServer
    from igaming_platform_amd.proto import risk_v1 as P
    cfg = Config()
    cfg.server.audit_db = str(tmp_path / "audit.db")
    eng = RiskEngine(cfg, backend="cpu", capacity=60)
    txs = _txs(50, np.random.default_rng(9))
    out = eng.score_tx_many_bytes([eng._tx_bytes(t) for t in txs], [0.0] * len(txs))
    resp = [P.ScoreTransactionResponse.FromString(b) for b in out]
    assert eng.flush_audit(cfg.server.audit_db) == 50 and eng.auditlog.pending() == 0
    db = sqlite3.connect(cfg.server.audit_db)
    rows = db.execute("SELECT account_id, score, rule_score, action, reason_codes FROM risk_scores ORDER BY id").fetchall()
    names = {v: k.lower() for k, v in P.ACTION.items()}
    for t, r, (aid, sc, rs, act, reasons) in zip(txs, resp, rows):
        assert (aid, sc, rs) == (t["account_id"], r.score, r.rule_score)
        assert names[r.action].endswith(act) and json.loads(reasons) == list(r.reason_codes)
    eng.score_tx_many_bytes([eng._tx_bytes(t) for t in txs[:7]], [0.0] * 7)
    srv = HttpServer(eng).start()
    try:
        req = urllib.request.Request(f"http://127.0.0.1:{srv.port}/admin/flush_audit", data=b"", method="POST")
        with urllib.request.urlopen(req, timeout=30) as r:
            assert json.loads(r.read()) == {"rows": 7}
    finally:
        srv.stop()
    assert db.execute("SELECT COUNT(*) FROM risk_scores").fetchone()[0] == 57


def test_audit_version_stamped_at_score_time_and_explain_logged(tmp_path):
    """rows scored before a model reload keep the old model version; explain()
    (ScoreWithExplanation, /debug/score) and score() are audited like the wire paths."""
    import sqlite3
    from igaming_platform_amd.onnx import builders
    cfg = Config()
    cfg.server.audit_db = str(tmp_path / "audit.db")
    eng = RiskEngine(cfg, backend="cpu", capacity=60)
    txs = _txs(6, np.random.default_rng(3))
    eng.score(txs[:3])
    eng.explain(txs[3])
    eng.reload_model(builders.build("logistic", n_features=30).SerializeToString())
    eng.score(txs[4:6])
    assert eng.flush_audit(cfg.server.audit_db) == 6
    vers = [r[0] for r in sqlite3.connect(cfg.server.audit_db).execute(
        "SELECT model_version FROM risk_scores ORDER BY id")]
    assert vers == ["1"] * 4 + ["2"] * 2


def test_audit_flush_into_db_without_ltv_table_and_failure_keeps_rows(tmp_path):
    """The schema script runs on every flush (an existing DB with only risk_scores gains
    ltv_predictions), and a failed write puts the drained rows back."""
    import sqlite3
    cfg = Config()
    path = str(tmp_path / "old.db")
    db = sqlite3.connect(path)
    db.execute("CREATE TABLE risk_scores (id INTEGER PRIMARY KEY AUTOINCREMENT, account_id TEXT, score INT,"
               " rule_score INT, ml_score REAL, action TEXT, reason_codes TEXT, model_version TEXT, created_at REAL)")
    db.commit()
    db.close()
    cfg.server.audit_db = path
    eng = RiskEngine(cfg, backend="cpu", capacity=60)
    vip = GL.PlayerFeatures(days_since_registration=400, days_since_last_bet=1, days_since_last_deposit=2,
                            sessions_per_week=6, deposit_frequency=5, net_revenue=20000, bet_count=500)
    eng.set_players(["vip"], [vip])
    eng.predict_ltv("vip")
    eng.score(_txs(4, np.random.default_rng(1)))
    assert eng.flush_audit(path) == 5
    eng.score(_txs(3, np.random.default_rng(2)))
    bad = str(tmp_path / "no_such_dir" / "x.db")
    with pytest.raises(sqlite3.OperationalError):
        eng.flush_audit(bad)
    assert eng.auditlog.pending() == 3
    assert eng.flush_audit(path) == 3
    assert sqlite3.connect(path).execute("SELECT COUNT(*) FROM risk_scores").fetchone()[0] == 7


def test_audit_disabled_without_audit_db():
    eng = RiskEngine(Config(), backend="cpu", capacity=20)
    eng.score(_txs(3, np.random.default_rng(1)))
    assert eng.auditlog.pending() == 0


def test_velocity_rate_limit_counters_and_features():
    """GetVelocity / CheckRateLimit / IncrementCounter / Set+GetFeature / DeleteAccountFeatures
    (redis_store.go:171-240)."""
    eng = RiskEngine(Config(), backend="cpu", capacity=50)
    evs = [dict(account_id="v1", amount=100, transaction_type="bet", ts=NOW - d) for d in (30, 100, 1000, 4000, 59)]
    eng.ingest_events(evs)
    assert eng.get_velocity("v1", now=NOW) == (2, 3, 4)          # 30 s, 59 s | +100 s | +1000 s (4000 s: out)
    assert eng.get_velocity("nobody", now=NOW) == (0, 0, 0)
    assert eng.check_rate_limit("v1", max_per_min=2, max_per_hour=100, now=NOW)
    assert not eng.check_rate_limit("v1", max_per_min=3, max_per_hour=5, now=NOW)
    assert eng.check_rate_limit("v1", max_per_min=3, max_per_hour=4, now=NOW)
    eng.set_scoring(max_tx_per_minute=10, max_tx_per_hour=4)   # defaults: the live config
    assert list(eng.check_rate_limit_batch(["v1", "nobody"], now=NOW)) == [True, False]
    assert eng.increment_counter("bonus:claims:v1", 60, now=NOW) == 1
    assert eng.increment_counter("bonus:claims:v1", 60, now=NOW + 10) == 2
    assert eng.increment_counter("bonus:claims:v1", 60, now=NOW + 71) == 1  # expired 60 s after the last INCR
    eng.set_feature("v1", "kyc_level", 3, ttl_s=100, now=NOW)
    assert eng.get_feature("v1", "kyc_level", now=NOW + 50) == "3"
    assert eng.get_feature("v1", "kyc_level", now=NOW + 101) is None
    eng.set_feature("v1", "vip", "gold", now=NOW)
    eng.delete_account_features(["v1"])
    assert eng.get_feature("v1", "vip", now=NOW) is None
    assert eng.get_velocity("v1", now=NOW) == (0, 0, 0)


def test_feature_importance_from_the_loaded_model():
    from igaming_platform_amd.features.store_ops import STATIC_IMPORTANCE
    from igaming_platform_amd.onnx import builders
    assert RiskEngine(Config(), backend="cpu", capacity=10).get_feature_importance() == STATIC_IMPORTANCE
    cfg = Config()
    cfg.features.width = 128
    imp = RiskEngine(cfg, backend="cpu", capacity=10,
                     fraud_model=builders.build("stacked", n_trees=20, depth=4).SerializeToString()).get_feature_importance()
    assert imp and abs(sum(imp.values()) - 1) < 1e-9 and all(v > 0 for v in imp.values())
    assert list(imp.values()) == sorted(imp.values(), reverse=True)
    assert set(imp) <= set(__import__("igaming_platform_amd.features.store_ops", fromlist=["x"]).input_names(128))
    lg = RiskEngine(Config(), backend="cpu", capacity=10,
                    fraud_model=builders.build("logistic", n_features=30).SerializeToString()).get_feature_importance()
    assert len(lg) == 30 and "tx_count_1m" in lg


def test_cached_hll_estimates_follow_the_registers(tmp_path):
    """AcctRT's cached HyperLogLog estimates (hll_dev_n / hll_ip_n, refreshed by every path that
    raises a register: PFCOUNT on a cached cardinality, redis_store.go:80-81) equal the estimate
    of the account's register file after every batch, across a TTL expiry (the reset path) -
    and a snapshot written before the cache existed (version 1, counts zero) restores them."""
    from igaming_platform_amd.golden.hll import count_many
    from igaming_platform_amd.layouts import ACCTRT
    eng = RiskEngine(Config(), backend="cpu", capacity=256)
    rng = np.random.default_rng(31)
    sc = eng.backends[0].sc
    ttl = eng.cfg.features.hll_ttl_s

    def check():
        st = sc.state()
        rt = st["rt"].reshape(-1, ACCTRT.itemsize).view(ACCTRT).reshape(-1)
        hll = st["hll"].reshape(len(rt), 2, 256)
        np.testing.assert_array_equal(rt["hll_dev_n"], count_many(hll[:, 0]))
        np.testing.assert_array_equal(rt["hll_ip_n"], count_many(hll[:, 1]))
        return rt, hll
    for step, now in enumerate((NOW, NOW + 60, NOW + ttl + 100, NOW + ttl + 160)):
        eng.score(_txs(200, rng), now=now)
        rt, hll = check()
    assert rt["hll_dev_n"].max() > 1 and rt["hll_ip_n"].max() > 1
    # an old snapshot: same state with the cached estimates zeroed and version 1
    path = str(tmp_path / "old.npz")
    st = sc.state()
    rt0 = st["rt"].copy().reshape(-1, ACCTRT.itemsize).view(ACCTRT).reshape(-1)
    rt0["hll_dev_n"] = rt0["hll_ip_n"] = 0
    np.savez(path, version=np.array([1]), ring_size=np.array([eng.cfg.features.ring_size]),
             **{**st, "rt": rt0.view(np.uint8).reshape(-1)})
    eng2 = RiskEngine(Config(), backend="cpu", capacity=256)
    eng2.backends[0].restore(path)
    st2 = eng2.backends[0].sc.state()
    np.testing.assert_array_equal(st2["rt"], st["rt"])

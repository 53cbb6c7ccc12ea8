"""The native HTTP/2 gRPC server (csrc/runtime/h2grpc.cpp, api/native_grpc.py) with real grpc
clients: every unary risk.v1 RPC and health Check, error statuses, ScoreTransaction through the
serving core without Python, the engine's Python path while the native path is off, concurrency
over many connections and a multi-MB ScoreBatch. Reference: services/risk/cmd/main.go:72-258."""
import time
from concurrent.futures import ThreadPoolExecutor

import grpc
import numpy as np
import pytest

from igaming_platform_amd.api.grpc_server import RiskServer
from igaming_platform_amd.api.native_grpc import NativeRiskServer
from igaming_platform_amd.clients.risk_client import RiskClient
from igaming_platform_amd.config import Config
from igaming_platform_amd.engine.risk_engine import RiskEngine
from igaming_platform_amd.golden import ltv as GL
from igaming_platform_amd.proto import risk_v1 as P


@pytest.fixture(scope="module")
def nstack():
    eng = RiskEngine(Config(), backend="cpu", capacity=4000)
    assert eng.core is not None
    srv = NativeRiskServer(eng, port=0, workers=2).start()
    cli = RiskClient(f"127.0.0.1:{srv.port}", timeout_s=30.0)
    yield eng, srv, cli
    cli.close()
    srv.stop()
    eng.close()


def test_scoring_rpcs_go_through_the_core(nstack):
    eng, srv, cli = nstack
    st0 = srv.stats()
    r = cli.score("n-1", 2_000_000, "deposit", device_id="d", ip_address="1.1.1.1")
    assert r.score == 24 and r.action == P.ACTION["ACTION_APPROVE"] and list(r.reason_codes) == ["NEW_ACCOUNT_LARGE_TX"]
    assert r.rule_score == 30 and r.HasField("features") and r.features.tx_count_1m == 0
    b = cli.score_batch([dict(account_id="n-1", amount=10, transaction_type="bet")] * 5)
    assert len(b.results) == 5 and all(x.features.tx_count_1m == 1 for x in b.results)
    st = srv.stats()
    assert st["hot_tx"] - st0["hot_tx"] == 1 and st["hot_batch"] - st0["hot_batch"] == 1


def test_same_answers_as_the_python_server():
    """The same request stream through the native server and through the grpc.aio server of an
    identical engine: identical responses (processing_time_ms aside)."""
    engs = [RiskEngine(Config(), backend="cpu", capacity=500) for _ in range(2)]
    a = NativeRiskServer(engs[0], port=0, workers=1).start()
    b = RiskServer(engs[1], port=0).start()
    ca, cb = RiskClient(f"127.0.0.1:{a.port}", timeout_s=30.0), RiskClient(f"127.0.0.1:{b.port}", timeout_s=30.0)
    try:
        rng = np.random.default_rng(3)
        for i in range(60):
            kw = dict(account_id=f"acc-{int(rng.integers(0, 12))}", amount=int(rng.choice([500, 150000, 2_000_000])),
                      transaction_type=["deposit", "withdraw", "bet", "win"][i % 4], device_id=f"dev-{i % 5}")
            x = ca.score(kw["account_id"], kw["amount"], kw["transaction_type"], device_id=kw["device_id"])
            y = cb.score(kw["account_id"], kw["amount"], kw["transaction_type"], device_id=kw["device_id"])
            for m in (x, y):  # wall-clock fields: the two servers see the call a moment apart
                m.response_time_ms = 0
                m.features.time_since_last_tx_sec = m.features.session_duration_sec = 0
            assert x == y
        for id_ in ("acc-1", "acc-3"):
            fa, fb = ca.get_features(id_).features, cb.get_features(id_).features
            for f in (fa, fb):
                f.time_since_last_tx_sec = f.session_duration_sec = 0
            assert fa == fb
    finally:
        ca.close()
        cb.close()
        a.stop()
        b.stop(0.5)
        for e in engs:
            e.close()


def test_cold_rpcs_errors_and_health(nstack):
    eng, srv, cli = nstack
    eng.set_players(["nl-1"], [GL.PlayerFeatures(days_since_registration=3, net_revenue=30)])
    r = cli.predict_ltv("nl-1")
    assert r.account_id == "nl-1" and r.segment == P.SEGMENT["SEGMENT_HIGH"]
    assert cli.player_segment("nl-1").segment == r.segment
    assert not cli.check_bonus_abuse("nl-1", "welcome").is_abuser
    with pytest.raises(grpc.RpcError) as e:
        cli.predict_ltv("")
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT and "account_id" in e.value.details()
    assert cli.add_to_blacklist("device", "nbad", "chargeback", "analyst").success
    assert cli.check_blacklist(device_id="nbad").is_blacklisted
    assert "KNOWN_FRAUDSTER" in cli.score("nbl", 10, "bet", device_id="nbad").reason_codes
    u = cli.update_thresholds(75, 45)
    assert (u.block_threshold, u.review_threshold) == (75, 45)
    g = cli.get_thresholds()
    assert (g.block_threshold, g.review_threshold) == (75, 45)
    cli.update_thresholds(80, 50)
    assert cli.health("") == "SERVING" and cli.health(P.SERVICE) == "SERVING"
    with pytest.raises(grpc.RpcError) as e:
        cli.health("no.such.Service")
    assert e.value.code() == grpc.StatusCode.NOT_FOUND
    with pytest.raises(grpc.RpcError) as e:
        cli.channel.unary_unary("/risk.v1.RiskService/NoSuchMethod")(b"", timeout=10)
    assert e.value.code() == grpc.StatusCode.UNIMPLEMENTED


def test_internal_errors_and_bad_payloads(nstack, monkeypatch):
    eng, srv, cli = nstack

    def boom(*a, **k):
        raise RuntimeError("kaboom")
    monkeypatch.setattr(eng, "get_thresholds", boom)
    with pytest.raises(grpc.RpcError) as e:
        cli.get_thresholds()
    assert e.value.code() == grpc.StatusCode.INTERNAL and e.value.details() == "internal server error"
    # a ScoreTransaction payload the wire parser refuses: INVALID_ARGUMENT from the core
    with pytest.raises(grpc.RpcError) as e:
        cli.channel.unary_unary(P.method_path("ScoreTransaction"))(b"\x0a\xff\xff\xff\xff\x0f", timeout=10)
    assert e.value.code() in (grpc.StatusCode.INVALID_ARGUMENT, grpc.StatusCode.INTERNAL)


def test_python_path_while_the_native_path_is_off(nstack):
    """With a fault injected the engine refuses the native path; the watcher turns the hot flag
    off and ScoreTransaction is served by the engine's Python path (fault semantics kept)."""
    eng, srv, cli = nstack
    eng.faults.set("backend_error", shard=0)
    try:
        t_end = time.time() + 5
        while time.time() < t_end and srv.stats()["cold"] == srv.stats()["cold"] and eng._native_ok():
            time.sleep(0.05)
        time.sleep(0.3)  # the watcher's period
        c0 = srv.stats()["cold"]
        r = cli.score("off-1", 500, "bet")
        assert r.action in (1, 2, 3)
        assert srv.stats()["cold"] == c0 + 1
    finally:
        eng.faults.clear()


def test_many_connections_and_a_large_batch(nstack):
    eng, srv, cli = nstack
    addr = f"127.0.0.1:{srv.port}"
    chans = [grpc.insecure_channel(addr) for _ in range(8)]
    call = [c.unary_unary(P.method_path("ScoreTransaction")) for c in chans]
    req = [P.ScoreTransactionRequest(account_id=f"mc-{i % 300}", amount=100 + i, transaction_type="bet")
           .SerializeToString() for i in range(2000)]

    def one(i):
        return P.ScoreTransactionResponse.FromString(call[i % 8](req[i], timeout=30))
    with ThreadPoolExecutor(32) as ex:
        out = list(ex.map(one, range(2000)))
    assert all(1 <= r.action <= 3 for r in out)
    # a 8192-transaction ScoreBatch (~1 MB request, ~1.5 MB response) through flow control
    txs = [P.ScoreTransactionRequest(account_id=f"big-{i % 1000}", amount=10 + i, transaction_type="deposit",
                                     device_id=f"d{i % 17}") for i in range(8192)]
    body = P.ScoreBatchRequest(transactions=txs).SerializeToString()
    resp = P.ScoreBatchResponse.FromString(chans[0].unary_unary(P.method_path("ScoreBatch"))(body, timeout=60))
    assert len(resp.results) == 8192
    for c in chans:
        c.close()
    assert srv.stats()["connections"] >= 1


def test_native_load_generator_against_the_native_server(nstack):
    """csrc/runtime/h2grpc.cpp grpc_load (the open-loop client of tools/bench_e2e.py): every
    scheduled call answered, latencies from the scheduled send times."""
    from igaming_platform_amd.native import native
    eng, srv, cli = nstack
    body = [P.ScoreTransactionRequest(account_id=f"lg-{i}", amount=100, transaction_type="bet").SerializeToString()
            for i in range(64)]
    r = native().grpc_load("127.0.0.1", srv.port, P.method_path("ScoreTransaction"), body, 1000.0, 1.0, 4, 512)
    assert r["errors"] == 0 and r["sent"] == 1000 and len(r["latency_ms"]) == 1000
    assert float(np.median(r["latency_ms"])) < 1000 and r["elapsed"] >= 1.0


def test_unary_in_flight_cap_with_concurrent_batches():
    """ServeCore Options.unary_depth (GpuConfig.unary_depth): while unary calls arrive the core
    keeps at most that many steps in flight, the full serve_depth otherwise. With a cap of 1
    under concurrent ScoreTransaction and ScoreBatch traffic every call is still answered, and a
    batch's rows all see the account's 128 earlier rows (8 batches x 16) in their 1-minute window."""
    cfg = Config()
    cfg.gpu.serve_depth, cfg.gpu.unary_depth = 4, 1
    eng = RiskEngine(cfg, backend="cpu", capacity=4000)
    srv = NativeRiskServer(eng, port=0, workers=2).start()
    addr = f"127.0.0.1:{srv.port}"
    chans = [grpc.insecure_channel(addr) for _ in range(4)]
    try:
        tx = [c.unary_unary(P.method_path("ScoreTransaction")) for c in chans]
        sb = chans[0].unary_unary(P.method_path("ScoreBatch"))
        req = [P.ScoreTransactionRequest(account_id=f"ud-{i % 50}", amount=100 + i, transaction_type="bet")
               .SerializeToString() for i in range(400)]
        body = P.ScoreBatchRequest(transactions=[P.ScoreTransactionRequest(
            account_id="ud-batch", amount=10, transaction_type="bet")] * 16).SerializeToString()

        def one(i):
            if i % 50 == 0:
                return len(P.ScoreBatchResponse.FromString(sb(body, timeout=30)).results)
            return P.ScoreTransactionResponse.FromString(tx[i % 4](req[i], timeout=30)).action
        with ThreadPoolExecutor(16) as ex:
            out = list(ex.map(one, range(400)))
        assert all(o == 16 for i, o in enumerate(out) if i % 50 == 0)
        assert all(1 <= o <= 3 for i, o in enumerate(out) if i % 50)
        # the batch account's rows: 8 earlier batches x 16 rows, scored at the batch clock
        last = P.ScoreBatchResponse.FromString(sb(body, timeout=30))
        assert {r.features.tx_count_1m for r in last.results} == {8 * 16}
    finally:
        for c in chans:
            c.close()
        srv.stop()
        eng.close()

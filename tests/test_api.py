"""T3: every risk.v1 RPC over a real in-process gRPC server (CPU backend), the health and
reflection services, the interceptors and the HTTP side endpoints."""
import json
import threading
import time
import urllib.request

import grpc
import pytest

from igaming_platform_amd.api.grpc_server import RiskServer
from igaming_platform_amd.api.http_server import HttpServer
from igaming_platform_amd.clients.risk_client import RiskClient
from igaming_platform_amd.config import Config
from igaming_platform_amd.engine.risk_engine import RiskEngine
from igaming_platform_amd.golden import ltv as GL
from igaming_platform_amd.proto import reflection_v1 as RV
from igaming_platform_amd.proto import risk_v1 as P


@pytest.fixture(scope="module")
def stack():
    eng = RiskEngine(Config(), backend="cpu", capacity=1000)
    gs = RiskServer(eng, port=0, max_batch=64, wait_us=500).start()
    hs = HttpServer(eng, port=0).start()
    cli = RiskClient(f"127.0.0.1:{gs.port}", timeout_s=30.0)  # first calls pay lazy init on a loaded box
    yield eng, gs, hs, cli
    cli.close()
    gs.stop(0.5)
    hs.stop()


def _http(hs, path):
    with urllib.request.urlopen(f"http://127.0.0.1:{hs.port}{path}", timeout=5) as r:
        return r.status, r.read().decode()


def test_descriptor_contract():
    """Field numbers of the hot messages (risk.proto Appendix B)."""
    d = P.ScoreTransactionRequest.DESCRIPTOR
    assert {f.name: f.number for f in d.fields} == {
        "account_id": 1, "player_id": 2, "amount": 3, "transaction_type": 4, "currency": 5, "game_id": 6,
        "round_id": 7, "ip_address": 8, "device_id": 9, "fingerprint": 10, "user_agent": 11, "session_id": 12,
        "metadata": 13}
    d = P.ScoreTransactionResponse.DESCRIPTOR
    assert [f.number for f in d.fields] == [1, 2, 3, 4, 5, 6, 7]
    assert len(P.FeatureVector.DESCRIPTOR.fields) == 26
    assert P.ACTION == {"ACTION_UNSPECIFIED": 0, "ACTION_APPROVE": 1, "ACTION_REVIEW": 2, "ACTION_BLOCK": 3}
    svc = P.M["ScoreBatchRequest"].DESCRIPTOR.file.services_by_name["RiskService"]
    assert [m.name for m in svc.methods] == [m[0] for m in P.METHODS]


def test_score_transaction_and_batch(stack):
    eng, gs, hs, cli = stack
    r = cli.score("api-1", 2_000_000, "deposit", device_id="d", ip_address="1.1.1.1")
    assert r.score == 24 and r.action == P.ACTION["ACTION_APPROVE"] and list(r.reason_codes) == ["NEW_ACCOUNT_LARGE_TX"]
    assert r.rule_score == 30 and r.HasField("features") and r.features.tx_count_1m == 0
    b = cli.score_batch([dict(account_id="api-1", amount=10, transaction_type="bet")] * 5)
    assert len(b.results) == 5 and all(x.features.tx_count_1m == 1 for x in b.results)


def test_concurrent_unary_calls_are_micro_batched(stack):
    eng, gs, hs, cli = stack
    native = gs.native_tx is not None   # the serving core's FIFO is the micro-batcher
    before = eng.core.stats(False)["steps"] if native else gs.batcher.batches
    unary0 = eng.core.stats(False)["unary"] if native else 0
    out, errs = [], []

    def worker(i):
        try:
            out.append(cli.score(f"conc-{i % 7}", 100 + i, "bet").score)
        except Exception as e:  # pragma: no cover
            errs.append(e)

    th = [threading.Thread(target=worker, args=(i,)) for i in range(48)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errs and len(out) == 48
    if native:
        st = eng.core.stats(False)
        assert st["unary"] - unary0 == 48
        assert st["steps"] - before <= 48   # never more than one step per call
        # a burst of concurrent calls (grpc futures, one client thread): they share steps
        import grpc as _g
        ch = _g.insecure_channel(f"127.0.0.1:{gs.port}")
        call = ch.unary_unary(P.method_path("ScoreTransaction"))
        s0 = eng.core.stats(False)["steps"]
        futs = [call.future(P.ScoreTransactionRequest(account_id=f"burst-{i % 9}", amount=100 + i,
                                                      transaction_type="bet").SerializeToString(), timeout=30)
                for i in range(256)]
        got = [P.ScoreTransactionResponse.FromString(f.result()) for f in futs]
        ch.close()
        assert len(got) == 256 and all(1 <= g.action <= 3 for g in got)
        assert eng.core.stats(False)["steps"] - s0 <= 256
        # calls queued while the device is busy share one micro-batch: hold a core (an engine
        # of its own: the server's poller drains this one's completions), queue 300 unary
        # requests, release it -> one device step answers all of them
        from igaming_platform_amd.engine.risk_engine import RiskEngine
        e2 = RiskEngine(Config(), backend="cpu", capacity=512)
        e2.core.pause()
        s1 = e2.core.stats(False)["steps"]
        e2.core.submit_tx_many([P.ScoreTransactionRequest(account_id=f"held-{i % 11}", amount=50 + i,
                                                          transaction_type="deposit").SerializeToString()
                                for i in range(300)], list(range(10_000, 10_300)))
        e2.core.resume()
        done, t_end = [], time.time() + 30
        while len(done) < 300 and time.time() < t_end:
            done += e2.core.poll(4096, 200_000)
        e2.close()
        assert sorted(t for t, _, _ in done) == list(range(10_000, 10_300)) and all(e is None for _, _, e in done)
        assert e2.core.stats(False)["steps"] - s1 == 1
    else:
        assert gs.batcher.batches - before < 48   # at least some calls shared a device batch


def test_ltv_segment_abuse(stack):
    eng, gs, hs, cli = stack
    eng.set_players(["ltv-1"], [GL.PlayerFeatures(days_since_registration=3, net_revenue=30)])
    r = cli.predict_ltv("ltv-1")
    assert r.account_id == "ltv-1" and r.segment == P.SEGMENT["SEGMENT_HIGH"] and r.predicted_at.seconds > 0
    s = cli.player_segment("ltv-1")
    assert s.segment == r.segment and list(s.recommended_actions)[0] == r.next_best_action
    a = cli.check_bonus_abuse("ltv-1", "welcome")
    assert not a.is_abuser
    with pytest.raises(grpc.RpcError) as e:
        cli.predict_ltv("")
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT


def test_concurrent_cold_rpcs_are_micro_batched(stack):
    """PredictLTV / GetPlayerSegment / CheckBonusAbuse calls in flight together merge into one
    batched engine call (one LTV launch / one feature read + GRU launch per shard), and each
    caller still gets its own account's answer."""
    from concurrent.futures import ThreadPoolExecutor
    eng, gs, _, cli = stack
    ids = [f"cold-{i}" for i in range(48)]
    eng.set_players(ids, [GL.PlayerFeatures(days_since_registration=10 + i, net_revenue=50 * i) for i in range(48)])
    want_ltv = {i: eng.predict_ltv(i).predicted_ltv for i in ids}
    lb, ab = gs.ltv_batcher.batches, gs.abuse_batcher.batches
    with ThreadPoolExecutor(48) as ex:
        ltv = list(ex.map(lambda i: cli.predict_ltv(i), ids))
        seg = list(ex.map(lambda i: cli.player_segment(i), ids))
        abu = list(ex.map(lambda i: cli.check_bonus_abuse(i), ids))
    assert [r.account_id for r in ltv] == ids and [r.account_id for r in seg] == ids
    assert all(r.predicted_ltv == pytest.approx(want_ltv[i], rel=1e-6) for r, i in zip(ltv, ids))
    assert all(not r.is_abuser for r in abu)
    assert gs.ltv_batcher.items >= 96 and gs.abuse_batcher.items >= 48
    assert gs.ltv_batcher.batches - lb < 96 and gs.abuse_batcher.batches - ab < 48


def test_blacklist_rpcs(stack):
    eng, gs, hs, cli = stack
    r = cli.add_to_blacklist("device", "bad-dev", "chargeback", "analyst")
    assert r.success and r.id
    c = cli.check_blacklist(device_id="bad-dev", ip_address="9.9.9.9")
    assert c.is_blacklisted and c.matches[0].type == "device" and c.matches[0].reason == "chargeback"
    assert not cli.check_blacklist(device_id="fine").is_blacklisted
    s = cli.score("bl-acc", 10, "bet", device_id="bad-dev")
    assert "KNOWN_FRAUDSTER" in s.reason_codes
    with pytest.raises(grpc.RpcError) as e:
        cli.add_to_blacklist("phone", "123")
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT


def test_features_and_thresholds(stack):
    eng, gs, hs, cli = stack
    cli.score("feat-1", 777, "deposit")
    f = cli.get_features("feat-1")
    assert f.account_id == "feat-1" and f.features.tx_count_1h == 1 and f.features.tx_sum_1h == 777
    u = cli.update_thresholds(75, 45)
    assert u.success and (u.block_threshold, u.review_threshold) == (75, 45)
    g = cli.get_thresholds()
    assert (g.block_threshold, g.review_threshold) == (75, 45)
    assert json.loads(_http(hs, "/debug/thresholds")[1]) == {"block_threshold": 75, "review_threshold": 45}  # Q7
    cli.update_thresholds(80, 50)


def test_health_and_reflection(stack):
    eng, gs, hs, cli = stack
    assert cli.health("") == "SERVING" and cli.health(P.SERVICE) == "SERVING"
    M = RV.M["grpc.reflection.v1alpha"]
    call = cli.channel.stream_stream("/grpc.reflection.v1alpha.ServerReflection/ServerReflectionInfo",
                                     request_serializer=lambda m: m.SerializeToString(),
                                     response_deserializer=M["ServerReflectionResponse"].FromString)
    reqs = [M["ServerReflectionRequest"](list_services="*"),
            M["ServerReflectionRequest"](file_containing_symbol="risk.v1.RiskService")]
    resp = list(call(iter(reqs), timeout=5))
    names = [s.name for s in resp[0].list_services_response.service]
    assert P.SERVICE in names and "grpc.health.v1.Health" in names
    from google.protobuf import descriptor_pb2
    fds = [descriptor_pb2.FileDescriptorProto.FromString(b) for b in resp[1].file_descriptor_response.file_descriptor_proto]
    assert "risk/v1/risk.proto" in [f.name for f in fds] and "google/protobuf/timestamp.proto" in [f.name for f in fds]


def test_http_endpoints_and_metrics(stack):
    eng, gs, hs, cli = stack
    cli.score("feat-http", 777, "deposit")  # this test's own RPC (xdist may run it before the others)
    assert _http(hs, "/health") == (200, "OK")
    assert _http(hs, "/ready") == (200, "Ready")
    code, body = _http(hs, "/debug/score?account_id=http-1&amount=500000&type=deposit")
    assert code == 200 and "NEW_ACCOUNT_LARGE_TX" in body
    code, body = _http(hs, "/metrics")
    assert 'risk_requests_total{code="OK",method="ScoreTransaction"}' in body
    assert "risk_action_total" in body and "risk_latency_seconds_bucket" in body
    code, body = _http(hs, "/debug/features?account_id=feat-http")
    assert json.loads(body)["tx_sum_1h"] == 777


def test_recovery_interceptor_maps_internal_errors(stack, monkeypatch):
    eng, gs, hs, cli = stack

    def boom(*a, **k):
        raise RuntimeError("kaboom")

    monkeypatch.setattr(eng, "get_thresholds", boom)
    with pytest.raises(grpc.RpcError) as e:
        cli.get_thresholds()
    assert e.value.code() == grpc.StatusCode.INTERNAL and e.value.details() == "internal server error"

"""Native account RPCs (csrc/runtime/acct_core.cpp, engine/acct.py): PredictLTV,
GetPlayerSegment and CheckBonusAbuse from request bytes to response bytes without Python, on
CPU devices here (GPU twins in tests/test_acct_gpu.py). Every answer must equal the Python
servicer's (api/grpc_server.py RiskServicer over engine/ltv.py / engine/abuse.py), byte for byte
except PredictLTVResponse.predicted_at; the multi-process tests route accounts owned by other
ranks over the node-shared mailbox and compare every rank's answers with a single-process engine.
Reference: proto/risk/v1/risk.proto:16-20, 95-145."""
import os
import socket
import time

import numpy as np
import pytest

NOW = 1_700_000_000


def _players(n, seed):
    from igaming_platform_amd.golden import ltv as GL
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        out.append(GL.PlayerFeatures(
            days_since_registration=int(rng.integers(0, 600)), days_since_last_deposit=int(rng.integers(0, 60)),
            days_since_last_bet=int(rng.integers(0, 60)), sessions_per_week=float(rng.uniform(0, 8)),
            deposit_frequency=float(rng.uniform(0, 6)), net_revenue=float(rng.uniform(-500, 40000)),
            total_deposits=float(rng.uniform(0, 50000)), total_withdrawals=float(rng.uniform(0, 50000)),
            bet_count=int(rng.integers(0, 400)), bonuses_claimed=int(rng.integers(0, 6)),
            games_played=int(rng.integers(0, 12)), bonus_conversion_rate=float(rng.uniform(0, 1)),
            push_enabled=bool(rng.integers(0, 2)), has_vip_manager=bool(rng.integers(0, 2)),
            support_tickets=int(rng.integers(0, 6))))
    return out


def _populate(eng, n=30):
    """Profiles, warehouse rows, scored traffic (device links) and event histories."""
    from igaming_platform_amd.layouts import ACCTBATCH
    ids = [f"acc-{i}" for i in range(n)]
    eng.set_players(ids, _players(n, 1))
    rows = np.zeros(n, ACCTBATCH)
    rows["present"] = 1
    rows["total_deposits"] = np.arange(n) * 700
    rows["bonus_claim_count"] = np.arange(n) % 6
    rows["bonus_wager_complete"] = (np.arange(n) % 5) / 5.0
    rows["account_created_at"] = NOW - (np.arange(n) % 10) * 86400
    eng.load_batch_features(ids, rows)
    rng = np.random.default_rng(2)
    for step in range(3):
        eng.score([dict(account_id=f"acc-{int(a)}", amount=int(rng.choice([500, 150000])), transaction_type="bet",
                        device_id=f"dev-{int(a) % 7}", ip_address=f"10.0.{int(a)}.{int(rng.integers(0, 4))}")
                   for a in rng.integers(0, n, 50)], now=NOW - 100 + step)
    eng.ingest_events([dict(account_id=f"acc-{i % n}", amount=100 * i, transaction_type="deposit", ts=NOW - 300 + i)
                       for i in range(120)])
    eng._flush_links()
    return ids + ["nobody", "ghost-1"]


def _requests(ids):
    from igaming_platform_amd.native import native
    from igaming_platform_amd.proto import risk_v1 as P
    N = native()
    out = []
    for a in ids:
        out.append((N.RPC_LTV, P.PredictLTVRequest(account_id=a)))
        out.append((N.RPC_SEGMENT, P.GetPlayerSegmentRequest(account_id=a)))
        out.append((N.RPC_ABUSE, P.CheckBonusAbuseRequest(account_id=a, bonus_id="welcome")))
    return out


def _ask(router, reqs, now=NOW, timeout=20.0):
    """Submit every request; returns [(bytes, err)] in request order."""
    for i, (rpc, m) in enumerate(reqs):
        router.submit(rpc, m.SerializeToString(), i, 0, now)
    got = {}
    t_end = time.time() + timeout
    while len(got) < len(reqs) and time.time() < t_end:
        for tag, b, e in router.poll(4096, 50000):
            got[int(tag)] = (b, e)
    assert len(got) == len(reqs), f"{len(reqs) - len(got)} answers missing"
    return [got[i] for i in range(len(reqs))]


def _python_answer(eng, rpc, m, now=NOW):
    from igaming_platform_amd.api.grpc_server import RiskServicer
    from igaming_platform_amd.native import native
    N = native()
    svc = RiskServicer(eng)
    if rpc == N.RPC_LTV:
        r = svc.PredictLTV(m, None)
        r.ClearField("predicted_at")
    elif rpc == N.RPC_SEGMENT:
        r = svc.GetPlayerSegment(m, None)
    else:
        r = svc.abuse_response(eng.check_bonus_abuse(m.account_id, m.bonus_id, now=now))
    return r.SerializeToString()


def _normalise(rpc, b):
    from igaming_platform_amd.native import native
    from igaming_platform_amd.proto import risk_v1 as P
    if rpc == native().RPC_LTV:
        r = P.PredictLTVResponse.FromString(b)
        assert r.predicted_at.seconds > 1_600_000_000  # stamped with the wall clock when answered
        r.ClearField("predicted_at")
        return r.SerializeToString()
    return b


@pytest.mark.parametrize("models", ["rules", "models"])
def test_native_account_rpcs_equal_python_path(models):
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.risk_engine import RiskEngine
    from igaming_platform_amd.onnx import builders
    kw = {}
    if models == "models":
        kw = dict(ltv_model=builders.build("ltv_mlp", n_features=64, width=64, layers=2).SerializeToString(),
                  abuse_model=builders.build("gru", seq=100, hidden=64, layers=2).SerializeToString())
    eng = RiskEngine(Config(), backend="cpu", capacity=64, **kw)
    assert eng.acct is not None and all(eng.acct.serves(r) for r in (1, 2, 3))
    ids = _populate(eng)
    reqs = _requests(ids)
    got = _ask(eng.acct.router, reqs)
    signals = set()
    for (rpc, m), (b, e) in zip(reqs, got):
        assert e is None, e
        assert _normalise(rpc, b) == _python_answer(eng, rpc, m), (rpc, m)
        if rpc == 3:
            from igaming_platform_amd.proto import risk_v1 as P
            signals.update(P.CheckBonusAbuseResponse.FromString(b).signals)
    # the comparison covered the rule signals, shared devices and (with a model) the GRU
    assert {"BONUS_ONLY_PLAYER", "SHARED_DEVICE", "LOW_WAGER_COMPLETION"} <= signals
    st = eng.acct.router.stats(1)
    assert st["items"] == 2 * len(ids) and st["steps"] >= 1
    eng.close()


def test_native_account_rpc_errors():
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.risk_engine import RiskEngine
    from igaming_platform_amd.proto import risk_v1 as P
    eng = RiskEngine(Config(), backend="cpu", capacity=16)
    r = eng.acct.router
    r.submit(1, P.PredictLTVRequest(account_id="").SerializeToString(), 7, 0, NOW)
    r.submit(3, b"\x0a\xff", 8, 0, NOW)  # truncated length-delimited field
    got = {}
    t_end = time.time() + 5
    while len(got) < 2 and time.time() < t_end:
        for tag, b, e in r.poll(16, 50000):
            got[int(tag)] = e
    assert got[7] == "invalid: account_id is required"
    assert got[8].startswith("pb: ")
    eng.close()


def test_native_grpc_serves_account_rpcs_hot():
    """Through the native HTTP/2 server: the three RPCs go to the router (hot_acct), answers equal
    the Python servicer, an empty account id is INVALID_ARGUMENT."""
    import grpc
    from igaming_platform_amd.api.native_grpc import NativeRiskServer
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.risk_engine import RiskEngine
    from igaming_platform_amd.proto import risk_v1 as P
    eng = RiskEngine(Config(), backend="cpu", capacity=64)
    ids = _populate(eng)
    srv = NativeRiskServer(eng, port=0).start()
    try:
        ch = grpc.insecure_channel(f"127.0.0.1:{srv.port}")
        calls = {1: ("PredictLTV", P.PredictLTVResponse), 2: ("GetPlayerSegment", P.GetPlayerSegmentResponse),
                 3: ("CheckBonusAbuse", P.CheckBonusAbuseResponse)}
        for rpc, m in _requests(ids[:8] + ["nobody"]):
            name, resp = calls[rpc]
            f = ch.unary_unary(f"/risk.v1.RiskService/{name}", request_serializer=lambda x: x.SerializeToString(),
                               response_deserializer=resp.FromString)
            got = f(m, timeout=10)
            if rpc == 1:
                got.ClearField("predicted_at")
            assert got.SerializeToString() == _python_answer(eng, rpc, m, now=int(time.time()))
        f = ch.unary_unary("/risk.v1.RiskService/PredictLTV", request_serializer=lambda x: x.SerializeToString(),
                           response_deserializer=P.PredictLTVResponse.FromString)
        with pytest.raises(grpc.RpcError) as ei:
            f(P.PredictLTVRequest(account_id=""), timeout=10)
        assert ei.value.code() == grpc.StatusCode.INVALID_ARGUMENT
        assert "account_id is required" in ei.value.details()
        st = srv.stats()
        assert st["hot_acct"] == 28 and st["hot_failures"] == 0
        ch.close()
    finally:
        srv.stop()
        eng.close()


def test_failed_hot_call_is_retried_through_the_cold_table():
    """a hot call the native core fails (here a model device whose executor
    throws) is answered by the cold handler table, which sees the path with '#retry:<error>'."""
    import grpc
    from igaming_platform_amd.native import native
    from igaming_platform_amd.onnx import builders
    from igaming_platform_amd.proto import risk_v1 as P
    N = native()
    idx = N.AccountIndex(64)
    idx.lookup(["a"], True)
    rows = np.zeros((64, 25), np.float32)
    present = np.ones(64, np.uint8)
    bad = N.Executor(N.OnnxModel.from_bytes(builders.build("ltv_mlp", n_features=64, width=64, layers=2)
                                            .SerializeToString()))
    dev = N.CpuLtvDevice(rows, present, None, bad, in_name="not-the-input", width=64, depth=2, cap=64)
    router = N.AcctRouter([idx])
    router.attach(dev)
    seen = []

    def cold(path, body):
        seen.append(path)
        return P.PredictLTVResponse(account_id="from-cold").SerializeToString()
    srv = N.GrpcServer(None, cold, 2, 0, acct=router)
    port = srv.start("127.0.0.1", 0, 1)
    try:
        ch = grpc.insecure_channel(f"127.0.0.1:{port}")
        f = ch.unary_unary("/risk.v1.RiskService/PredictLTV", request_serializer=lambda x: x.SerializeToString(),
                           response_deserializer=P.PredictLTVResponse.FromString)
        assert f(P.PredictLTVRequest(account_id="a"), timeout=10).account_id == "from-cold"
        assert len(seen) == 1 and seen[0].startswith("/risk.v1.RiskService/PredictLTV#retry:")
        assert "missing input" in seen[0]
        st = srv.stats()
        assert st["hot_acct"] == 1 and st["hot_failures"] == 1 and "missing input" in srv.last_failure()
        ch.close()
    finally:
        srv.stop()
        router.stop()


def test_mailbox_routes_accounts_to_their_owner_rank():
    """Two routers of one node (ranks 0 and 1, one process here): calls for accounts the other
    rank owns travel over the /dev/shm mailbox and come back with the owner's answer; a call to a
    dead owner fails after the remote deadline instead of hanging."""
    from igaming_platform_amd.engine.serving import shm_token
    from igaming_platform_amd.native import native
    from igaming_platform_amd.proto import risk_v1 as P
    from igaming_platform_amd.utils.hashing import SEED_ACCOUNT, id_hash
    N = native()
    name = shm_token() + "-mb"
    idx = [N.AccountIndex(64), N.AccountIndex(64)]
    ids = [f"acct-{i}" for i in range(24)]
    owners = [id_hash(a, SEED_ACCOUNT) % 2 for a in ids]
    assert 0 < sum(owners) < len(ids)
    tabs = []
    for o in range(2):
        mine = [a for a, w in zip(ids, owners) if w == o]
        slots, _ = idx[o].lookup(mine, True)
        rows = np.zeros((64, 25), np.float32)
        present = np.zeros(64, np.uint8)
        for s, a in zip(slots, mine):
            rows[s] = np.arange(25) + int(a.split("-")[1])  # a distinct profile per account
            present[s] = 1
        tabs.append((rows, present))
    r0 = N.AcctRouter(idx, 0, name, True)
    r1 = N.AcctRouter(idx, 1, name, False)
    r0.unlink_shared()
    devs = []
    try:
        for r, (rows, present) in zip((r0, r1), tabs):
            d = N.CpuLtvDevice(rows, present, None, None, depth=2, cap=64)
            devs.append(d)
            r.attach(d)
        reqs = [(1, P.PredictLTVRequest(account_id=a)) for a in ids]
        a0 = _ask(r0, reqs)
        a1 = _ask(r1, reqs)
        assert all(e is None for _, e in a0 + a1)
        assert [_normalise(1, b) for b, _ in a0] == [_normalise(1, b) for b, _ in a1]
        assert r0.remote_out == sum(owners) and r1.remote_out == len(ids) - sum(owners)
        # the answers come from the owners' profiles, not an empty row (whose LTV is 0)
        ltv = [P.PredictLTVResponse.FromString(b).predicted_ltv for b, _ in a0]
        assert all(v > 0 for v in ltv)
        r1.stop()  # the owner of rank 1's accounts is gone: rank 0's calls expire
        r0.remote_timeout_us = 200_000
        remote = [m for m, w in zip(reqs, owners) if w == 1][:2]
        out = _ask(r0, remote, timeout=5)
        assert all(b is None and "did not answer" in e for b, e in out)
        assert r0.remote_expired == 2
    finally:
        r0.stop()
        r1.stop()


def test_owner_without_core_and_oversize_replies_take_the_cold_path():
    """a call whose owner has no model core of that kind, or whose answer does not fit
    one mailbox record (CheckBonusAbuse with 15 linked ids of 150 bytes), comes back to the
    ingress as an error marked ``cold: `` - the native gRPC server then answers it through its
    cold (Python) path WITHOUT failing the shard over - never as a truncated response marked OK."""
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.acct import cpu_abuse_device
    from igaming_platform_amd.engine.risk_engine import RiskEngine
    from igaming_platform_amd.engine.serving import shm_token
    from igaming_platform_amd.native import native
    from igaming_platform_amd.proto import risk_v1 as P
    from igaming_platform_amd.utils.hashing import SEED_ACCOUNT, id_hash
    N = native()
    eng = RiskEngine(Config(), backend="cpu", capacity=256)   # rank 1's shard: its CPU scorer + index
    idx = [N.AccountIndex(256), eng.registry.index[0]]
    name = shm_token() + "-mb"
    r0 = N.AcctRouter(idx, 0, name, True)
    r1 = N.AcctRouter(idx, 1, name, False)
    r0.unlink_shared()
    try:
        r1.attach(cpu_abuse_device(eng.backends[0], None, 64))   # rank 1: abuse core only, no LTV core
        short = next(a for a in (f"short-{i}" for i in range(100)) if id_hash(a, SEED_ACCOUNT) % 2 == 1)
        longs = [("L%03d-" % i) + "x" * 145 for i in range(15)]
        keys = []
        for a in [short] + longs:
            o = id_hash(a, SEED_ACCOUNT) % 2
            sl, _ = idx[o].lookup([a], True)
            keys.append((o << 32) | int(sl[0]))
        L = N.LinkIndex(16)
        L.add(np.full(len(keys), 777, np.uint64), np.array(keys, np.int64))   # one shared device
        r1.set_links(L)
        # PredictLTV for an account of rank 1 asked on rank 0: no LTV core on the owner
        (b, e), = _ask(r0, [(N.RPC_LTV, P.PredictLTVRequest(account_id=short))])
        assert b is None and e.startswith("cold: ") and "no native model core" in e
        # CheckBonusAbuse: asked on the owner the answer is whole (15 linked ids, ~2.3 KB) ...
        ask = [(N.RPC_ABUSE, P.CheckBonusAbuseRequest(account_id=short, bonus_id="b"))]
        (b1, e1), = _ask(r1, ask)
        assert e1 is None and len(b1) > 2032
        assert sorted(P.CheckBonusAbuseResponse.FromString(b1).linked_accounts) == sorted(longs)
        # ... asked on rank 0 it does not fit a reply record: marked cold, never truncated
        (b0, e0), = _ask(r0, ask)
        assert b0 is None and e0.startswith("cold: ") and "exceeds the mailbox record" in e0
        assert r1.reply_oversize == 1
    finally:
        r0.stop()
        r1.stop()
        eng.close()


# ----------------------------------------------------------------------------- multi-process
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spmd_worker(rank, world, port, q, barrier, lm, am):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.risk_engine import RiskEngine, serve_shard
    from igaming_platform_amd.parallel.comm import TorchComm
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = TorchComm("gloo")
    try:
        if rank == 0:
            eng = RiskEngine(Config(), backend="cpu", capacity=128, spmd=comm, ltv_model=lm, abuse_model=am)
            ids = _populate(eng)
            barrier.wait(120)           # state loaded: every rank asks
            got = _ask(eng.acct.router, _requests(ids))
            barrier.wait(120)
            py = [_python_answer(eng, rpc, m) for rpc, m in _requests(ids)]  # the SPMD Python path (cold ops)
            eng.close()
            q.put(("ok", 0, got, py))
        else:
            out = {}

            def ingress(node):  # this rank's own calls through its router, after rank 0 loaded state
                barrier.wait(120)
                ids = [f"acc-{i}" for i in range(30)] + ["nobody", "ghost-1"]
                out["got"] = _ask(node.acct.router, _requests(ids))
                barrier.wait(120)
            serve_shard(Config(), comm, backend="cpu", capacity=128, ingress=ingress, ltv_model=lm, abuse_model=am)
            q.put(("ok", rank, out["got"], None))
    except Exception:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put(("err", traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.dist
@pytest.mark.parametrize("world", [2, 3])
def test_every_rank_serves_account_rpcs_owner_routed(world):
    """gloo world 2/3 (CPU shards): every rank answers PredictLTV / GetPlayerSegment /
    CheckBonusAbuse for every account through its own native router (the owner's model device,
    reached over the /dev/shm mailbox for other ranks' accounts); all answers equal a
    single-process engine, and the SPMD Python path (cold ops) agrees as well."""
    import torch.multiprocessing as mp
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.risk_engine import RiskEngine
    from igaming_platform_amd.onnx import builders
    lm = builders.build("ltv_mlp", n_features=64, width=64, layers=2).SerializeToString()
    am = builders.build("gru", seq=100, hidden=64, layers=2).SerializeToString()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    barrier = ctx.Barrier(world)
    port = _free_port()
    procs = [ctx.Process(target=_spmd_worker, args=(r, world, port, q, barrier, lm, am)) for r in range(world)]
    [p.start() for p in procs]
    msgs = [q.get(timeout=300) for _ in range(world)]
    [p.join(timeout=60) for p in procs]
    errs = [m[1] for m in msgs if m[0] == "err"]
    assert not errs, errs[0]
    ref = RiskEngine(Config(), backend="cpu", capacity=128, ltv_model=lm, abuse_model=am)
    ids = _populate(ref)
    reqs = _requests(ids)
    want = [_python_answer(ref, rpc, m) for rpc, m in reqs]
    for m in msgs:
        got = [_normalise(rpc, b) for (rpc, _), (b, e) in zip(reqs, m[2])]
        assert all(e is None for _, e in m[2])
        assert got == want, f"rank {m[1]} answers differ"
        if m[3] is not None:
            assert m[3] == want  # rank 0's SPMD Python path (OP_LTV / OP_ABUSE / OP_FEATMANY)
    ref.close()


def test_router_pause_holds_new_steps_until_resume():
    """AcctRouter.pause (used by a config refresh: the devices' config blocks are rewritten with
    no step in flight) holds every new device step; resume releases them, nothing is lost."""
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.risk_engine import RiskEngine
    from igaming_platform_amd.onnx import builders
    lm = builders.build("ltv_mlp", n_features=64, width=64, layers=2).SerializeToString()
    eng = RiskEngine(Config(), backend="cpu", capacity=256, ltv_model=lm)
    ids = _populate(eng)
    reqs = [x for x in _requests(ids) if x[0] == 1][:8]
    r = eng.acct.router
    r.pause()
    for i, (rpc, m) in enumerate(reqs):
        r.submit(rpc, m.SerializeToString(), i, 0, NOW)
    assert r.poll(64, 200000) == []            # held: no step issued while paused
    r.resume()
    got = {}
    t_end = time.time() + 20
    while len(got) < len(reqs) and time.time() < t_end:
        for tag, b, e in r.poll(64, 50000):
            got[int(tag)] = (b, e)
    assert sorted(got) == list(range(len(reqs))) and all(e is None for _, e in got.values())
    eng.acct.refresh()                          # pause / refresh / resume round trip
    assert len(_ask(r, reqs)) == len(reqs)
    eng.close()

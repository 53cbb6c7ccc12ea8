"""T5 on the GPU: the owner-routed RCCL exchange (csrc/kernels/exchange.hip, engine/dp.py)
through RCCL's single-rank path on one MI355X. The exchange scorer must give bit-identical
results, features and feature-store state to the plain single-GPU pipeline, and the SPMD
serving engine (world 1) must answer exactly like the plain GPU engine."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
NOW = 1_760_000_000


def _setup(width=128, n_acc=2048, seed=0):
    import torch
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.features.device_store import DeviceFeatureStore
    from igaming_platform_amd.models.plan import compile_onnx, to_device
    from igaming_platform_amd.native import native
    from igaming_platform_amd.onnx import builders
    from igaming_platform_amd.utils.synth import make_population
    dev = torch.device("cuda", 0)
    cfg = Config()
    cfg.features.width = width
    cfg.gpu.buckets = [64, 256]
    pop = make_population(n_acc, width - 30, seed=seed, fast_hash=True)
    m = native().OnnxModel.from_bytes(builders.stacked(n_trees=30).SerializeToString())

    def store():
        s = DeviceFeatureStore(n_acc, cfg.features, dev, max_events=256)
        s.set_batch_features(np.arange(n_acc), pop.batch)
        s.set_ext(np.arange(n_acc), pop.ext)
        for i in range(20):
            s.blacklist.add("device", f"bad-{i}")
        s.sync_tables()
        return s

    return cfg, pop, store, to_device(compile_onnx(m), dev), dev


def test_exchange_scorer_matches_plain_pipeline():
    import torch
    from igaming_platform_amd.engine.dp import DpGpuScorer
    from igaming_platform_amd.engine.scorer import GpuScorer
    from igaming_platform_amd.parallel.exchange import rccl_comms
    from igaming_platform_amd.utils.synth import make_requests
    cfg, pop, mk_store, plan, dev = _setup()
    s_ref, s_dp = mk_store(), mk_store()
    ref = GpuScorer(cfg, s_ref, plan=plan, model="plan", device=dev, pipeline_depth=3)
    ref.capture()
    dp = DpGpuScorer(cfg, s_dp, rccl_comms(0, 1), world=1, rank=0, senders=1, cbuckets=[64, 256], plan=plan,
                     model="plan", device=dev, pipeline_depth=3)
    dp.capture()
    rng = np.random.default_rng(5)
    for step in range(12):  # > 3 batches in flight: slot reuse and dedup-region rotation
        n = int(rng.choice([1, 40, 64, 200, 256]))
        req = make_requests(pop, n, rng, NOW + step, hot_frac=0.3, unknown_frac=0.02)
        wf = bool(step % 2)
        want, want_f = ref.wait(ref.submit(req, now=NOW + step, want_features=wf), unpack=False)
        p = dp.submit_rows(dp.next_slot(), req, np.zeros(n, np.int64), NOW + step, want_features=wf)
        res, feats = dp.wait_x(p)
        assert p.C == (64 if n <= 64 else 256)
        np.testing.assert_array_equal(np.ascontiguousarray(res).view(np.int32).reshape(-1, 2), want)
        if wf:
            np.testing.assert_array_equal(np.ascontiguousarray(feats).view(np.int32).reshape(-1, 32), want_f)
        assert dp.route_overflow(p.slot, p.C) == 0
    torch.cuda.synchronize(dev)
    for k in ("ring_ts", "ring_amt", "hll", "rt"):  # identical score-then-update state
        assert torch.equal(getattr(s_ref, k), getattr(s_dp, k)), k
    # device metrics count exactly the rows this GPU scored
    m_ref, m_dp = ref.read_metrics(), dp.read_metrics()
    np.testing.assert_array_equal(m_ref, m_dp)
    # ordered teardown: graphs holding communicator references first, then ncclCommDestroy
    dp.close()
    assert not any(c.alive for c in dp.comms)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init_pg(backend, **kw):
    """init_process_group on a fresh local port; a port handed out by the kernel can be taken
    again before the store binds it (EADDRINUSE): then another one."""
    import torch.distributed as dist
    for attempt in range(5):
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
        try:
            dist.init_process_group(backend, rank=0, world_size=1, **kw)
            return
        except dist.DistNetworkError:
            if attempt == 4:
                raise


@pytest.mark.parametrize("results,rows", [("a2a", "rccl"), ("d2h", "rccl"), ("d2h", "shm")])
def test_spmd_engine_world1_matches_plain_gpu_engine(monkeypatch, results, rows):
    """The SPMD serving engine at world 1 (its native core driving the exchange pipeline)
    answers exactly like the plain GPU engine, with the results returning through the result
    all-to-all or through the per-GPU D2H copies into the node-shared region (IGP_XCHG_RESULTS),
    and the rows reaching their owner through the RCCL row all-to-all or the node-shared rows
    region (IGP_XCHG_ROWS; shm: no communicator at all)."""
    import torch
    import torch.distributed as dist
    monkeypatch.setenv("IGP_XCHG_RESULTS", results)
    monkeypatch.setenv("IGP_XCHG_ROWS", rows)
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.risk_engine import RiskEngine
    from igaming_platform_amd.parallel.comm import TorchComm
    _init_pg("nccl", device_id=torch.device("cuda", 0))
    spmd = plain = None
    try:
        cfg = Config()
        cfg.gpu.buckets = [64, 256]
        spmd = RiskEngine(cfg, backend="gpu", capacity=1024, spmd=TorchComm("nccl", "cuda:0"))
        plain = RiskEngine(cfg, backend="gpu", capacity=1024)
        assert spmd.local.scorer.__class__.__name__ == "DpGpuScorer"
        assert (spmd.local.scorer.rshm is not None) == (results == "d2h")
        assert spmd.local.scorer.stage_ops  # state (+ d2h: model) stages as recorded launches
        assert spmd.local.scorer.rows_shm == (rows == "shm")
        assert len(spmd.local.scorer.comms) == (0 if rows == "shm" else 2)
        if results == "d2h":
            assert not os.path.exists(spmd.local.scorer.rshm["path"])  # unlinked once every rank mapped it
        rng = np.random.default_rng(2)
        types = ["deposit", "withdraw", "bet", "win"]
        for e in (spmd, plain):
            e.add_to_blacklist("device", "dev-3", "x", "t")
        for step in range(4):
            txs = [dict(account_id=f"acc-{int(a)}", amount=int(rng.choice([500, 150000, 2_000_000])),
                        transaction_type=types[int(rng.integers(0, 4))], device_id=f"dev-{int(a) % 7}",
                        ip_address=f"10.0.{int(a)}.1") for a in rng.integers(0, 60, 150)]
            a, b = spmd.score(txs, now=NOW + step), plain.score(txs, now=NOW + step)
            for x, y in zip(a, b):
                assert (x["score"], x["action"], x["reason_codes"], x["rule_score"], x["ml_score"]) == \
                       (y["score"], y["action"], y["reason_codes"], y["rule_score"], y["ml_score"])
                assert x["features"].tobytes() == y["features"].tobytes()
        assert spmd.group.runner.rows_scored == 600
    finally:
        for e in (spmd, plain):
            if e is not None:
                e.close()
        dist.destroy_process_group()


def test_spmd_engines_close_and_destroy_their_communicators(monkeypatch):
    """two SPMD world-1 engines created and closed one after the other in one
    process. Each close stops the serving core, destroys the exchange graphs (RCCL keeps a
    reference on a communicator per graph that captured its collectives) and then both RCCL
    communicators; the second engine's set-up, scoring and teardown then run in a process with
    no communicator left over from the first."""
    import torch
    import torch.distributed as dist
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.risk_engine import RiskEngine
    from igaming_platform_amd.parallel.comm import TorchComm
    monkeypatch.setenv("IGP_XCHG_ROWS", "rccl")  # the communicator lifecycle (rows region: none)
    for round_ in range(2):
        _init_pg("gloo")
        eng = None
        try:
            cfg = Config()
            cfg.gpu.buckets = [64, 256]
            eng = RiskEngine(cfg, backend="gpu", capacity=1024, spmd=TorchComm("gloo"))
            sc = eng.local.scorer
            assert sc.__class__.__name__ == "DpGpuScorer" and all(c.alive for c in sc.comms)
            rng = np.random.default_rng(round_)
            txs = [dict(account_id=f"acc-{int(a)}", amount=5000, transaction_type="bet", device_id=f"d-{int(a)}",
                        ip_address="10.0.0.1") for a in rng.integers(0, 60, 200)]
            out = eng.score(txs, now=NOW + round_)
            assert len(out) == 200
            comms = list(sc.comms)
            eng.close()
            eng = None
            assert not any(c.alive for c in comms), round_
            assert not sc.xgraphs
        finally:
            if eng is not None:
                eng.close()
            dist.destroy_process_group()
        torch.cuda.synchronize()


@pytest.mark.parametrize("world,C", [(2, 64), (3, 40), (8, 16)])
def test_exchange_kernels_multi_sender_layout(world, C):
    """exchange_compact / exchange_scatter on a receive buffer holding several senders' chunks
    (the N > 1 layout RCCL delivers) against their host twins (parallel/exchange.py)."""
    import torch
    from igaming_platform_amd.layouts import FEATREC, REQREC
    from igaming_platform_amd.native import hipk
    from igaming_platform_amd.parallel.exchange import build_chunks, compact, scatter_results
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(world)
    recv = np.zeros(world * (C + 1), REQREC)
    for p in range(world):  # chunk p = what sender p routed to this rank
        n = int(rng.integers(0, C + 1))
        rows = np.zeros(n, REQREC)
        rows["slot"] = rng.integers(0, 1000, n)
        rows["tx_type"] = rng.integers(0, 4, n) | (p << 8)
        rows["amount"] = rng.integers(1, 10**6, n)
        rows["dev_hash"] = rng.integers(1, 2**62, n)
        recv[p * (C + 1):(p + 1) * (C + 1)] = build_chunks(rows, np.zeros(n, np.int64), 1, C)[0]
    cap = world * C
    d_recv = torch.from_numpy(recv.view(np.uint8).copy()).to(dev)
    slab = torch.zeros(16 + 48 * cap, dtype=torch.uint8, device=dev)
    route = torch.full((cap + 1,), -7, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    hipk().exchange_compact(d_recv.data_ptr(), slab.data_ptr() + 16, slab.data_ptr(), route.data_ptr(), world, C, cap, s)
    torch.cuda.synchronize()
    rows_ref, route_ref = compact(recv, world, C)
    n = int(slab[:4].view(torch.int32).item())
    assert n == len(rows_ref)
    got = slab[16:16 + 48 * n].cpu().numpy().view(REQREC)
    np.testing.assert_array_equal(got.view(np.uint8), rows_ref.view(np.uint8))
    np.testing.assert_array_equal(route[:n].cpu().numpy(), route_ref)
    assert int(route[cap].item()) == 0
    # scatter: result + feature rows of the compact rows back into per-sender chunks
    res = rng.integers(0, 2**31, (cap, 2)).astype(np.int32)
    feats = rng.integers(0, 2**31, (cap, 32)).astype(np.int32)
    send = torch.zeros(world * C * 136, dtype=torch.uint8, device=dev)
    d_res, d_feat = torch.from_numpy(res).to(dev), torch.from_numpy(feats).to(dev)
    hipk().exchange_scatter(slab.data_ptr(), route.data_ptr(), d_res.data_ptr(), d_feat.data_ptr(), send.data_ptr(),
                            C, cap, s)
    torch.cuda.synchronize()
    want = scatter_results(res[:n].view(np.uint32), feats[:n].copy().view(FEATREC).reshape(-1), route_ref, world, C)
    got = send.cpu().numpy().reshape(world, C * 136)
    mask = scatter_results(np.ones((n, 2), np.uint32), np.ones(n, FEATREC), route_ref, world, C) != 0
    np.testing.assert_array_equal(got[mask], want[mask])


@pytest.mark.parametrize("world,C", [(1, 64), (3, 40), (8, 16)])
def test_exchange_compact_from_the_node_shared_rows_region(world, C):
    """The rows-region copy stage: exchange_compact reading this owner's chunk of every sender's
    block straight from page-locked host memory ([sender][owner][C + 1], sender stride
    world * (C + 1)) and copying the batch header along equals the host twin over the chunks
    this owner would have received from the all-to-all."""
    import torch
    from igaming_platform_amd.layouts import REQREC
    from igaming_platform_amd.native import hipk
    from igaming_platform_amd.parallel.exchange import build_chunks, compact
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(100 + world)
    me = world - 1
    region = torch.zeros(world * world * (C + 1) * 48, dtype=torch.uint8).pin_memory()
    blocks = region.numpy().view(REQREC).reshape(world, world * (C + 1))
    for p in range(world):  # sender p's block: its chunks for every owner (<= C rows each)
        owners = np.repeat(np.arange(world), rng.integers(0, C + 1, world))
        rng.shuffle(owners)
        n = len(owners)
        rows = np.zeros(n, REQREC)
        rows["slot"] = rng.integers(0, 1000, n)
        rows["tx_type"] = rng.integers(0, 4, n) | (p << 8)
        rows["amount"] = rng.integers(1, 10**6, n)
        rows["ts"] = NOW + p
        blocks[p] = build_chunks(rows, owners, world, C)[0]
    recv = np.concatenate([blocks[p, me * (C + 1):(me + 1) * (C + 1)] for p in range(world)])
    cap = world * C
    slab = torch.zeros(16 + 48 * cap, dtype=torch.uint8, device=dev)
    route = torch.full((cap + 1,), -7, dtype=torch.int32, device=dev)
    hdr = torch.tensor([0, 4242, NOW & 0xFFFFFFFF, NOW >> 32], dtype=torch.int32).pin_memory()
    first = region.data_ptr() + me * (C + 1) * 48
    hipk().exchange_compact(first, slab.data_ptr() + 16, slab.data_ptr(), route.data_ptr(), world, C, cap,
                            torch.cuda.current_stream().cuda_stream, world * (C + 1), hdr.data_ptr())
    torch.cuda.synchronize()
    rows_ref, route_ref = compact(recv, world, C)
    n = int(slab[:4].view(torch.int32).item())
    assert n == len(rows_ref) and int(slab[4:8].view(torch.int32).item()) == 4242
    got = slab[16:16 + 48 * n].cpu().numpy().view(REQREC)
    np.testing.assert_array_equal(got.view(np.uint8), rows_ref.view(np.uint8))
    np.testing.assert_array_equal(route[:n].cpu().numpy(), route_ref)
    # the serving copy stage: the dedup insert compacts the same chunks itself (one kernel)
    from igaming_platform_amd.engine.scorer import GpuScorer
    from igaming_platform_amd.ops import kernels as K
    cfg, pop, mk_store, plan, dev = _setup()
    store = mk_store()
    sc = GpuScorer(cfg, store, plan=plan, model="plan", device=dev, pipeline_depth=2)
    slab2 = torch.zeros(16 + 48 * cap, dtype=torch.uint8, device=dev)
    route2 = torch.full((cap + 1,), -7, dtype=torch.int32, device=dev)
    K.dedup_insert(store, sc.cfg_dev, slab2[16:], cap, slab2[:16].view(torch.int64),
                   xsrc=dict(recv=first, pstride=world * (C + 1), N=world, C=C, route=route2, hdr=hdr.data_ptr()))
    torch.cuda.synchronize()
    assert int(slab2[:4].view(torch.int32).item()) == n and int(slab2[4:8].view(torch.int32).item()) == 4242
    np.testing.assert_array_equal(slab2[16:16 + 48 * n].cpu().numpy(), got.view(np.uint8))
    np.testing.assert_array_equal(route2[:n].cpu().numpy(), route_ref)
    assert int(route2[cap].item()) == 0


def test_exchange_rank_fits_the_hardware_queue_budget():
    """one exchange rank runs on at most GPU_MAX_HW_QUEUES (4) distinct
    streams, default stream included, and owns exactly two communicators (the exchange's rows
    and results RcclComms); no torch NCCL process group is created (engine/dp.py stream map)."""
    import torch
    import torch.distributed as dist
    from igaming_platform_amd.engine import dp as DP
    from igaming_platform_amd.parallel.exchange import rccl_comms
    cfg, pop, mk_store, plan, dev = _setup()
    sc = DP.DpGpuScorer(cfg, mk_store(), rccl_comms(0, 1), world=1, rank=0, senders=1, cbuckets=[64, 256],
                        plan=plan, model="plan", device=dev, pipeline_depth=3)
    sc.capture()
    m = sc.stream_map()
    assert len(set(m.values())) == len(set(DP.stream_roles().values())) <= DP.HW_QUEUES == 4
    assert m["rows_a2a"] == m["h2d"] and m["results_a2a"] == m["model"]  # the collectives share streams
    assert len(sc.comms) == DP.EXCHANGE_COMMUNICATORS == 2
    assert not dist.is_initialized() or dist.get_backend() != "nccl"


def test_exchange_world1_same_accounts_in_one_step_follow_fifo_order():
    """The ordering contract on the GPU exchange (engine/dp.py) at world 1: two ScoreBatch
    requests over the same accounts queued into ONE exchange step are applied in FIFO (then row)
    order and scored against the pre-step state - equal to a plain GPU engine scoring their
    concatenation as one batch; the next step sees both."""
    import threading
    import time
    import torch
    import torch.distributed as dist
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.risk_engine import RiskEngine
    from igaming_platform_amd.parallel.comm import TorchComm
    from igaming_platform_amd.proto import risk_v1 as P
    _init_pg("nccl", device_id=torch.device("cuda", 0))
    spmd = plain = None
    try:
        cfg = Config()
        cfg.gpu.buckets = [64, 256]
        spmd = RiskEngine(cfg, backend="gpu", capacity=1024, spmd=TorchComm("nccl", "cuda:0"))
        plain = RiskEngine(cfg, backend="gpu", capacity=1024)
        rng = np.random.default_rng(4)
        types = ["deposit", "withdraw", "bet", "win"]

        def payload(n):
            return P.ScoreBatchRequest(transactions=[
                P.ScoreTransactionRequest(account_id=f"same-{int(a)}", amount=int(rng.choice([500, 150000, 2_000_000])),
                                          transaction_type=types[int(rng.integers(0, 4))],
                                          device_id=f"dv-{int(rng.integers(0, 9))}", ip_address=f"10.7.{int(a)}.1")
                for a in rng.integers(0, 6, n)]).SerializeToString()

        def decode(b):
            out = []
            for x in P.ScoreBatchResponse.FromString(b).results:
                x.response_time_ms = 0
                out.append(x.SerializeToString())
            return out
        core = spmd.core
        for rnd in range(3):
            reqs = [payload(40), payload(25)]
            now = NOW + 30 * rnd
            got, seqs = [None, None], [None, None]

            def call(i):
                got[i] = decode(core.score_batch(reqs[i], now, 0))
                seqs[i] = type(core).last_timings()[7]
            core.pause()
            th = []
            for i in range(2):  # queued in this order, both before the step is formed
                th.append(threading.Thread(target=call, args=(i,)))
                th[-1].start()
                while core.pending_items() < i + 1:
                    time.sleep(0.001)
            core.resume()
            [t.join() for t in th]
            assert seqs[0] == seqs[1]  # one exchange step
            txs = [t for r in reqs for t in P.ScoreBatchRequest.FromString(r).transactions]
            want = decode(plain.score_batch_bytes(P.ScoreBatchRequest(transactions=txs).SerializeToString(), now=now))
            assert got[0] + got[1] == want
    finally:
        # the engines stop their exchange / cores before the process group goes away, also when
        # an assertion failed (destroying the group under a running exchange aborts the process)
        for e in (spmd, plain):
            if e is not None:
                e.close()
        dist.destroy_process_group()


def test_two_rank_processes_serve_through_the_node_shared_exchange():
    """The multi-rank serving path on real GPU processes: ``bench.py --gpus 2`` under
    torch.distributed.run with both ranks on this box's one GPU (bench.py gpu_index: the
    node-shared rows / results regions open no RCCL communicator, so two ranks may share a
    device). Every rank ingests requests spread over both owners; the run must finish with both
    ranks answering, the rows-region mode named in the line and the exchange waits accounted."""
    import json
    import subprocess
    import sys
    import tempfile
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "w2.json")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
               "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
               "--steps", "2", "--warmup", "1", "--threads", "4", "--rounds", "4", "--accounts", "65536",
               "--json-out", out]
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        r = subprocess.run(cmd, cwd=root, env=env, timeout=110, capture_output=True, text=True)
        assert r.returncode == 0, r.stdout[-1500:] + r.stderr[-3000:]
        with open(out) as f:
            d = json.load(f)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["value"] > 0
    assert "node-shared pinned rows region" in d["config"]["serving"]
    w = d["exchange_waits_us_rank0"]
    assert w["submits"] > 0 and w["owner_wait_max_us"] >= 0

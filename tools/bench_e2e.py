#!/usr/bin/env python3
"""End-to-end scoring benches (VERDICT r1 "put the real request path in the timed region"):

``--scope e2e``  raw ``ScoreBatchRequest`` bytes -> C++ wire parse -> AccountIndex lookup of the
                 UUID account-id strings -> ReqRec pack -> GPU pipeline -> C++ response
                 serialisation (FeatureVector per row included), in-process, T caller threads
                 (``RiskEngine.score_batch_bytes``: what the ScoreBatch handler runs).
``--scope grpc`` the same server behind ``grpc.aio`` on 127.0.0.1: client processes send raw
                 ``ScoreBatch`` payloads, or unary ``ScoreTransaction`` calls that the
                 micro-batcher merges into device batches (``--rpc tx``).

Synthetic data: UUID account ids with warehouse batch features and 98 extended features loaded
through the engine's own loaders; random-init cfg3 weights (GBDT 100 x d7 -> MLP 32-256-1).
Prints one JSON line with "scope", throughput and p50/p99 latency (client-measured for grpc)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
import uuid

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BASELINE_P99_MS = 50.0  # README.md:58
TYPES = ["deposit", "withdraw", "bet", "win"]


def account_id(i: int) -> str:
    return str(uuid.UUID(int=(i * 0x9E3779B97F4A7C15 + 0x632BE59BD9B4E019) & ((1 << 128) - 1), version=4))


def make_payloads(n_accounts: int, n_payloads: int, batch: int, seed: int):
    """Serialized ScoreBatchRequest messages of ``batch`` transactions each."""
    from igaming_platform_amd.proto import risk_v1 as P
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n_payloads):
        acc = rng.integers(0, n_accounts, batch)
        amt = np.maximum(1, rng.lognormal(7.5, 1.6, batch)).astype(np.int64)
        typ = rng.choice(4, batch, p=[0.25, 0.1, 0.55, 0.1])
        dev = rng.integers(0, 6, batch)
        req = P.ScoreBatchRequest(transactions=[
            P.ScoreTransactionRequest(account_id=account_id(int(a)), amount=int(m), transaction_type=TYPES[int(t)],
                                      currency="EUR", device_id=f"dev-{int(a)}-{int(d)}",
                                      ip_address=f"10.{int(a) % 250}.{int(a) // 250 % 250}.{int(d)}",
                                      fingerprint=f"fp-{int(a)}-{int(d)}", session_id=f"s-{int(a)}")
            for a, m, t, d in zip(acc, amt, typ, dev)])
        out.append(req.SerializeToString())
    return out


def _varint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _field(num: int, data: bytes) -> bytes:
    return _varint(num << 3 | 2) + _varint(len(data)) + data


def spread_payloads(n_accounts: int, n_payloads: int, batch: int, seed: int, zipf: float = 0.0, stats=None):
    """ScoreBatchRequest bytes whose accounts cover the population: uniform account ids, or
    Zipf(``zipf``)-distributed ranks (``zipf`` > 1). Encoded directly (byte-identical to the
    protobuf serializer's output for these fields), so 128+ requests of 8192 transactions build in
    seconds. Same field set as :func:`make_payloads`."""
    rng = np.random.default_rng(seed)
    cur = _field(5, b"EUR")
    types = [_field(4, t.encode()) for t in TYPES]
    out = []
    seen = []
    for _ in range(n_payloads):
        acc = ((rng.zipf(zipf, batch) - 1) % n_accounts) if zipf > 1 else rng.integers(0, n_accounts, batch)
        seen.append(acc)
        amt = np.maximum(1, rng.lognormal(7.5, 1.6, batch)).astype(np.int64).tolist()
        typ = rng.choice(4, batch, p=[0.25, 0.1, 0.55, 0.1]).tolist()
        dev = rng.integers(0, 6, batch).tolist()
        parts = []
        for a, m, t, d in zip(acc.tolist(), amt, typ, dev):
            body = b"".join((_field(1, account_id(a).encode()), b"\x18" + _varint(m), types[t], cur,
                             _field(8, f"10.{a % 250}.{a // 250 % 250}.{d}".encode()),
                             _field(9, f"dev-{a}-{d}".encode()), _field(10, f"fp-{a}-{d}".encode()),
                             _field(12, f"s-{a}".encode())))
            parts.append(_field(1, body))
        out.append(b"".join(parts))
    if stats is not None:  # how much of the population the stream touches
        stats["distinct_accounts"] = int(len(np.unique(np.concatenate(seen))))
        stats["transactions"] = n_payloads * batch
    return out


def tx_payloads(n_accounts: int, n: int, seed: int):
    from igaming_platform_amd.proto import risk_v1 as P
    rng = np.random.default_rng(seed)
    return [P.ScoreTransactionRequest(account_id=account_id(int(a)), amount=int(rng.integers(100, 500000)),
                                      transaction_type=TYPES[int(rng.integers(0, 4))], device_id=f"dev-{int(a)}-0",
                                      ip_address="10.0.0.1").SerializeToString()
            for a in rng.integers(0, n_accounts, n)]


# per-column scale of the synthetic 25-column player profile (uniform in [0, scale))
PROFILE_SCALE = np.array([900, 90, 60, 500, 10, 120, 1e5, 8e4, 3e4, 500, 8, 5e3, 2e5, 1.8e5, 3000, 1, 80, 60, 20, 15,
                          1, 1, 1, 1, 8])


def fill_event_rings(store, seed: int = 77) -> None:
    """Full 100-event histories in a GPU shard's HBM event rings (random bf16 events for every
    slot, ring counts full): the GRU runs its 100 steps over real-looking inputs."""
    import torch
    from igaming_platform_amd.layouts import ACCTRT
    g = torch.Generator(device=store.device)
    g.manual_seed(seed)
    cap = store.ev.shape[0]
    for s0 in range(0, cap, 1 << 16):
        n = min(1 << 16, cap - s0)
        ev = torch.randn((n, store.ev.shape[1], store.ev.shape[2]), generator=g, device=store.device)
        store.ev[s0:s0 + n].copy_(ev.to(torch.bfloat16).view(torch.int16))
    rt = store.rt.view(-1, store.rt.shape[1])
    rt[:, ACCTRT.fields["ev_count"][1] // 4] = store.ev.shape[1]
    torch.cuda.synchronize(store.device)


def build_cold_engine(accounts: int, backend: str, precision: str = "fp32"):
    """Engine with the cfg 4 LTV MLP and the cfg 5 abuse GRU loaded, player profiles for every
    account and (GPU) full 100-event histories in the HBM event rings (PredictLTV /
    GetPlayerSegment / CheckBonusAbuse benches). ``precision``: the models' dense numerics
    (fp32 = the ONNX f32 contract: split bf16x3 MFMA; bf16)."""
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.risk_engine import RiskEngine
    from igaming_platform_amd.onnx import builders
    cfg = Config()
    cfg.gpu.buckets = [64, 512, 4096]
    cfg.gpu.max_batch = 4096
    cfg.ltv_model.precision = cfg.abuse_model.precision = precision
    eng = RiskEngine(cfg, backend=backend, capacity=accounts + 1024,
                     ltv_model=builders.build("ltv_mlp", n_features=256, width=512, layers=4).SerializeToString(),
                     abuse_model=builders.build("gru", seq=100, in_dim=16, hidden=256).SerializeToString())
    rng = np.random.default_rng(5)
    ids = [account_id(i) for i in range(accounts)]
    slots, owners = eng.registry.resolve_ids(ids, insert=True)
    step = 1 << 18
    for s0 in range(0, accounts, step):
        n = min(step, accounts - s0)
        rows = np.floor(rng.uniform(0, 1, (n, 25)) * PROFILE_SCALE)
        eng.ltv.set_rows(slots[s0:s0 + n], owners[s0:s0 + n], rows.astype(np.float32),
                         rng.normal(0, 1, (n, 231)).astype(np.float32))
    if backend == "gpu":
        fill_event_rings(eng.backends[0].store)
    return eng


def acct_request(rpc: str, account: str) -> bytes:
    """One PredictLTV / GetPlayerSegment / CheckBonusAbuse request body."""
    from igaming_platform_amd.proto import risk_v1 as P
    m = {"ltv": lambda a: P.PredictLTVRequest(account_id=a),
         "segment": lambda a: P.GetPlayerSegmentRequest(account_id=a),
         "abuse": lambda a: P.CheckBonusAbuseRequest(account_id=a, bonus_id="welcome")}[rpc](account)
    return m.SerializeToString()


def acct_payloads(accounts: int, rpc: str, n: int, seed: int, zipf: float = 0.0):
    """Request bodies of PredictLTV / GetPlayerSegment / CheckBonusAbuse over the population:
    uniform account ids, or Zipf-distributed ranks with exponent ``zipf`` (> 1)."""
    rng = np.random.default_rng(seed)
    acc = (rng.zipf(zipf, n) - 1) % accounts if zipf > 1 else rng.integers(0, accounts, n)
    return [acct_request(rpc, account_id(int(a))) for a in acc]


def run_cold_engine(a) -> dict:
    """The batched engine calls behind the micro-batched cold RPCs, in-process (4096 accounts each)."""
    eng = build_cold_engine(a.accounts, a.backend)
    rng = np.random.default_rng(9)
    fn = eng.predict_ltv_batch if a.rpc == "ltv" else eng.check_bonus_abuse_batch
    batches = [[account_id(int(i)) for i in rng.integers(0, a.accounts, 4096)] for _ in range(4)]
    for i in range(3):
        fn(batches[i % 4])
    lat = []
    t0 = time.perf_counter()
    for i in range(a.steps):
        t = time.perf_counter()
        fn(batches[i % 4])
        lat.append((time.perf_counter() - t) * 1e3)
    el = time.perf_counter() - t0
    eng.close()
    return dict(metric=f"{'PredictLTV' if a.rpc == 'ltv' else 'CheckBonusAbuse'} answers/sec (batched engine call, "
                       f"4096 accounts, in-process)", value=a.steps * 4096 / el, unit="answers/s",
                scope="engine_batched", n_gpus=1 if a.backend == "gpu" else 0, steps=a.steps,
                data="synthetic (UUID ids, random-init cfg4 / cfg5 weights)",
                p50_latency_ms=float(np.percentile(lat, 50)), p99_latency_ms=float(np.percentile(lat, 99)))


FRAUD_MODELS = {"cfg3": ("cfg3 GBDT(100,d7,128f)+MLP(32-256-1)", 128),
                "cfg1": ("cfg1 logistic regression over 32 features (Gemm -> Sigmoid)", 32)}


def fraud_model_bytes(model: str) -> bytes:
    from igaming_platform_amd.onnx import builders
    if model == "cfg1":
        return builders.build("logistic", n_features=32).SerializeToString()
    return builders.build("stacked").SerializeToString()


def build_engine(accounts: int, batch: int, backend: str, model: str = "cfg3"):
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.risk_engine import RiskEngine
    from igaming_platform_amd.layouts import ACCTBATCH
    from igaming_platform_amd.utils.synth import make_population
    cfg = Config()
    cfg.features.width = FRAUD_MODELS[model][1]
    cfg.gpu.buckets = sorted({64, 512, 2048, batch})
    cfg.gpu.max_batch = batch
    eng = RiskEngine(cfg, backend=backend, capacity=accounts + 1024, fraud_model=fraud_model_bytes(model))
    pop = make_population(accounts, 98, seed=3, fast_hash=True)
    ids = [account_id(i) for i in range(accounts)]
    step = 1 << 18
    for s in range(0, accounts, step):
        eng.load_batch_features(ids[s:s + step], np.asarray(pop.batch[s:s + step], ACCTBATCH))
        eng.load_ext_features(ids[s:s + step], pop.ext[s:s + step])
    return eng


def run_e2e(a) -> dict:
    eng = build_engine(a.accounts, a.batch, a.backend)
    payloads = make_payloads(a.accounts, a.payloads, a.batch, seed=11)
    n_req = a.batch
    for i in range(a.warmup):  # windows / HLLs fill, graphs warm
        eng.score_batch_bytes(payloads[i % len(payloads)])
    lat, lock = [], threading.Lock()
    counter = {"i": 0}

    def worker():
        while True:
            with lock:
                i = counter["i"]
                if i >= a.steps:
                    return
                counter["i"] = i + 1
            t0 = time.perf_counter()
            out = eng.score_batch_bytes(payloads[i % len(payloads)], t0)
            dt = (time.perf_counter() - t0) * 1e3
            assert len(out) > n_req  # every response carries n_req ScoreTransactionResponse messages
            with lock:
                lat.append(dt)

    th = [threading.Thread(target=worker) for _ in range(a.threads)]
    core = getattr(eng, "core", None)
    if core is not None:
        core.stats(True)
    t0 = time.perf_counter()
    [t.start() for t in th]
    [t.join() for t in th]
    el = time.perf_counter() - t0
    stages = {}
    if core is not None:  # per-stage host cost of the native path, ns per row (summed over threads)
        st = core.stats(True)
        rows = max(int(st["rows"]), 1)
        stages = {k[:-3] + "_ns_per_row": round(st[k] / rows, 1)
                  for k in ("parse_ns", "resolve_ns", "pack_ns", "submit_ns", "copy_ns", "serialize_ns")}
        stages.update(device_us_per_step=round(st["device_ns"] / max(int(st["steps"]), 1) / 1e3, 1),
                      steps=int(st["steps"]), mean_rows_per_step=round(st["rows"] / max(int(st["steps"]), 1), 1))
    eng.close()
    return dict(metric="fraud scores/sec (risk.v1.ScoreBatch bytes in -> bytes out, in-process)",
                value=a.steps * n_req / el, unit="scores/s", scope="e2e", n_gpus=1 if a.backend == "gpu" else 0,
                steps=a.steps, warmup=a.warmup, ms_per_step=el / a.steps * 1e3, higher_is_better=True,
                scaling="weak", vs_baseline=None, dtype="fp32", data="synthetic (UUID ids, random-init cfg3 weights)",
                config=dict(model="cfg3 GBDT(100,d7,128f)+MLP(32-256-1)", batch_per_request=n_req,
                            caller_threads=a.threads, accounts=a.accounts,
                            path=("native serving core (engine/serving.py): C++ parse -> AccountIndex(UUID) -> "
                                  "FIFO -> stepper packs + launches -> completion -> C++ serialize, no Python "
                                  "per batch" if core is not None else
                                  "C++ parse -> AccountIndex(UUID) -> pack -> GPU graphs -> C++ serialize")),
                host_stages=stages,
                p50_latency_ms=float(np.percentile(lat, 50)), p99_latency_ms=float(np.percentile(lat, 99)),
                latency_baseline_ms=BASELINE_P99_MS,
                latency_vs_baseline=BASELINE_P99_MS / float(np.percentile(lat, 99)))


def _client(i, port, kind, accounts, batch, n_payloads, t_start, t_end, q):
    import grpc
    from igaming_platform_amd.proto import risk_v1 as P
    ch = grpc.insecure_channel(f"127.0.0.1:{port}", options=[("grpc.max_receive_message_length", 256 << 20),
                                                             ("grpc.max_send_message_length", 256 << 20)])
    if kind == "batch":
        call = ch.unary_unary(P.method_path("ScoreBatch"))
        payloads = make_payloads(accounts, n_payloads, batch, seed=100 + i)
        per = batch
    elif kind in ("ltv", "abuse"):
        rpc, req = (("PredictLTV", P.PredictLTVRequest) if kind == "ltv" else ("CheckBonusAbuse", P.CheckBonusAbuseRequest))
        call = ch.unary_unary(P.method_path(rpc))
        rng = np.random.default_rng(100 + i)
        payloads = [req(account_id=account_id(int(x))).SerializeToString() for x in rng.integers(0, accounts, 4096)]
        per = 1
    else:
        call = ch.unary_unary(P.method_path("ScoreTransaction"))
        payloads = tx_payloads(accounts, 4096, seed=100 + i)
        per = 1
    lat, errs, k = [], 0, 0
    while time.time() < t_start - 1.0:  # connect / warm before the window
        call(payloads[k % len(payloads)], timeout=30)
        k += 1
    while time.time() < t_end:
        t0 = time.perf_counter()
        try:
            call(payloads[k % len(payloads)], timeout=30)
        except Exception:
            errs += 1
            continue
        finally:
            k += 1
        if time.time() >= t_start:
            lat.append((time.perf_counter() - t0) * 1e3)
    ch.close()
    q.put((lat, errs, per))


def _open_loop_client(i, port, accounts, rates, seconds, t_start, q):
    """One load-generator process: open-loop unary ScoreTransaction over grpc.aio. Calls are
    issued on a fixed schedule (rate / clients per second) whatever the server's pace, up to
    4096 in flight; a call's latency counts from its SCHEDULED send time, so a server that
    falls behind shows up as growing latency, not as a lower offered load."""
    import asyncio
    import grpc
    from igaming_platform_amd.proto import risk_v1 as P
    payloads = tx_payloads(accounts, 8192, seed=300 + i)

    async def main():
        ch = grpc.aio.insecure_channel(f"127.0.0.1:{port}")
        call = ch.unary_unary(P.method_path("ScoreTransaction"))
        for k in range(200):  # connect + warm
            await call(payloads[k], timeout=30)
        out = []
        t_level = t_start
        for rate in rates:
            while time.time() < t_level:
                await asyncio.sleep(0.001)
            lat, errs, sent, kinds = [], [0], 0, {}
            sem = asyncio.Semaphore(4096)
            loop = asyncio.get_running_loop()
            t0 = loop.time()
            interval = 1.0 / rate

            async def one(t_sched, body):
                try:
                    await call(body, timeout=30)
                    lat.append((loop.time() - t_sched) * 1e3)
                except Exception as e:
                    errs[0] += 1
                    k = str(getattr(e, "code", lambda: type(e).__name__)())
                    kinds[k] = kinds.get(k, 0) + 1
                finally:
                    sem.release()
            tasks = []
            while True:
                t_sched = t0 + sent * interval
                if t_sched >= t0 + seconds:
                    break
                d = t_sched - loop.time()
                if d > 0:
                    await asyncio.sleep(d)
                await sem.acquire()
                tasks.append(asyncio.ensure_future(one(t_sched, payloads[sent % len(payloads)])))
                sent += 1
            await asyncio.gather(*tasks)
            out.append((rate, sent, lat, errs[0], loop.time() - t0, kinds))
            t_level += seconds + 2.0
        await ch.close()
        return out
    q.put(asyncio.run(main()))


def make_server(a, eng, batching: bool):
    """--server native (default): the C++ HTTP/2 server (api/native_grpc.py); aio: grpc.aio."""
    if a.server == "native":
        from igaming_platform_amd.api.native_grpc import NativeRiskServer
        return NativeRiskServer(eng, port=0, workers=a.server_workers, batching=batching).start()
    from igaming_platform_amd.api.grpc_server import RiskServer
    return RiskServer(eng, port=0, batching=batching, workers=16).start()


def server_desc(a) -> str:
    if a.server == "native":
        return (f"native HTTP/2 (libnghttp2, {a.server_workers} epoll workers, SO_REUSEPORT); ScoreTransaction "
                "straight into the serving core")
    return "grpc.aio, raw-bytes handlers, native serving core FIFO (NativeUnary)"


def run_grpc_open_loop(a) -> dict:
    """Unary ScoreTransaction throughput vs latency: offered load stepped through ``--rates``
    (whole-node calls/s, split over ``--clients`` processes), open loop."""
    import multiprocessing as mp
    eng = build_engine(a.accounts, a.batch, a.backend, a.model)
    srv = make_server(a, eng, batching=True)
    rates = [int(x) for x in a.rates.split(",")]
    if a.client == "native":
        return _native_open_loop(a, eng, srv, rates)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    lead = 30.0
    t_start = time.time() + lead
    per = [r / a.clients for r in rates]
    procs = [ctx.Process(target=_open_loop_client, args=(i, srv.port, a.accounts, per, a.seconds, t_start, q))
             for i in range(a.clients)]
    [p.start() for p in procs]
    res = [q.get(timeout=lead + len(rates) * (a.seconds + 2) + 300) for _ in procs]
    [p.join() for p in procs]
    st = eng.core.stats(False) if getattr(eng, "core", None) is not None else None
    srv.stop(0.5) if a.server != "native" else srv.stop()
    eng.close()
    curve = []
    for li, rate in enumerate(rates):
        lat = [x for r in res for x in r[li][2]]
        sent = sum(r[li][1] for r in res)
        errs = sum(r[li][3] for r in res)
        dur = max(r[li][4] for r in res)
        kinds = {}
        for r in res:
            for k, v in r[li][5].items():
                kinds[k] = kinds.get(k, 0) + v
        curve.append(dict(offered_per_s=rate, achieved_per_s=round(len(lat) / dur, 1), calls=sent, errors=errs,
                          error_kinds=kinds,
                          p50_ms=round(float(np.percentile(lat, 50)), 3) if lat else None,
                          p99_ms=round(float(np.percentile(lat, 99)), 3) if lat else None))
    ok = [c for c in curve if c["p99_ms"] is not None and c["p99_ms"] < BASELINE_P99_MS and c["errors"] == 0
          and c["achieved_per_s"] >= 0.95 * c["offered_per_s"]]
    best = max(ok, key=lambda c: c["achieved_per_s"]) if ok else None
    return dict(metric="unary risk.v1.ScoreTransaction over gRPC: throughput vs latency (open loop)",
                value=best["achieved_per_s"] if best else 0.0, unit="calls/s",
                value_is="highest offered rate answered in full with p99 < 50 ms", scope="grpc_unary_open_loop",
                n_gpus=1 if a.backend == "gpu" else 0, data="synthetic (UUID ids, random-init cfg3 weights)",
                config=dict(model=FRAUD_MODELS[a.model][0], clients=a.clients, seconds_per_level=a.seconds,
                            server=server_desc(a),
                            client="grpc.aio open loop, latency from the scheduled send time"),
                curve=curve, best=best,
                mean_rows_per_device_step=(round(st["rows"] / max(st["steps"], 1), 1) if st else None),
                latency_baseline_ms=BASELINE_P99_MS)


RPC_PATHS = {"tx": "ScoreTransaction", "ltv": "PredictLTV", "segment": "GetPlayerSegment", "abuse": "CheckBonusAbuse"}
RPC_MODELS = {"tx": "cfg3 GBDT(100,d7,128f)+MLP(32-256-1)",
              "ltv": "cfg4 LTV MLP 4x512 over 256 features (HBM tables) + K9, fused chain",
              "segment": "cfg4 LTV MLP 4x512 over 256 features (HBM tables) + K9, fused chain",
              "abuse": "cfg5 GRU 2x256 over the last 100 events (HBM event rings) + K1 rule signals + links"}


def _curve_result(a, curve, st) -> dict:
    ok = [c for c in curve if c["p99_ms"] is not None and c["p99_ms"] < BASELINE_P99_MS and c["errors"] == 0
          and c["achieved_per_s"] >= 0.95 * c["offered_per_s"]]
    best = max(ok, key=lambda c: c["achieved_per_s"]) if ok else None
    rpc = RPC_PATHS[a.rpc]
    return dict(metric=f"unary risk.v1.{rpc} over gRPC: throughput vs latency (open loop)",
                value=best["achieved_per_s"] if best else 0.0, unit="calls/s",
                value_is="highest offered rate answered in full with p99 < 50 ms", scope="grpc_unary_open_loop",
                n_gpus=1 if a.backend == "gpu" else 0,
                data=f"synthetic (UUID ids over {a.accounts} accounts"
                     + (f", Zipf({a.zipf}) account ranks" if a.zipf > 1 else ", uniform") + ", random-init weights)",
                dtype=getattr(a, "numerics", "fp32"),
                config=dict(model=FRAUD_MODELS[a.model][0] if a.rpc == "tx" else RPC_MODELS[a.rpc],
                            clients=a.clients, seconds_per_level=a.seconds, backend=a.backend,
                            server=server_desc(a),
                            client=("native HTTP/2 open loop (libnghttp2, one connection per thread)" if a.client == "native"
                                    else "grpc.aio open loop") + ", latency from the scheduled send time"),
                curve=curve, best=best,
                mean_rows_per_device_step=(round(st["rows"] / max(st["steps"], 1), 1) if st else None),
                latency_baseline_ms=BASELINE_P99_MS)


def _native_open_loop(a, eng, srv, rates) -> dict:
    """The offered-load curve from the C++ load generator (csrc/runtime/h2grpc.cpp grpc_load):
    ``--clients`` HTTP/2 connections, each on its own thread."""
    from igaming_platform_amd.native import native
    from igaming_platform_amd.proto import risk_v1 as P
    payloads = (tx_payloads(a.accounts, 8192, seed=300) if a.rpc == "tx"
                else acct_payloads(a.accounts, a.rpc, 1 << 16, 300, a.zipf))
    path = P.method_path(RPC_PATHS[a.rpc])
    native().grpc_load("127.0.0.1", srv.port, path, payloads, 2000.0, 1.0, a.clients, 4096)  # warm
    curve = []
    for rate in rates:
        r = native().grpc_load("127.0.0.1", srv.port, path, payloads, float(rate), a.seconds, a.clients, 8192)
        lat = np.asarray(r["latency_ms"])
        curve.append(dict(offered_per_s=rate, achieved_per_s=round(len(lat) / float(r["elapsed"]), 1), calls=int(r["sent"]),
                          errors=int(r["errors"]), error_kinds={},
                          p50_ms=round(float(np.percentile(lat, 50)), 3) if len(lat) else None,
                          p99_ms=round(float(np.percentile(lat, 99)), 3) if len(lat) else None))
        print(json.dumps(curve[-1]), flush=True)
        time.sleep(1.0)
    if a.rpc == "tx":
        st = eng.core.stats(False) if getattr(eng, "core", None) is not None else None
    else:  # the native account router's device steps (None: served on the Python path)
        acct = getattr(eng, "acct", None)
        st = acct.router.stats(3 if a.rpc == "abuse" else 1) if acct is not None else None
    out_srv = srv.stats()
    srv.stop()
    eng.close()
    res = _curve_result(a, curve, st)
    res["server_stats"] = out_srv
    return res


def run_grpc(a) -> dict:
    import multiprocessing as mp
    cold = a.rpc in ("ltv", "abuse")
    eng = build_cold_engine(a.accounts, a.backend) if cold else build_engine(a.accounts, a.batch, a.backend)
    srv = make_server(a, eng, batching=a.rpc != "batch")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    lead = 25.0  # client start-up (import + payload generation) happens before the window
    t_end = time.time() + lead + a.seconds
    procs = [ctx.Process(target=_client, args=(i, srv.port, a.rpc, a.accounts,
                                               a.batch, 4, t_end - a.seconds, t_end, q))
             for i in range(a.clients)]
    [p.start() for p in procs]
    res = [q.get(timeout=a.seconds + lead + 300) for _ in procs]
    [p.join() for p in procs]
    batcher = None if a.server == "native" else {"tx": srv.batcher, "ltv": srv.ltv_batcher,
                                                 "abuse": srv.abuse_batcher}.get(a.rpc)
    srv.stop(0.5) if a.server != "native" else srv.stop()
    eng.close()
    lat = [x for r in res for x in r[0]]
    per = res[0][2]
    calls = len(lat)
    names = {"batch": "fraud scores/sec (risk.v1.ScoreBatch over gRPC)",
             "tx": "fraud scores/sec (unary risk.v1.ScoreTransaction over gRPC, micro-batched)",
             "ltv": "PredictLTV answers/sec (unary over gRPC, micro-batched)",
             "abuse": "CheckBonusAbuse answers/sec (unary over gRPC, micro-batched)"}
    mean_batch = (batcher.items / max(batcher.batches, 1)) if batcher is not None else None
    return dict(metric=names[a.rpc], mean_device_batch=mean_batch,
                value=calls * per / a.seconds, unit="scores/s", scope="grpc", n_gpus=1 if a.backend == "gpu" else 0,
                higher_is_better=True, dtype="fp32", data="synthetic (UUID ids, random-init weights)",
                config=dict(model={"ltv": "cfg4 LTV MLP 4x512 (bf16) + K9", "abuse": "cfg5 GRU 2x256 over 100 events"
                                   " + rule signals"}.get(a.rpc, "cfg3 GBDT(100,d7,128f)+MLP(32-256-1)"),
                            rpc=a.rpc, clients=a.clients,
                            seconds=a.seconds, transactions_per_call=per, accounts=a.accounts,
                            server=server_desc(a)),
                calls=calls, errors=sum(r[1] for r in res),
                p50_latency_ms=float(np.percentile(lat, 50)), p99_latency_ms=float(np.percentile(lat, 99)),
                latency_baseline_ms=BASELINE_P99_MS,
                latency_vs_baseline=BASELINE_P99_MS / float(np.percentile(lat, 99)))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--scope", default="e2e", choices=["e2e", "grpc", "engine_batched"])
    ap.add_argument("--rpc", default="batch", choices=["batch", "tx", "ltv", "segment", "abuse"])
    ap.add_argument("--zipf", type=float, default=0.0, help="account-id distribution: Zipf exponent (> 1), 0 uniform")
    ap.add_argument("--numerics", default="fp32", choices=["fp32", "bf16"], help="cfg4 / cfg5 model numerics")
    ap.add_argument("--backend", default="gpu", choices=["gpu", "cpu"])
    ap.add_argument("--model", default="cfg3", choices=sorted(FRAUD_MODELS),
                    help="fraud model of the ScoreTransaction / ScoreBatch scopes (cfg1: CPU logistic, BASELINE config 1)")
    ap.add_argument("--accounts", type=int, default=1 << 20)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--payloads", type=int, default=6)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--json-out", default="")
    ap.add_argument("--open-loop", action="store_true", help="--scope grpc --rpc tx: offered-load curve")
    ap.add_argument("--server", default="native", choices=["native", "aio"], help="--scope grpc: the gRPC server")
    ap.add_argument("--server-workers", type=int, default=4, help="--server native: epoll worker threads")
    ap.add_argument("--client", default="native", choices=["native", "aio"],
                    help="--open-loop load generator: C++ HTTP/2 (default) or grpc.aio processes")
    ap.add_argument("--rates", default="2000,5000,8000,12000,16000,24000",
                    help="--open-loop: offered whole-node unary calls/s per level")
    a = ap.parse_args(argv)
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
    if a.scope == "grpc" and a.rpc in ("ltv", "segment", "abuse") and a.open_loop:
        eng = build_cold_engine(a.accounts, a.backend, a.numerics)
        out = _native_open_loop(a, eng, make_server(a, eng, batching=True), [int(x) for x in a.rates.split(",")])
    elif a.scope == "grpc" and a.rpc == "tx" and a.open_loop:
        out = run_grpc_open_loop(a)
    else:
        out = {"e2e": run_e2e, "grpc": run_grpc, "engine_batched": run_cold_engine}[a.scope](a)
    line = json.dumps(out)
    print(line, flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())

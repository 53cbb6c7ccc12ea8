#!/usr/bin/env python3
"""Mixed traffic on one GPU: the serving bench's ScoreBatch load plus open-loop
CheckBonusAbuse and unary ScoreTransaction over the native HTTP/2 server, all at once.

The reference calls CheckBonusAbuse from the node that scores wallet traffic
(/root/reference/services/bonus/internal/service/bonus_engine.go:268-275 for the award path,
services/wallet/internal/service/wallet_service.go:261-279 for the per-transaction risk check).
Here one engine holds the cfg3 fraud model, the cfg4 LTV MLP and the cfg5 abuse GRU; the run is

  phase A  ScoreBatch alone: ``--threads`` in-process ingress threads, 8192-transaction requests
           through the native serving core (as bench.py's serving scope) for ``--seconds``
  phase B  the same ScoreBatch load + ``--abuse-rate`` CheckBonusAbuse/s + ``--tx-rate``
           ScoreTransaction/s, open loop from the native load generator (C++ HTTP/2 clients,
           latency from the scheduled send time) over ``--clients`` connections each

and reports the ScoreBatch throughput of both phases (the loss the unary traffic costs it), the
unary p50 / p99, the abuse device's cluster fallbacks (gru_wsx clusters that did not become
co-resident) and the device steps of each path. One JSON line (``--json-out``).

Usage: python tools/bench_mixed.py [--seconds 5] [--abuse-rate 100000] [--tx-rate 200000]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")


def build(accounts: int, abuse_max_batch: int = 0, abuse_priority: bool = False, acct_depth: int = 2,
          serve_depth: int = 0):
    """One engine: cfg3 fraud model (8192-row micro-batches), cfg4 LTV MLP, cfg5 abuse GRU; warehouse
    rows + ext rows for every account, profile rows for the LTV model, full event rings."""
    import bench_e2e as E
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.risk_engine import RiskEngine
    from igaming_platform_amd.layouts import ACCTBATCH
    from igaming_platform_amd.onnx import builders
    from igaming_platform_amd.utils.synth import make_population
    cfg = Config()
    cfg.features.width = 128
    cfg.gpu.buckets = [64, 512, 2048, 8192]
    cfg.gpu.max_batch = 8192
    cfg.abuse.max_batch = abuse_max_batch
    cfg.abuse.high_priority = abuse_priority
    cfg.gpu.acct_depth = acct_depth
    if serve_depth > 0:
        cfg.gpu.serve_depth = serve_depth
    eng = RiskEngine(cfg, backend="gpu", capacity=accounts + 4096, fraud_model=E.fraud_model_bytes("cfg3"),
                     ltv_model=builders.build("ltv_mlp", n_features=256, width=512, layers=4).SerializeToString(),
                     abuse_model=builders.build("gru", seq=100, in_dim=16, hidden=256).SerializeToString())
    pop = make_population(accounts, 98, seed=3, fast_hash=True)
    ids = [E.account_id(i) for i in range(accounts)]
    rng = np.random.default_rng(5)
    step = 1 << 18
    for s in range(0, accounts, step):
        eng.load_batch_features(ids[s:s + step], np.asarray(pop.batch[s:s + step], ACCTBATCH))
        eng.load_ext_features(ids[s:s + step], pop.ext[s:s + step])
        slots, owners = eng.registry.resolve_ids(ids[s:s + step], insert=True)
        n = len(slots)
        eng.ltv.set_rows(slots, owners, np.floor(rng.uniform(0, 1, (n, 25)) * E.PROFILE_SCALE).astype(np.float32),
                         rng.normal(0, 1, (n, 231)).astype(np.float32))
    E.fill_event_rings(eng.backends[0].store)
    return eng


def batch_load(eng, payloads, threads: int, seconds: float, t_base: int, rows_per_request: int = 8192,
               rate: float = 0.0):
    """ScoreBatch from ``threads`` ingress threads for ``seconds``: closed loop, or paced open
    loop at ``rate`` requests/s (request k of thread w due at t0 + (k * threads + w) / rate;
    latency from the due time). Returns (rows/s, p50, p99 ms, requests)."""
    core = eng.core
    lock = threading.Lock()
    lat, rows, starts = [], [0], []
    t_start = time.perf_counter()
    t_end = t_start + seconds
    counter = [0]

    def worker(w):
        k = 0
        while time.perf_counter() < t_end:
            due = None
            if rate > 0:
                due = t_start + (k * threads + w) / rate
                k += 1
                if due >= t_end:
                    return
                wait = due - time.perf_counter()
                if wait > 0:
                    time.sleep(wait)
            with lock:
                i = counter[0]
                counter[0] += 1
            t0 = time.perf_counter_ns() if due is None else int(due * 1e9)
            out = core.score_batch(payloads[i % len(payloads)], t_base + i // 50, time.perf_counter_ns())
            dt = (time.perf_counter_ns() - t0) / 1e6
            if not out:
                raise RuntimeError("empty ScoreBatch response")
            with lock:
                lat.append(dt)
                starts.append(t0 / 1e6 - t_start * 1e3)
                rows[0] += rows_per_request
    th = [threading.Thread(target=worker, args=(w,)) for w in range(threads)]
    t0 = time.perf_counter()
    [t.start() for t in th]
    [t.join() for t in th]
    el = time.perf_counter() - t0
    batch_load.stalls = stall_windows(np.asarray(starts), np.asarray(lat), 5.0)
    return rows[0] / el, float(np.percentile(lat, 50)), float(np.percentile(lat, 99)), counter[0]


def open_loop(port: int, rpc: str, payloads, rate: float, seconds: float, conns: int, out: dict):
    from igaming_platform_amd.native import native
    from igaming_platform_amd.proto import risk_v1 as P
    path = P.method_path({"abuse": "CheckBonusAbuse", "tx": "ScoreTransaction"}[rpc])
    r = native().grpc_load("127.0.0.1", port, path, payloads, float(rate), float(seconds), int(conns), 8192)
    lat = np.asarray(r["latency_ms"])
    out[rpc] = dict(offered_per_s=rate, achieved_per_s=round(len(lat) / float(r["elapsed"]), 1), calls=int(r["sent"]),
                    errors=int(r["errors"]),
                    p50_ms=round(float(np.percentile(lat, 50)), 3) if len(lat) else None,
                    p99_ms=round(float(np.percentile(lat, 99)), 3) if len(lat) else None,
                    stall_windows=stall_windows(np.asarray(r["sched_ms"]), lat, 5.0))


def stall_windows(t_ms, lat_ms, over_ms: float, bin_ms: float = 50.0, top: int = 12):
    """Where a run's tail comes from: the 50-ms windows (by scheduled send / start time) whose
    worst latency exceeds ``over_ms``, as [window start ms, calls in it, calls over, worst ms]."""
    if len(t_ms) == 0 or len(t_ms) != len(lat_ms):
        return []
    b = (np.asarray(t_ms) // bin_ms).astype(np.int64)
    out = []
    for w in np.unique(b[lat_ms > over_ms]):
        m = b == w
        out.append([int(w * bin_ms), int(m.sum()), int((lat_ms[m] > over_ms).sum()), round(float(lat_ms[m].max()), 2)])
    out.sort(key=lambda x: -x[3])
    return sorted(out[:top])


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--accounts", type=int, default=1 << 20)
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--threads", type=int, default=8, help="ScoreBatch ingress threads")
    ap.add_argument("--abuse-rate", type=float, default=100000.0)
    ap.add_argument("--tx-rate", type=float, default=200000.0)
    ap.add_argument("--clients", type=int, default=4, help="HTTP/2 connections per open-loop RPC")
    ap.add_argument("--server-workers", type=int, default=4)
    ap.add_argument("--abuse-max-batch", type=int, default=0, help="AbuseConfig.max_batch (0: the largest bucket)")
    ap.add_argument("--abuse-priority", type=int, default=0, help="AbuseConfig.high_priority")
    ap.add_argument("--acct-depth", type=int, default=2, help="GpuConfig.acct_depth (abuse device slots)")
    ap.add_argument("--serve-depth", type=int, default=0, help="GpuConfig.serve_depth (scoring pipeline slots; 0: the config's)")
    ap.add_argument("--batch-rate", type=float, default=0.0,
                    help="ScoreBatch requests/s, paced open loop over --threads (0: closed loop)")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args(argv)
    import bench_e2e as E
    from igaming_platform_amd.api.native_grpc import NativeRiskServer
    from igaming_platform_amd.utils.synth import NOW0
    eng = build(a.accounts, a.abuse_max_batch, bool(a.abuse_priority), a.acct_depth, a.serve_depth)
    srv = NativeRiskServer(eng, port=0, workers=a.server_workers, batching=True).start()
    payloads = E.spread_payloads(a.accounts, 64, 8192, seed=11)
    abuse_p = E.acct_payloads(a.accounts, "abuse", 1 << 16, 300)
    tx_p = E.tx_payloads(a.accounts, 8192, seed=300)
    # warm: graphs, histories, both unary paths
    batch_load(eng, payloads, a.threads, 2.0, NOW0 - 3600)
    warm = {}
    open_loop(srv.port, "abuse", abuse_p, 2000, 1.0, a.clients, warm)
    open_loop(srv.port, "tx", tx_p, 2000, 1.0, a.clients, warm)
    dev = [d for d in eng.acct.devices if hasattr(d, "driver") and hasattr(d.driver, "fallbacks")]
    fb0 = sum(int(d.driver.fallbacks) for d in dev)
    acct0 = eng.acct.router.stats(3, True)
    alone = batch_load(eng, payloads, a.threads, a.seconds, NOW0, rate=a.batch_rate)
    time.sleep(1.0)
    # the unary load alone (the same two open loops, no ScoreBatch): what the GPU sharing costs it
    solo = {}
    th = [threading.Thread(target=open_loop, args=(srv.port, "abuse", abuse_p, a.abuse_rate, a.seconds, a.clients, solo)),
          threading.Thread(target=open_loop, args=(srv.port, "tx", tx_p, a.tx_rate, a.seconds, a.clients, solo))]
    [t.start() for t in th]
    [t.join() for t in th]
    time.sleep(1.0)
    eng.acct.router.stats(3, True)
    eng.core.stats(True)
    res = {}
    th = [threading.Thread(target=open_loop, args=(srv.port, "abuse", abuse_p, a.abuse_rate, a.seconds, a.clients, res)),
          threading.Thread(target=open_loop, args=(srv.port, "tx", tx_p, a.tx_rate, a.seconds, a.clients, res))]
    [t.start() for t in th]
    mixed = batch_load(eng, payloads, a.threads, a.seconds, NOW0 + 600, rate=a.batch_rate)
    [t.join() for t in th]
    st = eng.acct.router.stats(3, False)
    sv = dict(eng.core.stats(False))
    ns = max(int(sv.get("steps", 1)), 1)
    serve = {k: sv[k] for k in ("items", "rows", "steps", "unary", "max_step_rows") if k in sv}
    serve.update({k[:-3] + "_us_per_step": round(sv[k] / ns / 1e3, 1) for k in sv if k.endswith("_ns")})
    fb = sum(int(d.driver.fallbacks) for d in dev) - fb0
    out = dict(metric="mixed traffic on one GPU: ScoreBatch load + open-loop CheckBonusAbuse + ScoreTransaction",
               n_gpus=1, seconds=a.seconds, data="synthetic (UUID ids over %d accounts, random-init cfg3/cfg4/cfg5 "
                                                "weights, full 100-event histories)" % a.accounts,
               scorebatch_alone=dict(scores_per_s=round(alone[0], 1), p50_ms=round(alone[1], 3), p99_ms=round(alone[2], 3),
                                     requests=alone[3]),
               scorebatch_mixed=dict(scores_per_s=round(mixed[0], 1), p50_ms=round(mixed[1], 3), p99_ms=round(mixed[2], 3),
                                     requests=mixed[3], stall_windows=batch_load.stalls),
               stall_windows_what="[window start ms, calls, calls over 5 ms, worst ms] per 50-ms window with a call over "
                                  "5 ms; ScoreBatch windows by request start, unary windows by scheduled send (the load "
                                  "generator starts its schedule ~200 ms after the ScoreBatch threads)",
               scorebatch_loss_pct=round(100.0 * (1 - mixed[0] / alone[0]), 2),
               check_bonus_abuse=res.get("abuse"), score_transaction=res.get("tx"),
               unary_without_scorebatch=dict(check_bonus_abuse=solo.get("abuse"), score_transaction=solo.get("tx")),
               abuse_cluster_fallbacks=fb,
               abuse_rows_per_device_step=round(st.get("items", 0) / max(int(st.get("steps", 1)), 1), 1),
               # where an abuse call's time goes in the mixed phase (acct_core.h AcctStats): queueing
               # before its step, the step on the device, the answer writing (link lookups included)
               abuse_device_us_per_step=round(st.get("device_ns", 0) / max(int(st.get("steps", 1)), 1) / 1e3, 1),
               abuse_queue_us_per_call=round(st.get("queue_ns", 0) / max(int(st.get("items", 1)), 1) / 1e3, 1),
               abuse_finish_us_per_step=round(st.get("finish_ns", 0) / max(int(st.get("steps", 1)), 1) / 1e3, 1),
               abuse_steps=int(st.get("steps", 0)),
               link_read_timeouts=int(getattr(eng.links, "read_timeouts", 0) or 0) if getattr(eng, "links", None) else None,
               link_lock_takeovers=int(getattr(eng.links, "takeovers", 0) or 0) if getattr(eng, "links", None) else None,
               config=dict(scorebatch_threads=a.threads, clients_per_rpc=a.clients, server_workers=a.server_workers,
                           scorebatch_offered_per_s=(a.batch_rate * 8192 if a.batch_rate > 0 else "closed loop"),
                           abuse_max_batch=a.abuse_max_batch, abuse_high_priority=bool(a.abuse_priority),
                           acct_depth=a.acct_depth, serve_depth=eng.cfg.gpu.serve_depth,
                           models="cfg3 GBDT(100,d7,128f)+MLP(32-256-1) fp32; cfg5 GRU 2x256 x 100 events fp32 split"),
               server_stats=srv.stats(), serve_core_mixed=serve)
    srv.stop()
    eng.close()
    line = json.dumps(out)
    print(line, flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())

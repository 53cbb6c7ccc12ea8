#!/usr/bin/env python3
"""Config 1: risk.v1.ScoreTransaction end to end over gRPC on the CPU path (C++ executor,
32-feature logistic model, batch = 1 — no micro-batching), N concurrent unary clients.
Prints one JSON line: scores/s + p50/p99 latency (client-measured, includes gRPC)."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def client(i, port, accounts, t_start, t_end, q):
    from igaming_platform_amd.clients.risk_client import RiskClient
    from igaming_platform_amd.proto import risk_v1 as P
    c = RiskClient(f"127.0.0.1:{port}")
    rng = np.random.default_rng(i)
    types = ["deposit", "withdraw", "bet", "win"]
    lat, errs = [], 0
    while time.time() < t_end:
        req = P.ScoreTransactionRequest(account_id=f"acc-{int(rng.integers(0, accounts))}",
                                        amount=int(rng.integers(100, 500000)),
                                        transaction_type=types[int(rng.integers(0, 4))],
                                        device_id=f"dev-{int(rng.integers(0, 50000))}", ip_address="10.0.0.1")
        t0 = time.perf_counter()
        try:
            c.call("ScoreTransaction", req)
        except Exception:
            errs += 1
            continue
        if time.time() >= t_start:
            lat.append((time.perf_counter() - t0) * 1e3)
    c.close()
    q.put((lat, errs))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--accounts", type=int, default=10000)
    a = ap.parse_args()
    from igaming_platform_amd.api.grpc_server import RiskServer
    from igaming_platform_amd.clients.risk_client import RiskClient
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.risk_engine import RiskEngine
    from igaming_platform_amd.onnx import builders
    from igaming_platform_amd.proto import risk_v1 as P
    cfg = Config()
    cfg.features.width = 32
    eng = RiskEngine(cfg, backend="cpu", capacity=a.accounts * 2,
                     fraud_model=builders.build("logistic", n_features=32).SerializeToString())
    srv = RiskServer(eng, port=0, batching=False).start()
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    t_end = time.time() + 3.0 + a.seconds   # clients start measuring 3 s from now (after spawn)
    procs = [ctx.Process(target=client, args=(i, srv.port, a.accounts, t_end - a.seconds, t_end, q))
             for i in range(a.clients)]
    [p.start() for p in procs]
    res = [q.get(timeout=a.seconds + 120) for _ in procs]
    [p.join() for p in procs]
    srv.stop(0.5)
    lat = [x for r in res for x in r[0]]
    errs = sum(r[1] for r in res)
    el = a.seconds
    out = dict(metric="fraud scores/sec (risk.v1.ScoreTransaction over gRPC, CPU executor)", value=len(lat) / el,
               unit="scores/s", n_gpus=0, higher_is_better=True, dtype="fp32", data="synthetic",
               config=dict(model="cfg1 32-feature logistic (Gemm+Sigmoid), C++ CPU executor", batch=1,
                           clients=a.clients, seconds=a.seconds),
               p50_latency_ms=float(np.percentile(lat, 50)), p99_latency_ms=float(np.percentile(lat, 99)),
               latency_baseline_ms=50.0, errors=errs)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())

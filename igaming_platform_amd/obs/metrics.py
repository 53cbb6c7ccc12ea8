"""Prometheus metrics of the risk service.

The reference exposes only Go runtime metrics and lists the intended ones in a no-op
interceptor (services/risk/cmd/main.go:170, 344-353; ``ModelMetrics`` onnx_model.go:359-365).
These are those, plus the GPU-side ones. Each engine owns its own registry so several
engines (tests, multi-tenant) never collide.
"""
from __future__ import annotations

import threading

import numpy as np
from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest
from prometheus_client.core import CounterMetricFamily

LAT_BUCKETS = (0.0001, 0.00025, 0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5)
ACTIONS = {1: "approve", 2: "review", 3: "block"}


class Metrics:
    def __init__(self):
        r = self.registry = CollectorRegistry()
        self.requests = Counter("risk_requests_total", "RPCs by method and status code", ["method", "code"], registry=r)
        self.latency = Histogram("risk_latency_seconds", "RPC latency", ["method"], buckets=LAT_BUCKETS, registry=r)
        # decision counters: plain accumulators on the hot path, exported at scrape time
        self._lock = threading.Lock()
        self._dec = [0] * 11
        self._act = [0] * 4
        self._n = self._ml_high = self._bl = 0
        # native serving cores count their own decisions (engine/serving.py core_metrics)
        self.sources = []
        self._fast = {}
        # the engine's LinkIndex (CheckBonusAbuse linked_accounts): its lock counters at scrape
        self.links = None
        r.register(_DecisionCollector(self))
        self.batch_size = Histogram("gpu_batch_size", "rows per device micro-batch",
                                    buckets=(1, 8, 64, 256, 1024, 4096, 8192), registry=r)
        self.step = Histogram("gpu_step_seconds", "device step time by phase", ["phase"], buckets=LAT_BUCKETS,
                              registry=r)
        self.queue_depth = Gauge("gpu_queue_depth", "requests waiting in the micro-batcher", ["gpu"], registry=r)
        self.gpu_healthy = Gauge("gpu_healthy", "1 if the shard is serving from its GPU", ["gpu"], registry=r)
        self.collective = Histogram("rccl_seconds", "collective time by op", ["op"], buckets=LAT_BUCKETS, registry=r)
        self.audit_evicted = Counter("risk_audit_evicted_rows_total",
                                     "audit rows dropped from the ring before a flush", registry=r)
        self.fallbacks = Counter("risk_fallback_total", "rows scored by the CPU fallback", ["reason"], registry=r)
        self.accounts = Gauge("risk_accounts", "accounts resident in the feature store", ["gpu"], registry=r)

    def fast_rpc(self, method: str) -> "_FastRpc":
        """risk_requests_total{OK} / risk_latency_seconds children of a hot RPC, resolved once."""
        f = self._fast.get(method)
        if f is None:
            f = self._fast[method] = _FastRpc(self, method)
        return f

    def observe_results(self, res: np.ndarray, feats=None) -> None:
        """Decision accounting from ResultRec rows (uint32 [n,2])."""
        n = len(res)
        if n == 0:
            return
        if n <= 8:  # unary path: plain ints, no numpy temporaries
            with self._lock:
                for p in res[:, 0].tolist():
                    self._dec[min((p & 0xFF) // 10, 10)] += 1
                    self._act[(p >> 16) & 3] += 1
                    self._ml_high += (p >> 28) & 1
                    self._bl += (p >> 27) & 1
                self._n += n
            return
        p = res[:, 0].astype(np.uint32)
        dec = np.bincount(np.minimum((p & 0xFF) // 10, 10), minlength=11)
        act = np.bincount((p >> 16) & 3, minlength=4)
        hi = int(np.count_nonzero(p & (1 << 28)))
        bl = int(np.count_nonzero(p & (1 << 27)))
        with self._lock:
            for i in range(11):
                self._dec[i] += int(dec[i])
            for i in range(4):
                self._act[i] += int(act[i])
            self._ml_high += hi
            self._bl += bl
            self._n += n

    def render(self) -> bytes:
        return generate_latest(self.registry)


class _DecisionCollector:
    def __init__(self, m: Metrics):
        self.m = m

    def collect(self):
        m = self.m
        with m._lock:
            dec, act, n, hi, bl = list(m._dec), list(m._act), m._n, m._ml_high, m._bl
        for src in list(m.sources):
            c = src()
            if not c:
                continue
            dec = [a + b for a, b in zip(dec, c["deciles"])]
            act = [a + b for a, b in zip(act, c["actions"])]
            n, hi, bl = n + c["scored"], hi + c["ml_high"], bl + c["blacklisted"]
        c = CounterMetricFamily("risk_scores", "transactions scored")
        c.add_metric([], n)
        yield c
        c = CounterMetricFamily("risk_score_bucket", "final scores by decile", labels=["decile"])
        for d, v in enumerate(dec):
            c.add_metric([str(d * 10)], v)
        yield c
        c = CounterMetricFamily("risk_action", "decisions by action", labels=["action"])
        for a, name in ACTIONS.items():
            c.add_metric([name], act[a])
        yield c
        c = CounterMetricFamily("risk_ml_high_risk", "ML score above the high-risk threshold")
        c.add_metric([], hi)
        yield c
        c = CounterMetricFamily("risk_blacklist_hits", "requests matching the blacklist")
        c.add_metric([], bl)
        yield c
        links = m.links
        if links is not None:
            c = CounterMetricFamily("risk_link_read_timeouts", "linked-account lookups answered empty because "
                                    "the link index lock was busy past its bounded wait")
            c.add_metric([], int(links.read_timeouts))
            yield c
            c = CounterMetricFamily("risk_link_lock_takeovers", "link index locks taken over from a dead process")
            c.add_metric([], int(links.takeovers))
            yield c



class _FastRpc:
    """OK calls of one hot RPC through pre-resolved metric children (no label lookup per call)."""

    def __init__(self, m: "Metrics", method: str):
        self._count = m.requests.labels(method=method, code="OK")
        self._lat = m.latency.labels(method=method)

    def observe(self, dt: float) -> None:
        self._count.inc()
        self._lat.observe(dt)

"""Prometheus metrics of the risk service.

The reference exposes only Go runtime metrics and lists the intended ones in a no-op
interceptor (services/risk/cmd/main.go:170, 344-353; ``ModelMetrics`` onnx_model.go:359-365).
These are those, plus the GPU-side ones. Each engine owns its own registry so several
engines (tests, multi-tenant) never collide.
"""
from __future__ import annotations

import numpy as np
from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

LAT_BUCKETS = (0.0001, 0.00025, 0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5)
ACTIONS = {1: "approve", 2: "review", 3: "block"}


class Metrics:
    def __init__(self):
        r = self.registry = CollectorRegistry()
        self.requests = Counter("risk_requests_total", "RPCs by method and status code", ["method", "code"], registry=r)
        self.latency = Histogram("risk_latency_seconds", "RPC latency", ["method"], buckets=LAT_BUCKETS, registry=r)
        self.scores = Counter("risk_scores_total", "transactions scored", registry=r)
        self.score_bucket = Counter("risk_score_bucket_total", "final scores by decile", ["decile"], registry=r)
        self.actions = Counter("risk_action_total", "decisions by action", ["action"], registry=r)
        self.ml_high = Counter("risk_ml_high_risk_total", "ML score above the high-risk threshold", registry=r)
        self.blacklist_hits = Counter("risk_blacklist_hits_total", "requests matching the blacklist", registry=r)
        self.batch_size = Histogram("gpu_batch_size", "rows per device micro-batch",
                                    buckets=(1, 8, 64, 256, 1024, 4096, 8192), registry=r)
        self.step = Histogram("gpu_step_seconds", "device step time by phase", ["phase"], buckets=LAT_BUCKETS,
                              registry=r)
        self.queue_depth = Gauge("gpu_queue_depth", "requests waiting in the micro-batcher", ["gpu"], registry=r)
        self.gpu_healthy = Gauge("gpu_healthy", "1 if the shard is serving from its GPU", ["gpu"], registry=r)
        self.collective = Histogram("rccl_seconds", "collective time by op", ["op"], buckets=LAT_BUCKETS, registry=r)
        self.fallbacks = Counter("risk_fallback_total", "rows scored by the CPU fallback", ["reason"], registry=r)
        self.accounts = Gauge("risk_accounts", "accounts resident in the feature store", ["gpu"], registry=r)

    def observe_results(self, res: np.ndarray, feats=None) -> None:
        """Vectorised decision accounting from ResultRec rows (uint32 [n,2])."""
        n = len(res)
        if n == 0:
            return
        p = res[:, 0].astype(np.uint32)
        score = (p & 0xFF).astype(np.int64)
        action = ((p >> 16) & 3).astype(np.int64)
        reasons = p >> 20
        self.scores.inc(n)
        dec = np.bincount(np.minimum(score // 10, 10), minlength=11)
        for d, c in enumerate(dec):
            if c:
                self.score_bucket.labels(decile=str(d * 10)).inc(int(c))
        act = np.bincount(action, minlength=4)
        for a, name in ACTIONS.items():
            if act[a]:
                self.actions.labels(action=name).inc(int(act[a]))
        hi = int(np.count_nonzero(reasons & (1 << 8)))
        if hi:
            self.ml_high.inc(hi)
        bl = int(np.count_nonzero(reasons & (1 << 7)))
        if bl:
            self.blacklist_hits.inc(bl)

    def render(self) -> bytes:
        return generate_latest(self.registry)

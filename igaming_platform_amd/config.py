"""Typed configuration for the MI355X risk engine.

One config tree, loaded from defaults -> optional YAML file -> environment variables.
Environment names are the reference's (``services/risk/cmd/main.go:55-70``;
``services/wallet/cmd/main.go:54-62``) so a deployment of the reference can switch
without renaming anything; ``MODEL_PATH`` is accepted as an alias of
``FRAUD_MODEL_PATH`` (reference quirk Q18, ``deploy/docker-compose.yml:173``).

Scoring defaults are ``DefaultConfig()`` of ``services/risk/internal/scoring/engine.go:215-228``
and the rule weights of ``engine.go:246-257``. Unlike the reference wiring
(``services/risk/cmd/main.go:121-126``, quirk Q5) env overrides are applied on top of
the defaults, so MLWeight/RuleWeight are never silently zero.
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

# Reason codes in rule order (engine.go:17-28). Bit i of the device reason mask is
# REASON_CODES[i]; the order is also the order of ``reason_codes`` in responses.
REASON_CODES: List[str] = [
    "HIGH_VELOCITY",            # bit 0  rule 1
    "NEW_ACCOUNT_LARGE_TX",     # bit 1  rule 2
    "MULTIPLE_DEVICES",         # bit 2  rule 3
    "IP_COUNTRY_MISMATCH",      # bit 3  rule 4 (many IPs; reference quirk Q12)
    "VPN_DETECTED",             # bit 4  rule 5
    "RAPID_DEPOSIT_WITHDRAW",   # bit 5  rule 6
    "BONUS_ABUSE",              # bit 6  rule 7
    "KNOWN_FRAUDSTER",          # bit 7  rule 8
    "ML_HIGH_RISK",             # bit 8  appended after the rules when ml > 0.7
    "SUSPICIOUS_PATTERN",       # bit 9  defined, never emitted by the reference rules
    "MULTI_ACCOUNT",            # bit 10 defined in risk.proto:274, never emitted
    "DEVICE_FINGERPRINT_MISMATCH",  # bit 11 risk.proto:275, never emitted
]
REASON_BIT = {name: i for i, name in enumerate(REASON_CODES)}

TX_TYPES = ["deposit", "withdraw", "bet", "win", "refund", "bonus"]
TX_TYPE_ID = {name: i for i, name in enumerate(TX_TYPES)}
TX_UNKNOWN = 255

ACTION_APPROVE, ACTION_REVIEW, ACTION_BLOCK = 1, 2, 3  # risk.proto:84-89
ACTION_NAMES = {1: "approve", 2: "review", 3: "block"}


@dataclass
class RuleWeights:
    """Per-reason weights (engine.go:246-257)."""
    high_velocity: int = 20
    new_account_large_tx: int = 30
    ip_country_mismatch: int = 25
    multiple_devices: int = 15
    suspicious_pattern: int = 20
    vpn_detected: int = 15
    known_fraudster: int = 50
    rapid_deposit_withdraw: int = 25
    bonus_abuse: int = 20
    ml_high_risk: int = 30  # defined but never added to the score (quirk Q13)

    def by_reason(self) -> Dict[str, int]:
        return {
            "HIGH_VELOCITY": self.high_velocity,
            "NEW_ACCOUNT_LARGE_TX": self.new_account_large_tx,
            "IP_COUNTRY_MISMATCH": self.ip_country_mismatch,
            "MULTIPLE_DEVICES": self.multiple_devices,
            "SUSPICIOUS_PATTERN": self.suspicious_pattern,
            "VPN_DETECTED": self.vpn_detected,
            "KNOWN_FRAUDSTER": self.known_fraudster,
            "RAPID_DEPOSIT_WITHDRAW": self.rapid_deposit_withdraw,
            "BONUS_ABUSE": self.bonus_abuse,
            "ML_HIGH_RISK": self.ml_high_risk,
        }


@dataclass
class ScoringConfig:
    """Thresholds, rule parameters and ensemble weights (engine.go:196-228)."""
    block_threshold: int = 80
    review_threshold: int = 50
    max_tx_per_minute: int = 10
    max_tx_per_hour: int = 100          # only used by the rate limiter (redis_store.go:196-203)
    new_account_days: int = 7
    large_deposit_amount: int = 100000  # cents
    max_devices_per_day: int = 3
    max_ips_per_day: int = 5
    ml_weight: float = 0.6
    rule_weight: float = 0.4
    ml_high_risk_threshold: float = 0.7  # engine.go:285
    ml_error_score: float = 0.5          # engine.go:281
    weights: RuleWeights = field(default_factory=RuleWeights)


@dataclass
class FeatureConfig:
    """Feature-store and feature-vector shape.

    ``log_transform``: "log1p" (default for new models) or "identity" (the reference's
    stub ``log1p`` at ``onnx_model.go:193-195``, quirk Q1).
    ``sum_mode``: "sliding" (exact 1h sum from the tx ring) or "compat" (INCRBY with a
    TTL refreshed on every event, ``redis_store.go:136-138``, quirk Q8).
    """
    width: int = 30              # model input width; columns >= 30 come from the ext table
    log_transform: str = "log1p"
    sum_mode: str = "sliding"
    ring_size: int = 256         # per-account tx ring entries (exact 1m/5m/1h windows)
    hll_p: int = 8               # HyperLogLog precision (2^p one-byte registers)
    event_ring: int = 100        # per-account event history for the GRU (cfg 5)
    event_dim: int = 16
    session_ttl_s: int = 1800    # redis_store.go:157-160
    last_tx_ttl_s: int = 7 * 86400
    hll_ttl_s: int = 86400
    sum_ttl_s: int = 3600


@dataclass
class ModelConfig:
    path: str = ""
    kind: str = "auto"           # auto | onnx | heuristic | none
    input_name: str = "input"    # onnx_model.go:37
    output_name: str = "output"  # onnx_model.go:38
    precision: str = "fp32"      # dense-layer numerics on the GPU: fp32 (reference) | bf16


@dataclass
class GPUConfig:
    devices: int = 1
    max_batch: int = 8192
    wait_us: int = 200           # micro-batcher close timeout
    buckets: List[int] = field(default_factory=lambda: [64, 256, 1024, 4096, 8192])
    accounts_per_gpu: int = 1 << 20
    blacklist_capacity: int = 1 << 16
    use_graphs: bool = True
    fallback: str = "cpu"        # on GPU fault: cpu | fail
    batch_timeout_ms: int = 2000  # watchdog: a device batch slower than this marks the shard unhealthy
    # failure handling (engine/risk_engine.py): a quarantined shard whose late batches drained
    # returns to service; one still unhealthy after rehome_after_s (or any remote shard of a
    # failed SPMD group) is rebuilt on a surviving device from snapshot_dir
    auto_recover: bool = True
    rehome_after_s: float = 30.0
    rehome_grace_s: float = 5.0   # SPMD: wait this long for survivors' final snapshots
    snapshot_dir: str = ""        # where snapshots are written / re-homed shards restore from
    spmd_heartbeat_s: float = 2.0  # SPMD liveness op period (0: off)
    # native serving core (csrc/runtime/serve_core.cpp, engine/serving.py): request bytes ->
    # response bytes without Python on the hot path; the unary micro-batcher is its FIFO
    native_serving: bool = True
    serve_depth: int = 6          # pipeline slots (batches in flight) of a shard's device (<= 7; profiles/r6/ad)
    unary_depth: int = 4          # steps in flight while unary calls are arriving (ServeCore Options.unary_depth)
    serve_finishers: int = 2      # unary response threads
    exchange_timeout_s: float = 10.0  # multi-rank step deadline: a peer that misses it failed
    # native account RPCs (csrc/runtime/acct_core.cpp, engine/acct.py): PredictLTV,
    # GetPlayerSegment, CheckBonusAbuse micro-batched on the owner's model devices
    native_acct: bool = True
    acct_depth: int = 2           # pipeline slots of each account-model device


@dataclass
class ServerConfig:
    grpc_port: int = 9082        # services/risk/cmd/main.go:57
    http_port: int = 8082        # services/risk/cmd/main.go:58
    log_level: str = "info"
    shutdown_grace_s: float = 30.0
    http_timeout_s: float = 10.0
    audit_db: str = ""           # SQLite file the risk_scores audit ring drains into ("" = in-memory only)
    audit_ring_rows: int = 1 << 24  # native audit ring of the serving core (24 B/row: 384 MiB at 16.7M rows)
    audit_mode: str = "auto"     # auto | sqlite | segments (engine/audit.py)
    audit_direct_max: int = 262144  # auto: larger native backlogs go through segment files


@dataclass
class AbuseConfig:
    """CheckBonusAbuse decision threshold (engine/abuse.py documents the signal weights) and the
    native abuse device's micro-batching on a GPU shard that also scores transactions:
    ``max_batch`` caps the rows of one device step (0: the shard's largest batch bucket);
    ``cluster_kernel`` runs steps of <= 256 rows on the weight-stationary split GRU clusters
    (gru_wsx.hip), which read no weights per timestep: the batch-parallel kernel streams the
    2.5 MB weight set through L2 every timestep of every workgroup, and beside a ScoreBatch
    load that cost the scoring path 64-79 % of its throughput (profiles/r6/i);
    ``high_priority`` creates the abuse streams at high queue priority, off by default: on the
    box it made the abuse path slower, not faster - unary CheckBonusAbuse p99 391 ms at high
    priority vs 1.9 ms at normal priority with no ScoreBatch load (tools/bench_mixed.py,
    profiles/r6/f)."""
    threshold: float = 0.7
    max_batch: int = 0
    high_priority: bool = False
    cluster_kernel: bool = True
    # longest wait of a CheckBonusAbuse micro-batch for the link inserts queued before its calls
    # (acct_core.h AbuseParams.link_wait_us)
    link_wait_us: int = 200


@dataclass
class Config:
    server: ServerConfig = field(default_factory=ServerConfig)
    scoring: ScoringConfig = field(default_factory=ScoringConfig)
    features: FeatureConfig = field(default_factory=FeatureConfig)
    fraud_model: ModelConfig = field(default_factory=ModelConfig)
    ltv_model: ModelConfig = field(default_factory=ModelConfig)
    abuse_model: ModelConfig = field(default_factory=ModelConfig)
    gpu: GPUConfig = field(default_factory=GPUConfig)
    abuse: AbuseConfig = field(default_factory=AbuseConfig)

    # ------------------------------------------------------------------ loading
    @classmethod
    def load(cls, path: Optional[str] = None, env: Optional[Dict[str, str]] = None) -> "Config":
        cfg = cls()
        if path:
            import yaml
            with open(path) as f:
                data = yaml.safe_load(f) or {}
            _merge(cfg, data)
        cfg.apply_env(os.environ if env is None else env)
        cfg.validate()
        return cfg

    def apply_env(self, env) -> None:
        def geti(name, cur):
            v = env.get(name)
            if v in (None, ""):
                return cur
            # Go's fmt.Sscanf("%d") semantics: leading integer, 0 on garbage
            s = v.strip()
            digits = ""
            for i, ch in enumerate(s):
                if ch.isdigit() or (i == 0 and ch in "+-"):
                    digits += ch
                else:
                    break
            try:
                return int(digits)
            except ValueError:
                return 0

        s = self.server
        s.grpc_port = geti("GRPC_PORT", s.grpc_port)
        s.http_port = geti("HTTP_PORT", s.http_port)
        s.log_level = env.get("LOG_LEVEL", s.log_level) or s.log_level
        s.audit_db = env.get("AUDIT_DB", s.audit_db)
        s.audit_ring_rows = int(env.get("AUDIT_RING_ROWS", s.audit_ring_rows))
        s.audit_mode = env.get("AUDIT_MODE", s.audit_mode)
        s.audit_direct_max = int(env.get("AUDIT_DIRECT_MAX", s.audit_direct_max))
        sc = self.scoring
        sc.block_threshold = geti("BLOCK_THRESHOLD", sc.block_threshold)
        sc.review_threshold = geti("REVIEW_THRESHOLD", sc.review_threshold)
        sc.max_tx_per_minute = geti("MAX_TX_PER_MINUTE", sc.max_tx_per_minute)
        sc.max_tx_per_hour = geti("MAX_TX_PER_HOUR", sc.max_tx_per_hour)
        fm = env.get("FRAUD_MODEL_PATH") or env.get("MODEL_PATH")
        if fm:
            self.fraud_model.path = fm
        if env.get("LTV_MODEL_PATH"):
            self.ltv_model.path = env["LTV_MODEL_PATH"]
        if env.get("ABUSE_MODEL_PATH"):
            self.abuse_model.path = env["ABUSE_MODEL_PATH"]
        self.gpu.devices = geti("RISK_GPUS", self.gpu.devices)
        self.gpu.max_batch = geti("RISK_MAX_BATCH", self.gpu.max_batch)
        self.gpu.wait_us = geti("RISK_BATCH_WAIT_US", self.gpu.wait_us)
        self.gpu.batch_timeout_ms = geti("RISK_BATCH_TIMEOUT_MS", self.gpu.batch_timeout_ms)
        self.gpu.snapshot_dir = env.get("RISK_SNAPSHOT_DIR", self.gpu.snapshot_dir) or self.gpu.snapshot_dir
        ns = env.get("RISK_NATIVE_SERVING")
        if ns not in (None, ""):
            self.gpu.native_serving = ns.strip().lower() not in ("0", "false", "no", "off")
        na = env.get("RISK_NATIVE_ACCT")
        if na is not None:
            self.gpu.native_acct = na.strip().lower() not in ("0", "false", "no", "off")
        lt = env.get("RISK_LOG_TRANSFORM")
        if lt:
            self.features.log_transform = lt

    def validate(self) -> None:
        f = self.features
        if f.log_transform not in ("log1p", "identity"):
            raise ValueError(f"features.log_transform must be log1p|identity, got {f.log_transform!r}")
        if f.sum_mode not in ("sliding", "compat"):
            raise ValueError(f"features.sum_mode must be sliding|compat, got {f.sum_mode!r}")
        if f.ring_size % 64 != 0 or not (64 <= f.ring_size <= 4096):
            raise ValueError("features.ring_size must be a multiple of 64 in [64, 4096]")
        if f.hll_p != 8:
            raise ValueError("features.hll_p: only p=8 (256 registers, one per 4 lanes x 64) is built")
        if f.width < 30:
            raise ValueError("features.width must be >= 30 (the reference feature vector)")
        if self.gpu.max_batch > max(self.gpu.buckets):
            raise ValueError("gpu.max_batch exceeds the largest graph bucket")

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)


def _merge(obj, data: Dict[str, Any]) -> None:
    for k, v in data.items():
        if not hasattr(obj, k):
            raise KeyError(f"unknown config key {k!r} for {type(obj).__name__}")
        cur = getattr(obj, k)
        if dataclasses.is_dataclass(cur) and isinstance(v, dict):
            _merge(cur, v)
        else:
            setattr(obj, k, v)

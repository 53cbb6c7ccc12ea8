"""Feature-store auxiliary operations of the reference's Redis store and the model's feature
importance:

* ``GetVelocity`` (redis_store.go:171-193): 1 min / 5 min / 1 h transaction counts. Here they
  come from the device tx ring through K1 (the same window edges as the scoring path,
  ``>= now - w`` inclusive like ZCOUNT [min, +inf]), batched: one K1 launch per shard for many
  accounts (``backends.features_many``).
* ``CheckRateLimit`` (:196-203): count_1m >= max_per_min or count_1h >= max_per_hour; the
  defaults are the scoring config's MaxTxPerMinute / MaxTxPerHour (the only consumer of
  MaxTxPerHour in the reference, engine.go:215-228).
* ``IncrementCounter`` (:206-215), ``SetFeature`` / ``GetFeature`` (:218-227): named host
  counters and per-account string features with TTLs (:class:`KVStore`, Redis INCR+EXPIRE /
  SET with TTL / GET semantics, expiry checked on read). ``DeleteAccountFeatures`` (:230-240)
  also drops the account's named features.
* ``GetFeatureImportance`` (onnx_model.go:329-345): the reference returns a static map; here it
  is derived from the loaded model: split counts per input feature of the tree ensembles
  (XGBoost "weight" importance: the ONNX file carries no gains), otherwise the column L1 norms of
  the first dense layer; the built-in heuristic model keeps the reference's static map.
"""
from __future__ import annotations

import threading
import time
from typing import Dict, Optional, Tuple

import numpy as np

# onnx_model.go:329-345, returned verbatim for the built-in heuristic (mockPredict) model
STATIC_IMPORTANCE = {
    "is_vpn": 0.15, "is_tor": 0.12, "tx_count_1min": 0.10, "unique_devices": 0.10, "account_age": 0.09,
    "tx_amount": 0.08, "bonus_only_player": 0.08, "unique_ips": 0.07, "time_since_last": 0.06,
    "net_deposit": 0.05, "other": 0.10,
}


class KVStore:
    """Named counters and per-account features with TTLs (the reference's generic Redis keys).
    Thread-safe; expired keys read as absent and are purged lazily."""

    def __init__(self, max_keys: int = 1 << 20):
        self._d: Dict[str, Tuple[object, float]] = {}
        self._lock = threading.Lock()
        self.max_keys = int(max_keys)

    def _live(self, key: str, now: float):
        v = self._d.get(key)
        if v is None:
            return None
        if v[1] and v[1] <= now:
            del self._d[key]
            return None
        return v

    def _purge(self, now: float) -> None:
        if len(self._d) < self.max_keys:
            return
        for k in [k for k, (_, exp) in self._d.items() if exp and exp <= now]:
            del self._d[k]
        if len(self._d) >= self.max_keys:
            raise RuntimeError("KVStore full")

    def incr(self, key: str, ttl_s: float, now: Optional[float] = None) -> int:
        """INCR key; EXPIRE key ttl (both every call, like the reference pipeline)."""
        now = time.time() if now is None else now
        with self._lock:
            v = self._live(key, now)
            n = (int(v[0]) if v is not None else 0) + 1
            self._purge(now)
            self._d[key] = (n, now + ttl_s if ttl_s > 0 else 0.0)
            return n

    def set(self, key: str, value, ttl_s: float = 0.0, now: Optional[float] = None) -> None:
        now = time.time() if now is None else now
        with self._lock:
            self._purge(now)
            self._d[key] = (str(value), now + ttl_s if ttl_s > 0 else 0.0)

    def get(self, key: str, now: Optional[float] = None) -> Optional[str]:
        now = time.time() if now is None else now
        with self._lock:
            v = self._live(key, now)
            return None if v is None else str(v[0])

    def delete_prefix(self, prefix: str) -> int:
        with self._lock:
            ks = [k for k in self._d if k.startswith(prefix)]
            for k in ks:
                del self._d[k]
            return len(ks)


def feature_key(account_id: str, feature: str) -> str:
    return f"features:{account_id}:{feature}"   # redis_store.go:220


def input_names(width: int):
    from ..golden.features import MODEL_INPUT_NAMES
    return list(MODEL_INPUT_NAMES[:width]) + [f"ext_{i}" for i in range(max(width - len(MODEL_INPUT_NAMES), 0))]


def plan_importance(plan, width: int) -> Dict[str, float]:
    """Normalised importance per model input column of a compiled plan (models/plan.py)."""
    score = np.zeros(width, np.float64)
    trees = [s for s in plan.steps if s.kind == "tree"]
    if trees:
        for t in trees:
            if t.layout == "sparse":  # pointer layout: [N][4] int32 {meta, thr, left, right}, leaves mode 7
                nodes = np.asarray(t.nodes_np, np.int32).reshape(-1, 4)
                meta = nodes[:, 0].view(np.uint32)
                feat = meta[((meta >> 16) & 7) != 7] & 0xFFFF
            else:  # complete layout: [T][2^D-1][2] f32 {thr, meta}, padding nodes have +inf thresholds
                nodes = np.asarray(t.nodes_np, np.float32).reshape(-1, 2)
                real = np.isfinite(nodes[:, 0])
                feat = nodes[:, 1].view(np.uint32)[real] & 0xFFFF
            score += np.bincount(feat.astype(np.int64), minlength=width)[:width]
    else:
        first = next((s for s in plan.steps if s.kind in ("dense", "head")), None)
        if first is not None:
            w = first.w1_np if first.kind == "head" else first.w_np   # [N, K]
            score[:min(width, w.shape[1])] = np.abs(w).sum(axis=0)[:width]
    tot = score.sum()
    names = input_names(width)
    if tot <= 0:
        return {}
    out = {names[i]: float(score[i] / tot) for i in np.argsort(-score) if score[i] > 0}
    return out

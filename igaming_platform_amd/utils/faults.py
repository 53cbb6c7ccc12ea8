"""Fault injection hooks: ``FAULT_INJECT="backend_error:shard=0,model_error"``.

Names used by the engine: ``backend_error`` (a shard's scoring step raises -> the shard is
marked unhealthy and its rows go to the CPU fallback), ``gpu_timeout:ms=N`` (a real N ms
device stall is queued ahead of the shard's batch, so the watchdog deadline fires),
``model_error`` (ML fails -> ml_error_score, engine.go:279-282),
``feature_store_down`` (features unavailable -> partial features, engine.go:267-270),
``xchg_stall_results:file=P`` (once file P exists, a CPU exchange owner keeps stepping but
stops publishing its results: its peers' steps fail at the deadline, then the group fails
over; tests/test_failover.py).
"""
from __future__ import annotations

import os
import threading
from typing import Dict, Optional


class Faults:
    def __init__(self, spec: Optional[str] = None):
        self._lock = threading.Lock()
        self._active: Dict[str, Dict[str, str]] = {}
        self.load(os.environ.get("FAULT_INJECT", "") if spec is None else spec)

    def load(self, spec: str) -> None:
        with self._lock:
            self._active.clear()
            for item in filter(None, (s.strip() for s in spec.split(","))):
                name, _, args = item.partition(":")
                kv = {}
                for a in filter(None, args.split(";")):
                    k, _, v = a.partition("=")
                    kv[k.strip()] = v.strip()
                self._active[name.strip()] = kv

    def set(self, name: str, **kv) -> None:
        with self._lock:
            self._active[name] = {k: str(v) for k, v in kv.items()}

    def clear(self, name: Optional[str] = None) -> None:
        with self._lock:
            if name is None:
                self._active.clear()
            else:
                self._active.pop(name, None)

    def params(self, name: str) -> Dict[str, str]:
        with self._lock:
            return dict(self._active.get(name, {}))

    def any_active(self) -> bool:
        with self._lock:
            return bool(self._active)

    def active(self, name: str, **match) -> bool:
        with self._lock:
            kv = self._active.get(name)
            if kv is None:
                return False
            return all(k not in kv or kv[k] == str(v) for k, v in match.items())


class InjectedFault(RuntimeError):
    pass

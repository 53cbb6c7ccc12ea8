"""Native serving: the scoring hot path as one GIL-free C++ pipeline per shard.

``_native.ServeCore`` (csrc/runtime/serve_core.cpp) takes raw risk.v1 request bytes and
returns response bytes: wire parse -> AccountIndex resolve -> owner sort -> a FIFO of work
items -> device micro-batches (a stepper thread packs the pinned slab and launches the slot
through the device's C function table, csrc/include/device_ops.h) -> a completion thread
waits for slots in order -> callers copy their result rows and serialise. Unary
ScoreTransaction calls are 1-row items of the same FIFO (the micro-batcher), answered
through a completion queue the gRPC layer polls.

Devices (``device_ops()`` owners):

* the single-GPU pipeline (engine/scorer.py ``PipeDriver``)
* the owner-routed RCCL exchange of a multi-rank group (engine/dp.py ``XchgDriver``): every
  rank ingests; ranks keep their step sequences aligned through a ``StepClock`` in
  /dev/shm (no host collective per step)
* CPU shards: ``CpuDevice`` (one shard) and ``ShmXchgDevice`` (a CPU rank of a multi-process
  group, the exchange over /dev/shm)

Reference: the hot path it replaces is ``ScoringEngine.Score``
(services/risk/internal/scoring/engine.go:262-323) behind the gRPC handler the reference
never registers (services/risk/cmd/main.go:142); its only scaling story is "horizontal
scaling with stateless services" (README.md:157-160).
"""
from __future__ import annotations

import os
import secrets
from typing import Optional, Sequence

from ..native import native


class XchgDevice:
    """``device_ops()`` of a data-parallel scorer's exchange driver at chunk capacity C."""

    def __init__(self, scorer, C: int):
        self.scorer, self.C = scorer, int(C)

    def device_ops(self) -> int:
        return self.scorer.xdriver.device_ops(self.C)


def gpu_device(scorer):
    """The device object of a GPU scorer for the serving core (None: no native driver)."""
    if getattr(scorer, "xdriver", None) is not None:
        return XchgDevice(scorer, scorer.cbuckets[-1])
    d = getattr(scorer, "driver", None)
    return d


def make_core(indexes: Sequence, device, cfg, rank: int = 0, clock=None, seq0: int = 0, features: bool = True):
    g = cfg.gpu
    timeout_us = int(g.batch_timeout_ms * 1000) if g.batch_timeout_ms > 0 else -1
    return native().ServeCore(list(indexes), device, rank, clock, max_wait_us=int(g.wait_us), timeout_us=timeout_us,
                               finishers=int(g.serve_finishers), features=features, seq0=int(seq0),
                               unary_depth=int(g.unary_depth))


def shm_token() -> str:
    """A fresh name prefix for the /dev/shm regions of one serving group."""
    return f"igp-{os.getpid()}-{secrets.token_hex(4)}"


def core_metrics(core) -> Optional[dict]:
    """Decision counters of a core (cumulative) for /metrics."""
    if core is None:
        return None
    s = core.stats(False)
    return dict(deciles=list(s["deciles"]), actions=list(s["actions"]), ml_high=int(s["ml_high"]),
                blacklisted=int(s["blacklisted"]), scored=int(s["scored"]))

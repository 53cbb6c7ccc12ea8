"""CheckBonusAbuse service (risk.proto:135-145).

The reference defines the RPC and calls it from the bonus engine (bonus_engine.go:268-275)
but has no server implementation, so the semantics here are this framework's own, built
from signals the reference already computes:

* rule signals from the account's live feature row (K1 on a synthetic request):
  BONUS_ONLY_PLAYER (engine.go:384-386), LOW_WAGER_COMPLETION, MULTIPLE_DEVICES /
  MULTIPLE_IPS (the rule-3/4 limits), VPN_PROXY_TOR, HIGH_VELOCITY (rule-1 limit);
* SHARED_DEVICE / MULTI_ACCOUNT from the device<->account link index (linked_accounts);
* SEQUENCE_MODEL: config 5's GRU (2x256 over the last 100 events, K4 reading the HBM
  event ring directly) when an abuse model is loaded.

abuse_score = max(rule score, model score) when a model is present, else the rule score;
rule score = min(1, sum of the weights of the signals that fired). is_abuser: score >= threshold.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..layouts import FR_BONUS_ONLY, FR_PROXY, FR_TOR, FR_VPN

SIGNAL_WEIGHTS: Dict[str, float] = {
    "BONUS_ONLY_PLAYER": 0.35,
    "LOW_WAGER_COMPLETION": 0.2,
    "MULTIPLE_DEVICES": 0.15,
    "MULTIPLE_IPS": 0.1,
    "VPN_PROXY_TOR": 0.1,
    "HIGH_VELOCITY": 0.1,
    "SHARED_DEVICE": 0.25,
    "SEQUENCE_MODEL": 0.0,   # contributes through the model score
}


@dataclass
class AbuseResult:
    is_abuser: bool
    abuse_score: float
    signals: List[str] = field(default_factory=list)
    linked_accounts: List[str] = field(default_factory=list)
    model_score: Optional[float] = None


def rule_signals(feat, scoring, n_linked: int) -> List[str]:
    s = []
    flags = int(feat["flags"])
    if flags & FR_BONUS_ONLY:
        s.append("BONUS_ONLY_PLAYER")
    if int(feat["bonus_claim_count"]) > 0 and float(feat["bonus_wager_completion_rate"]) < 0.3:
        s.append("LOW_WAGER_COMPLETION")
    if int(feat["unique_devices_24h"]) > scoring.max_devices_per_day:
        s.append("MULTIPLE_DEVICES")
    if int(feat["unique_ips_24h"]) > scoring.max_ips_per_day:
        s.append("MULTIPLE_IPS")
    if flags & (FR_VPN | FR_PROXY | FR_TOR):
        s.append("VPN_PROXY_TOR")
    if int(feat["tx_count_1m"]) > scoring.max_tx_per_minute:
        s.append("HIGH_VELOCITY")
    if n_linked > 0:
        s.append("SHARED_DEVICE")
    return s


class AbuseGpu:
    """K4 over the event rings of one GPU shard, one launch per batch of slots."""

    def __init__(self, store, plan, bmax: int = 8192):
        import torch
        from ..ops import kernels as K
        self.torch, self.K = torch, K
        self.store = store
        self.device = store.device
        steps = plan.steps
        n = sum(1 for s in steps if s.kind == "gru")
        head = steps[n] if n < len(steps) else None
        self.gp = K.GruPack(steps[:n], head, self.device)
        if self.gp.head_w is None:
            raise ValueError("abuse model must end in an N=1 head (probability)")
        self.T = steps[0].seq or store.ev.shape[1]
        if self.T > store.ev.shape[1]:
            raise ValueError(f"abuse model sequence length {self.T} exceeds the event ring {store.ev.shape[1]}")
        self.bmax = bmax
        self.slots = torch.zeros(bmax, dtype=torch.int32, device=self.device)
        self.out = torch.zeros(bmax, dtype=torch.float32, device=self.device)
        self.stream = torch.cuda.Stream(device=self.device)
        self._lock = threading.Lock()

    def launch(self, n: int) -> None:
        self.K.gru(self.gp, n, self.T, out=self.out, store=self.store, slots=self.slots)

    def score_slots(self, slots: np.ndarray) -> np.ndarray:
        torch = self.torch
        res = []
        with self._lock:
            for i in range(0, len(slots), self.bmax):
                chunk = np.ascontiguousarray(slots[i:i + self.bmax], np.int32)
                with torch.cuda.stream(self.stream):
                    self.slots[:len(chunk)].copy_(torch.from_numpy(chunk), non_blocking=False)
                    self.launch(len(chunk))
                    r = self.out[:len(chunk)].cpu()
                res.append(r.numpy())
        return np.concatenate(res) if res else np.zeros(0, np.float32)


class AbuseService:
    def __init__(self, engine, threshold: float = 0.7, gpu: Optional[List[AbuseGpu]] = None, executor=None,
                 input_name: str = "input", output_name: str = "output", group=None, group_model: bool = False):
        self.engine = engine
        self.group = group              # SPMD: the GRU runs on the rank that owns the account
        self.group_model = group_model
        self.threshold = float(threshold)
        self.gpu = gpu
        self.executor = executor
        self.input_name, self.output_name = input_name, output_name

    @property
    def has_model(self) -> bool:
        return self.gpu is not None or self.executor is not None or self.group_model

    def model_scores(self, owner: int, slots: np.ndarray) -> Optional[np.ndarray]:
        if self.group_model:
            return self.group.abuse_scores(slots, np.full(len(slots), owner, np.int32))
        if self.gpu is not None:
            return self.gpu[owner % len(self.gpu)].score_slots(slots)
        if self.executor is not None:
            be = self.engine.backends[owner]
            X = np.stack([be.event_history(int(s)) if s >= 0 else np.zeros_like(be.event_history(0))
                          for s in slots], axis=1)
            y = self.executor.run({self.input_name: X.astype(np.float32)})
            return np.asarray(y.get(self.output_name, list(y.values())[-1]), np.float32).reshape(-1)
        return None

    def check(self, account_ids: Sequence[str], now: int) -> List[AbuseResult]:
        eng = self.engine
        slots, owners = eng.registry.resolve_ids(list(account_ids), insert=False)
        out: List[Optional[AbuseResult]] = [None] * len(account_ids)
        for o in np.unique(owners):
            sel = np.nonzero(owners == o)[0]
            ms = self.model_scores(int(o), slots[sel]) if self.has_model else None
            for k, i in enumerate(sel):
                s = int(slots[i])
                if s < 0:
                    out[i] = AbuseResult(False, 0.0, [], [])
                    continue
                feat = eng.backends[int(o)].features(s, now)
                linked = eng.linked_accounts(int(o), s)
                sig = rule_signals(feat, eng.scoring, len(linked))
                score = min(1.0, sum(SIGNAL_WEIGHTS[x] for x in sig))
                mscore = None
                if ms is not None:
                    mscore = float(ms[k])
                    if mscore >= self.threshold:
                        sig.append("SEQUENCE_MODEL")
                    score = max(score, mscore)
                out[i] = AbuseResult(score >= self.threshold, float(score), sig, linked, mscore)
        return out  # type: ignore[return-value]

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

import os
import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..layouts import FR_BONUS_ONLY, FR_PROXY, FR_TOR, FR_VPN
from ..obs.logging import get_logger

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


def rule_signal_columns(feats: np.ndarray, scoring) -> Dict[str, np.ndarray]:
    """The rule signals of :func:`rule_signals` for a whole FEATREC batch (numpy columns)."""
    flags = feats["flags"].astype(np.int64)
    return {
        "BONUS_ONLY_PLAYER": (flags & FR_BONUS_ONLY) != 0,
        "LOW_WAGER_COMPLETION": (feats["bonus_claim_count"] > 0) & (feats["bonus_wager_completion_rate"] < 0.3),
        "MULTIPLE_DEVICES": feats["unique_devices_24h"] > scoring.max_devices_per_day,
        "MULTIPLE_IPS": feats["unique_ips_24h"] > scoring.max_ips_per_day,
        "VPN_PROXY_TOR": (flags & (FR_VPN | FR_PROXY | FR_TOR)) != 0,
        "HIGH_VELOCITY": feats["tx_count_1m"] > scoring.max_tx_per_minute,
    }


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


log = get_logger("abuse")


class AbuseGpu:
    """K4 over the HBM event rings of one GPU shard. Requests carry only slots; one captured
    hipGraph per bucket: H2D [n | slots] -> fused 2-layer GRU + head (reads the rings) -> D2H."""

    def __init__(self, store, plan, bmax: int = 8192, buckets: Sequence[int] = (), use_graphs: bool = True,
                 depth: int = 2, overlap: bool = False):
        import torch
        from ..ops import kernels as K
        self.torch, self.K = torch, K
        self.store = store
        self.device = store.device
        # the shard's _native.StateClock when it also scores (engine/backends.py wait_state): each
        # batch then reads the store after every scoring batch issued before it
        self.state_clock = None
        steps = plan.steps
        from .runner import GruModel
        # fp32 plans (the ONNX f32 contract, default): the f32-faithful split GRU; bf16 plans: bf16 MFMA
        bmax_ = max([int(b) for b in buckets] or [bmax])
        self.gm = GruModel(steps, self.device, getattr(plan, "precision", "fp32") != "bf16", bmax_)
        if not self.gm.has_head:
            raise ValueError("abuse model must end in an N=1 head (probability)")
        self.gp = self.gm.packs[0]  # (the weight-stationary path and its fallback live on this pack)
        self.T = steps[0].seq or store.ev.shape[1]
        if self.T > store.ev.shape[1]:
            raise ValueError(f"abuse model sequence length {self.T} exceeds the event ring {store.ev.shape[1]}")
        self.buckets = sorted(set(int(b) for b in (buckets or [bmax])))
        B = self.bmax = self.buckets[-1]
        dev = self.device
        self.depth = depth
        # overlap (a process whose only device work is this model, e.g. the cfg5 bench): one
        # stream per pipeline slot (own device slab / output), so the next slot's batch runs
        # beside a batch-parallel launch that leaves CUs free (the 32-row split GRU fills 128 of
        # 256 CUs at 4096 rows). The weight-stationary cluster kernel needs the whole chip
        # co-resident and a bidirectional model shares its intermediates: both stay on one
        # stream, as does a serving rank (its streams are budgeted to the 4 hardware queues,
        # engine/dp.py).
        multi = overlap and not self.gp.ws_ok and not self.gm.bidirectional and depth > 1
        if multi:
            # the split cluster kernel (gru_wsx) keeps one workspace per pack (counters, hand-off
            # slab, head partials): launches on several streams at once would share it (ADVICE
            # r5), so with one stream per slot every bucket runs the batch-parallel kernel
            for gp in self.gm.packs:
                gp.wsx_ok = False
        self.n_streams = depth if multi else 1
        if self.gm.split:  # 32-row split tiles leave half the chip to the next slot's batch
            rows = int(os.environ.get("IGP_GRU_X3_ROWS", "32" if multi else "16"))
            for gp in self.gm.packs:
                gp.x3_rows = rows
        self.dev_slabs = [torch.zeros(16 + 4 * B, dtype=torch.uint8, device=dev) for _ in range(self.n_streams)]
        self.outs = [torch.zeros(B, dtype=torch.float32, device=dev) for _ in range(self.n_streams)]
        self.streams = [torch.cuda.Stream(device=dev) for _ in range(self.n_streams)]
        self.dev_slab, self.out, self.stream = self.dev_slabs[0], self.outs[0], self.streams[0]
        self.host = [torch.zeros(16 + 4 * B, dtype=torch.uint8).pin_memory() for _ in range(depth)]
        self.host_out = [torch.zeros(B, dtype=torch.float32).pin_memory() for _ in range(depth)]
        self.graphs: Dict[tuple, object] = {}
        self.use_graphs = use_graphs
        self._slot = 0
        self._lock = threading.Lock()
        self._slot_locks = [threading.Lock() for _ in range(depth)]

    def slot_stream(self, slot: int):
        return self.streams[slot % self.n_streams]

    def slot_out(self, slot: int):
        return self.outs[slot % self.n_streams]

    def _body(self, slot: int, b: int) -> None:
        slab, out = self.dev_slabs[slot % self.n_streams], self.outs[slot % self.n_streams]
        slab[:16 + 4 * b].copy_(self.host[slot][:16 + 4 * b], non_blocking=True)
        self.gm.run(b, self.T, out, store=self.store, slots=slab[16:].view(self.torch.int32),
                    m_ptr=slab[:4].view(self.torch.int32))
        self.host_out[slot][:b].copy_(out[:b], non_blocking=True)

    def _pack(self, slot: int, slots: np.ndarray, b: int) -> None:
        h = self.host[slot].numpy()
        h[:4].view(np.int32)[0] = len(slots)
        v = h[16:16 + 4 * b].view(np.int32)
        v[:len(slots)] = slots
        v[len(slots):] = -1

    def capture(self) -> None:
        torch = self.torch
        if not self.use_graphs:
            return
        with torch.cuda.device(self.device):
            for b in self.buckets:
                for slot in range(self.depth):
                    self._pack(slot, np.zeros(0, np.int32), b)
                    s = self.slot_stream(slot)  # capture on the replay stream: no extra streams / queues
                    s.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(s):
                        self._body(slot, b)
                    torch.cuda.current_stream().wait_stream(s)
                    g = torch.cuda.CUDAGraph()
                    with self.K.graph_capture(g, s):
                        self._body(slot, b)
                    self.graphs[(b, slot)] = g
            torch.cuda.synchronize(self.device)

    def bucket_for(self, n: int) -> int:
        for b in self.buckets:
            if n <= b:
                return b
        raise ValueError(f"abuse batch of {n} exceeds {self.bmax}")

    def next_slot(self) -> int:
        with self._lock:
            s = self._slot
            self._slot = (self._slot + 1) % self.depth
        return s

    def submit_packed(self, slot: int, n: int):
        torch = self.torch
        b = self.bucket_for(max(n, 1))
        st = self.slot_stream(slot)
        with torch.cuda.stream(st):
            if self.state_clock is not None:
                self.state_clock.wait(st.cuda_stream)
            g = self.graphs.get((b, slot))
            if g is not None:
                g.replay()
            else:
                self._body(slot, b)
            ev = torch.cuda.Event()
            ev.record(st)
        return slot, n, ev

    def submit(self, slots: np.ndarray):
        slot = self.next_slot()
        self._slot_locks[slot].acquire()
        self._pack(slot, np.asarray(slots, np.int32), self.bucket_for(max(len(slots), 1)))
        with self._lock:
            return self.submit_packed(slot, len(slots))

    def wait(self, p, release: bool = True) -> np.ndarray:
        slot, n, ev = p
        try:
            ev.synchronize()
            out = self.host_out[slot][:n].numpy().copy()
            if (self.gp.ws_ok or self.gp.wsx_ok) and n and np.isnan(out).any():
                out = self._ws_fallback(slot, n)
            return out
        finally:
            if release:
                self._slot_locks[slot].release()

    def _ws_fallback(self, slot: int, n: int) -> np.ndarray:
        """A weight-stationary cluster launch gave up (its workgroups were not co-resident):
        switch this model to the batch-parallel K4, re-capture, and recompute the batch."""
        torch = self.torch
        log.error("abuse GRU: cluster kernel timed out; falling back to the batch-parallel kernel")
        with self._lock:
            torch.cuda.synchronize(self.device)
            self.gp.disable_ws()
            b = self.bucket_for(max(n, 1))
            with torch.cuda.stream(self.slot_stream(slot)):
                self._body(slot, b)
            self.slot_stream(slot).synchronize()
            out = self.host_out[slot][:n].numpy().copy()
            self.graphs.clear()
            self.capture()
        return out

    def score_slots(self, slots: np.ndarray) -> np.ndarray:
        out = [self.wait(self.submit(slots[i:i + self.bmax])) for i in range(0, len(slots), self.bmax)]
        return np.concatenate(out) if out else np.zeros(0, np.float32)


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
            g = self.gpu[owner % len(self.gpu)]
            return g.score_slots(slots) if g is not None else None  # None: shard being re-homed
        if self.executor is not None:
            be = self.engine.backends[owner]
            X = np.stack([be.event_history(int(s)) if s >= 0 else np.zeros_like(be.event_history(0))
                          for s in slots], axis=1)
            y = self.executor.run({self.input_name: X.astype(np.float32)})
            return np.asarray(y.get(self.output_name, list(y.values())[-1]), np.float32).reshape(-1)
        return None

    def check(self, account_ids: Sequence[str], now: int) -> List[AbuseResult]:
        """Batched: per owner shard ONE feature read (K1 over all the batch's accounts) and ONE
        GRU launch (cfg 5's model over their event rings), then the host-side signals."""
        eng = self.engine
        slots, owners = eng.registry.resolve_ids(list(account_ids), insert=False)
        out: List[Optional[AbuseResult]] = [None] * len(account_ids)
        for o in np.unique(owners):
            sel = np.nonzero(owners == o)[0]
            if not eng.healthy[int(o)]:  # shard lost with its worker / quarantined: no state to check
                for i in sel.tolist():
                    out[i] = AbuseResult(False, 0.0, [], [])
                continue
            ms = self.model_scores(int(o), slots[sel]) if self.has_model else None
            known = slots[sel] >= 0
            cols = {}
            if known.any():
                feats = eng.backends[int(o)].features_many(slots[sel][known], now)
                cols = {k: v.tolist() for k, v in rule_signal_columns(feats, eng.scoring).items()}
            fi = (np.cumsum(known) - 1).tolist()
            if known.any():
                eng._flush_links()
            for k, i in enumerate(sel.tolist()):
                s = int(slots[i])
                if s < 0:
                    out[i] = AbuseResult(False, 0.0, [], [])
                    continue
                linked = eng.linked_accounts(int(o), s, flush=False)
                sig = [name for name, col in cols.items() if col[fi[k]]]
                if linked:
                    sig.append("SHARED_DEVICE")
                score = min(1.0, sum(SIGNAL_WEIGHTS[x] for x in sig))
                mscore = None
                if ms is not None:
                    mscore = float(ms[k])
                    if mscore >= self.threshold:
                        sig.append("SEQUENCE_MODEL")
                    score = max(score, mscore)
                out[i] = AbuseResult(score >= self.threshold, float(score), sig, linked, mscore)
        return out  # type: ignore[return-value]

"""PredictLTV / GetPlayerSegment service (risk.proto:95-129).

Reference: ``LTVPredictor`` (services/risk/internal/prediction/ltv.go:113-151) reads a
``PlayerDataSource`` that has no implementation anywhere in the reference. Here the player
profile is a host-resident table (one row of ``golden.ltv.PLAYER_COLUMNS`` per account,
loaded by the warehouse job / ``set_players``), and prediction runs:

* GPU (:class:`LtvGpu`): one captured hipGraph per batch bucket —
  H2D [model input | player rows] -> optional learned LTV model (config 4: MLP 4x512 on
  MFMA, ``DeviceModel``) -> K9 ``ltv_segment`` (churn, segment, survival, confidence, NBA,
  with the model output replacing the formula LTV before the churn adjustment) -> D2H.
* CPU: the golden float64 formula (+ the model through the C++ executor).

The learned model's input row is :func:`ltv_model_input`: signed log1p of the 25 profile
columns followed by the account's extra LTV features (zeros when none are loaded).
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..golden import ltv as GL

N_COLS = len(GL.PLAYER_COLUMNS)


def ltv_model_input(pf: np.ndarray, ext: Optional[np.ndarray], width: int) -> np.ndarray:
    pf = np.asarray(pf, np.float32).reshape(-1, N_COLS)
    x = np.zeros((len(pf), width), np.float32)
    x[:, :N_COLS] = np.sign(pf) * np.log1p(np.abs(pf))
    if ext is not None and width > N_COLS:
        e = np.asarray(ext, np.float32).reshape(len(pf), -1)
        w = min(e.shape[1], width - N_COLS)
        x[:, N_COLS:N_COLS + w] = e[:, :w]
    return x


@dataclass
class LtvResult:
    account_id: str
    predicted_ltv: float
    segment: int
    churn_risk: float
    survival_days: int
    confidence: float
    next_best_action: str
    found: bool = True

    def recommended_actions(self) -> List[str]:
        return recommended_from(self.segment, self.next_best_action)


def recommended_from(seg: int, nba: str) -> List[str]:
    """GetPlayerSegment.recommended_actions: the NBA first, then the segment's playbook."""
    acts = [nba]
    for a in GL.SEGMENT_PLAYBOOK.get(seg, []):
        if a not in acts:
            acts.append(a)
    return acts


class PlayerTable:
    """Host player-profile rows keyed by (owner, slot) of the account registry."""

    def __init__(self, capacity: int, world: int = 1, ext_width: int = 0):
        self.rows = [np.zeros((capacity, N_COLS), np.float32) for _ in range(world)]
        self.present = [np.zeros(capacity, bool) for _ in range(world)]
        self.ext = [np.zeros((capacity, ext_width), np.float32) if ext_width else None for _ in range(world)]
        self.lock = threading.Lock()

    def set(self, owner: int, slots: np.ndarray, rows: np.ndarray, ext: Optional[np.ndarray] = None) -> None:
        with self.lock:
            self.rows[owner][slots] = rows
            self.present[owner][slots] = True
            if ext is not None and self.ext[owner] is not None:
                self.ext[owner][slots] = ext[:, : self.ext[owner].shape[1]]

    def get(self, owner: int, slots: np.ndarray):
        with self.lock:
            ok = (slots >= 0)
            s = np.where(ok, slots, 0)
            rows = self.rows[owner][s].copy()
            present = self.present[owner][s] & ok
            ext = self.ext[owner][s].copy() if self.ext[owner] is not None else None
        rows[~present] = 0
        return rows, present, ext


class LtvGpu:
    """Graph-captured K3 (optional model) + K9 pipeline on one GPU."""

    def __init__(self, device, plan=None, buckets: Sequence[int] = (64, 256, 1024, 4096, 8192),
                 in_width: int = 0, use_graphs: bool = True, depth: int = 2):
        import torch
        from ..ops import kernels as K
        from .runner import DeviceModel
        self.torch, self.K = torch, K
        self.device = K.as_device(device)
        self.buckets = sorted(set(int(b) for b in buckets))
        B = self.buckets[-1]
        self.bmax = B
        self.plan = plan
        self.in_width = (plan.in_width if plan is not None else 0) or in_width
        self.model = DeviceModel(plan, self.device, self.buckets) if plan is not None else None
        if self.model is not None and plan.out_width < 1:
            raise ValueError("LTV model must produce at least one output column")
        dev = self.device
        self.w = self.in_width
        row_bytes = 4 * (self.w + N_COLS)
        self.slab_bytes = 16 + row_bytes * B
        self.dev_slab = torch.zeros(self.slab_bytes, dtype=torch.uint8, device=dev)
        self.n_ptr = self.dev_slab[:4].view(torch.int32)
        self.depth = depth
        self.host = [torch.zeros(self.slab_bytes, dtype=torch.uint8).pin_memory() for _ in range(depth)]
        self.host_out = [torch.zeros((B, 6), dtype=torch.float32).pin_memory() for _ in range(depth)]
        self.out = torch.zeros((B, 6), dtype=torch.float32, device=dev)
        self.stream = torch.cuda.Stream(device=dev)
        self.graphs: Dict[tuple, object] = {}
        self._slot = 0
        self.use_graphs = use_graphs
        self._lock = threading.Lock()

    def _views(self, b: int):
        t = self.torch
        X = self.dev_slab[16:16 + 4 * self.w * b].view(t.float32).view(b, self.w) if self.w else None
        off = 16 + 4 * self.w * b
        pf = self.dev_slab[off: off + 4 * N_COLS * b].view(t.float32).view(b, N_COLS)
        return X, pf

    def _body(self, slot: int, b: int) -> None:
        nbytes = 16 + 4 * (self.w + N_COLS) * b
        self.dev_slab[:nbytes].copy_(self.host[slot][:nbytes], non_blocking=True)
        X, pf = self._views(b)
        ml = None
        if self.model is not None:
            y = self.model.run(X, b, m_ptr=self.n_ptr)
            ml = y[:b, 0] if y.shape[1] == 1 else y[:b, 0].contiguous()
        self.K.ltv(pf, self.out[:b], model_ltv=ml)
        self.host_out[slot][:b].copy_(self.out[:b], non_blocking=True)

    def capture(self) -> None:
        torch = self.torch
        if not self.use_graphs:
            return
        with torch.cuda.device(self.device):
            for b in self.buckets:
                for slot in range(self.depth):
                    s = torch.cuda.Stream(device=self.device)
                    s.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(s):
                        self._body(slot, b)
                    torch.cuda.current_stream().wait_stream(s)
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=s):
                        self._body(slot, b)
                    self.graphs[(b, slot)] = g
            torch.cuda.synchronize(self.device)

    def bucket_for(self, n: int) -> int:
        for b in self.buckets:
            if n <= b:
                return b
        raise ValueError(f"LTV batch of {n} exceeds {self.bmax}")

    def host_views(self, slot: int, b: int):
        h = self.host[slot].numpy()
        X = h[16:16 + 4 * self.w * b].view(np.float32).reshape(b, self.w) if self.w else None
        off = 16 + 4 * self.w * b
        pf = h[off: off + 4 * N_COLS * b].view(np.float32).reshape(b, N_COLS)
        return X, pf

    def submit_packed(self, slot: int, n: int):
        torch = self.torch
        b = self.bucket_for(max(n, 1))
        self.host[slot].numpy()[:4].view(np.int32)[0] = n
        with torch.cuda.stream(self.stream):
            g = self.graphs.get((b, slot))
            if g is not None:
                g.replay()
            else:
                self._body(slot, b)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return slot, n, ev

    def next_slot(self) -> int:
        s = self._slot
        self._slot = (self._slot + 1) % self.depth
        return s

    def wait(self, p) -> np.ndarray:
        slot, n, ev = p
        ev.synchronize()
        return self.host_out[slot][:n].numpy().copy()

    def predict_rows(self, pf: np.ndarray, X: Optional[np.ndarray]) -> np.ndarray:
        """[n, 25] profile rows (+ model input) -> [n, 6] (ltv, churn, survival, conf, seg, nba)."""
        out = []
        for i in range(0, max(len(pf), 1), self.bmax):
            chunk = pf[i:i + self.bmax]
            n = len(chunk)
            with self._lock:
                slot = self.next_slot()
                b = self.bucket_for(max(n, 1))
                hx, hp = self.host_views(slot, b)
                hp[:n] = chunk
                hp[n:] = 0
                if hx is not None:
                    hx[:n] = X[i:i + n] if X is not None else 0
                    hx[n:] = 0
                p = self.submit_packed(slot, n)
            out.append(self.wait(p))
        return np.concatenate(out) if out else np.zeros((0, 6), np.float32)


class LtvService:
    def __init__(self, registry, world: int = 1, gpu: Optional[List[LtvGpu]] = None, executor=None,
                 model_width: int = 0, output_name: str = "output", input_name: str = "input"):
        self.registry = registry
        self.table = PlayerTable(registry.capacity, world, ext_width=max(model_width - N_COLS, 0))
        self.gpu = gpu
        self.executor = executor
        self.model_width = model_width
        self.input_name, self.output_name = input_name, output_name

    def set_players(self, account_ids: Sequence[str], features: Sequence[GL.PlayerFeatures],
                    ext: Optional[np.ndarray] = None) -> None:
        slots, owners = self.registry.resolve_ids(list(account_ids), insert=True)
        rows = np.array([f.row() for f in features], np.float32).reshape(-1, N_COLS)
        for o in np.unique(owners):
            sel = np.nonzero((owners == o) & (slots >= 0))[0]
            self.table.set(int(o), slots[sel], rows[sel], None if ext is None else np.asarray(ext)[sel])

    def predict(self, account_ids: Sequence[str]) -> List[LtvResult]:
        slots, owners = self.registry.resolve_ids(list(account_ids), insert=False)
        out: List[Optional[LtvResult]] = [None] * len(account_ids)
        for o in np.unique(owners):
            sel = np.nonzero(owners == o)[0]
            rows, present, ext = self.table.get(int(o), slots[sel])
            X = ltv_model_input(rows, ext, self.model_width) if self.model_width else None
            if self.gpu is not None:
                res = self.gpu[int(o) % len(self.gpu)].predict_rows(rows, X)
            else:
                res = self._cpu(rows, X)
            for k, i in enumerate(sel):
                r = res[k]
                out[i] = LtvResult(account_ids[i], float(r[0]), int(r[4]), float(r[1]), int(r[2]), float(r[3]),
                                   GL.NBA_CODES[int(r[5])], found=bool(present[k]))
        return out  # type: ignore[return-value]

    def _cpu(self, rows: np.ndarray, X: Optional[np.ndarray]) -> np.ndarray:
        ml = None
        if self.executor is not None and X is not None and len(rows):
            y = self.executor.run({self.input_name: X})
            ml = np.asarray(y.get(self.output_name, list(y.values())[-1]), np.float32).reshape(len(rows), -1)[:, 0]
        res = np.zeros((len(rows), 6), np.float32)
        for k, row in enumerate(rows):
            f = GL.PlayerFeatures.from_row(row)
            p = GL.predict(f, None if ml is None else float(ml[k]))
            res[k] = (p.predicted_ltv, p.churn_risk, p.survival_days, p.confidence, p.segment,
                      GL.NBA_ID[p.next_best_action])
        return res

    def segment_players(self, account_ids: Sequence[str]) -> Dict[int, List[str]]:
        """``SegmentPlayers`` (ltv.go:401-414)."""
        groups: Dict[int, List[str]] = {}
        for r in self.predict(account_ids):
            groups.setdefault(r.segment, []).append(r.account_id)
        return groups

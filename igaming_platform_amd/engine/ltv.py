"""PredictLTV / GetPlayerSegment service (risk.proto:95-129).

Reference: ``LTVPredictor`` (services/risk/internal/prediction/ltv.go:113-151) reads a
``PlayerDataSource`` that has no implementation anywhere in the reference. Here the player
profile is a table with one row of ``golden.ltv.PLAYER_COLUMNS`` per account (loaded by
the warehouse job / ``set_players``; a host mirror plus, on GPUs, an HBM-resident copy in
the same slot space as the fraud feature store), and prediction runs:

* GPU (:class:`LtvGpu`): requests carry only slots; one captured hipGraph per bucket —
  H2D [n | slots] -> ``ltv_assemble`` (model input gathered from the HBM tables) -> learned
  LTV model (config 4: MLP 4x512 on MFMA, ``DeviceModel``) -> K9 ``ltv_segment`` (churn,
  segment, survival, confidence, NBA; the model output replaces the formula LTV before the
  churn adjustment) -> D2H [n, 6].
* CPU: the golden float64 formula (+ the model through the C++ executor).

The learned model's input row is :func:`ltv_model_input`: signed log1p of the 25 profile
columns followed by the account's extra LTV features (zeros when none are loaded).
"""
from __future__ import annotations

import os
import threading
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..golden import ltv as GL
from ..obs.logging import get_logger

N_COLS = len(GL.PLAYER_COLUMNS)



log = get_logger("ltv")

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

    def get(self, owner: int, slots: np.ndarray, with_rows: bool = True):
        """(rows, present, ext) of ``slots``; ``with_rows=False`` (GPU path: the device holds the
        tables) returns only the presence mask."""
        with self.lock:
            ok = (slots >= 0)
            s = np.where(ok, slots, 0)
            present = self.present[owner][s] & ok
            if not with_rows:
                return None, present, None
            rows = self.rows[owner][s].copy()
            ext = self.ext[owner][s].copy() if self.ext[owner] is not None else None
        rows[~present] = 0
        if ext is not None:
            ext[~present] = 0  # an empty profile has no extra features either (the device gathers zeros)
        return rows, present, ext


class LtvGpu:
    """Player profiles resident in HBM; one captured hipGraph per batch bucket:
    H2D [n | slots] -> ltv_assemble (model input gathered from the tables) -> MLP (MFMA)
    -> K9 (reads the profile rows by slot) -> D2H [n, 6]."""

    def __init__(self, device, capacity: int, plan=None, buckets: Sequence[int] = (64, 256, 1024, 4096, 8192),
                 in_width: int = 0, use_graphs: bool = True, depth: int = 2):
        import torch
        from ..ops import kernels as K
        from .runner import DeviceModel
        self.torch, self.K = torch, K
        self.device = K.as_device(device)
        self.buckets = sorted(set(int(b) for b in buckets))
        B = self.bmax = self.buckets[-1]
        self.plan = plan
        self.w = (plan.in_width if plan is not None else 0) or in_width
        if plan is not None and self.w < N_COLS:
            raise ValueError(f"LTV model input ({self.w}) must hold the {N_COLS} profile columns")
        self.model = DeviceModel(plan, self.device, self.buckets) if plan is not None else None
        # a dense chain (cfg 4: 256 -> 4 x 512 -> 1) runs as ONE fused kernel with the table
        # gather and K9 in it (csrc/kernels/mlp_fused.hip); IGP_MLP_FUSED=0: layer kernels. The
        # step replays a captured graph (recorded direct launches measured slower here: cfg4 96.4
        # vs 172.7 M/s, profiles/r2/direct3; the native account device records them instead)
        self.chain = None
        # the fused chain (mlp_fused.hip): bf16 plans as bf16 MFMA, fp32 plans in its split
        # mode (bf16 hi/lo pairs, three MFMAs per product: f32-faithful); IGP_MLP_SPLIT=0 sends
        # fp32 plans to the per-layer f32 MFMA kernels instead
        split_ok = os.environ.get("IGP_MLP_SPLIT", "1") != "0"
        if (plan is not None and (plan.precision == "bf16" or split_ok) and os.environ.get("IGP_MLP_FUSED", "1") != "0"
                and K.MlpChainPack.eligible(plan.steps)):
            self.chain = K.MlpChainPack(plan.steps, self.device, split=plan.precision != "bf16")
        dev = self.device
        self.capacity = int(capacity)
        self.pf_tab = torch.zeros((self.capacity, N_COLS), dtype=torch.float32, device=dev)
        self.ext_w = max(self.w - N_COLS, 0) if plan is not None else 0
        self.ext_tab = torch.zeros((self.capacity, self.ext_w), dtype=torch.float32, device=dev) if self.ext_w else None
        self.X = torch.zeros((B, self.w), dtype=torch.float32, device=dev) if plan is not None else None
        self.depth = depth
        self.host = [torch.zeros(16 + 4 * B, dtype=torch.uint8).pin_memory() for _ in range(depth)]
        self.host_out = [torch.zeros((B, 6), dtype=torch.float32).pin_memory() for _ in range(depth)]
        # the fused chain keeps no state between launches: each pipeline slot gets its own device
        # buffers and stream, so batch i+1's H2D / kernel overlap batch i's kernel / D2H (the
        # layer-kernel path shares the DeviceModel activations and stays on one stream)
        n_bufs = depth if self.chain is not None else 1
        # the chain's K9 epilogue stores each row's 6 outputs into the slot's pinned host buffer
        # (24 B per row through the fabric) instead of device memory + a D2H copy kernel: cfg4
        # fp32 124-129 -> 136-137 M/s, bf16 189-190 -> 200 M/s (profiles/r3/zb). 0: the copy
        self._host_out = self.chain is not None and os.environ.get("IGP_LTV_HOST_OUT", "1") == "1"
        # IGP_LTV_HOST_IN=1: the chain also reads the request slab ([n | slots], 4 B per row) from
        # the slot's pinned buffer, skipping the H2D copy (the slot lock keeps it unchanged until
        # the batch was waited for)
        self._host_in = self._host_out and os.environ.get("IGP_LTV_HOST_IN", "0") == "1"
        self._slabs = [torch.zeros(16 + 4 * B, dtype=torch.uint8, device=dev) for _ in range(n_bufs)]
        self._outs = [torch.zeros((B, 6), dtype=torch.float32, device=dev) for _ in range(n_bufs)]
        self._streams = [torch.cuda.Stream(device=dev) for _ in range(n_bufs)]
        self._use(0)
        self.graphs: Dict[tuple, object] = {}
        self._slot = 0
        self.use_graphs = use_graphs
        self._lock = threading.Lock()
        self._slot_locks = [threading.Lock() for _ in range(depth)]

    def _use(self, slot: int) -> None:
        """Point the step buffers at pipeline slot ``slot``'s (a no-op with one buffer set)."""
        i = slot % len(self._slabs)
        self.dev_slab, self.out, self.stream = self._slabs[i], self._outs[i], self._streams[i]
        self.n_ptr = self.dev_slab[:4].view(self.torch.int32)
        self.slots = self.dev_slab[16:].view(self.torch.int32)

    # ---- tables
    def set_rows(self, slots: np.ndarray, rows: np.ndarray, ext: Optional[np.ndarray] = None) -> None:
        torch = self.torch
        idx = torch.as_tensor(np.asarray(slots, np.int64), device=self.device)
        with torch.cuda.stream(self.stream):
            self.pf_tab.index_copy_(0, idx, torch.as_tensor(np.asarray(rows, np.float32), device=self.device))
            if ext is not None and self.ext_tab is not None:
                e = np.zeros((len(slots), self.ext_w), np.float32)
                w = min(self.ext_w, np.asarray(ext).shape[1])
                e[:, :w] = np.asarray(ext, np.float32)[:, :w]
                self.ext_tab.index_copy_(0, idx, torch.as_tensor(e, device=self.device))
        self.stream.synchronize()

    # ---- the step
    def _body(self, slot: int, b: int) -> None:
        K = self.K
        cp = K.memcpy_async
        if not self._host_in:
            cp(self.dev_slab, self.host[slot], 16 + 4 * b)
        nout = b * self.out.shape[1] * self.out.element_size()
        if self.chain is not None:
            ws = slot % len(self._slabs)
            def run(**kw):
                K.mlp_chain(self.chain, b, pf_tab=self.pf_tab, ext_tab=self.ext_tab, ws_key=ws, **kw)
            if self._host_out:  # the epilogue writes the slot's pinned rows: no D2H copy kernel
                if self._host_in:  # ... and the kernel reads [n | slots] from the pinned slab: no H2D
                    hs = self.host[slot]
                    run(slots=hs[16:16 + 4 * b].view(self.torch.int32), ltv_out=self.host_out[slot],
                        m_ptr=hs[:4].view(self.torch.int32))
                    return
                run(slots=self.slots, ltv_out=self.host_out[slot], m_ptr=self.n_ptr)
                return
            run(slots=self.slots, ltv_out=self.out, m_ptr=self.n_ptr)
            cp(self.host_out[slot], self.out, nout)
            return
        ml = None
        if self.model is not None:
            K.ltv_assemble(self.slots, self.pf_tab, self.ext_tab, self.X, b, m_ptr=self.n_ptr)
            y = self.model.run(self.X, b, m_ptr=self.n_ptr)
            ml = y[:b, 0]
        K.ltv(self.pf_tab, self.out, model_ltv=ml, slots=self.slots, rows=b)
        cp(self.host_out[slot], self.out, nout)

    def capture(self) -> None:
        torch = self.torch
        if not self.use_graphs:
            return
        with torch.cuda.device(self.device):
            for b in self.buckets:
                for slot in range(self.depth):
                    self._use(slot)
                    self._pack(slot, np.zeros(0, np.int32), b)
                    s = self.stream  # capture on the replay stream: no extra streams / hardware queues
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
        raise ValueError(f"LTV batch of {n} exceeds {self.bmax}")

    def _pack(self, slot: int, slots: np.ndarray, b: int) -> None:
        h = self.host[slot].numpy()
        h[:4].view(np.int32)[0] = len(slots)
        v = h[16:16 + 4 * b].view(np.int32)
        v[:len(slots)] = slots
        v[len(slots):] = -1

    def next_slot(self) -> int:
        with self._lock:
            s = self._slot
            self._slot = (self._slot + 1) % self.depth
        return s

    def submit_packed(self, slot: int, n: int):
        torch = self.torch
        b = self.bucket_for(max(n, 1))
        self._use(slot)
        with torch.cuda.stream(self.stream):
            g = self.graphs.get((b, slot))
            if g is None:
                self._body(slot, b)
            else:
                g.replay()
            ev = torch.cuda.Event()
            ev.record(self.stream)
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
            return self.host_out[slot][:n].numpy().copy()
        finally:
            if release:
                self._slot_locks[slot].release()

    def predict_slots(self, slots: np.ndarray) -> np.ndarray:
        """slots -> [n, 6] (ltv, churn, survival, confidence, segment, nba)."""
        out = [self.wait(self.submit(slots[i:i + self.bmax])) for i in range(0, max(len(slots), 1), self.bmax)]
        return np.concatenate(out) if out else np.zeros((0, 6), np.float32)


class LtvService:
    """``gpu``: the LtvGpu of each local owner (indexed owner % len). ``group`` (SPMD rank 0): the
    rows and predictions of accounts owned by other ranks go to their rank (OP_LTVROWS / OP_LTV
    over the control plane); ``rank``: the owner this process holds (SPMD)."""

    def __init__(self, registry, world: int = 1, gpu: Optional[List[LtvGpu]] = None, executor=None,
                 model_width: int = 0, output_name: str = "output", input_name: str = "input", group=None,
                 rank: Optional[int] = None):
        self.registry = registry
        self.table = PlayerTable(registry.capacity, world, ext_width=max(model_width - N_COLS, 0))
        self.gpu = gpu
        self.executor = executor
        self.model_width = model_width
        self.input_name, self.output_name = input_name, output_name
        self.group = group
        self.rank = rank

    def _remote(self, o: int) -> bool:
        return self.group is not None and self.rank is not None and int(o) != self.rank

    def set_players(self, account_ids: Sequence[str], features: Sequence[GL.PlayerFeatures],
                    ext: Optional[np.ndarray] = None) -> None:
        slots, owners = self.registry.resolve_ids(list(account_ids), insert=True)
        rows = np.array([f.row() for f in features], np.float32).reshape(-1, N_COLS)
        self.set_rows(slots, owners, rows, ext)

    def set_rows(self, slots: np.ndarray, owners: np.ndarray, rows: np.ndarray, ext=None) -> None:
        slots, owners = np.asarray(slots, np.int32), np.asarray(owners, np.int32)
        rows = np.asarray(rows, np.float32).reshape(-1, N_COLS)
        if self.group is not None and self.rank is not None:
            remote = (owners != self.rank) & (slots >= 0)
            if remote.any():  # every rank applies the rows it owns (one control-plane op)
                self.group.ltv_rows(slots[remote], owners[remote], rows[remote],
                                    None if ext is None else np.asarray(ext, np.float32)[remote])
        for o in np.unique(owners):
            if self._remote(o):
                continue
            sel = np.nonzero((owners == o) & (slots >= 0))[0]
            e = None if ext is None else np.asarray(ext)[sel]
            self.table.set(int(o), slots[sel], rows[sel], e)
            if self.gpu is not None:
                self.gpu[int(o) % len(self.gpu)].set_rows(slots[sel], rows[sel], e)

    def predict_owner_slots(self, o: int, slots: np.ndarray):
        """[n, 6] rows (ltv, churn, survival, confidence, segment, nba) of owner ``o``'s ``slots``
        on this process's shard, and the profile-present mask."""
        rows, present, ext = self.table.get(int(o), np.asarray(slots, np.int32), with_rows=self.gpu is None)
        if self.gpu is not None:
            return self.gpu[int(o) % len(self.gpu)].predict_slots(np.where(present, slots, -1)), present
        X = ltv_model_input(rows, ext, self.model_width) if self.model_width else None
        return self._cpu(rows, X), present

    def predict(self, account_ids: Sequence[str]) -> List[LtvResult]:
        slots, owners = self.registry.resolve_ids(list(account_ids), insert=False)
        out: List[Optional[LtvResult]] = [None] * len(account_ids)
        nba = GL.NBA_CODES
        for o in np.unique(owners):
            sel = np.nonzero(owners == o)[0]
            if self._remote(o):
                res, present = self.group.ltv_predict(slots[sel], np.full(len(sel), o, np.int32))
            else:
                res, present = self.predict_owner_slots(int(o), slots[sel])
            # columns -> Python scalars in bulk (tolist) before building the per-account results
            ltv, churn, surv, conf = (res[:, c].astype(np.float64).tolist() for c in (0, 1, 2, 3))
            seg, act = res[:, 4].astype(np.int64).tolist(), res[:, 5].astype(np.int64).tolist()
            pres = present.tolist()
            for k, i in enumerate(sel.tolist()):
                out[i] = LtvResult(account_ids[i], ltv[k], seg[k], churn[k], int(surv[k]), conf[k], nba[act[k]],
                                   found=pres[k])
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

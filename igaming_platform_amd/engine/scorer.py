"""GPU scoring pipeline for one MI355X (one feature shard, one model replica).

One micro-batch = one captured hipGraph replay:

  H2D  pinned slab [BatchHdr | ReqRec x n] -> device slab            (one copy)
  K1   feature_assemble (+blacklist, +ip-intel, +HLL counts, +rules) -> X, FeatRec
  K2/K3/K4  model steps of the compiled ONNX plan                      -> ml
  K5   ensemble + action (+K10 metrics histogram)                      -> ResultRec
  K6   feature_update: the batch's own transactions (score-then-update, engine.go:486-488)
  D2H  ResultRec [n] -> pinned result buffer                           (one copy)

Graphs are captured per (batch bucket, pipeline slot); a batch is padded to the smallest
bucket >= n and kernels read the live count from the device header, so padded rows are
inert. Thresholds/weights live in a device config block (``cfg_dev``): UpdateThresholds
is a 176-byte copy, never a re-capture. Pipeline slots double-buffer the pinned host
memory so the host packs batch i+1 while the GPU runs batch i.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np
import torch

from ..config import Config
from ..layouts import (BATCHHDR, FEATREC, MODEL_HEURISTIC, MODEL_NONE, MODEL_OUTPUT, REQREC, score_cfg,
                       unpack_results)
from ..models.plan import Plan
from ..ops import kernels as K
from .runner import DeviceModel

HDR_BYTES = 16
REQ_BYTES = REQREC.itemsize


@dataclass
class Pending:
    slot: int
    n: int
    bucket: int
    event: "torch.cuda.Event"
    t_submit: float
    want_features: bool


class GpuScorer:
    def __init__(self, cfg: Config, store, plan: Optional[Plan] = None, model: str = "plan",
                 device=None, pipeline_depth: int = 2, update_features: bool = True,
                 use_graphs: Optional[bool] = None, owner_filter: bool = False, rank: int = 0):
        self.cfg = cfg
        # broadcast serving (multi-GPU): every rank sees the whole batch, scores only the rows
        # whose owner byte (ReqRec.tx_type bits 8-15) is its rank, zeroes the rest
        self.owner_filter = bool(owner_filter)
        self.rank = int(rank)
        self.store = store
        self.device = K.as_device(device) if device is not None else store.device
        self.plan = plan
        if plan is None and model == "plan":
            model = "none"
        self.model = model
        self.update_features = update_features
        self.use_graphs = cfg.gpu.use_graphs if use_graphs is None else use_graphs
        self.buckets = sorted(set(int(b) for b in cfg.gpu.buckets))
        self.bmax = self.buckets[-1]
        if store.dmax < self.bmax:
            raise ValueError("store.max_events must cover the largest bucket (score-then-update)")
        self.width = cfg.features.width
        if plan is not None and plan.in_width > 0 and plan.in_width != self.width:
            raise ValueError(f"model input width {plan.in_width} != features.width {self.width}")
        dev = self.device
        B = self.bmax
        self.slab_bytes = HDR_BYTES + REQ_BYTES * B
        self.dev_slab = torch.zeros(self.slab_bytes, dtype=torch.uint8, device=dev)
        self.hdr = self.dev_slab[:HDR_BYTES].view(torch.int64)
        self.n_ptr = self.dev_slab[:4].view(torch.int32)
        self.req = self.dev_slab[HDR_BYTES:]
        self.depth = int(pipeline_depth)
        self.host_slab = [torch.zeros(self.slab_bytes, dtype=torch.uint8).pin_memory() for _ in range(self.depth)]
        self.host_slab_np = [t.numpy() for t in self.host_slab]
        self.X = torch.zeros((B, self.width), dtype=torch.float32, device=dev)
        self.feat = torch.zeros((B, 32), dtype=torch.int32, device=dev)
        self.res = torch.zeros((B, 2), dtype=torch.int32, device=dev)
        self.host_res = [torch.zeros((B, 2), dtype=torch.int32).pin_memory() for _ in range(self.depth)]
        self.host_feat = [torch.zeros((B, 32), dtype=torch.int32).pin_memory() for _ in range(self.depth)]
        self.metrics = torch.zeros(128, dtype=torch.int64, device=dev)
        self._alloc_model_buffers()
        self.cfg_dev = torch.zeros(176, dtype=torch.uint8, device=dev)
        self.refresh_config()
        self.graphs: Dict[tuple, "torch.cuda.CUDAGraph"] = {}
        self._slot = 0
        self._seq = 0
        self._lock = threading.Lock()
        self.stream = torch.cuda.Stream(device=dev)
        self.batches = 0

    # ------------------------------------------------------------------ buffers / config
    def _alloc_model_buffers(self):
        self.model_dev = None
        self.step_out: List[torch.Tensor] = []
        self.tree_partial = None
        self.tree_groups: Dict[int, int] = {}
        self.ml = None
        if self.plan is None:
            return
        if any(s.kind == "gru" for s in self.plan.steps):
            raise ValueError("fraud scoring models take a feature vector; GRU models run in the abuse scorer")
        self.model_dev = DeviceModel(self.plan, self.device, self.buckets)
        self.step_out = self.model_dev.step_out
        self.tree_partial = self.model_dev.tree_partial
        self.tree_groups = self.model_dev.tree_groups
        self.ml = self.model_dev.out

    def refresh_config(self, scoring=None) -> None:
        """Write the device config block (thresholds, weights, table sizes). The last
        ``scoring`` given stays in force for later refreshes (e.g. a blacklist sync)."""
        if scoring is not None:
            self.scoring = scoring
        scoring = getattr(self, "scoring", None) or self.cfg.scoring
        kind = {"none": MODEL_NONE, "heuristic": MODEL_HEURISTIC, "plan": MODEL_OUTPUT}[self.model]
        ml_col = self.plan.ml_col if self.plan is not None else 0
        ml_stride = self.plan.out_width if self.plan is not None else 1
        c = score_cfg(self.cfg, kind, ml_col=ml_col, ml_stride=ml_stride, sc=scoring,
                      owner_filter=self.owner_filter, my_rank=self.rank, **self.store.table_params())
        self.store.sync_tables()
        self.cfg_dev.copy_(torch.from_numpy(c.view(np.uint8).copy()))

    # ------------------------------------------------------------------ the step
    def _kernels(self, bucket: int) -> None:
        upd = self.update_features
        K.feature_assemble(self.store, self.hdr, self.cfg_dev, self.req, self.X, self.feat, bucket, dedup=upd)
        if self.model_dev is not None:
            self.model_dev.run(self.X, bucket, m_ptr=self.n_ptr)
        ud = K.update_args(self.store, self.cfg_dev, self.req, bucket, hdr=self.hdr, region=-1) if upd else None
        K.ensemble(self.hdr, self.cfg_dev, self.feat, self.X, self.ml, self.res, bucket, self.metrics, upd=ud)
        if upd:
            K.update_segments(self.store, self.cfg_dev, self.req, bucket, self.hdr)

    def _body(self, slot: int, bucket: int, with_features: bool = False) -> None:
        nbytes = HDR_BYTES + REQ_BYTES * bucket
        self.dev_slab[:nbytes].copy_(self.host_slab[slot][:nbytes], non_blocking=True)
        self._kernels(bucket)
        self.host_res[slot][:bucket].copy_(self.res[:bucket], non_blocking=True)
        if with_features:
            self.host_feat[slot][:bucket].copy_(self.feat[:bucket], non_blocking=True)

    def capture(self) -> None:
        """Capture one graph per (bucket, pipeline slot); run each once eagerly first."""
        if not self.use_graphs:
            return
        with torch.cuda.device(self.device):
            for b in self.buckets:
                for slot in range(self.depth):
                    self._write_hdr(slot, 0, 0)
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
        raise ValueError(f"batch of {n} exceeds the largest bucket {self.bmax}")

    def _write_hdr(self, slot: int, n: int, now: int) -> None:
        h = self.host_slab_np[slot][:HDR_BYTES].view(BATCHHDR)
        h["n"] = n
        h["seq"] = self._seq
        h["now"] = now

    def slab_view(self, slot: int, n: int) -> np.ndarray:
        return self.host_slab_np[slot][HDR_BYTES:HDR_BYTES + REQ_BYTES * n].view(REQREC)

    def next_slot(self) -> int:
        with self._lock:
            s = self._slot
            self._slot = (self._slot + 1) % self.depth
        return s

    def submit_packed(self, slot: int, n: int, now: int, want_features: bool = False) -> Pending:
        """Launch a batch whose ReqRec rows are already in ``slab_view(slot, n)``."""
        b = self.bucket_for(max(n, 1))
        self._seq += 1
        self._write_hdr(slot, n, now)
        t0 = time.perf_counter()
        with torch.cuda.stream(self.stream):
            g = self.graphs.get((b, slot))
            if g is not None and not want_features:
                g.replay()
            else:
                self._body(slot, b, with_features=want_features)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.batches += 1
        return Pending(slot, n, b, ev, t0, want_features)

    def submit_into(self, slot: int, req: np.ndarray, now: Optional[int] = None,
                    want_features: bool = False) -> Pending:
        n = len(req)
        now = int(time.time()) if now is None else int(now)
        v = self.slab_view(slot, n)
        v[:] = req
        v["ts"] = now
        return self.submit_packed(slot, n, now, want_features)

    def submit(self, req: np.ndarray, now: Optional[int] = None, want_features: bool = False) -> Pending:
        """``req``: REQREC structured array (rows; ts is overwritten with ``now``)."""
        n = len(req)
        now = int(time.time()) if now is None else int(now)
        slot = self.next_slot()
        v = self.slab_view(slot, n)
        v[:] = req
        v["ts"] = now
        return self.submit_packed(slot, n, now, want_features)

    def wait(self, p: Pending, unpack: bool = True):
        p.event.synchronize()
        res = self.host_res[p.slot][:p.n].numpy().copy()
        feats = self.host_feat[p.slot][:p.n].numpy().copy() if p.want_features else None
        if not unpack:
            return res, feats
        out = unpack_results(res)
        if feats is not None:
            out["features"] = feats.view(FEATREC).reshape(-1)
        out["latency_ms"] = (time.perf_counter() - p.t_submit) * 1e3
        return out

    def score(self, req: np.ndarray, now: Optional[int] = None, want_features: bool = False):
        return self.wait(self.submit(req, now, want_features))

    def read_metrics(self, reset: bool = False) -> np.ndarray:
        m = self.metrics.cpu().numpy().copy()
        if reset:
            self.metrics.zero_()
        return m

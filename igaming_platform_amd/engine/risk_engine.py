"""RiskEngine: the risk.v1 service logic behind the gRPC layer.

Reference: ``ScoringEngine`` (services/risk/internal/scoring/engine.go:179-543) wired as the
commented block of services/risk/cmd/main.go:98-142, plus the RPCs the reference declares
but never serves (PredictLTV, GetPlayerSegment, CheckBonusAbuse, blacklist, GetFeatures).

Hot path (ScoreBatch / micro-batched ScoreTransaction), all columnar:
  request bytes -> C++ wire codec (RequestBatch) -> C++ AccountIndex (owner, slot)
  -> REQREC rows per owner shard -> backend (GPU graph or CPU golden) -> ResultRec
  -> C++ serializer -> response bytes.
Thresholds are an immutable ``ScoringConfig`` snapshot swapped under a lock and pushed to
every shard's device config block (fixes the unguarded read of quirk Q6).
"""
from __future__ import annotations

import dataclasses
import functools
import json
import os
import threading
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..config import ACTION_NAMES, Config, REASON_CODES
from ..features.tables import Blacklist, IPIntel
from ..golden import scoring as GS
from ..layouts import ACCTBATCH, FEATREC, REQREC, unpack_results
from ..native import native
from ..obs.logging import get_logger
from ..obs.metrics import Metrics
from ..utils.faults import Faults, InjectedFault
from .audit import AuditLog
from .backends import CpuBackend, GpuBackend, NativeCpuBackend
from .registry import AccountRegistry
from ..parallel.spmd import GroupFailure

log = get_logger("engine")


def _load_onnx(src):
    """bytes | path | _native.OnnxModel -> _native.OnnxModel (None if src is falsy)."""
    if not src:
        return None
    N = native()
    if isinstance(src, (bytes, bytearray)):
        return N.OnnxModel.from_bytes(bytes(src))
    if isinstance(src, str):
        with open(src, "rb") as f:
            return N.OnnxModel.from_bytes(f.read())
    return src


class RiskEngine:
    def __init__(self, cfg: Optional[Config] = None, backend: str = "auto", devices: Optional[Sequence[int]] = None,
                 capacity: Optional[int] = None, fraud_model=None, ltv_model=None, abuse_model=None,
                 shards: int = 1, capture: bool = True, faults: Optional[Faults] = None, spmd=None):
        """``spmd``: a comm (parallel.comm.TorchComm) when this is rank 0 of a one-process-per-GPU
        group; every other rank runs :func:`serve_shard`. Accounts are then owned by ranks."""
        import copy
        self.cfg = copy.deepcopy(cfg) if cfg is not None else Config()
        cfg = self.cfg
        self.faults = faults or Faults()
        self.metrics = Metrics()
        N = native()
        self.N = N
        if backend == "auto":
            backend = "cpu"
            try:
                import torch
                if torch.cuda.is_available():
                    backend = "gpu"
            except Exception:
                pass
        self.kind = backend
        self.group = None
        if spmd is not None:
            import torch
            self.devices = [torch.cuda.current_device()] if backend == "gpu" else []
            world = spmd.world
        elif backend == "gpu":
            import torch
            if devices is None:
                devices = list(range(min(max(cfg.gpu.devices, 1), torch.cuda.device_count())))
            self.devices = list(devices)
            world = len(self.devices)
        else:
            if backend not in ("cpu", "golden"):
                raise ValueError(f"backend must be auto|gpu|cpu|golden, got {backend!r}")
            self.devices = []
            world = max(int(shards), 1)
        self.world = world
        self.capacity = int(capacity or cfg.gpu.accounts_per_gpu)
        self.registry = AccountRegistry(self.capacity, world)
        self.blacklist = Blacklist(cfg.gpu.blacklist_capacity)
        self.ipintel = IPIntel(cfg.gpu.blacklist_capacity)
        self.links = N.LinkIndex(8)  # 8 most recent accounts per device / devices per account
        self.metrics.links = self.links
        # link inserts run off the scoring path on one background thread (C++, GIL released);
        # linked_accounts() waits for the inserts already queued
        import concurrent.futures as _cf
        self._link_pool = _cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="risk-links")
        self._link_pending: List = []
        self._lock = threading.RLock()
        self.scoring = cfg.scoring
        # risk_scores / ltv_predictions audit (engine/audit.py): on when AUDIT_DB is configured
        self.auditlog = make_auditlog(cfg, "r0")
        from ..features.store_ops import KVStore
        self.kv = KVStore()  # IncrementCounter / SetFeature / GetFeature keys (redis_store.go:206-227)

        # ---- models
        fm = _load_onnx(fraud_model if fraud_model is not None else cfg.fraud_model.path)
        mkind = cfg.fraud_model.kind
        if mkind == "auto":
            mkind = "onnx" if fm is not None else "heuristic"  # missing model -> mockPredict (onnx_model.go:51-60)
        if mkind == "onnx" and fm is None:
            raise ValueError("fraud_model.kind=onnx but no model given")
        if mkind == "onnx":
            dims = fm.inputs()[0][2]
            w = int(dims[-1]) if dims and int(dims[-1]) > 0 else cfg.features.width
            if w != cfg.features.width:
                if cfg.features.width != 30:
                    raise ValueError(f"model input width {w} != features.width {cfg.features.width}")
                # columns >= 30 are the account's extra features (warehouse ext table)
                cfg.features.width = w
        self.model_kind = mkind
        self.fraud_onnx = fm
        self._capture = capture
        self._abuse_am = abuse_model if abuse_model is not None else cfg.abuse_model.path
        # failure handling state (see _group_failed / rehome)
        self._snapshot_dir = cfg.gpu.snapshot_dir or None
        self.failover = dict(group_failed=False, error=None, rehomed=[], rehome_errors={})
        self.rehome_done = threading.Event()
        self._rehome_threads: List[threading.Thread] = []
        self.model_version = 1
        self.backends: List = []
        self.healthy = [True] * world
        self.core = None
        if spmd is not None:
            from ..parallel.spmd import ShardProxy, ShardRunner, SpmdGroup
            node = SpmdNode(cfg, spmd, backend, self.capacity, fm, mkind, self.blacklist, self.ipintel,
                            capture=capture)
            self.node = node
            self.registry = node.registry  # node-shared: every rank resolves ids to the same slots
            local = node.local
            self.local = local
            self.core = node.core
            self.links = node.links  # node-shared: links recorded by every rank's ingress
            self.metrics.links = self.links
            self.auditlog = node.audit  # the node's core writes its native ring
            self._audit_evicted_seen = 0
            from . import serving
            self.metrics.sources.append(lambda c=node.core: serving.core_metrics(c))
            abuse_gpu = make_abuse_gpu(cfg, local, self._abuse_am)
            self.group = SpmdGroup(spmd, ShardRunner(spmd, local, abuse_gpu, node.core),
                                   heartbeat_s=cfg.gpu.spmd_heartbeat_s,
                                   used_fn=lambda: [self.registry.size(o) for o in range(self.world)],
                                   on_failure=self._group_failed)
            self._spmd_abuse_gpu = abuse_gpu
            self.backends = [ShardProxy(self.group, o, local) for o in range(world)]
        elif backend == "gpu":
            from ..models.plan import compile_onnx, to_device
            for r, d in enumerate(self.devices):
                plan = (to_device(compile_onnx(fm), f"cuda:{d}", cfg.fraud_model.precision)
                        if mkind == "onnx" else None)
                model = {"onnx": "plan", "heuristic": "heuristic", "none": "none"}[mkind]
                be = GpuBackend(cfg, self.capacity, f"cuda:{d}", plan=plan, model=model,
                                blacklist=self.blacklist, ipintel=self.ipintel, capture=capture)
                be.on_drained = functools.partial(self._on_drained, r)
                self.backends.append(be)
                self.metrics.gpu_healthy.labels(gpu=str(d)).set(1)
        else:
            for _ in range(world):
                self.backends.append(self._cpu_backend(mkind, fm, backend, self.capacity))
        # native serving core of a single-shard engine (engine/serving.py): request bytes ->
        # response bytes without Python on the hot path, and the only issuer of the shard's
        # device batches (SPMD: the node's core, above)
        if spmd is None and world == 1 and cfg.gpu.native_serving:
            self._attach_core(self.backends[0])
        self.fallback = None
        if cfg.gpu.fallback == "cpu":  # degraded tier: CPU scorer without the shard's feature state
            self.fallback = self._cpu_backend(mkind, fm, "golden" if backend == "golden" else "cpu", 1)

        # ---- LTV / abuse services
        from .abuse import AbuseGpu, AbuseService
        from .ltv import LtvGpu, LtvService
        lm = _load_onnx(ltv_model if ltv_model is not None else cfg.ltv_model.path)
        am = _load_onnx(abuse_model if abuse_model is not None else cfg.abuse_model.path)
        ltv_width = int(lm.inputs()[0][2][-1]) if lm is not None else 0
        self.ltv_model_version = "onnx-1" if lm is not None else "rules"  # ltv.go:113-151 formula
        if spmd is not None:
            lg = None
            if backend == "gpu":
                from ..models.plan import compile_onnx, to_device
                dev = f"cuda:{self.devices[0]}"
                lplan = to_device(compile_onnx(lm), dev, cfg.ltv_model.precision) if lm is not None else None
                g = LtvGpu(dev, self.capacity, lplan,
                           buckets=cfg.gpu.buckets, in_width=ltv_width, use_graphs=capture)
                g.capture()
                lg = [g]
            self.ltv = LtvService(self.registry, world, gpu=lg, model_width=ltv_width,
                                  executor=N.Executor(lm) if (lm is not None and lg is None) else None,
                                  group=self.group, rank=0)
            self.group.runner.ltv = self.ltv
            self.abuse = AbuseService(self, threshold=cfg.abuse.threshold, group=self.group,
                                      executor=N.Executor(am) if (am is not None and backend != "gpu") else None,
                                      group_model=am is not None and backend == "gpu")
        elif backend == "gpu":
            from ..models.plan import compile_onnx, to_device
            lg = []
            for d in self.devices:
                lp = to_device(compile_onnx(lm), f"cuda:{d}", cfg.ltv_model.precision) if lm is not None else None
                g = LtvGpu(f"cuda:{d}", self.capacity, lp, buckets=cfg.gpu.buckets, in_width=ltv_width,
                           use_graphs=capture)
                g.capture()
                lg.append(g)
            self.ltv = LtvService(self.registry, world, gpu=lg, model_width=ltv_width)
            ag = None
            if am is not None:
                ag = []
                for r, d in enumerate(self.devices):
                    ap = to_device(compile_onnx(am), f"cuda:{d}", cfg.abuse_model.precision)
                    g = AbuseGpu(self.backends[r].store, ap, buckets=cfg.gpu.buckets, use_graphs=capture)
                    g.state_clock = getattr(self.backends[r], "state_clock", None)
                    g.capture()
                    ag.append(g)
            self.abuse = AbuseService(self, threshold=cfg.abuse.threshold, gpu=ag)
        else:
            self.ltv = LtvService(self.registry, world, executor=N.Executor(lm) if lm is not None else None,
                                  model_width=ltv_width)
            self.abuse = AbuseService(self, threshold=cfg.abuse.threshold,
                                      executor=N.Executor(am) if am is not None else None)
        # ---- native account RPCs (engine/acct.py, csrc/runtime/acct_core.cpp): PredictLTV,
        # GetPlayerSegment and CheckBonusAbuse bytes -> bytes without Python, micro-batched on this
        # process's model devices (SPMD: the node's router, owner-routed over /dev/shm)
        self.acct = None
        if cfg.gpu.native_acct and backend != "golden" and (spmd is not None or (world == 1 and cfg.gpu.native_serving)):
            self._attach_acct(spmd is not None, am)
        self.started_at = time.time()
        if self.group is not None:
            self.group.start_heartbeat()
        log.info("risk engine ready", extra={"fields": dict(backend=backend, shards=world, capacity=self.capacity,
                                                              model=mkind)})

    def _attach_core(self, be, indexes=None, rank: int = 0, clock=None) -> None:
        from . import serving
        if be.kind == "gpu":
            dev = be.native_device()
            seq0 = be.scorer._seq
        elif hasattr(be, "native_device"):
            dev = be.native_device(self.cfg.gpu.serve_depth, self.cfg.gpu.max_batch)
            seq0 = 0
        else:
            return  # golden (pure Python) shards keep the Python path
        if dev is None:
            return
        core = serving.make_core(indexes if indexes is not None else [self.registry.index[0]], dev, self.cfg,
                                 rank=rank, clock=clock, seq0=seq0)
        core.set_links(self.links)
        be.attach_core(core)
        self.core = core
        self._attach_audit(core, indexes if indexes is not None else [self.registry.index[0]])
        self.metrics.sources.append(lambda c=core: serving.core_metrics(c))

    def _attach_audit(self, core, indexes) -> None:
        """risk_scores audit of the core's rows: its native ring (csrc/runtime/audit.cpp),
        drained by :meth:`flush_audit` next to the Python rings."""
        attach_audit_ring(self.auditlog, self.cfg, core, indexes, int(self.model_version))
        self._audit_evicted_seen = 0

    def _attach_acct(self, spmd: bool, am) -> None:
        from . import acct as A
        try:
            if spmd:
                acct = self.node.acct
                local, owner = self.local, 0
            else:
                acct = A.NativeAcct([self.registry.index[0]])
                local, owner = self.backends[0], 0
            plan = A.abuse_device_plan(self.cfg, am, local.device) if (am is not None and local.kind == "gpu") else None
            A.attach_models(acct, self.cfg, local, ltv=self.ltv, owner=owner, abuse_model=am, abuse_plan=plan,
                            audit=bool(self.cfg.server.audit_db), rank=0)  # as every worker rank
            acct.router.set_links(self.links)
            self.acct = acct
            if spmd:
                self.group.runner.acct = acct
        except Exception as e:  # the Python path keeps serving these RPCs
            log.error("native account RPCs unavailable", extra={"fields": dict(error=str(e))})
            self.acct = None

    def on_core_failure(self, msg: str) -> None:
        """A hot call failed inside a native core (device error / deadline): the same handling
        as :meth:`score_batch_bytes` - the group fails over (SPMD) or the shard is marked
        unhealthy, so later calls take the Python path with its fallback."""
        e = RuntimeError(f"native serving failure: {msg}")
        g = self.group
        if g is not None:
            try:
                g.fail(e)
            except Exception:  # GroupFailure: the failover runs in _group_failed
                pass
        else:
            self._mark_unhealthy(0, e)

    def _native_ok(self) -> bool:
        """Whether a request may take the all-native path (the Python path keeps fault
        injection and the degraded-shard fallback)."""
        return self.core is not None and all(self.healthy) and not self.faults.any_active()

    def _cpu_backend(self, mkind, fm, kind: str = "cpu", capacity: int = 1):
        if kind == "cpu":
            return make_local_backend(self.cfg, "cpu", capacity, fm, mkind, self.blacklist, self.ipintel)
        if mkind == "onnx":
            from ..models.plan import executor_output
            ml_col, out_name = executor_output(fm, self.cfg.fraud_model.output_name)
            in_name = fm.inputs()[0][0]
            return CpuBackend(self.cfg, model="plan", executor=self.N.Executor(fm), input_name=in_name,
                              output_name=out_name, ml_col=ml_col, blacklist=self.blacklist, ipintel=self.ipintel)
        return CpuBackend(self.cfg, model=mkind, blacklist=self.blacklist, ipintel=self.ipintel)

    # ================================================================== scoring (columnar)
    def _score_parsed(self, rb, now: int, want_features: bool = True):
        """RequestBatch -> (ResultRec [n,2] uint32, FeatRec [n] or None)."""
        n = len(rb)
        version = self.model_version  # read before scoring: a concurrent reload bumps it after its swap
        slots, owners, _ = self.registry.resolve_batch(rb, insert=True)
        req = np.empty(n, REQREC)
        rb.pack_reqrec(slots, req.view(np.uint8), now, None)
        g = self.group
        if g is not None:  # owner-routed exchange: each rank scores its own rows
            try:
                try:
                    res, feats = self.core.score_rows(req.view(np.uint8), owners, now, bool(want_features))
                    feats = feats.view(FEATREC).reshape(-1) if feats is not None else None
                except RuntimeError as e:  # a peer missed the step deadline: the group failed
                    raise g.fail(e) from e
                audited = self.auditlog.native is not None  # the core's ring has these rows
            except GroupFailure:
                # the batch died with the group (some rows may have been applied on their
                # shards): answer all of it from the stateless fallback; later batches go to
                # the local and re-homed shards (_group_failed)
                res, feats = self._fallback_score(req, now, want_features, "group_failed")
                audited = False
            self._add_links(rb, slots, owners)
            self._observe(rb, res, version, audited)
            return res, feats, slots, owners
        res = np.zeros((n, 2), np.uint32)
        feats = np.zeros(n, FEATREC) if want_features else None
        groups = [(0, None)] if self.world == 1 else [(o, np.nonzero(owners == o)[0]) for o in range(self.world)]
        pend = []
        for o, sel in groups:
            sub = req if sel is None else req[sel]
            if len(sub) == 0:
                continue
            pend.append((o, sel, sub, self._submit(o, sub, now, want_features)))
        # rows the serving core scored are in its native audit ring already (world 1 only)
        audited = self.auditlog.native is not None
        for o, sel, sub, p in pend:
            r, f, via_core = self._collect(o, sub, now, want_features, p)
            audited = audited and via_core
            if sel is None:
                res[:], feats = r, f
            else:
                res[sel] = r
                if want_features:
                    feats[sel] = f
        self._add_links(rb, slots, owners)
        self._observe(rb, res, version, audited)
        return res, feats, slots, owners

    def _add_links(self, rb, slots: np.ndarray, owners: np.ndarray) -> None:
        """(device, account) co-occurrences of a batch -> the link index, asynchronously."""
        dev = rb.columns()["device_hash"]
        keys = (owners.astype(np.int64) << 32) | np.where(slots >= 0, slots, -1)
        with self._lock:
            self._link_pending = [f for f in self._link_pending if not f.done()]
            if len(self._link_pending) >= 8:  # the worker fell behind: insert inline (bounded queue)
                self.links.add(dev, keys)
                return
            self._link_pending.append(self._link_pool.submit(self.links.add, dev, keys))

    def _flush_links(self) -> None:
        with self._lock:
            pend, self._link_pending = self._link_pending, []
        for f in pend:
            f.result()

    def _observe(self, rb, res: np.ndarray, version: int, audited: bool = False) -> None:
        """Metrics + the risk_scores audit entry of one scored batch (every scoring entry point
        goes through :meth:`_score_parsed`, so ScoreWithExplanation and /debug/score are logged
        too). ``version`` is the model version the batch was scored with; ``audited``: the
        serving core's native ring holds the batch already."""
        self.metrics.observe_results(res)
        self.metrics.batch_size.observe(len(res))
        if self.auditlog.enabled and not audited:
            before = self.auditlog.evicted_rows
            self.auditlog.record_scores(rb.account_id, res, version)
            if self.auditlog.evicted_rows != before:
                self.metrics.audit_evicted.inc(self.auditlog.evicted_rows - before)

    def _submit(self, o: int, sub: np.ndarray, now: int, want_features: bool):
        be = self.backends[o]
        if not self.healthy[o] and self.fallback is not None:
            return ("fallback", None)
        try:
            if self.faults.active("backend_error", shard=o):
                raise InjectedFault(f"injected backend error on shard {o}")
            if be.kind == "gpu" and self.faults.active("gpu_timeout", shard=o):
                # a real device stall ahead of the batch: the watchdog deadline has to catch it
                ms = float(self.faults.params("gpu_timeout").get("ms", 3 * self.cfg.gpu.batch_timeout_ms))
                be.stall(ms)
            return ("ok", (be, be.submit(sub, now, want_features)))
        except Exception as e:  # shard failure -> degrade to the CPU fallback
            self._mark_unhealthy(o, e)
            return ("fallback", None)

    def _collect(self, o: int, sub: np.ndarray, now: int, want_features: bool, p):
        state, h = p
        if state == "ok":
            be, h = h
            try:
                if be.kind == "gpu":
                    r, f = be.collect(h, timeout_s=self.cfg.gpu.batch_timeout_ms / 1e3)
                else:
                    r, f = be.collect(h)
                return r, f, getattr(be, "core", None) is not None
            except Exception as e:
                self._mark_unhealthy(o, e)
        r, f = self._fallback_score(sub, now, want_features, "shard_unhealthy", shard=o)
        return r, f, False

    def _fallback_score(self, sub: np.ndarray, now: int, want_features: bool, reason: str, shard=None):
        if self.fallback is None:
            raise RuntimeError(f"shard {shard if shard is not None else '*'} failed and no fallback is configured")
        self.metrics.fallbacks.labels(reason=reason).inc(len(sub))
        # the fallback has no feature state for this shard: partial features (engine.go:267-270)
        fb = sub.copy()
        fb["slot"] = -1
        return self.fallback.score(fb, now, want_features, update=False)

    def _mark_unhealthy(self, o: int, err: Exception) -> None:
        first = self.healthy[o]
        if first:
            log.error("shard unhealthy", extra={"fields": dict(shard=o, error=str(err))})
        self.healthy[o] = False
        if self.devices and o < len(self.devices):
            self.metrics.gpu_healthy.labels(gpu=str(self.devices[o])).set(0)
        if (first and self.group is None and self.kind == "gpu" and self.cfg.gpu.auto_recover
                and len(self.devices) > 1 and not self.failover["group_failed"]):
            # a shard that neither drains nor recovers is rebuilt on a surviving GPU
            t = threading.Timer(self.cfg.gpu.rehome_after_s, self._rehome_if_still_unhealthy, args=(o,))
            t.daemon = True
            t.start()

    def recover(self, shard: Optional[int] = None) -> None:
        """Mark shard(s) healthy again (after an operator or watchdog check)."""
        for o in ([shard] if shard is not None else range(self.world)):
            self.healthy[o] = True
            if self.devices and o < len(self.devices):
                self.metrics.gpu_healthy.labels(gpu=str(self.devices[o])).set(1)

    # ---- failure handling: drain, failover, re-home
    def _on_drained(self, o: int, be) -> None:
        """A quarantined GPU shard's late batches all completed: its state is consistent (each
        late batch applied its events once), so it returns to service (``auto_recover``)."""
        if self.cfg.gpu.auto_recover and self.backends[o] is be and not self.healthy[o]:
            log.info("shard drained, back in service", extra={"fields": dict(shard=o)})
            self.recover(o)

    def _rehome_if_still_unhealthy(self, o: int) -> None:
        if self.healthy[o] or self._snapshot_dir is None:
            return
        alive = [d for k, d in enumerate(self.devices) if self.healthy[k] and k != o]
        if not alive:
            return
        try:
            self.rehome(o, device=alive[0])
        except Exception as e:
            log.error("re-home failed", extra={"fields": dict(shard=o, error=str(e))})

    def _group_failed(self, err: BaseException) -> None:
        """SPMD group failure (called once, by the thread whose collective failed): rank 0
        leaves the group and serves alone. Its own shard keeps its state (a GPU shard drops
        the RCCL exchange and runs the single-GPU pipeline on the same HBM store); every
        remote shard is unhealthy (rows -> stateless fallback) until :meth:`rehome` rebuilds
        it here from the snapshot directory, on a background thread."""
        with self._lock:
            g = self.group
            if g is None:
                return
            self.group = None
        self.failover.update(group_failed=True, error=str(err), t_failed=time.time())
        log.error("spmd group failed: failing over to rank 0", extra={"fields": dict(error=str(err))})
        g.abandon()
        local = self.local
        core, self.core = self.core, None
        if core is not None:
            try:
                core.abort()  # no convergence with the dead peer; later batches take the Python path
            except Exception as e:
                log.error("serving core abort failed", extra={"fields": dict(error=str(e))})
            local.core = None
        try:
            if local.kind == "gpu":
                local.leave_exchange()
        except Exception as e:  # rank 0's own device is stuck too: everything falls back
            log.error("local shard unusable after the group failure", extra={"fields": dict(error=str(e))})
            self._mark_unhealthy(0, e)
        self.backends = [local] + [DeadShard(o) for o in range(1, self.world)]
        for o in range(1, self.world):
            self.healthy[o] = False
        ag = getattr(self, "_spmd_abuse_gpu", None)
        self.abuse.group, self.abuse.group_model = None, False
        if ag is not None:
            self.abuse.gpu = [ag] + [None] * (self.world - 1)
        if self.cfg.gpu.auto_recover and self._snapshot_dir is not None:
            t = threading.Thread(target=self._rehome_all, args=(list(range(1, self.world)), True), daemon=True,
                                 name="spmd-rehome")
            self._rehome_threads.append(t)
            t.start()
        else:
            self.rehome_done.set()

    def _rehome_all(self, owners, wait_final: bool) -> None:
        try:
            for o in owners:
                try:
                    self.rehome(o, wait_final=wait_final)
                except Exception as e:
                    self.failover["rehome_errors"][o] = str(e)
                    log.error("re-home failed", extra={"fields": dict(shard=o, error=str(e))})
        finally:
            self.rehome_done.set()

    def rehome(self, o: int, directory: Optional[str] = None, device=None, wait_final: bool = False) -> int:
        """Rebuild shard ``o`` in this process from its snapshot in ``directory`` (default: the
        last snapshot directory) and put it back in service; returns the accounts restored.
        ``device``: GPU ordinal for a GPU shard (default: this process's device).
        ``wait_final``: first wait up to ``rehome_grace_s`` for the shard's final snapshot
        (written by a surviving SPMD worker when the group failed). The engine's account
        registry is live on rank 0, so every account keeps its slot."""
        directory = directory or self._snapshot_dir
        if directory is None:
            raise ValueError("no snapshot directory to re-home from")
        if wait_final:
            marker = os.path.join(directory, f"shard{o}.final")
            t_end = time.time() + self.cfg.gpu.rehome_grace_s
            t_fail = self.failover.get("t_failed", 0) - 60
            while time.time() < t_end and not (os.path.exists(marker) and os.path.getmtime(marker) >= t_fail):
                time.sleep(0.05)
        kind = self.kind if self.kind in ("gpu", "golden") else "cpu"
        if kind == "gpu":
            import torch
            from ..features.device_store import DeviceFeatureStore
            dev = int(device) if device is not None else torch.cuda.current_device()
            # a re-homed shard needs a whole store on this device: refuse (the shard stays on the
            # fallback) instead of running the survivor out of HBM
            need = DeviceFeatureStore.estimate_bytes(self.cfg.features, self.capacity)
            free, _ = torch.cuda.mem_get_info(dev)
            if need > 0.9 * free:
                raise MemoryError(f"re-homing shard {o} needs ~{need / 2**30:.1f} GiB, "
                                  f"{free / 2**30:.1f} GiB free on cuda:{dev}")
            with torch.cuda.device(dev):
                be = make_local_backend(self.cfg, "gpu", self.capacity, self.fraud_onnx, self.model_kind,
                                        self.blacklist, self.ipintel, rank=o, capture=self._capture)
        else:
            be = make_local_backend(self.cfg, kind, self.capacity, self.fraud_onnx, self.model_kind,
                                    self.blacklist, self.ipintel, rank=o)
        path = os.path.join(directory, f"shard{o}.{be.snapshot_ext}")
        n = 0
        if os.path.exists(path):
            if be.kind == "gpu":
                n = be.store.restore(path)
            else:
                be.restore(path)
                n = self.registry.size(o)
        else:
            log.error("no snapshot for shard: it restarts empty", extra={"fields": dict(shard=o, path=path)})
        be.refresh_config(self.scoring)
        if be.kind == "gpu":
            be.on_drained = functools.partial(self._on_drained, o)
            if self.abuse.gpu is not None and self._abuse_am is not None:
                self.abuse.gpu[o] = make_abuse_gpu(self.cfg, be, self._abuse_am)
        self.backends[o] = be
        self.failover["rehomed"].append(dict(shard=o, path=path, accounts=int(n), t=time.time()))
        self.recover(o)
        log.info("shard re-homed", extra={"fields": dict(shard=o, path=path, accounts=int(n))})
        return int(n)

    # ---- wire-level entry points (gRPC handlers call these with raw bytes)
    def score_batch_bytes(self, data: bytes, t0: Optional[float] = None, now: Optional[int] = None) -> bytes:
        t0 = time.perf_counter() if t0 is None else t0
        now = int(time.time()) if now is None else int(now)
        if self._native_ok():
            try:
                return self.core.score_batch(data, now, int(t0 * 1e9))
            except RuntimeError as e:  # device failure / deadline: the Python path falls back
                if "ServeCore" not in str(e):
                    raise
                g = self.group
                if g is not None:
                    try:
                        g.fail(e)
                    except Exception:  # GroupFailure: the failover below serves this batch
                        pass
                else:
                    self._mark_unhealthy(0, e)
        rb = self.N.RequestBatch()
        rb.parse_batch(data)
        res, feats, slots, owners = self._score_parsed(rb, now)
        ms = np.full(len(rb), int((time.perf_counter() - t0) * 1e3), np.int64)
        return self.N.serialize_batch_response(res, feats.view(np.int32).reshape(-1, 32) if feats is not None else None, ms)

    def score_tx_bytes(self, data: bytes, t0: Optional[float] = None) -> bytes:
        return self.score_tx_many_bytes([data], [t0 if t0 is not None else time.perf_counter()])[0]

    def score_tx_many_bytes(self, items: List[bytes], t0s: Sequence[float]) -> List[bytes]:
        """Micro-batcher path: many unary requests, one device batch, one response each."""
        rb = self.N.RequestBatch()
        rb.parse_tx_list(items)
        res, feats, _, _ = self._score_parsed(rb, int(time.time()))
        now = time.perf_counter()
        ms = np.array([int((now - t) * 1e3) for t in t0s], np.int64)
        return self.N.serialize_tx_responses(res, feats.view(np.int32).reshape(-1, 32) if feats is not None else None, ms)

    def flush_audit(self, path: str) -> int:
        """Drain the score audit ring into the ``risk_scores`` table of the SQLite database at
        ``path`` and the LTV ring (PredictLTV / GetPlayerSegment answers) into
        ``ltv_predictions`` (deploy/schema.sql; the reference declares both tables,
        init-db.sql:122-155, and never writes them). Rows survive a failed write. Returns the
        number of rows written."""
        try:
            return self.auditlog.flush(path)
        finally:
            ring = self.auditlog.native
            if ring is not None:  # native-ring evictions -> the Prometheus counter
                ev = int(ring.evicted)
                if ev > self._audit_evicted_seen:
                    self.metrics.audit_evicted.inc(ev - self._audit_evicted_seen)
                    self._audit_evicted_seen = ev

    # ================================================================== python-level API
    def _tx_bytes(self, tx: Dict) -> bytes:
        from ..proto import risk_v1 as P
        m = P.ScoreTransactionRequest()
        for k, v in tx.items():
            if k == "metadata":
                m.metadata.update(v)
            else:
                setattr(m, k, v)
        return m.SerializeToString()

    def score(self, txs: Sequence[Dict], now: Optional[int] = None) -> List[Dict]:
        """Score dict transactions (ScoreTransactionRequest field names). Returns dicts."""
        rb = self.N.RequestBatch()
        rb.parse_tx_list([self._tx_bytes(t) for t in txs])
        res, feats, slots, _ = self._score_parsed(rb, int(time.time()) if now is None else int(now))
        cols = unpack_results(res)
        out = []
        for i in range(len(txs)):
            mask = int(cols["reasons"][i])
            out.append(dict(score=int(cols["score"][i]), action=int(cols["action"][i]),
                            action_name=ACTION_NAMES.get(int(cols["action"][i]), "?"),
                            reason_codes=[REASON_CODES[b] for b in range(len(REASON_CODES)) if mask >> b & 1],
                            rule_score=int(cols["rule_score"][i]), ml_score=float(cols["ml"][i]),
                            features=feats[i] if feats is not None else None))
        return out

    def explain(self, tx: Dict, now: Optional[int] = None) -> str:
        """``ScoreWithExplanation`` (engine.go:507-543)."""
        t0 = time.perf_counter()
        r = self.score([tx], now)[0]
        f = r["features"]
        fd = {k: (f[k].item() if hasattr(f[k], "item") else f[k]) for k in FEATREC.names} if f is not None else {}
        fl = int(fd.get("flags", 0))
        fd.update(is_vpn=bool(fl & 1), is_proxy=bool(fl & 2), bonus_only_player=bool(fl & 16))
        sr = GS.ScoreResult(r["score"], r["action"], r["reason_codes"], r["rule_score"], r["ml_score"], fd,
                            int((time.perf_counter() - t0) * 1e3))
        return GS.explain(self.scoring, sr)

    def get_features(self, account_id: str, now: Optional[int] = None) -> np.ndarray:
        now = int(time.time()) if now is None else int(now)
        slot, owner = self.registry.resolve(account_id, insert=False)
        if slot < 0 or self.faults.active("feature_store_down"):
            r = np.zeros(1, FEATREC)[0]
            r["flags"] = 64  # partial
            r["slot"] = -1
            return r
        return self.backends[owner].features(slot, now)

    def get_features_bytes(self, account_id: str, now: Optional[int] = None) -> bytes:
        rec = np.array([self.get_features(account_id, now)], FEATREC)
        return self.N.serialize_feature_vector(rec.view(np.int32))

    # ---- thresholds (engine.go:491-504)
    def get_thresholds(self):
        s = self.scoring
        return s.block_threshold, s.review_threshold

    def update_thresholds(self, block: int, review: int):
        if not (0 <= review <= 100 and 0 <= block <= 100):
            raise ValueError("thresholds must be in [0, 100]")
        with self._lock:
            self.scoring = dataclasses.replace(self.scoring, block_threshold=int(block), review_threshold=int(review))
            self._push_config()
        log.info("thresholds updated", extra={"fields": dict(block=block, review=review)})
        return self.get_thresholds()

    # ---- model hot-reload: versioned, broadcast to every shard
    def reload_model(self, fraud_model) -> int:
        """Swap the fraud model (ONNX bytes or path; None/b"" = the built-in heuristic) on every
        shard between batches; feature state, thresholds and metrics are kept. The input width
        must match the running feature layout. Returns the new model version."""
        raw = fraud_model
        if isinstance(raw, str):
            with open(raw, "rb") as f:
                raw = f.read()
        raw = bytes(raw or b"")
        fm = _load_onnx(raw)
        mkind = "onnx" if fm is not None else "heuristic"
        if fm is not None:
            dims = fm.inputs()[0][2]
            w = int(dims[-1]) if dims and int(dims[-1]) > 0 else self.cfg.features.width
            if w != self.cfg.features.width:
                raise ValueError(f"model input width {w} != running features.width {self.cfg.features.width}")
        with self._lock:
            if self.group is not None:
                self.group.reload_model(raw)
            else:
                for be in self.backends:
                    be.swap_model(fm, mkind, version=self.model_version + 1)
            if self.fallback is not None:
                self.fallback.swap_model(fm, mkind)
            self.fraud_onnx, self.model_kind = fm, mkind
            self.model_version += 1
        log.info("fraud model reloaded", extra={"fields": dict(version=self.model_version, kind=mkind)})
        return self.model_version

    def set_scoring(self, **kw) -> None:
        """Replace any ScoringConfig fields (rule limits, weights) atomically."""
        with self._lock:
            self.scoring = dataclasses.replace(self.scoring, **kw)
            self._push_config()

    def _push_config(self) -> None:
        if self.group is not None:
            self.backends[0].refresh_config(self.scoring)  # every rank's runner refreshes its router too
            return
        for be in self.backends:
            be.refresh_config(self.scoring)
        if self.fallback is not None:
            self.fallback.refresh_config(self.scoring)
        acct = getattr(self, "acct", None)
        if acct is not None:
            acct.set_abuse(self.scoring, self.cfg.abuse.threshold, self.cfg.abuse.link_wait_us)
            acct.refresh()

    # ---- blacklist (risk.proto:151-181; redis_store.go:251-293)
    def add_to_blacklist(self, type_: str, value: str, reason: str = "", created_by: str = "",
                         expires_at: int = 0):
        with self._lock:
            e = self.blacklist.add(type_, value, reason, created_by, expires_at=expires_at, now=int(time.time()))
            self._push_config()
        return e

    def check_blacklist(self, device_id: str = "", fingerprint: str = "", ip: str = "", email: str = "",
                        now: Optional[int] = None):
        now = int(time.time()) if now is None else int(now)
        return self.blacklist.check(now, device_id=device_id, fingerprint=fingerprint, ip=ip, email=email)

    def set_ip_intel(self, ip: str, vpn: bool = False, proxy: bool = False, tor: bool = False) -> None:
        with self._lock:
            self.ipintel.set(ip, vpn, proxy, tor)
            self._push_config()

    # ---- feature ingestion (event path)
    def ingest_events(self, events: Sequence[Dict]) -> int:
        """TransactionEvents -> ordered feature update on the owner shard (no scoring).
        Each event: account_id, amount, transaction_type, ts (unix s), device_id, ip_address."""
        if not events:
            return 0
        rb = self.N.RequestBatch()
        rb.parse_tx_list([self._tx_bytes({k: v for k, v in e.items() if k != "ts"}) for e in events])
        slots, owners, _ = self.registry.resolve_batch(rb, insert=True)
        req = np.empty(len(events), REQREC)
        rb.pack_reqrec(slots, req.view(np.uint8), 0, None)
        req["ts"] = [int(e.get("ts") or time.time()) for e in events]
        for o in range(self.world):
            sel = owners == o
            if np.any(sel):
                self.backends[o].ingest(req[sel])
        self._add_links(rb, slots, owners)
        return len(events)

    # ---- warehouse batch features (engine.go:127-140 / the hourly job, main.go:227-236)
    def load_batch_features(self, account_ids: Sequence[str], rows: np.ndarray) -> None:
        rows = np.asarray(rows, ACCTBATCH)
        slots, owners = self.registry.resolve_ids(list(account_ids), insert=True)
        for o in range(self.world):
            sel = np.nonzero((owners == o) & (slots >= 0))[0]
            if len(sel):
                self.backends[o].set_batch_rows(slots[sel], rows[sel])

    def load_ext_features(self, account_ids: Sequence[str], ext: np.ndarray) -> None:
        slots, owners = self.registry.resolve_ids(list(account_ids), insert=True)
        ext = np.asarray(ext, np.float32)
        for o in range(self.world):
            sel = np.nonzero((owners == o) & (slots >= 0))[0]
            if len(sel):
                self.backends[o].set_ext(slots[sel], ext[sel])

    def delete_account_features(self, account_ids: Sequence[str]) -> None:
        """``DeleteAccountFeatures`` (redis_store.go:230-240): the shard state and the account's
        named features."""
        from ..features.store_ops import feature_key
        for a in account_ids:
            self.kv.delete_prefix(feature_key(a, ""))
        slots, owners = self.registry.resolve_ids(list(account_ids), insert=False)
        for o in range(self.world):
            sel = np.nonzero((owners == o) & (slots >= 0))[0]
            if len(sel):
                self.backends[o].reset_accounts(slots[sel])

    # ---- feature-store auxiliary operations (redis_store.go:171-240) and feature importance
    def get_velocity_batch(self, account_ids: Sequence[str], now: Optional[int] = None) -> np.ndarray:
        """``GetVelocity`` for many accounts: int32 [n, 3] = (count_1m, count_5m, count_1h), one
        feature read (K1 launch on a GPU shard) per shard; unknown accounts count 0."""
        now = int(time.time()) if now is None else int(now)
        slots, owners = self.registry.resolve_ids(list(account_ids), insert=False)
        out = np.zeros((len(slots), 3), np.int32)
        for o in np.unique(owners):
            sel = np.nonzero((owners == o) & (slots >= 0))[0]
            if len(sel):
                f = self.backends[int(o)].features_many(slots[sel], now)
                out[sel] = np.stack([f["tx_count_1m"], f["tx_count_5m"], f["tx_count_1h"]], 1)
        return out

    def get_velocity(self, account_id: str, now: Optional[int] = None) -> Tuple[int, int, int]:
        c = self.get_velocity_batch([account_id], now)[0]
        return int(c[0]), int(c[1]), int(c[2])

    def check_rate_limit_batch(self, account_ids: Sequence[str], max_per_min: Optional[int] = None,
                               max_per_hour: Optional[int] = None, now: Optional[int] = None) -> np.ndarray:
        """``CheckRateLimit``: count_1m >= max_per_min or count_1h >= max_per_hour (defaults: the
        live MaxTxPerMinute / MaxTxPerHour)."""
        s = self.scoring
        mpm = s.max_tx_per_minute if max_per_min is None else int(max_per_min)
        mph = s.max_tx_per_hour if max_per_hour is None else int(max_per_hour)
        v = self.get_velocity_batch(account_ids, now)
        return (v[:, 0] >= mpm) | (v[:, 2] >= mph)

    def check_rate_limit(self, account_id: str, max_per_min: Optional[int] = None,
                         max_per_hour: Optional[int] = None, now: Optional[int] = None) -> bool:
        return bool(self.check_rate_limit_batch([account_id], max_per_min, max_per_hour, now)[0])

    def increment_counter(self, key: str, ttl_s: float, now: Optional[float] = None) -> int:
        """``IncrementCounter``: INCR + EXPIRE of a named counter."""
        return self.kv.incr(key, ttl_s, now)

    def set_feature(self, account_id: str, feature: str, value, ttl_s: float = 0.0,
                    now: Optional[float] = None) -> None:
        """``SetFeature``: an account-scoped named value with a TTL."""
        from ..features.store_ops import feature_key
        self.kv.set(feature_key(account_id, feature), value, ttl_s, now)

    def get_feature(self, account_id: str, feature: str, now: Optional[float] = None) -> Optional[str]:
        """``GetFeature``: the value or None (Redis nil) when absent / expired."""
        from ..features.store_ops import feature_key
        return self.kv.get(feature_key(account_id, feature), now)

    def get_feature_importance(self) -> Dict[str, float]:
        """``GetFeatureImportance`` (onnx_model.go:329-345) of the loaded fraud model."""
        from ..features.store_ops import STATIC_IMPORTANCE, plan_importance
        if self.model_kind != "onnx" or self.fraud_onnx is None:
            return dict(STATIC_IMPORTANCE)
        from ..models.plan import compile_onnx
        return plan_importance(compile_onnx(self.fraud_onnx), self.cfg.features.width)

    # ---- LTV / segment / abuse
    def set_players(self, account_ids, features, ext=None) -> None:
        self.ltv.set_players(account_ids, features, ext)

    def predict_ltv(self, account_id: str):
        return self.predict_ltv_batch([account_id])[0]

    def predict_ltv_batch(self, account_ids: Sequence[str]):
        out = self.ltv.predict(account_ids)
        self.auditlog.record_ltv(out, self.ltv_model_version)
        return out

    def check_bonus_abuse(self, account_id: str, bonus_id: str = "", now: Optional[int] = None):
        return self.check_bonus_abuse_batch([account_id], now)[0]

    def check_bonus_abuse_batch(self, account_ids: Sequence[str], now: Optional[int] = None):
        """CheckBonusAbuse for many accounts: one K1 feature read and one GRU launch per shard
        (the gRPC layer's micro-batcher merges concurrent unary calls into one of these)."""
        now = int(time.time()) if now is None else int(now)
        return self.abuse.check(list(account_ids), now)

    def linked_accounts(self, owner: int, slot: int, limit: int = 16, flush: bool = True) -> List[str]:
        if flush:  # the inserts of batches scored so far
            self._flush_links()
        keys = self.links.linked((int(owner) << 32) | int(slot), limit)
        return [self.registry.id_of(int(k) >> 32, int(k) & 0xFFFFFFFF) for k in keys]

    def shard_metrics(self) -> Optional[np.ndarray]:
        """[shards, 128] K10 device counters per shard (SPMD: one all-reduce over the group;
        CPU shards report only their row count), or None when no shard keeps device counters."""
        g = self.group
        if g is not None:
            try:
                return g.shard_metrics()
            except GroupFailure:
                return None
        rows = []
        for be in self.backends:
            m = be.metrics() if hasattr(be, "metrics") and be.kind == "gpu" else None
            rows.append(np.zeros(128, np.int64) if m is None else np.asarray(m, np.int64)[:128])
        return np.stack(rows) if any(r.any() for r in rows) else None

    # ---- health / durability
    def close(self) -> None:
        """Release the SPMD workers (rank 0 only) and stop the serving core."""
        if getattr(self, "acct", None) is not None:
            self.acct.stop()
        if self.group is not None:
            self.group.stop()  # also stops this rank's core (every rank converges)
            self.group = None
            if getattr(self, "node", None) is not None:
                self.node.close()  # the exchange graphs, then the RCCL communicators
        elif self.core is not None:
            self.core.stop()
        self.auditlog.close()  # the segment loader (segments left over resume on the next start)

    def health(self) -> Dict:
        fo = self.failover
        return dict(backend=self.kind, shards=self.world, healthy=list(self.healthy),
                    accounts=[self.registry.size(o) for o in range(self.world)],
                    uptime_s=round(time.time() - self.started_at, 1),
                    failover=dict(group_failed=fo["group_failed"], error=fo["error"],
                                  rehomed=[r["shard"] for r in fo["rehomed"]]))

    def ready(self) -> bool:
        return all(self.healthy) or self.fallback is not None

    def snapshot(self, directory: str) -> None:
        """Feature shards + account registry -> ``directory`` (restart keeps velocity windows;
        a failed shard is re-homed from here)."""
        os.makedirs(directory, exist_ok=True)
        self._snapshot_dir = directory
        meta = dict(version=1, world=self.world, kind=self.kind, ids=[])
        for o in range(self.world):
            n = self.registry.size(o)
            meta["ids"].append([self.registry.id_of(o, s) for s in range(n)])
            if self.group is not None:
                continue
            be = self.backends[o]
            path = os.path.join(directory, f"shard{o}.{be.snapshot_ext}")
            if be.kind == "gpu":
                be.store.snapshot(path, n_used=max(n, 1))
            else:
                be.snapshot(path)
        if self.group is not None:
            self.group.snapshot(directory, [self.registry.size(o) for o in range(self.world)])
        tmp = os.path.join(directory, "registry.json.tmp")
        with open(tmp, "w") as f:
            json.dump(meta, f)
        os.replace(tmp, os.path.join(directory, "registry.json"))

    def restore(self, directory: str) -> int:
        with open(os.path.join(directory, "registry.json")) as f:
            meta = json.load(f)
        if meta["world"] != self.world:
            raise ValueError(f"snapshot has {meta['world']} shards, engine has {self.world}")
        total = 0
        for o in range(self.world):
            ids = meta["ids"][o]
            if ids:
                got, _ = self.registry.index[o].lookup(ids, True)
                if list(got) != list(range(len(ids))):
                    raise ValueError("registry must be empty before restore")
            total += len(ids)
            if self.group is not None:
                continue
            be = self.backends[o]
            path = os.path.join(directory, f"shard{o}.{be.snapshot_ext}")
            if be.kind == "gpu":
                be.store.restore(path)
            else:
                be.restore(path)
        if self.group is not None:
            self.group.restore(directory)
        return total


class ShardUnavailable(RuntimeError):
    """The shard's process died with the SPMD group and is being re-homed."""


class DeadShard:
    """Stand-in for a shard lost with its SPMD worker until :meth:`RiskEngine.rehome` rebuilds
    it: scoring skips it (its rows go to the fallback), state ops fail fast, config pushes and
    model swaps are no-ops (the rebuilt shard takes the engine's current config and model)."""

    kind = "dead"

    def __init__(self, owner: int):
        self.o = owner

    def refresh_config(self, scoring=None) -> None:
        pass

    def swap_model(self, fm, mkind: str, version=None) -> None:
        pass

    def metrics(self):
        return None

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)

        def unavailable(*a, **k):
            raise ShardUnavailable(f"shard {self.o} is being re-homed after its worker failed")
        return unavailable


# ============================================================================ shard construction
def make_local_backend(cfg: Config, kind: str, capacity: int, fm, mkind: str, blacklist, ipintel,
                       owner_filter: bool = False, rank: int = 0, capture: bool = True, comm=None,
                       results_shm: Optional[str] = None):
    """The backend of THIS process's shard (used by SPMD rank 0 and by every worker rank).
    ``comm``: the SPMD group; a GPU shard then joins the owner-routed RCCL exchange (two
    communicators of its own, created collectively here) and scores only its own rows."""
    if kind == "gpu":
        import torch
        from ..models.plan import compile_onnx, to_device
        dev = f"cuda:{torch.cuda.current_device()}"
        plan = to_device(compile_onnx(fm), dev, cfg.fraud_model.precision) if mkind == "onnx" else None
        model = {"onnx": "plan", "heuristic": "heuristic", "none": "none"}[mkind]
        exchange = None
        if comm is not None:
            from ..parallel.exchange import chunk_capacity, rccl_comms
            from .dp import rows_mode
            # rows and results through the node-shared regions: no communicator (engine/dp.py
            # rows_mode); otherwise the two RCCL communicators of the all-to-alls
            rows_shm = bool(results_shm) and rows_mode() == "shm"
            # every rank ingests: each step carries up to C rows per (sender, owner) pair
            exchange = dict(comms=[] if rows_shm else rccl_comms(comm.rank, comm.world), world=comm.world,
                            senders=comm.world, cbuckets=[chunk_capacity(max(cfg.gpu.buckets), comm.world)],
                            rows_shm=rows_shm)
            if results_shm:  # per-GPU D2H result path instead of the result all-to-all
                exchange["results_shm"] = results_shm
        return GpuBackend(cfg, capacity, dev, plan=plan, model=model, blacklist=blacklist, ipintel=ipintel,
                          capture=capture, owner_filter=owner_filter, rank=rank, exchange=exchange)
    N = native()
    cls = CpuBackend if kind == "golden" else NativeCpuBackend
    kw = {} if kind == "golden" else {"capacity": capacity}
    if mkind == "onnx":
        from ..models.plan import executor_output
        ml_col, out_name = executor_output(fm, cfg.fraud_model.output_name)
        return cls(cfg, model="plan", executor=N.Executor(fm), input_name=fm.inputs()[0][0],
                   output_name=out_name, ml_col=ml_col, blacklist=blacklist, ipintel=ipintel, **kw)
    return cls(cfg, model=mkind, blacklist=blacklist, ipintel=ipintel, **kw)


def make_abuse_gpu(cfg: Config, local, abuse_model):
    am = _load_onnx(abuse_model)
    if am is None or local.kind != "gpu":
        return None
    from ..models.plan import compile_onnx, to_device
    from .abuse import AbuseGpu
    g = AbuseGpu(local.store, to_device(compile_onnx(am), str(local.device), cfg.abuse_model.precision),
                 buckets=cfg.gpu.buckets)
    g.state_clock = getattr(local, "state_clock", None)
    g.capture()
    return g


def worker_acct(cfg: Config, node, ltv_model=None, abuse_model=None):
    """A worker rank's LTV shard (the profile rows of the accounts it owns) and its native
    account-RPC router with the LTV / abuse devices attached. Returns (ltv, acct or None)."""
    from .ltv import LtvGpu, LtvService
    lm = _load_onnx(ltv_model if ltv_model is not None else cfg.ltv_model.path)
    am = _load_onnx(abuse_model if abuse_model is not None else cfg.abuse_model.path)
    width = int(lm.inputs()[0][2][-1]) if lm is not None else 0
    local = node.local
    gpu = None
    if local.kind == "gpu":
        from ..models.plan import compile_onnx, to_device
        lp = to_device(compile_onnx(lm), str(local.device), cfg.ltv_model.precision) if lm is not None else None
        g = LtvGpu(str(local.device), node.registry.capacity, lp, buckets=cfg.gpu.buckets, in_width=width)
        g.capture()
        gpu = [g]
    ltv = LtvService(node.registry, node.world, gpu=gpu, model_width=width, rank=node.rank,
                     executor=native().Executor(lm) if (lm is not None and gpu is None) else None)
    acct = node.acct if cfg.gpu.native_acct else None
    if acct is not None:
        from . import acct as A
        try:
            plan = A.abuse_device_plan(cfg, am, local.device) if (am is not None and local.kind == "gpu") else None
            A.attach_models(acct, cfg, local, ltv=ltv, owner=node.rank, abuse_model=am, abuse_plan=plan,
                            audit=bool(cfg.server.audit_db), rank=node.rank)
        except Exception as e:
            log.error("native account RPCs unavailable on this rank", extra={"fields": dict(error=str(e))})
            acct = None
    return ltv, acct


def serve_shard(cfg: Config, comm, backend: str = "gpu", capacity: Optional[int] = None, fraud_model=None,
                abuse_model=None, capture: bool = True, ingress=None, on_node=None, ltv_model=None):
    """Worker rank (>= 1) of an SPMD group: build the same local shard as rank 0 and serve
    its cold ops until rank 0 stops the group; ``ingress(node)``, when given, runs this rank's
    own traffic through its serving core on a thread meanwhile. Returns (ops served, rows
    this shard scored)."""
    from ..parallel.spmd import run_worker
    node = worker_node(cfg, comm, backend, capacity, fraud_model, capture)
    ltv, acct = worker_acct(cfg, node, ltv_model, abuse_model)
    started = on_node(node) if on_node is not None else None  # e.g. this rank's gRPC listener
    if ingress is not None:  # this rank's own traffic, beside the cold-op loop
        import threading
        th = threading.Thread(target=ingress, args=(node,), name=f"ingress-{comm.rank}", daemon=True)
        th.start()
    abuse_gpu = make_abuse_gpu(cfg, node.local, abuse_model if abuse_model is not None else cfg.abuse_model.path)
    try:
        out = run_worker(comm, node.local, abuse_gpu, node.core, ltv=ltv, acct=acct,
                         abuse_threshold=cfg.abuse.threshold,
                         abuse_link_wait_us=cfg.abuse.link_wait_us)
    finally:
        if started is not None and hasattr(started, "stop"):
            started.stop(1.0)
    if ingress is not None:
        th.join(60)
    if node.local.kind == "gpu" and getattr(node.local.scorer, "comms", None):
        node.close()  # graphs, then the communicators (no leak across the process lifetime)
    return out


def make_auditlog(cfg: Config, tag: str) -> AuditLog:
    """The risk_scores / ltv_predictions audit log of a process (on when AUDIT_DB is set);
    segments an earlier process left behind are loaded in the background."""
    s = cfg.server
    log_ = AuditLog(enabled=bool(s.audit_db), mode=s.audit_mode, direct_max=s.audit_direct_max,
                    tag=f"{tag}-p{os.getpid()}")
    if log_.enabled:
        log_.resume_loading(s.audit_db)
    return log_


def attach_audit_ring(auditlog: AuditLog, cfg: Config, core, indexes, model_version: int = 1) -> None:
    if not auditlog.enabled:
        return
    ring = native().AuditRing(int(cfg.server.audit_ring_rows))
    core.set_audit(ring)
    core.set_model_version(int(model_version))
    auditlog.attach_native(ring, indexes)


def worker_node(cfg: Config, comm, backend: str = "gpu", capacity: Optional[int] = None, fraud_model=None,
                capture: bool = True) -> "SpmdNode":
    """The serving objects of a worker rank (>= 1): local shard, node-shared registry, core."""
    fm = _load_onnx(fraud_model if fraud_model is not None else cfg.fraud_model.path)
    mkind = cfg.fraud_model.kind
    if mkind == "auto":
        mkind = "onnx" if fm is not None else "heuristic"
    return SpmdNode(cfg, comm, backend, int(capacity or cfg.gpu.accounts_per_gpu), fm, mkind,
                    Blacklist(cfg.gpu.blacklist_capacity), IPIntel(cfg.gpu.blacklist_capacity), capture=capture)


class SpmdNode:
    """One rank's serving objects in a one-process-per-GPU (or per CPU shard) group:

    * its local shard joined to the owner-routed exchange (GPU: two RCCL communicators of its
      own and the XchgDriver; CPU: the /dev/shm exchange),
    * the node-shared account registry (every rank resolves ids to the same owner slots),
    * the step clock shared with the peers,
    * the serving core that ingests this rank's traffic and issues its exchange steps.

    The /dev/shm regions are created by rank 0, opened by the others after a barrier and
    unlinked once every rank mapped them (nothing is left behind if a process dies later)."""

    def __init__(self, cfg: Config, comm, backend: str, capacity: int, fm, mkind: str, blacklist, ipintel,
                 capture: bool = True):
        from . import serving
        from ..parallel.exchange import chunk_capacity
        rank, world = comm.rank, comm.world
        self.rank, self.world = rank, world
        prefix = comm.bcast_bytes(serving.shm_token().encode() if rank == 0 else None, 0).decode()
        # IGP_XCHG_RESULTS=d2h: results return through a node-shared pinned region (each owner's
        # scatter kernel writes its rows for every sender into it over PCIe) instead of the result
        # all-to-all over xGMI
        # (default: same-box world-1 A/B 95 vs 86 M scores/s, profiles/r5/xchg)
        self.results_mode = os.environ.get("IGP_XCHG_RESULTS", "d2h")
        if self.results_mode not in ("a2a", "d2h"):
            raise ValueError("IGP_XCHG_RESULTS must be a2a or d2h")
        rshm = f"{prefix}-res" if (backend == "gpu" and self.results_mode == "d2h") else None
        if backend != "gpu":
            self.results_mode = "a2a"  # the CPU exchange (/dev/shm) has one result path
        self.local = make_local_backend(cfg, backend, capacity, fm, mkind, blacklist, ipintel, rank=rank,
                                        capture=capture, comm=comm if backend == "gpu" else None, results_shm=rshm)
        C = chunk_capacity(max(cfg.gpu.buckets), world)
        op_t = getattr(comm, "op_timeout", None)
        timeout_s = min(cfg.gpu.exchange_timeout_s, op_t.total_seconds()) if op_t else cfg.gpu.exchange_timeout_s

        def regions(create: bool):
            reg = AccountRegistry(capacity, world, shm_prefix=prefix, create=create)
            clock = native().StepClock(f"{prefix}-clock", world, rank, create)
            # the account-RPC mailbox (engine/acct.py): PredictLTV / GetPlayerSegment /
            # CheckBonusAbuse of accounts another rank owns travel to it over /dev/shm
            from .acct import NativeAcct
            self.acct = NativeAcct(reg.index, rank, f"{prefix}-acct", create) if backend != "golden" else None
            # the device <-> account link index every rank's ingress records into and every
            # rank's CheckBonusAbuse reads (linked_accounts across ingress ranks)
            self.links = native().LinkIndex(8, 1 << 18, f"{prefix}-links", create)
            if self.local.kind == "gpu":
                dev = self.local.native_device()
            else:
                dev = self.local.exchange_device(f"{prefix}-xchg", world, rank, cfg.gpu.serve_depth, C, create,
                                                 timeout_s)
            return reg, clock, dev
        if rank == 0:
            self.registry, self.clock, dev = regions(True)
        comm.barrier()
        if rank != 0:
            self.registry, self.clock, dev = regions(False)
        comm.barrier()
        if rank == 0:
            self.registry.unlink_shared()
            self.clock.unlink_shared()
            if self.acct is not None:
                self.acct.router.unlink_shared()
            self.links.unlink_shared()
            if hasattr(dev, "unlink_shared"):
                dev.unlink_shared()
            if rshm:  # every rank mapped it while building its shard (before the barriers)
                try:
                    os.unlink("/dev/shm/" + rshm)
                except FileNotFoundError:
                    pass
        seq0 = self.local.scorer._seq if self.local.kind == "gpu" else 0
        self.core = serving.make_core(self.registry.index, dev, cfg, rank=rank, clock=self.clock, seq0=seq0)
        self.core.set_links(self.links)
        if self.acct is not None:
            self.acct.router.set_links(self.links)
        self.local.attach_core(self.core)
        self.cfg = cfg
        # risk_scores audit of the rows this rank ingests (each rank drains its own ring)
        self.audit = make_auditlog(cfg, f"r{rank}")
        attach_audit_ring(self.audit, cfg, self.core, self.registry.index)

    def flush_audit(self, path: str) -> int:
        return self.audit.flush(path)

    def start_audit_flusher(self, every_s: float, log=None) -> None:
        """Worker ranks: drain the audit ring every ``every_s`` (rank 0's serve loop does its own)."""
        if not self.audit.enabled:
            return
        from .audit import flush_if_configured
        self._audit_stop = threading.Event()

        def loop():
            while not self._audit_stop.wait(every_s):
                flush_if_configured(self, log)
            flush_if_configured(self, log)
        self._audit_thread = threading.Thread(target=loop, name="audit-flush", daemon=True)
        self._audit_thread.start()

    def close(self) -> None:
        """Ordered shutdown of this rank: the account router and the serving core stop issuing
        device steps, then the local shard releases its exchange (graphs, then the RCCL
        communicators: engine/dp.py DpGpuScorer.close). Idempotent."""
        acct = getattr(self, "acct", None)
        if acct is not None:
            acct.stop()
        if self.core is not None:
            self.core.stop()
        if hasattr(self.local, "close"):
            self.local.close()

    def stop_audit_flusher(self) -> None:
        if getattr(self, "_audit_stop", None) is not None:
            self._audit_stop.set()
            self._audit_thread.join(60)
        self.audit.close()

    def score_batch_bytes(self, data: bytes, now: Optional[int] = None) -> bytes:
        """This rank's ingress: ScoreBatch request bytes -> response bytes."""
        import time as _t
        return self.core.score_batch(data, int(_t.time()) if now is None else int(now), _t.perf_counter_ns())

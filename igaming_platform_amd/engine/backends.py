"""Scoring backends behind the RiskEngine facade.

Both take REQREC rows (slot already resolved by the registry) and return the same thing —
``(res, feats)``: ResultRec ``uint32[n,2]`` (what the C++ wire serializer consumes) and
optionally FeatRec rows — so the API layer, clients and tests are backend-agnostic:

* :class:`CpuBackend` — the golden semantics (``golden/``) with ONNX models run by the C++
  CPU executor (``csrc/runtime/executor.cpp``). This is config 1 (BASELINE.json: unary
  ScoreTransaction on CPU, heuristic model, batch 1) and the fallback when no GPU is present.
* :class:`GpuBackend` — one MI355X shard: HBM feature store + captured-graph scorer.

Reference: services/risk/internal/scoring/engine.go:152-303 (Score), 486-488 (score-then-update).
"""
from __future__ import annotations

import threading
import time
from typing import Optional, Tuple

import numpy as np

from ..config import Config, REASON_BIT
from ..golden import scoring as GS
from ..golden.features import BatchFeatures, GoldenFeatureStore, TxEvent, model_input
from ..layouts import (ACCTBATCH, FEATREC, FR_BLACKLISTED, FR_BONUS_ONLY, FR_PARTIAL, FR_PROXY, FR_TOR,
                       FR_VPN, REQREC, pack_results)
from ..features.tables import Blacklist, IPIntel

Result = Tuple[np.ndarray, Optional[np.ndarray]]


def _featrec_from_golden(f, row, bl: bool, rule: int, reasons) -> np.ndarray:
    r = np.zeros(1, FEATREC)[0]
    for k in FEATREC.names:
        if k in f and not isinstance(f[k], bool):
            r[k] = f[k]
    flags = (FR_VPN if f["is_vpn"] else 0) | (FR_PROXY if f["is_proxy"] else 0) | (FR_TOR if f["is_tor"] else 0)
    flags |= (FR_BONUS_ONLY if f["bonus_only_player"] else 0) | (FR_BLACKLISTED if bl else 0)
    flags |= FR_PARTIAL if f.get("_partial") else 0
    r["flags"] = flags
    r["tx_type"] = int(row["tx_type"]) & 0xFF
    r["slot"] = int(row["slot"])
    r["amount"] = int(row["amount"])
    r["rule_score"] = rule
    r["rule_reasons"] = sum(1 << REASON_BIT[x] for x in reasons)
    return r


def cpu_model_spec(cfg: Config, fm, mkind: str) -> dict:
    """Model arguments of a CPU backend for an ONNX model ``fm`` (``mkind`` "onnx") or a
    built-in model kind ("heuristic" / "none")."""
    if mkind != "onnx":
        return dict(model=mkind, executor=None, input_name="input", output_name=cfg.fraud_model.output_name, ml_col=0)
    from ..models.plan import executor_output
    ml_col, out_name = executor_output(fm, cfg.fraud_model.output_name)
    from ..native import native
    return dict(model="plan", executor=native().Executor(fm), input_name=fm.inputs()[0][0], output_name=out_name,
                ml_col=ml_col)


class CpuBackend:
    """Golden-semantics scorer on the host (the pure-Python spec; ``backend="golden"``)."""

    kind = "cpu"
    snapshot_ext = "json"

    def __init__(self, cfg: Config, model: str = "heuristic", executor=None, input_name: str = "input",
                 output_name: str = "output", ml_col: int = 0,
                 blacklist: Optional[Blacklist] = None, ipintel: Optional[IPIntel] = None):
        if model == "plan" and executor is None:
            model = "none"
        self.cfg = cfg
        self.model = model
        self.executor, self.input_name, self.output_name, self.ml_col = executor, input_name, output_name, ml_col
        self.store = GoldenFeatureStore(cfg.features)
        self.blacklist = blacklist or Blacklist()
        self.ipintel = ipintel or IPIntel()
        self.scoring = cfg.scoring
        self._lock = threading.RLock()
        self._tables_version = None
        self.refresh_config()

    # ------------------------------------------------------------------ state
    def _sync_tables(self) -> None:
        v = (self.blacklist.table.version, self.ipintel.table.version)
        if v == self._tables_version:
            return
        # from the hash tables (what every rank holds), exactly like the device probe (K7)
        b = self.blacklist.table
        self.store.blacklist = {int(k): int(x) for k, x in zip(b.keys, b.vals) if int(k) != 0}
        t = self.ipintel.table
        self.store.ip_intel = {int(k): int(x) for k, x in zip(t.keys.view(np.uint64), t.vals) if int(k) != 0}
        self._tables_version = v

    def swap_model(self, fm, mkind: str, version: Optional[int] = None) -> None:
        """Model hot-reload: the next batch scores with the new model (feature state kept)."""
        spec = cpu_model_spec(self.cfg, fm, mkind)
        with self._lock:
            self.model = spec["model"]
            self.executor, self.input_name = spec["executor"], spec["input_name"]
            self.output_name, self.ml_col = spec["output_name"], spec["ml_col"]

    def refresh_config(self, scoring=None) -> None:
        with self._lock:
            if scoring is not None:
                self.scoring = scoring
            self._sync_tables()

    def set_batch_rows(self, slots, rows) -> None:
        with self._lock:
            for s, b in zip(slots, np.asarray(rows, ACCTBATCH)):
                if not b["present"]:
                    self.store.set_batch(str(int(s)), None)
                    continue
                self.store.set_batch(str(int(s)), BatchFeatures(
                    total_deposits=int(b["total_deposits"]), total_withdrawals=int(b["total_withdrawals"]),
                    deposit_count=int(b["deposit_count"]), withdraw_count=int(b["withdraw_count"]),
                    total_bets=int(b["total_bets"]), total_wins=int(b["total_wins"]),
                    bet_count=int(b["bet_count"]), win_count=int(b["win_count"]),
                    avg_bet_size=float(b["avg_bet_size"]), account_created_at=int(b["account_created_at"]),
                    bonus_claim_count=int(b["bonus_claim_count"]),
                    bonus_wager_complete=float(b["bonus_wager_complete"])))

    def set_ext(self, slots, ext) -> None:
        with self._lock:
            for s, e in zip(slots, ext):
                self.store.set_ext(str(int(s)), e)

    def reset_accounts(self, slots) -> None:
        with self._lock:
            for s in slots:
                self.store.accounts.pop(str(int(s)), None)

    def ingest(self, events: np.ndarray) -> None:
        with self._lock:
            for row in events:
                s = int(row["slot"])
                if s >= 0:
                    self.store.apply(TxEvent(str(s), int(row["amount"]), int(row["tx_type"]) & 0xFF,
                                             int(row["dev_hash"]), int(row["ip_hash"]), int(row["ts"])))

    # ------------------------------------------------------------------ scoring
    def _features(self, row, now: int):
        s = int(row["slot"])
        key = str(s) if s >= 0 else "__unknown__"
        f = self.store.raw_features(key, now, ip_hash=int(row["ip_hash"]))
        if s < 0:
            f["_partial"] = True
        bl = self.store.blacklisted([int(row["dev_hash"]), int(row["fp_hash"]), int(row["ip_hash"])], now)
        amount, tx = int(row["amount"]), int(row["tx_type"]) & 0xFF
        rule, reasons = GS.apply_rules(self.scoring, f, amount, tx, bl)
        st = self.store.accounts.get(key) if s >= 0 else None
        x = model_input(f, amount, tx, self.cfg.features.log_transform, self.cfg.features.width,
                        st.ext if st is not None else None)
        return f, bl, rule, reasons, x

    def _ml(self, X: np.ndarray):
        n = len(X)
        if self.model == "none" or n == 0:
            return [None] * n
        if self.model == "heuristic":
            return [GS.heuristic_predict(x) for x in X]
        try:
            y = self.executor.run({self.input_name: np.ascontiguousarray(X, np.float32)})
            yv = y[self.output_name] if self.output_name in y else list(y.values())[-1]
            yv = np.asarray(yv, np.float32).reshape(n, -1)[:, self.ml_col]
        except Exception:  # model error -> neutral score (engine.go:279-282)
            return [self.scoring.ml_error_score] * n
        return [self.scoring.ml_error_score if not np.isfinite(v) else GS.clamp01_f32(v) for v in yv]

    def score(self, req: np.ndarray, now: Optional[int] = None, want_features: bool = True,
              update: bool = True) -> Result:
        now = int(time.time()) if now is None else int(now)
        n = len(req)
        sc = np.zeros(n, np.int32); rs = np.zeros(n, np.int32); act = np.zeros(n, np.int32)
        rmask = np.zeros(n, np.int32); mlv = np.zeros(n, np.float32)
        feats = np.zeros(n, FEATREC)
        with self._lock:
            self._sync_tables()
            rows = [self._features(r, now) for r in req]
            ml = self._ml(np.stack([r[4] for r in rows]) if n else np.zeros((0, self.cfg.features.width)))
            for i, (f, bl, rule, reasons, _) in enumerate(rows):
                score, action, rr, m = GS.ensemble(self.scoring, rule, reasons, ml[i])
                sc[i], act[i], rs[i], mlv[i] = score, action, rule, m
                rmask[i] = sum(1 << REASON_BIT[r] for r in rr)
                if want_features:
                    feats[i] = _featrec_from_golden(f, req[i], bl, rule, reasons)
            if update:  # score-then-update, in request order (engine.go:486-488)
                for row in req:
                    s = int(row["slot"])
                    if s >= 0:
                        self.store.apply(TxEvent(str(s), int(row["amount"]), int(row["tx_type"]) & 0xFF,
                                                 int(row["dev_hash"]), int(row["ip_hash"]), now))
        res = pack_results(sc, rs, act, rmask, mlv, np.full(n, self.model != "none"))
        return res, (feats if want_features else None)

    def submit(self, req: np.ndarray, now: Optional[int] = None, want_features: bool = True):
        return self.score(req, now, want_features)

    def collect(self, pending) -> Result:
        return pending

    def features(self, slot: int, now: int) -> np.ndarray:
        r = np.zeros(1, REQREC)
        r["slot"], r["tx_type"] = slot, 255
        with self._lock:
            self._sync_tables()
            f, bl, rule, reasons, _ = self._features(r[0], now)
        return _featrec_from_golden(f, r[0], bl, rule, reasons)

    def features_many(self, slots, now: int) -> np.ndarray:
        return np.array([self.features(int(s), now) for s in slots], FEATREC).reshape(-1)

    def event_history(self, slot: int) -> np.ndarray:
        with self._lock:
            return self.store.event_history(str(slot))

    def metrics(self) -> Optional[np.ndarray]:
        return None

    # ------------------------------------------------------------------ durability
    def snapshot(self, path: str) -> None:
        """JSON snapshot of the host feature state (our own file format; no pickle)."""
        import base64
        import dataclasses
        import json
        import os
        out = {}
        with self._lock:
            for k, st in self.store.accounts.items():
                d = {f.name: getattr(st, f.name) for f in dataclasses.fields(st)}
                d["hll_dev"] = base64.b64encode(bytes(st.hll_dev)).decode()
                d["hll_ip"] = base64.b64encode(bytes(st.hll_ip)).decode()
                d["batch"] = dataclasses.asdict(st.batch) if st.batch is not None else None
                d["ext"] = None if st.ext is None else np.asarray(st.ext, np.float32).tolist()
                d["events"] = [np.asarray(e, np.float32).tolist() for e in st.events]
                out[k] = d
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(dict(version=1, ring_size=self.cfg.features.ring_size, accounts=out), f)
        os.replace(tmp, path)

    def restore(self, path: str) -> int:
        import base64
        import json
        from ..golden.features import AccountState
        with open(path) as f:
            data = json.load(f)
        if data["ring_size"] != self.cfg.features.ring_size:
            raise ValueError("snapshot ring size differs from the configured ring size")
        with self._lock:
            for k, d in data["accounts"].items():
                d["hll_dev"] = bytearray(base64.b64decode(d["hll_dev"]))
                d["hll_ip"] = bytearray(base64.b64decode(d["hll_ip"]))
                d["batch"] = BatchFeatures(**d["batch"]) if d["batch"] is not None else None
                d["ext"] = None if d["ext"] is None else np.asarray(d["ext"], np.float32)
                d["events"] = [np.asarray(e, np.float32) for e in d["events"]]
                self.store.accounts[k] = AccountState(**d)
        return len(data["accounts"])


class BatchTimeout(TimeoutError):
    """A device batch overran the watchdog deadline (its slot is quarantined until it drains)."""


class GpuBackend:
    """One GPU shard: HBM feature store + captured-graph scorer."""

    kind = "gpu"
    snapshot_ext = "npz"

    def __init__(self, cfg: Config, capacity: int, device, plan=None, model: str = "plan",
                 blacklist: Optional[Blacklist] = None, ipintel: Optional[IPIntel] = None,
                 capture: bool = True, owner_filter: bool = False, rank: int = 0, exchange: Optional[dict] = None):
        """``exchange``: dict(comms, world, senders, cbuckets) -> the shard is one rank of an
        owner-routed data-parallel group (engine/dp.py): batches arrive through the RCCL
        exchange and only this GPU's own rows are scored."""
        import torch
        from ..features.device_store import DeviceFeatureStore
        self.torch = torch
        self.cfg = cfg
        from ..ops.kernels import as_device
        self.device = as_device(device)
        self.exchange = exchange
        self.rank = rank
        self.owner_filter = owner_filter
        dmax = exchange["senders"] * max(exchange["cbuckets"]) if exchange else max(cfg.gpu.buckets)
        self.store = DeviceFeatureStore(capacity, cfg.features, self.device, events=True,
                                        blacklist=blacklist, ipintel=ipintel, max_events=dmax)
        self.blacklist, self.ipintel = self.store.blacklist, self.store.ipintel
        # read-your-writes for every reader of this shard's store (GetFeatures, event history,
        # CheckBonusAbuse steps): each scoring driver publishes its batches' state-stage events
        # here, a reader's stream waits for the latest one (csrc/kernels/state_clock.h). One clock
        # per shard, kept across scorer rebuilds (failover, hot reload)
        from ..ops import kernels as _K
        self.state_clock = _K._mod().StateClock()
        # the exchange scorer too runs serve_depth slots (it was pinned to 3 while the dedup ring
        # held 4 regions; at 3 the serving core's stepper waited ~50 us per step for a slot,
        # round-5 slot-cycle stats)
        self.scorer = self._make_scorer(plan, model, cfg.gpu.serve_depth if cfg.gpu.native_serving else 2)
        if capture and self.scorer.use_graphs:
            self.scorer.capture()
        self._lock = threading.RLock()
        self._slot_locks = [threading.Lock() for _ in range(self.scorer.depth)]
        self._fx = None
        self._watch = None               # EventWatch (csrc/kernels/watch.hip), made on first use
        self.quarantined: set = set()    # slots whose batch overran its deadline, not yet drained
        self.on_drained = None           # callback(backend) once every quarantined slot drained
        self.timeouts = 0
        # native serving core (engine/serving.py): once attached, EVERY batch of this shard goes
        # through it (its stepper owns the driver's slots and batch sequence)
        self.core = None
        self._core_pool = None

    def native_device(self):
        """The scorer's device object for the serving core (None: no native driver)."""
        from .serving import gpu_device
        return gpu_device(self.scorer)

    def attach_core(self, core) -> None:
        import concurrent.futures as cf
        self.core = core
        self._core_pool = cf.ThreadPoolExecutor(max_workers=8, thread_name_prefix=f"core-{self.device}")

    def swap_model(self, fm, mkind: str, version: Optional[int] = None) -> None:
        """Model hot-reload: drain the shard, build a scorer for the new plan on the same HBM
        feature store (new graphs, same store, batch sequence and metrics carried over so the
        dedup region ring stays consistent), swap it in. Scoring resumes with the new model;
        ``version`` becomes the serving core's audit stamp while nothing is in flight."""
        from ..models.plan import compile_onnx, to_device
        torch = self.torch
        plan = to_device(compile_onnx(fm), self.device, self.cfg.fraud_model.precision) if mkind == "onnx" else None
        model = {"onnx": "plan", "heuristic": "heuristic", "none": "none"}[mkind]
        core = self.core
        with self._lock:
            if core is not None:
                core.pause()  # every issued step completed (exchange: every rank converged)
            for lk in self._slot_locks:
                lk.acquire()
            try:
                old = self.scorer
                torch.cuda.synchronize(self.device)
                sc = self._make_scorer(plan, model, old.depth, use_graphs=old.use_graphs)
                # dedup regions rotate by batch seq (one is still dirty)
                sc._seq = core.seq if core is not None else old._seq
                sc.metrics = old.metrics
                sc.refresh_config(getattr(old, "scoring", None))
                if old.graphs and sc.use_graphs:
                    sc.capture()
                torch.cuda.synchronize(self.device)
                self.scorer = sc
                if core is not None:
                    core.set_device(self.native_device())
                    if version is not None:
                        core.set_model_version(int(version))
            finally:
                for lk in self._slot_locks:
                    lk.release()
                if core is not None:
                    core.resume()

    def _make_scorer(self, plan, model: str, depth: int, use_graphs=None):
        if self.exchange is not None:
            from .dp import DpGpuScorer, map_results_region
            x = self.exchange
            if isinstance(x.get("results_shm"), str):  # mapped once; a hot reload's scorer reuses it
                x["results_shm"] = map_results_region(x["results_shm"], depth, x["world"], max(x["cbuckets"]),
                                                      rows=bool(x.get("rows_shm")))
            sc = DpGpuScorer(self.cfg, self.store, x["comms"], x["world"], self.rank, x["senders"], x["cbuckets"],
                             plan=plan, model=model, device=self.device, pipeline_depth=depth,
                             results_shm=x.get("results_shm"))
        else:
            from .scorer import GpuScorer
            sc = GpuScorer(self.cfg, self.store, plan=plan, model=model, device=self.device, pipeline_depth=depth,
                           owner_filter=self.owner_filter, rank=self.rank, use_graphs=use_graphs)
        sc.state_clock = self.state_clock  # before capture(), which makes the native driver
        return sc

    def wait_state(self, stream) -> None:
        """Order ``stream`` (a torch stream) after the last scoring batch's state stage issued so
        far on this shard (read-your-writes, csrc/kernels/state_clock.h)."""
        self.state_clock.wait(stream.cuda_stream)

    def exchange_score(self, req: Optional[np.ndarray], owners: Optional[np.ndarray], C: int, now: int,
                       want_features: bool, timeout_s: Optional[float] = None) -> Result:
        """One owner-routed exchange step (collective over the group): this rank's ingress
        rows (None on a non-ingress rank) go to their owners; this GPU scores the rows it
        owns; returns the ingress rows' (res, feats) in request order. ``timeout_s``: the
        step's deadline (past it the RCCL communicators are aborted, TimeoutError)."""
        sc = self.scorer
        with self._lock:
            slot = sc.next_slot()
        self._slot_locks[slot].acquire()
        try:
            with self._lock:
                if req is None:
                    p = sc.submit_chunks(slot, C, now, None, want_features)
                else:
                    p = sc.submit_rows(slot, req, owners, now, want_features, C=C)
            res, feats = sc.wait_x(p, timeout_s=timeout_s)
        finally:
            self._slot_locks[slot].release()
        if req is None:
            return res, feats
        return res, (feats.copy() if feats is not None else None)

    def refresh_config(self, scoring=None) -> None:
        with self._lock:
            with self.torch.cuda.stream(self.scorer.stream):
                self.scorer.refresh_config(scoring)
            self.scorer.stream.synchronize()

    def set_batch_rows(self, slots, rows) -> None:
        with self._lock:
            self.store.set_batch_features(np.asarray(slots), rows)
            self.torch.cuda.synchronize(self.device)

    def set_ext(self, slots, ext) -> None:
        with self._lock:
            self.store.set_ext(np.asarray(slots), ext)
            self.torch.cuda.synchronize(self.device)

    def reset_accounts(self, slots) -> None:
        with self._lock:
            self.store.reset_accounts(slots)
            self.torch.cuda.synchronize(self.device)

    def ingest(self, events: np.ndarray) -> None:
        """IngestEvents: ordered feature update without scoring (standalone dedup region)."""
        from ..ops import kernels as K
        torch = self.torch
        with self._lock:
            for i in range(0, len(events), self.store.dmax):
                chunk = np.ascontiguousarray(events[i:i + self.store.dmax], REQREC)
                t = torch.from_numpy(chunk.view(np.uint8).copy()).to(self.device)
                with torch.cuda.stream(self.scorer.stream):
                    K.feature_update(self.store, self.scorer.cfg_dev, t, len(chunk), n=len(chunk))
                self.scorer.stream.synchronize()

    def submit(self, req: np.ndarray, now: Optional[int] = None, want_features: bool = True):
        """Launch the batch (chunks of the largest bucket); returns a handle for :meth:`collect`.
        A pipeline slot's pinned buffers are reused only after its results were collected."""
        if self.core is not None:
            rows = np.ascontiguousarray(req, REQREC).view(np.uint8)
            fut = self._core_pool.submit(self.core.score_rows, rows, None, int(now), bool(want_features))
            return ("core", fut, bool(want_features))
        sc = self.scorer
        pend = []
        n = len(req)
        for i in range(0, max(n, 1), sc.bmax):
            chunk = req[i:i + sc.bmax]
            with self._lock:
                slot = sc.next_slot()
            self._slot_locks[slot].acquire()
            try:
                with self._lock:
                    pend.append(sc.submit_into(slot, chunk, now, want_features))
            except BaseException:
                self._slot_locks[slot].release()
                raise
        return pend

    def collect(self, pend, timeout_s: Optional[float] = None) -> Result:
        """Results of :meth:`submit`'s batches. ``timeout_s``: the watchdog deadline per batch,
        an event wait (no polling). A batch that overruns it is quarantined with every batch
        behind it: their slots stay locked (never reused) until a drain thread has seen them
        complete, then ``on_drained`` fires; the caller gets :class:`BatchTimeout`."""
        if isinstance(pend, tuple) and pend[0] == "core":
            try:
                res, feat = pend[1].result()
            except RuntimeError as e:
                if "deadline" in str(e):  # the core answered at the deadline; the step drains later
                    self._quarantine_core()
                    raise BatchTimeout(f"GPU batch exceeded its deadline on {self.device}") from e
                raise
            return np.asarray(res, np.uint32).reshape(-1, 2), (feat.view(FEATREC).reshape(-1) if pend[2] else None)
        res, feats = [], []
        release = list(pend)
        try:
            for i, p in enumerate(pend):
                if timeout_s is not None and not self.scorer.done(p):
                    if self._watch is None:
                        from ..native import hipk
                        self._watch = hipk().EventWatch()
                    if not self._watch.wait_for(self.scorer.done_event(p), timeout_s * 1e3):
                        release = list(pend[:i])
                        self._quarantine(list(pend[i:]))
                        raise BatchTimeout(f"GPU batch exceeded {timeout_s * 1e3:.0f} ms on {self.device}")
                r, f = self.scorer.wait(p, unpack=False)
                res.append(r.view(np.uint32).reshape(-1, 2))
                if f is not None:
                    feats.append(f.view(FEATREC).reshape(-1))
        finally:
            for p in release:
                self._slot_locks[p.slot].release()
        want = bool(pend) and pend[0].want_features
        return np.concatenate(res), (np.concatenate(feats) if want else None)

    def stall(self, ms: float) -> None:
        """Fault injection: queue a ``ms`` device stall on the copy stream (ahead of the next
        batch's graphs)."""
        from ..native import hipk
        hipk().stall(self.scorer.cstream.cuda_stream, float(ms) * 1e3)

    def _quarantine_core(self) -> None:
        """The serving core keeps an overrunning step's slot until the device finished it;
        watch for that, then report the shard drained (``on_drained``)."""
        import time as _t
        with self._lock:
            self.timeouts += 1
            self.quarantined.add("core")
        core = self.core

        def drain():
            _t.sleep(0.01)
            while core.late_steps > 0:
                _t.sleep(0.005)
            with self._lock:
                self.quarantined.discard("core")
            cb = self.on_drained
            if cb is not None and not self.quarantined:
                cb(self)
        threading.Thread(target=drain, daemon=True, name=f"gpu-drain-{self.device}").start()

    def _quarantine(self, pend) -> None:
        """Keep the overrunning batches' slots out of service and drain them on a thread that
        blocks (GIL released) until the device finishes them; a batch that never finishes
        keeps its slot quarantined (the engine re-homes the shard after ``rehome_after_s``)."""
        with self._lock:
            self.timeouts += 1
            self.quarantined.update(p.slot for p in pend)
        sc = self.scorer

        def drain():
            for p in pend:
                try:
                    sc.wait(p, unpack=False)
                except Exception:  # device error: the slot stays quarantined
                    return
                with self._lock:
                    self.quarantined.discard(p.slot)
                self._slot_locks[p.slot].release()
            cb = self.on_drained
            if cb is not None and not self.quarantined:
                cb(self)
        threading.Thread(target=drain, daemon=True, name=f"gpu-drain-{self.device}").start()

    def close(self) -> None:
        """Release the exchange (graphs, then the RCCL communicators) once the serving core that
        issues its steps has stopped; a plain single-GPU shard holds nothing to release."""
        sc = self.scorer
        if self.exchange is not None and hasattr(sc, "close"):
            sc.close()

    def leave_exchange(self, timeout_s: float = 5.0) -> None:
        """Failover (rank 0 of a failed SPMD group): abort the RCCL exchange and serve this
        shard through the plain single-GPU pipeline on the same HBM store (new scorer and
        graphs; batch sequence and metrics carried over)."""
        if self.exchange is None:
            return
        torch = self.torch
        old = self.scorer
        with self._lock:
            old.abort_exchange()
            ev = torch.cuda.Event()
            ev.record(old.mstream)
            from ..native import hipk
            if not hipk().EventWatch().wait_for(int(ev.cuda_event), timeout_s * 1e3):
                raise TimeoutError("the exchange streams did not drain after the abort")
            torch.cuda.synchronize(self.device)
            old.release_graphs()  # their references to the aborted communicators go now, not at GC
            self.exchange = None
            sc = self._make_scorer(old.plan, old.model, 2, use_graphs=old.use_graphs)
            sc._seq = old._seq
            sc.metrics = old.metrics
            sc.refresh_config(getattr(old, "scoring", None))
            if sc.use_graphs:
                sc.capture()
            torch.cuda.synchronize(self.device)
            self._slot_locks = [threading.Lock() for _ in range(sc.depth)]
            self.scorer = sc

    def score(self, req: np.ndarray, now: Optional[int] = None, want_features: bool = True,
              update: bool = True) -> Result:
        if not update:
            raise ValueError("the GPU scorer always applies score-then-update")
        return self.collect(self.submit(req, now, want_features))

    FX_ROWS = 1024  # rows per K1 launch of the feature read path

    def features(self, slot: int, now: int) -> np.ndarray:
        """GetFeatures: K1 on a synthetic request for ``slot`` (no update)."""
        return self.features_many(np.array([slot], np.int32), now)[0]

    def features_many(self, slots, now: int) -> np.ndarray:
        """Feature rows of many accounts in one K1 launch per 1024 (no update): batched
        GetFeatures / the CheckBonusAbuse rule signals. Returns FEATREC [n]."""
        from ..ops import kernels as K
        torch = self.torch
        slots = np.asarray(slots, np.int32)
        out = np.zeros(len(slots), FEATREC)
        R = self.FX_ROWS
        st = self.scorer.stream
        with self._lock:
            if self._fx is None:
                # zero-filled ON the stream that uses them: torch.zeros on the default stream
                # raced the first read's slab copy on the state stream (the fill landed after the
                # copy: n = 0, every row inert -> the one-off all-zero GetFeatures of round 4,
                # profiles/NOTES.md "read consistency")
                with torch.cuda.stream(st):
                    self._fx = dict(slab=torch.zeros(16 + 48 * R, dtype=torch.uint8, device=self.device),
                                    X=torch.zeros((R, self.cfg.features.width), dtype=torch.float32,
                                                  device=self.device),
                                    feat=torch.zeros((R, 32), dtype=torch.int32, device=self.device))
            fx = self._fx
            for i in range(0, len(slots), R):
                sl = slots[i:i + R]
                n = len(sl)
                h = np.zeros(1, [("n", "<i4"), ("seq", "<i4"), ("now", "<i8")])
                h["n"], h["now"] = n, now
                r = np.zeros(n, REQREC)
                r["slot"], r["tx_type"], r["ts"] = sl, 255 | (self.scorer.rank << 8), now
                buf = np.concatenate([h.view(np.uint8), r.view(np.uint8)])
                bucket = 64 if n <= 64 else R
                with torch.cuda.stream(st):
                    self.wait_state(st)  # every scoring batch issued before this read (read-your-writes)
                    fx["slab"][:len(buf)].copy_(torch.from_numpy(buf))
                    K.feature_assemble(self.store, fx["slab"][:16].view(torch.int64), self.scorer.cfg_dev,
                                       fx["slab"][16:16 + 48 * bucket], fx["X"], fx["feat"], bucket)
                    host = fx["feat"][:n].cpu()
                out[i:i + n] = host.numpy().view(FEATREC).reshape(-1)
        return out

    def event_history(self, slot: int) -> np.ndarray:
        """[event_ring, event_dim] f32, oldest first, right-aligned (GRU input)."""
        torch = self.torch
        st = self.scorer.stream
        with self._lock, torch.cuda.stream(st):
            self.wait_state(st)  # after the state stage of every batch issued so far
            raw = self.store.ev[slot].cpu().numpy()
            rt = self.store.read_rt(slot)
        ev = (raw.view(np.uint16).astype(np.uint32) << 16).view(np.float32)
        R = ev.shape[0]
        head, cnt = int(rt["ev_head"]), min(int(rt["ev_count"]), R)
        out = np.zeros_like(ev)
        if cnt:
            idx = [(head - cnt + i) % R for i in range(cnt)]
            out[R - cnt:] = ev[idx]
        return out

    def metrics(self) -> np.ndarray:
        return self.scorer.read_metrics()


class NativeCpuBackend:
    """CPU shard on the C++ ``CpuScorer`` (csrc/runtime/cpu_scorer.cpp): the same SoA state and
    record formats as the GPU store, GIL released while scoring. The default CPU backend."""

    kind = "cpu"
    snapshot_ext = "npz"

    def __init__(self, cfg: Config, capacity: int, model: str = "heuristic", executor=None,
                 input_name: str = "input", output_name: str = "output", ml_col: int = 0,
                 blacklist: Optional[Blacklist] = None, ipintel: Optional[IPIntel] = None):
        from ..native import native
        if model == "plan" and executor is None:
            model = "none"
        self.cfg = cfg
        self.model = model
        f = cfg.features
        self.sc = native().CpuScorer(int(capacity), f.ring_size, f.event_ring, f.event_dim, f.width - 30)
        self.sc.set_model(executor if model == "plan" else None, input_name, output_name, ml_col)
        self.blacklist = blacklist or Blacklist()
        self.ipintel = ipintel or IPIntel()
        self.scoring = cfg.scoring
        self._tables_version = None
        self._lock = threading.RLock()
        self.refresh_config()

    core = None

    def native_device(self, depth: int = 2, cap: int = 8192):
        """A CpuDevice over this shard's CpuScorer for the serving core."""
        from ..native import native
        self._device = native().CpuDevice(self.sc, int(depth), int(cap))
        return self._device

    def attach_core(self, core) -> None:
        self.core = core

    def exchange_device(self, shm_name: str, world: int, rank: int, depth: int, C: int, create: bool,
                        timeout_s: float):
        """This shard as one rank of a CPU data-parallel group: the owner-routed exchange over
        /dev/shm (csrc/runtime/cpu_device.cpp ShmXchgDevice)."""
        from ..native import native
        self._device = native().ShmXchgDevice(self.sc, shm_name, int(world), int(rank), int(depth), int(C),
                                              bool(create), float(timeout_s))
        from ..utils.faults import Faults
        f = Faults()  # FAULT_INJECT=xchg_stall_results:file=P - this owner stops publishing results
        if f.active("xchg_stall_results"):
            self._device.debug_stall_results_when(f.params("xchg_stall_results")["file"])
        return self._device

    @property
    def rows_scored(self) -> int:
        """Rows this shard scored through the exchange (its own accounts only)."""
        d = getattr(self, "_device", None)
        return int(d.rows_scored) if d is not None and hasattr(d, "rows_scored") else 0

    def swap_model(self, fm, mkind: str, version: Optional[int] = None) -> None:
        """Model hot-reload: the C++ scorer's executor is replaced between batches (with the
        serving core paused, so ``version`` stamps exactly the rows of the new model)."""
        spec = cpu_model_spec(self.cfg, fm, mkind)
        core = self.core
        with self._lock:
            if core is not None:
                core.pause()
            try:
                self.model = spec["model"]
                self.sc.set_model(spec["executor"] if self.model == "plan" else None, spec["input_name"],
                                  spec["output_name"], spec["ml_col"])
                self.refresh_config()
                if core is not None and version is not None:
                    core.set_model_version(int(version))
            finally:
                if core is not None:
                    core.resume()

    def refresh_config(self, scoring=None) -> None:
        from ..layouts import MODEL_HEURISTIC, MODEL_NONE, MODEL_OUTPUT, score_cfg
        with self._lock:
            if scoring is not None:
                self.scoring = scoring
            b, t = self.blacklist.table, self.ipintel.table
            kind = {"none": MODEL_NONE, "heuristic": MODEL_HEURISTIC, "plan": MODEL_OUTPUT}[self.model]
            c = score_cfg(self.cfg, kind, sc=self.scoring, bl_mask=b.mask, bl_max_probe=max(b.max_probe, 1),
                          ip_mask=t.mask, ip_max_probe=max(t.max_probe, 1))
            self.sc.set_cfg(c.view(np.uint8))
            v = (b.version, t.version)
            if v != self._tables_version:
                self.sc.set_tables(b.keys, b.vals, t.keys, t.vals)
                self._tables_version = v

    def _sync(self) -> None:
        if (self.blacklist.table.version, self.ipintel.table.version) != self._tables_version:
            self.refresh_config()

    def set_batch_rows(self, slots, rows) -> None:
        self.sc.set_batch(np.asarray(slots, np.int32), np.ascontiguousarray(rows, ACCTBATCH).view(np.uint8))

    def set_ext(self, slots, ext) -> None:
        if self.cfg.features.width > 30:
            self.sc.set_ext(np.asarray(slots, np.int32), np.asarray(ext, np.float32).reshape(len(slots), -1))

    def reset_accounts(self, slots) -> None:
        self.sc.reset(np.asarray(slots, np.int32))

    def ingest(self, events: np.ndarray) -> None:
        self.sc.ingest(np.ascontiguousarray(events, REQREC).view(np.uint8))

    def score(self, req: np.ndarray, now: Optional[int] = None, want_features: bool = True,
              update: bool = True) -> Result:
        now = int(time.time()) if now is None else int(now)
        self._sync()
        if self.core is not None and update:  # batches of this shard go through its serving core
            res, feat = self.core.score_rows(np.ascontiguousarray(req, REQREC).view(np.uint8), None, now,
                                             bool(want_features))
            return res, (feat.view(FEATREC).reshape(-1) if feat is not None else None)
        res, feat = self.sc.score(np.ascontiguousarray(req, REQREC).view(np.uint8), now, update, want_features)
        return res, (feat.view(FEATREC).reshape(-1) if feat is not None else None)

    def submit(self, req: np.ndarray, now: Optional[int] = None, want_features: bool = True):
        return self.score(req, now, want_features)

    def collect(self, pending) -> Result:
        return pending

    def features(self, slot: int, now: int) -> np.ndarray:
        self._sync()
        return self.sc.features(int(slot), int(now)).view(FEATREC)[0]

    def features_many(self, slots, now: int) -> np.ndarray:
        self._sync()
        return np.array([self.sc.features(int(s), int(now)).view(FEATREC)[0] for s in slots], FEATREC).reshape(-1)

    def event_history(self, slot: int) -> np.ndarray:
        return self.sc.event_history(int(slot))

    def metrics(self):
        return None

    def snapshot(self, path: str) -> None:
        import os
        st = self.sc.state()
        tmp = path + ".tmp.npz"
        # version 2: AcctRT carries the cached HLL estimates (version 1 files get them rebuilt)
        np.savez(tmp, version=np.array([2]), ring_size=np.array([self.cfg.features.ring_size]), **st)
        os.replace(tmp, path)

    def restore(self, path: str) -> int:
        with np.load(path, allow_pickle=False) as z:
            if int(z["ring_size"][0]) != self.cfg.features.ring_size:
                raise ValueError("snapshot ring size differs from the configured ring size")
            st = {k: z[k] for k in ("ring_ts", "ring_amt", "hll", "rt", "batch", "ext", "ev")}
            if int(z["version"][0]) < 2 and st["rt"].size:  # before AcctRT cached the HLL estimates
                from ..golden.hll import refresh_cached_counts
                from ..layouts import ACCTRT
                rt = np.ascontiguousarray(st["rt"]).copy()
                refresh_cached_counts(st["hll"], rt.view(np.uint8).reshape(-1, ACCTRT.itemsize).view(ACCTRT).reshape(-1))
                st["rt"] = rt
            self.sc.load_state(st)
        return self.sc.capacity

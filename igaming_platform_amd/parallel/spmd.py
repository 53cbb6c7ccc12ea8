"""SPMD multi-GPU serving: one process per GPU, every rank ingests.

Data parallelism by account owner (``owner = XXH64(account_id) % world``):
every account's feature state lives on exactly one rank. The hot path is each rank's native
serving core (engine/serving.py, csrc/runtime/serve_core.cpp): its own ingress (gRPC
listener / bench threads) parses and resolves requests through the node-shared account
registry (/dev/shm), and its stepper issues owner-routed exchange steps (RCCL all-to-all over
xGMI between GPUs, /dev/shm between CPU shards): every rank scores ONLY the rows it owns and
the results return to the ingress rank. Ranks keep their step sequences aligned through a
shared step clock; no host collective, no lock and no header broadcast per step.

This module is the control plane (cold ops) over gloo: rank 0 broadcasts an op (thresholds,
blacklist/ip tables, warehouse rows, GetFeatures, event histories, GRU abuse scores,
snapshots, model reloads) and every rank applies it to its local shard; state-changing ops
end with a barrier, so a request any rank ingests after the op returned sees it everywhere.

Failure handling (reference: engine.go:279-282 degrades a failed model call,
cmd/main.go:329-342 recovers a failed handler): every collective rank 0 issues carries a
deadline (:mod:`.comm`), a heartbeat op (OP_PING, an all-reduce of ones) runs every
``heartbeat_s`` so a dead worker is noticed while the API is idle too, and an exchange step a
peer never joins fails at the step deadline. The first failure marks the group failed
(:class:`GroupFailure`) and calls ``on_failure``: the engine then scores that batch on its
stateless fallback, leaves the group and re-homes every remote shard onto rank 0 from its
snapshot (engine/risk_engine.py ``_group_failed``). A surviving worker whose collective fails
aborts its serving core and writes a final snapshot of its shard next to the periodic ones
(``shard<r>.<ext>`` + ``shard<r>.final``) before it exits, so its state is re-homed without
loss; a dead worker's shard comes back from its last periodic snapshot.
"""
from __future__ import annotations

import dataclasses
import io
import json
import logging
import os
import threading
import time

import numpy as np

from ..config import RuleWeights, ScoringConfig
from ..layouts import ACCTBATCH, FEATREC, REQREC  # noqa: F401  (REQREC: OP_INGEST rows)

OP_INGEST, OP_CONFIG, OP_TABLES, OP_BATCH, OP_EXT, OP_FEATURES, OP_RESET, OP_STOP, OP_EVHIST, \
    OP_ABUSE, OP_SNAPSHOT, OP_RESTORE, OP_RELOAD, OP_FEATMANY, OP_PING, OP_METRICS, OP_LTVROWS, OP_LTV = range(2, 20)
MUTATING = (OP_INGEST, OP_CONFIG, OP_TABLES, OP_BATCH, OP_EXT, OP_RESET, OP_RELOAD, OP_LTVROWS)
LTV_COLS = 25  # golden.ltv.PLAYER_COLUMNS
MET_WORDS = 128   # K10 device counter block (csrc/include/records.h MET_*); [106] = rows scored

log = logging.getLogger("igaming_platform_amd.spmd")

# slots beyond the last count rank 0 announced that a survivor's final snapshot also covers
# (accounts created since the previous heartbeat)
FINAL_SNAPSHOT_MARGIN = 65536


class GroupFailure(RuntimeError):
    """A collective of the SPMD group failed or missed its deadline (a rank died or hung)."""


def owners_of(req: np.ndarray) -> np.ndarray:
    return (req["tx_type"] >> 8) & 0xFF


def _tables_bytes(blacklist, ipintel) -> bytes:
    buf = io.BytesIO()
    bt, it = blacklist.table, ipintel.table
    np.savez(buf, bl_keys=bt.keys, bl_vals=bt.vals, bl_meta=np.array([bt.max_probe, bt.n], np.int64),
             ip_keys=it.keys, ip_vals=it.vals, ip_meta=np.array([it.max_probe, it.n], np.int64))
    return buf.getvalue()


def _load_tables(data: bytes, blacklist, ipintel) -> None:
    with np.load(io.BytesIO(data), allow_pickle=False) as z:
        for tab, p in ((blacklist.table, "bl"), (ipintel.table, "ip")):
            if len(z[f"{p}_keys"]) != tab.cap:
                raise ValueError("table capacity differs across ranks")
            with tab._lock:
                tab.keys[:] = z[f"{p}_keys"]
                tab.vals[:] = z[f"{p}_vals"]
                tab.max_probe, tab.n = int(z[f"{p}_meta"][0]), int(z[f"{p}_meta"][1])
                tab.version += 1


def scoring_to_json(s: ScoringConfig) -> bytes:
    return json.dumps(dataclasses.asdict(s)).encode()


def scoring_from_json(b: bytes) -> ScoringConfig:
    d = json.loads(b.decode())
    d["weights"] = RuleWeights(**d["weights"])
    return ScoringConfig(**d)


class ShardRunner:
    """What every rank (0 included) executes for one cold op on its local backend."""

    def __init__(self, comm, backend, abuse_gpu=None, core=None, ltv=None):
        self.comm = comm
        self.be = backend
        self.rank = comm.rank
        self.abuse_gpu = abuse_gpu
        self.core = core  # this rank's serving core (paused around snapshots / restores)
        self.ltv = ltv    # this rank's LTV shard (engine/ltv.py LtvService holding its own accounts)
        self.acct = None  # this rank's native account-RPC router (engine/acct.py NativeAcct)
        self.abuse_threshold = 0.7
        self.abuse_link_wait_us = 200
        self.model_version = 1  # fraud-model reloads applied (audit stamp of the core's rows)
        self.snapshot_dir = None  # the directory of the last OP_SNAPSHOT (final snapshot on failure)
        self.used = [0] * comm.world  # slots in use per rank (the shared registry, via OP_PING)

    @property
    def rows_scored(self) -> int:
        """Rows this rank scored through the exchange (its own accounts only): the device
        metrics row counter on a GPU shard (K10, reads the device), the host count otherwise."""
        if self.be.kind == "gpu":
            return int(self.be.scorer.read_metrics()[106])
        return int(getattr(self.be, "rows_scored", 0))

    def local_metrics(self) -> np.ndarray:
        """This shard's K10 counters (GPU), or just its exchange row count (CPU shards)."""
        m = np.zeros(MET_WORDS, np.int64)
        if self.be.kind == "gpu":
            v = np.asarray(self.be.scorer.read_metrics(), np.int64)
            m[:min(len(v), MET_WORDS)] = v[:MET_WORDS]
        else:
            m[106] = self.rows_scored
        return m

    def _mine(self, owners: np.ndarray) -> np.ndarray:
        return owners == self.rank

    def _quiesced(self, fn):
        """Run ``fn`` with this rank's serving core paused (every rank does the same for the
        same op, so the exchange converges to one step count first)."""
        if self.core is None:
            return fn()
        self.core.pause()
        try:
            return fn()
        finally:
            self.core.resume()

    def handle(self, op: int, hdr: np.ndarray, payload: bytes):
        out = self._handle(op, hdr, payload)
        if op in MUTATING:
            # a request ingested anywhere after the op returned must see it on every shard
            self.comm.barrier()
        return out

    def _handle(self, op: int, hdr: np.ndarray, payload: bytes):
        n, now, aux, aux2 = int(hdr[1]), int(hdr[2]), int(hdr[3]), int(hdr[4])
        if op == OP_METRICS:  # every shard's K10 counter block, one row per rank (sum-reduce)
            out = np.zeros((self.comm.world, MET_WORDS), np.int64)
            out[self.rank] = self.local_metrics()
            return self.comm.sum_i64(out.reshape(-1)).reshape(self.comm.world, MET_WORDS)
        if op == OP_PING:  # heartbeat: payload = slots in use per rank; all-reduce proves liveness
            if payload:
                self.used = np.frombuffer(payload, np.int64).tolist()
            return self.comm.sum_i64(np.ones(1, np.int64))
        if op == OP_INGEST:
            ev = np.frombuffer(payload, REQREC).copy()
            mine = self._mine(owners_of(ev))
            if np.any(mine):
                self.be.ingest(ev[mine])
            return None
        if op == OP_CONFIG:
            sc = scoring_from_json(payload)
            self.be.refresh_config(sc)
            if self.acct is not None:  # the abuse signal limits of this rank's native router
                self.acct.set_abuse(sc, self.abuse_threshold, self.abuse_link_wait_us)
                self.acct.refresh()
            return None
        if op == OP_RELOAD:  # payload: ONNX bytes (empty: built-in heuristic)
            from ..native import native
            fm = native().OnnxModel.from_bytes(payload) if payload else None
            # every rank counts the reloads it applied: the same audit version stamp group-wide
            self.model_version += 1
            self.be.swap_model(fm, "onnx" if fm is not None else "heuristic", version=self.model_version)
            return None
        if op == OP_TABLES:
            _load_tables(payload, self.be.blacklist, self.be.ipintel)
            self.be.refresh_config(None)
            if self.acct is not None:
                self.acct.refresh()
            return None
        if op in (OP_BATCH, OP_EXT, OP_RESET):
            slots = np.frombuffer(payload[:4 * n], np.int32)
            owners = np.frombuffer(payload[4 * n:8 * n], np.int32)
            mine = self._mine(owners)
            body = payload[8 * n:]
            if np.any(mine):
                if op == OP_BATCH:
                    self.be.set_batch_rows(slots[mine], np.frombuffer(body, ACCTBATCH)[mine])
                elif op == OP_EXT:
                    self.be.set_ext(slots[mine], np.frombuffer(body, np.float32).reshape(n, -1)[mine])
                else:
                    self.be.reset_accounts(slots[mine])
            return None
        if op == OP_FEATURES:  # aux = owner, aux2 = slot
            rec = np.zeros(1, FEATREC)
            if aux == self.rank:
                rec[0] = self.be.features(aux2, now)
            return self.comm.sum_i64(rec.view(np.int64).reshape(-1))
        if op == OP_FEATMANY:  # payload: slots | owners; each rank fills the rows it owns
            slots = np.frombuffer(payload[:4 * n], np.int32)
            owners = np.frombuffer(payload[4 * n:8 * n], np.int32)
            recs = np.zeros(n, FEATREC)
            mine = self._mine(owners)
            if np.any(mine):
                recs[mine] = self.be.features_many(slots[mine], now)
            return self.comm.sum_i64(recs.view(np.int64).reshape(-1))
        if op == OP_EVHIST:
            h = None
            if aux == self.rank:
                h = np.ascontiguousarray(self.be.event_history(aux2), np.float32)
            shape = np.asarray(hdr[5:7], np.int64)
            buf = np.zeros(int(shape[0]) * int(shape[1]), np.float32) if h is None else h.reshape(-1)
            return self.comm.sum_i64(np.pad(buf, (0, len(buf) % 2)).view(np.int64))
        if op == OP_ABUSE:
            slots = np.frombuffer(payload[:4 * n], np.int32)
            owners = np.frombuffer(payload[4 * n:8 * n], np.int32)
            out = np.zeros(n, np.float32)
            mine = self._mine(owners)
            if np.any(mine) and self.abuse_gpu is not None:
                out[mine] = self.abuse_gpu.score_slots(slots[mine])
            return self.comm.sum_i64(np.pad(out, (0, n % 2)).view(np.int64))
        if op == OP_LTVROWS:  # payload: slots | owners | rows [n, 25] f32 | ext [n, aux] f32
            slots = np.frombuffer(payload[:4 * n], np.int32)
            owners = np.frombuffer(payload[4 * n:8 * n], np.int32)
            rows = np.frombuffer(payload[8 * n:8 * n + 4 * LTV_COLS * n], np.float32).reshape(n, LTV_COLS)
            ext = np.frombuffer(payload[8 * n + 4 * LTV_COLS * n:], np.float32).reshape(n, aux) if aux else None
            mine = self._mine(owners)
            if np.any(mine) and self.ltv is not None:
                self.ltv.set_rows(slots[mine], owners[mine], rows[mine], None if ext is None else ext[mine])
            return None
        if op == OP_LTV:  # payload: slots | owners -> [n, 7] f32 (6 outputs + profile present), sum-reduced
            slots = np.frombuffer(payload[:4 * n], np.int32)
            owners = np.frombuffer(payload[4 * n:8 * n], np.int32)
            out = np.zeros((n, 7), np.float32)
            mine = self._mine(owners)
            if np.any(mine) and self.ltv is not None:
                res, present = self.ltv.predict_owner_slots(self.rank, slots[mine])
                out[mine, :6] = res
                out[mine, 6] = present
            flat = out.reshape(-1)
            return self.comm.sum_i64(np.pad(flat, (0, len(flat) % 2)).view(np.int64))
        if op in (OP_SNAPSHOT, OP_RESTORE):  # payload: {"dir": ..., "used": [slots in use per rank]}
            import os
            meta = json.loads(payload.decode())
            path = os.path.join(meta["dir"], f"shard{self.rank}.{self.be.snapshot_ext}")
            if op == OP_SNAPSHOT:
                self.snapshot_dir = meta["dir"]
                self.used = [int(u) for u in meta["used"]] or self.used
                if self.be.kind == "gpu":
                    self._quiesced(lambda: self.be.store.snapshot(path, n_used=max(int(meta["used"][self.rank]), 1)))
                else:
                    self._quiesced(lambda: self.be.snapshot(path))
            elif self.be.kind == "gpu":
                self._quiesced(lambda: self.be.store.restore(path))
            else:
                self._quiesced(lambda: self.be.restore(path))
            self.comm.barrier()
            return None
        raise ValueError(f"unknown op {op}")

    def final_snapshot(self) -> str:
        """After the group failed: this shard's current state -> the snapshot directory of the
        last OP_SNAPSHOT (+ a ``.final`` marker rank 0's re-home waits for). Returns the path
        ('' when no snapshot directory is known)."""
        if not self.snapshot_dir or self.rank == 0:
            return ""
        path = os.path.join(self.snapshot_dir, f"shard{self.rank}.{self.be.snapshot_ext}")
        if self.be.kind == "gpu":
            xd = getattr(self.be.scorer, "abort_exchange", None)
            if xd is not None:
                xd()  # unblock the RCCL exchange kernels still waiting on the dead peer
        if self.core is not None:
            self.core.abort()  # no convergence with a dead peer; steps in flight fail at their deadline
        if self.be.kind == "gpu":
            cap = self.be.store.capacity
            self.be.store.snapshot(path, n_used=min(cap, max(int(self.used[self.rank]), 1) + FINAL_SNAPSHOT_MARGIN))
        else:
            self.be.snapshot(path)
        tmp = os.path.join(self.snapshot_dir, f"shard{self.rank}.final.tmp")
        with open(tmp, "w") as f:
            json.dump(dict(rank=self.rank, time=time.time()), f)
        os.replace(tmp, os.path.join(self.snapshot_dir, f"shard{self.rank}.final"))
        return path


class SpmdGroup:
    """Rank 0's handle on the group: issues an op to every rank and runs its own share.
    Ops are serialised (one collective sequence at a time) by a lock."""

    def __init__(self, comm, runner: ShardRunner, heartbeat_s: float = 0.0, used_fn=None, on_failure=None):
        """``heartbeat_s`` > 0: an OP_PING every that many seconds (liveness while idle; its
        payload tells the workers how many slots rank 0's registry gives each shard, from
        ``used_fn()``). ``on_failure(exc)``: called once, from the thread whose collective
        failed, when the group fails."""
        if comm.rank != 0:
            raise ValueError("SpmdGroup lives on rank 0; other ranks call run_worker()")
        self.comm = comm
        self.runner = runner
        self.world = comm.world
        self._lock = threading.Lock()
        self.failed: BaseException = None
        self.on_failure = on_failure
        self.used_fn = used_fn
        self.heartbeats = 0
        self._stop = threading.Event()
        self._hb = None
        self.heartbeat_s = float(heartbeat_s)

    def start_heartbeat(self) -> None:
        """Start the liveness op (call once the owner of ``on_failure`` is fully built)."""
        if self._hb is None and self.heartbeat_s > 0 and self.world > 1:
            self._hb = threading.Thread(target=self._heartbeat, args=(self.heartbeat_s,), daemon=True,
                                        name="spmd-heartbeat")
            self._hb.start()

    def fail(self, e: BaseException) -> "GroupFailure":
        """A hot-path exchange step failed (a peer missed its deadline): the group is failed."""
        return self._fail(e)

    def _fail(self, e: BaseException) -> "GroupFailure":
        first = self.failed is None
        if first:
            self.failed = e
            log.error("spmd group failed: %s", e)
            self._stop.set()
        if first and self.on_failure is not None:
            self.on_failure(e)
        return e if isinstance(e, GroupFailure) else GroupFailure(str(e))

    def _collective(self, fn):
        """Run ``fn`` (one op's collectives) under the group lock; a failure or missed deadline
        marks the group failed and raises :class:`GroupFailure` (now and on every later op)."""
        with self._lock:
            if self.failed is not None:
                raise GroupFailure(f"spmd group failed earlier: {self.failed}")
            try:
                return fn()
            except GroupFailure:
                raise
            except Exception as e:  # gloo: timeout / connection reset by a dead peer
                err = e
        raise self._fail(err) from err

    def _issue(self, op: int, payload: bytes = b"", n: int = 0, now: int = 0, aux: int = 0, aux2: int = 0,
               extra=(0, 0)):
        hdr = np.array([op, n, now, aux, aux2, extra[0], extra[1], 0], np.int64)

        def run():
            self.comm.bcast_i64(hdr, 0)
            self.comm.bcast_bytes(payload, 0)
            return self.runner.handle(op, hdr, payload)
        return self._collective(run)

    def ping(self) -> int:
        """One heartbeat: every rank answers (returns the number of live ranks)."""
        used = self.used_fn() if self.used_fn is not None else [0] * self.world
        payload = np.asarray(used, np.int64).tobytes()
        out = self._issue(OP_PING, payload)
        self.heartbeats += 1
        return int(out[0])

    def _heartbeat(self, every: float) -> None:
        while not self._stop.wait(every):
            try:
                self.ping()
            except GroupFailure:
                return

    # ---- cold path
    def ingest(self, ev: np.ndarray) -> None:
        self._issue(OP_INGEST, np.ascontiguousarray(ev).tobytes(), n=len(ev))

    def refresh_config(self, scoring: ScoringConfig) -> None:
        self._issue(OP_CONFIG, scoring_to_json(scoring))

    def sync_tables(self, blacklist, ipintel) -> None:
        self._issue(OP_TABLES, _tables_bytes(blacklist, ipintel))

    def reload_model(self, onnx_bytes: bytes) -> None:
        self._issue(OP_RELOAD, onnx_bytes)

    def _rows(self, op, slots, owners, body: bytes = b"") -> None:
        n = len(slots)
        self._issue(op, np.asarray(slots, np.int32).tobytes() + np.asarray(owners, np.int32).tobytes() + body, n=n)

    def set_batch_rows(self, slots, owners, rows) -> None:
        self._rows(OP_BATCH, slots, owners, np.ascontiguousarray(rows, ACCTBATCH).tobytes())

    def set_ext(self, slots, owners, ext) -> None:
        self._rows(OP_EXT, slots, owners, np.ascontiguousarray(ext, np.float32).tobytes())

    def reset_accounts(self, slots, owners) -> None:
        self._rows(OP_RESET, slots, owners)

    def features(self, owner: int, slot: int, now: int) -> np.ndarray:
        return self._issue(OP_FEATURES, now=now, aux=owner, aux2=slot).view(FEATREC)[0].copy()

    def features_many(self, slots, owners, now: int) -> np.ndarray:
        n = len(slots)
        out = self._issue(OP_FEATMANY, np.asarray(slots, np.int32).tobytes() + np.asarray(owners, np.int32).tobytes(),
                          n=n, now=now)
        return out.view(FEATREC).reshape(-1)[:n].copy()

    def event_history(self, owner: int, slot: int, shape) -> np.ndarray:
        out = self._issue(OP_EVHIST, aux=owner, aux2=slot, extra=shape)
        return out.view(np.float32)[: shape[0] * shape[1]].reshape(shape).copy()

    def abuse_scores(self, slots, owners) -> np.ndarray:
        n = len(slots)
        out = self._issue(OP_ABUSE, np.asarray(slots, np.int32).tobytes() + np.asarray(owners, np.int32).tobytes(),
                          n=n)
        return out.view(np.float32)[:n].copy()

    def ltv_rows(self, slots, owners, rows, ext=None) -> None:
        n = len(slots)
        w = 0 if ext is None else int(np.asarray(ext).shape[1])
        body = np.ascontiguousarray(rows, np.float32).tobytes()
        if ext is not None:
            body += np.ascontiguousarray(ext, np.float32).tobytes()
        self._issue(OP_LTVROWS, np.asarray(slots, np.int32).tobytes() + np.asarray(owners, np.int32).tobytes() + body,
                    n=n, aux=w)

    def ltv_predict(self, slots, owners):
        """[n, 6] LTV rows of accounts owned by any rank, and their profile-present mask."""
        n = len(slots)
        out = self._issue(OP_LTV, np.asarray(slots, np.int32).tobytes() + np.asarray(owners, np.int32).tobytes(), n=n)
        v = out.view(np.float32)[:7 * n].reshape(n, 7)
        return v[:, :6].copy(), v[:, 6] > 0.5

    def shard_metrics(self) -> np.ndarray:
        """[world, 128] device counters of every shard (one all-reduce; /metrics)."""
        return self._issue(OP_METRICS)

    def snapshot(self, directory: str, used) -> None:
        self._issue(OP_SNAPSHOT, json.dumps({"dir": directory, "used": [int(u) for u in used]}).encode())

    def restore(self, directory: str) -> None:
        self._issue(OP_RESTORE, json.dumps({"dir": directory, "used": []}).encode())

    def stop(self) -> None:
        """Release the workers (no-op once the group failed: they leave on their own); every
        rank then stops its serving core (the cores converge on one final step count)."""
        self._stop.set()
        if self.failed is not None:
            return
        hdr = np.array([OP_STOP, 0, 0, 0, 0, 0, 0, 0], np.int64)
        try:
            self._collective(lambda: self.comm.bcast_i64(hdr, 0))
        except GroupFailure:
            return
        if self.runner.core is not None:
            self.runner.core.stop()

    def abandon(self) -> None:
        """After a failure: stop the heartbeat and tear the process group down, which makes the
        surviving workers' pending collectives fail at once (they then write their final
        snapshots and exit) instead of waiting for the group timeout."""
        self._stop.set()
        try:
            import torch.distributed as dist
            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception as e:  # already broken: nothing left to release
            log.warning("destroy_process_group after failure: %s", e)


def run_worker(comm, backend, abuse_gpu=None, core=None, ltv=None, acct=None, abuse_threshold: float = 0.7,
               abuse_link_wait_us: int = 200):
    """Cold-op loop of ranks >= 1 until rank 0 sends STOP (the rank's serving core keeps
    ingesting and stepping on its own threads meanwhile). Returns (ops served, rows scored).
    When a collective fails (rank 0 or a peer died / the group was torn down), the shard
    aborts its core, writes its final snapshot (if rank 0 ever sent a snapshot directory) and
    the loop returns."""
    runner = ShardRunner(comm, backend, abuse_gpu, core, ltv)
    runner.acct, runner.abuse_threshold = acct, float(abuse_threshold)
    runner.abuse_link_wait_us = int(abuse_link_wait_us)
    served = 0
    while True:
        try:
            # idle wait for rank 0's next op: no per-op deadline (rank 0's heartbeats keep the
            # group timeout from firing while the API is idle)
            hdr = comm.bcast_i64(np.zeros(8, np.int64), 0, deadline=False)
            op = int(hdr[0])
            if op == OP_STOP:
                if acct is not None:
                    acct.stop()
                if core is not None:
                    core.stop()
                return served, runner.rows_scored
            payload = comm.bcast_bytes(None, 0)
            runner.handle(op, hdr, payload)
        except Exception as e:
            log.error("spmd worker %d: group failed (%s); writing the final snapshot", comm.rank, e)
            try:
                path = runner.final_snapshot()
                if path:
                    log.info("spmd worker %d: final snapshot %s", comm.rank, path)
            except Exception as e2:  # the shard itself is broken: rank 0 falls back to the periodic snapshot
                log.error("spmd worker %d: final snapshot failed: %s", comm.rank, e2)
            return served, -1
        served += 1


class ShardProxy:
    """Backend-shaped handle for owner ``o`` of an SPMD group (cold-path ops only; the
    engine sends scoring batches to the whole group at once)."""

    kind = "spmd"

    def __init__(self, group: SpmdGroup, owner: int, local):
        self.g, self.o, self.local = group, owner, local
        self.blacklist, self.ipintel = local.blacklist, local.ipintel

    def refresh_config(self, scoring=None) -> None:
        if self.o == 0:  # one broadcast for the whole group
            self.g.sync_tables(self.blacklist, self.ipintel)
            if scoring is not None:
                self.g.refresh_config(scoring)

    def ingest(self, ev: np.ndarray) -> None:
        ev = ev.copy()
        ev["tx_type"] = (ev["tx_type"] & 0xFF) | (self.o << 8)
        self.g.ingest(ev)

    def set_batch_rows(self, slots, rows) -> None:
        self.g.set_batch_rows(slots, np.full(len(slots), self.o, np.int32), rows)

    def set_ext(self, slots, ext) -> None:
        self.g.set_ext(slots, np.full(len(slots), self.o, np.int32), ext)

    def reset_accounts(self, slots) -> None:
        self.g.reset_accounts(slots, np.full(len(slots), self.o, np.int32))

    def features(self, slot: int, now: int) -> np.ndarray:
        return self.g.features(self.o, int(slot), now)

    def features_many(self, slots, now: int) -> np.ndarray:
        return self.g.features_many(slots, np.full(len(slots), self.o, np.int32), now)

    def event_history(self, slot: int) -> np.ndarray:
        shape = self.local.event_history(0).shape
        return self.g.event_history(self.o, int(slot), shape)

    def metrics(self):
        return None

"""Data-parallel GPU scorer: the three-stream scoring pipeline of :mod:`.scorer` behind the
owner-routed RCCL exchange of :mod:`..parallel.exchange` (one process per GPU).

Per micro-batch on every rank (``csrc/kernels/exchange.hip`` XchgDriver; no host sync, no
row-count read-back):

  xs stream    H2D  the ingress rank's chunks [world][1 + C] ReqRec + the batch header, then
               the RCCL all-to-all of the chunks (each owner gets its rows from every sender)
  copy stream  exchange_compact -> contiguous owned rows + BatchHdr.n; K6a dedup insert
  state stream K1 feature_assemble + score-then-update (unchanged graphs)
  model stream trees / MLP head / K5 ensemble -> exchange_scatter into result chunks
  ys stream    RCCL all-to-all of the results back to the senders; D2H to pinned memory

Each GPU scores only its own accounts' rows (``senders * C`` rows at most per batch: one
sender for the serving front end on rank 0, every rank in ``bench.py --gpus N``). With a
world of 1 the same code runs through RCCL's single-rank path (tests on a 1-GPU box).

Ordering contract for one account reached through several ingress ranks (two wallet
connections landing on different ranks under SO_REUSEPORT). Every rank issues the same
sequence of exchange steps (the step clock). A request's rows ride in the step its rank's
serving core formed when it took them from its FIFO (``ServeCore.last_timings()`` reports the
step); within a step the owner compacts the rows by sender rank, then by the sender's row order
(the sender's FIFO order, then the request's row order), scores every row of the step against
the account state the previous steps left (score-then-update, engine.go:485-488, batch
semantics: rows of one step do not see each other), and applies the rows' events in that same
(step, sender rank, row) order, each exactly once. The responses and the resulting state are
therefore those of a single engine fed, step by step, the senders' rows concatenated in rank
order (tests/test_dist.py ``test_cross_ingress_ordering_contract_same_accounts``,
tests/test_dp_gpu.py ``test_exchange_world1_same_accounts_in_one_step_follow_fifo_order``).
Which step a request lands in depends on arrival time, exactly as the order of two
independent connections to one server does.
"""
from __future__ import annotations

import copy
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..layouts import REQREC
from ..native import hipk
from ..ops import kernels as K
from ..parallel.exchange import FEAT_BYTES, RES_BYTES, build_chunks, gather_results, result_width
from .scorer import GpuScorer

REQ = REQREC.itemsize

# Per-rank stream -> hardware-queue map of the exchange pipeline. HIP multiplexes a process's
# streams onto GPU_MAX_HW_QUEUES hardware queues (4 on the boxes, HIP's default); a fifth
# stream would share a queue with one of these and serialise behind it. The two RCCL
# all-to-alls (IGP_XCHG_ROWS=rccl) therefore run on the copy and model streams:
#   default  allocations, cold reads (GetFeatures readouts order on the state stream)
#   copy     H2D chunks + header, row all-to-all (communicator 0), compaction, dedup insert
#   state    K1 feature assembly + state update (owns the HBM feature store)
#   model    trees / head / K5, result scatter, result all-to-all (communicator 1), D2H
# Communicators per rank: the two exchange RcclComms (rows, results; their kernels run on the
# streams above, RCCL opens no stream of its own for them) and the gloo control plane (CPU).
# With the node-shared rows and results regions (IGP_XCHG_ROWS=shm, IGP_XCHG_RESULTS=d2h: the
# serving default) a rank has no RCCL communicator at all: copy = compact from the rows region
# + dedup insert, state, model + scatter into the results region - three streams + default.
# No torch NCCL process group exists on the serving path. (Round 5's A/B mode with two
# CU-masked streams of their own for the collectives was removed: it exceeded the queue budget.)
HW_QUEUES = 4
EXCHANGE_COMMUNICATORS = 2


def rows_mode() -> str:
    """How rows reach their owners (IGP_XCHG_ROWS): ``shm`` (default) through the node-shared
    rows region - every sender packs its per-owner chunks into page-locked /dev/shm and each
    owner's copy stage compacts its chunks straight from host memory (the rows cross PCIe once,
    host -> owner, as in the single-GPU pipeline; no collective on the hot path); ``rccl``: an
    H2D copy to the ingress GPU, then the RCCL row all-to-all over xGMI. The requests arrive in
    host memory either way, so the all-to-all adds a hop: at world 1 the exchange path measured
    94 M scores/s against 129 M for the plain pipeline on the same box (profiles/r6/a)."""
    m = os.environ.get("IGP_XCHG_ROWS", "shm")
    if m not in ("shm", "rccl"):
        raise ValueError("IGP_XCHG_ROWS must be shm or rccl")
    return m


def map_results_region(name: str, depth: int, world: int, cmax: int, rows: bool = False) -> dict:
    """The node-shared result region of the per-GPU D2H result path (IGP_XCHG_RESULTS=d2h):
    [depth][owner][sender][cmax][W] result chunks + one 64-B flag line per (slot, owner); with
    ``rows`` also the rows region (IGP_XCHG_ROWS=shm): [depth][sender][owner][cmax + 1] ReqRec
    chunks + one 64-B flag line per (slot, sender).
    Every rank opens the same name (O_CREAT, same size: no creation order needed); the group's
    creator unlinks it once every rank mapped it. Page-locked, so the owners' device copies into
    it are asynchronous DMA (and nodes of the captured model graphs)."""
    import ctypes
    import mmap
    W = RES_BYTES + FEAT_BYTES
    owner_stride = world * cmax * W
    slot_stride = world * owner_stride
    data = depth * slot_stride
    sender_stride = world * (cmax + 1) * REQ
    rows_slot_stride = world * sender_stride
    rows_at = data + depth * world * 64
    rows_flags_at = rows_at + depth * rows_slot_stride
    size = rows_flags_at + depth * world * 64 if rows else data + depth * world * 64
    path = "/dev/shm/" + name.lstrip("/")
    fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o600)
    try:
        if os.fstat(fd).st_size < size:
            os.ftruncate(fd, size)
        mm = mmap.mmap(fd, size)
    finally:
        os.close(fd)
    base = ctypes.addressof(ctypes.c_char.from_buffer(mm))
    hipk().host_register(base, size)
    out = dict(name=name, path=path, mm=mm, base=base, size=size, owner_stride=owner_stride, slot_stride=slot_stride,
               flags=base + data, depth=depth, world=world, cmax=cmax, rows=None)
    if rows:
        out["rows"] = dict(base=base + rows_at, slot_stride=rows_slot_stride, sender_stride=sender_stride,
                           flags=base + rows_flags_at, offset=rows_at)
    return out


def stream_roles() -> dict:
    """role -> the stream that carries it."""
    return dict(default="default", h2d="copy", rows_a2a="copy", compact="copy", features="state",
                model="model", results_a2a="model", d2h="model")


@dataclass
class XPending:
    slot: int
    C: int
    n: int
    gather: Optional[np.ndarray]
    want_features: bool
    t_submit: float


class DpGpuScorer(GpuScorer):
    """GpuScorer whose batches arrive through the exchange. ``cbuckets``: chunk capacities
    (rows per owner per sender); the scorer graphs run ``senders * C`` rows."""

    fenc_to_host = False  # the result all-to-all carries the device feature images to the senders

    def __init__(self, cfg, store, comms: Sequence, world: int, rank: int, senders: int,
                 cbuckets: Sequence[int], plan=None, model: str = "plan", device=None, pipeline_depth: int = 3,
                 update_features: bool = True, results_shm: Optional[str] = None):
        """``results_shm``: name of a node-shared /dev/shm region for the per-GPU D2H result
        path (every rank opens the same name; the creator of the group unlinks it once all
        mapped it): owners copy their results for every sender into it instead of the result
        all-to-all (IGP_XCHG_RESULTS=d2h, :meth:`_attach_results_shm`)."""
        self.world, self.senders = int(world), int(senders)
        if not 1 <= self.senders <= self.world:
            raise ValueError("senders must be in [1, world]")
        if self.world > hipk().XCHG_MAX_WORLD:
            raise ValueError("world too large for the exchange kernels")
        self.cbuckets = sorted(set(int(c) for c in cbuckets))
        cfg = copy.deepcopy(cfg)
        cfg.gpu.buckets = [self.senders * c for c in self.cbuckets]
        super().__init__(cfg, store, plan=plan, model=model, device=device, pipeline_depth=pipeline_depth,
                         update_features=update_features, use_graphs=True, owner_filter=False, rank=rank)
        self.comms = list(comms or [])
        cmax, dev = self.cbuckets[-1], self.device
        self.xbytes_max = self.world * (cmax + 1) * REQ
        self.rbytes_max = self.world * cmax * (RES_BYTES + FEAT_BYTES)
        for sb in self.slots:
            sb.xsend = torch.zeros(self.xbytes_max, dtype=torch.uint8, device=dev)
            sb.xrecv = torch.zeros(self.xbytes_max, dtype=torch.uint8, device=dev)
            sb.route = torch.zeros(self.bmax + 1, dtype=torch.int32, device=dev)
            sb.rsend = torch.zeros(self.rbytes_max, dtype=torch.uint8, device=dev)
            sb.rrecv = torch.zeros(self.rbytes_max, dtype=torch.uint8, device=dev)
        self.host_x = [torch.zeros(self.xbytes_max, dtype=torch.uint8).pin_memory() for _ in range(self.depth)]
        self.host_x_np = [t.numpy() for t in self.host_x]
        self.host_rr = [torch.zeros(self.rbytes_max, dtype=torch.uint8).pin_memory() for _ in range(self.depth)]
        # the row all-to-all on the copy stream, the result all-to-all + D2H on the model stream:
        # two cross-stream hops per batch, as in the single-GPU pipeline
        self.xstream, self.ystream = self.cstream, self.mstream
        self.xgraphs = {}
        self.xdriver = None
        self._watch = None
        self.rshm = None
        if results_shm:
            self.rshm = (results_shm if isinstance(results_shm, dict)
                         else map_results_region(results_shm, self.depth, self.world, self.cbuckets[-1]))
            if (self.rshm["depth"], self.rshm["world"], self.rshm["cmax"]) != (self.depth, self.world, self.cbuckets[-1]):
                raise ValueError("results region shape does not match the scorer")
        # rows through the node-shared rows region (IGP_XCHG_ROWS=shm): no communicator at all
        self.rows_shm = self.rshm is not None and self.rshm.get("rows") is not None
        if self.rows_shm:
            r = self.rshm["rows"]
            # this sender's block of each slot: submit_rows packs its chunks there directly
            self.host_x_np = [np.frombuffer(self.rshm["mm"], np.uint8, r["sender_stride"],
                                            r["offset"] + s * r["slot_stride"] + self.rank * r["sender_stride"])
                              for s in range(self.depth)]
        elif len(self.comms) != 2:
            raise ValueError("the exchange needs two RCCL communicators (rows, results)")

    def stream_map(self) -> dict:
        """role -> HIP stream handle actually used by this rank (see :func:`stream_roles`)."""
        st = dict(default=torch.cuda.default_stream(self.device), copy=self.cstream, state=self.stream,
                  model=self.mstream, xs=self.xstream, ys=self.ystream)
        h = {k: v.cuda_stream for k, v in st.items()}
        roles = dict(default="default", h2d="copy", rows_a2a="xs", compact="copy", features="state",
                     model="model", results_a2a="ys", d2h="ys")
        return {r: h[s] for r, s in roles.items()}

    # ------------------------------------------------------------------ graph bodies
    @staticmethod
    def _direct_default() -> bool:
        # the state / model stages are recorded launches (see capture): no CU masks (same-box
        # world-1 A/B, 3 runs each: none 77.9 / 78.1 / 71.7 vs half 68.3 / 69.0 / 74.4 M
        # scores/s, profiles/r5/xchg)
        return True

    def cap(self, C: int) -> int:
        return self.senders * C

    def _send_body(self, slot: int, C: int) -> None:
        sb, nb = self.slots[slot], self.world * (C + 1) * REQ
        K.memcpy_async(sb.xsend, self.host_x[slot], nb)
        # the receive buffer's chunk counts are zeroed ahead of the all-to-all: an aborted
        # collective (failover) then leaves zero rows to compact instead of a stale chunk; the
        # same kernel brings the batch header from the pinned slab (no 16-byte copy job)
        hipk().exchange_clear(sb.xrecv.data_ptr(), self.world, C, torch.cuda.current_stream().cuda_stream,
                              self.host_slab[slot].data_ptr(), sb.dev_slab.data_ptr())

    def _post_body(self, slot: int, C: int) -> None:
        sb, b = self.slots[slot], self.cap(C)
        hipk().exchange_compact(sb.xrecv.data_ptr(), sb.req.data_ptr(), sb.dev_slab.data_ptr(), sb.route.data_ptr(),
                                self.world, C, b, torch.cuda.current_stream().cuda_stream)
        if self.update_features:
            K.dedup_insert(self.store, self.cfg_dev, sb.req, b, sb.hdr)

    def _rows_post_body(self, slot: int, C: int) -> None:
        """Rows-region copy stage, one kernel: the dedup insert reads this owner's chunk of every
        sender's block straight from page-locked host memory, compacts the rows (with their route
        and the batch header) into the slot's device rows and registers them - as the
        single-GPU pipeline's insert reads its pinned slab."""
        sb, b, r = self.slots[slot], self.cap(C), self.rshm["rows"]
        first = r["base"] + slot * r["slot_stride"] + self.rank * (C + 1) * REQ
        if self.update_features:
            K.dedup_insert(self.store, self.cfg_dev, sb.req, b, sb.hdr,
                           xsrc=dict(recv=first, pstride=r["sender_stride"] // REQ, N=self.world, C=C,
                                     route=sb.route, hdr=self.host_slab[slot].data_ptr()))
            return
        hipk().exchange_compact(first, sb.req.data_ptr(), sb.dev_slab.data_ptr(), sb.route.data_ptr(),
                                self.world, C, b, torch.cuda.current_stream().cuda_stream,
                                r["sender_stride"] // REQ, self.host_slab[slot].data_ptr())

    def _routed(self, slot: int, C: int, with_features: bool) -> Optional[dict]:
        """Rows-region exchange with feature images: K5 writes each result and K1 each image
        straight into the row's sender chunk of the results region (no scatter kernel, no device
        copy of the images): dict(base, route, C, stride) of the result rows, else None."""
        if not (self.rows_shm and with_features):
            return None
        return dict(base=self._region(slot), route=self.slots[slot].route, C=C, stride=C * (RES_BYTES + FEAT_BYTES))

    def _fenc_route(self, slot: int, bucket: int):
        if not self.rows_shm:
            return None
        C = bucket // self.senders
        r = self._routed(slot, C, True)
        return dict(r, base=r["base"] + C * RES_BYTES)

    def _xmodel_body(self, slot: int, C: int, with_features: bool, send: int = 0) -> None:
        """The model, K5, and the scatter of each row's result (+ feature image) into its
        sender's chunk of ``send`` (default: the slot's device buffer for the result
        all-to-all). Rows-region exchange with features: K5 writes the rows in place (routed)."""
        sb, b = self.slots[slot], self.cap(C)
        routed = self._routed(slot, C, with_features)
        if routed is not None:
            if sb.model is not None and sb.model.fuses_ensemble(b):
                ens = K.ensemble_args(sb.hdr, self.cfg_dev, sb.feat, sb.X, sb.model.step_out[-1], sb.res, b,
                                      self.metrics, host_route=routed)
                sb.model.run(sb.X, b, m_ptr=sb.n_ptr, ens=ens)
            else:
                ml = sb.model.run(sb.X, b, m_ptr=sb.n_ptr) if sb.model is not None else None
                K.ensemble(sb.hdr, self.cfg_dev, sb.feat, sb.X, ml, sb.res, b, self.metrics, host_route=routed)
            return
        if sb.model is not None and sb.model.fuses_ensemble(b):
            ens = K.ensemble_args(sb.hdr, self.cfg_dev, sb.feat, sb.X, sb.model.step_out[-1], sb.res, b, self.metrics)
            sb.model.run(sb.X, b, m_ptr=sb.n_ptr, ens=ens)
        else:
            ml = sb.model.run(sb.X, b, m_ptr=sb.n_ptr) if sb.model is not None else None
            K.ensemble(sb.hdr, self.cfg_dev, sb.feat, sb.X, ml, sb.res, b, self.metrics)
        hipk().exchange_scatter(sb.dev_slab.data_ptr(), sb.route.data_ptr(), sb.res.data_ptr(),
                                (sb.fenc if sb.fenc is not None else sb.feat).data_ptr() if with_features else 0,
                                send or sb.rsend.data_ptr(), C, b,
                                torch.cuda.current_stream().cuda_stream)

    # ---- collectives captured into the graphs (RCCL stream capture)
    def _a2a_rows(self, slot: int, C: int) -> None:
        sb = self.slots[slot]
        self.comms[0].all_to_all(sb.xsend.data_ptr(), sb.xrecv.data_ptr(), (C + 1) * REQ,
                                 torch.cuda.current_stream().cuda_stream)

    def _a2a_results(self, slot: int, C: int, with_features: bool) -> None:
        sb, W = self.slots[slot], result_width(with_features)
        self.comms[1].all_to_all(sb.rsend.data_ptr(), sb.rrecv.data_ptr(), C * W,
                                 torch.cuda.current_stream().cuda_stream)
        nb = self.world * C * W
        self.host_rr[slot][:nb].copy_(sb.rrecv[:nb], non_blocking=True)

    def _sendpost_body(self, slot: int, C: int) -> None:
        self._send_body(slot, C)
        self._a2a_rows(slot, C)
        self._post_body(slot, C)

    def _region(self, slot: int) -> int:
        """This owner's block of the node-shared results region for ``slot`` (0: no region)."""
        r = self.rshm
        return 0 if r is None else r["base"] + slot * r["slot_stride"] + self.rank * r["owner_stride"]

    def _model_results_body(self, slot: int, C: int, with_features: bool) -> None:
        if self.rshm is not None:
            # node-shared results: the scatter writes this owner's rows for every sender straight
            # into its block of the pinned host region (the senders read their chunk of every
            # owner's block) - no result all-to-all and no D2H copy job
            self._xmodel_body(slot, C, with_features, send=self._region(slot))
            return
        self._xmodel_body(slot, C, with_features)
        self._a2a_results(slot, C, with_features)

    def capture(self) -> None:
        """Capture send / post / state / model / model+features graphs per (C, slot), each on
        the stream it replays on, and hand them to the native exchange driver. The two all-to-alls
        and the D2H copy are captured into the send and model graphs too (three graph launches
        per batch)."""
        dev = self.device
        if self.rows_shm:
            return self._capture_rows_shm()
        # the stages are always graph replays: recorded direct launches with driver-issued
        # collectives measured 67.4 vs 100.9 M scores/s at world 1 (profiles/r2/direct3), and the
        # collective-free state stage as recorded launches 91.7 / 90.4 vs 90.7 / 104.0
        # (profiles/r2/xab); both were removed in round 5
        self.direct = False
        self.captured = True
        with torch.cuda.device(dev):
            for C in self.cbuckets:
                for slot in range(self.depth):
                    self._write_hdr(slot, 0, 0)
                    gs = []
                    if self.captured:
                        bodies = ((lambda: self._sendpost_body(slot, C), self.cstream),
                                  None,
                                  (lambda: self._state_body(slot, self.cap(C)), self.stream),
                                  (lambda: self._model_results_body(slot, C, False), self.mstream),
                                  (lambda: self._model_results_body(slot, C, True), self.mstream))
                    else:
                        bodies = ((lambda: self._send_body(slot, C), self.xstream),
                                  (lambda: self._post_body(slot, C), self.cstream),
                                  (lambda: self._state_body(slot, self.cap(C)), self.stream),
                                  (lambda: self._xmodel_body(slot, C, False, self._region(slot)), self.mstream),
                                  (lambda: self._xmodel_body(slot, C, True, self._region(slot)), self.mstream))
                    for item in bodies:
                        if item is None:
                            gs.append(None)
                            continue
                        body, s = item
                        s.wait_stream(torch.cuda.current_stream())
                        with torch.cuda.stream(s):
                            body()
                        torch.cuda.current_stream().wait_stream(s)
                        g = torch.cuda.CUDAGraph()
                        with K.graph_capture(g, s):
                            body()
                        gs.append(g)
                    self.xgraphs[(C, slot)] = tuple(gs)
            torch.cuda.synchronize(dev)
        m = hipk()
        d = m.XchgDriver(self.cstream.cuda_stream, self.stream.cuda_stream, self.mstream.cuda_stream,
                         self.xstream.cuda_stream, self.ystream.cuda_stream, self.depth, self.world,
                         self.comms[0], self.comms[1])
        for slot, sb in enumerate(self.slots):
            d.set_slot(slot, self.host_slab[slot].data_ptr(), self.host_x[slot].data_ptr(),
                       self.host_rr[slot].data_ptr(), sb.xsend.data_ptr(), sb.xrecv.data_ptr(), sb.rsend.data_ptr(),
                       sb.rrecv.data_ptr(), self.xbytes_max, self.rbytes_max)
        for (C, slot), g in self.xgraphs.items():
            d.set_graphs(C, slot, *[0 if x is None else x.raw_cuda_graph_exec() for x in g])
        # captured mode: the collective-free stages also as recorded launches (oplist.h), which
        # the driver issues instead of their graphs - the state stage always, the model stages
        # when the results go through the node-shared region (no result all-to-all inside them).
        # A two-kernel hipGraphLaunch costs ~20 us of host time and one thread issues every step
        # (profiles/NOTES.md round 5). GRU plans keep graphs (as the single-GPU pipeline).
        self.stage_ops = self.captured and not any(s.kind == "gru" for s in (self.plan.steps if self.plan else []))
        if self.stage_ops:
            with torch.cuda.device(dev):
                for (C, slot) in self.xgraphs:
                    lists = []
                    bodies = [lambda: self._state_body(slot, self.cap(C))]
                    if self.rshm is not None:
                        bodies += [lambda: self._xmodel_body(slot, C, False, self._region(slot)),
                                   lambda: self._xmodel_body(slot, C, True, self._region(slot))]
                    for body in bodies:
                        with K.Recorder() as r:
                            body()
                        lists.append(r.ops)
                    d.set_stage_ops(C, slot, *lists)
        d.set_captured(self.captured)
        if self.rshm is not None:
            r = self.rshm
            d.set_results_shm(r["base"], r["slot_stride"], r["owner_stride"], r["flags"], self.rank)
            # every wait for the other owners is bounded (a hung owner fails the step, then the
            # group fails over): the serving deadline's headroom for the late-step drain
            ms = getattr(getattr(self, "cfg", None), "gpu", None)
            ms = int(ms.batch_timeout_ms) if ms is not None and ms.batch_timeout_ms > 0 else 5000
            d.set_owner_deadline_us(2 * ms * 1000)
        if getattr(self, "state_clock", None) is not None:
            d.set_state_clock(self.state_clock)
        self.xdriver = d
        self.driver = None  # the three-graph driver of the single-GPU path is not used here

    def _capture_rows_shm(self) -> None:
        """Rows and results through the node-shared regions: the three stages as recorded
        launches (oplist.h) issued by the native driver - copy (compact from the rows region +
        dedup insert), state (K1 + update), model (trees / head / K5 + scatter into the results
        region). GRU plans keep graphs for the state / model stages (not recordable)."""
        dev = self.device
        self.direct = False
        self.captured = False
        self.stage_ops = not any(s.kind == "gru" for s in (self.plan.steps if self.plan else []))
        m = hipk()
        d = m.XchgDriver(self.cstream.cuda_stream, self.stream.cuda_stream, self.mstream.cuda_stream,
                         self.xstream.cuda_stream, self.ystream.cuda_stream, self.depth, self.world, None, None)
        for slot, sb in enumerate(self.slots):
            d.set_slot(slot, self.host_slab[slot].data_ptr(), self.host_x[slot].data_ptr(),
                       self.host_rr[slot].data_ptr(), sb.xsend.data_ptr(), sb.xrecv.data_ptr(), sb.rsend.data_ptr(),
                       sb.rrecv.data_ptr(), self.xbytes_max, self.rbytes_max)
        with torch.cuda.device(dev):
            for C in self.cbuckets:
                for slot in range(self.depth):
                    self._write_hdr(slot, 0, 0)
                    with K.Recorder() as r:
                        self._rows_post_body(slot, C)
                    d.set_copy_ops(C, slot, r.ops)
                    stages = [lambda: self._state_body(slot, self.cap(C)),
                              lambda: self._xmodel_body(slot, C, False, self._region(slot)),
                              lambda: self._xmodel_body(slot, C, True, self._region(slot))]
                    if self.stage_ops:
                        lists = []
                        for body in stages:
                            with K.Recorder() as r:
                                body()
                            lists.append(r.ops)
                        d.set_stage_ops(C, slot, *lists)
                        continue
                    gs = []
                    for body, st in zip(stages, (self.stream, self.mstream, self.mstream)):
                        st.wait_stream(torch.cuda.current_stream())
                        with torch.cuda.stream(st):
                            body()
                        torch.cuda.current_stream().wait_stream(st)
                        g = torch.cuda.CUDAGraph()
                        with K.graph_capture(g, st):
                            body()
                        gs.append(g)
                    self.xgraphs[(C, slot)] = (None, None, *gs)
                    d.set_graphs(C, slot, 0, 0, *[g.raw_cuda_graph_exec() for g in gs])
            torch.cuda.synchronize(dev)
        rs = self.rshm
        d.set_results_shm(rs["base"], rs["slot_stride"], rs["owner_stride"], rs["flags"], self.rank)
        ms = self.cfg.gpu.batch_timeout_ms if self.cfg.gpu.batch_timeout_ms > 0 else 5000
        d.set_owner_deadline_us(int(2 * ms * 1000))
        rw = rs["rows"]
        d.set_rows_shm(rw["base"], rw["slot_stride"], rw["sender_stride"], rw["flags"])
        if getattr(self, "state_clock", None) is not None:
            d.set_state_clock(self.state_clock)
        self.xdriver = d
        self.driver = None

    # ------------------------------------------------------------------ batches
    def cbucket_for(self, c: int) -> int:
        for b in self.cbuckets:
            if c <= b:
                return b
        raise ValueError(f"{c} rows for one owner exceed the largest chunk capacity {self.cbuckets[-1]}")

    def submit_chunks(self, slot: int, C: int, now: int, chunks: Optional[np.ndarray] = None,
                      want_features: bool = False, n: int = 0, gather: Optional[np.ndarray] = None,
                      prefilled: bool = False) -> XPending:
        """Launch one exchange step with prebuilt ``chunks`` (REQREC [world * (C + 1)], from
        :func:`build_chunks`; None: this rank ingests nothing this step, unless ``prefilled``:
        the chunks were built in the slot's pinned buffer already)."""
        import time
        if self.xdriver is None:
            raise RuntimeError("DpGpuScorer.capture() has not run")
        self._seq += 1
        t0 = time.perf_counter()
        nb = self.world * (C + 1) * REQ
        if prefilled:
            src = 0
        elif chunks is None:
            hx = self.host_x_np[slot][:nb].view(REQREC)
            hx["slot"][np.arange(self.world) * (C + 1)] = 0
            src = 0
        else:
            if chunks.dtype != REQREC or len(chunks) != self.world * (C + 1):
                raise ValueError("chunks must be REQREC [world * (C + 1)]")
            src = chunks.ctypes.data
        self.xdriver.submit(slot, C, self._seq, int(now), src, nb if src else 0, bool(want_features))
        self._cur = slot
        self.batches += 1
        return XPending(slot, C, n, gather, want_features, t0)

    def submit_rows(self, slot: int, req: np.ndarray, owners: np.ndarray, now: int,
                    want_features: bool = False, C: Optional[int] = None) -> XPending:
        """Ingress: route REQREC ``req`` by ``owners`` and launch."""
        from ..parallel.exchange import max_owner_count
        C = C or self.cbucket_for(max(max_owner_count(owners, self.world), 1))
        buf = self.host_x_np[slot][:self.world * (C + 1) * REQ].view(REQREC)
        _, gather, _ = build_chunks(np.asarray(req, REQREC), owners, self.world, C, out=buf)
        return self.submit_chunks(slot, C, now, None, want_features, n=len(req), gather=gather, prefilled=True)

    def wait_x(self, p: XPending, gather: bool = True, timeout_s: Optional[float] = None):
        """Block until the step's results are on the host. ``gather``: return (res, feats) of
        the ingress rows in request order; else the raw result chunks. ``timeout_s``: the
        step's deadline (event wait, csrc/kernels/watch.hip); past it the RCCL communicators
        are aborted (a peer died inside the all-to-all) and TimeoutError is raised."""
        if timeout_s is not None:
            if self._watch is None:
                self._watch = hipk().EventWatch()
            if not self._watch.wait_for(self.xdriver.done_event(p.slot), timeout_s * 1e3):
                codes = self.abort_exchange()
                raise TimeoutError(f"exchange step exceeded {timeout_s:.1f} s (RCCL async errors {codes})")
        self.xdriver.wait(p.slot)
        W = result_width(p.want_features)
        raw = self.host_rr[p.slot][:self.world * p.C * W].numpy()
        if not gather:
            return raw
        if p.gather is None or p.n == 0:
            return np.zeros((0, 2), np.uint32), None
        return gather_results(raw, p.gather, self.world, p.C, p.want_features)

    def route_overflow(self, slot: int, C: int) -> int:
        """Rows dropped by the compact kernel because they exceeded ``senders * C`` (always 0
        when every sender respects the chunk capacity; a test hook)."""
        return int(self.slots[slot].route[self.cap(C)].item())

    def done(self, p) -> bool:
        return self.xdriver.query(p.slot)

    def release_graphs(self) -> None:
        """Destroy the exchange graphs / op lists and the driver that replays them. RCCL keeps a
        reference on a communicator for every graph that captured one of its collectives, and
        ncclCommDestroy waits until those graphs are gone: destroying the communicators while the
        scorer still held its graphs is the hang of round 4 (reverted e878694)."""
        self.xdriver = None
        for gs in self.xgraphs.values():
            for g in gs:
                if hasattr(g, "reset"):  # torch.cuda.CUDAGraph: hipGraphExecDestroy + hipGraphDestroy
                    g.reset()
        self.xgraphs.clear()

    def close(self) -> None:
        """Ordered teardown (the reference drains and stops,
        services/risk/cmd/main.go:239-257): the serving core that issues steps must be stopped by
        the caller first; then the device drains, the graphs holding communicator references are
        destroyed, and both communicators are destroyed (ncclCommDestroy). Idempotent."""
        if getattr(self, "_closed", False):
            return
        self._closed = True
        import torch
        torch.cuda.synchronize(self.device)  # every issued step (collectives included) finished
        self.release_graphs()
        torch.cuda.synchronize(self.device)
        for c in self.comms:
            c.destroy()

    def abort_exchange(self) -> List[int]:
        """Failover: abort both communicators (cancels collectives still waiting on a dead peer
        so the streams drain). Returns their async error codes read before the abort."""
        codes = []
        for c in self.comms:
            try:
                codes.append(int(c.async_error()))
                c.abort()
            except Exception:  # already torn down
                codes.append(-1)
        return codes


def exchange_buckets(batch_buckets: Sequence[int]) -> List[int]:
    """Chunk capacities for the rank-0 serving front end: any micro-batch of up to the largest
    bucket fits (one sender), routed per owner into the smallest fitting chunk."""
    return sorted(set(int(b) for b in batch_buckets))

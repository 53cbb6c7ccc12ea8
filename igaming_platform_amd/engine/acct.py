"""Native account-RPC serving: PredictLTV, GetPlayerSegment and CheckBonusAbuse without Python.

``_native.AcctRouter`` (csrc/runtime/acct_core.cpp) takes the request bytes of the three RPCs
(from the native HTTP/2 server or a caller), reads the account id, routes it to the rank that
owns the account (``XXH64(id) % world``; other ranks through a node-shared /dev/shm mailbox),
micro-batches the owner's rows on its model device and writes the response bytes in C++. This
module builds the model devices of one rank (the C ABI of csrc/include/model_ops.h):

* GPU LTV: :class:`LtvNativeDevice` - per (bucket, slot) the recorded launch of the fused chain
  (csrc/kernels/mlp_fused.hip: profile gather from HBM + MLP 4x512 on MFMA + K9 epilogue), which
  reads the slot array from the pinned slab and stores the 6 outputs per row into pinned host
  memory: one kernel launch per micro-batch, no copies;
* GPU abuse: :class:`AbuseNativeDevice` - per (bucket, slot) a captured graph: H2D of the live
  rows, K1 (features.hip) writing the FeatRec rows into pinned host memory, the GRU
  (gru.hip / gru_ws.hip) over the HBM event rings, the score D2H;
* CPU: ``_native.CpuLtvDevice`` / ``_native.CpuAbuseDevice`` (csrc/runtime/acct_devices.cpp).

Python twins of the semantics (the per-call path that serves when the native path is off):
engine/ltv.py ``LtvService``, engine/abuse.py ``AbuseService``. Reference:
proto/risk/v1/risk.proto:16-20 (the RPCs), services/bonus/internal/service/bonus_engine.go:269
(every bonus award calls CheckBonusAbuse), services/risk/internal/prediction/ltv.go:113-151.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from ..native import native
from ..obs.logging import get_logger
from .abuse import SIGNAL_WEIGHTS

log = get_logger("acct")

SIGNAL_ORDER = ("BONUS_ONLY_PLAYER", "LOW_WAGER_COMPLETION", "MULTIPLE_DEVICES", "MULTIPLE_IPS", "VPN_PROXY_TOR",
                "HIGH_VELOCITY", "SHARED_DEVICE")  # csrc/runtime/acct_core.h AbuseParams.w


class LtvNativeDevice:
    """The LTV step of one GPU shard for the native core (``model_ops()``)."""

    def __init__(self, g, depth: int = 2):
        import torch
        from ..ops import kernels as K
        self.g, self.depth = g, int(depth)
        B = self.cap = g.bmax
        dev = g.device
        self.slabs = [torch.zeros(16 + 4 * B, dtype=torch.uint8).pin_memory() for _ in range(self.depth)]
        self.outs = [torch.zeros((B, 6), dtype=torch.float32).pin_memory() for _ in range(self.depth)]
        self.stream = torch.cuda.Stream(device=dev)
        # one stream per slot when the step is the recorded chain (no shared scratch): small
        # micro-batches of consecutive slots then run side by side
        self.streams = [self.stream] + ([torch.cuda.Stream(device=dev) for _ in range(self.depth - 1)]
                                        if g.chain is not None else [])
        m = K._mod()
        self.driver = m.ModelDriver([st.cuda_stream for st in self.streams], m.MODEL_LTV, self.depth, B,
                                    1 if g.plan is not None else 0,
                                    0, [t.data_ptr() for t in self.slabs], [t.data_ptr() for t in self.outs], [])
        self.graphs = []
        self._dev = None
        with torch.cuda.device(dev):
            for b in g.buckets:
                for slot in range(self.depth):
                    if g.chain is not None:
                        # [n | slots] read from the pinned slab, 6 outputs per row stored into the
                        # pinned rows (no H2D / D2H copy): one fused kernel
                        hs = self.slabs[slot]
                        kw = dict(slots=hs[16:16 + 4 * b].view(torch.int32), pf_tab=g.pf_tab, ext_tab=g.ext_tab,
                                  ltv_out=self.outs[slot], m_ptr=hs[:4].view(torch.int32))
                        with K.Recorder() as r:
                            K.mlp_chain(g.chain, b, **kw)
                        self.driver.set_ops(b, slot, r.ops)
                    else:
                        self.driver.set_graph(b, slot, self._capture(slot, b))
            torch.cuda.synchronize(dev)

    def _capture(self, slot: int, b: int) -> int:
        """Graph of the layer-kernel / formula path (no fused chain): H2D [n | slots], the model
        input gather + model + K9, D2H of the rows (own buffers: the Python path keeps its own)."""
        import torch
        from ..ops import kernels as K
        from .runner import DeviceModel
        g = self.g
        if self._dev is None:
            B = self.cap
            self._dev = dict(slab=torch.zeros(16 + 4 * B, dtype=torch.uint8, device=g.device),
                             out=torch.zeros((B, 6), dtype=torch.float32, device=g.device),
                             X=torch.zeros((B, g.w), dtype=torch.float32, device=g.device) if g.plan is not None else None,
                             model=DeviceModel(g.plan, g.device, g.buckets) if g.plan is not None else None)
        d = self._dev

        def body():
            K.memcpy_async(d["slab"], self.slabs[slot], 16 + 4 * b)
            slots, n_ptr = d["slab"][16:].view(torch.int32), d["slab"][:4].view(torch.int32)
            ml = None
            if d["model"] is not None:
                K.ltv_assemble(slots, g.pf_tab, g.ext_tab, d["X"], b, m_ptr=n_ptr)
                ml = d["model"].run(d["X"], b, m_ptr=n_ptr)[:b, 0]
            K.ltv(g.pf_tab, d["out"], model_ltv=ml, slots=slots, rows=b)
            K.memcpy_async(self.outs[slot], d["out"], b * 24)
        s = self.stream
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            body()
        torch.cuda.current_stream().wait_stream(s)
        gr = torch.cuda.CUDAGraph()
        with K.graph_capture(gr, s):
            body()
        self.graphs.append(gr)
        return gr.raw_cuda_graph_exec()

    def model_ops(self) -> int:
        return self.driver.model_ops()


class AbuseNativeDevice:
    """The CheckBonusAbuse step of one GPU shard for the native core: K1 feature rows of the
    accounts (the rule signals) and, with an abuse model, the GRU over their event rings."""

    def __init__(self, backend, plan=None, buckets=(64, 512, 4096), depth: int = 2, rank: int = 0,
                 max_batch: int = 0, priority: int = 0, cluster_kernel: bool = True):
        import torch
        from ..ops import kernels as K
        from .runner import GruModel
        self.be, self.depth = backend, int(depth)
        store, sc = backend.store, backend.scorer
        dev = store.device
        self.buckets = sorted(set(int(b) for b in buckets))
        if max_batch > 0:  # AbuseConfig.max_batch: smaller device steps (the cluster kernel's range)
            self.buckets = sorted({b for b in self.buckets if b < max_batch} | {int(max_batch)})
        B = self.cap = self.buckets[-1]
        if B > store.dmax:
            raise ValueError("abuse bucket larger than the store's batch capacity")
        self.gm = None
        if plan is not None:
            self.gm = GruModel(plan.steps, dev, getattr(plan, "precision", "fp32") != "bf16", B)
            if not self.gm.has_head:
                raise ValueError("abuse model must end in an N=1 head (probability)")
            # the bf16 cluster kernel (gru_ws.hip) needs the whole chip co-resident, which a
            # serving rank sharing it with the scoring pipeline cannot promise: off. The split
            # clusters for small batches (gru_wsx.hip, <= half the chip per launch) with
            # ``cluster_kernel`` (AbuseConfig, default on), with a second graph per step on the
            # batch-parallel kernel that the driver switches to if a cluster gives up (NaN
            # scores, model_driver.hip check_fallback). The step graphs hold no counter-reset
            # memset: with one, cluster launches stalled up to their 200 ms bound (cfg5 serving
            # 0.22 M checks/s at p99 204 ms vs 1.14 M at p99 15 ms without, profiles/r6/g, r6/i)
            for gp in self.gm.packs:
                gp.disable_ws(keep_wsx=cluster_kernel)
            if any(gp.wsx_ok for gp in self.gm.packs):
                # 128- and 256-row buckets: micro-batches up to 256 rows run on the clusters
                # (8 x 16 CUs at 256 rows)
                self.buckets = sorted(set(self.buckets) | {b for b in (128, 256) if b < B})
            self.T = plan.steps[0].seq or store.ev.shape[1]
        self.req_off = 16 + 4 * B
        nb = self.req_off + 48 * B
        self.slabs = [torch.zeros(nb, dtype=torch.uint8).pin_memory() for _ in range(self.depth)]
        self.out0 = [torch.zeros(B, dtype=torch.float32).pin_memory() for _ in range(self.depth)]
        self.out1 = [torch.zeros((B, 32), dtype=torch.int32).pin_memory() for _ in range(self.depth)]
        # the scorer's device config block, copied: a model reload replaces the scorer (and its
        # block) while these graphs keep their pointers (refresh() re-copies it)
        self.cfg_dev = sc.cfg_dev.clone()
        width = sc.width
        self.stream = torch.cuda.Stream(device=dev, priority=priority)
        # one stream per slot: a few hundred rows of 100-step GRU fill a few dozen CUs, so the
        # slots' steps run side by side (a bidirectional model shares the pack's direction
        # buffers between slots and keeps one stream)
        shared = self.gm is not None and self.gm.bidirectional
        self.streams = [self.stream] if shared else [self.stream] + [
            torch.cuda.Stream(device=dev, priority=priority) for _ in range(self.depth - 1)]
        self.bufs = [dict(slab=torch.zeros(nb, dtype=torch.uint8, device=dev),
                          X=torch.zeros((B, width), dtype=torch.float32, device=dev),
                          feat=torch.zeros((B, 32), dtype=torch.int32, device=dev),
                          out=torch.zeros(B, dtype=torch.float32, device=dev)) for _ in range(self.depth)]
        m = K._mod()
        self.driver = m.ModelDriver([st.cuda_stream for st in self.streams], m.MODEL_ABUSE, self.depth, B,
                                    1 if self.gm else 0,
                                    int(rank), [t.data_ptr() for t in self.slabs], [t.data_ptr() for t in self.out0],
                                    [t.data_ptr() for t in self.out1])
        # every step reads the store after the scoring batches issued before it (state_clock.h)
        if getattr(backend, "state_clock", None) is not None:
            self.driver.set_state_clock(backend.state_clock)
        if self.gm is not None and any(gp.wsx_ok for gp in self.gm.packs):
            # the split GRU clusters (buckets <= 256: up to half the chip per launch) run one
            # launch at a time on a stream of their own; larger buckets keep a stream per slot
            self.small_stream = torch.cuda.Stream(device=dev, priority=priority)
            self.driver.set_small_stream(self.small_stream.cuda_stream, 256)
        self.graphs = []
        wsx = self.gm is not None and any(gp.wsx_ok for gp in self.gm.packs)
        with torch.cuda.device(dev):
            for b in self.buckets:
                # rows per workgroup of the batch-parallel split GRU, per bucket: 16-row tiles for
                # the small steps of unary traffic, 32-row tiles (half the chip at 4096 rows) for
                # the full steps, so a slot's step runs beside the next slot's as in the cfg5
                # engine bench (one 16-row-tile step filled the chip: 1.7-1.8 vs 2.6 M checks/s,
                # profiles/r6/s, round-4 sweep profiles/r4/m/gru_x3_sweep.json)
                if self.gm is not None and self.gm.split and len(self.streams) > 1:
                    for gp in self.gm.packs:
                        gp.x3_rows = 32 if b >= 2048 else 16
                for slot in range(self.depth):
                    self.driver.set_graph(b, slot, self._capture(slot, b))
                    if wsx:  # the same step on the batch-parallel kernel (the fallback body)
                        for gp in self.gm.packs:
                            gp.wsx_ok = False
                        try:
                            self.driver.set_alt_graph(b, slot, self._capture(slot, b))
                        finally:
                            for gp in self.gm.packs:
                                gp.wsx_ok = True
            torch.cuda.synchronize(dev)

    def _body(self, slot: int, b: int) -> None:
        import torch
        from ..ops import kernels as K
        d, h, ro = self.bufs[slot], self.slabs[slot], self.req_off
        K.memcpy_async(d["slab"], h, 16 + 4 * b)                       # header + slots
        K.memcpy_async(d["slab"][ro:], h[ro:], 48 * b)                 # synthetic request rows
        store = self.be.store
        K.feature_assemble(store, d["slab"][:16].view(torch.int64), self.cfg_dev, d["slab"][ro:ro + 48 * b], d["X"],
                           d["feat"], b, fenc=self.out1[slot])
        if self.gm is not None:
            self.gm.run(b, self.T, d["out"], store=store, slots=d["slab"][16:16 + 4 * b].view(torch.int32),
                        m_ptr=d["slab"][:4].view(torch.int32))
            K.memcpy_async(self.out0[slot], d["out"], 4 * b)

    def _capture(self, slot: int, b: int) -> int:
        import torch
        from ..ops import kernels as K
        h = self.slabs[slot].numpy()
        h[:4].view(np.int32)[0] = 0
        s = self.streams[slot % len(self.streams)]
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._body(slot, b)
        torch.cuda.current_stream().wait_stream(s)
        gr = torch.cuda.CUDAGraph()
        with K.graph_capture(gr, s):
            self._body(slot, b)
        self.graphs.append(gr)
        return gr.raw_cuda_graph_exec()

    def refresh(self) -> None:
        """Re-copy the scorer's config block (thresholds / table sizes) between batches."""
        import torch
        sc = self.be.scorer
        with torch.cuda.stream(self.stream):
            self.cfg_dev.copy_(sc.cfg_dev, non_blocking=True)
        self.stream.synchronize()

    def model_ops(self) -> int:
        return self.driver.model_ops()


def cpu_ltv_device(ltv, owner: int, cap: int, depth: int = 2):
    """CPU LTV device over ``ltv`` (engine/ltv.py LtvService)'s host table of ``owner``."""
    t = ltv.table
    return native().CpuLtvDevice(t.rows[owner], t.present[owner].view(np.uint8), t.ext[owner], ltv.executor,
                                 ltv.input_name, ltv.output_name, int(ltv.model_width), int(depth), int(cap))


def cpu_abuse_device(backend, model, cap: int, in_name: str = "input", out_name: str = "output", depth: int = 2):
    """CPU abuse device over a CpuBackend's C++ scorer (features + event histories)."""
    ex = native().Executor(model) if model is not None else None
    return native().CpuAbuseDevice(backend.sc, ex, in_name, out_name, int(depth), int(cap))


class NativeAcct:
    """One rank's native account-RPC router and the model devices attached to it."""

    def __init__(self, indexes, rank: int = 0, mailbox: str = "", create: bool = False):
        self.router = native().AcctRouter(list(indexes), int(rank), mailbox, bool(create))
        self.devices = []

    def attach(self, device, cfg) -> None:
        g = cfg.gpu
        timeout_us = int(g.batch_timeout_ms * 1000) if g.batch_timeout_ms > 0 else -1
        self.router.attach(device, max_wait_us=int(g.wait_us), timeout_us=timeout_us,
                           finishers=int(g.serve_finishers))
        self.devices.append(device)

    def set_abuse(self, scoring, threshold: float, link_wait_us: int = 200) -> None:
        self.router.set_abuse(int(scoring.max_devices_per_day), int(scoring.max_ips_per_day),
                              int(scoring.max_tx_per_minute), float(threshold),
                              [float(SIGNAL_WEIGHTS[k]) for k in SIGNAL_ORDER], link_wait_us=int(link_wait_us))

    def refresh(self) -> None:
        """Re-copy the devices' config blocks with no step in flight (a device's slots run on
        their own streams, so a copy on one stream could otherwise overlap a step on another)."""
        devs = [d for d in self.devices if hasattr(d, "refresh")]
        if not devs:
            return
        self.router.pause()
        try:
            for d in devs:
                d.refresh()
        finally:
            self.router.resume()

    def serves(self, rpc: int) -> bool:
        return bool(self.router.serves(int(rpc)))

    def stop(self) -> None:
        self.router.stop()


def attach_models(acct: NativeAcct, cfg, backend, ltv=None, owner: int = 0, abuse_model=None, abuse_plan=None,
                  audit: bool = False, rank: int = 0) -> None:
    """Build and attach this rank's LTV and abuse devices (``backend``: the local shard).
    ``audit``: LTV answers must reach the ltv_predictions audit log, which the Python path
    writes - the LTV device then stays off the native path."""
    depth = max(2, int(cfg.gpu.acct_depth))
    if ltv is not None and not audit:
        if backend.kind == "gpu" and ltv.gpu is not None:
            acct.attach(LtvNativeDevice(ltv.gpu[owner % len(ltv.gpu)], depth), cfg)
        elif backend.kind == "cpu":
            acct.attach(cpu_ltv_device(ltv, owner, max(cfg.gpu.buckets), depth), cfg)
    if backend.kind == "gpu":
        # (torch maps a large negative priority to the highest the device allows)
        acct.attach(AbuseNativeDevice(backend, abuse_plan, buckets=cfg.gpu.buckets, depth=depth, rank=rank,
                                      max_batch=int(cfg.abuse.max_batch),
                                      priority=-100 if cfg.abuse.high_priority else 0,
                                      cluster_kernel=bool(cfg.abuse.cluster_kernel)), cfg)
    elif backend.kind == "cpu" and hasattr(backend, "sc"):
        acct.attach(cpu_abuse_device(backend, abuse_model, max(cfg.gpu.buckets),
                                     cfg.abuse_model.input_name, cfg.abuse_model.output_name, depth), cfg)
    acct.set_abuse(cfg.scoring, cfg.abuse.threshold, cfg.abuse.link_wait_us)


def abuse_device_plan(cfg, abuse_model, device) -> Optional[object]:
    """The device plan of the abuse model (None without one)."""
    if abuse_model is None:
        return None
    from ..models.plan import compile_onnx, to_device
    return to_device(compile_onnx(abuse_model), str(device), cfg.abuse_model.precision)

"""Typed launch wrappers for the gfx950 kernels in ``_hipk``.

Every wrapper checks — on the host, before the launch — that operands live on the same GPU,
are contiguous, have the dtype the kernel reads and are at least as large as the grid will
index (a kernel fault can reset every GPU of a node, so nothing is left to the device).
All launches go to the caller's current torch stream and are hipGraph-capturable.
"""
from __future__ import annotations

import contextlib

import os

from typing import Optional

import torch

from ..features.device_store import DEDUP_STANDALONE
from ..layouts import check_layouts
from ..native import hipk

ACT = {"none": 0, "relu": 1, "sigmoid": 2, "tanh": 3}
_checked = False


def _mod():
    global _checked
    m = hipk()
    if not _checked:
        check_layouts(m)
        _checked = True
    return m


def as_device(device) -> torch.device:
    """torch.device with an explicit index ("cuda" -> "cuda:<current>")."""
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def memcpy_async(dst: torch.Tensor, src: torch.Tensor, nbytes: int) -> None:
    """Stream-ordered copy of ``nbytes`` between contiguous tensors (pinned host <-> device),
    recordable by the native driver's direct-launch mode (csrc/kernels/oplist.h)."""
    if nbytes > dst.numel() * dst.element_size() or nbytes > src.numel() * src.element_size():
        raise ValueError("memcpy_async: nbytes exceeds a tensor")
    if not (dst.is_contiguous() and src.is_contiguous()):
        raise ValueError("memcpy_async: tensors must be contiguous")
    _mod().memcpy_async(dst.data_ptr(), src.data_ptr(), int(nbytes), _stream())


@contextlib.contextmanager
def graph_capture(g, stream):
    """``torch.cuda.graph(g, stream=stream)`` with the garbage collector paused for the capture:
    a collection inside it can destroy native objects of an earlier pipeline (HIP events,
    drivers) whose HIP calls are illegal while a stream captures and abort the process."""
    import gc
    was = gc.isenabled()
    gc.disable()
    try:
        with torch.cuda.graph(g, stream=stream):
            yield
    finally:
        if was:
            gc.enable()


class Recorder:
    """``with Recorder() as r: body()`` -> ``r.ops``: the body's launches as a native op list
    (nothing runs on the device while recording)."""

    def __enter__(self):
        _mod().record_begin()
        self.ops = None
        return self

    def __exit__(self, *exc):
        self.ops = _mod().record_end()
        return False


def _need(t: Optional[torch.Tensor], name: str, dtype=None, min_numel: int = 0, device=None):
    if t is None:
        raise ValueError(f"{name}: tensor required")
    if not t.is_cuda:
        raise ValueError(f"{name}: must be a GPU tensor")
    if device is not None and t.device != device:
        raise ValueError(f"{name}: on {t.device}, expected {device}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if dtype is not None and t.dtype not in (dtype if isinstance(dtype, tuple) else (dtype,)):
        raise ValueError(f"{name}: dtype {t.dtype}, expected {dtype}")
    if t.numel() < min_numel:
        raise ValueError(f"{name}: {t.numel()} elements < {min_numel} required")
    return t.data_ptr()


def _opt(t: Optional[torch.Tensor], name: str, **kw):
    return None if t is None else _need(t, name, **kw)


def _host_or_dev(t: Optional[torch.Tensor], name: str, min_numel: int, device, dtype=torch.float32):
    """Pointer to a GPU tensor on ``device`` or to a pinned (device-mapped) host tensor that the
    kernel reads / writes through the fabric."""
    if t is None or t.is_cuda:
        return _opt(t, name, dtype=dtype, min_numel=min_numel, device=device)
    if not t.is_pinned() or not t.is_contiguous() or t.dtype != dtype or t.numel() < min_numel:
        raise ValueError(f"{name}: host tensor must be contiguous, pinned, {dtype}, >= {min_numel} elements")
    return t.data_ptr()


# --------------------------------------------------------------------------- K1
def feature_assemble(store, hdr: torch.Tensor, cfg_dev: torch.Tensor, req: torch.Tensor,
                     X: torch.Tensor, feat: torch.Tensor, n_rows: int, dedup: bool = False,
                     trace: Optional[torch.Tensor] = None, fenc: Optional[torch.Tensor] = None,
                     fenc_route: Optional[dict] = None) -> None:
    """K1. ``dedup=True``: score-then-update. :func:`dedup_insert` must have registered the
    batch first; K1 then applies each single-event account's event and opens the segments
    that :func:`update_segments` applies afterwards (dedup ring region by batch seq).
    ``fenc`` [rows, 32] int32: each row's 128-byte D2H feature image - the raw FeatRec, or the
    encoded risk.v1 FeatureVector body for rows whose ReqRec.tx_type carries FV_ENC_BIT. A pinned
    host tensor is written through the fabric (one coalesced 128-B store per row), so the image
    needs no D2H copy. ``fenc_route``: dict(base=host address, route=int32 tensor, C=, stride=):
    the images go to their senders' chunks of the exchange's node-shared results region instead
    (row i at base + p * stride + j * 128, route[i] = p * C + j)."""
    dev = store.device
    if X.dim() != 2 or X.shape[1] < 30 + store.ext_width:
        raise ValueError("X must be [rows, >= 30 + ext_width]")
    if dedup and n_rows > store.dmax:
        raise ValueError("score-then-update batch larger than the store's dedup capacity")
    d = dict(
        hdr=_need(hdr, "hdr", torch.int64, 2, dev), cfg=_need(cfg_dev, "cfg", torch.uint8, 176, dev),
        req=_need(req, "req", torch.uint8, 48 * n_rows, dev),
        ring_ts=_need(store.ring_ts, "ring_ts", torch.int32), ring_amt=_need(store.ring_amt, "ring_amt", torch.int64),
        hll=_need(store.hll, "hll", torch.uint8), rt=_need(store.rt, "rt", torch.int32),
        batch=_need(store.batch, "batch", torch.int32), ext=_need(store.ext, "ext", torch.float32),
        bl_keys=_need(store.bl_keys, "bl_keys", torch.int64), bl_exp=_need(store.bl_exp, "bl_exp", torch.int32),
        ip_keys=_need(store.ip_keys, "ip_keys", torch.int64), ip_flags=_need(store.ip_flags, "ip_flags", torch.int32),
        hll_lc=_need(store.hll_lc, "hll_lc", torch.int32, 257),
        X=_need(X, "X", torch.float32, X.shape[1] * n_rows, dev),
        feat=_need(feat, "feat", torch.int32, 32 * n_rows, dev),
        fenc=_host_or_dev(fenc, "fenc", 32 * n_rows, dev, torch.int32),
        dbuf=_need(store.dbuf, "dbuf", torch.int32) if dedup else None, dcap=int(store.dcap), dmax=int(store.dmax),
        x_stride=int(X.shape[1]), ring_size=int(store.ring_ts.shape[1]), n_rows=int(n_rows),
        # every wave's 16 trace words (features.hip): 4 waves per 16 rows
        trace=_opt(trace, "trace", dtype=torch.int64, min_numel=((int(n_rows) + 15) // 16) * 64, device=dev),
    )
    if dedup:
        d["upd"] = update_args(store, cfg_dev, req, n_rows, hdr=hdr, region=-1)
    if fenc_route is not None:
        if fenc is not None:
            raise ValueError("feature_assemble: fenc or fenc_route")
        d.update(fenc=int(fenc_route["base"]), fenc_route=_need(fenc_route["route"], "route", torch.int32, n_rows, dev),
                 fenc_c=int(fenc_route["C"]), fenc_stride=int(fenc_route["stride"]))
    _mod().feature_assemble(d, _stream())


# --------------------------------------------------------------------------- K6
def update_args(store, cfg_dev: torch.Tensor, req: torch.Tensor, n_max: int, n: int = 0,
                hdr: Optional[torch.Tensor] = None, region: int = DEDUP_STANDALONE) -> dict:
    dev = store.device
    if n_max > store.dmax:
        raise ValueError(f"feature_update: {n_max} events > store dedup capacity {store.dmax}")
    if region < 0 and hdr is None:
        raise ValueError("ring dedup region needs the batch header")
    if store.ev is not None and store.ev.shape[2] != 16:
        raise ValueError("event ring dim must be 16")
    return dict(
        cfg=_need(cfg_dev, "cfg", torch.uint8, 176, dev), hdr=_opt(hdr, "hdr", dtype=torch.int64, min_numel=2),
        n=int(n), n_max=int(n_max), req=_need(req, "req", torch.uint8, 48 * n_max, dev),
        ring_ts=_need(store.ring_ts, "ring_ts", torch.int32), ring_amt=_need(store.ring_amt, "ring_amt", torch.int64),
        hll=_need(store.hll, "hll", torch.uint8), rt=_need(store.rt, "rt", torch.int32),
        ev=_opt(store.ev, "ev", dtype=torch.int16),
        ring_size=int(store.ring_ts.shape[1]),
        ev_ring=int(store.ev.shape[1]) if store.ev is not None else 0,
        ev_dim=int(store.ev.shape[2]) if store.ev is not None else 0,
        dbuf=_need(store.dbuf, "dbuf", torch.int32), dcap=int(store.dcap), dmax=int(store.dmax), region=int(region),
        hll_lc=_need(store.hll_lc, "hll_lc", torch.int32, 257),
    )


def feature_update(store, cfg_dev: torch.Tensor, req: torch.Tensor, n_max: int, n: int = 0) -> None:
    """Standalone ordered event ingestion (event bus / history replay): ``n`` events."""
    if n > n_max:
        raise ValueError("n > n_max")
    d = update_args(store, cfg_dev, req, n_max, n=n, region=DEDUP_STANDALONE)
    _mod().feature_update(d, _stream())


def dedup_insert(store, cfg_dev: torch.Tensor, req: torch.Tensor, n_max: int, hdr: torch.Tensor,
                 src: Optional[torch.Tensor] = None, xsrc: Optional[dict] = None) -> None:
    """Scorer head: register the batch's accounts in its dedup region (before K1), with the
    per-account row lists and the multi-event account list :func:`update_segments` reads.
    ``src``: the pinned host slab [BatchHdr | ReqRec x n_max] - the kernel reads the batch from
    it and writes ``hdr`` / ``req`` itself (no H2D copy before it). ``xsrc``: the rows-region
    exchange - dict(recv=host address of sender 0's chunk for this owner, pstride=records between
    senders, N=senders, C=chunk capacity, route=int32 [n_max + 1], hdr=host address of the batch
    header): the kernel compacts the chunks into ``req`` itself (launch.h UpdateArgs)."""
    d = update_args(store, cfg_dev, req, n_max, hdr=hdr, region=-1)
    if src is not None:
        d["src"] = _host_or_dev(src, "src", 16 + 48 * n_max, store.device, torch.uint8)
    if xsrc is not None:
        d.update(xrecv=int(xsrc["recv"]), xpstride=int(xsrc["pstride"]), xn=int(xsrc["N"]), xc=int(xsrc["C"]),
                 route=_need(xsrc["route"], "route", torch.int32, n_max + 1, store.device), xhdr=int(xsrc["hdr"]))
    d["insert_only"] = 1
    _mod().feature_update(d, _stream())


def update_segments(store, cfg_dev: torch.Tensor, req: torch.Tensor, n_max: int, hdr: torch.Tensor) -> None:
    """Scorer tail (after K1): ordered apply of the multi-event accounts (insert before K1,
    single-event accounts in K1), then clear the dedup region of batch seq + DEDUP_AHEAD (launch.h)."""
    d = update_args(store, cfg_dev, req, n_max, hdr=hdr, region=-1)
    d["segments_only"] = 1
    _mod().feature_update(d, _stream())


# --------------------------------------------------------------------------- K2
def _tree_dict(tp, X: torch.Tensor, out: Optional[torch.Tensor], n_rows: int, partial, groups: int,
               no_finish: bool, trace, ens) -> dict:
    dev = X.device
    if tp.k not in (1, 2, 4, 8, 16, 32, 64):
        raise ValueError(f"tree kernel built for K in 1,2,4,8,16,32,64; got {tp.k}")
    if X.shape[1] <= tp.max_feature:
        raise ValueError("X narrower than the ensemble's largest feature id")
    if groups > 1 and (partial is None or partial.numel() < groups * n_rows * tp.k):
        raise ValueError("grouped tree launch needs a [groups, rows, K] partial buffer")
    if no_finish and groups <= 1:
        raise ValueError("no_finish needs a grouped launch")
    if out is None and not no_finish:
        raise ValueError("tree_ensemble: out required")
    if ens is not None and (groups <= 1 or no_finish or ens.get("ml") != out.data_ptr()):
        raise ValueError("tree_ensemble: ensemble fusion needs a grouped launch whose output is the ml input")
    d = dict(
        X=_need(X, "X", torch.float32, X.shape[1] * n_rows), nodes=_need(tp.nodes, "nodes", torch.float32, device=dev),
        leaves=_need(tp.leaves, "leaves", torch.float32, device=dev), base=_opt(tp.base, "base", dtype=torch.float32),
        out=_opt(out, "out", dtype=torch.float32, min_numel=tp.n_out * n_rows), x_stride=int(X.shape[1]),
        n_rows=int(n_rows), n_trees=tp.n_trees, depth=tp.depth, k=tp.k, n_out=tp.n_out, post=tp.post,
        average=tp.average, binary_class=tp.binary_class, all_positive=tp.all_positive,
        groups=int(groups), partial=_opt(partial, "partial", dtype=torch.float32), no_finish=int(no_finish),
        all_leq=int(tp.all_leq), trace=_opt(trace, "trace", dtype=torch.int64, min_numel=64), ens=ens,
    )
    if tp.nodes.numel() < tp.n_trees * ((1 << tp.depth) - 1) * 2:
        raise ValueError("node table smaller than n_trees * (2^depth - 1)")
    if tp.leaves.numel() < tp.n_trees * (1 << tp.depth) * tp.k:
        raise ValueError("leaf table smaller than n_trees * 2^depth * K")
    if tp.n_trees * (1 << tp.depth) * tp.k >= 2 ** 31:
        raise ValueError("leaf table too large for the kernel's 32-bit offsets")
    return d


def tree_ensemble(tp, X: torch.Tensor, out: Optional[torch.Tensor], n_rows: int,
                  partial: Optional[torch.Tensor] = None, groups: int = 1, no_finish: bool = False,
                  trace: Optional[torch.Tensor] = None, ens: Optional[dict] = None) -> None:
    """``tp``: models.plan.TreeStep with device tensors. ``trace``: int64 [64] phase timestamps
    (wall_clock64) of 8 sample workgroups, for tools/tree_bench.py. ``ens``
    (:func:`ensemble_args` with ``ml`` = ``out``, grouped launches only): the scorer's K5
    ensemble runs in the finish kernel's epilogue."""
    _mod().tree_ensemble(_tree_dict(tp, X, out, n_rows, partial, groups, no_finish, trace, ens), _stream())


def tree_head_ok(tp, hs, groups: int) -> bool:
    """Whether :func:`tree_head` runs this tree -> head pair in one launch (K = 32 leaf vectors
    without a post transform, grouped, f32 head with k_pad 32)."""
    return (tp.layout != "sparse" and tp.k == 32 and 1 < groups <= 16 and tp.post == 0 and tp.binary_class < 0
            and hs.k == 32 and hs.w1.dtype == torch.float32 and hs.w1.shape[1] == 32 and 0 < hs.n1 <= 512
            and ACT.get(hs.act1, -1) in (0, 1, 2, 3))


def tree_head(tp, hs, X: torch.Tensor, Y: torch.Tensor, n_rows: int, partial: torch.Tensor, groups: int,
              tile_cnt: torch.Tensor, m_ptr: Optional[torch.Tensor] = None, ens: Optional[dict] = None) -> None:
    """K2 -> K3 -> K5 of the stacked model in ONE launch (trees.hip tree_head_kernel): the
    grouped tree ensemble's last-arriving block per 64-row tile reduces the tile's group
    partials and runs the f32 head and the fused ensemble on it. ``tile_cnt``: int32 zeros,
    one per 64-row tile (the kernel leaves them zero)."""
    if not tree_head_ok(tp, hs, groups):
        raise ValueError("tree_head: unsupported tree / head shapes")
    if tile_cnt.dtype != torch.int32 or tile_cnt.numel() < -(-n_rows // 64) or tile_cnt.device != X.device:
        raise ValueError("tree_head: tile counters")
    dt = _tree_dict(tp, X, None, n_rows, partial, groups, True, None, None)
    dt["tile_cnt"] = tile_cnt.data_ptr()
    dh = _head_dict(hs, None, Y, n_rows, m_ptr, (partial, groups, tp), None, ens)
    _mod().tree_head(dt, dh, _stream())


def tree_sparse(tp, X: torch.Tensor, out: torch.Tensor, n_rows: int, partial: Optional[torch.Tensor] = None,
                groups: int = 1) -> None:
    """K2b: ``tp`` a sparse-layout TreeStep with device tensors (pointer layout validated by
    :func:`models.plan.validate_sparse` at upload). ``partial``: [groups, rows, K] scratch."""
    dev = X.device
    if tp.layout != "sparse":
        raise ValueError("tree_sparse needs a sparse-layout TreeStep")
    if X.shape[1] <= tp.max_feature:
        raise ValueError("X narrower than the ensemble's largest feature id")
    if groups > 1 and (partial is None or partial.numel() < groups * n_rows * tp.k):
        raise ValueError("grouped tree launch needs a [groups, rows, K] partial buffer")
    n_nodes = tp.nodes.shape[0]
    d = dict(X=_need(X, "X", torch.float32, X.shape[1] * n_rows, device=dev),
             nodes=_need(tp.nodes, "nodes", torch.int32, 4 * n_nodes, device=dev),
             roots=_need(tp.roots, "roots", torch.int32, tp.n_trees, device=dev),
             leaf_w=_need(tp.leaf_w, "leaf_w", torch.float32, device=dev),
             leaf_has=_need(tp.leaf_has, "leaf_has", torch.uint8, tp.leaf_w.numel(), device=dev),
             base=_opt(tp.base, "base", dtype=torch.float32, min_numel=1 if tp.binary_class >= 0 else tp.k),
             out=_need(out, "out", torch.float32, tp.n_out * n_rows, device=dev), x_stride=int(X.shape[1]),
             n_rows=int(n_rows), n_trees=tp.n_trees, depth=tp.depth, k=tp.k, n_out=tp.n_out, post=tp.post,
             aggregate=tp.aggregate, binary_class=tp.binary_class, all_positive=tp.all_positive,
             feat_w=int(max(tp.max_feature, 0) + 1), groups=int(groups),
             partial=_opt(partial, "partial", dtype=torch.float32))
    if out.dim() == 2 and out.shape[1] != tp.n_out:
        raise ValueError("out must have n_out columns")
    _mod().tree_sparse(d, _stream())


# --------------------------------------------------------------------------- K3
def dense(X: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor], Y: torch.Tensor,
          M: int, N: int, K: int, act: str = "none", m_ptr: Optional[torch.Tensor] = None) -> None:
    """Y[:M,:N] = act(X[:M,:K] W^T + b); W bf16 [N_pad(128), K_pad(64)] from models.plan."""
    dev = X.device
    if X.dtype not in (torch.float32, torch.bfloat16) or Y.dtype not in (torch.float32, torch.bfloat16):
        raise ValueError("dense: X and Y must be float32 or bfloat16")
    if W.dtype not in (torch.bfloat16, torch.float32) or W.dim() != 2:
        raise ValueError("dense: W must be 2-D bfloat16 or float32")
    if N == 1:
        if W.shape[1] < K:
            raise ValueError("dense: W narrower than K")
    elif W.shape[0] % 128 or W.shape[1] % 64 or W.shape[0] < N or W.shape[1] < K:
        raise ValueError("dense: W must be padded to [N_pad % 128 == 0, K_pad % 64 == 0]")
    if X.shape[1] < K or Y.shape[1] < N or X.shape[0] < M or Y.shape[0] < M:
        raise ValueError("dense: operand shapes smaller than M/N/K")
    if bias is not None and bias.numel() < N:
        raise ValueError("dense: bias shorter than N")
    d = dict(X=_need(X, "X", device=dev), W=_need(W, "W", device=dev), bias=_opt(bias, "bias", dtype=torch.float32),
             Y=_need(Y, "Y", device=dev), m_ptr=_opt(m_ptr, "m_ptr", dtype=torch.int32), M=int(M), N=int(N),
             K=int(K), ldx=int(X.shape[1]), ldy=int(Y.shape[1]), ldw=int(W.shape[1]),
             x_bf16=int(X.dtype == torch.bfloat16), y_bf16=int(Y.dtype == torch.bfloat16), act=ACT[act],
             w_f32=int(W.dtype == torch.float32))
    if N == 1:
        _mod().gemv(d, _stream())
    else:
        _mod().gemm(d, _stream())


JOIN_OPS = {"add": 0, "concat": 1}


def join(op: str, A: torch.Tensor, B: torch.Tensor, Y: torch.Tensor, M: int, na: int, nb: int,
         m_ptr: Optional[torch.Tensor] = None) -> None:
    """DAG join (join.hip): ``add`` Y[:M, :na] = A + B; ``concat`` Y[:M, :na+nb] = [A | B]."""
    dev = Y.device
    for t, name in ((A, "A"), (B, "B"), (Y, "Y")):
        if t.dim() != 2 or t.dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"join: {name} must be 2-D float32 or bfloat16")
    width = na if op == "add" else na + nb
    if op not in JOIN_OPS or (op == "add" and na != nb):
        raise ValueError("join: op add (equal widths) or concat")
    if A.shape[1] < na or B.shape[1] < nb or Y.shape[1] < width or min(A.shape[0], B.shape[0], Y.shape[0]) < M:
        raise ValueError("join: operand shapes smaller than M / widths")
    d = dict(A=_need(A, "A", device=dev), B=_need(B, "B", device=dev), Y=_need(Y, "Y", device=dev),
             m_ptr=_opt(m_ptr, "m_ptr", dtype=torch.int32), M=int(M), na=int(na), nb=int(nb), op=JOIN_OPS[op],
             lda=int(A.shape[1]), ldb=int(B.shape[1]), ldy=int(Y.shape[1]), a_bf16=int(A.dtype == torch.bfloat16),
             b_bf16=int(B.dtype == torch.bfloat16), y_bf16=int(Y.dtype == torch.bfloat16))
    _mod().join(d, _stream())


def mlp_head(hs, X: Optional[torch.Tensor], Y: torch.Tensor, M: int, m_ptr: Optional[torch.Tensor] = None,
             tree_partial=None, trace: Optional[torch.Tensor] = None, ens: Optional[dict] = None) -> None:
    """``hs``: models.plan.HeadStep. Y[:M, 0] = act2(act1(X W1^T + b1) . w2 + b2).
    ``tree_partial=(slab, groups, tree_step)``: X is the preceding tree ensemble's unreduced
    group partials [groups, M, K]; the head reduces them while staging (no finisher launch).
    ``ens``: :func:`ensemble_args` of the scorer's K5 on this Y (model column 0): the head's
    epilogue runs the ensemble of its rows, replacing the standalone ensemble launch."""
    _mod().mlp_head(_head_dict(hs, X, Y, M, m_ptr, tree_partial, trace, ens), _stream())


def _head_dict(hs, X, Y, M, m_ptr, tree_partial, trace, ens) -> dict:
    if tree_partial is not None:
        slab, groups, ts = tree_partial
        if ts.k != hs.k or slab.numel() < groups * M * hs.k or ts.post != 0 or ts.binary_class >= 0:
            raise ValueError("mlp_head: tree partial slab does not match the head")
        X = slab
    dev = X.device
    if X.dtype not in (torch.float32, torch.bfloat16):
        raise ValueError("mlp_head: X must be float32 or bfloat16")
    if tree_partial is None and (X.shape[1] < hs.k or X.shape[0] < M):
        raise ValueError("mlp_head: operand shapes")
    if Y.shape[0] < M or Y.dtype != torch.float32:
        raise ValueError("mlp_head: output shape/dtype")
    if hs.w1.shape[0] < -(-hs.n1 // 64) * 64 or hs.w1.shape[1] % 32 or hs.w1.shape[1] < hs.k:
        raise ValueError("mlp_head: W1 padding")
    w1_f32 = hs.w1.dtype == torch.float32
    if w1_f32 and hs.w1.shape[1] * 4 * -(-hs.n1 // 64) * 64 > (1 << 30):
        raise ValueError("mlp_head: f32 W1 too large")
    d = dict(X=_need(X, "X", device=dev), W1=_need(hs.w1, "W1", (torch.bfloat16, torch.float32), device=dev),
             w1_f32=int(w1_f32),
             b1=_opt(hs.b1, "b1", dtype=torch.float32, min_numel=hs.n1),
             w2=_need(hs.w2, "w2", torch.float32, hs.n1, dev), b2=float(hs.b2),
             Y=_need(Y, "Y", torch.float32, M, dev), m_ptr=_opt(m_ptr, "m_ptr", dtype=torch.int32),
             M=int(M), K=int(hs.k), N1=int(hs.n1), k_pad=int(hs.w1.shape[1]), ldx=int(X.shape[1]) if X.dim() == 2 else hs.k,
             ldy=int(Y.shape[1]), x_bf16=int(X.dtype == torch.bfloat16), act1=ACT[hs.act1], act2=ACT[hs.act2])
    if tree_partial is not None:
        slab, groups, ts = tree_partial
        d.update(partial=_need(slab, "partial", torch.float32, groups * M * hs.k, dev), ldx=hs.k,
                 pbase=_opt(ts.base, "pbase", dtype=torch.float32, min_numel=hs.k), groups=int(groups),
                 p_average=int(ts.average), p_ntrees=int(ts.n_trees))
    if trace is not None:
        d["trace"] = _need(trace, "trace", torch.int64, 64, dev)
    if ens is not None:
        if ens["n_rows"] > M:
            raise ValueError("mlp_head: fused ensemble covers more rows than the head")
        d["ens"] = ens
    return d


# --------------------------------------------------------------------------- K5 / K10
def ensemble_args(hdr, cfg_dev, feat, X, ml: Optional[torch.Tensor], out, n_rows: int,
                  metrics: Optional[torch.Tensor] = None, host_out: Optional[torch.Tensor] = None,
                  host_route: Optional[dict] = None) -> dict:
    """``host_out``: pinned host int32 [>= n_rows, 2] rows the kernel also writes (the D2H
    copy of the results is then not needed). ``host_route``: dict(base=host address,
    route=int32 tensor, C=, stride=): the live rows go to their senders' chunks of the exchange's
    results region instead (row i at base + p * stride + j * 8, route[i] = p * C + j)."""
    dev = feat.device
    d = dict(hdr=_need(hdr, "hdr", torch.int64, 2, dev), cfg=_need(cfg_dev, "cfg", torch.uint8, 176, dev),
             feat=_need(feat, "feat", torch.int32, 32 * n_rows, dev),
             X=_need(X, "X", torch.float32, X.shape[1] * n_rows, dev), x_stride=int(X.shape[1]),
             ml=_opt(ml, "ml", dtype=torch.float32), out=_need(out, "out", torch.int32, 2 * n_rows, dev),
             metrics=_opt(metrics, "metrics", dtype=torch.int64, min_numel=128), n_rows=int(n_rows))
    if ml is not None and ml.numel() < n_rows:
        raise ValueError("ensemble: model output shorter than the batch")
    if host_out is not None:
        if host_out.is_cuda or not host_out.is_pinned() or host_out.dtype != torch.int32 or \
                not host_out.is_contiguous() or host_out.numel() < 2 * n_rows:
            raise ValueError("ensemble: host_out must be pinned contiguous int32 [>= n_rows, 2]")
        d["host_out"] = host_out.data_ptr()
    if host_route is not None:
        if host_out is not None:
            raise ValueError("ensemble: host_out or host_route")
        d.update(host_out=int(host_route["base"]), route=_need(host_route["route"], "route", torch.int32, n_rows, dev),
                 route_c=int(host_route["C"]), route_stride=int(host_route["stride"]))
    return d


def ensemble(hdr, cfg_dev, feat, X, ml: Optional[torch.Tensor], out, n_rows: int,
             metrics: Optional[torch.Tensor] = None, host_out: Optional[torch.Tensor] = None,
             host_route: Optional[dict] = None) -> None:
    _mod().ensemble(ensemble_args(hdr, cfg_dev, feat, X, ml, out, n_rows, metrics, host_out, host_route), _stream())


# --------------------------------------------------------------------------- K9
def ltv(pf: torch.Tensor, out: torch.Tensor, model_ltv: Optional[torch.Tensor] = None,
        slots: Optional[torch.Tensor] = None, rows: Optional[int] = None) -> None:
    """K9. ``pf`` is [B, 25] rows, or (with ``slots``) the [C, 25] device player table."""
    if pf.dim() != 2 or pf.shape[1] != 25:
        raise ValueError("ltv: player features must be [B, 25]")
    B = pf.shape[0] if slots is None else int(rows)
    if slots is not None:
        _need(slots, "slots", torch.int32, B)
    d = dict(pf=_need(pf, "pf", torch.float32), out=_need(out, "out", torch.float32, 6 * B),
             ltv_model=_opt(model_ltv, "ltv_model", dtype=torch.float32, min_numel=B), B=int(B),
             slots=None if slots is None else slots.data_ptr())
    _mod().ltv(d, _stream())


def ltv_assemble(slots: torch.Tensor, pf_tab: torch.Tensor, ext_tab: Optional[torch.Tensor], X: torch.Tensor,
                 n_rows: int, m_ptr: Optional[torch.Tensor] = None) -> None:
    """LTV model input rows gathered from the device-resident player tables."""
    dev = X.device
    if X.dim() != 2 or pf_tab.dim() != 2 or pf_tab.shape[1] != 25 or X.shape[0] < n_rows:
        raise ValueError("ltv_assemble: shapes")
    ext_w = 0 if ext_tab is None else int(ext_tab.shape[1])
    if ext_tab is not None and ext_tab.shape[0] != pf_tab.shape[0]:
        raise ValueError("ltv_assemble: table row counts differ")
    if X.shape[1] < 25:
        raise ValueError("ltv_assemble: model input narrower than the profile")
    d = dict(slots=_need(slots, "slots", torch.int32, n_rows, dev), pf_tab=_need(pf_tab, "pf_tab", torch.float32, device=dev),
             ext_tab=_opt(ext_tab, "ext_tab", dtype=torch.float32, device=dev), ext_w=ext_w,
             X=_need(X, "X", torch.float32, X.shape[1] * n_rows, dev), x_w=int(X.shape[1]),
             m_ptr=_opt(m_ptr, "m_ptr", dtype=torch.int32, device=dev), n_rows=int(n_rows))
    _mod().ltv_assemble(d, _stream())


# --------------------------------------------------------------------------- K4
def pack_fragments(w, k_pad: int, ks_major: bool = False) -> torch.Tensor:
    """[N, K] float -> bf16 MFMA B-fragment order P[N/16][k_pad/32][64 lanes][8]
    (lane l of tile (nt, ks) holds W[nt*16 + (l&15)][ks*32 + 8*(l>>4) .. +8]).
    ``ks_major``: P[k_pad/32][N/16][64][8] - the tiles one k-step reads across all columns are
    contiguous. The chain kernels stream weights that way: every CU of an XCD reads the same
    k-step at about the same time, and with N/16-major order those 1-KB tiles sat NKS KB apart,
    i.e. on the same few L2 channels."""
    import numpy as np
    w = np.asarray(w, np.float32)
    n, k = w.shape
    if n % 16 or k > k_pad or k_pad % 32:
        raise ValueError("pack_fragments: N must be a multiple of 16 and K <= k_pad (multiple of 32)")
    buf = np.zeros((n, k_pad), np.float32)
    buf[:, :k] = w
    # [nt, 16 rows, ks, 4 kgroups, 8] -> [nt, ks, kgroup, row, 8] (lane = kgroup*16 + row)
    t = buf.reshape(n // 16, 16, k_pad // 32, 4, 8).transpose(0, 2, 3, 1, 4)
    if ks_major:
        t = t.transpose(1, 0, 2, 3, 4)
    return torch.from_numpy(np.ascontiguousarray(t).reshape(-1)).to(torch.bfloat16)


class GruPack:
    """Device weights of a 1-2 layer GRU chain (+ optional N=1 head) for the K4 kernel."""

    def __init__(self, layers, head=None, device="cuda", split: bool = False, reverse: bool = False):
        """``split``: f32-faithful mode (gru.hip layer_step_x3): each weight also as its bf16
        residual w - bf16(w); the kernel runs three MFMAs per product on (hi, lo) pairs.
        ``reverse``: ONNX direction=reverse for every layer (the kernels read the sequence last
        step first: forward recurrences over the time-reversed input give the same states)."""
        import numpy as np
        if not 1 <= len(layers) <= 2:
            raise ValueError("gru: 1 or 2 stacked layers are lowered")
        H = layers[0].hidden
        if H not in (64, 128, 256):
            raise ValueError("gru: hidden size must be 64, 128 or 256")
        if layers[0].in_dim % 8 or layers[0].in_dim > 64:
            raise ValueError("gru: input dim must be a multiple of 8, <= 64")
        if len(layers) == 2 and (layers[1].hidden != H or layers[1].in_dim != H):
            raise ValueError("gru: layer 2 must be H -> H")
        if len({int(l.linear_before_reset) for l in layers}) != 1:
            raise ValueError("gru: layers must share linear_before_reset")
        self.H, self.I, self.n_layers = H, layers[0].in_dim, len(layers)
        self.reverse = bool(reverse)
        self.waves = 0
        self.lbr = int(layers[0].linear_before_reset)
        dev = as_device(device)
        self.split = bool(split)
        self.x3_rows = 16  # rows per workgroup of the split kernel (32: see AbuseGpu overlap)
        self.layers = []

        def residual(w):
            w = np.ascontiguousarray(w, np.float32)
            return w - torch.from_numpy(w).to(torch.bfloat16).float().numpy()
        for i, l in enumerate(layers):
            kx = H if i == 1 else (32 if l.in_dim <= 32 else 64)
            self.layers.append(dict(W=pack_fragments(l.w_np, kx).to(dev), R=pack_fragments(l.r_np, H).to(dev),
                                    Wlo=pack_fragments(residual(l.w_np), kx).to(dev) if self.split else None,
                                    Rlo=pack_fragments(residual(l.r_np), H).to(dev) if self.split else None,
                                    bias=torch.from_numpy(np.ascontiguousarray(l.b_np, np.float32)).to(dev),
                                    kx_pad=kx, lbr=self.lbr))
        self.head_w = self.head_b = None
        self.head_act = 0
        if head is not None:
            if head.n != 1 or head.k != H or head.act not in ("none", "sigmoid"):
                raise ValueError("gru: head must be dense H -> 1 with none/sigmoid")
            self.head_w = torch.from_numpy(np.ascontiguousarray(head.w_np[0], np.float32)).to(dev)
            self.head_b = float(head.b_np[0]) if head.b_np is not None else 0.0
            self.head_act = ACT[head.act]
        self.device = dev
        # weight-stationary cluster kernels for 2 x 256, lbr = 1, I <= 32: bf16 (gru_ws.hip, 8
        # members per 128 / 64 rows) and, for small f32-faithful batches, the split variant
        # (gru_wsx.hip, 16 members per 32 rows; the launcher picks it up to n_cu / 4 workgroups)
        shape_ok = self.n_layers == 2 and H == 256 and self.lbr == 1 and self.I <= 32
        self.ws_ok = shape_ok and not self.split
        self.wsx_ok = shape_ok and self.split
        self._ws = None
        self._ws_old = []  # superseded workspaces stay alive: captured graphs keep their pointers
        self.ws_err = torch.zeros(1, dtype=torch.int32, device=dev) if (self.ws_ok or self.wsx_ok) else None

    def workspace(self, n_rows: int):
        """Hand-off slabs / counters / head partials for ``n_rows`` (grow-only)."""
        if self.wsx_ok:  # 32-row clusters of 16 members: [2 parities][16][4 blocks][32][16] bf16
            ncl = -(-int(n_rows) // 32)
            if self._ws is None or self._ws["clusters"] < ncl:
                if self._ws is not None:
                    self._ws_old.append(self._ws)
                dev = self.device
                self._ws = dict(clusters=ncl, sync=torch.zeros(ncl * 16, dtype=torch.int32, device=dev),
                                x=torch.zeros(ncl * 2 * 16 * 4 * 32 * 16, dtype=torch.int16, device=dev),
                                part=torch.zeros(ncl * 16 * 32, dtype=torch.float32, device=dev))
            return self._ws
        if not self.ws_ok:
            return None
        ncl = -(-int(n_rows) // 128)
        if self._ws is None or self._ws["clusters"] < ncl:
            if self._ws is not None:
                self._ws_old.append(self._ws)
            dev = self.device
            self._ws = dict(clusters=ncl,
                            # 16 counters per 128-row cluster, or per 64-row cluster (ws = 3)
                            sync=torch.zeros(ncl * 32, dtype=torch.int32, device=dev),
                            x=torch.zeros(ncl * 2 * 8 * 2 * 128 * 32, dtype=torch.int16, device=dev),
                            part=torch.zeros(ncl * 8 * 128, dtype=torch.float32, device=dev))
        return self._ws

    def ws_failed(self) -> bool:
        """True if a cluster launch ever timed out waiting for a non-resident member."""
        return bool(self.ws_err is not None and int(self.ws_err.item()) != 0)

    def disable_ws(self, keep_wsx: bool = False) -> None:
        """After a failed cluster launch (NaN outputs / ws_err): counters back to 0 and every
        later launch on the batch-parallel kernel (callers re-capture their graphs).
        ``keep_wsx``: only the bf16 cluster kernel (a caller that falls back on its own)."""
        self.ws_ok = False
        if keep_wsx:
            return
        self.wsx_ok = False
        for w in [self._ws] + self._ws_old:
            if w is not None:
                w["sync"].zero_()
        if self.ws_err is not None:
            self.ws_err.zero_()


# default cluster layout: 1 one 128-row cluster per CU, 3 two 64-row clusters per CU
_GRU_WS_MODE = int(os.environ.get("IGP_GRU_WS_MODE", "3"))


def gru(gp: GruPack, n_rows: int, T: int, out: Optional[torch.Tensor] = None, yh: Optional[torch.Tensor] = None,
        X: Optional[torch.Tensor] = None, store=None, slots: Optional[torch.Tensor] = None,
        m_ptr: Optional[torch.Tensor] = None, tile_rows: int = 0, waves: int = 0, pipeline: int = 1,
        ws: Optional[int] = None, ws_trace: Optional[torch.Tensor] = None) -> None:
    """K4. Input either dense ``X`` f32 [T, rows, I] or the store's event rings for ``slots``.
    ``ws``: 0 the batch-parallel kernel; 1 the weight-stationary cluster kernel when the model
    shape allows it; 2 the same with its two-half hand-off pipeline; 3 two 64-row clusters per
    CU (gru_ws2_kernel); None: IGP_GRU_WS_MODE (3)."""
    if ws is None:
        ws = _GRU_WS_MODE
    if ws not in (0, 1, 2, 3):
        raise ValueError("gru: ws must be 0..3")
    dev = gp.device
    d = dict(n_layers=gp.n_layers, H=gp.H, T=int(T), I=gp.I, n_rows=int(n_rows),
             m_ptr=_opt(m_ptr, "m_ptr", dtype=torch.int32, device=dev), tile_rows=int(tile_rows),
             waves=int(waves or gp.waves), pipeline=int(pipeline))
    w = gp.workspace(n_rows) if ws else None
    if w is not None:
        d.update(ws=int(ws), ws_clusters=w["clusters"], ws_sync=w["sync"].data_ptr(), ws_x=w["x"].data_ptr(),
                 ws_part=w["part"].data_ptr(), ws_err=gp.ws_err.data_ptr(),
                 ws_trace=_opt(ws_trace, "ws_trace", dtype=torch.int64, min_numel=64 * 8 + 4 + 1024, device=dev))
    if gp.split:
        d["split"] = 1
        if not tile_rows:
            d["tile_rows"] = int(gp.x3_rows)
    if gp.reverse:
        d["reverse"] = 1
    for i, l in enumerate(gp.layers):
        d[f"l{i}_W"] = _need(l["W"], "W", torch.bfloat16, device=dev)
        d[f"l{i}_R"] = _need(l["R"], "R", torch.bfloat16, device=dev)
        if gp.split:
            d[f"l{i}_Wlo"] = _need(l["Wlo"], "Wlo", torch.bfloat16, device=dev)
            d[f"l{i}_Rlo"] = _need(l["Rlo"], "Rlo", torch.bfloat16, device=dev)
        d[f"l{i}_bias"] = _need(l["bias"], "bias", torch.float32, 6 * gp.H, dev)
        d[f"l{i}_kx_pad"] = l["kx_pad"]
        d[f"l{i}_lbr"] = l["lbr"]
    if X is not None:
        if X.dim() != 3 or X.shape[0] < T or X.shape[1] < n_rows or X.shape[2] != gp.I:
            raise ValueError(f"gru: X must be [T>={T}, rows>={n_rows}, {gp.I}]")
        d.update(mode=0, X=_need(X, "X", torch.float32, device=dev), x_rows=int(X.shape[1]))
    else:
        if store is None or slots is None or store.ev is None:
            raise ValueError("gru: need X or (store with event rings, slots)")
        if store.ev.shape[2] != gp.I or store.ev.shape[1] < T:
            raise ValueError("gru: event ring width / length does not match the model")
        d.update(mode=1, ev=_need(store.ev, "ev", torch.int16, device=dev),
                 rt=_need(store.rt, "rt", torch.int32, device=dev),
                 slots=_need(slots, "slots", torch.int32, n_rows, dev), ev_ring=int(store.ev.shape[1]))
    if yh is not None:
        d["yh"] = _need(yh, "yh", torch.float32, n_rows * gp.H, dev)
    if gp.head_w is not None:
        if out is None:
            raise ValueError("gru: a model with a head needs out")
        d.update(head_w=_need(gp.head_w, "head_w", torch.float32, gp.H, dev), head_b=gp.head_b,
                 head_act=gp.head_act, out=_need(out, "out", torch.float32, n_rows, dev))
    elif yh is None:
        raise ValueError("gru: nothing to write (no head, no yh)")
    _mod().gru(d, _stream())


# --------------------------------------------------------------------------- K3 fused MLP chain
class MlpChainPack:
    """Device weights of a dense chain for the fused kernel (csrc/kernels/mlp_fused.hip):
    ``steps`` = DenseStep* + HeadStep (models/plan.py). Each layer's bf16 W [N][K_pad] (K padded
    with zeros to a multiple of 64), f32 bias; the head's N -> 1 vector in f32."""

    MAX_LAYERS = 8

    @staticmethod
    def eligible(steps) -> bool:
        if not steps or steps[-1].kind != "head" or any(s.kind != "dense" for s in steps[:-1]):
            return False
        if any(getattr(s, "src", None) is not None for s in steps):
            return False  # DAG plans run step by step (engine/runner.py)
        if len(steps) > MlpChainPack.MAX_LAYERS:
            return False
        widths = [s.n for s in steps[:-1]] + [steps[-1].n1]
        ks = [s.k for s in steps[:-1]] + [steps[-1].k]
        if any(n % 64 or n < 64 or n > 512 for n in widths) or any(k < 1 or k > 512 for k in ks):
            return False
        return all(ks[i] == widths[i - 1] for i in range(1, len(ks)))

    def __init__(self, steps, device, split: bool = False):
        """``split``: f32-faithful mode - each weight also as its bf16 residual w - bf16(w), and
        the kernel runs three MFMAs per product on (hi, lo) pairs (mlp_fused.hip SPLIT)."""
        import numpy as np
        if not self.eligible(steps):
            raise ValueError("mlp_chain: the plan is not a dense chain the fused kernel covers")
        dev = as_device(device)
        self.split = bool(split)
        self.layers = []
        for s in steps:
            w = np.asarray(s.w1_np if s.kind == "head" else s.w_np, np.float32)
            b = s.b1_np if s.kind == "head" else s.b_np
            n, k = w.shape
            kp = -(-k // 64) * 64
            # MFMA B-fragment order (pack_fragments, k-step major): one 1 KB contiguous wave load
            # per 16x32 tile, a k-step's tiles of all columns contiguous
            lo = None
            if self.split:
                hi = torch.from_numpy(np.ascontiguousarray(w)).to(torch.bfloat16).float().numpy()
                lo = pack_fragments(w - hi, kp, ks_major=True).to(dev)
            self.layers.append(dict(W=pack_fragments(w, kp, ks_major=True).to(dev), Wlo=lo,
                                    b=None if b is None else torch.from_numpy(np.ascontiguousarray(b, np.float32)).to(dev),
                                    N=n, K=kp, act=ACT[s.act1 if s.kind == "head" else s.act]))
        head = steps[-1]
        self.w2 = torch.from_numpy(np.ascontiguousarray(head.w2_np, np.float32)).to(dev)
        self.b2, self.act2 = float(head.b2), ACT[head.act2]
        self.in_live = steps[0].k
        self.in_w = self.layers[0]["K"]
        self.device = dev

    def waves(self) -> int:
        """Waves per workgroup: 8 needs every layer width to be a multiple of 128."""
        # 8: +11 % cfg4 over 4 (same-box A/B, NOTES.md)
        return 8 if all(l["N"] % 128 == 0 for l in self.layers) else 4


def mlp_chain(pk: MlpChainPack, n_rows: int, X: Optional[torch.Tensor] = None, slots: Optional[torch.Tensor] = None,
              pf_tab: Optional[torch.Tensor] = None, ext_tab: Optional[torch.Tensor] = None,
              ml: Optional[torch.Tensor] = None, ltv_out: Optional[torch.Tensor] = None,
              m_ptr: Optional[torch.Tensor] = None, ws_key: int = 0) -> None:
    """Fused dense chain + N=1 head over ``n_rows`` rows. Input: dense ``X`` [rows, >= in] f32, or
    the LTV gather (``slots`` into ``pf_tab`` [C, 25] / ``ext_tab`` [C, ext_w]); outputs ``ml``
    [rows] and/or the K9 rows ``ltv_out`` [rows, 6] (a GPU tensor, or a pinned host tensor that
    the epilogue writes through the fabric: no D2H copy). ``ws_key`` is accepted for call-site
    compatibility (the one-workgroup chain keeps no workspace)."""
    dev = pk.device
    d = dict(n_rows=int(n_rows), n_layers=len(pk.layers), in_w=pk.in_w, in_live=pk.in_live,
             rows_per_block=int(os.environ.get("IGP_MLP_ROWS", "64")), waves=pk.waves(),
             m_ptr=_host_or_dev(m_ptr, "m_ptr", 1, dev, torch.int32), w2=_need(pk.w2, "w2", torch.float32, device=dev),
             b2=pk.b2, act2=pk.act2,
             ml=_opt(ml, "ml", dtype=torch.float32, min_numel=n_rows, device=dev),
             ltv_out=_host_or_dev(ltv_out, "ltv_out", 6 * n_rows, dev))
    if slots is not None:
        if pf_tab is None or pf_tab.dim() != 2 or pf_tab.shape[1] != 25:
            raise ValueError("mlp_chain: LTV gather needs the [C, 25] profile table")
        ext_w = 0 if ext_tab is None else int(ext_tab.shape[1])
        if 25 + ext_w < pk.in_live:
            raise ValueError("mlp_chain: tables narrower than the model input")
        if slots is None:
            raise ValueError("slots: tensor required")
        d.update(slots=_host_or_dev(slots, "slots", n_rows, dev, torch.int32),
                 pf_tab=_need(pf_tab, "pf_tab", torch.float32, device=dev),
                 ext_tab=_opt(ext_tab, "ext_tab", dtype=torch.float32, device=dev), ext_w=ext_w)
    else:
        if X is None or X.dim() != 2 or X.shape[1] < pk.in_live or X.shape[0] < n_rows:
            raise ValueError("mlp_chain: X must be [>= rows, >= model input]")
        if ltv_out is not None:
            raise ValueError("mlp_chain: the K9 epilogue needs slots")
        d.update(X=_need(X, "X", torch.float32, device=dev), ldx=int(X.shape[1]))
    if ml is None and ltv_out is None:
        raise ValueError("mlp_chain: nothing to write")
    for i, l in enumerate(pk.layers):
        d[f"l{i}_W"] = _need(l["W"], "W", torch.bfloat16, l["N"] * l["K"], dev)
        if pk.split:
            d[f"l{i}_Wlo"] = _need(l["Wlo"], "Wlo", torch.bfloat16, l["N"] * l["K"], dev)
        d[f"l{i}_b"] = _opt(l["b"], "b", dtype=torch.float32, min_numel=l["N"], device=dev)
        d[f"l{i}_N"], d[f"l{i}_K"], d[f"l{i}_act"] = l["N"], l["K"], l["act"]
    if pk.split:
        # 64 rows x 8 waves (hi + lo tiles in LDS once): 123-128 vs 91 M predictions/s for 32
        # rows, same box (profiles/r3/x); 4-wave chains keep 32
        rows = int(os.environ.get("IGP_MLP_SPLIT_ROWS", "64" if d["waves"] == 8 else "32"))
        d.update(split=1, rows_per_block=rows if d["waves"] == 8 else 32)
    _mod().mlp_chain(d, _stream())

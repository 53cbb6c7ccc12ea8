"""Owner-routed row exchange: the data-parallel hot path of multi-GPU serving and of
``bench.py --gpus N`` (reference scaling claim: README.md:157-160).

Every rank may ingest requests. Each row goes to the rank that owns its account
(``owner = XXH64(account_id) % world``), every rank scores ONLY the rows it owns, and the
packed results return to the ingress rank. The wire format is the same on GPUs (RCCL over
xGMI, device-resident, ``csrc/kernels/exchange.hip``) and on CPU shards (torch.distributed
over gloo, :class:`HostExchange`):

  send buffer   N chunks of (1 + C) REQREC records; record 0 of chunk ``o`` is a header whose
                ``slot`` field holds the number of rows for owner ``o`` (<= C, the chunk capacity)
  all-to-all    chunk ``o`` of every sender lands in the owner's receive buffer
  owner         compacts the received rows (sender order, then row order) and scores them
  result buffer N chunks of C result records (ResultRec 8 B, + FeatRec 128 B when features
                are wanted), record j of chunk ``p`` answering row j that sender ``p`` sent
  all-to-all    back to the senders, who un-permute with the gather index of :func:`build_chunks`

All collectives are fixed-size per chunk capacity C (a batch bucket), so nothing needs the
row counts on the host of the receiving rank.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import numpy as np

from ..layouts import FEATREC, REQREC

RES_BYTES = 8
FEAT_BYTES = FEATREC.itemsize


def chunk_rows(C: int) -> int:
    return C + 1


def result_width(want_features: bool) -> int:
    return RES_BYTES + (FEAT_BYTES if want_features else 0)


def build_chunks(req: np.ndarray, owners: np.ndarray, world: int, C: int,
                 out: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Rows -> the send buffer of the exchange.

    Returns ``(buf, gather, counts)``: ``buf`` REQREC ``[world * (C + 1)]``, ``gather[i]`` =
    ``owner * C + j`` (row i's position in the returned results) and the per-owner counts.
    Raises if an owner receives more than ``C`` rows (callers pick C >= the largest count,
    or split the batch)."""
    n = len(req)
    owners = np.asarray(owners, np.int64)
    if n and (owners.min() < 0 or owners.max() >= world):
        raise ValueError("owner out of range")
    counts = np.bincount(owners, minlength=world).astype(np.int64)
    if n and counts.max() > C:
        raise ValueError(f"owner receives {int(counts.max())} rows > chunk capacity {C}")
    if out is None:
        out = np.zeros(world * (C + 1), REQREC)
    elif len(out) < world * (C + 1) or out.dtype != REQREC:
        raise ValueError("chunk buffer too small")
    order = np.argsort(owners, kind="stable")
    starts = np.zeros(world, np.int64)
    starts[1:] = np.cumsum(counts)[:-1]
    j = np.empty(n, np.int64)
    j[order] = np.arange(n) - np.repeat(starts, counts)
    dst = owners * (C + 1) + 1 + j
    out[dst] = req
    hdr = np.arange(world) * (C + 1)
    out[hdr] = np.zeros(1, REQREC)
    out["slot"][hdr] = counts
    return out, owners * C + j, counts


def max_owner_count(owners: np.ndarray, world: int) -> int:
    return int(np.bincount(np.asarray(owners, np.int64), minlength=world).max()) if len(owners) else 0


def compact(recv: np.ndarray, world: int, C: int) -> Tuple[np.ndarray, np.ndarray]:
    """Host twin of the ``exchange_compact`` kernel: received chunks -> (rows, route)."""
    recv = recv.reshape(world, C + 1)
    counts = np.clip(recv["slot"][:, 0], 0, C)
    rows = np.concatenate([recv[p, 1:1 + counts[p]] for p in range(world)]) if world else np.zeros(0, REQREC)
    route = np.concatenate([p * C + np.arange(counts[p]) for p in range(world)]).astype(np.int64)
    rows = rows.copy()
    rows["tx_type"] &= 0xFF
    return rows, route


def scatter_results(res: np.ndarray, feats: Optional[np.ndarray], route: np.ndarray, world: int,
                    C: int) -> np.ndarray:
    """Host twin of ``exchange_scatter``: results of compact rows -> the result send buffer
    ``uint8 [world, C * W]`` (C ResultRec, then C FeatRec when ``feats`` is given)."""
    W = result_width(feats is not None)
    buf = np.zeros((world, C * W), np.uint8)
    p, j = route // C, route % C
    r = buf[:, :C * RES_BYTES].reshape(world, C, RES_BYTES)  # views (split of the last axis)
    r[p, j] = np.ascontiguousarray(res, np.uint32).view(np.uint8).reshape(-1, RES_BYTES)
    if feats is not None:
        f = buf[:, C * RES_BYTES:].reshape(world, C, FEAT_BYTES)
        f[p, j] = np.ascontiguousarray(feats).view(np.uint8).reshape(-1, FEAT_BYTES)
    return buf


def gather_results(recv: np.ndarray, gather: np.ndarray, world: int, C: int,
                   want_features: bool) -> Tuple[np.ndarray, Optional[np.ndarray]]:
    """Received result chunks -> (ResultRec uint32 [n, 2], FeatRec [n] or None) in the
    ingress order (``gather`` from :func:`build_chunks`)."""
    W = result_width(want_features)
    buf = np.asarray(recv).view(np.uint8).reshape(world, C * W)
    res = np.ascontiguousarray(buf[:, :C * RES_BYTES]).view(np.uint32).reshape(world * C, 2)[gather]
    feats = None
    if want_features:
        feats = np.ascontiguousarray(buf[:, C * RES_BYTES:]).view(FEATREC).reshape(world * C)[gather]
    return res, feats


class HostExchange:
    """The exchange over torch.distributed CPU tensors (gloo): CPU shards in SPMD serving and
    the multi-process CPU tests. ``score_fn(rows, want_features) -> (res, feats)`` scores
    this rank's owned rows; ``rows_scored`` counts them (tests assert owned-rows-only)."""

    def __init__(self, rank: int, world: int, comm=None):
        """``comm``: a :class:`~.comm.TorchComm` (its per-op deadline bounds both all-to-alls);
        None: plain torch.distributed calls on the default group."""
        self.rank, self.world = rank, world
        self.comm = comm
        self.rows_scored = 0
        self.batches = 0

    def _a2a(self, send: np.ndarray, per_peer: int) -> np.ndarray:
        if self.world == 1:
            return send.copy()
        if self.comm is not None and hasattr(self.comm, "all_to_all_bytes"):
            return self.comm.all_to_all_bytes(send, per_peer)
        import torch
        import torch.distributed as dist
        s = torch.from_numpy(np.ascontiguousarray(send).view(np.uint8).reshape(-1))
        r = torch.empty(self.world * per_peer, dtype=torch.uint8)
        dist.all_to_all_single(r, s)
        return r.numpy()

    def step(self, req: Optional[np.ndarray], owners: Optional[np.ndarray], C: int, want_features: bool,
             score_fn):
        """One exchange step (collective: every rank calls it with the same C/want_features;
        non-ingress ranks pass ``req=None``). Returns the ingress rows' (res, feats)."""
        world = self.world
        if req is None or len(req) == 0:
            buf, gather = build_chunks(np.zeros(0, REQREC), np.zeros(0, np.int64), world, C)[:2]
        else:
            buf, gather = build_chunks(req, owners, world, C)[:2]
        recv = self._a2a(buf.view(np.uint8), (C + 1) * REQREC.itemsize).view(REQREC)
        rows, route = compact(recv, world, C)
        self.batches += 1
        self.rows_scored += len(rows)
        if len(rows):
            res, feats = score_fn(rows, want_features)
        else:
            res, feats = np.zeros((0, 2), np.uint32), (np.zeros(0, FEATREC) if want_features else None)
        out = scatter_results(res, feats if want_features else None, route, world, C)
        back = self._a2a(out, C * result_width(want_features))
        if req is None or len(req) == 0:
            return np.zeros((0, 2), np.uint32), (np.zeros(0, FEATREC) if want_features else None)
        return gather_results(back, gather, world, C, want_features)


# --------------------------------------------------------------------------------- RCCL
def rccl_lib_path() -> str:
    import torch
    return os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so.1")


def rccl_comms(rank: int, world: int, n: int = 2):
    """``n`` RCCL communicators of our own over the ranks of the current torch.distributed
    group (rank 0 makes the unique ids; one object broadcast). The exchange uses two: one for
    the row all-to-all, one for the result all-to-all, so the two directions of consecutive
    micro-batches progress independently."""
    from ..native import hipk
    m = hipk()
    lib = rccl_lib_path()
    ids = [m.rccl_unique_id(lib) for _ in range(n)] if rank == 0 else [None] * n
    if world > 1:
        import torch.distributed as dist
        dist.broadcast_object_list(ids, src=0)
    return [m.RcclComm(lib, rank, world, bytes(u)) for u in ids]


def chunk_capacity(batch: int, world: int, slack: float = 1.125, align: int = 64) -> int:
    """Per-owner chunk capacity for a rank ingesting ``batch`` hash-routed rows per step."""
    if world == 1:
        return batch
    c = int(np.ceil(batch * slack / world))
    return min(batch, -(-c // align) * align)

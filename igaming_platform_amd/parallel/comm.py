"""Collectives for the serving/bench data-parallel paths.

One process per GPU; ``torch.distributed`` with backend ``nccl`` (= RCCL over xGMI on ROCm)
for device tensors, or ``gloo`` for CPU tests. Every message is tiny (a batch slab of
48 B/request, 8 B result records, a 1 KiB metrics block), so the collectives are latency-
bound: the API moves host numpy buffers through ONE pre-allocated staging tensor per
direction instead of allocating per call. A :class:`LoopbackComm` (world 1) lets the same
code run single-process.

Failure handling (the reference bounds every call with a context deadline and recovers a
panicking handler, services/risk/cmd/main.go:329-342): the process group is created with a
timeout (``RISK_SPMD_TIMEOUT_S``, default 30 s) and every collective rank 0 issues waits at
most ``RISK_SPMD_OP_TIMEOUT_S`` (default 10 s, ``Work.wait(timeout)``), so a dead or stuck
rank surfaces as an exception on rank 0 instead of a hang. Serving runs this control plane
over gloo even on GPUs: an RCCL timeout would tear the rank-0 process down, and the hot path
moves its rows over RCCL communicators of its own (parallel/exchange.py) anyway.
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

import numpy as np


def spmd_timeouts():
    """(group timeout, per-op deadline) in seconds from RISK_SPMD_TIMEOUT_S / _OP_TIMEOUT_S."""
    return (float(os.environ.get("RISK_SPMD_TIMEOUT_S", "30")),
            float(os.environ.get("RISK_SPMD_OP_TIMEOUT_S", "10")))


def init_from_env(backend: Optional[str] = None, device=None, timeout_s: Optional[float] = None,
                  op_timeout_s: Optional[float] = None):
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_* (127.0.0.1 default) with a
    group timeout; returns a :class:`TorchComm` whose collectives carry the per-op deadline."""
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    t_group, t_op = spmd_timeouts()
    timeout_s = t_group if timeout_s is None else timeout_s
    op_timeout_s = t_op if op_timeout_s is None else op_timeout_s
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if not dist.is_initialized():
        kw = {}
        if backend == "nccl" and device is not None:
            kw["device_id"] = torch.device(device)
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return TorchComm(backend, device, op_timeout_s=op_timeout_s)


class LoopbackComm:
    rank, world = 0, 1

    def bcast_bytes(self, data: Optional[bytes], src: int = 0) -> bytes:
        return data

    def bcast_i64(self, arr: np.ndarray, src: int = 0, deadline: bool = True) -> np.ndarray:
        return arr

    def all_to_all_bytes(self, send: np.ndarray, per_peer: int) -> np.ndarray:
        return np.ascontiguousarray(send).view(np.uint8).reshape(-1).copy()

    def sum_i64(self, arr: np.ndarray) -> np.ndarray:
        return arr

    def gather_bytes(self, data: bytes, dst: int = 0):
        return [data]

    def barrier(self) -> None:
        pass


class TorchComm:
    """Host-buffer collectives over a torch.distributed process group. With ``op_timeout_s``
    every collective waits at most that long (``deadline=False`` opts out: a worker's idle
    wait for rank 0's next op, bounded by the group timeout and rank 0's heartbeats)."""

    def __init__(self, backend: str, device=None, cap_bytes: int = 1 << 20, op_timeout_s: Optional[float] = None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.backend = backend
        self.op_timeout = datetime.timedelta(seconds=op_timeout_s) if op_timeout_s else None
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        if backend == "nccl":
            self.dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        else:
            self.dev = torch.device("cpu")
        self._hdr = torch.zeros(2, dtype=torch.int64, device=self.dev)
        self._cap = 0
        self._buf = None
        self._grow(cap_bytes)

    def _grow(self, n: int) -> None:
        if n > self._cap:
            self._cap = max(n, 2 * self._cap)
            self._buf = self.torch.zeros(self._cap, dtype=self.torch.uint8, device=self.dev)

    def _wait(self, work, deadline: bool = True) -> None:
        if deadline and self.op_timeout is not None:
            work.wait(timeout=self.op_timeout)
        else:
            work.wait()

    def bcast_bytes(self, data: Optional[bytes], src: int = 0) -> bytes:
        """Length-prefixed broadcast (2 collectives: length, then payload)."""
        torch = self.torch
        if self.rank == src:
            self._hdr[0] = len(data)
        self._wait(self.dist.broadcast(self._hdr, src, async_op=True))
        n = int(self._hdr[0].item())
        self._grow(n)
        if self.rank == src and n:
            self._buf[:n].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
        if n:
            self._wait(self.dist.broadcast(self._buf[:n], src, async_op=True))
        return bytes(self._buf[:n].cpu().numpy()) if n else b""

    def bcast_i64(self, arr: np.ndarray, src: int = 0, deadline: bool = True) -> np.ndarray:
        t = self.torch.from_numpy(np.ascontiguousarray(arr, np.int64)).to(self.dev)
        self._wait(self.dist.broadcast(t, src, async_op=True), deadline)
        return t.cpu().numpy()

    def sum_i64(self, arr: np.ndarray) -> np.ndarray:
        t = self.torch.from_numpy(np.ascontiguousarray(arr, np.int64)).to(self.dev)
        self._wait(self.dist.all_reduce(t, async_op=True))
        return t.cpu().numpy()

    def all_to_all_bytes(self, send: np.ndarray, per_peer: int) -> np.ndarray:
        """Equal ``per_peer``-byte blocks to / from every rank (the host exchange)."""
        torch = self.torch
        s = torch.from_numpy(np.ascontiguousarray(send).view(np.uint8).reshape(-1)).to(self.dev)
        r = torch.empty(self.world * per_peer, dtype=torch.uint8, device=self.dev)
        self._wait(self.dist.all_to_all_single(r, s, async_op=True))
        return r.cpu().numpy()

    def gather_bytes(self, data: bytes, dst: int = 0):
        """Equal-length payloads from every rank -> list on every rank (all_gather)."""
        torch = self.torch
        n = len(data)
        src = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(self.dev) if n else \
            torch.zeros(0, dtype=torch.uint8, device=self.dev)
        out = torch.zeros(n * self.world, dtype=torch.uint8, device=self.dev)
        if n:
            self._wait(self.dist.all_gather_into_tensor(out, src, async_op=True))
        host = out.cpu().numpy()
        return [bytes(host[r * n:(r + 1) * n]) for r in range(self.world)]

    def barrier(self) -> None:
        self._wait(self.dist.barrier(async_op=True))

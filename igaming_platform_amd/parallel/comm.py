"""Collectives for the serving/bench data-parallel paths.

One process per GPU; ``torch.distributed`` with backend ``nccl`` (= RCCL over xGMI on ROCm)
for device tensors, or ``gloo`` for CPU tests. Every message is tiny (a batch slab of
48 B/request, 8 B result records, a 1 KiB metrics block), so the collectives are latency-
bound: the API moves host numpy buffers through ONE pre-allocated staging tensor per
direction instead of allocating per call. A :class:`LoopbackComm` (world 1) lets the same
code run single-process.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np


def init_from_env(backend: Optional[str] = None, device=None):
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_* (127.0.0.1 default)."""
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if not dist.is_initialized():
        kw = {}
        if backend == "nccl" and device is not None:
            kw["device_id"] = torch.device(device)
        dist.init_process_group(backend, **kw)
    return TorchComm(backend, device)


class LoopbackComm:
    rank, world = 0, 1

    def bcast_bytes(self, data: Optional[bytes], src: int = 0) -> bytes:
        return data

    def bcast_i64(self, arr: np.ndarray, src: int = 0) -> np.ndarray:
        return arr

    def sum_i64(self, arr: np.ndarray) -> np.ndarray:
        return arr

    def gather_bytes(self, data: bytes, dst: int = 0):
        return [data]

    def barrier(self) -> None:
        pass


class TorchComm:
    """Host-buffer collectives over a torch.distributed process group."""

    def __init__(self, backend: str, device=None, cap_bytes: int = 1 << 20):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.backend = backend
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

    def bcast_bytes(self, data: Optional[bytes], src: int = 0) -> bytes:
        """Length-prefixed broadcast (2 collectives: length, then payload)."""
        torch = self.torch
        if self.rank == src:
            self._hdr[0] = len(data)
        self.dist.broadcast(self._hdr, src)
        n = int(self._hdr[0].item())
        self._grow(n)
        if self.rank == src and n:
            self._buf[:n].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
        if n:
            self.dist.broadcast(self._buf[:n], src)
        return bytes(self._buf[:n].cpu().numpy()) if n else b""

    def bcast_i64(self, arr: np.ndarray, src: int = 0) -> np.ndarray:
        t = self.torch.from_numpy(np.ascontiguousarray(arr, np.int64)).to(self.dev)
        self.dist.broadcast(t, src)
        return t.cpu().numpy()

    def sum_i64(self, arr: np.ndarray) -> np.ndarray:
        t = self.torch.from_numpy(np.ascontiguousarray(arr, np.int64)).to(self.dev)
        self.dist.all_reduce(t)
        return t.cpu().numpy()

    def gather_bytes(self, data: bytes, dst: int = 0):
        """Equal-length payloads from every rank -> list on every rank (all_gather)."""
        torch = self.torch
        n = len(data)
        src = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(self.dev) if n else \
            torch.zeros(0, dtype=torch.uint8, device=self.dev)
        out = torch.zeros(n * self.world, dtype=torch.uint8, device=self.dev)
        if n:
            self.dist.all_gather_into_tensor(out, src)
        host = out.cpu().numpy()
        return [bytes(host[r * n:(r + 1) * n]) for r in range(self.world)]

    def barrier(self) -> None:
        self.dist.barrier()

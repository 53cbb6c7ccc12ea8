"""Account registry: account id -> (owner GPU, slot in that GPU's feature shard).

Routing is by account owner, ``owner = XXH64(account_id) % world`` (SURVEY §2.5 DP), so all of
an account's state lives on one GPU and the hot path needs no cross-GPU feature traffic.
Each owner has its own C++ :class:`AccountIndex` (lock-free open addressing, exact id
verification). In multi-rank serving every rank ingests, so the indexes live in /dev/shm and
every rank of the node maps the same ones (``shm_prefix``): an account gets one slot on its
owner whichever rank saw it first.
"""
from __future__ import annotations

import threading
from typing import Sequence, Tuple

import numpy as np

from ..native import native
from ..utils.hashing import SEED_ACCOUNT


class AccountRegistry:
    def __init__(self, capacity_per_owner: int, world: int = 1, shm_prefix: str = "", create: bool = True):
        N = native()
        self.world = int(world)
        self.capacity = int(capacity_per_owner)
        if shm_prefix:
            self.index = [N.AccountIndex(self.capacity, f"{shm_prefix}-acct{o}", create) for o in range(self.world)]
        else:
            self.index = [N.AccountIndex(self.capacity) for _ in range(self.world)]
        self._lock = threading.Lock()

    def unlink_shared(self) -> None:
        """Drop the /dev/shm names (every rank has mapped the indexes; mappings stay valid)."""
        for ix in self.index:
            if ix.shared:
                ix.unlink_shared()

    def owner_of_hash(self, h: np.ndarray) -> np.ndarray:
        return (np.asarray(h, np.uint64) % np.uint64(self.world)).astype(np.int32)

    def resolve_batch(self, batch, insert: bool = True) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """``batch``: _native.RequestBatch -> (slots, owners, fresh). Unknown accounts get a slot
        on their owner when ``insert`` (their events must accumulate); -1 when the shard is full."""
        cols = batch.columns()
        owners = self.owner_of_hash(cols["account_hash"])
        n = len(owners)
        if self.world == 1:
            slots, fresh = self.index[0].lookup_batch(batch, insert)
            return np.asarray(slots, np.int32), owners, np.asarray(fresh, bool)
        slots = np.full(n, -1, np.int32)
        fresh = np.zeros(n, bool)
        for o in range(self.world):
            mine = owners == o
            if not mine.any():
                continue
            s, f = self.index[o].lookup_batch(batch, insert, mine)  # C++, GIL released
            slots[mine] = s[mine]
            fresh[mine] = np.asarray(f, bool)[mine]
        return slots, owners, fresh

    def resolve_ids(self, ids: Sequence[str], insert: bool = False) -> Tuple[np.ndarray, np.ndarray]:
        ids = list(ids)
        if self.world == 1:  # digests and lookups in C++ (GIL released)
            s, _ = self.index[0].lookup(ids, insert)
            return np.asarray(s, np.int32), np.zeros(len(ids), np.int32)
        h = native().id_hashes(ids, SEED_ACCOUNT)
        owners = self.owner_of_hash(h)
        slots = np.full(len(ids), -1, np.int32)
        for o in range(self.world):
            sel = np.nonzero(owners == o)[0]
            if len(sel):
                s, _ = self.index[o].lookup([ids[i] for i in sel], insert)
                slots[sel] = s
        return slots, owners

    def resolve(self, account_id: str, insert: bool = False) -> Tuple[int, int]:
        s, o = self.resolve_ids([account_id], insert)
        return int(s[0]), int(o[0])

    def size(self, owner: int = 0) -> int:
        return len(self.index[owner])

    def id_of(self, owner: int, slot: int) -> str:
        return self.index[owner].id_of(int(slot))

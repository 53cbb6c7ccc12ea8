"""Host-authoritative open-addressing hash sets mirrored to the device.

Blacklist (``redis_store.go:244-293``: Redis sets per type) and IP intelligence (the
reference's ``IPIntelligence`` interface, ``engine.go:158-171``, which has no implementation)
are small, rarely-written tables. The host keeps the authoritative copy plus metadata
(reason, created_by, created_at, id); the device gets the (key, value) arrays and is probed
by ``feature_assemble`` with exactly this layout: slot = low 32 bits of the key & mask,
linear probing, key 0 = empty.
"""
from __future__ import annotations

import threading
import uuid
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np

from ..utils.hashing import TYPE_SEEDS, id_hash


class HashSet64:
    def __init__(self, capacity: int):
        cap = 16
        while cap < capacity:
            cap <<= 1
        self.cap = cap
        self.mask = cap - 1
        self.keys = np.zeros(cap, np.uint64)
        self.vals = np.zeros(cap, np.uint32)
        self.max_probe = 0
        self.n = 0
        self.version = 0
        self._lock = threading.Lock()

    def _slot(self, key: int) -> int:
        return int(key & 0xFFFFFFFF) & self.mask

    def put(self, key: int, val: int) -> None:
        if key == 0:
            raise ValueError("key 0 is reserved")
        with self._lock:
            i = self._slot(key)
            for p in range(self.cap):
                k = int(self.keys[i])
                if k == key or k == 0:
                    if k == 0:
                        if self.n + 1 > self.cap * 3 // 4:
                            raise RuntimeError("hash set full")
                        self.n += 1
                    self.keys[i] = np.uint64(key)
                    self.vals[i] = np.uint32(val)
                    self.max_probe = max(self.max_probe, p + 1)
                    self.version += 1
                    return
                i = (i + 1) & self.mask
            raise RuntimeError("hash set full")

    def get(self, key: int) -> Optional[int]:
        if key == 0:
            return None
        i = self._slot(key)
        for _ in range(self.max_probe):
            k = int(self.keys[i])
            if k == 0:
                return None
            if k == key:
                return int(self.vals[i])
            i = (i + 1) & self.mask
        return None


@dataclass
class BlacklistEntry:
    id: str
    type: str
    value: str
    reason: str
    created_by: str
    created_at: int
    expires_at: int  # 0 = never


class Blacklist:
    """All four reference types (device, ip, fingerprint, email: risk.proto:152,
    init-db.sql:158-170) with optional expiry (quirk Q19: the Redis store had neither)."""

    TYPES = ("device", "ip", "fingerprint", "email")

    def __init__(self, capacity: int = 1 << 16):
        self.table = HashSet64(capacity)
        self.entries: Dict[int, BlacklistEntry] = {}

    def add(self, type_: str, value: str, reason: str = "", created_by: str = "",
            expires_at: int = 0, now: int = 0) -> BlacklistEntry:
        if type_ not in self.TYPES:
            raise ValueError(f"unknown blacklist type: {type_}")
        if not value:
            raise ValueError("blacklist value must be non-empty")
        key = id_hash(value, TYPE_SEEDS[type_])
        e = BlacklistEntry(str(uuid.uuid4()), type_, value, reason, created_by, now, int(expires_at))
        self.entries[key] = e
        self.table.put(key, int(expires_at) & 0xFFFFFFFF)
        return e

    def check(self, now: int, device_id: str = "", fingerprint: str = "", ip: str = "",
              email: str = "") -> List[BlacklistEntry]:
        out = []
        for t, v in (("device", device_id), ("fingerprint", fingerprint), ("ip", ip), ("email", email)):
            if not v:
                continue
            e = self.entries.get(id_hash(v, TYPE_SEEDS[t]))
            if e is not None and (e.expires_at == 0 or now < e.expires_at):
                out.append(e)
        return out

    def active_keys(self, now: int) -> Dict[int, int]:
        return {k: e.expires_at for k, e in self.entries.items()
                if e.expires_at == 0 or now < e.expires_at}


class IPIntel:
    """IP -> {vpn, proxy, tor} flags (bit 0/1/2), keyed like the request's ip digest."""

    VPN, PROXY, TOR = 1, 2, 4

    def __init__(self, capacity: int = 1 << 16):
        self.table = HashSet64(capacity)

    def set(self, ip: str, vpn: bool = False, proxy: bool = False, tor: bool = False) -> None:
        flags = (self.VPN if vpn else 0) | (self.PROXY if proxy else 0) | (self.TOR if tor else 0)
        self.table.put(id_hash(ip, TYPE_SEEDS["ip"]), flags)

    def flags(self, ip: str) -> int:
        v = self.table.get(id_hash(ip, TYPE_SEEDS["ip"]))
        return v or 0

"""64-bit identity hashing shared by host, C++ runtime and device tables.

Every string identifier that reaches the GPU is reduced to a 64-bit XXH64 digest with a
per-type seed, so the device never sees strings:

* account ids -> routing (owner GPU = h % world) and the account index,
* device ids / IPs -> HyperLogLog registers (index = low 8 bits, rank from the rest),
* device / fingerprint / ip / email -> blacklist keys (open-addressing set on device).

The reference keeps the raw strings in Redis keys (``redis_store.go:25-35, 244-248``).
Digest 0 is reserved for "absent" (empty string); a real digest of 0 is remapped to 1.

``xxh64`` here is a pure-Python implementation of the public XXH64 algorithm; the
C++ runtime has its own (``csrc/runtime/xxh64.h``) and tests cross-check both against
the ``xxhash`` package when it is importable.
"""
from __future__ import annotations

from typing import Iterable, List

MASK = (1 << 64) - 1
P1 = 0x9E3779B185EBCA87
P2 = 0xC2B2AE3D27D4EB4F
P3 = 0x165667B19E3779F9
P4 = 0x85EBCA77C2B2AE63
P5 = 0x27D4EB2F165667C5

SEED_ACCOUNT = 0x41434354  # "ACCT"
SEED_DEVICE = 0x44455649   # "DEVI"
SEED_FINGERPRINT = 0x46505249  # "FPRI"
SEED_IP = 0x49504144       # "IPAD"
SEED_EMAIL = 0x454D4149    # "EMAI"

TYPE_SEEDS = {
    "device": SEED_DEVICE,
    "fingerprint": SEED_FINGERPRINT,
    "ip": SEED_IP,
    "email": SEED_EMAIL,
}


def _rotl(x: int, r: int) -> int:
    return ((x << r) | (x >> (64 - r))) & MASK


def _round(acc: int, lane: int) -> int:
    acc = (acc + lane * P2) & MASK
    acc = _rotl(acc, 31)
    return (acc * P1) & MASK


def _merge(acc: int, val: int) -> int:
    acc ^= _round(0, val)
    return (acc * P1 + P4) & MASK


def xxh64(data: bytes, seed: int = 0) -> int:
    n = len(data)
    i = 0
    if n >= 32:
        v1 = (seed + P1 + P2) & MASK
        v2 = (seed + P2) & MASK
        v3 = seed & MASK
        v4 = (seed - P1) & MASK
        while i + 32 <= n:
            v1 = _round(v1, int.from_bytes(data[i:i + 8], "little"))
            v2 = _round(v2, int.from_bytes(data[i + 8:i + 16], "little"))
            v3 = _round(v3, int.from_bytes(data[i + 16:i + 24], "little"))
            v4 = _round(v4, int.from_bytes(data[i + 24:i + 32], "little"))
            i += 32
        h = (_rotl(v1, 1) + _rotl(v2, 7) + _rotl(v3, 12) + _rotl(v4, 18)) & MASK
        h = _merge(h, v1)
        h = _merge(h, v2)
        h = _merge(h, v3)
        h = _merge(h, v4)
    else:
        h = (seed + P5) & MASK
    h = (h + n) & MASK
    while i + 8 <= n:
        k1 = _round(0, int.from_bytes(data[i:i + 8], "little"))
        h ^= k1
        h = (_rotl(h, 27) * P1 + P4) & MASK
        i += 8
    if i + 4 <= n:
        h ^= (int.from_bytes(data[i:i + 4], "little") * P1) & MASK
        h = (_rotl(h, 23) * P2 + P3) & MASK
        i += 4
    while i < n:
        h ^= (data[i] * P5) & MASK
        h = (_rotl(h, 11) * P1) & MASK
        i += 1
    h ^= h >> 33
    h = (h * P2) & MASK
    h ^= h >> 29
    h = (h * P3) & MASK
    h ^= h >> 32
    return h


def id_hash(value: str, seed: int) -> int:
    """Digest of an identifier; 0 means absent (empty string)."""
    if not value:
        return 0
    h = xxh64(value.encode("utf-8"), seed)
    return h if h != 0 else 1


def id_hashes(values: Iterable[str], seed: int) -> List[int]:
    return [id_hash(v, seed) for v in values]


def to_i64(h: int) -> int:
    """Reinterpret an unsigned 64-bit digest as int64 (torch has no uint64 arithmetic)."""
    return h - (1 << 64) if h >= (1 << 63) else h


def from_i64(h: int) -> int:
    return h & MASK

"""Golden HyperLogLog (p = 8) — the spec for the device HLL update/count kernels.

Replaces Redis PFADD/PFCOUNT on ``features:<id>:devices:24h`` / ``ips:24h``
(``redis_store.go:80-81, 141-152``). Redis' estimator and hash are not reproduced
bit-for-bit (not observable by clients); the counts agree with the exact distinct
count within HLL error, and for the cardinalities the rules look at (<= ~20) the
linear-counting branch is used, which is exact up to register collisions.

Register update: idx = h & 255, w = h >> 8 (56 bits), rank = clz56(w) + 1 (57 if w == 0),
reg[idx] = max(reg[idx], rank).
Estimate: E = alpha * m^2 / sum(2^-reg); if E <= 2.5 m and V (zero registers) > 0,
E = m * ln(m / V). Count = floor(E + 0.5).
"""
from __future__ import annotations

import math

P = 8
M = 1 << P
ALPHA = 0.7213 / (1.0 + 1.079 / M)


def rank_of(h: int) -> int:
    w = h >> P
    if w == 0:
        return 64 - P + 1
    return (64 - P) - w.bit_length() + 1


def add(regs: bytearray, h: int) -> None:
    if h == 0:
        return
    idx = h & (M - 1)
    r = rank_of(h)
    if r > regs[idx]:
        regs[idx] = r


def linear_count(v: int) -> int:
    """Linear-counting estimate for ``v`` zero registers (the device reads a table of these)."""
    return int(math.floor(M * math.log(M / v) + 0.5))


def count(regs) -> int:
    z = 0.0
    v = 0
    for r in regs:
        z += math.ldexp(1.0, -int(r))
        if r == 0:
            v += 1
    e = ALPHA * M * M / z
    if e <= 2.5 * M and v > 0:
        e = M * math.log(M / v)
    return int(math.floor(e + 0.5))


def count_many(regs) -> "np.ndarray":
    """:func:`count` of every row of ``regs`` (uint8 [n, 256]) at once (numpy; the same sums:
    every partial sum of 2^-r is exact in double). Used to rebuild the cached estimates of
    AcctRT (hll_dev_n / hll_ip_n) when a snapshot is loaded."""
    import numpy as np
    r = np.asarray(regs, np.uint8).reshape(-1, M).astype(np.int64)
    z = np.ldexp(1.0, -r).sum(axis=1)
    v = (r == 0).sum(axis=1)
    e = ALPHA * M * M / z
    lc = np.array([0] + [linear_count(k) for k in range(1, M + 1)], np.int64)
    out = np.floor(e + 0.5).astype(np.int64)
    small = (e <= 2.5 * M) & (v > 0)
    out[small] = lc[v[small]]
    return out.astype(np.int32)


def refresh_cached_counts(hll, rt) -> None:
    """Rewrite AcctRT's cached estimates (structured ``rt`` [n] ACCTRT, in place) from the
    register files ``hll`` (uint8 [n, 512]: device HLL then ip HLL)."""
    import numpy as np
    h = np.asarray(hll, np.uint8).reshape(len(rt), 2, M)
    rt["hll_dev_n"] = count_many(h[:, 0])
    rt["hll_ip_n"] = count_many(h[:, 1])


"""Deterministic synthetic accounts and transaction streams (BASELINE: "synthetic transaction
streams"). The same generator feeds the golden model, the device store, tests and benches.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from ..golden.features import BatchFeatures, TxEvent
from ..layouts import ACCTBATCH, REQREC
from .hashing import SEED_DEVICE, SEED_FINGERPRINT, SEED_IP, id_hash

NOW0 = 1_760_000_000  # 2025-10-09, a fixed synthetic clock


@dataclass
class Population:
    ids: List[str]
    batch: np.ndarray          # ACCTBATCH [n]
    ext: np.ndarray            # f32 [n, E]
    dev_pool: np.ndarray       # u64 [n, P] per-account device digests
    ip_pool: np.ndarray        # u64 [n, P]
    fp_pool: np.ndarray        # u64 [n, P]

    def golden_batch(self, i: int) -> Optional[BatchFeatures]:
        b = self.batch[i]
        if not b["present"]:
            return None
        return BatchFeatures(
            total_deposits=int(b["total_deposits"]), total_withdrawals=int(b["total_withdrawals"]),
            deposit_count=int(b["deposit_count"]), withdraw_count=int(b["withdraw_count"]),
            total_bets=int(b["total_bets"]), total_wins=int(b["total_wins"]), bet_count=int(b["bet_count"]),
            win_count=int(b["win_count"]), avg_bet_size=float(b["avg_bet_size"]),
            account_created_at=int(b["account_created_at"]), bonus_claim_count=int(b["bonus_claim_count"]),
            bonus_wager_complete=float(b["bonus_wager_complete"]))


def _digests(prefix: str, n: int, seed: int) -> np.ndarray:
    return np.array([id_hash(f"{prefix}{i}", seed) for i in range(n)], dtype=np.uint64)


def make_population(n: int, ext_width: int, seed: int = 0, now: int = NOW0, pool: int = 6,
                    missing_batch_frac: float = 0.05, fast_hash: bool = False) -> Population:
    rng = np.random.default_rng(seed)
    ids = [f"acct-{i:08d}" for i in range(n)]
    b = np.zeros(n, ACCTBATCH)
    dep_cnt = rng.poisson(6, n)
    b["deposit_count"] = dep_cnt
    b["total_deposits"] = (dep_cnt * rng.lognormal(8.5, 1.2, n)).astype(np.int64)
    wd_cnt = rng.poisson(2, n)
    b["withdraw_count"] = wd_cnt
    b["total_withdrawals"] = (b["total_deposits"] * rng.uniform(0, 1.3, n)).astype(np.int64)
    bets = rng.poisson(80, n)
    b["bet_count"] = bets
    b["win_count"] = (bets * rng.uniform(0.2, 0.6, n)).astype(np.int32)
    b["total_bets"] = (bets * rng.lognormal(6, 1, n)).astype(np.int64)
    b["total_wins"] = (b["total_bets"] * rng.uniform(0.7, 1.1, n)).astype(np.int64)
    b["avg_bet_size"] = (b["total_bets"] / np.maximum(bets, 1)).astype(np.float32)
    b["account_created_at"] = now - rng.integers(0, 800 * 86400, n)
    b["bonus_claim_count"] = rng.poisson(1.5, n)
    b["bonus_wager_complete"] = rng.uniform(0, 1, n).astype(np.float32)
    b["present"] = (rng.uniform(0, 1, n) >= missing_batch_frac).astype(np.int32)
    ext = rng.uniform(0, 1, (n, max(ext_width, 0))).astype(np.float32)
    if fast_hash:
        # large populations: digests drawn directly (same distribution, no per-string hashing)
        dev = rng.integers(1, 2 ** 63, (n, pool), dtype=np.int64).astype(np.uint64)
        ip = rng.integers(1, 2 ** 63, (n, pool), dtype=np.int64).astype(np.uint64)
        fp = rng.integers(1, 2 ** 63, (n, pool), dtype=np.int64).astype(np.uint64)
    else:
        dev = np.stack([_digests(f"dev-{i}-", pool, SEED_DEVICE) for i in range(n)]) if n else np.zeros((0, pool), np.uint64)
        ip = (np.stack([_digests(f"10.{i % 250}.{i // 250 % 250}.", pool, SEED_IP) for i in range(n)]) if n
              else np.zeros((0, pool), np.uint64))
        fp = np.stack([_digests(f"fp-{i}-", pool, SEED_FINGERPRINT) for i in range(n)]) if n else np.zeros((0, pool), np.uint64)
    return Population(ids, b, ext, dev, ip, fp)


def make_requests(pop: Population, n: int, rng: np.random.Generator, now: int,
                  slots: Optional[np.ndarray] = None, spread_s: int = 0, hot_frac: float = 0.0,
                  unknown_frac: float = 0.0) -> np.ndarray:
    """REQREC rows. ``spread_s`` spreads ts over [now - spread_s, now]; ``hot_frac`` sends that
    fraction of traffic to 16 hot accounts (velocity / multi-device patterns)."""
    n_acc = len(pop.ids)
    r = np.zeros(n, REQREC)
    acc = rng.integers(0, n_acc, n)
    if hot_frac > 0:
        hot = rng.uniform(0, 1, n) < hot_frac
        acc[hot] = rng.integers(0, min(16, n_acc), hot.sum())
    r["slot"] = acc if slots is None else slots[acc]
    if unknown_frac > 0:
        r["slot"][rng.uniform(0, 1, n) < unknown_frac] = -1
    r["tx_type"] = rng.choice([0, 1, 2, 3], n, p=[0.25, 0.1, 0.55, 0.1])
    r["amount"] = np.maximum(1, rng.lognormal(7.5, 1.6, n)).astype(np.int64)
    P = pop.dev_pool.shape[1]
    pick = rng.integers(0, P, n)
    r["dev_hash"] = pop.dev_pool[acc, pick]
    r["ip_hash"] = pop.ip_pool[acc, rng.integers(0, P, n)]
    r["fp_hash"] = pop.fp_pool[acc, pick]
    # some requests without device / ip (empty strings upstream)
    r["dev_hash"][rng.uniform(0, 1, n) < 0.03] = 0
    r["ip_hash"][rng.uniform(0, 1, n) < 0.03] = 0
    if spread_s > 0:
        r["ts"] = now - np.sort(rng.integers(0, spread_s, n))[::-1]
    else:
        r["ts"] = now
    return r


def to_events(pop: Population, req: np.ndarray) -> List[TxEvent]:
    out = []
    for row in req:
        s = int(row["slot"])
        if s < 0:
            continue
        out.append(TxEvent(account=pop.ids[s], amount=int(row["amount"]), tx_type=int(row["tx_type"]),
                           device_hash=int(row["dev_hash"]), ip_hash=int(row["ip_hash"]), ts=int(row["ts"])))
    return out

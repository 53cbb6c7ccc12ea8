"""Golden feature store + feature extraction — the executable spec for the device kernels.

Reference semantics being reproduced (file:line under /root/reference):

* real-time window features: ``services/risk/internal/features/redis_store.go:60-116``
  (ZCOUNT ts >= now-60/-300/-3600 inclusive, PFCOUNT, GET last_tx / session_start),
* event application: ``redis_store.go:119-168`` (ZADD, INCRBY+EXPIRE 1h, PFADD+EXPIRE 24h,
  SET last_tx EX 7d, SETNX session_start + EXPIRE 30min),
* feature assembly: ``services/risk/internal/scoring/engine.go:326-417``,
* model input order + normalisation: ``services/risk/internal/ml/onnx_model.go:86-205``.

Deliberate, documented differences:
* Q8: 1h sum is an exact sliding sum over the tx ring (``sum_mode="sliding"``); the
  reference's INCRBY-with-refreshed-TTL is available as ``sum_mode="compat"``.
* Q9: the ring keeps duplicate (ts, amount) pairs; Redis' ZSET member dedupes them.
* Q1: ``log_transform="identity"`` reproduces the reference stub ``log1p(x)=x``.
* The ring holds the last ``ring_size`` events; window counts saturate at that size
  (default 256 >= the 200 normalisation cap of tx_count_1h).
* TTLs are evaluated against event/scoring timestamps (alive iff now < expiry).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from ..config import FeatureConfig, TX_TYPE_ID
from . import hll

F32 = np.float32

# proto FeatureVector field order (risk.proto:197-235); index i is model input i.
FEATURE_NAMES = [
    "tx_count_1m", "tx_count_5m", "tx_count_1h", "tx_sum_1h", "tx_avg_1h",
    "unique_devices_24h", "unique_ips_24h", "ip_country_changes_7d", "device_age_days",
    "account_age_days", "total_deposits", "total_withdrawals", "net_deposit",
    "deposit_count", "withdraw_count", "time_since_last_tx_sec", "session_duration_sec",
    "avg_bet_size", "win_rate", "is_vpn", "is_proxy", "is_tor", "disposable_email",
    "bonus_claim_count", "bonus_wager_completion_rate", "bonus_only_player",
]
MODEL_INPUT_NAMES = FEATURE_NAMES + ["tx_amount", "tx_type_deposit", "tx_type_withdraw", "tx_type_bet"]

IPF_VPN, IPF_PROXY, IPF_TOR = 1, 2, 4


@dataclass
class BatchFeatures:
    """Warehouse (ClickHouse) per-account aggregates, ``engine.go:127-140``."""
    total_deposits: int = 0
    total_withdrawals: int = 0
    deposit_count: int = 0
    withdraw_count: int = 0
    total_bets: int = 0
    total_wins: int = 0
    bet_count: int = 0
    win_count: int = 0
    avg_bet_size: float = 0.0
    account_created_at: int = 0   # unix seconds
    bonus_claim_count: int = 0
    bonus_wager_complete: float = 0.0


@dataclass
class AccountState:
    ring_ts: List[int]
    ring_amt: List[int]
    head: int = 0
    hll_dev: bytearray = field(default_factory=lambda: bytearray(hll.M))
    hll_dev_exp: int = 0
    hll_ip: bytearray = field(default_factory=lambda: bytearray(hll.M))
    hll_ip_exp: int = 0
    last_tx: int = 0
    last_tx_exp: int = 0
    session_start: int = 0
    session_exp: int = 0
    sum_compat: int = 0
    sum_compat_exp: int = 0
    batch: Optional[BatchFeatures] = None
    ext: Optional[np.ndarray] = None
    events: List[np.ndarray] = field(default_factory=list)
    last_event_ts: int = 0


@dataclass
class TxEvent:
    """``TransactionEvent`` (engine.go:143-150 / redis_store.go:47-54), ids pre-hashed."""
    account: str
    amount: int
    tx_type: int
    device_hash: int
    ip_hash: int
    ts: int


def minmax(x: F32, lo: float, hi: float) -> F32:
    """``minMaxScale`` (onnx_model.go:197-205), float32 arithmetic."""
    x = F32(x)
    if x < F32(lo):
        return F32(0.0)
    if x > F32(hi):
        return F32(1.0)
    return F32((x - F32(lo)) / (F32(hi) - F32(lo)))


def log_t(x, mode: str) -> F32:
    """``logTransform`` (onnx_model.go:187-195); identity mode = quirk Q1."""
    x = F32(x)
    if x <= 0:
        return F32(0.0)
    if mode == "identity":
        return x
    return F32(math.log1p(float(x)))


EVENT_DIM = 16


def encode_event(amount: int, tx_type: int, ts: int, prev_ts: int, new_device: bool,
                 new_ip: bool, dim: int = EVENT_DIM) -> np.ndarray:
    """Per-event feature row for the bonus-abuse GRU (cfg 5). Our design (no reference).

    [log1p(amount)/16, one-hot(type: deposit,withdraw,bet,win,refund,bonus), log1p(dt)/12,
     sin/cos(hour of day), new_device, new_ip, amount>=1e5, 1] -> 16 f32.
    """
    v = np.zeros(dim, dtype=F32)
    v[0] = F32(math.log1p(max(amount, 0)) / 16.0)
    if 0 <= tx_type < 6:
        v[1 + tx_type] = 1.0
    dt = ts - prev_ts if prev_ts > 0 and ts >= prev_ts else 0
    v[7] = F32(math.log1p(dt) / 12.0)
    hour = (ts % 86400) / 3600.0
    v[8] = F32(math.sin(2 * math.pi * hour / 24.0))
    v[9] = F32(math.cos(2 * math.pi * hour / 24.0))
    v[10] = 1.0 if new_device else 0.0
    v[11] = 1.0 if new_ip else 0.0
    v[12] = 1.0 if amount >= 100000 else 0.0
    v[13] = 1.0
    return v


class GoldenFeatureStore:
    """Per-account state with the reference's Redis semantics on a ring buffer."""

    def __init__(self, cfg: Optional[FeatureConfig] = None):
        self.cfg = cfg or FeatureConfig()
        self.accounts: Dict[str, AccountState] = {}
        self.ip_intel: Dict[int, int] = {}
        self.blacklist: Dict[int, int] = {}   # key hash -> expires_at (0 = never)

    def state(self, account: str) -> AccountState:
        st = self.accounts.get(account)
        if st is None:
            r = self.cfg.ring_size
            st = AccountState(ring_ts=[0] * r, ring_amt=[0] * r)
            self.accounts[account] = st
        return st

    # ------------------------------------------------------------ writes
    def set_batch(self, account: str, b: Optional[BatchFeatures]) -> None:
        st = self.state(account)
        if b is not None:
            b.avg_bet_size = float(F32(b.avg_bet_size))
            b.bonus_wager_complete = float(F32(b.bonus_wager_complete))
        st.batch = b

    def set_ext(self, account: str, ext: Optional[np.ndarray]) -> None:
        self.state(account).ext = None if ext is None else np.asarray(ext, dtype=F32)

    def apply(self, ev: TxEvent) -> None:
        """``UpdateRealTimeFeatures`` (redis_store.go:119-168) on the ring representation."""
        c = self.cfg
        st = self.state(ev.account)
        now = ev.ts
        st.ring_ts[st.head] = now
        st.ring_amt[st.head] = ev.amount
        st.head = (st.head + 1) % c.ring_size
        if now >= st.sum_compat_exp:
            st.sum_compat = 0
        st.sum_compat += ev.amount
        st.sum_compat_exp = now + c.sum_ttl_s
        new_dev = new_ip = False
        if ev.device_hash:
            if now >= st.hll_dev_exp:
                st.hll_dev = bytearray(hll.M)
            before = st.hll_dev[ev.device_hash & (hll.M - 1)]
            hll.add(st.hll_dev, ev.device_hash)
            new_dev = st.hll_dev[ev.device_hash & (hll.M - 1)] != before
            st.hll_dev_exp = now + c.hll_ttl_s
        if ev.ip_hash:
            if now >= st.hll_ip_exp:
                st.hll_ip = bytearray(hll.M)
            before = st.hll_ip[ev.ip_hash & (hll.M - 1)]
            hll.add(st.hll_ip, ev.ip_hash)
            new_ip = st.hll_ip[ev.ip_hash & (hll.M - 1)] != before
            st.hll_ip_exp = now + c.hll_ttl_s
        st.last_tx = now
        st.last_tx_exp = now + c.last_tx_ttl_s
        if now >= st.session_exp or st.session_start == 0:
            st.session_start = now
        st.session_exp = now + c.session_ttl_s
        st.events.append(encode_event(ev.amount, ev.tx_type, now, st.last_event_ts, new_dev, new_ip,
                                      c.event_dim))
        if len(st.events) > c.event_ring:
            st.events.pop(0)
        st.last_event_ts = now

    # ------------------------------------------------------------ reads
    def raw_features(self, account: str, now: int, ip_hash: int = 0) -> Dict[str, object]:
        """Assemble the 26-field FeatureVector (engine.go:326-417)."""
        c = self.cfg
        st = self.accounts.get(account)
        f: Dict[str, object] = {k: 0 for k in FEATURE_NAMES}
        for k in ("tx_avg_1h", "avg_bet_size", "win_rate", "bonus_wager_completion_rate"):
            f[k] = 0.0
        for k in ("is_vpn", "is_proxy", "is_tor", "disposable_email", "bonus_only_player"):
            f[k] = False
        partial = True
        if st is not None:
            c1 = c5 = c60 = 0
            s60 = 0
            for ts, amt in zip(st.ring_ts, st.ring_amt):
                if ts == 0:
                    continue
                if ts >= now - 60:
                    c1 += 1
                if ts >= now - 300:
                    c5 += 1
                if ts >= now - 3600:
                    c60 += 1
                    s60 += amt
            f["tx_count_1m"], f["tx_count_5m"], f["tx_count_1h"] = c1, c5, c60
            if c.sum_mode == "sliding":
                f["tx_sum_1h"] = s60
            else:
                f["tx_sum_1h"] = st.sum_compat if now < st.sum_compat_exp else 0
            f["unique_devices_24h"] = hll.count(st.hll_dev) if now < st.hll_dev_exp else 0
            f["unique_ips_24h"] = hll.count(st.hll_ip) if now < st.hll_ip_exp else 0
            if st.last_tx > 0 and now < st.last_tx_exp:
                f["time_since_last_tx_sec"] = now - st.last_tx
            if st.session_start > 0 and now < st.session_exp:
                f["session_duration_sec"] = now - st.session_start
            b = st.batch
            if b is not None:
                partial = False
                f["total_deposits"] = b.total_deposits
                f["total_withdrawals"] = b.total_withdrawals
                f["net_deposit"] = b.total_deposits - b.total_withdrawals
                f["deposit_count"] = b.deposit_count
                f["withdraw_count"] = b.withdraw_count
                f["avg_bet_size"] = float(F32(b.avg_bet_size))
                d = now - b.account_created_at
                f["account_age_days"] = int(d / 86400) if d >= 0 else -int((-d) / 86400)
                f["bonus_claim_count"] = b.bonus_claim_count
                f["bonus_wager_completion_rate"] = float(F32(b.bonus_wager_complete))
                if b.bet_count > 0:
                    f["win_rate"] = float(F32(b.win_count / b.bet_count))
                f["bonus_only_player"] = b.bonus_claim_count > 3 and b.total_deposits < 5000
        if ip_hash:
            fl = self.ip_intel.get(ip_hash, 0)
            f["is_vpn"] = bool(fl & IPF_VPN)
            f["is_proxy"] = bool(fl & IPF_PROXY)
            f["is_tor"] = bool(fl & IPF_TOR)
        if f["tx_count_1h"] > 0:
            f["tx_avg_1h"] = float(F32(f["tx_sum_1h"] / f["tx_count_1h"]))
        f["_partial"] = partial
        return f

    def blacklisted(self, hashes, now: int) -> bool:
        for h in hashes:
            if h and h in self.blacklist:
                exp = self.blacklist[h]
                if exp == 0 or now < exp:
                    return True
        return False

    def event_history(self, account: str) -> np.ndarray:
        c = self.cfg
        out = np.zeros((c.event_ring, c.event_dim), dtype=F32)
        st = self.accounts.get(account)
        if st is not None and st.events:
            ev = np.stack(st.events)
            out[c.event_ring - len(ev):] = ev   # oldest first, right-aligned
        return out


def model_input(f: Dict[str, object], amount: int, tx_type: int, mode: str, width: int = 30,
                ext: Optional[np.ndarray] = None) -> np.ndarray:
    """``ToSlice`` + ``Normalize`` (onnx_model.go:133-184) into a fresh buffer (quirk Q2)."""
    x = np.zeros(width, dtype=F32)
    x[0] = minmax(f["tx_count_1m"], 0, 20)
    x[1] = minmax(f["tx_count_5m"], 0, 50)
    x[2] = minmax(f["tx_count_1h"], 0, 200)
    x[3] = log_t(f["tx_sum_1h"], mode)
    x[4] = F32(f["tx_avg_1h"])
    x[5] = minmax(f["unique_devices_24h"], 0, 10)
    x[6] = minmax(f["unique_ips_24h"], 0, 20)
    x[7] = F32(f["ip_country_changes_7d"])
    x[8] = F32(f["device_age_days"])
    x[9] = minmax(f["account_age_days"], 0, 365)
    x[10] = log_t(f["total_deposits"], mode)
    x[11] = log_t(f["total_withdrawals"], mode)
    x[12] = F32(f["net_deposit"])
    x[13] = F32(f["deposit_count"])
    x[14] = F32(f["withdraw_count"])
    x[15] = minmax(f["time_since_last_tx_sec"], 0, 86400)
    x[16] = F32(f["session_duration_sec"])
    x[17] = F32(f["avg_bet_size"])
    x[18] = F32(f["win_rate"])
    x[19] = F32(1.0 if f["is_vpn"] else 0.0)
    x[20] = F32(1.0 if f["is_proxy"] else 0.0)
    x[21] = F32(1.0 if f["is_tor"] else 0.0)
    x[22] = F32(1.0 if f["disposable_email"] else 0.0)
    x[23] = F32(f["bonus_claim_count"])
    x[24] = F32(f["bonus_wager_completion_rate"])
    x[25] = F32(1.0 if f["bonus_only_player"] else 0.0)
    x[26] = log_t(amount, mode)
    x[27] = F32(1.0 if tx_type == TX_TYPE_ID["deposit"] else 0.0)
    x[28] = F32(1.0 if tx_type == TX_TYPE_ID["withdraw"] else 0.0)
    x[29] = F32(1.0 if tx_type == TX_TYPE_ID["bet"] else 0.0)
    if width > 30:
        if ext is not None:
            x[30:] = np.asarray(ext, dtype=F32)[: width - 30]
    return x

"""HBM-resident feature store shard (one per GPU) — replaces the reference's Redis store.

Layout (structure-of-arrays, one row per account slot, sized for 288 GB HBM3E):

=================  ==========================  ==================================================
tensor             shape / dtype               reference equivalent (redis_store.go)
=================  ==========================  ==================================================
``ring_ts``        [C, R] int32 (unix s)       ZSET ``features:<id>:tx_history`` scores (:25-35)
``ring_amt``       [C, R] int64 (cents)        ZSET members ``ts:amount``
``hll``            [C, 2, 256] uint8           PFADD ``devices:24h`` / ``ips:24h`` (:140-152)
``rt``             [C] AcctRT (64 B)           last_tx / session_start / tx_sum TTL keys (:136-162)
``batch``          [C] AcctBatch (80 B)        ClickHouse batch features (engine.go:127-140)
``ext``            [C, W-30] float32           extended warehouse features (model width > 30)
``ev``             [C, 100, 16] bf16           event history for the bonus-abuse GRU (cfg 5)
=================  ==========================  ==================================================

With R = 256 a slot costs ~4.5 KB (+3.2 KB with the GRU event ring), i.e. ~35-60 M accounts
per MI355X at 60 % of HBM. The host never mirrors the per-event state (the GPU is the
store); :meth:`snapshot` / :meth:`restore` give durability (the reference relied on Redis
AOF, ``deploy/docker-compose.yml:29``).
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import numpy as np

from ..config import FeatureConfig
from ..golden.hll import linear_count as hll_linear_count
from ..layouts import ACCTBATCH, ACCTRT
from .tables import Blacklist, IPIntel

DEDUP_LIST = 64  # events per account per batch kept in a dedup list (launch.h DEDUP_LIST)
DEDUP_REGIONS = 9  # 8 scorer ring regions (by batch seq) + 1 standalone ingestion region (launch.h)
DEDUP_STANDALONE = 8


def dedup_hot_cap(n_max: int) -> int:
    """Hot-account pairs per region (update.h dedup_hot_cap)."""
    return n_max // (DEDUP_LIST + 1) + 1


def dedup_region_size(cap: int, n_max: int) -> int:
    """int32 words of one dedup region (update.h dedup_region_size)."""
    return (5 * cap + cap * DEDUP_LIST + 2 * n_max + 4 + 2 * dedup_hot_cap(n_max) + 15) & ~15


def _pow2_at_least(n: int) -> int:
    c = 1
    while c < n:
        c <<= 1
    return c


class DeviceFeatureStore:
    def __init__(self, capacity: int, fcfg: FeatureConfig, device="cuda", events: bool = True,
                 blacklist: Optional[Blacklist] = None, ipintel: Optional[IPIntel] = None,
                 max_events: int = 8192):
        import torch
        self.torch = torch
        self.capacity = int(capacity)
        self.cfg = fcfg
        d = torch.device(device)
        if d.type == "cuda" and d.index is None:
            d = torch.device("cuda", torch.cuda.current_device())
        self.device = d
        C, R = self.capacity, fcfg.ring_size
        z = dict(device=self.device)
        self.ring_ts = torch.zeros((C, R), dtype=torch.int32, **z)
        self.ring_amt = torch.zeros((C, R), dtype=torch.int64, **z)
        self.hll = torch.zeros((C, 512), dtype=torch.uint8, **z)
        self.rt = torch.zeros((C, ACCTRT.itemsize // 4), dtype=torch.int32, **z)
        self.batch = torch.zeros((C, ACCTBATCH.itemsize // 4), dtype=torch.int32, **z)
        self.ext_width = fcfg.width - 30
        self.ext = torch.zeros((C, max(self.ext_width, 1)), dtype=torch.float32, **z)
        self.events = events
        self.ev = (torch.zeros((C, fcfg.event_ring, fcfg.event_dim), dtype=torch.int16, **z)
                   if events else None)
        self.blacklist = blacklist or Blacklist()
        self.ipintel = ipintel or IPIntel()
        self.bl_keys = torch.zeros(self.blacklist.table.cap, dtype=torch.int64, **z)
        self.bl_exp = torch.zeros(self.blacklist.table.cap, dtype=torch.int32, **z)
        self.ip_keys = torch.zeros(self.ipintel.table.cap, dtype=torch.int64, **z)
        self.ip_flags = torch.zeros(self.ipintel.table.cap, dtype=torch.int32, **z)
        self._bl_version = -1
        self._ip_version = -1
        # HLL linear-counting table floor(m ln(m / V) + 0.5), V = zero registers (golden/hll.py)
        self.hll_lc = torch.tensor([0] + [hll_linear_count(v) for v in range(1, 257)], dtype=torch.int32,
                                   device=self.device)
        self.max_events = int(max_events)
        # dedup scratch for ordered score-then-update: scorer ring regions + standalone
        self.dmax = self.max_events
        self.dcap = _pow2_at_least(2 * self.max_events)
        # per region (csrc/kernels/update.h dedup_region): keys/first/count/fill/done [cap],
        # per-account event lists [cap][DEDUP_LIST], multi-account list [dmax], 4 counters, the
        # batch's row -> applied account slot array [dmax], the hot-account list [hot_cap] pairs
        # (update.h dedup_region_size; checked against the extension by layouts.check_layouts)
        self.dregion = dedup_region_size(self.dcap, self.dmax)
        self.dbuf = torch.empty(DEDUP_REGIONS * self.dregion, dtype=torch.int32, **z)
        self.reset_dedup()

    def reset_dedup(self) -> None:
        r = self.dbuf.view(DEDUP_REGIONS, self.dregion)
        r[:, : self.dcap].fill_(-1)                            # keys
        r[:, self.dcap: 2 * self.dcap].fill_(0x7FFFFFFF)        # first
        r[:, 2 * self.dcap: 5 * self.dcap].zero_()              # count, fill, done
        r[:, (5 + DEDUP_LIST) * self.dcap + self.dmax:].zero_()  # counters

    # ------------------------------------------------------------------ sizing
    def bytes_per_account(self) -> int:
        b = self.ring_ts[0].numel() * 4 + self.ring_amt[0].numel() * 8 + 512
        b += ACCTRT.itemsize + ACCTBATCH.itemsize + self.ext[0].numel() * 4
        if self.ev is not None:
            b += self.ev[0].numel() * 2
        return b

    def memory_bytes(self) -> int:
        return self.bytes_per_account() * self.capacity

    @staticmethod
    def _per_account(fcfg: FeatureConfig, events: bool = True) -> int:
        per = fcfg.ring_size * 12 + 512 + ACCTRT.itemsize + ACCTBATCH.itemsize + max(fcfg.width - 30, 1) * 4
        if events:
            per += fcfg.event_ring * fcfg.event_dim * 2
        return per

    @staticmethod
    def capacity_for(fcfg: FeatureConfig, hbm_bytes: int, fraction: float = 0.6, events: bool = True) -> int:
        return int(hbm_bytes * fraction // DeviceFeatureStore._per_account(fcfg, events))

    @staticmethod
    def estimate_bytes(fcfg: FeatureConfig, capacity: int, events: bool = True) -> int:
        """HBM a store of ``capacity`` accounts takes (per-account arrays; tables and dedup
        scratch are small)."""
        return DeviceFeatureStore._per_account(fcfg, events) * int(capacity)

    # ------------------------------------------------------------------ writes
    def set_batch_features(self, slots: np.ndarray, rows: np.ndarray) -> None:
        """Bulk-load warehouse aggregates (the hourly batch job, risk main.go:227-236)."""
        rows = np.ascontiguousarray(rows, dtype=ACCTBATCH)
        t = self.torch.from_numpy(rows.view(np.int32).reshape(len(rows), -1).copy())
        idx = self.torch.as_tensor(np.asarray(slots, np.int64), device=self.device)
        self.batch.index_copy_(0, idx, t.to(self.device))

    def set_ext(self, slots: np.ndarray, ext: np.ndarray) -> None:
        if self.ext_width <= 0:
            return
        idx = self.torch.as_tensor(np.asarray(slots, np.int64), device=self.device)
        self.ext.index_copy_(0, idx, self.torch.as_tensor(np.asarray(ext, np.float32), device=self.device))

    def reset_accounts(self, slots) -> None:
        """``DeleteAccountFeatures`` (redis_store.go:230-240) for the given slots."""
        idx = self.torch.as_tensor(np.asarray(slots, np.int64), device=self.device)
        for t in (self.ring_ts, self.ring_amt, self.hll, self.rt, self.batch, self.ext):
            t.index_fill_(0, idx, 0)
        if self.ev is not None:
            self.ev.index_fill_(0, idx, 0)

    def sync_tables(self) -> bool:
        """Upload blacklist / ip-intel tables if the host copy changed. Returns True if so."""
        changed = False
        bt = self.blacklist.table
        if bt.version != self._bl_version:
            self.bl_keys.copy_(self.torch.from_numpy(bt.keys.view(np.int64).copy()))
            self.bl_exp.copy_(self.torch.from_numpy(bt.vals.view(np.int32).copy()))
            self._bl_version = bt.version
            changed = True
        it = self.ipintel.table
        if it.version != self._ip_version:
            self.ip_keys.copy_(self.torch.from_numpy(it.keys.view(np.int64).copy()))
            self.ip_flags.copy_(self.torch.from_numpy(it.vals.view(np.int32).copy()))
            self._ip_version = it.version
            changed = True
        return changed

    def table_params(self) -> Dict[str, int]:
        return dict(bl_mask=self.blacklist.table.mask, bl_max_probe=max(self.blacklist.table.max_probe, 1),
                    ip_mask=self.ipintel.table.mask, ip_max_probe=max(self.ipintel.table.max_probe, 1))

    # ------------------------------------------------------------------ reads (debug / GetFeatures)
    def read_rt(self, slot: int) -> np.ndarray:
        return self.rt[slot].cpu().numpy().view(ACCTRT)[0]

    def read_batch(self, slot: int) -> np.ndarray:
        return self.batch[slot].cpu().numpy().view(ACCTBATCH)[0]

    # ------------------------------------------------------------------ durability
    def snapshot(self, path: str, n_used: Optional[int] = None) -> None:
        """Versioned snapshot of the first ``n_used`` slots (device -> host -> file)."""
        n = self.capacity if n_used is None else int(n_used)
        arrs = {
            # version 2: AcctRT carries the cached HLL estimates (version 1 files get them rebuilt)
            "version": np.array([2], np.int32),
            "ring_size": np.array([self.cfg.ring_size], np.int32),
            "ring_ts": self.ring_ts[:n].cpu().numpy(), "ring_amt": self.ring_amt[:n].cpu().numpy(),
            "hll": self.hll[:n].cpu().numpy(), "rt": self.rt[:n].cpu().numpy(),
            "batch": self.batch[:n].cpu().numpy(), "ext": self.ext[:n].cpu().numpy(),
        }
        if self.ev is not None:
            arrs["ev"] = self.ev[:n].cpu().numpy()
        tmp = path + ".tmp.npz"
        np.savez(tmp, **arrs)
        os.replace(tmp, path if path.endswith(".npz") else path)

    def restore(self, path: str) -> int:
        with np.load(path, allow_pickle=False) as z:
            if int(z["ring_size"][0]) != self.cfg.ring_size:
                raise ValueError("snapshot ring size differs from the configured ring size")
            n = z["ring_ts"].shape[0]
            if n > self.capacity:
                raise ValueError("snapshot larger than the store capacity")
            rt = z["rt"].copy()
            if int(z["version"][0]) < 2 and n:  # written before AcctRT cached the HLL estimates
                from ..golden.hll import refresh_cached_counts
                v = rt.reshape(n, -1).view(ACCTRT).reshape(-1)
                refresh_cached_counts(z["hll"], v)
            for name in ("ring_ts", "ring_amt", "hll", "batch", "ext"):
                getattr(self, name)[:n].copy_(self.torch.from_numpy(z[name]))
            self.rt[:n].copy_(self.torch.from_numpy(rt))
            if self.ev is not None and "ev" in z:
                self.ev[:n].copy_(self.torch.from_numpy(z["ev"]))
        return n

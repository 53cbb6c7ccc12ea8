"""numpy structured dtypes mirroring ``csrc/include/records.h`` (host <-> device records).

``check_layouts()`` compares the itemsizes with the ``sizeof`` values exported by the
compiled extension, so a drift between C and Python fails loudly.
"""
from __future__ import annotations

import numpy as np

from .config import Config, ScoringConfig

FEATREC = np.dtype([
    ("tx_count_1m", "<i4"), ("tx_count_5m", "<i4"), ("tx_count_1h", "<i4"), ("flags", "<i4"),
    ("tx_sum_1h", "<i8"), ("tx_avg_1h", "<f4"), ("unique_devices_24h", "<i4"),
    ("unique_ips_24h", "<i4"), ("ip_country_changes_7d", "<i4"), ("device_age_days", "<i4"),
    ("account_age_days", "<i4"), ("total_deposits", "<i8"), ("total_withdrawals", "<i8"),
    ("net_deposit", "<i8"), ("deposit_count", "<i4"), ("withdraw_count", "<i4"),
    ("time_since_last_tx_sec", "<i4"), ("session_duration_sec", "<i4"), ("avg_bet_size", "<f4"),
    ("win_rate", "<f4"), ("bonus_claim_count", "<i4"), ("bonus_wager_completion_rate", "<f4"),
    ("tx_type", "<i4"), ("slot", "<i4"), ("amount", "<i8"), ("rule_reasons", "<i4"),
    ("rule_score", "<i4"),
])
FR_VPN, FR_PROXY, FR_TOR, FR_DISPOSABLE, FR_BONUS_ONLY, FR_BLACKLISTED, FR_PARTIAL = 1, 2, 4, 8, 16, 32, 64
FR_NOT_OWNED = 128

ACCTRT = np.dtype([
    ("hll_dev_exp", "<u4"), ("hll_ip_exp", "<u4"), ("last_tx", "<u4"), ("last_tx_exp", "<u4"),
    ("session_start", "<u4"), ("session_exp", "<u4"), ("sum_exp", "<u4"), ("last_event_ts", "<u4"),
    ("sum_compat", "<i8"), ("ring_head", "<i4"), ("ev_head", "<i4"), ("ev_count", "<i4"),
    ("hll_dev_n", "<i4"), ("hll_ip_n", "<i4"), ("pad", "<i4"),
])

ACCTBATCH = np.dtype([
    ("total_deposits", "<i8"), ("total_withdrawals", "<i8"), ("total_bets", "<i8"),
    ("total_wins", "<i8"), ("account_created_at", "<i8"), ("deposit_count", "<i4"),
    ("withdraw_count", "<i4"), ("bet_count", "<i4"), ("win_count", "<i4"), ("avg_bet_size", "<f4"),
    ("bonus_claim_count", "<i4"), ("bonus_wager_complete", "<f4"), ("present", "<i4"),
    ("pad", "<i4", (2,)),
])

SCORECFG = np.dtype([
    ("block_threshold", "<i4"), ("review_threshold", "<i4"), ("max_tx_per_minute", "<i4"),
    ("new_account_days", "<i4"), ("large_deposit_amount", "<i8"), ("max_devices_per_day", "<i4"),
    ("max_ips_per_day", "<i4"), ("ml_weight", "<f8"), ("rule_weight", "<f8"),
    ("ml_high_risk", "<f8"), ("ml_error_score", "<f8"),
    ("w_high_velocity", "<i4"), ("w_new_account_large_tx", "<i4"), ("w_multiple_devices", "<i4"),
    ("w_ip_country_mismatch", "<i4"), ("w_vpn", "<i4"), ("w_rapid_deposit_withdraw", "<i4"),
    ("w_bonus_abuse", "<i4"), ("w_known_fraudster", "<i4"),
    ("model_kind", "<i4"), ("ml_col", "<i4"), ("ml_stride", "<i4"), ("log_identity", "<i4"),
    ("sum_compat", "<i4"), ("session_ttl", "<i4"), ("last_tx_ttl", "<i4"), ("hll_ttl", "<i4"),
    ("sum_ttl", "<i4"), ("bl_mask", "<i4"), ("bl_max_probe", "<i4"), ("ip_mask", "<i4"),
    ("ip_max_probe", "<i4"), ("ext_width", "<i4"), ("owner_filter", "<i4"), ("my_rank", "<i4"),
    ("pad", "<i4", (4,)),
])

REQREC = np.dtype([
    ("slot", "<i4"), ("tx_type", "<i4"), ("amount", "<i8"), ("dev_hash", "<u8"),
    ("fp_hash", "<u8"), ("ip_hash", "<u8"), ("ts", "<i8"),
])

BATCHHDR = np.dtype([("n", "<i4"), ("seq", "<i4"), ("now", "<i8")])

MODEL_NONE, MODEL_HEURISTIC, MODEL_OUTPUT = 0, 1, 2


def check_layouts(mod) -> None:
    for name, dt in (("SCORECFG", SCORECFG), ("FEATREC", FEATREC), ("ACCTRT", ACCTRT),
                     ("ACCTBATCH", ACCTBATCH), ("REQREC", REQREC)):
        want = getattr(mod, "SIZEOF_" + name)
        if dt.itemsize != want:
            raise RuntimeError(f"layout drift: {name} is {dt.itemsize} B in Python, {want} B in C")
    from .features.device_store import DEDUP_LIST, DEDUP_REGIONS, dedup_region_size
    if (getattr(mod, "DEDUP_LIST", DEDUP_LIST), getattr(mod, "DEDUP_REGIONS", DEDUP_REGIONS)) != (DEDUP_LIST,
                                                                                                 DEDUP_REGIONS):
        raise RuntimeError("layout drift: dedup scratch layout differs between Python and C")
    f = getattr(mod, "dedup_region_size", None)
    if f is not None and any(f(c, n) != dedup_region_size(c, n) for c, n in ((16384, 8192), (1024, 300), (64, 1))):
        raise RuntimeError("layout drift: dedup region size differs between Python and C")


def score_cfg(cfg: Config, model_kind: int, ml_col: int = 0, ml_stride: int = 1,
              bl_mask: int = 0, bl_max_probe: int = 0, ip_mask: int = 0, ip_max_probe: int = 0,
              sc: ScoringConfig = None, owner_filter: bool = False, my_rank: int = 0) -> np.ndarray:
    sc = sc or cfg.scoring
    f = cfg.features
    w = sc.weights
    c = np.zeros(1, SCORECFG)
    c["block_threshold"] = sc.block_threshold
    c["review_threshold"] = sc.review_threshold
    c["max_tx_per_minute"] = sc.max_tx_per_minute
    c["new_account_days"] = sc.new_account_days
    c["large_deposit_amount"] = sc.large_deposit_amount
    c["max_devices_per_day"] = sc.max_devices_per_day
    c["max_ips_per_day"] = sc.max_ips_per_day
    c["ml_weight"] = sc.ml_weight
    c["rule_weight"] = sc.rule_weight
    c["ml_high_risk"] = sc.ml_high_risk_threshold
    c["ml_error_score"] = sc.ml_error_score
    c["w_high_velocity"] = w.high_velocity
    c["w_new_account_large_tx"] = w.new_account_large_tx
    c["w_multiple_devices"] = w.multiple_devices
    c["w_ip_country_mismatch"] = w.ip_country_mismatch
    c["w_vpn"] = w.vpn_detected
    c["w_rapid_deposit_withdraw"] = w.rapid_deposit_withdraw
    c["w_bonus_abuse"] = w.bonus_abuse
    c["w_known_fraudster"] = w.known_fraudster
    c["model_kind"] = model_kind
    c["ml_col"] = ml_col
    c["ml_stride"] = ml_stride
    c["log_identity"] = 1 if f.log_transform == "identity" else 0
    c["sum_compat"] = 1 if f.sum_mode == "compat" else 0
    c["session_ttl"] = f.session_ttl_s
    c["last_tx_ttl"] = f.last_tx_ttl_s
    c["hll_ttl"] = f.hll_ttl_s
    c["sum_ttl"] = f.sum_ttl_s
    c["bl_mask"] = bl_mask
    c["bl_max_probe"] = bl_max_probe
    c["ip_mask"] = ip_mask
    c["ip_max_probe"] = ip_max_probe
    c["ext_width"] = f.width - 30
    c["owner_filter"] = 1 if owner_filter else 0
    c["my_rank"] = my_rank
    return c


def unpack_results(res: np.ndarray):
    """ResultRec[n] (uint32 [n,2]) -> dict of columns."""
    res = np.ascontiguousarray(res).view(np.uint32).reshape(-1, 2)
    p = res[:, 0]
    return {
        "score": (p & 0xFF).astype(np.int32),
        "rule_score": ((p >> 8) & 0xFF).astype(np.int32),
        "action": ((p >> 16) & 0x3).astype(np.int32),
        "ml_present": ((p >> 18) & 1).astype(bool),
        "reasons": (p >> 20).astype(np.int32),
        "ml": res[:, 1].view(np.float32).copy(),
    }


def pack_results(score, rule_score, action, reasons, ml, ml_present) -> np.ndarray:
    """Columns -> ResultRec[n] (uint32 [n,2]); inverse of :func:`unpack_results`."""
    n = len(score)
    out = np.zeros((n, 2), np.uint32)
    out[:, 0] = ((np.asarray(score, np.uint32) & 0xFF) | ((np.asarray(rule_score, np.uint32) & 0xFF) << 8)
                 | ((np.asarray(action, np.uint32) & 0x3) << 16)
                 | (np.asarray(ml_present, np.uint32) << 18) | (np.asarray(reasons, np.uint32) << 20))
    out[:, 1] = np.asarray(ml, np.float32).view(np.uint32)
    return out

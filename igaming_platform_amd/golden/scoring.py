"""Golden rules, heuristic model, ensemble and action — spec for the ``rules_ensemble`` kernel.

* Rules 1-8 + cap: ``services/risk/internal/scoring/engine.go:420-483`` (weights :246-257).
* Ensemble + action: ``engine.go:276-310`` (truncating int(), cap 100, block >= / review >=).
* Heuristic model (``mockPredict``, the reference's no-model fallback):
  ``services/risk/internal/ml/onnx_model.go:258-308`` — evaluated in float64 with the
  same addition order so scores match bit-for-bit; comparisons are on float32 inputs
  (Go compares float32 fields against untyped constants converted to float32).
* ``ScoreWithExplanation``: ``engine.go:507-543``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from ..config import (ACTION_APPROVE, ACTION_BLOCK, ACTION_NAMES, ACTION_REVIEW, REASON_BIT,
                      REASON_CODES, ScoringConfig, TX_TYPE_ID)

F32 = np.float32


@dataclass
class ScoreResult:
    score: int
    action: int
    reasons: List[str]
    rule_score: int
    ml_score: float
    features: Dict[str, object] = field(default_factory=dict)
    response_time_ms: int = 0

    @property
    def reason_mask(self) -> int:
        m = 0
        for r in self.reasons:
            m |= 1 << REASON_BIT[r]
        return m


def apply_rules(cfg: ScoringConfig, f: Dict[str, object], amount: int, tx_type: int,
                blacklisted: bool):
    w = cfg.weights
    total = 0
    reasons: List[str] = []
    if f["tx_count_1m"] > cfg.max_tx_per_minute:
        total += w.high_velocity
        reasons.append("HIGH_VELOCITY")
    if f["account_age_days"] < cfg.new_account_days and amount > cfg.large_deposit_amount:
        total += w.new_account_large_tx
        reasons.append("NEW_ACCOUNT_LARGE_TX")
    if f["unique_devices_24h"] > cfg.max_devices_per_day:
        total += w.multiple_devices
        reasons.append("MULTIPLE_DEVICES")
    if f["unique_ips_24h"] > cfg.max_ips_per_day:
        total += w.ip_country_mismatch
        reasons.append("IP_COUNTRY_MISMATCH")
    if f["is_vpn"] or f["is_proxy"] or f["is_tor"]:
        total += w.vpn_detected
        reasons.append("VPN_DETECTED")
    if f["time_since_last_tx_sec"] < 300 and tx_type == TX_TYPE_ID["withdraw"]:
        td = int(f["total_deposits"])
        # Go int64: total_deposits*80/100 truncates toward zero
        q = abs(td * 80) // 100
        lim = q if td * 80 >= 0 else -q
        if f["deposit_count"] > 0 and int(f["total_withdrawals"]) > lim:
            total += w.rapid_deposit_withdraw
            reasons.append("RAPID_DEPOSIT_WITHDRAW")
    if f["bonus_only_player"]:
        total += w.bonus_abuse
        reasons.append("BONUS_ABUSE")
    if blacklisted:
        total += w.known_fraudster
        reasons.append("KNOWN_FRAUDSTER")
    return min(total, 100), reasons


def heuristic_predict(x: np.ndarray) -> float:
    """``mockPredict`` on the normalised model input (float64 accumulation, same order)."""
    x = np.asarray(x, dtype=F32)
    s = 0.0
    if x[0] > F32(0.5):
        s += 0.2
    if x[2] > F32(0.5):
        s += 0.15
    if x[5] > F32(0.3):
        s += 0.15
    if x[6] > F32(0.25):
        s += 0.1
    if x[19] > 0 or x[20] > 0:
        s += 0.15
    if x[21] > 0:
        s += 0.25
    if x[9] < F32(0.02) and x[26] > F32(0.5):
        s += 0.2
    if x[25] > 0:
        s += 0.15
    if x[15] < F32(0.01) and x[28] > 0:
        if x[11] > F32(x[10] * F32(0.8)):
            s += 0.2
    return min(s, 1.0)


def ensemble(cfg: ScoringConfig, rule_score: int, reasons: List[str], ml: Optional[float],
             block: Optional[int] = None, review: Optional[int] = None):
    """Returns (score, action, reasons, ml). ``ml=None`` means no model configured."""
    reasons = list(reasons)
    if ml is None:
        mlv = 0.0
    else:
        mlv = float(ml)
        if mlv > cfg.ml_high_risk_threshold:
            reasons.append("ML_HIGH_RISK")
    final = int(cfg.rule_weight * float(rule_score) + cfg.ml_weight * (mlv * 100.0))
    final = min(final, 100)
    b = cfg.block_threshold if block is None else block
    r = cfg.review_threshold if review is None else review
    if final >= b:
        action = ACTION_BLOCK
    elif final >= r:
        action = ACTION_REVIEW
    else:
        action = ACTION_APPROVE
    return final, action, reasons, mlv


def clamp01_f32(v: float) -> float:
    """ORT output clamp (onnx_model.go:246-252) on a float32 result, widened to float64."""
    v = F32(v)
    if v < 0:
        v = F32(0.0)
    if v > 1:
        v = F32(1.0)
    return float(v)


def reasons_from_mask(mask: int) -> List[str]:
    return [REASON_CODES[i] for i in range(len(REASON_CODES)) if mask >> i & 1]


def explain(cfg: ScoringConfig, res: ScoreResult) -> str:
    """Human-readable breakdown (``ScoreWithExplanation``, engine.go:507-543)."""
    w = cfg.weights.by_reason()
    f = res.features
    lines = [
        "",
        "Fraud Score Analysis",
        "====================",
        f"Final Score: {res.score}/100",
        f"Action: {ACTION_NAMES.get(res.action, '?')}",
        f"Response Time: {res.response_time_ms}ms",
        "",
        f"Rule Contribution: {res.rule_score}",
        f"ML Contribution: {res.ml_score:.2f} ({res.ml_score:.2f} * 100)",
        "",
        "Triggered Rules:",
    ]
    for r in res.reasons:
        lines.append(f"  - {r} (+{w.get(r, 0)})")
    lines += [
        "",
        "Key Features:",
        f"  - Transaction velocity (1h): {f.get('tx_count_1h', 0)} txs, sum: {f.get('tx_sum_1h', 0)}",
        f"  - Unique devices (24h): {f.get('unique_devices_24h', 0)}",
        f"  - Account age: {f.get('account_age_days', 0)} days",
        f"  - VPN/Proxy: {'true' if (f.get('is_vpn') or f.get('is_proxy')) else 'false'}",
        f"  - Bonus abuse signal: {'true' if f.get('bonus_only_player') else 'false'}",
        "",
    ]
    return "\n".join(lines)

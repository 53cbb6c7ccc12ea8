"""Golden LTV / churn / segment / next-best-action — spec for the ``ltv_segment`` kernel.

Reproduces ``services/risk/internal/prediction/ltv.go:113-382`` (``LTVPredictor``) and the
simpler ``LTVModel`` formula of ``services/risk/internal/ml/onnx_model.go:405-490``.
All arithmetic is float64 like the Go code.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, fields
from typing import List

SEGMENTS = ["unspecified", "vip", "high", "medium", "low", "churning"]  # risk.proto:122-129
SEG_VIP, SEG_HIGH, SEG_MEDIUM, SEG_LOW, SEG_CHURNING = 1, 2, 3, 4, 5

NBA_CODES = [
    "NO_ACTION", "SEND_WINBACK_BONUS", "SEND_ENGAGEMENT_EMAIL", "VIP_MANAGER_CALL",
    "EXCLUSIVE_EVENT_INVITE", "ASSIGN_VIP_MANAGER", "RETENTION_BONUS", "LOYALTY_REWARD",
    "SUGGEST_BONUS", "RECOMMEND_NEW_GAMES", "STANDARD_PROMOTION", "ONBOARDING_GUIDE",
    "SMALL_DEPOSIT_BONUS",
]
NBA_ID = {n: i for i, n in enumerate(NBA_CODES)}

# Device column order of the player-feature table (ltv.go:38-78, numeric fields only).
PLAYER_COLUMNS = [
    "days_since_registration", "days_since_last_deposit", "days_since_last_bet",
    "total_active_days", "sessions_per_week", "avg_session_duration", "total_deposits",
    "total_withdrawals", "net_revenue", "avg_deposit_amount", "deposit_frequency",
    "largest_deposit", "total_bets", "total_wins", "bet_count", "win_rate", "avg_bet_size",
    "games_played", "bonuses_claimed", "bonus_wagering_completed", "bonus_conversion_rate",
    "push_enabled", "email_opt_in", "has_vip_manager", "support_tickets",
]


@dataclass
class PlayerFeatures:
    days_since_registration: int = 0
    days_since_last_deposit: int = 0
    days_since_last_bet: int = 0
    total_active_days: int = 0
    sessions_per_week: float = 0.0
    avg_session_duration: float = 0.0
    total_deposits: float = 0.0
    total_withdrawals: float = 0.0
    net_revenue: float = 0.0
    avg_deposit_amount: float = 0.0
    deposit_frequency: float = 0.0
    largest_deposit: float = 0.0
    total_bets: float = 0.0
    total_wins: float = 0.0
    bet_count: int = 0
    win_rate: float = 0.0
    avg_bet_size: float = 0.0
    games_played: int = 0
    bonuses_claimed: int = 0
    bonus_wagering_completed: int = 0
    bonus_conversion_rate: float = 0.0
    push_enabled: bool = False
    email_opt_in: bool = False
    has_vip_manager: bool = False
    support_tickets: int = 0
    country: str = ""
    payment_method: str = ""
    favorite_game_category: str = ""

    def row(self) -> List[float]:
        return [float(getattr(self, c)) for c in PLAYER_COLUMNS]

    @classmethod
    def from_row(cls, row) -> "PlayerFeatures":
        kw = {}
        types = {f.name: f.type for f in fields(cls)}
        for c, v in zip(PLAYER_COLUMNS, row):
            t = types[c]
            if t in ("int", int):
                kw[c] = int(v)
            elif t in ("bool", bool):
                kw[c] = bool(v)
            else:
                kw[c] = float(v)
        return cls(**kw)


@dataclass
class LTVPrediction:
    predicted_ltv: float
    segment: int
    churn_risk: float
    survival_days: int
    confidence: float
    next_best_action: str


def engagement(f: PlayerFeatures) -> float:
    s = 0.0
    if f.days_since_last_bet < 3:
        s += 0.3
    elif f.days_since_last_bet < 7:
        s += 0.2
    elif f.days_since_last_bet < 14:
        s += 0.1
    if f.sessions_per_week >= 5:
        s += 0.2
    elif f.sessions_per_week >= 3:
        s += 0.15
    elif f.sessions_per_week >= 1:
        s += 0.1
    if f.deposit_frequency >= 4:
        s += 0.2
    elif f.deposit_frequency >= 2:
        s += 0.15
    elif f.deposit_frequency >= 1:
        s += 0.1
    if f.push_enabled:
        s += 0.1
    if f.email_opt_in:
        s += 0.1
    if f.has_vip_manager:
        s += 0.1
    return min(s, 1.0)


def churn_risk(f: PlayerFeatures) -> float:
    r = 0.0
    if f.days_since_last_bet > 30:
        r += 0.5
    elif f.days_since_last_bet > 14:
        r += 0.3
    elif f.days_since_last_bet > 7:
        r += 0.15
    if f.sessions_per_week < 1 and f.days_since_registration > 30:
        r += 0.2
    if f.days_since_last_deposit > 30:
        r += 0.2
    if f.support_tickets > 3:
        r += 0.1
    if f.total_withdrawals > f.total_deposits:
        r += 0.1
    return min(r, 1.0)


def base_ltv(f: PlayerFeatures) -> float:
    if f.days_since_registration < 30:
        monthly = f.net_revenue / float(max(f.days_since_registration, 1)) * 30
        return monthly * 12
    monthly = f.net_revenue / float(f.days_since_registration) * 30
    remaining = 12.0 * engagement(f)
    return f.net_revenue + monthly * remaining


def segment_of(ltv: float, churn: float) -> int:
    if churn > 0.7:
        return SEG_CHURNING
    if ltv >= 10000:
        return SEG_VIP
    if ltv >= 1000:
        return SEG_HIGH
    if ltv >= 100:
        return SEG_MEDIUM
    return SEG_LOW


def survival(f: PlayerFeatures, churn: float) -> int:
    d = 90.0 * (1.0 + engagement(f)) * (1.0 - churn)
    return int(max(d, 0.0))


def next_best_action(seg: int, f: PlayerFeatures, churn: float) -> str:
    if seg == SEG_CHURNING:
        return "SEND_WINBACK_BONUS" if f.net_revenue > 0 else "SEND_ENGAGEMENT_EMAIL"
    if seg == SEG_VIP:
        return "VIP_MANAGER_CALL" if f.days_since_last_deposit > 7 else "EXCLUSIVE_EVENT_INVITE"
    if seg == SEG_HIGH:
        if not f.has_vip_manager:
            return "ASSIGN_VIP_MANAGER"
        if churn > 0.3:
            return "RETENTION_BONUS"
        return "LOYALTY_REWARD"
    if seg == SEG_MEDIUM:
        if f.bonuses_claimed < 3:
            return "SUGGEST_BONUS"
        if f.games_played < 5:
            return "RECOMMEND_NEW_GAMES"
        return "STANDARD_PROMOTION"
    if seg == SEG_LOW:
        if f.days_since_registration < 7:
            return "ONBOARDING_GUIDE"
        if f.bonus_conversion_rate > 0.8:
            return "NO_ACTION"
        return "SMALL_DEPOSIT_BONUS"
    return "NO_ACTION"


def confidence(f: PlayerFeatures) -> float:
    c = 0.0
    if f.days_since_registration > 90:
        c += 0.3
    elif f.days_since_registration > 30:
        c += 0.2
    else:
        c += 0.1
    if f.bet_count > 100:
        c += 0.3
    elif f.bet_count > 20:
        c += 0.2
    else:
        c += 0.1
    if f.deposit_frequency > 2:
        c += 0.2
    elif f.deposit_frequency > 0:
        c += 0.1
    if f.days_since_last_bet < 7:
        c += 0.2
    elif f.days_since_last_bet < 30:
        c += 0.1
    return min(c, 1.0)


def predict(f: PlayerFeatures, ltv_override: float = None) -> LTVPrediction:
    """``LTVPredictor.Predict`` (ltv.go:113-151). ``ltv_override`` replaces the formula
    LTV with a learned model's output (cfg 4 MLP) before the churn adjustment."""
    ltv = base_ltv(f) if ltv_override is None else float(ltv_override)
    churn = churn_risk(f)
    adjusted = ltv * (1 - churn * 0.5)
    seg = segment_of(adjusted, churn)
    return LTVPrediction(
        predicted_ltv=adjusted,
        segment=seg,
        churn_risk=churn,
        survival_days=survival(f, churn),
        confidence=confidence(f),
        next_best_action=next_best_action(seg, f, churn),
    )


SEGMENT_PLAYBOOK = {
    SEG_VIP: ["EXCLUSIVE_EVENT_INVITE", "VIP_MANAGER_CALL"],
    SEG_HIGH: ["LOYALTY_REWARD", "RETENTION_BONUS"],
    SEG_MEDIUM: ["STANDARD_PROMOTION", "SUGGEST_BONUS"],
    SEG_LOW: ["SMALL_DEPOSIT_BONUS", "ONBOARDING_GUIDE"],
    SEG_CHURNING: ["SEND_WINBACK_BONUS", "SEND_ENGAGEMENT_EMAIL"],
}


def recommended_actions(seg: int, f: PlayerFeatures, churn: float) -> List[str]:
    """GetPlayerSegment.recommended_actions: the NBA first, then segment-generic actions."""
    acts = [next_best_action(seg, f, churn)]
    for a in SEGMENT_PLAYBOOK.get(seg, []):
        if a not in acts:
            acts.append(a)
    return acts


# ---------------------------------------------------------------- simple LTVModel
def simple_model_predict(days_since_registration: float, days_since_last_deposit: float,
                         days_since_last_bet: float, sessions_per_week: float,
                         net_revenue: float, deposit_frequency: float, games_played: float,
                         bonus_conversion_rate: float) -> float:
    """``LTVModel.Predict`` (onnx_model.go:405-432) with its helpers (:434-490)."""
    current = float(net_revenue)
    days = float(days_since_registration)
    if days < 1:
        days = 1
    monthly = current / days * 30
    e = 0.0
    if days_since_last_bet < 3:
        e += 0.3
    elif days_since_last_bet < 7:
        e += 0.2
    if sessions_per_week >= 5:
        e += 0.2
    elif sessions_per_week >= 3:
        e += 0.15
    if deposit_frequency >= 4:
        e += 0.2
    elif deposit_frequency >= 2:
        e += 0.15
    if games_played >= 10:
        e += 0.15
    if bonus_conversion_rate > 0.5:
        e += 0.15
    e = min(e, 1.0)
    r = 0.0
    if days_since_last_bet > 30:
        r += 0.5
    elif days_since_last_bet > 14:
        r += 0.3
    if days_since_last_deposit > 30:
        r += 0.2
    if sessions_per_week < 1 and days_since_registration > 30:
        r += 0.2
    r = min(r, 1.0)
    return (current + monthly * 12.0 * e) * (1.0 - r * 0.5)


def _isfinite(x: float) -> bool:
    return not (math.isinf(x) or math.isnan(x))

"""Bonus rules engine (services/bonus/internal/service/bonus_engine.go).

* The YAML DSL (``bonus_rules:`` list; schema bonus_engine.go:39-99) is parsed with
  ``yaml.safe_load`` and validated into dataclasses — unknown keys and bad types fail loudly.
* Eligibility: active, one-time claims, player conditions, schedule (date range, weekday
  names, and the HH:MM window the reference parses but never enforces — quirk Q16).
* Awards call the risk service's CheckBonusAbuse first (fail-open on error,
  bonus_engine.go:268-275), compute the amount (deposit match capped by max_bonus; fixed
  amounts for no-deposit / freebet; cashback on net losses) and the wagering requirement,
  credit the bonus balance through the wallet and publish ``bonus.awarded``.
* ``min_deposit`` is enforced when ``enforce_min_deposit`` (the reference parses it and never
  checks, Q16); PlayerInfo.total_deposits is the deposit COUNT, as in the reference.
* Wagering: contribution = bet x game weight % (0 if excluded / not eligible); completion
  releases the bonus. Max-bet (percent of bonus and absolute) is checked before a bet.
"""
from __future__ import annotations

import dataclasses
import datetime as dt
import time
import uuid
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import yaml

from ..events import bus as EB
from ..obs.logging import get_logger

log = get_logger("bonus")

TYPES = ("deposit_match", "no_deposit", "free_spins", "cashback", "freebet", "reload")
WEEKDAYS = ["monday", "tuesday", "wednesday", "thursday", "friday", "saturday", "sunday"]


class BonusError(Exception):
    def __init__(self, code: str, message: str):
        super().__init__(f"{code}: {message}")
        self.code, self.message = code, message


@dataclass
class Schedule:
    days_of_week: List[str] = field(default_factory=list)
    start_time: str = ""      # HH:MM (UTC)
    end_time: str = ""
    start_date: str = ""      # YYYY-MM-DD
    end_date: str = ""


@dataclass
class Conditions:
    min_deposits_lifetime: int = 0
    min_account_age_days: int = 0
    max_account_age_days: int = 0
    required_segment: str = ""
    excluded_segments: List[str] = field(default_factory=list)
    countries: List[str] = field(default_factory=list)
    excluded_countries: List[str] = field(default_factory=list)


@dataclass
class BonusRule:
    id: str
    name: str
    type: str
    description: str = ""
    match_percent: int = 0
    max_bonus: int = 0
    min_deposit: int = 0
    fixed_amount: int = 0
    free_spins_count: int = 0
    cashback_percent: int = 0
    wagering_multiplier: int = 0
    max_bet_percent: int = 0
    max_bet_absolute: int = 0
    eligible_games: List[str] = field(default_factory=list)
    excluded_games: List[str] = field(default_factory=list)
    game_weights: Dict[str, int] = field(default_factory=dict)
    expiry_days: int = 30
    schedule: Optional[Schedule] = None
    conditions: Optional[Conditions] = None
    active: bool = True
    one_time: bool = False
    promo_code: str = ""


def _build(cls, d: dict, where: str):
    if not isinstance(d, dict):
        raise ValueError(f"{where}: mapping expected")
    names = {f.name: f for f in dataclasses.fields(cls)}
    unknown = set(d) - set(names)
    if unknown:
        raise ValueError(f"{where}: unknown keys {sorted(unknown)}")
    kw = {}
    for k, v in d.items():
        if k == "schedule" and v is not None:
            v = _build(Schedule, v, f"{where}.schedule")
        elif k == "conditions" and v is not None:
            v = _build(Conditions, v, f"{where}.conditions")
        kw[k] = v
    return cls(**kw)


def load_rules(text: str) -> List[BonusRule]:
    data = yaml.safe_load(text) or {}
    rules = []
    seen = set()
    for i, d in enumerate(data.get("bonus_rules", [])):
        r = _build(BonusRule, d, f"bonus_rules[{i}]")
        if r.type not in TYPES:
            raise ValueError(f"rule {r.id}: unknown type {r.type!r}")
        if r.id in seen:
            raise ValueError(f"duplicate rule id {r.id}")
        for pct in (r.match_percent, r.max_bet_percent, r.cashback_percent):
            if not 0 <= int(pct) <= 1000:
                raise ValueError(f"rule {r.id}: percentage out of range")
        if r.schedule:
            for day in r.schedule.days_of_week:
                if day.lower() not in WEEKDAYS:
                    raise ValueError(f"rule {r.id}: bad weekday {day!r}")
        seen.add(r.id)
        rules.append(r)
    return rules


def load_rules_file(path: str) -> List[BonusRule]:
    with open(path) as f:
        return load_rules(f.read())


@dataclass
class PlayerInfo:
    """bonus_engine.go:144-151 (total_deposits is a count, like the reference)."""
    account_id: str
    account_age_days: int = 0
    total_deposits: int = 0
    segment: str = ""
    country: str = ""
    total_bonus_claims: int = 0


@dataclass
class PlayerBonus:
    id: str
    account_id: str
    rule_id: str
    type: str
    status: str
    bonus_amount: int
    wagering_required: int
    wagering_progress: int = 0
    free_spins_total: int = 0
    free_spins_used: int = 0
    awarded_at: float = 0.0
    expires_at: float = 0.0
    completed_at: Optional[float] = None
    trigger_tx_id: Optional[str] = None
    promo_code: Optional[str] = None


class BonusEngine:
    def __init__(self, rules: List[BonusRule], repo, risk=None, players=None, wallet=None,
                 bus: Optional[EB.EventBus] = None, enforce_min_deposit: bool = True, clock=time.time):
        """``risk``: object with check_bonus_abuse(account_id, bonus_id) -> (is_abuser, score, signals)
        (risk.v1 CheckBonusAbuse); ``players``: callable account_id -> PlayerInfo;
        ``wallet``: WalletService (credits the bonus balance)."""
        self.rules = rules
        self.by_id = {r.id: r for r in rules}
        self.repo, self.risk, self.players, self.wallet, self.bus = repo, risk, players, wallet, bus
        self.enforce_min_deposit = enforce_min_deposit
        self.clock = clock

    @classmethod
    def from_file(cls, path: str, repo, **kw) -> "BonusEngine":
        return cls(load_rules_file(path), repo, **kw)

    # ---- lookup
    def get_rule(self, rule_id: str) -> Optional[BonusRule]:
        return self.by_id.get(rule_id)

    def all_rules(self) -> List[BonusRule]:
        return [r for r in self.rules if r.active]

    # ---- eligibility
    def _player(self, account_id: str) -> PlayerInfo:
        if self.players is None:
            return PlayerInfo(account_id)
        return self.players(account_id)

    def check_conditions(self, rule: BonusRule, p: PlayerInfo) -> bool:
        c = rule.conditions
        if c is None:
            return True
        if c.min_deposits_lifetime and p.total_deposits < c.min_deposits_lifetime:
            return False
        if c.min_account_age_days and p.account_age_days < c.min_account_age_days:
            return False
        if c.max_account_age_days and p.account_age_days > c.max_account_age_days:
            return False
        if c.required_segment and p.segment != c.required_segment:
            return False
        if p.segment in c.excluded_segments:
            return False
        if c.countries and p.country not in c.countries:
            return False
        if p.country in c.excluded_countries:
            return False
        return True

    def check_schedule(self, rule: BonusRule, now: Optional[float] = None) -> bool:
        s = rule.schedule
        if s is None:
            return True
        t = dt.datetime.fromtimestamp(self.clock() if now is None else now, dt.timezone.utc)
        if s.start_date and t.date() < dt.date.fromisoformat(s.start_date):
            return False
        if s.end_date and t.date() > dt.date.fromisoformat(s.end_date):
            return False
        if s.days_of_week and WEEKDAYS[t.weekday()] not in [d.lower() for d in s.days_of_week]:
            return False
        hm = t.strftime("%H:%M")
        if s.start_time and hm < s.start_time:
            return False
        if s.end_time and hm > s.end_time:
            return False
        return True

    def eligible(self, account_id: str, promo_code: str = "") -> List[BonusRule]:
        p = self._player(account_id)
        out = []
        for r in self.rules:
            if not r.active or (r.promo_code and r.promo_code != promo_code):
                continue
            if r.one_time and self.repo.count_by_rule_and_account(r.id, account_id) > 0:
                continue
            if self.check_conditions(r, p) and self.check_schedule(r):
                out.append(r)
        return out

    # ---- amounts
    @staticmethod
    def bonus_amount(rule: BonusRule, deposit: int, net_loss: int = 0) -> int:
        if rule.type in ("deposit_match", "reload"):
            return min(deposit * rule.match_percent // 100, rule.max_bonus) if rule.max_bonus else \
                deposit * rule.match_percent // 100
        if rule.type == "cashback":
            v = max(net_loss, 0) * rule.cashback_percent // 100
            return min(v, rule.max_bonus) if rule.max_bonus else v
        return rule.fixed_amount

    @staticmethod
    def wager_contribution(rule: BonusRule, category: str, bet: int) -> int:
        if category in rule.excluded_games:
            return 0
        if rule.eligible_games and category not in rule.eligible_games:
            return 0
        return bet * int(rule.game_weights.get(category, 100)) // 100

    # ---- lifecycle
    def award(self, account_id: str, rule_id: str, deposit_amount: int = 0, trigger_tx_id: Optional[str] = None,
              promo_code: Optional[str] = None, net_loss: int = 0) -> PlayerBonus:
        rule = self.by_id.get(rule_id)
        if rule is None:
            raise BonusError("RULE_NOT_FOUND", f"bonus rule not found: {rule_id}")
        if not rule.active:
            raise BonusError("RULE_INACTIVE", "bonus rule is not active")
        if rule.promo_code and rule.promo_code != (promo_code or ""):
            raise BonusError("PROMO_CODE", "promo code required")
        p = self._player(account_id)
        if not self.check_conditions(rule, p) or not self.check_schedule(rule):
            raise BonusError("NOT_ELIGIBLE", "player not eligible for this bonus")
        if self.enforce_min_deposit and rule.min_deposit and rule.type in ("deposit_match", "reload") \
                and deposit_amount < rule.min_deposit:
            raise BonusError("MIN_DEPOSIT", f"deposit {deposit_amount} below minimum {rule.min_deposit}")
        if self.risk is not None:
            try:
                is_abuser, score, signals = self.risk.check_bonus_abuse(account_id, rule_id)
            except Exception as e:  # fail-open (bonus_engine.go:270-271)
                log.warning("abuse check failed", extra={"fields": dict(error=str(e))})
            else:
                if is_abuser:
                    self._publish(EB.risk_event(EB.FRAUD_DETECTED, account_id, int(score * 100), "bonus_blocked",
                                                list(signals)), EB.EXCHANGE_RISK)
                    raise BonusError("ABUSE_SUSPECTED", f"bonus blocked: suspected abuse ({', '.join(signals)})")
        if rule.one_time and self.repo.count_by_rule_and_account(rule.id, account_id) > 0:
            raise BonusError("ALREADY_CLAIMED", "bonus already claimed")
        amount = self.bonus_amount(rule, deposit_amount, net_loss)
        if amount <= 0 and rule.type != "free_spins":
            raise BonusError("ZERO_AMOUNT", "calculated bonus amount is zero")
        now = self.clock()
        b = PlayerBonus(id=str(uuid.uuid4()), account_id=account_id, rule_id=rule.id, type=rule.type, status="active",
                        bonus_amount=amount, wagering_required=amount * rule.wagering_multiplier,
                        free_spins_total=rule.free_spins_count, awarded_at=now,
                        expires_at=now + rule.expiry_days * 86400, trigger_tx_id=trigger_tx_id, promo_code=promo_code)
        if b.wagering_required == 0 and rule.type != "free_spins":
            b.status, b.completed_at = "completed", now
        self.repo.create(b)
        if self.wallet is not None and amount > 0:
            self.wallet.grant_bonus(account_id, amount, f"bonus:{b.id}", bonus_id=b.id)
        self._publish(EB.bonus_event(EB.BONUS_AWARDED, dict(bonus_id=b.id, account_id=account_id, rule_id=rule.id,
                                                            type=rule.type, amount=amount,
                                                            wagering_required=b.wagering_required,
                                                            wagering_progress=0)))
        log.info("bonus awarded", extra={"fields": dict(bonus_id=b.id, account_id=account_id, rule_id=rule.id,
                                                        amount=amount)})
        return b

    def process_wager(self, account_id: str, bet: int, game_id: str = "", category: str = "") -> List[PlayerBonus]:
        done = []
        for b in self.repo.active_by_account(account_id):
            rule = self.by_id.get(b.rule_id)
            if rule is None:
                continue
            c = self.wager_contribution(rule, category, bet)
            if c == 0:
                continue
            b.wagering_progress += c
            self.repo.log(b.id, "wager", c, b.wagering_progress)
            if b.wagering_progress >= b.wagering_required:
                b.status, b.completed_at = "completed", self.clock()
                done.append(b)
                self._publish(EB.bonus_event(EB.BONUS_COMPLETED, dict(
                    bonus_id=b.id, account_id=account_id, rule_id=b.rule_id, type=b.type, amount=b.bonus_amount,
                    wagering_required=b.wagering_required, wagering_progress=b.wagering_progress)))
            self.repo.update(b)
        return done

    def check_max_bet(self, account_id: str, bet: int) -> None:
        for b in self.repo.active_by_account(account_id):
            rule = self.by_id.get(b.rule_id)
            if rule is None:
                continue
            if rule.max_bet_percent > 0:
                cap = b.bonus_amount * rule.max_bet_percent // 100
                if bet > cap:
                    from ..wallet.domain import WalletError
                    raise WalletError("BONUS_RESTRICTION", f"bet {bet} exceeds {rule.max_bet_percent}% of bonus ({cap})")
            if rule.max_bet_absolute > 0 and bet > rule.max_bet_absolute:
                from ..wallet.domain import WalletError
                raise WalletError("BONUS_RESTRICTION", f"bet {bet} exceeds absolute max {rule.max_bet_absolute}")

    def expire(self, now: Optional[float] = None) -> int:
        n = 0
        for b in self.repo.expired(self.clock() if now is None else now):
            b.status = "expired"
            self.repo.update(b)
            self.repo.log(b.id, "expire", b.bonus_amount)
            self._publish(EB.bonus_event(EB.BONUS_EXPIRED, dict(bonus_id=b.id, account_id=b.account_id,
                                                                rule_id=b.rule_id, type=b.type,
                                                                amount=b.bonus_amount)))
            n += 1
        return n

    def forfeit(self, account_id: str) -> int:
        n = 0
        for b in self.repo.active_by_account(account_id):
            b.status = "forfeited"
            self.repo.update(b)
            self.repo.log(b.id, "forfeit", b.bonus_amount)
            n += 1
        return n

    def _publish(self, ev: EB.Event, exchange: str = EB.EXCHANGE_BONUS) -> None:
        if self.bus is not None:
            self.bus.publish(exchange, ev)


class GrpcAbuseChecker:
    """``RiskChecker`` (bonus_engine.go:139-141) over risk.v1 CheckBonusAbuse."""

    def __init__(self, client):
        self.c = client

    def check_bonus_abuse(self, account_id: str, bonus_id: str):
        r = self.c.check_bonus_abuse(account_id, bonus_id)
        return bool(r.is_abuser), float(r.abuse_score), list(r.signals)


class EngineAbuseChecker:
    def __init__(self, engine):
        self.e = engine

    def check_bonus_abuse(self, account_id: str, bonus_id: str):
        r = self.e.check_bonus_abuse(account_id, bonus_id)
        return r.is_abuser, r.abuse_score, r.signals

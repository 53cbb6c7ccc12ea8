"""Currency-tagged decimal money (the reference's ``pkg/money``, money.go:16-261).

The services move int64 cents (as the reference's services do); this type is for API edges,
reports and bonus maths: exact decimal arithmetic, currency mismatch and insufficient-funds
errors, percentages with banker-free half-up rounding to cents, JSON and SQLite adapters.
"""
from __future__ import annotations

import json
import sqlite3
from dataclasses import dataclass
from decimal import ROUND_HALF_UP, Decimal, InvalidOperation
from typing import Union

CENT = Decimal("0.01")
Number = Union[int, str, Decimal, float]


class MoneyError(ValueError):
    pass


class CurrencyMismatch(MoneyError):
    pass


class InsufficientFunds(MoneyError):
    pass


def _dec(v: Number) -> Decimal:
    try:
        d = Decimal(str(v)) if isinstance(v, float) else Decimal(v)
    except (InvalidOperation, TypeError) as e:
        raise MoneyError(f"invalid amount: {v!r}") from e
    if not d.is_finite():
        raise MoneyError(f"invalid amount: {v!r}")
    return d


@dataclass(frozen=True)
class Money:
    amount: Decimal
    currency: str

    def __post_init__(self):
        if not (isinstance(self.currency, str) and len(self.currency) == 3 and self.currency.isalpha()):
            raise MoneyError(f"invalid currency code: {self.currency!r}")
        object.__setattr__(self, "currency", self.currency.upper())
        object.__setattr__(self, "amount", _dec(self.amount))

    # ---- construction
    @classmethod
    def parse(cls, s: str, currency: str) -> "Money":
        return cls(_dec(s.strip()), currency)

    @classmethod
    def from_cents(cls, cents: int, currency: str) -> "Money":
        return cls(Decimal(int(cents)) * CENT, currency)

    @classmethod
    def zero(cls, currency: str) -> "Money":
        return cls(Decimal(0), currency)

    # ---- conversion
    def cents(self) -> int:
        return int((self.amount / CENT).to_integral_value(ROUND_HALF_UP))

    def rounded(self) -> "Money":
        return Money(self.amount.quantize(CENT, ROUND_HALF_UP), self.currency)

    def __str__(self) -> str:
        return f"{self.amount.quantize(CENT, ROUND_HALF_UP)} {self.currency}"

    # ---- arithmetic
    def _same(self, o: "Money") -> None:
        if not isinstance(o, Money):
            raise TypeError("Money expected")
        if o.currency != self.currency:
            raise CurrencyMismatch(f"currency mismatch: {self.currency} vs {o.currency}")

    def add(self, o: "Money") -> "Money":
        self._same(o)
        return Money(self.amount + o.amount, self.currency)

    def sub(self, o: "Money") -> "Money":
        """Subtract; raises :class:`InsufficientFunds` when the result would be negative."""
        self._same(o)
        r = self.amount - o.amount
        if r < 0:
            raise InsufficientFunds(f"insufficient funds: {self} - {o}")
        return Money(r, self.currency)

    def percent(self, pct: Number) -> "Money":
        return Money((self.amount * _dec(pct) / 100).quantize(CENT, ROUND_HALF_UP), self.currency)

    def mul(self, k: Number) -> "Money":
        return Money(self.amount * _dec(k), self.currency)

    __add__ = add
    __sub__ = sub

    # ---- comparison
    def cmp(self, o: "Money") -> int:
        self._same(o)
        return (self.amount > o.amount) - (self.amount < o.amount)

    def __lt__(self, o: "Money") -> bool:
        return self.cmp(o) < 0

    def __le__(self, o: "Money") -> bool:
        return self.cmp(o) <= 0

    def is_zero(self) -> bool:
        return self.amount == 0

    def is_positive(self) -> bool:
        return self.amount > 0

    def is_negative(self) -> bool:
        return self.amount < 0

    # ---- serialisation
    def to_json(self) -> str:
        return json.dumps({"amount": str(self.amount), "currency": self.currency})

    @classmethod
    def from_json(cls, s: str) -> "Money":
        d = json.loads(s)
        return cls(_dec(d["amount"]), d["currency"])


# SQLite column round trip ("12.34 EUR"), the analogue of the reference's sql Scanner/Valuer
sqlite3.register_adapter(Money, lambda m: f"{m.amount} {m.currency}")


def money_from_sql(b: bytes) -> Money:
    amt, cur = b.decode().split()
    return Money(_dec(amt), cur)


sqlite3.register_converter("MONEY", money_from_sql)

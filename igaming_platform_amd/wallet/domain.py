"""Wallet domain model (services/wallet/internal/domain/models.go:12-225)."""
from __future__ import annotations

import time
import uuid
from dataclasses import dataclass, field
from typing import Dict, Optional

# account status (models.go:24-30)
ACTIVE, SUSPENDED, CLOSED = "active", "suspended", "closed"
# transaction types and status (models.go:79-98)
DEPOSIT, WITHDRAW, BET, WIN, REFUND = "deposit", "withdraw", "bet", "win", "refund"
BONUS_GRANT, BONUS_WAGER, ADJUSTMENT = "bonus_grant", "bonus_wager", "adjustment"
PENDING, COMPLETED, FAILED, REVERSED = "pending", "completed", "failed", "reversed"
CREDIT_TYPES = (DEPOSIT, WIN, REFUND, BONUS_GRANT)
DEBIT_TYPES = (WITHDRAW, BET, BONUS_WAGER)
CLEARING_ACCOUNT = "00000000-0000-0000-0000-000000000000"


class WalletError(Exception):
    """Typed error; ``code`` is one of wallet.proto's error codes (wallet.proto:233-241)."""

    def __init__(self, code: str, message: str, **details):
        super().__init__(f"{code}: {message}")
        self.code, self.message, self.details = code, message, {k: str(v) for k, v in details.items()}


def not_found(what: str = "account") -> WalletError:
    return WalletError("ACCOUNT_NOT_FOUND", f"{what} not found")


class ConcurrentUpdate(WalletError):
    def __init__(self):
        super().__init__("CONCURRENT_UPDATE", "concurrent update detected")


@dataclass
class Account:
    player_id: str
    currency: str = "USD"
    balance: int = 0
    bonus: int = 0
    status: str = ACTIVE
    version: int = 1
    id: str = field(default_factory=lambda: str(uuid.uuid4()))
    created_at: float = field(default_factory=time.time)
    updated_at: float = field(default_factory=time.time)

    def can_transact(self) -> bool:
        return self.status == ACTIVE

    def total_balance(self) -> int:
        return self.balance + self.bonus

    def withdrawable(self) -> int:
        return self.balance       # bonus money is never withdrawable (models.go:71-74)


@dataclass
class Transaction:
    account_id: str
    idempotency_key: str
    type: str
    amount: int
    balance_before: int
    balance_after: int
    status: str = PENDING
    reference: str = ""
    game_id: Optional[str] = None
    round_id: Optional[str] = None
    risk_score: Optional[int] = None
    metadata: Dict[str, str] = field(default_factory=dict)
    id: str = field(default_factory=lambda: str(uuid.uuid4()))
    created_at: float = field(default_factory=time.time)
    completed_at: Optional[float] = None

    def complete(self) -> None:
        self.status = COMPLETED
        self.completed_at = time.time()

    def fail(self) -> None:
        self.status = FAILED

    def is_credit(self) -> bool:
        return self.type in CREDIT_TYPES

    def is_debit(self) -> bool:
        return self.type in DEBIT_TYPES


@dataclass
class LedgerEntry:
    transaction_id: str
    account_id: str
    entry_type: str        # debit | credit
    amount: int
    balance_after: int
    description: str = ""
    id: str = field(default_factory=lambda: str(uuid.uuid4()))
    created_at: float = field(default_factory=time.time)


@dataclass
class BalanceSnapshot:
    account_id: str
    balance: int
    bonus: int
    currency: str
    at: float = field(default_factory=time.time)

    @property
    def total(self) -> int:
        return self.balance + self.bonus

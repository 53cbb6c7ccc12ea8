"""WalletService — money movements with risk checks (services/wallet/internal/service/
wallet_service.go:141-704), re-built as a thin client of risk.v1.

Every operation: idempotency -> account validation -> risk check -> transaction row ->
optimistic-locked balance update -> ledger -> complete -> event. Unlike the reference the
whole sequence runs in ONE unit of work (a failure leaves nothing half-written), the ledger
is double-entry against the platform clearing account, events go through a transactional
outbox, and Refund (declared in wallet.proto, missing from the Go service) is implemented.

Risk semantics (wallet_service.go:263-272, 380-389, 598-608):
  Deposit / Bet: fail-OPEN (risk unavailable -> proceed), reject if score >= block.
  Withdraw:      fail-CLOSED (risk unavailable -> RISK_REVIEW), reject if score >= review.
  Win / Refund:  no risk check. Bet spends bonus money first (wallet_service.go:410-419).
"""
from __future__ import annotations

import time
from typing import List, Optional, Protocol, Sequence, Tuple

from ..events import bus as EB
from ..obs.logging import get_logger
from .domain import (ACTIVE, BET, CLEARING_ACCOUNT, COMPLETED, DEBIT_TYPES, DEPOSIT, REFUND, REVERSED, WIN,
                     WITHDRAW, Account, ConcurrentUpdate, LedgerEntry, Transaction, WalletError, not_found)
from .repository import (AccountRepository, AuditRepository, Database, LedgerRepository, TransactionRepository)

log = get_logger("wallet")


class RiskScorer(Protocol):
    def score(self, account_id: str, amount: int, tx_type: str, ip: str = "", device_id: str = "",
              fingerprint: str = "", game_id: str = "", session_id: str = "") -> Tuple[int, List[str]]:
        ...


class GrpcRisk:
    """RiskScorer over the risk.v1 gRPC API (wallet_service.go:40-42 ``RiskService``)."""

    def __init__(self, client, timeout_s: float = 2.0):
        self.c = client
        self.timeout = timeout_s

    def score(self, account_id, amount, tx_type, ip="", device_id="", fingerprint="", game_id="", session_id=""):
        from ..proto import risk_v1 as P
        r = self.c.call("ScoreTransaction", P.ScoreTransactionRequest(
            account_id=account_id, amount=amount, transaction_type=tx_type, ip_address=ip, device_id=device_id,
            fingerprint=fingerprint, game_id=game_id, session_id=session_id), timeout=self.timeout)
        return int(r.score), list(r.reason_codes)


class EngineRisk:
    """RiskScorer calling an in-process RiskEngine (single-binary deployments, tests)."""

    def __init__(self, engine):
        self.e = engine

    def score(self, account_id, amount, tx_type, ip="", device_id="", fingerprint="", game_id="", session_id=""):
        r = self.e.score([dict(account_id=account_id, amount=amount, transaction_type=tx_type, ip_address=ip,
                               device_id=device_id, fingerprint=fingerprint, game_id=game_id,
                               session_id=session_id)])[0]
        return r["score"], r["reason_codes"]


class WalletService:
    def __init__(self, db: Optional[Database] = None, risk: Optional[RiskScorer] = None,
                 bus: Optional[EB.EventBus] = None, block_threshold: int = 80, review_threshold: int = 50,
                 bonus=None, retries: int = 3):
        self.db = db or Database()
        self.accounts = AccountRepository(self.db)
        self.txs = TransactionRepository(self.db)
        self.ledger = LedgerRepository(self.db)
        self.audit = AuditRepository(self.db)
        self.risk = risk
        self.bus = bus
        self.block_threshold = block_threshold    # RISK_BLOCK_THRESHOLD (wallet main.go:54-62)
        self.review_threshold = review_threshold  # RISK_REVIEW_THRESHOLD
        self.bonus = bonus                        # optional BonusEngine: max-bet + wagering + forfeits
        self.retries = retries

    # ------------------------------------------------------------------ accounts
    def create_account(self, player_id: str, currency: str = "USD") -> Account:
        """Idempotent by player (wallet_service.go:189-219)."""
        if not player_id:
            raise WalletError("INVALID_ARGUMENT", "player_id is required")
        with self.db.unit_of_work():
            a = self.accounts.get_by_player(player_id)
            if a is not None:
                return a
            a = self.accounts.create(Account(player_id=player_id, currency=(currency or "USD").upper()))
            self._emit(EB.EXCHANGE_WALLET, EB.Event(EB.ACCOUNT_CREATED, "wallet-service", a.id,
                                                    {"account_id": a.id, "player_id": player_id,
                                                     "currency": a.currency}))
        self._flush_outbox()
        return a

    def get_account(self, account_id: str = "", player_id: str = "") -> Account:
        if account_id:
            return self.accounts.get_by_id(account_id)
        a = self.accounts.get_by_player(player_id) if player_id else None
        if a is None:
            raise not_found()
        return a

    def get_balance(self, account_id: str) -> Account:
        return self.accounts.get_by_id(account_id)

    def set_status(self, account_id: str, status: str) -> None:
        self.accounts.get_by_id(account_id)
        self.accounts.update_status(account_id, status)

    # ------------------------------------------------------------------ internals
    def _active(self, account_id: str) -> Account:
        a = self.accounts.get_by_id(account_id)
        if a.status != ACTIVE:
            raise WalletError("ACCOUNT_SUSPENDED", f"account is {a.status}")
        return a

    @staticmethod
    def _amount(amount: int) -> None:
        if int(amount) <= 0:
            raise WalletError("INVALID_AMOUNT", "amount must be positive")

    def _risk(self, account_id: str, amount: int, tx_type: str, fail_closed: bool, limit: int, **ctx):
        if self.risk is None:
            return None
        try:
            score, reasons = self.risk.score(account_id, amount, tx_type, **ctx)
        except Exception as e:  # risk unavailable
            if fail_closed:
                log.warning("risk unavailable, holding withdrawal", extra={"fields": dict(error=str(e))})
                raise WalletError("RISK_REVIEW", "withdrawal pending: risk service unavailable")
            log.warning("risk unavailable, proceeding", extra={"fields": dict(error=str(e))})
            return None
        if score >= limit:
            code = "RISK_REVIEW" if fail_closed else "RISK_BLOCKED"
            self._emit_now(EB.EXCHANGE_RISK, EB.risk_event(EB.RISK_BLOCKED, account_id, score,
                                                           code.lower(), reasons))
            raise WalletError(code, f"transaction {'requires review' if fail_closed else 'blocked by risk'}: "
                                    f"score={score}", score=score, reasons=",".join(reasons))
        return score

    def _ledger(self, tx: Transaction, account: Account, description: str) -> None:
        """Double entry: the account side and the contra posting on the clearing account."""
        credit = tx.is_credit()
        self.ledger.create(LedgerEntry(tx.id, tx.account_id, "credit" if credit else "debit", tx.amount,
                                       tx.balance_after, description))
        clearing_after = self.ledger.clearing_balance() + (-tx.amount if credit else tx.amount)
        self.ledger.create(LedgerEntry(tx.id, CLEARING_ACCOUNT, "debit" if credit else "credit", tx.amount,
                                       clearing_after, description))

    def _emit(self, exchange: str, ev: EB.Event) -> None:
        self.audit.outbox(exchange, ev.type, ev.to_json().decode())

    def _emit_now(self, exchange: str, ev: EB.Event) -> None:
        if self.bus is not None:
            self.bus.publish(exchange, ev)

    def _flush_outbox(self) -> None:
        """Relay committed outbox rows to the bus (at-least-once; consumers dedupe on event id)."""
        if self.bus is None:
            return
        rows = self.audit.pending_outbox(1000)
        for r in rows:
            self.bus.publish(r["exchange"], EB.Event.from_json(r["payload"].encode()), r["routing_key"])
        self.audit.mark_published([r["id"] for r in rows])

    def _run(self, fn):
        """Retry a unit of work on optimistic-lock conflicts."""
        for attempt in range(self.retries):
            try:
                with self.db.unit_of_work():
                    out = fn()
                self._flush_outbox()
                return out
            except ConcurrentUpdate:
                if attempt == self.retries - 1:
                    raise
                time.sleep(0.001 * (attempt + 1))

    def _commit(self, tx: Transaction, account: Account, balance: int, bonus: int, description: str,
                events: Sequence[str]) -> None:
        self.txs.create(tx)
        self.accounts.update_balance(account.id, balance, bonus, account.version)
        self._ledger(tx, account, description)
        tx.complete()
        self.txs.update(tx)
        for et in events:
            self._emit(EB.EXCHANGE_WALLET, EB.transaction_event(et, dict(
                transaction_id=tx.id, account_id=tx.account_id, type=tx.type, amount=tx.amount,
                balance_before=tx.balance_before, balance_after=tx.balance_after, status=tx.status,
                game_id=tx.game_id, round_id=tx.round_id, risk_score=tx.risk_score)))

    # ------------------------------------------------------------------ money movements
    def deposit(self, account_id: str, amount: int, idempotency_key: str, payment_method: str = "",
                reference: str = "", ip: str = "", device_id: str = "", fingerprint: str = ""):
        self._amount(amount)
        prev = self.txs.get_by_idempotency_key(account_id, idempotency_key)
        if prev is not None:
            return prev, prev.balance_after, prev.risk_score
        self._active(account_id)
        score = self._risk(account_id, amount, DEPOSIT, False, self.block_threshold, ip=ip, device_id=device_id,
                           fingerprint=fingerprint)

        def work():
            a = self._active(account_id)
            tx = Transaction(account_id, idempotency_key, DEPOSIT, amount, a.total_balance(),
                             a.total_balance() + amount, reference=reference or f"payment:{payment_method}",
                             risk_score=score, metadata={"payment_method": payment_method})
            self._commit(tx, a, a.balance + amount, a.bonus, "Deposit", [EB.TRANSACTION_COMPLETED, EB.DEPOSIT_RECEIVED])
            return tx, tx.balance_after, score
        return self._run(work)

    def bet(self, account_id: str, amount: int, idempotency_key: str, game_id: str = "", round_id: str = "",
            game_category: str = "", ip: str = "", device_id: str = "", session_id: str = ""):
        """Returns (tx, new_total, risk_score, real_deducted, bonus_deducted)."""
        self._amount(amount)
        prev = self.txs.get_by_idempotency_key(account_id, idempotency_key)
        if prev is not None:
            m = prev.metadata
            return prev, prev.balance_after, prev.risk_score, int(m.get("real", 0)), int(m.get("bonus", 0))
        a = self._active(account_id)
        if a.total_balance() < amount:
            raise WalletError("INSUFFICIENT_BALANCE", f"available={a.total_balance()} required={amount}")
        if self.bonus is not None:
            self.bonus.check_max_bet(account_id, amount)
        score = self._risk(account_id, amount, BET, False, self.block_threshold, ip=ip, device_id=device_id,
                           game_id=game_id, session_id=session_id)

        def work():
            a = self._active(account_id)
            if a.total_balance() < amount:
                raise WalletError("INSUFFICIENT_BALANCE", f"available={a.total_balance()} required={amount}")
            from_bonus = min(a.bonus, amount)
            from_real = amount - from_bonus
            tx = Transaction(account_id, idempotency_key, BET, amount, a.total_balance(), a.total_balance() - amount,
                             reference=f"game:{game_id}:round:{round_id}", game_id=game_id or None,
                             round_id=round_id or None, risk_score=score,
                             metadata={"real": str(from_real), "bonus": str(from_bonus), "category": game_category})
            self._commit(tx, a, a.balance - from_real, a.bonus - from_bonus, "Bet",
                         [EB.TRANSACTION_COMPLETED, EB.BET_PLACED])
            return tx, tx.balance_after, score, from_real, from_bonus
        out = self._run(work)
        if self.bonus is not None:
            self.bonus.process_wager(account_id, amount, game_id, game_category)
        return out

    def win(self, account_id: str, amount: int, idempotency_key: str, game_id: str = "", round_id: str = "",
            bet_transaction_id: str = "", win_type: str = "normal", metadata: Optional[dict] = None):
        self._amount(amount)
        prev = self.txs.get_by_idempotency_key(account_id, idempotency_key)
        if prev is not None:
            return prev, prev.balance_after
        self._active(account_id)
        if bet_transaction_id:
            bt = self.txs.get(bet_transaction_id)
            if bt is None or bt.account_id != account_id or bt.type != BET:
                raise WalletError("INVALID_OPERATION", "bet_transaction_id does not reference a bet of this account")

        def work():
            a = self._active(account_id)
            md = dict(metadata or {})
            md.update(win_type=win_type, bet_tx=bet_transaction_id)
            tx = Transaction(account_id, idempotency_key, WIN, amount, a.total_balance(), a.total_balance() + amount,
                             reference=f"game:{game_id}:round:{round_id}", game_id=game_id or None,
                             round_id=round_id or None, metadata=md)
            self._commit(tx, a, a.balance + amount, a.bonus, "Win", [EB.TRANSACTION_COMPLETED, EB.WIN_PAID])
            return tx, tx.balance_after
        return self._run(work)

    def withdraw(self, account_id: str, amount: int, idempotency_key: str, payout_method: str = "",
                 payout_details: str = "", ip: str = "", device_id: str = ""):
        """Returns (tx, new_total, risk_score, payout_status)."""
        self._amount(amount)
        prev = self.txs.get_by_idempotency_key(account_id, idempotency_key)
        if prev is not None:
            return prev, prev.balance_after, prev.risk_score, "pending"
        a = self._active(account_id)
        if a.withdrawable() < amount:
            raise WalletError("INSUFFICIENT_BALANCE", f"withdrawable={a.withdrawable()} required={amount}")
        score = self._risk(account_id, amount, WITHDRAW, True, self.review_threshold, ip=ip, device_id=device_id)

        def work():
            a = self._active(account_id)
            if a.withdrawable() < amount:
                raise WalletError("INSUFFICIENT_BALANCE", f"withdrawable={a.withdrawable()} required={amount}")
            tx = Transaction(account_id, idempotency_key, WITHDRAW, amount, a.total_balance(),
                             a.total_balance() - amount, reference=f"payout:{payout_method}", risk_score=score,
                             metadata={"payout_method": payout_method, "payout_details": payout_details})
            self._commit(tx, a, a.balance - amount, a.bonus, "Withdrawal",
                         [EB.TRANSACTION_COMPLETED, EB.WITHDRAWAL_COMPLETED])
            return tx, tx.balance_after, score, "pending"
        out = self._run(work)
        if self.bonus is not None:
            self.bonus.forfeit(account_id)   # early withdrawal forfeits active bonuses
        return out

    def refund(self, account_id: str, original_transaction_id: str, idempotency_key: str, reason: str = ""):
        """Reverse a completed debit (bet / withdrawal) back to the real balance."""
        prev = self.txs.get_by_idempotency_key(account_id, idempotency_key)
        if prev is not None:
            return prev, prev.balance_after
        orig = self.txs.get(original_transaction_id)
        if orig is None or orig.account_id != account_id:
            raise WalletError("TRANSACTION_NOT_FOUND", "original transaction not found")
        if orig.type not in DEBIT_TYPES or orig.status != COMPLETED:
            raise WalletError("INVALID_OPERATION", f"cannot refund a {orig.status} {orig.type}")

        def work():
            a = self._active(account_id)
            o = self.txs.get(original_transaction_id)
            if o.status != COMPLETED:
                raise WalletError("INVALID_OPERATION", "transaction already reversed")
            tx = Transaction(account_id, idempotency_key, REFUND, o.amount, a.total_balance(),
                             a.total_balance() + o.amount, reference=f"refund:{o.id}", game_id=o.game_id,
                             round_id=o.round_id, metadata={"original": o.id, "reason": reason})
            self._commit(tx, a, a.balance + o.amount, a.bonus, "Refund", [EB.TRANSACTION_COMPLETED])
            o.status = REVERSED
            self.txs.update(o)
            return tx, tx.balance_after
        return self._run(work)

    def grant_bonus(self, account_id: str, amount: int, idempotency_key: str, bonus_id: str = ""):
        """Credit bonus money (called by the bonus engine on award)."""
        self._amount(amount)
        from .domain import BONUS_GRANT

        def work():
            a = self._active(account_id)
            tx = Transaction(account_id, idempotency_key, BONUS_GRANT, amount, a.total_balance(),
                             a.total_balance() + amount, reference=f"bonus:{bonus_id}")
            self._commit(tx, a, a.balance, a.bonus + amount, "Bonus grant", [EB.TRANSACTION_COMPLETED])
            return tx
        prev = self.txs.get_by_idempotency_key(account_id, idempotency_key)
        return prev if prev is not None else self._run(work)

    # ------------------------------------------------------------------ history
    def history(self, account_id: str, limit: int = 50, offset: int = 0, types: Sequence[str] = (),
                t_from: Optional[float] = None, t_to: Optional[float] = None, game_id: str = ""):
        """(transactions, total, has_more); limit capped at 100 (wallet.proto:171)."""
        self.accounts.get_by_id(account_id)
        limit = max(1, min(int(limit or 50), 100))
        txs = self.txs.list_by_account(account_id, limit, offset, types, t_from, t_to, game_id)
        total = self.txs.count_by_account(account_id, types, t_from, t_to, game_id)
        return txs, total, offset + len(txs) < total

    def get_transaction(self, tx_id: str) -> Transaction:
        t = self.txs.get(tx_id)
        if t is None:
            raise WalletError("TRANSACTION_NOT_FOUND", "transaction not found")
        return t

"""SQLite repositories for the wallet and bonus services.

The reference's repositories are Postgres via sqlx (services/wallet/internal/repository/
postgres.go): account CRUD with optimistic locking (``WHERE version = $4``, :129-148), row
locks, transactions with idempotency lookup / history / per-round / daily stats (:172-317),
ledger with balance verification (:320-390) and a unit-of-work wrapper (:393-443). No Postgres
server exists here, so the same repository surface runs on SQLite (stdlib, WAL mode, one
writer at a time via ``BEGIN IMMEDIATE`` — the SQLite equivalent of ``SELECT ... FOR UPDATE``).
The schema is deploy/schema.sql.
"""
from __future__ import annotations

import json
import os
import sqlite3
import threading
import time
from contextlib import contextmanager
from typing import Iterator, List, Optional, Sequence

from .domain import CLEARING_ACCOUNT, Account, ConcurrentUpdate, LedgerEntry, Transaction, WalletError, not_found

SCHEMA = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                      "deploy", "schema.sql")


class Database:
    """One SQLite connection shared by the repositories; ``unit_of_work`` serialises writers."""

    def __init__(self, path: str = ":memory:"):
        self.path = path
        self.conn = sqlite3.connect(path, check_same_thread=False, isolation_level=None, timeout=30)
        self.conn.row_factory = sqlite3.Row
        if path != ":memory:":
            self.conn.execute("PRAGMA journal_mode=WAL")
        with open(SCHEMA) as f:
            self.conn.executescript(f.read())
        self._lock = threading.RLock()
        self._depth = 0

    @contextmanager
    def unit_of_work(self) -> Iterator[sqlite3.Connection]:
        """Atomic scope (nested scopes join the outer one)."""
        with self._lock:
            outer = self._depth == 0
            if outer:
                self.conn.execute("BEGIN IMMEDIATE")
            self._depth += 1
            try:
                yield self.conn
                self._depth -= 1
                if outer:
                    self.conn.execute("COMMIT")
            except BaseException:
                self._depth -= 1
                if outer:
                    self.conn.execute("ROLLBACK")
                raise

    def query(self, sql: str, args: Sequence = ()) -> List[sqlite3.Row]:
        with self._lock:
            return self.conn.execute(sql, args).fetchall()

    def execute(self, sql: str, args: Sequence = ()) -> sqlite3.Cursor:
        with self._lock:
            return self.conn.execute(sql, args)


def is_duplicate_key(e: Exception) -> bool:
    """postgres.go:446-453 (unique violation) for SQLite."""
    return isinstance(e, sqlite3.IntegrityError) and "UNIQUE" in str(e)


def _acct(r) -> Account:
    return Account(player_id=r["player_id"], currency=r["currency"], balance=r["balance"], bonus=r["bonus"],
                   status=r["status"], version=r["version"], id=r["id"], created_at=r["created_at"],
                   updated_at=r["updated_at"])


def _tx(r) -> Transaction:
    return Transaction(account_id=r["account_id"], idempotency_key=r["idempotency_key"], type=r["type"],
                       amount=r["amount"], balance_before=r["balance_before"], balance_after=r["balance_after"],
                       status=r["status"], reference=r["reference"] or "", game_id=r["game_id"],
                       round_id=r["round_id"], risk_score=r["risk_score"], metadata=json.loads(r["metadata"] or "{}"),
                       id=r["id"], created_at=r["created_at"], completed_at=r["completed_at"])


class AccountRepository:
    def __init__(self, db: Database):
        self.db = db

    def create(self, a: Account) -> Account:
        try:
            self.db.execute("INSERT INTO accounts(id, player_id, currency, balance, bonus, status, version, created_at, "
                            "updated_at) VALUES (?,?,?,?,?,?,?,?,?)",
                            (a.id, a.player_id, a.currency, a.balance, a.bonus, a.status, a.version, a.created_at,
                             a.updated_at))
        except sqlite3.IntegrityError as e:
            if is_duplicate_key(e):
                raise WalletError("DUPLICATE_ACCOUNT", f"player {a.player_id} already has an account") from e
            raise
        return a

    def get_by_id(self, account_id: str) -> Account:
        r = self.db.query("SELECT * FROM accounts WHERE id = ? AND status != 'system'", (account_id,))
        if not r:
            raise not_found()
        return _acct(r[0])

    def get_by_player(self, player_id: str) -> Optional[Account]:
        r = self.db.query("SELECT * FROM accounts WHERE player_id = ?", (player_id,))
        return _acct(r[0]) if r else None

    def update_balance(self, account_id: str, balance: int, bonus: int, expected_version: int) -> int:
        """Optimistic lock (postgres.go:129-148): succeeds only if nobody updated since the read."""
        try:
            cur = self.db.execute("UPDATE accounts SET balance = ?, bonus = ?, version = version + 1, updated_at = ? "
                                  "WHERE id = ? AND version = ?",
                                  (balance, bonus, time.time(), account_id, expected_version))
        except sqlite3.IntegrityError as e:
            raise WalletError("INSUFFICIENT_BALANCE", "balance would become negative") from e
        if cur.rowcount != 1:
            raise ConcurrentUpdate()
        return expected_version + 1

    def update_status(self, account_id: str, status: str) -> None:
        self.db.execute("UPDATE accounts SET status = ?, updated_at = ? WHERE id = ?", (status, time.time(), account_id))


class TransactionRepository:
    def __init__(self, db: Database):
        self.db = db

    def create(self, t: Transaction) -> Transaction:
        try:
            self.db.execute(
                "INSERT INTO transactions(id, account_id, idempotency_key, type, amount, balance_before, balance_after, "
                "status, reference, game_id, round_id, risk_score, metadata, created_at, completed_at) "
                "VALUES (?,?,?,?,?,?,?,?,?,?,?,?,?,?,?)",
                (t.id, t.account_id, t.idempotency_key, t.type, t.amount, t.balance_before, t.balance_after, t.status,
                 t.reference, t.game_id, t.round_id, t.risk_score, json.dumps(t.metadata), t.created_at,
                 t.completed_at))
        except sqlite3.IntegrityError as e:
            if is_duplicate_key(e):
                raise WalletError("DUPLICATE_TRANSACTION", "idempotency key already used") from e
            raise
        return t

    def update(self, t: Transaction) -> None:
        self.db.execute("UPDATE transactions SET status = ?, balance_after = ?, risk_score = ?, completed_at = ?, "
                        "metadata = ? WHERE id = ?",
                        (t.status, t.balance_after, t.risk_score, t.completed_at, json.dumps(t.metadata), t.id))

    def get(self, tx_id: str) -> Optional[Transaction]:
        r = self.db.query("SELECT * FROM transactions WHERE id = ?", (tx_id,))
        return _tx(r[0]) if r else None

    def get_by_idempotency_key(self, account_id: str, key: str) -> Optional[Transaction]:
        r = self.db.query("SELECT * FROM transactions WHERE account_id = ? AND idempotency_key = ?", (account_id, key))
        return _tx(r[0]) if r else None

    def list_by_account(self, account_id: str, limit: int = 50, offset: int = 0, types: Sequence[str] = (),
                        t_from: Optional[float] = None, t_to: Optional[float] = None,
                        game_id: str = "") -> List[Transaction]:
        sql, args = self._filter(account_id, types, t_from, t_to, game_id)
        rows = self.db.query("SELECT * FROM transactions " + sql + " ORDER BY created_at DESC, rowid DESC "
                             "LIMIT ? OFFSET ?", args + [int(limit), int(offset)])
        return [_tx(r) for r in rows]

    def count_by_account(self, account_id: str, types: Sequence[str] = (), t_from: Optional[float] = None,
                         t_to: Optional[float] = None, game_id: str = "") -> int:
        sql, args = self._filter(account_id, types, t_from, t_to, game_id)
        return int(self.db.query("SELECT COUNT(*) AS n FROM transactions " + sql, args)[0]["n"])

    @staticmethod
    def _filter(account_id, types, t_from, t_to, game_id):
        cond, args = ["account_id = ?"], [account_id]
        if types:
            cond.append("type IN (%s)" % ",".join("?" * len(types)))
            args += list(types)
        if t_from is not None:
            cond.append("created_at >= ?")
            args.append(t_from)
        if t_to is not None:
            cond.append("created_at <= ?")
            args.append(t_to)
        if game_id:
            cond.append("game_id = ?")
            args.append(game_id)
        return "WHERE " + " AND ".join(cond), args

    def by_round(self, game_id: str, round_id: str) -> List[Transaction]:
        return [_tx(r) for r in self.db.query("SELECT * FROM transactions WHERE game_id = ? AND round_id = ? "
                                              "ORDER BY created_at", (game_id, round_id))]

    def daily_stats(self, account_id: str, day_start: float) -> dict:
        rows = self.db.query("SELECT type, COUNT(*) AS n, SUM(amount) AS s FROM transactions WHERE account_id = ? "
                             "AND status = 'completed' AND created_at >= ? AND created_at < ? GROUP BY type",
                             (account_id, day_start, day_start + 86400))
        return {r["type"]: {"count": r["n"], "sum": r["s"]} for r in rows}


class LedgerRepository:
    def __init__(self, db: Database):
        self.db = db

    def create(self, e: LedgerEntry) -> None:
        self.db.execute("INSERT INTO ledger_entries(id, transaction_id, account_id, entry_type, amount, balance_after, "
                        "description, created_at) VALUES (?,?,?,?,?,?,?,?)",
                        (e.id, e.transaction_id, e.account_id, e.entry_type, e.amount, e.balance_after, e.description,
                         e.created_at))

    def by_transaction(self, tx_id: str) -> List[LedgerEntry]:
        return [LedgerEntry(r["transaction_id"], r["account_id"], r["entry_type"], r["amount"], r["balance_after"],
                            r["description"], r["id"], r["created_at"])
                for r in self.db.query("SELECT * FROM ledger_entries WHERE transaction_id = ? ORDER BY rowid", (tx_id,))]

    def balance(self, account_id: str) -> int:
        r = self.db.query("SELECT COALESCE(SUM(CASE entry_type WHEN 'credit' THEN amount ELSE -amount END), 0) AS b "
                          "FROM ledger_entries WHERE account_id = ?", (account_id,))
        return int(r[0]["b"])

    def clearing_balance(self) -> int:
        return self.balance(CLEARING_ACCOUNT)

    def verify_balance(self, account: Account) -> bool:
        """postgres.go:376-390: the ledger must reproduce the stored total balance."""
        return self.balance(account.id) == account.total_balance()


class BonusRepository:
    """player_bonuses / bonus_transactions (the reference's BonusRepository interface has no
    implementation, bonus_engine.go:129-137)."""

    def __init__(self, db: Database):
        self.db = db

    COLS = ("id", "account_id", "rule_id", "type", "status", "bonus_amount", "wagering_required", "wagering_progress",
            "free_spins_total", "free_spins_used", "awarded_at", "expires_at", "completed_at", "trigger_tx_id",
            "promo_code")

    def create(self, b) -> None:
        self.db.execute("INSERT INTO player_bonuses(%s) VALUES (%s)" % (",".join(self.COLS), ",".join("?" * len(self.COLS))),
                        tuple(getattr(b, c) for c in self.COLS))
        self.log(b.id, "award", b.bonus_amount, b.wagering_progress, b.trigger_tx_id)

    def update(self, b) -> None:
        self.db.execute("UPDATE player_bonuses SET status = ?, wagering_progress = ?, free_spins_used = ?, "
                        "completed_at = ? WHERE id = ?",
                        (b.status, b.wagering_progress, b.free_spins_used, b.completed_at, b.id))

    def log(self, bonus_id: str, kind: str, amount: int, progress: Optional[int] = None, tx_id: Optional[str] = None):
        import uuid
        self.db.execute("INSERT INTO bonus_transactions(id, bonus_id, transaction_id, type, amount, progress_after, "
                        "created_at) VALUES (?,?,?,?,?,?,?)",
                        (str(uuid.uuid4()), bonus_id, tx_id, kind, int(amount), progress, time.time()))

    def _rows(self, sql: str, args=()):
        from ..bonus.engine import PlayerBonus
        return [PlayerBonus(**{c: r[c] for c in self.COLS}) for r in self.db.query(sql, args)]

    def get(self, bonus_id: str):
        r = self._rows("SELECT * FROM player_bonuses WHERE id = ?", (bonus_id,))
        return r[0] if r else None

    def active_by_account(self, account_id: str):
        return self._rows("SELECT * FROM player_bonuses WHERE account_id = ? AND status = 'active' "
                          "ORDER BY awarded_at, rowid", (account_id,))

    def count_by_rule_and_account(self, rule_id: str, account_id: str) -> int:
        return int(self.db.query("SELECT COUNT(*) AS n FROM player_bonuses WHERE rule_id = ? AND account_id = ?",
                                 (rule_id, account_id))[0]["n"])

    def expired(self, now: float):
        return self._rows("SELECT * FROM player_bonuses WHERE status = 'active' AND expires_at <= ?", (now,))

    def count_by_account(self, account_id: str) -> int:
        return int(self.db.query("SELECT COUNT(*) AS n FROM player_bonuses WHERE account_id = ?",
                                 (account_id,))[0]["n"])


class AuditRepository:
    """risk_scores / ltv_predictions / event_outbox writers (the reference declares these tables,
    init-db.sql:122-188, and never writes them)."""

    def __init__(self, db: Database):
        self.db = db

    def risk_score(self, account_id: str, score: int, rule_score: int, ml_score: float, action: str,
                   reasons: Sequence[str], transaction_id: Optional[str] = None, response_ms: int = 0) -> None:
        self.db.execute("INSERT INTO risk_scores(account_id, transaction_id, score, rule_score, ml_score, action, "
                        "reason_codes, response_ms, created_at) VALUES (?,?,?,?,?,?,?,?,?)",
                        (account_id, transaction_id, score, rule_score, ml_score, action, json.dumps(list(reasons)),
                         response_ms, time.time()))

    def outbox(self, exchange: str, routing_key: str, payload: str) -> str:
        import uuid
        i = str(uuid.uuid4())
        self.db.execute("INSERT INTO event_outbox(id, exchange, routing_key, payload, created_at) VALUES (?,?,?,?,?)",
                        (i, exchange, routing_key, payload, time.time()))
        return i

    def pending_outbox(self, limit: int = 100):
        return self.db.query("SELECT * FROM event_outbox WHERE published_at IS NULL ORDER BY created_at LIMIT ?",
                             (limit,))

    def mark_published(self, ids: Sequence[str]) -> None:
        now = time.time()
        for i in ids:
            self.db.execute("UPDATE event_outbox SET published_at = ?, attempts = attempts + 1 WHERE id = ?", (now, i))

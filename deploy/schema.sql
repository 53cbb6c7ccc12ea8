-- Platform schema (SQLite dialect; executed by igaming_platform_amd/wallet/repository.py).
-- Covers the ten tables of the reference schema (deploy/init-db.sql): wallet accounts,
-- transactions and ledger; bonuses; the risk audit tables; blacklists; the event outbox and
-- an audit log. Money is int64 cents everywhere. Differences from the reference:
--   * the ledger is real double-entry (every transaction posts to the account AND to the
--     platform clearing account, so each transaction's entries sum to zero);
--   * the optimistic-lock trigger only fires when a balance changes without a version bump
--     (the reference's trigger also rejected status-only updates, quirk Q15).

PRAGMA foreign_keys = ON;

CREATE TABLE IF NOT EXISTS accounts (
    id          TEXT PRIMARY KEY,
    player_id   TEXT NOT NULL UNIQUE,
    currency    TEXT NOT NULL DEFAULT 'USD' CHECK (length(currency) = 3),
    balance     INTEGER NOT NULL DEFAULT 0 CHECK (balance >= 0),
    bonus       INTEGER NOT NULL DEFAULT 0 CHECK (bonus >= 0),
    status      TEXT NOT NULL DEFAULT 'active' CHECK (status IN ('active', 'suspended', 'closed', 'system')),
    version     INTEGER NOT NULL DEFAULT 1,
    created_at  REAL NOT NULL,
    updated_at  REAL NOT NULL
);
CREATE INDEX IF NOT EXISTS ix_accounts_status ON accounts(status);

CREATE TABLE IF NOT EXISTS transactions (
    id               TEXT PRIMARY KEY,
    account_id       TEXT NOT NULL REFERENCES accounts(id),
    idempotency_key  TEXT NOT NULL,
    type             TEXT NOT NULL,
    amount           INTEGER NOT NULL CHECK (amount > 0),
    balance_before   INTEGER NOT NULL,
    balance_after    INTEGER NOT NULL,
    status           TEXT NOT NULL DEFAULT 'pending',
    reference        TEXT,
    game_id          TEXT,
    round_id         TEXT,
    risk_score       INTEGER,
    metadata         TEXT NOT NULL DEFAULT '{}',
    created_at       REAL NOT NULL,
    completed_at     REAL,
    UNIQUE (account_id, idempotency_key)
);
CREATE INDEX IF NOT EXISTS ix_tx_account_time ON transactions(account_id, created_at DESC);
CREATE INDEX IF NOT EXISTS ix_tx_round ON transactions(game_id, round_id);
CREATE INDEX IF NOT EXISTS ix_tx_type_status ON transactions(type, status);

CREATE TABLE IF NOT EXISTS ledger_entries (
    id              TEXT PRIMARY KEY,
    transaction_id  TEXT NOT NULL REFERENCES transactions(id),
    account_id      TEXT NOT NULL REFERENCES accounts(id),
    entry_type      TEXT NOT NULL CHECK (entry_type IN ('debit', 'credit')),
    amount          INTEGER NOT NULL CHECK (amount > 0),
    balance_after   INTEGER NOT NULL,
    description     TEXT,
    created_at      REAL NOT NULL
);
CREATE INDEX IF NOT EXISTS ix_ledger_account ON ledger_entries(account_id, created_at);
CREATE INDEX IF NOT EXISTS ix_ledger_tx ON ledger_entries(transaction_id);

CREATE TABLE IF NOT EXISTS player_bonuses (
    id                 TEXT PRIMARY KEY,
    account_id         TEXT NOT NULL,
    rule_id            TEXT NOT NULL,
    type               TEXT NOT NULL,
    status             TEXT NOT NULL DEFAULT 'active'
                       CHECK (status IN ('active', 'completed', 'expired', 'forfeited', 'cancelled')),
    bonus_amount       INTEGER NOT NULL,
    wagering_required  INTEGER NOT NULL,
    wagering_progress  INTEGER NOT NULL DEFAULT 0,
    free_spins_total   INTEGER NOT NULL DEFAULT 0,
    free_spins_used    INTEGER NOT NULL DEFAULT 0,
    awarded_at         REAL NOT NULL,
    expires_at         REAL NOT NULL,
    completed_at       REAL,
    trigger_tx_id      TEXT,
    promo_code         TEXT
);
CREATE INDEX IF NOT EXISTS ix_bonus_account_status ON player_bonuses(account_id, status);
CREATE INDEX IF NOT EXISTS ix_bonus_rule ON player_bonuses(rule_id, account_id);
CREATE INDEX IF NOT EXISTS ix_bonus_expiry ON player_bonuses(status, expires_at);

CREATE TABLE IF NOT EXISTS bonus_transactions (
    id              TEXT PRIMARY KEY,
    bonus_id        TEXT NOT NULL REFERENCES player_bonuses(id),
    transaction_id  TEXT,
    type            TEXT NOT NULL,           -- award | wager | release | forfeit | expire
    amount          INTEGER NOT NULL,
    progress_after  INTEGER,
    created_at      REAL NOT NULL
);

-- risk audit: every decision (the reference declares this table and never writes it)
CREATE TABLE IF NOT EXISTS risk_scores (
    id            INTEGER PRIMARY KEY AUTOINCREMENT,
    account_id    TEXT NOT NULL,
    transaction_id TEXT,
    score         INTEGER NOT NULL,
    rule_score    INTEGER NOT NULL,
    ml_score      REAL NOT NULL,
    action        TEXT NOT NULL,
    reason_codes  TEXT NOT NULL DEFAULT '[]',
    features      TEXT,
    model_version TEXT,
    response_ms   INTEGER,
    created_at    REAL NOT NULL
);
CREATE INDEX IF NOT EXISTS ix_risk_account_time ON risk_scores(account_id, created_at DESC);

CREATE TABLE IF NOT EXISTS ltv_predictions (
    id                INTEGER PRIMARY KEY AUTOINCREMENT,
    account_id        TEXT NOT NULL,
    predicted_ltv     REAL NOT NULL,
    segment           TEXT NOT NULL,
    churn_risk        REAL NOT NULL,
    survival_days     INTEGER,
    confidence        REAL,
    next_best_action  TEXT,
    model_version     TEXT,
    created_at        REAL NOT NULL
);

CREATE TABLE IF NOT EXISTS blacklists (
    id          TEXT PRIMARY KEY,
    type        TEXT NOT NULL CHECK (type IN ('device', 'ip', 'fingerprint', 'email')),
    value       TEXT NOT NULL,
    reason      TEXT,
    created_by  TEXT,
    created_at  REAL NOT NULL,
    expires_at  REAL,
    UNIQUE (type, value)
);

-- transactional outbox: events written in the same DB transaction as the state change
CREATE TABLE IF NOT EXISTS event_outbox (
    id            TEXT PRIMARY KEY,
    exchange      TEXT NOT NULL,
    routing_key   TEXT NOT NULL,
    payload       TEXT NOT NULL,
    created_at    REAL NOT NULL,
    published_at  REAL,
    attempts      INTEGER NOT NULL DEFAULT 0
);
CREATE INDEX IF NOT EXISTS ix_outbox_pending ON event_outbox(published_at, created_at);

CREATE TABLE IF NOT EXISTS audit_log (
    id          INTEGER PRIMARY KEY AUTOINCREMENT,
    entity      TEXT NOT NULL,
    entity_id   TEXT NOT NULL,
    action      TEXT NOT NULL,
    actor       TEXT,
    old_value   TEXT,
    new_value   TEXT,
    created_at  REAL NOT NULL
);

-- optimistic locking: a balance change must come with version = old.version + 1
CREATE TRIGGER IF NOT EXISTS trg_accounts_version
BEFORE UPDATE OF balance, bonus ON accounts
WHEN NEW.version != OLD.version + 1
BEGIN
    SELECT RAISE(ABORT, 'concurrent update detected');
END;

CREATE TRIGGER IF NOT EXISTS trg_accounts_audit
AFTER UPDATE OF status ON accounts
WHEN NEW.status != OLD.status
BEGIN
    INSERT INTO audit_log(entity, entity_id, action, old_value, new_value, created_at)
    VALUES ('account', NEW.id, 'status', OLD.status, NEW.status, NEW.updated_at);
END;

-- the platform clearing account: contra side of every ledger posting
INSERT OR IGNORE INTO accounts(id, player_id, currency, balance, bonus, status, version, created_at, updated_at)
VALUES ('00000000-0000-0000-0000-000000000000', '__platform_clearing__', 'USD', 0, 0, 'system', 1, 0, 0);
